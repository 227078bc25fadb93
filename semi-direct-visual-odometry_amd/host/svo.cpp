// svo.cpp — implementation of the C++ class-surface mirror (host/svo.hpp) over the C ABI.
#include <cstring>
#include "svo.hpp"

#include <algorithm>
#include <cmath>
#include <iomanip>
#include <random>
#include <string>
#include <unordered_map>

namespace svo_amd {

static void check(int rc) {
    if (rc != SVO_OK) throw Error(rc, std::string("svo: ") + svo_last_error());
}

Context::Context(int device) { check(svo_ctx_create(device, &m_ctx)); }
Context::~Context() { svo_ctx_destroy(m_ctx); }

Vec2 PinholeCamera::project2d(const Vec3& p) const { return {fx * (p[0] / p[2]) + cx, fy * (p[1] / p[2]) + cy}; }
Vec3 PinholeCamera::inverseProject2d(const Vec2& px) const {
    Vec3 v{(px[0] - cx) / fx, (px[1] - cy) / fy, 1.0};
    const double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    return {v[0] * (1.0 / n), v[1] * (1.0 / n), v[2] * (1.0 / n)};
}
bool PinholeCamera::isInFrame(const Vec2& p, double b) const {
    return p[0] >= b && p[1] >= b && p[0] < width - b && p[1] < height - b;
}

ImagePyramid::ImagePyramid(Context& ctx, std::size_t levels) : m_ctx(ctx), m_levels(levels) {}
ImagePyramid::ImagePyramid(Context& ctx, const uint8_t* img, int32_t w, int32_t h, std::size_t levels)
    : m_ctx(ctx), m_levels(levels) {
    createImagePyramid(img, w, h, levels);
}
ImagePyramid::~ImagePyramid() { clear(); }
void ImagePyramid::createImagePyramid(const uint8_t* img, int32_t w, int32_t h, std::size_t levels) {
    clear();
    m_levels = levels;
    check(svo_pyramid_set_create(m_ctx.get(), 1, w, h, (int32_t)levels, &m_set));
    check(svo_pyramid_set_upload(m_set, 0, 1, img));
    check(svo_pyramid_set_build(m_set, 0, 1));
    check(svo_ctx_synchronize(m_ctx.get()));
}
std::array<int32_t, 2> ImagePyramid::getImageSizeAtLevel(std::size_t level) const {
    std::array<int32_t, 2> s{0, 0};
    if (m_set) check(svo_pyramid_level_size(m_set, (int32_t)level, &s[0], &s[1]));
    return s;
}
std::vector<uint8_t> ImagePyramid::getImageAtLevel(std::size_t level) const {
    auto s = getImageSizeAtLevel(level);
    std::vector<uint8_t> out((size_t)s[0] * s[1]);
    check(svo_pyramid_set_download(m_set, 0, (int32_t)level, 0, out.data()));
    return out;
}
std::vector<uint8_t> ImagePyramid::getGradientAtLevel(std::size_t level) const {
    auto s = getImageSizeAtLevel(level);
    std::vector<uint8_t> out((size_t)s[0] * s[1]);
    check(svo_pyramid_set_download(m_set, 0, (int32_t)level, 1, out.data()));
    return out;
}
void ImagePyramid::clear() {
    if (m_set) svo_pyramid_set_destroy(m_set);
    m_set = nullptr;
}

Feature::Feature(Frame* frame, const Vec2& px)
    : m_frame(frame), m_pixelPosition(px), m_bearingVec(frame->m_camera->inverseProject2d(px)) {}

Frame::Frame(Context& ctx, std::shared_ptr<PinholeCamera> camera, const uint8_t* img, uint32_t maxImagePyramid,
             std::shared_ptr<Frame> lastKeyframe)
    : m_camera(std::move(camera)), m_imagePyramid(ctx, maxImagePyramid), m_lastKeyframe(std::move(lastKeyframe)) {
    static uint64_t frameCounter = 0;  // Frame::m_frameCounter
    m_id = frameCounter++;
    if (!img) throw std::runtime_error("Image Corrupted");  // src/frame.cpp:20-24
    m_imagePyramid.createImagePyramid(img, m_camera->width, m_camera->height, maxImagePyramid);
}

ImageAlignment::ImageAlignment(Context& ctx, uint32_t patchSize, int32_t minLevel, int32_t maxLevel, uint32_t numParameters,
                               int32_t medianMode)
    : m_ctx(ctx), m_params{(int32_t)patchSize, minLevel, maxLevel, medianMode} {
    if (numParameters != 6) throw Error(SVO_ERR_ARG, "ImageAlignment: numParameters must be 6");
}

ImageAlignment::~ImageAlignment() {
    if (m_batch) svo_align_batch_destroy(m_batch);
}

double ImageAlignment::align(std::shared_ptr<Frame>& refFrame, std::shared_ptr<Frame>& curFrame) {
    if (refFrame->numberObservation() == 0) return 0;  // src/image_alignment.cpp:27-28
    const auto& kf = refFrame->m_lastKeyframe;
    const int32_t nr = (int32_t)refFrame->numberObservation(), nk = (int32_t)kf->numberObservation();
    m_px.clear(); m_br.clear(); m_pt.clear(); m_hp.clear();
    for (const auto* fr : {refFrame.get(), kf.get()})
        for (const auto& f : fr->m_features) {
            m_px.insert(m_px.end(), f->m_pixelPosition.begin(), f->m_pixelPosition.end());
            m_br.insert(m_br.end(), f->m_bearingVec.begin(), f->m_bearingVec.end());
            const Vec3 p = f->m_point ? f->m_point->m_position : Vec3{0, 0, 0};
            m_pt.insert(m_pt.end(), p.begin(), p.end());
            m_hp.push_back(f->m_point ? 1 : 0);
        }
    const svo_camera cam = refFrame->m_camera->c();
    const bool same_cam = m_batch && std::memcmp(&cam, &m_batchCam, sizeof(cam)) == 0;
    if (!same_cam || nr + nk > m_batchCap) {  // grow-only: a new batch only for a larger frame or another camera
        if (m_batch) svo_align_batch_destroy(m_batch);
        m_batch = nullptr;
        int32_t grow = same_cam ? 2 * m_batchCap : 1;
        if (m_params.median_mode == SVO_MEDIAN_REFERENCE)  // doubling must not cross the reference-mode limit
            grow = std::min(grow, SVO_REF_MAX_SLOTS / (m_params.patch_size * m_params.patch_size));
        const int32_t cap = std::max(nr + nk, grow);
        check(svo_align_batch_create(m_ctx.get(), &cam, &m_params, 1, cap, &m_batch));
        m_batchCap = cap;
        m_batchCam = cam;
    }
    double err = 0.0;
    check(svo_align_batch_set_pair(m_batch, 0, refFrame->m_imagePyramid.set(), 0, kf->m_imagePyramid.set(), 0,
                                   curFrame->m_imagePyramid.set(), 0, refFrame->m_absPose.data(), kf->m_absPose.data(),
                                   curFrame->m_absPose.data(), nr, nk, m_px.data(), m_br.data(), m_pt.data(),
                                   m_hp.data()));
    check(svo_align_batch_run(m_batch));
    check(svo_align_batch_results(m_batch, curFrame->m_absPose.data(), &err, &m_status));
    return err;
}

FeatureAlignment::FeatureAlignment(Context& ctx, uint32_t patchSize, int32_t level, uint32_t numParameters)
    : m_ctx(ctx), m_patchSize(patchSize) {
    if (numParameters != 3) throw Error(SVO_ERR_ARG, "FeatureAlignment: numParameters must be 3");
    if (level != 0) throw Error(SVO_ERR_ARG, "FeatureAlignment works on level 0 (src/feature_alignment.cpp:69)");
}

double FeatureAlignment::align(const std::shared_ptr<Feature>& refFeature, const std::shared_ptr<Frame>& curFrame,
                               Vec2& pixelPos) {
    svo_camera cam = curFrame->m_camera->c();
    double err = 0.0;
    check(svo_feature_align(m_ctx.get(), &cam, (int32_t)m_patchSize, refFeature->m_frame->m_imagePyramid.set(), nullptr,
                            0, curFrame->m_imagePyramid.set(), 0, 1, refFeature->m_pixelPosition.data(),
                            pixelPos.data(), &err, &m_status));
    return err;
}

// ------------------------------------------------------------------ FeatureSelection
FeatureSelection::FeatureSelection(Context& ctx, int32_t width, int32_t height, int32_t cellSize)
    : m_ctx(ctx), m_width(width), m_height(height), m_cellSize(cellSize) {
    check(svo_feature_grid_size(width, height, cellSize, &m_gridRows, &m_gridCols));
    m_occupancyGrid.assign((size_t)m_gridRows * m_gridCols, 0);
}

void FeatureSelection::emit(std::shared_ptr<Frame>& frame, const std::vector<double>& px, const std::vector<double>& resp,
                            int32_t n) {
    for (int32_t i = 0; i < n; ++i) {  // Feature(frame, px, response, angle 0, level 0, EDGE) (:68-71)
        auto f = std::make_shared<Feature>(frame.get(), Vec2{px[2 * i], px[2 * i + 1]});
        f->m_gradientMagnitude = resp[i];
        frame->m_features.push_back(std::move(f));
    }
}

void FeatureSelection::gradientMagnitudeWithSSC(std::shared_ptr<Frame>& frame, uint32_t detectionThreshold,
                                                uint32_t numberCandidate, bool useBucketing) {
    const int32_t cap = useBucketing ? m_gridRows * m_gridCols : m_width * m_height;
    std::vector<double> px(2 * (size_t)cap), resp(cap);
    int32_t n = 0;
    check(svo_feature_select_ssc(m_ctx.get(), frame->m_imagePyramid.set(), 0, (int32_t)detectionThreshold,
                                 (int32_t)numberCandidate, useBucketing ? 1 : 0, m_cellSize, m_occupancyGrid.data(), cap,
                                 px.data(), resp.data(), &n, nullptr));
    emit(frame, px, resp, n);
}

void FeatureSelection::gradientMagnitudeByValue(std::shared_ptr<Frame>& frame, uint32_t detectionThreshold,
                                                bool useBucketing) {
    if (!useBucketing) throw Error(SVO_ERR_ARG, "svo: gradientMagnitudeByValue without bucketing is not supported");
    const int32_t cap = m_gridRows * m_gridCols;
    std::vector<double> px(2 * (size_t)cap), resp(cap);
    int32_t n = 0;
    check(svo_feature_select_by_value(m_ctx.get(), frame->m_imagePyramid.set(), 0, (int32_t)detectionThreshold,
                                      m_cellSize, m_occupancyGrid.data(), cap, px.data(), resp.data(), &n));
    emit(frame, px, resp, n);
}

void FeatureSelection::setExistingFeatures(const std::vector<std::shared_ptr<Feature>>& features) {
    for (const auto& f : features) setCellInGridOccupancy(f->m_pixelPosition);
}

void FeatureSelection::setCellInGridOccupancy(const Vec2& location) {  // :276-282
    const uint32_t idx = location[0] / m_cellSize;
    const uint32_t idy = location[1] / m_cellSize;
    m_occupancyGrid[idy * m_gridCols + idx] = 1;
}

void FeatureSelection::resetGridOccupancy() { std::fill(m_occupancyGrid.begin(), m_occupancyGrid.end(), 0); }

// ------------------------------------------------------------------ BundleAdjustment
BundleAdjustment::BundleAdjustment(Context& ctx, std::shared_ptr<PinholeCamera> camera, int32_t level,
                                   uint32_t numParameters)
    : m_ctx(ctx), m_camera(std::move(camera)) {
    if (numParameters != 6 || level != 0) throw Error(SVO_ERR_ARG, "svo: BundleAdjustment(camera, 0, 6) only");
}

double BundleAdjustment::optimizePose(std::shared_ptr<Frame>& frame) {
    const std::size_t n = frame->numberObservation();
    if (n == 0) return 0;  // src/bundle_adjustment.cpp:37-38
    m_refVisibility.resize(n, 0);
    std::vector<double> bearing(3 * n), point(3 * n, 0.0);
    std::vector<uint8_t> has(n, 0);
    for (std::size_t k = 0; k < n; ++k) {
        const auto& f = frame->m_features[k];
        for (int i = 0; i < 3; ++i) bearing[3 * k + i] = f->m_bearingVec[i];
        if (f->m_point) {
            has[k] = 1;
            for (int i = 0; i < 3; ++i) point[3 * k + i] = f->m_point->m_position[i];
        }
    }
    const int32_t off[2] = {0, (int32_t)n};
    double err = 0.0;
    check(svo_pose_optimize(m_ctx.get(), 1, off, bearing.data(), point.data(), has.data(), m_refVisibility.data(),
                            frame->m_absPose.data(), &err, &m_status));
    return err;
}

// ------------------------------------------------------------------ DepthEstimator
void DepthEstimator::addKeyframe(const std::shared_ptr<Frame>& frame, double depthMean, double depthMin) {
    const int32_t kf = (int32_t)m_keyframes.size();
    m_keyframes.push_back(frame);
    for (const auto& f : frame->m_features) {
        if (f->m_point) continue;  // initializeFilters: features without a point only
        svo_depth_seed sd{};
        check(svo_depth_seed_init(depthMean, depthMin, &sd));  // MixedGaussianFilter (src/mixed_gaussian_filter.cpp:7-24)
        sd.px[0] = f->m_pixelPosition[0];
        sd.px[1] = f->m_pixelPosition[1];
        for (int i = 0; i < 3; ++i) sd.bearing[i] = f->m_bearingVec[i];
        sd.kf = kf;
        m_seeds.push_back(sd);
        m_features.push_back(f);
    }
}

std::vector<std::pair<std::shared_ptr<Feature>, std::shared_ptr<Point>>> DepthEstimator::updateFilters(
    const std::shared_ptr<Frame>& frame) {
    std::vector<std::pair<std::shared_ptr<Feature>, std::shared_ptr<Point>>> out;
    const int32_t n = (int32_t)m_seeds.size();
    if (n == 0) return out;
    const int32_t nk = (int32_t)m_keyframes.size();
    std::vector<const svo_pyramid_set*> sets(nk);
    std::vector<int32_t> frames(nk, 0);
    std::vector<double> poses(7 * (size_t)nk);
    for (int32_t k = 0; k < nk; ++k) {
        sets[k] = m_keyframes[k]->m_imagePyramid.set();
        for (int i = 0; i < 7; ++i) poses[7 * k + i] = m_keyframes[k]->m_absPose[i];
    }
    std::vector<int32_t> outcome(n), cand_seed(n);
    std::vector<double> cand_points(3 * (size_t)n);
    int32_t n_out = 0, n_cand = 0;
    const svo_camera cam = frame->m_camera->c();
    std::vector<svo_depth_seed> seeds = m_seeds;
    check(svo_depth_update(m_ctx.get(), &cam, nk, sets.data(), frames.data(), poses.data(), frame->m_imagePyramid.set(),
                           0, frame->m_absPose.data(), n, seeds.data(), &n_out, outcome.data(), cand_points.data(),
                           cand_seed.data(), &n_cand));
    for (int32_t j = 0; j < n_cand; ++j)
        out.emplace_back(m_features[cand_seed[j]],
                         std::make_shared<Point>(Point{{cand_points[3 * j], cand_points[3 * j + 1], cand_points[3 * j + 2]}}));
    std::vector<std::shared_ptr<Feature>> keep;  // survivors, order kept (remove_if, :300-308)
    for (int32_t i = 0; i < n; ++i)
        if (outcome[i] == SVO_DEPTH_NO_MATCH || outcome[i] == SVO_DEPTH_UPDATED) keep.push_back(m_features[i]);
    m_features.swap(keep);
    seeds.resize(n_out);
    m_seeds.swap(seeds);
    return out;
}

// ------------------------------------------------------------------ Map
Map::Map(Context& ctx, std::shared_ptr<PinholeCamera> camera, int32_t cellSize, uint64_t seed)
    : m_ctx(ctx), m_camera(std::move(camera)), m_cellSize(cellSize) {
    m_gridCols = (m_camera->width + cellSize - 1) / cellSize;  // src/map.cpp:222-248
    m_gridRows = (m_camera->height + cellSize - 1) / cellSize;
    const int32_t n = m_gridCols * m_gridRows;
    m_cellOrders.resize(n);
    for (int32_t i = 0; i < n; ++i) m_cellOrders[i] = i;
    std::mt19937_64 rng(seed);
    std::shuffle(m_cellOrders.begin(), m_cellOrders.end(), rng);
    m_cellVisited.assign(n, 0);
}

void Map::reprojectMap(const std::shared_ptr<Frame>& refFrame, std::shared_ptr<Frame>& curFrame,
                       std::vector<std::pair<std::shared_ptr<Frame>, int32_t>>& overlapKeyFrames) {
    if (!refFrame->m_lastKeyframe) throw Error(SVO_ERR_ARG, "svo: reprojectMap needs refFrame->m_lastKeyframe");
    const std::shared_ptr<Frame> kfs[2] = {refFrame, refFrame->m_lastKeyframe};
    std::vector<std::shared_ptr<Feature>> feats;
    int32_t off[3] = {0, 0, 0};
    for (int k = 0; k < 2; ++k) {
        feats.insert(feats.end(), kfs[k]->m_features.begin(), kfs[k]->m_features.end());
        off[k + 1] = (int32_t)feats.size();
    }
    std::vector<std::shared_ptr<Point>> points;
    std::unordered_map<const Point*, int32_t> index;
    std::vector<int32_t> featPoint(std::max<size_t>(feats.size(), 1), -1);
    for (size_t i = 0; i < feats.size(); ++i) {
        const auto& pt = feats[i]->m_point;
        if (!pt) continue;
        auto it = index.emplace(pt.get(), (int32_t)points.size());
        if (it.second) points.push_back(pt);
        featPoint[i] = it.first->second;
    }
    const size_t np = std::max<size_t>(points.size(), 1);
    std::vector<double> pos(3 * np, 0.0);
    std::vector<uint32_t> type(np, 0);
    std::vector<uint64_t> last(np, 0);
    for (size_t i = 0; i < points.size(); ++i) {
        for (int j = 0; j < 3; ++j) pos[3 * i + j] = points[i]->m_position[j];
        type[i] = (uint32_t)points[i]->m_type;
        last[i] = points[i]->m_lastProjectedKFId;
    }
    const int32_t nCells = (int32_t)m_cellOrders.size();
    std::vector<int32_t> selFeat(nCells), selCell(nCells);
    std::vector<double> selPx(2 * (size_t)nCells);
    int32_t overlap[2] = {0, 0}, nSel = 0, matches = 0, trials = 0;
    const svo_camera cam = m_camera->c();
    check(svo_map_reproject_plan(&cam, m_cellSize, nCells, m_cellOrders.data(), curFrame->m_absPose.data(),
                                 curFrame->m_id, 2, off, featPoint.data(), (int32_t)points.size(), pos.data(),
                                 type.data(), last.data(), overlap, &nSel, selFeat.data(), selCell.data(),
                                 selPx.data(), &matches, &trials));
    for (size_t i = 0; i < points.size(); ++i) points[i]->m_lastProjectedKFId = last[i];
    for (int k = 0; k < 2; ++k) overlapKeyFrames.emplace_back(kfs[k], overlap[k]);
    m_matches = (uint32_t)matches;
    m_trials = (uint32_t)trials;
    if (nSel == 0) return;
    std::vector<const svo_pyramid_set*> sets(nSel);
    std::vector<int32_t> frames(nSel, 0), status(nSel);
    std::vector<double> refPx(2 * (size_t)nSel), err(nSel);
    for (int32_t i = 0; i < nSel; ++i) {
        const auto& f = feats[selFeat[i]];
        sets[i] = f->m_frame->m_imagePyramid.set();
        refPx[2 * i] = f->m_pixelPosition[0];
        refPx[2 * i + 1] = f->m_pixelPosition[1];
    }
    check(svo_feature_align_multi(m_ctx.get(), &cam, 7, sets.data(), frames.data(), curFrame->m_imagePyramid.set(), 0,
                                  nSel, refPx.data(), selPx.data(), err.data(), status.data()));
    for (int32_t i = 0; i < nSel; ++i) {  // src/map.cpp:558-569
        const auto& point = feats[selFeat[i]]->m_point;
        point->m_succeededProjection++;
        if (point->m_type == Point::PointType::UNKNOWN && point->m_succeededProjection > 10)
            point->m_type = Point::PointType::GOOD;
        auto feature = std::make_shared<Feature>(curFrame.get(), Vec2{selPx[2 * i], selPx[2 * i + 1]});
        curFrame->m_features.push_back(feature);
        feature->m_point = point;
        point->m_features.push_back(feature);
        m_cellVisited[selCell[i]] = 1;
    }
}

void Map::addNewCandidate(const std::shared_ptr<Feature>& feature, const std::shared_ptr<Point>& point) {
    point->m_type = Point::PointType::CANDIDATE;  // src/map.cpp:586-593
    m_candidates.push_back({feature, point, false});
}

void Map::addCandidateToFrame(std::shared_ptr<Frame>& frame) {
    const int32_t n = (int32_t)m_candidates.size();
    if (n == 0) return;
    std::vector<double> pos(3 * (size_t)n), px0(2 * (size_t)n);
    for (int32_t i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) pos[3 * i + j] = m_candidates[i].point->m_position[j];
    const svo_camera cam = m_camera->c();
    check(svo_world2image(&cam, frame->m_absPose.data(), n, pos.data(), px0.data()));
    const double w = frame->m_camera->width, h = frame->m_camera->height;
    std::vector<int32_t> elig, cells;
    for (int32_t i = 0; i < n; ++i) {  // isInFrame(px, 3) and a free cell (:600-606)
        const double x = px0[2 * i], y = px0[2 * i + 1];
        if (!(x >= 3 && y >= 3 && x < w - 3 && y < h - 3)) continue;
        const int32_t cell = (int32_t)y / m_cellSize * m_gridCols + (int32_t)x / m_cellSize;
        if (m_cellVisited[cell]) continue;
        elig.push_back(i);
        cells.push_back(cell);
    }
    const int32_t ne = (int32_t)elig.size();
    if (ne == 0) return;
    std::vector<const svo_pyramid_set*> sets(ne);
    std::vector<int32_t> frames(ne, 0), status(ne);
    std::vector<double> refPx(2 * (size_t)ne), px(2 * (size_t)ne), err(ne);
    for (int32_t j = 0; j < ne; ++j) {
        const auto& f = m_candidates[elig[j]].feature;
        sets[j] = f->m_frame->m_imagePyramid.set();
        refPx[2 * j] = f->m_pixelPosition[0];
        refPx[2 * j + 1] = f->m_pixelPosition[1];
        px[2 * j] = px0[2 * elig[j]];
        px[2 * j + 1] = px0[2 * elig[j] + 1];
    }
    check(svo_feature_align_multi(m_ctx.get(), &cam, 7, sets.data(), frames.data(), frame->m_imagePyramid.set(), 0, ne,
                                  refPx.data(), px.data(), err.data(), status.data()));
    for (int32_t j = 0; j < ne; ++j) {  // list order: a cell taken earlier in this loop is skipped (:607-624)
        if (m_cellVisited[cells[j]] || !(err[j] < 50.0)) continue;
        Candidate& c = m_candidates[elig[j]];
        auto feature = std::make_shared<Feature>(frame.get(), Vec2{px[2 * j], px[2 * j + 1]});
        frame->m_features.push_back(feature);
        c.point->m_features.push_back(c.feature);
        c.point->m_features.push_back(feature);
        c.feature->m_point = c.point;
        feature->m_point = c.point;
        c.matched = true;
        m_cellVisited[cells[j]] = 1;
    }
    removeMatchedCandidate();  // (:626)
}

void Map::removeMatchedCandidate() {  // src/map.cpp:629-634
    m_candidates.erase(std::remove_if(m_candidates.begin(), m_candidates.end(), [](const Candidate& c) { return c.matched; }),
                       m_candidates.end());
}

// ------------------------------------------------------------------ trajectory / feature dump
namespace utils {
void writeInFile(const Pose& refAbsPose, std::ostream& w) {
    double m[12];
    check(svo_pose_matrix3x4_inverse(refAbsPose.data(), m));
    w << std::setprecision(6);
    for (int i = 0; i < 12; ++i) w << (i ? " " : "") << m[i];
    w << std::endl;
}

void writeAllInfoFile(const Frame& ref, const Frame& cur, std::ostream& w) {
    for (std::size_t i = 0; i < ref.numberObservation(); i++) {
        const Vec2& r = ref.m_features[i]->m_pixelPosition;
        const Vec2& c = cur.m_features[i]->m_pixelPosition;
        const Vec3& p = ref.m_features[i]->m_point->m_position;
        w << std::setprecision(6) << r[0] << " " << r[1] << " " << c[0] << " " << c[1] << " " << p[0] << " " << p[1]
          << " " << p[2] << std::endl;
    }
}

void writeFeaturesInfoFile(const Frame& ref, const Frame& cur, std::ostream& w) {
    for (std::size_t i = 0; i < ref.numberObservation(); i++) {
        const Vec2& r = ref.m_features[i]->m_pixelPosition;
        const Vec2& c = cur.m_features[i]->m_pixelPosition;
        w << std::setprecision(6) << r[0] << " " << r[1] << " " << c[0] << " " << c[1] << std::endl;
    }
}
}  // namespace utils

}  // namespace svo_amd
