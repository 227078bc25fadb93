// adapter.cpp -- the INTEGRATION.md adapter bodies, compiled (test infrastructure): the code a maintainer puts
// behind the reference's class surface, over the C ABI of include/svo_c.h.  tests/test_adapter.py compiles this
// file against tests/cpp/ref_types.hpp (the shapes of the reference's Frame / Feature / Point / camera types) and
// checks that every block between "// >>> name" and "// <<< name" appears verbatim in INTEGRATION.md.
//
// Error convention: the reference's align() never throws and returns its RMSE (0 without ref
// features, NaN when nothing is visible, -1 for Non_Suff_Points).  Every svo_* return is checked; on any failure
// the adapter leaves the frame's pose (or the pixel position) untouched and returns NaN.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include "ref_types.hpp"

int32_t g_svo_device = 0;

// >>> context
// one context per host thread (the main thread runs align, src/system.cpp:312); nullptr while none can be made
static svo_ctx* ctx() {
    static thread_local svo_ctx* c = nullptr;
    if (!c && svo_ctx_create(g_svo_device, &c) != SVO_OK) c = nullptr;
    return c;
}
static const double kNaN = std::numeric_limits<double>::quiet_NaN();
// <<< context

// >>> ImageAlignment::align
double ImageAlignment::align(std::shared_ptr<Frame>& ref, std::shared_ptr<Frame>& cur) {
    if (ref->numberObservation() == 0) return 0.0;                         // :27-28
    const auto& kf = ref->m_lastKeyframe;                                   // :30-31 (must be non-null)
    std::vector<double> px, br, pt; std::vector<uint8_t> hp;
    for (const Frame* fr : {ref.get(), kf.get()})                           // slot order :85-121
        for (const auto& f : fr->m_features) {
            px.insert(px.end(), {f->m_pixelPosition.x(), f->m_pixelPosition.y()});
            br.insert(br.end(), {f->m_bearingVec.x(), f->m_bearingVec.y(), f->m_bearingVec.z()});
            const Eigen::Vector3d P = f->m_point ? f->m_point->m_position : Eigen::Vector3d::Zero();
            pt.insert(pt.end(), {P.x(), P.y(), P.z()});
            hp.push_back(f->m_point != nullptr);
        }
    const int32_t nr = (int32_t)ref->m_features.size(), nk = (int32_t)kf->m_features.size();
    svo_camera cam{ref->m_camera->fx(), ref->m_camera->fy(), ref->m_camera->cx(), ref->m_camera->cy(),
                   ref->m_camera->width(), ref->m_camera->height()};
    // the reference's own robust scale (std::nth_element post-state), bit for bit; SVO_MEDIAN_EXACT is the faster
    // exact-order-statistic variant.  One grow-only batch per thread: no device allocation
    // per frame (recreated only when the feature count or the parameters grow / change).  The capacity only sizes
    // buffers: each run picks its robust-scale kernel from the frame's own vector ((nr + nk) * patch^2).
    svo_align_params prm{(int32_t)m_patchSize, m_minLevel, m_maxLevel, SVO_MEDIAN_REFERENCE};
    static thread_local svo_align_batch* b = nullptr;
    static thread_local int32_t cap = 0;
    static thread_local svo_align_params have{};
    svo_ctx* c = ctx();
    if (!c) return kNaN;                                                    // no device: pose untouched
    if (!b || nr + nk > cap || std::memcmp(&have, &prm, sizeof prm) != 0) {
        if (b) svo_align_batch_destroy(b);
        b = nullptr;
        // doubling, clamped to the reference-mode limit (SVO_REF_MAX_SLOTS residual slots per pair)
        const int32_t want = std::max(nr + nk, std::min(2 * cap, SVO_REF_MAX_SLOTS / (int32_t)(m_patchSize * m_patchSize)));
        if (svo_align_batch_create(c, &cam, &prm, 1, want, &b) != SVO_OK) { b = nullptr; cap = 0; return kNaN; }
        cap = want;
        have = prm;
    }
    // pyramids: the frames' device-resident svo_pyramid_set (see ImagePyramid below)
    if (svo_align_batch_set_pair(b, 0, ref->m_imagePyramid.set(), 0, kf->m_imagePyramid.set(), 0,
                                 cur->m_imagePyramid.set(), 0, ref->m_absPose.data(), kf->m_absPose.data(),
                                 cur->m_absPose.data(), nr, nk, px.data(), br.data(), pt.data(), hp.data()) != SVO_OK)
        return kNaN;
    if (svo_align_batch_run(b) != SVO_OK) return kNaN;
    double pose[7], err; int32_t status;
    if (svo_align_batch_results(b, pose, &err, &status) != SVO_OK) return kNaN;
    cur->m_absPose = Sophus::SE3d(Eigen::Quaterniond(pose[3], pose[0], pose[1], pose[2]),
                                  Eigen::Vector3d(pose[4], pose[5], pose[6]));   // params() order qx..qw tx..tz
    return err;
}
// <<< ImageAlignment::align

// >>> ImagePyramid
void ImagePyramid::createImagePyramid(const cv::Mat& base, const std::size_t levels) {
    if (m_set) svo_pyramid_set_destroy(m_set);                               // the stacks are rebuilt, not appended
    m_set = nullptr;
    svo_ctx* c = ctx();
    if (!c || svo_pyramid_set_create(c, 1, base.cols, base.rows, (int32_t)levels, &m_set) != SVO_OK) {
        m_set = nullptr;                                                     // align() then returns NaN
        return;
    }
    if (svo_pyramid_set_upload(m_set, 0, 1, base.ptr<uint8_t>()) != SVO_OK ||   // CV_8UC1, continuous
        svo_pyramid_set_build(m_set, 0, 1) != SVO_OK) {
        svo_pyramid_set_destroy(m_set);
        m_set = nullptr;
    }
}
ImagePyramid::~ImagePyramid() {
    if (m_set) svo_pyramid_set_destroy(m_set);
}
// <<< ImagePyramid

// >>> ImagePyramid getters
// host copies on demand of the device stacks (the reference keeps cv::Mat stacks, src/image_pyramid.cpp:54-124).
// Every svo_* return is checked: without a set, past the last level or on any failure a getter returns an empty Mat
// (rows = cols = 0) and the sizes are (0, 0), as the reference's getImageSizeAtLevel past the last level.
std::size_t ImagePyramid::getSizeImagePyramid() const {
    std::size_t n = 0;
    int32_t w = 0, h = 0;
    while (m_set && svo_pyramid_level_size(m_set, (int32_t)n, &w, &h) == SVO_OK && w > 0) ++n;
    return n;
}
cv::Size ImagePyramid::getImageSizeAtLevel(const std::size_t level) const {
    int32_t w = 0, h = 0;
    if (!m_set || level >= (std::size_t)INT32_MAX || svo_pyramid_level_size(m_set, (int32_t)level, &w, &h) != SVO_OK)
        return cv::Size(0, 0);
    return cv::Size(w, h);
}
cv::Size ImagePyramid::getBaseImageSize() const { return getImageSizeAtLevel(0); }
const cv::Mat& ImagePyramid::hostLevel(const std::size_t level, const int32_t gradient) const {
    const cv::Size sz = getImageSizeAtLevel(level);
    m_none = cv::Mat();
    if (sz.width == 0) return m_none;                                        // no set, or past the last level
    std::vector<cv::Mat>& cache = gradient ? m_hostGradients : m_hostImages;
    if (cache.size() <= level) cache.resize(level + 1);
    cv::Mat& m = cache[level];
    m.create(sz.height, sz.width, CV_8UC1);
    if (svo_pyramid_set_download(m_set, 0, (int32_t)level, gradient, m.ptr<uint8_t>()) != SVO_OK) m = cv::Mat();
    return m;
}
const cv::Mat& ImagePyramid::getImageAtLevel(const std::size_t level) const { return hostLevel(level, 0); }
const cv::Mat& ImagePyramid::getGradientAtLevel(const std::size_t level) const { return hostLevel(level, 1); }
const cv::Mat& ImagePyramid::getBaseImage() const { return hostLevel(0, 0); }
const cv::Mat& ImagePyramid::getBaseGradientImage() const { return hostLevel(0, 1); }
// the non-const overloads hand out the same host copy (writes to it do not reach the device stacks)
cv::Mat& ImagePyramid::getImageAtLevel(const std::size_t level) {
    return const_cast<cv::Mat&>(static_cast<const ImagePyramid&>(*this).getImageAtLevel(level));
}
cv::Mat& ImagePyramid::getGradientAtLevel(const std::size_t level) {
    return const_cast<cv::Mat&>(static_cast<const ImagePyramid&>(*this).getGradientAtLevel(level));
}
const std::vector<cv::Mat>& ImagePyramid::getAllImages() const {
    const std::size_t n = getSizeImagePyramid();
    for (std::size_t l = 0; l < n; ++l) hostLevel(l, 0);
    m_hostImages.resize(n);
    return m_hostImages;
}
// <<< ImagePyramid getters

// >>> FeatureAlignment::align
double FeatureAlignment::align(const std::shared_ptr<Feature>& ref, const std::shared_ptr<Frame>& cur,
                               Eigen::Vector2d& pixelPos) {
    svo_ctx* c = ctx();
    if (!c) return kNaN;
    svo_camera cam{cur->m_camera->fx(), cur->m_camera->fy(), cur->m_camera->cx(), cur->m_camera->cy(),
                   cur->m_camera->width(), cur->m_camera->height()};
    double rpx[2] = {ref->m_pixelPosition.x(), ref->m_pixelPosition.y()}, px[2] = {pixelPos.x(), pixelPos.y()};
    double err; int32_t status;
    if (svo_feature_align(c, &cam, (int32_t)m_patchSize, ref->m_frame->m_imagePyramid.set(), nullptr, 0,
                          cur->m_imagePyramid.set(), 0, 1, rpx, px, &err, &status) != SVO_OK)
        return kNaN;                                                         // pixelPos untouched
    pixelPos = {px[0], px[1]};
    return err;
}
// <<< FeatureAlignment::align
