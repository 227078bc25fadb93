// svo.hpp — C++ mirror of the reference's alignment class surface over the C ABI (include/svo_c.h).
//
// The reference's callers (src/system.cpp:313, src/map.cpp:538,608, src/frame.cpp:26) use
//   ImageAlignment(patchSize, minLevel, maxLevel, numParameters); double align(ref, cur);
//   FeatureAlignment(patchSize, level, numParameters);            double align(feature, cur, pixelPos);
//   ImagePyramid(baseImage, maxPyramidLevel) + getters.
// The same names, argument meaning and error behaviour are kept here over self-contained types
// (Eigen / Sophus / OpenCV are absent from this image; INTEGRATION.md shows the adapter a maintainer adds
// to feed cv::Mat / Sophus::SE3d / Eigen::Vector2d through these types unchanged).
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <utility>
#include <vector>

#include "svo_c.h"

namespace svo_amd {

using Pose = std::array<double, 7>;  // Sophus::SE3d::params(): qx qy qz qw tx ty tz
using Vec2 = std::array<double, 2>;
using Vec3 = std::array<double, 3>;

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& msg) : std::runtime_error(msg), code(code) {}
    int code;
};

class Context {
public:
    explicit Context(int device = 0);
    ~Context();
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    svo_ctx* get() const { return m_ctx; }

private:
    svo_ctx* m_ctx = nullptr;
};

struct PinholeCamera {  // include/pinhole_camera.hpp:16 (undistorted)
    int32_t width, height;
    double fx, fy, cx, cy;
    Vec2 project2d(const Vec3& p) const;
    Vec3 inverseProject2d(const Vec2& px) const;
    bool isInFrame(const Vec2& p, double boundary = 0.0) const;
    svo_camera c() const { return {fx, fy, cx, cy, width, height}; }
};

// ImagePyramid (include/image_pyramid.hpp:23-149): device resident; copy/move deleted like the reference.
class ImagePyramid {
public:
    ImagePyramid(Context& ctx, std::size_t maxPyramidLevel);
    ImagePyramid(Context& ctx, const uint8_t* baseImage, int32_t width, int32_t height, std::size_t maxPyramidLevel);
    ImagePyramid(const ImagePyramid&) = delete;
    ImagePyramid& operator=(const ImagePyramid&) = delete;
    ~ImagePyramid();
    void createImagePyramid(const uint8_t* baseImage, int32_t width, int32_t height, std::size_t maxPyramidLevel);
    std::vector<uint8_t> getImageAtLevel(std::size_t level) const;
    std::vector<uint8_t> getGradientAtLevel(std::size_t level) const;
    std::vector<uint8_t> getBaseImage() const { return getImageAtLevel(0); }
    std::vector<uint8_t> getBaseGradientImage() const { return getGradientAtLevel(0); }
    std::size_t getSizeImagePyramid() const { return m_set ? m_levels : 0; }
    std::array<int32_t, 2> getImageSizeAtLevel(std::size_t level) const;  // (width, height); (0,0) past the top
    std::array<int32_t, 2> getBaseImageSize() const { return getImageSizeAtLevel(0); }
    void clear();
    const svo_pyramid_set* set() const { return m_set; }

private:
    Context& m_ctx;
    svo_pyramid_set* m_set = nullptr;
    std::size_t m_levels;
};

struct Frame;
struct Feature;
struct Point {  // include/point.hpp:14-40 (the members the map's reprojection reads and writes)
    enum class PointType : uint32_t { GOOD = 0, DELETED = 1, CANDIDATE = 2, UNKNOWN = 3 };
    Vec3 m_position;
    PointType m_type = PointType::UNKNOWN;
    uint64_t m_lastProjectedKFId = ~(uint64_t)0;  // m_lastProjectedKFId(-1)
    uint32_t m_succeededProjection = 0;
    uint32_t m_failedProjection = 0;
    std::vector<std::weak_ptr<Feature>> m_features;  // observing features (weak: Frame owns them)
};
struct Feature {  // include/feature.hpp:14
    enum class FeatureType : uint32_t { EDGE = 0, CORNER = 1 };  // include/feature.hpp:19-23
    Frame* m_frame;
    Vec2 m_pixelPosition;
    Vec3 m_bearingVec;
    std::shared_ptr<Point> m_point;
    double m_gradientMagnitude = 1.0;    // src/feature.cpp:15
    double m_gradientOrientation = 0.0;
    FeatureType m_type = FeatureType::EDGE;
    Feature(Frame* frame, const Vec2& px);
};
struct Frame {  // include/frame.hpp:70-208 (the members the alignment path reads)
    Frame(Context& ctx, std::shared_ptr<PinholeCamera> camera, const uint8_t* img, uint32_t maxImagePyramid,
          std::shared_ptr<Frame> lastKeyframe = nullptr);
    std::shared_ptr<PinholeCamera> m_camera;
    Pose m_absPose{0, 0, 0, 1, 0, 0, 0};
    ImagePyramid m_imagePyramid;
    std::vector<std::shared_ptr<Feature>> m_features;
    std::shared_ptr<Frame> m_lastKeyframe;
    uint64_t m_id;  // Frame::m_frameCounter (src/frame.cpp:6-27)
    std::size_t numberObservation() const { return m_features.size(); }
};

// ImageAlignment (include/image_alignment.hpp:15-73)
// medianMode: SVO_MEDIAN_REFERENCE (default) reproduces the reference's robust scale bit for bit.
// The single-pair batch is kept and grown on demand (no device allocation per align() once warm).
class ImageAlignment {
public:
    ImageAlignment(Context& ctx, uint32_t patchSize, int32_t minLevel, int32_t maxLevel, uint32_t numParameters,
                   int32_t medianMode = SVO_MEDIAN_REFERENCE);
    ~ImageAlignment();
    ImageAlignment(const ImageAlignment&) = delete;
    ImageAlignment& operator=(const ImageAlignment&) = delete;
    double align(std::shared_ptr<Frame>& refFrame, std::shared_ptr<Frame>& curFrame);
    int32_t lastStatus() const { return m_status; }

private:
    Context& m_ctx;
    svo_align_params m_params;
    int32_t m_status = SVO_STATUS_FAILED;
    svo_align_batch* m_batch = nullptr;
    int32_t m_batchCap = 0;
    svo_camera m_batchCam{};
    std::vector<double> m_px, m_br, m_pt;
    std::vector<uint8_t> m_hp;
};

// FeatureAlignment (include/feature_alignment.hpp:15-43)
class FeatureAlignment {
public:
    FeatureAlignment(Context& ctx, uint32_t patchSize, int32_t level, uint32_t numParameters);
    double align(const std::shared_ptr<Feature>& refFeature, const std::shared_ptr<Frame>& curFrame, Vec2& pixelPos);
    int32_t lastStatus() const { return m_status; }

private:
    Context& m_ctx;
    uint32_t m_patchSize;
    int32_t m_status = SVO_STATUS_FAILED;
};

// FeatureSelection (include/feature_selection.hpp, src/feature_selection.cpp:19-287): the occupancy grid
// is a host member as in the reference; detection runs on the frame's device-resident gradient plane.
class FeatureSelection {
public:
    FeatureSelection(Context& ctx, int32_t width, int32_t height, int32_t cellSize);
    FeatureSelection(const FeatureSelection&) = delete;
    FeatureSelection& operator=(const FeatureSelection&) = delete;
    void gradientMagnitudeWithSSC(std::shared_ptr<Frame>& frame, uint32_t detectionThreshold, uint32_t numberCandidate,
                                  bool useBucketing);
    void gradientMagnitudeByValue(std::shared_ptr<Frame>& frame, uint32_t detectionThreshold, bool useBucketing);
    void setExistingFeatures(const std::vector<std::shared_ptr<Feature>>& features);
    void setCellInGridOccupancy(const Vec2& location);
    void resetGridOccupancy();
    const std::vector<uint8_t>& occupancyGrid() const { return m_occupancyGrid; }

private:
    void emit(std::shared_ptr<Frame>& frame, const std::vector<double>& px, const std::vector<double>& resp, int32_t n);
    Context& m_ctx;
    int32_t m_width, m_height, m_cellSize, m_gridRows, m_gridCols;
    std::vector<uint8_t> m_occupancyGrid;
};

// BundleAdjustment (include/bundle_adjustment.hpp, src/bundle_adjustment.cpp:30-166): optimizePose over the
// C ABI.  m_refVisibility is kept across calls like the reference's member (include/svo_c.h explains why
// a fresh object returns NaN).  Several frames at once: optimizePoses.
class BundleAdjustment {
public:
    BundleAdjustment(Context& ctx, std::shared_ptr<PinholeCamera> camera, int32_t level, uint32_t numParameters);
    double optimizePose(std::shared_ptr<Frame>& frame);
    int32_t lastStatus() const { return m_status; }
    const std::vector<uint8_t>& refVisibility() const { return m_refVisibility; }

private:
    Context& m_ctx;
    std::shared_ptr<PinholeCamera> m_camera;
    std::vector<uint8_t> m_refVisibility;
    int32_t m_status = SVO_STATUS_FAILED;
};

// DepthEstimator (include/depth_estimator.hpp, src/depth_estimator.cpp:175-309) without its worker thread:
// addKeyframe = initializeFilters for the keyframe's features without a point; updateFilters = one
// svo_depth_update over every seed.  Converged seeds come back as (feature, point) candidates in the
// reference's order (Map::addNewCandidate, src/map.cpp:586-593).
class DepthEstimator {
public:
    explicit DepthEstimator(Context& ctx) : m_ctx(ctx) {}
    void addKeyframe(const std::shared_ptr<Frame>& frame, double depthMean, double depthMin);
    std::vector<std::pair<std::shared_ptr<Feature>, std::shared_ptr<Point>>> updateFilters(const std::shared_ptr<Frame>& frame);
    std::size_t numberFilters() const { return m_seeds.size(); }
    const std::vector<svo_depth_seed>& seeds() const { return m_seeds; }

private:
    Context& m_ctx;
    std::vector<std::shared_ptr<Frame>> m_keyframes;  // svo_depth_seed::kf indexes this list
    std::vector<std::shared_ptr<Feature>> m_features; // the feature behind every seed
    std::vector<svo_depth_seed> m_seeds;
};

// Map (include/map.hpp, src/map.cpp:15-634): the reprojection half — reprojectMap (:260-570) as one
// host plan (svo_map_reproject_plan) plus one batched FeatureAlignment(7) launch, addNewCandidate
// (:586-593) and addCandidateToFrame (:595-627) with one launch for every candidate in a free cell.  The
// cell order is a seeded permutation (the reference shuffles with an unseeded std::random_device) or the
// caller's.
class Map {
public:
    Map(Context& ctx, std::shared_ptr<PinholeCamera> camera, int32_t cellSize, uint64_t seed = 0);
    void setCellOrder(const std::vector<int32_t>& order) { m_cellOrders = order; }
    void reprojectMap(const std::shared_ptr<Frame>& refFrame, std::shared_ptr<Frame>& curFrame,
                      std::vector<std::pair<std::shared_ptr<Frame>, int32_t>>& overlapKeyFrames);
    void addNewCandidate(const std::shared_ptr<Feature>& feature, const std::shared_ptr<Point>& point);
    void addCandidateToFrame(std::shared_ptr<Frame>& frame);
    void removeMatchedCandidate();  // src/map.cpp:629-634
    uint32_t m_matches = 0, m_trials = 0;
    std::vector<int32_t> m_cellOrders;
    std::vector<uint8_t> m_cellVisited;  // never cleared, as in the reference
    struct Candidate {
        std::shared_ptr<Feature> feature;
        std::shared_ptr<Point> point;
        bool matched;
    };
    std::vector<Candidate> m_candidates;

private:
    Context& m_ctx;
    std::shared_ptr<PinholeCamera> m_camera;
    int32_t m_cellSize, m_gridCols, m_gridRows;
};

// Trajectory and feature-dump text, through std::ostream like the reference.
namespace utils {
// System::writeInFile (src/system.cpp:635-640): refAbsPose.inverse().matrix3x4() at precision 6
void writeInFile(const Pose& refAbsPose, std::ostream& fileWriter);
// utils::writeAllInfoFile / writeFeaturesInfoFile (src/utils.cpp:62-81)
void writeAllInfoFile(const Frame& refFrame, const Frame& curFrame, std::ostream& fileWriter);
void writeFeaturesInfoFile(const Frame& refFrame, const Frame& curFrame, std::ostream& fileWriter);
}  // namespace utils

}  // namespace svo_amd
