// ref_types.hpp -- test infrastructure: the SHAPES of the reference's types that the INTEGRATION.md adapter
// touches, so that the adapter bodies (tests/cpp/adapter.cpp) compile here, where Eigen, Sophus and OpenCV are
// absent.  Only the members and accessors the adapter uses, with the reference's names and meaning:
//   Frame         include/frame.hpp:198-206   (m_camera, m_absPose, m_imagePyramid, m_features, m_lastKeyframe)
//   Feature       include/feature.hpp:29-38   (m_frame, m_pixelPosition, m_bearingVec, m_point)
//   Point         include/point.hpp:28        (m_position)
//   PinholeCamera include/pinhole_camera.hpp:55-64 (fx, fy, cx, cy, width, height)
//   ImageAlignment include/image_alignment.hpp:15-35, FeatureAlignment include/feature_alignment.hpp:15-31
//   ImagePyramid  include/image_pyramid.hpp:23-149 (the adapter replaces its cv::Mat stacks by one svo_pyramid_set)
// Eigen::Vector2d / Vector3d / Quaterniond and Sophus::SE3d are reduced to what the adapter calls
// (x(), y(), z(), Zero(), data() in Sophus params() order qx qy qz qw tx ty tz).  Not the reference's headers.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "svo_c.h"

namespace Eigen {
struct Vector2d {
    double v[2] = {0, 0};
    Vector2d() = default;
    Vector2d(double a, double b) : v{a, b} {}
    double x() const { return v[0]; }
    double y() const { return v[1]; }
};
struct Vector3d {
    double v[3] = {0, 0, 0};
    Vector3d() = default;
    Vector3d(double a, double b, double c) : v{a, b, c} {}
    double x() const { return v[0]; }
    double y() const { return v[1]; }
    double z() const { return v[2]; }
    static Vector3d Zero() { return {}; }
};
struct Quaterniond {  // Eigen's (w, x, y, z) constructor order
    double w, x, y, z;
    Quaterniond(double w_, double x_, double y_, double z_) : w(w_), x(x_), y(y_), z(z_) {}
};
}  // namespace Eigen

namespace Sophus {
struct SE3d {
    double p[7] = {0, 0, 0, 1, 0, 0, 0};  // params(): qx qy qz qw tx ty tz
    SE3d() = default;
    SE3d(const Eigen::Quaterniond& q, const Eigen::Vector3d& t) : p{q.x, q.y, q.z, q.w, t.x(), t.y(), t.z()} {}
    double* data() { return p; }
    const double* data() const { return p; }
};
}  // namespace Sophus

namespace cv {
constexpr int CV_8UC1 = 0;
struct Size {  // cv::Size(width, height)
    int width = 0, height = 0;
    Size() = default;
    Size(int w, int h) : width(w), height(h) {}
};
struct Mat {  // CV_8UC1, continuous
    int rows = 0, cols = 0;
    std::vector<uint8_t> buf;
    template <class T> const T* ptr() const { return reinterpret_cast<const T*>(buf.data()); }
    template <class T> T* ptr() { return reinterpret_cast<T*>(buf.data()); }
    void create(int r, int c, int /*type: CV_8UC1*/) {
        rows = r;
        cols = c;
        buf.assign((size_t)r * (size_t)c, 0);
    }
    bool empty() const { return buf.empty(); }
    Size size() const { return Size(cols, rows); }
};
}  // namespace cv
using cv::CV_8UC1;

class PinholeCamera {
public:
    PinholeCamera(double fx, double fy, double cx, double cy, int32_t w, int32_t h) : m_fx(fx), m_fy(fy), m_cx(cx), m_cy(cy), m_w(w), m_h(h) {}
    double fx() const { return m_fx; }
    double fy() const { return m_fy; }
    double cx() const { return m_cx; }
    double cy() const { return m_cy; }
    int32_t width() const { return m_w; }
    int32_t height() const { return m_h; }

private:
    double m_fx, m_fy, m_cx, m_cy;
    int32_t m_w, m_h;
};

class ImagePyramid {
public:
    ImagePyramid() = default;
    ImagePyramid(const ImagePyramid&) = delete;  // include/image_pyramid.hpp: copy and move deleted
    ~ImagePyramid();
    void createImagePyramid(const cv::Mat& baseImage, std::size_t levels);
    svo_pyramid_set* set() const { return m_set; }
    // the getters of include/image_pyramid.hpp:75-140 (const forms; the adapter adds the non-const ones)
    const std::vector<cv::Mat>& getAllImages() const;
    const cv::Mat& getImageAtLevel(std::size_t level) const;
    cv::Mat& getImageAtLevel(std::size_t level);
    const cv::Mat& getBaseImage() const;
    const cv::Mat& getBaseGradientImage() const;
    const cv::Mat& getGradientAtLevel(std::size_t level) const;
    cv::Mat& getGradientAtLevel(std::size_t level);
    std::size_t getSizeImagePyramid() const;
    cv::Size getImageSizeAtLevel(std::size_t level) const;
    cv::Size getBaseImageSize() const;

private:
    const cv::Mat& hostLevel(std::size_t level, int32_t gradient) const;
    svo_pyramid_set* m_set = nullptr;  // the adapter's member: the frame's device-resident stacks
    mutable std::vector<cv::Mat> m_hostImages, m_hostGradients;  // host copies the getters fill on demand
    mutable cv::Mat m_none;                                        // what a getter returns on failure (empty)
};

class Frame;
class Point {
public:
    Eigen::Vector3d m_position;
};
class Feature {
public:
    std::shared_ptr<Frame> m_frame;
    Eigen::Vector2d m_pixelPosition;
    Eigen::Vector3d m_bearingVec;
    std::shared_ptr<Point> m_point;
};
class Frame {
public:
    explicit Frame(std::shared_ptr<PinholeCamera> cam) : m_camera(std::move(cam)) {}
    std::size_t numberObservation() const { return m_features.size(); }
    const std::shared_ptr<PinholeCamera> m_camera;
    Sophus::SE3d m_absPose;
    ImagePyramid m_imagePyramid;
    std::vector<std::shared_ptr<Feature>> m_features;
    std::shared_ptr<Frame> m_lastKeyframe;
};

class ImageAlignment {
public:
    ImageAlignment(uint32_t patchSize, int32_t minLevel, int32_t maxLevel, uint32_t)
        : m_patchSize(patchSize), m_minLevel(minLevel), m_maxLevel(maxLevel) {}
    double align(std::shared_ptr<Frame>& refFrame, std::shared_ptr<Frame>& curFrame);

private:
    uint32_t m_patchSize;
    int32_t m_minLevel, m_maxLevel;
};

class FeatureAlignment {
public:
    FeatureAlignment(uint32_t patchSize, int32_t, uint32_t) : m_patchSize(patchSize) {}
    double align(const std::shared_ptr<Feature>& refFeature, const std::shared_ptr<Frame>& curFrame,
                 Eigen::Vector2d& pixelPos);

private:
    uint32_t m_patchSize;
};

// the adapter's context device (tests force an invalid one to check the failure path)
extern int32_t g_svo_device;
