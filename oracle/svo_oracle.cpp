// =====================================================================================================
//  svo_oracle.cpp — CPU restatement of the reference's direct-alignment hot path.
//
//  TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the timed CPU baseline
//  ("cpu_baseline.kind = port").  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
//  leg may load it.  The product (semi-direct-visual-odometry_amd/) never links or calls it.
//
//  It restates, function by function, the behaviour of amin-abouee/semi-direct-visual-odometry
//  (paths relative to the reference root):
//    ImagePyramid ........ src/image_pyramid.cpp:36-52 (cv::pyrDown + Simd::AbsGradientSaturatedSum,
//                          semantics per 3rd_party/simd/include/Simd/SimdLib.h:856-884)
//    ImageAlignment ...... src/image_alignment.cpp:25-387
//    FeatureAlignment .... src/feature_alignment.cpp:25-212
//    Optimizer::optimizeLM src/optimizer.cpp:162-370, tukeyWeighting :485-514, chi2 :470-483
//    algorithm:: ......... bilinear :885-905, median/MAD/sigma :834-872 (src/algorithm.cpp)
//    Frame / camera ...... src/frame.cpp:89-120, src/pinhole_camera.cpp:50-101,163-175
//    Depth filter ........ src/depth_estimator.cpp:192-357, src/algorithm.cpp:335-551,682-709,907-911,
//                          src/mixed_gaussian_filter.cpp:7-24
//
//  Third-party arithmetic restated (not vendored in the reference): Sophus SE3/SO3 (exp, product,
//  inverse, point action), Eigen quaternion->matrix, Eigen LDLT<Lower> with diagonal pivoting and
//  the D^+ pseudo-inverse, OpenCV pyrDown (5x5 binomial, BORDER_REFLECT_101, (s+128)>>8).
//  libstdc++ std::nth_element is used directly (same toolchain as the reference build).
//
//  Numeric conventions: compiled with -ffp-contract=off; every sum of a short vector is evaluated
//  left to right.  The reference's own binary (g++ -march=native) contracts FMAs, so its last
//  bits are not reproducible by anyone; parity is judged with the tolerances in DESIGN.md.
// =====================================================================================================
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <iomanip>
#include <sstream>
#include <string>
#include <limits>
#include <pthread.h>
#include <sched.h>
#include <thread>
#include <vector>

namespace oracle {

// ------------------------------------------------------------------ small linear algebra
struct V3 { double x, y, z; };
struct V2 { double x, y; };
static inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 scl(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline double norm(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

// Unit quaternion, Eigen coefficient order (x, y, z, w); Sophus params() = (qx,qy,qz,qw,tx,ty,tz).
struct Q { double x, y, z, w; };
struct SE3 { Q q; V3 t; };

// Eigen QuaternionBase::_transformVector (used by Sophus SO3 * point)
static inline V3 qrot(const Q& q, V3 v) {
    V3 qv{q.x, q.y, q.z};
    V3 uv = cross(qv, v);
    uv = add(uv, uv);
    return add(add(v, scl(uv, q.w)), cross(qv, uv));
}
static inline Q qconj(const Q& q) { return {-q.x, -q.y, -q.z, q.w}; }
// Sophus SO3 product (explicit Hamilton product) followed by the near-unit renormalisation
// (factor 2/(1+|q|^2) whenever |q|^2 != 1).
static inline Q qmul(const Q& a, const Q& b) {
    Q r{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
        a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
        a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x,
        a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
    double n2 = r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
    if (n2 != 1.0) {
        double f = 2.0 / (1.0 + n2);
        r.x *= f; r.y *= f; r.z *= f; r.w *= f;
    }
    return r;
}
static inline V3 act(const SE3& T, V3 p) { return add(qrot(T.q, p), T.t); }
static inline SE3 inverse(const SE3& T) {
    Q qi = qconj(T.q);
    return {qi, qrot(qi, scl(T.t, -1.0))};
}
static inline SE3 compose(const SE3& a, const SE3& b) { return {qmul(a.q, b.q), add(a.t, qrot(a.q, b.t))}; }
// Eigen QuaternionBase::toRotationMatrix, row-major R[3][3]
static inline void rotmat(const Q& q, double R[3][3]) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1.0 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
    R[1][0] = txy + twz; R[1][1] = 1.0 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1.0 - (txx + tyy);
}
// Frame::cameraInWorld  (src/frame.cpp:116-120):  C = -R^T t
static inline V3 camera_in_world(const SE3& T) {
    double R[3][3];
    rotmat(T.q, R);
    V3 c;
    c.x = (-R[0][0]) * T.t.x + (-R[1][0]) * T.t.y + (-R[2][0]) * T.t.z;
    c.y = (-R[0][1]) * T.t.x + (-R[1][1]) * T.t.y + (-R[2][1]) * T.t.z;
    c.z = (-R[0][2]) * T.t.x + (-R[1][2]) * T.t.y + (-R[2][2]) * T.t.z;
    return c;
}
// Sophus SE3::exp, tangent = (upsilon; omega), Constants<double>::epsilon() = 1e-10
static SE3 se3_exp(const double a[6]) {
    const V3 up{a[0], a[1], a[2]};
    const V3 om{a[3], a[4], a[5]};
    const double eps = 1e-10;
    const double theta_sq = om.x * om.x + om.y * om.y + om.z * om.z;
    double theta, imag, real;
    if (theta_sq < eps * eps) {
        theta = 0.0;
        const double theta_po4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
        theta = std::sqrt(theta_sq);
        const double half = 0.5 * theta;
        imag = std::sin(half) / theta;
        real = std::cos(half);
    }
    Q q{imag * om.x, imag * om.y, imag * om.z, real};
    // Omega = hat(omega), Omega^2
    const double W[3][3] = {{0.0, -om.z, om.y}, {om.z, 0.0, -om.x}, {-om.y, om.x, 0.0}};
    double W2[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) W2[i][j] = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
    double V[3][3];
    if (theta < eps) {
        rotmat(q, V);
    } else {
        const double c1 = (1.0 - std::cos(theta)) / (theta_sq);
        const double c2 = (theta - std::sin(theta)) / (theta_sq * theta);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) V[i][j] = ((i == j ? 1.0 : 0.0) + c1 * W[i][j]) + c2 * W2[i][j];
    }
    V3 t{V[0][0] * up.x + V[0][1] * up.y + V[0][2] * up.z, V[1][0] * up.x + V[1][1] * up.y + V[1][2] * up.z,
         V[2][0] * up.x + V[2][1] * up.y + V[2][2] * up.z};
    return {q, t};
}

// Eigen LDLT<MatrixXd, Lower>::compute + solve for an n x n system (n <= 6).
// Pivot = first index of max |diag| in the trailing block; D^+ zeroes |d| <= DBL_MIN.
static void ldlt_solve(int n, const double* Hin, const double* b, double* x) {
    double A[36];
    std::memcpy(A, Hin, sizeof(double) * n * n);  // row-major, only the lower triangle is read
    int perm[6];
    double tmp[6];
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double best = std::fabs(A[k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = std::fabs(A[i * n + i]);
            if (v > best) { best = v; piv = i; }
        }
        perm[k] = piv;
        if (piv != k) {
            for (int j = 0; j < k; ++j) std::swap(A[k * n + j], A[piv * n + j]);
            for (int i = piv + 1; i < n; ++i) std::swap(A[i * n + k], A[i * n + piv]);
            std::swap(A[k * n + k], A[piv * n + piv]);
            for (int i = k + 1; i < piv; ++i) {
                double t = A[i * n + k];
                A[i * n + k] = A[piv * n + i];
                A[piv * n + i] = t;
            }
        }
        if (k > 0) {
            for (int j = 0; j < k; ++j) tmp[j] = A[j * n + j] * A[k * n + j];
            double s = 0.0;
            for (int j = 0; j < k; ++j) s += A[k * n + j] * tmp[j];
            A[k * n + k] -= s;
            for (int i = k + 1; i < n; ++i) {
                double si = 0.0;
                for (int j = 0; j < k; ++j) si += A[i * n + j] * tmp[j];
                A[i * n + k] -= si;
            }
        }
        const double akk = A[k * n + k];
        const bool valid = std::fabs(akk) > 0.0;
        if (k == 0 && !valid) {  // whole diagonal zero: identity transpositions, nothing else
            for (int j = 0; j < n; ++j) perm[j] = j;
            break;
        }
        if (valid)
            for (int i = k + 1; i < n; ++i) A[i * n + k] /= akk;
    }
    for (int i = 0; i < n; ++i) x[i] = b[i];
    for (int k = 0; k < n; ++k) std::swap(x[k], x[perm[k]]);
    for (int i = 0; i < n; ++i) {  // L unit lower
        double s = x[i];
        for (int j = 0; j < i; ++j) s -= A[i * n + j] * x[j];
        x[i] = s;
    }
    for (int i = 0; i < n; ++i) {
        const double d = A[i * n + i];
        if (std::fabs(d) > DBL_MIN) x[i] /= d;
        else x[i] = 0.0;
    }
    for (int i = n - 1; i >= 0; --i) {  // L^T
        double s = x[i];
        for (int j = i + 1; j < n; ++j) s -= A[j * n + i] * x[j];
        x[i] = s;
    }
    for (int k = n - 1; k >= 0; --k) std::swap(x[k], x[perm[k]]);
}

// ------------------------------------------------------------------ camera  (src/pinhole_camera.cpp)
struct Camera {
    double fx, fy, cx, cy;
    int32_t width, height;
    V2 project2d(V3 p) const { return {fx * (p.x / p.z) + cx, fy * (p.y / p.z) + cy}; }  // :53-57 (d = 0)
    V3 inverse_project2d(double u, double v) const {                                     // :84-100
        V3 p{(u - cx) / fx, (v - cy) / fy, 1.0};
        return scl(p, 1.0 / norm(p));
    }
    bool is_in_frame(V2 p, double b) const {  // :163-168
        return p.x >= b && p.y >= b && p.x < width - b && p.y < height - b;
    }
};

// ------------------------------------------------------------------ image pyramid
struct LevelDims { int32_t w[16], h[16]; int64_t off[16]; int64_t total; };
static LevelDims level_dims(int32_t w, int32_t h, int32_t levels) {
    LevelDims d{};
    int64_t off = 0;
    for (int l = 0; l < levels; ++l) {
        d.w[l] = w; d.h[l] = h; d.off[l] = off;
        off += (int64_t)w * h;
        w = (w + 1) / 2;
        h = (h + 1) / 2;
    }
    d.total = off;
    return d;
}
static inline int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}
// cv::pyrDown, CV_8UC1, default dst size, BORDER_REFLECT_101
static void pyr_down(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    static const int k[5] = {1, 4, 6, 4, 1};
    for (int y = 0; y < dh; ++y)
        for (int x = 0; x < dw; ++x) {
            int s = 0;
            for (int i = 0; i < 5; ++i) {
                const uint8_t* row = src + (size_t)reflect101(2 * y + i - 2, sh) * sw;
                int rs = 0;
                for (int j = 0; j < 5; ++j) rs += k[j] * row[reflect101(2 * x + j - 2, sw)];
                s += k[i] * rs;
            }
            dst[(size_t)y * dw + x] = (uint8_t)((s + 128) >> 8);
        }
}
// Simd::AbsGradientSaturatedSum (SimdLib.h:856-884): border pixels 0
static void abs_gradient_saturated_sum(const uint8_t* src, int w, int h, uint8_t* dst) {
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            if (y == 0 || x == 0 || y == h - 1 || x == w - 1) { dst[(size_t)y * w + x] = 0; continue; }
            int dx = std::abs((int)src[(size_t)y * w + x + 1] - (int)src[(size_t)y * w + x - 1]);
            int dy = std::abs((int)src[(size_t)(y + 1) * w + x] - (int)src[(size_t)(y - 1) * w + x]);
            dst[(size_t)y * w + x] = (uint8_t)std::min(dx + dy, 255);
        }
}
// ImagePyramid::createImagePyramid (src/image_pyramid.cpp:36-52): level 0 = input; the gradient
// stack is pyrDown of the L0 gradient (not the gradient of each level).
static void build_pyramid(const uint8_t* img, int w, int h, int levels, uint8_t* out_img, uint8_t* out_grad) {
    LevelDims d = level_dims(w, h, levels);
    std::memcpy(out_img, img, (size_t)w * h);
    if (out_grad) abs_gradient_saturated_sum(img, w, h, out_grad);
    for (int l = 1; l < levels; ++l) {
        pyr_down(out_img + d.off[l - 1], d.w[l - 1], d.h[l - 1], out_img + d.off[l], d.w[l], d.h[l]);
        if (out_grad)
            pyr_down(out_grad + d.off[l - 1], d.w[l - 1], d.h[l - 1], out_grad + d.off[l], d.w[l], d.h[l]);
    }
}

struct Image { const uint8_t* p; int32_t w, h; uint8_t at(int y, int x) const { return p[(size_t)y * w + x]; } };

// algorithm::bilinearInterpolationDouble (src/algorithm.cpp:896-905)
static inline double bilinear_d(const Image& im, double x, double y) {
    const int32_t x1 = (int32_t)x, y1 = (int32_t)y, x2 = x1 + 1, y2 = y1 + 1;
    const double a = (x2 - x) * im.at(y1, x1) + (x - x1) * im.at(y1, x2);
    const double b = (x2 - x) * im.at(y2, x1) + (x - x1) * im.at(y2, x2);
    return (y2 - y) * a + (y - y1) * b;
}
// algorithm::bilinearInterpolation, float flavour (src/algorithm.cpp:885-894)
static inline float bilinear_f(const Image& im, double x, double y) {
    const int x1 = (int)x, y1 = (int)y, x2 = x1 + 1, y2 = y1 + 1;
    const float a = (float)((x2 - x) * im.at(y1, x1) + (x - x1) * im.at(y1, x2));
    const float b = (float)((x2 - x) * im.at(y2, x1) + (x - x1) * im.at(y2, x2));
    return (float)((y2 - y) * (double)a + (y - y1) * (double)b);
}

// ------------------------------------------------------------------ robust statistics
// median_mode 0: the reference (std::nth_element on a copy of the FULL vector, odd/even decided by
// the total length; the even case reads vec[mid-1] from the libstdc++ post-partition state,
// src/algorithm.cpp:834-853).  median_mode 1: true order statistics (what a radix select returns).
// mid == 0 with an even length reads vec[-1] in the reference (UB); both modes use vec[mid] there.
static double compute_median(const std::vector<double>& in, uint32_t n_valid, int mode) {
    std::vector<double> v(in);
    if (v.empty()) return std::numeric_limits<double>::quiet_NaN();
    const uint32_t mid = n_valid / 2;
    if (mode == 0) {
        std::nth_element(v.begin(), v.begin() + mid, v.end());
        if (v.size() % 2 != 0 || mid == 0) return v[mid];
        return (v[mid - 1] + v[mid]) / 2.0;
    }
    std::nth_element(v.begin(), v.begin() + mid, v.end());
    const double hi = v[mid];
    if (v.size() % 2 != 0 || mid == 0) return hi;
    const double lo = *std::max_element(v.begin(), v.begin() + mid);
    return (lo + hi) / 2.0;
}
static double compute_mad(const std::vector<double>& in, uint32_t n_valid, int mode, double* med_out) {
    const double med = compute_median(in, n_valid, mode);
    if (med_out) *med_out = med;
    std::vector<double> diff(in.size());
    for (size_t i = 0; i < in.size(); ++i) diff[i] = std::fabs(in[i] - med);
    return compute_median(diff, n_valid, mode);
}

// ------------------------------------------------------------------ Optimizer (src/optimizer.cpp)
enum Status : int32_t {
    Success = 0, Max_Coff_Dx = 1, Non_In_Dx = 2, Small_Step_Size = 3, Lambda_Value = 4, Norm_Inf_Diff = 5,
    Non_Suff_Points = 6, Increase_Chi_Squred_Error = 7, Small_Chi_Squred_Error = 8, Failed = 9
};

struct LevelTrace {  // per-level debug record (mirrors svo_level_debug in include/svo_c.h)
    int32_t level, n_ref_vis, n_vis, status;
    double median, mad, sigma, chi2, lambda, err;
    double H[36], g[6], dx[6];
};

// test infrastructure: when set (oracle_image_align_vectors), each level's tukey_weighting appends the residual vector it
// sees (the reference's feature-major slots, DBL_MAX for an invisible slot) and its n_valid
static thread_local double* g_vec_dump = nullptr;
static thread_local int64_t g_vec_cap = 0, g_vec_used = 0;
static thread_local uint32_t* g_vec_nvalid = nullptr;
static thread_local int32_t g_vec_levels = 0;

struct Optimizer {
    int nu;                       // number of unknowns
    int median_mode = 0;
    std::vector<double> J;        // M x nu, row-major
    std::vector<double> r, w;
    std::vector<uint8_t> vis;
    double H[36], g[6], dx[6];
    LevelTrace* trace = nullptr;
    explicit Optimizer(int n) : nu(n) {}

    void init_parameters(size_t M) {  // :378-385
        J.assign(M * nu, 0.0);
        r.resize(M);
        w.resize(M);
        vis.resize(M);
    }
    void reset_all() {  // :387-396 (Jacobian not cleared)
        std::fill(r.begin(), r.end(), std::numeric_limits<double>::max());
        std::fill(w.begin(), w.end(), 0.0);
        std::fill(vis.begin(), vis.end(), 0);
    }
    void tukey_weighting(uint32_t n_valid) {  // :485-514
        if (g_vec_dump && g_vec_used + (int64_t)r.size() <= g_vec_cap) {
            std::memcpy(g_vec_dump + g_vec_used, r.data(), r.size() * sizeof(double));
            g_vec_used += (int64_t)r.size();
            g_vec_nvalid[g_vec_levels++] = n_valid;
        }
        double med = 0.0;
        const double mad = compute_mad(r, n_valid, median_mode, &med);
        double sigma = 1.482602218505602 * mad;
        if (trace) { trace->median = med; trace->mad = mad; }
        if (sigma <= std::numeric_limits<double>::epsilon()) sigma = std::numeric_limits<double>::epsilon();
        if (trace) trace->sigma = sigma;
        const double c = 4.6851 * sigma;
        const double c2 = c * c;
        for (size_t i = 0; i < vis.size(); ++i)
            if (vis[i]) {
                const double a = std::fabs(r[i]);
                if (a <= c) {
                    const double t = 1.0 - (r[i] * r[i]) / c2;
                    w[i] = t * t;
                } else {
                    w[i] = 0.0;
                }
            }
    }
    double chi2() const {  // :470-483
        double s = 0.0;
        for (size_t i = 0; i < vis.size(); ++i)
            if (vis[i]) s += r[i] * r[i] * w[i];
        return s;
    }
    void normal_equations() {  // :279-280, H = J^T W J, g = J^T W r (row order)
        std::fill(H, H + 36, 0.0);
        std::fill(g, g + 6, 0.0);
        const size_t M = r.size();
        for (size_t k = 0; k < M; ++k) {
            const double wk = w[k];
            if (wk == 0.0) continue;  // exact-zero rows add exact zeros (0*DBL_MAX = 0 in the reference)
            const double* Jk = &J[k * nu];
            for (int i = 0; i < nu; ++i) {
                const double jw = Jk[i] * wk;
                for (int j = 0; j < nu; ++j) H[i * nu + j] += jw * Jk[j];
                g[i] += jw * r[k];
            }
        }
    }
    // Optimizer::optimizeLM<T> (:162-370).  The loop is restated in full; with normDiffPose fixed at
    // 0 (:186, :327 commented out) it always leaves after the first damped step (:328).
    template <typename T>
    std::pair<int32_t, double> optimize_lm(T& params, const std::function<uint32_t(T&)>& residual_fn,
                                           const std::function<void(T&, const double*)>& update_fn,
                                           const std::function<void(T&)>& jacobian_fn = nullptr) {
        const size_t M = r.size();
        int32_t status = Failed;
        if (M < (size_t)nu) return {Non_Suff_Points, -1.0};
        uint32_t cur_iter = 0;
        const uint32_t max_iter = 20;
        double step = 0.0, norm_diff = 0.0, chi = 0.0, pre_chi = 0.0;
        uint32_t n_proj = 0, pre_n_proj = 0;
        double lambda = 1e-2, nuf = 2.0;
        reset_all();
        if (jacobian_fn) std::fill(J.begin(), J.end(), 0.0);  // resetAllParameters(computeJacobian = true)
        n_proj = residual_fn(params);
        tukey_weighting(n_proj);
        chi = chi2();
        T pre_params = params;
        std::vector<double> pre_r, pre_w;
        std::vector<uint8_t> pre_vis;
        bool success_iter = true;
        while (cur_iter < max_iter) {
            if (success_iter) {
                pre_params = params; pre_chi = chi; pre_r = r; pre_w = w; pre_vis = vis; pre_n_proj = n_proj;
                status = Success;
            }
            if (jacobian_fn) jacobian_fn(params);  // :242-243
            normal_equations();
            if (cur_iter == 0) {
                double mx = H[0];
                for (int i = 1; i < nu; ++i) mx = std::max(mx, H[i * nu + i]);
                lambda *= mx;
            }
            for (int i = 0; i < nu; ++i) H[i * nu + i] += lambda;
            if (trace) {
                std::memcpy(trace->H, H, sizeof(double) * nu * nu);
                std::memcpy(trace->g, g, sizeof(double) * nu);
                trace->lambda = lambda;
            }
            ldlt_solve(nu, H, g, dx);
            if (trace) std::memcpy(trace->dx, dx, sizeof(double) * nu);
            update_fn(params, dx);
            bool big = false, nan = false;
            for (int i = 0; i < nu; ++i) { big |= dx[i] > 1e3; nan |= std::isnan(dx[i]); }
            if (big) { status = Max_Coff_Dx; break; }
            if (nan) { status = Non_In_Dx; break; }
            step = 0.0;
            for (int i = 0; i < nu; ++i) step += dx[i] * dx[i];
            if (step < 1e-16 || lambda >= 1e14 || lambda <= 1e-14 || norm_diff < 1e-3) {
                status = step < 1e-16 ? Small_Step_Size : status;
                status = std::fabs(lambda) >= 1e14 ? Lambda_Value : status;
                break;
            }
            // unreachable with normDiffPose == 0; kept for completeness of the restatement
            std::fill(r.begin(), r.end(), std::numeric_limits<double>::max());
            std::fill(w.begin(), w.end(), 0.0);
            std::fill(vis.begin(), vis.end(), 0);
            n_proj = residual_fn(params);
            tukey_weighting(n_proj);
            chi = chi2();
            const double rho = pre_chi - chi;
            if (rho > 0.0) {
                lambda *= std::max(1.0 / 3.0, 1.0 - std::pow(2 * rho - 1, 3));
                nuf = 2.0;
                success_iter = true;
            } else {
                lambda *= nuf;
                nuf *= 2;
                success_iter = false;
                chi = pre_chi; params = pre_params; r = pre_r; w = pre_w; vis = pre_vis; n_proj = pre_n_proj;
            }
            ++cur_iter;
        }
        const double rmse = std::sqrt(chi / n_proj);
        if (trace) { trace->chi2 = chi; trace->n_vis = (int32_t)n_proj; trace->status = status; trace->err = rmse; }
        return {status, rmse};
    }
};

// ------------------------------------------------------------------ frames & features
struct Frame;
struct Feature {
    V2 px;
    V3 bearing;
    bool has_point;
    V3 point;
    const Frame* frame;
};
struct Frame {
    SE3 pose;
    const uint8_t* pyr;   // packed image stack
    const uint8_t* grad;  // packed gradient stack (may be null when unused)
    LevelDims dims;
    std::vector<Feature> features;
    const Frame* last_kf;
    Image level(int l) const { return {pyr + dims.off[l], dims.w[l], dims.h[l]}; }
    Image grad_level(int l) const { return {grad + dims.off[l], dims.w[l], dims.h[l]}; }
    V3 camera2world(V3 p) const { return act(inverse(pose), p); }  // src/frame.cpp:94-97
};

// ------------------------------------------------------------------ ImageAlignment (src/image_alignment.cpp)
struct ImageAlignment {
    uint32_t half, area;  // area = (2h+1)^2 (loop footprint; = p^2 for odd p)
    int32_t min_level, max_level;
    Optimizer opt;
    std::vector<double> ref_patches;  // numFeatures x area
    std::vector<uint8_t> ref_vis;
    const Camera* cam;
    ImageAlignment(uint32_t patch, int32_t minl, int32_t maxl, const Camera* c)
        : half(patch / 2), area((2 * (patch / 2) + 1) * (2 * (patch / 2) + 1)), min_level(minl), max_level(maxl), opt(6), cam(c) {}

    static void image_jac(double J[2][6], V3 p, double fx, double fy) {  // :194-248
        const double x = p.x, y = p.y, z = p.z, x2 = x * x, y2 = y * y, z2 = z * z;
        J[0][0] = fx / z; J[0][1] = 0.0; J[0][2] = -(fx * x) / z2; J[0][3] = -(fx * x * y) / z2;
        J[0][4] = (fx * x2) / z2 + fx; J[0][5] = -(fx * y) / z;
        J[1][0] = 0.0; J[1][1] = fy / z; J[1][2] = -(fy * y) / z2; J[1][3] = -(fy * y2) / z2 - fy;
        J[1][4] = (fy * x * y) / z2; J[1][5] = (fy * x) / z;
    }
    bool jac_single(const Feature& f, const Image& im, int32_t border, V3 C, double scale, double fx, double fy, uint32_t& cnt) {
        const double u = f.px.x * scale, v = f.px.y * scale;  // :138-149
        const int32_t ui = (int32_t)std::floor(u), vi = (int32_t)std::floor(v);
        if ((ui - border) < 0 || (vi - border) < 0 || (ui + border) >= im.w || (vi + border) >= im.h) return false;
        ref_vis[cnt] = 1;
        const double depth = norm(sub(f.point, C));  // :153-155
        const V3 pc = scl(f.bearing, depth);
        const V3 pw = f.frame->camera2world(pc);
        double Jimg[2][6];
        image_jac(Jimg, pw, fx, fy);
        uint32_t k = 0;
        const int32_t h = (int32_t)half;
        for (int32_t y = -h; y <= h; ++y)
            for (int32_t x = -h; x <= h; ++x, ++k) {  // :169-189
                const double row = v + y, col = u + x;
                ref_patches[(size_t)cnt * area + k] = bilinear_d(im, col, row);
                const double dx = 0.5 * (bilinear_d(im, col + 1, row) - bilinear_d(im, col - 1, row));
                const double dy = 0.5 * (bilinear_d(im, col, row + 1) - bilinear_d(im, col, row - 1));
                double* Jr = &opt.J[((size_t)cnt * area + k) * 6];
                for (int j = 0; j < 6; ++j) Jr[j] = dx * Jimg[0][j] + dy * Jimg[1][j];
            }
        ++cnt;
        return true;
    }
    void compute_jacobian(const Frame& ref, int level) {  // :69-126
        std::fill(ref_vis.begin(), ref_vis.end(), 0);
        std::fill(ref_patches.begin(), ref_patches.end(), 0.0);
        const int32_t border = (int32_t)half + 2;
        const double dom = (double)(1 << level), scale = 1.0 / dom;
        const double fx = cam->fx / dom, fy = cam->fy / dom;
        uint32_t cnt = 0;
        const Image ri = ref.level(level);
        const V3 rc = camera_in_world(ref.pose);
        for (const auto& f : ref.features) {
            if (!f.has_point) { ++cnt; continue; }
            if (!jac_single(f, ri, border, rc, scale, fx, fy, cnt)) { ++cnt; continue; }
        }
        const Frame& kf = *ref.last_kf;
        const Image ki = kf.level(level);
        const V3 kc = camera_in_world(kf.pose);
        for (const auto& f : kf.features) {
            if (!f.has_point) { ++cnt; continue; }
            if (!jac_single(f, ki, border, kc, scale, fx, fy, cnt)) { ++cnt; continue; }
        }
    }
    bool res_single(const Feature& f, const Image& im, const SE3& pose, int32_t border, V3 C, double scale, uint32_t& cnt, uint32_t& n) {
        const double depth = norm(sub(f.point, C));  // :320-340
        const V3 pc = scl(f.bearing, depth);
        const V3 pw = f.frame->camera2world(pc);
        const V3 cp = act(pose, pw);
        const V2 uv = cam->project2d(cp);
        const double u = uv.x * scale, v = uv.y * scale;
        const int32_t ui = (int32_t)std::floor(u), vi = (int32_t)std::floor(v);
        if (!f.has_point || (ui - border) < 0 || (vi - border) < 0 || (ui + border) >= im.w || (vi + border) >= im.h) return false;
        uint32_t k = 0;
        const int32_t h = (int32_t)half;
        for (int32_t y = -h; y <= h; ++y)
            for (int32_t x = -h; x <= h; ++x, ++k, ++n) {
                const double cur = bilinear_d(im, u + x, v + y);
                const size_t idx = (size_t)cnt * area + k;
                opt.r[idx] = cur - ref_patches[idx];  // :359
                opt.vis[idx] = 1;
            }
        ++cnt;
        return true;
    }
    uint32_t compute_residuals(const Frame& ref, const Frame& cur, int level, const SE3& pose) {  // :251-308
        const Image ci = cur.level(level);
        const int32_t border = (int32_t)half + 2;
        const double scale = 1.0 / (double)(1 << level);
        const V3 rc = camera_in_world(ref.pose);
        uint32_t cnt = 0, n = 0;
        for (const auto& f : ref.features) {
            if (!ref_vis[cnt]) { ++cnt; continue; }
            if (!res_single(f, ci, pose, border, rc, scale, cnt, n)) { ++cnt; continue; }
        }
        const Frame& kf = *ref.last_kf;
        const V3 kc = camera_in_world(kf.pose);
        for (const auto& f : kf.features) {
            if (!ref_vis[cnt]) { ++cnt; continue; }
            if (!res_single(f, ci, pose, border, kc, scale, cnt, n)) { ++cnt; continue; }
        }
        return n;
    }
    double align(const Frame& ref, Frame& cur, int32_t* status_out, LevelTrace* traces) {  // :25-67
        if (ref.features.empty()) { if (status_out) *status_out = Failed; return 0.0; }
        const size_t nf = ref.features.size() + ref.last_kf->features.size();
        const size_t M = nf * area;
        ref_patches.assign(nf * area, 0.0);
        opt.init_parameters(M);
        ref_vis.assign(nf, 0);
        double err = 0.0;
        int32_t st = Failed;
        for (int32_t level = max_level; level >= min_level; --level) {
            compute_jacobian(ref, level);
            LevelTrace* tr = traces ? &traces[level] : nullptr;
            if (tr) {
                std::memset(tr, 0, sizeof(*tr));
                tr->level = level;
                int32_t c = 0;
                for (uint8_t b : ref_vis) c += b;
                tr->n_ref_vis = c;
            }
            opt.trace = tr;
            auto resid = [&](SE3& p) -> uint32_t { return compute_residuals(ref, cur, level, p); };
            auto upd = [&](SE3& p, const double* dx) {  // :372-380  pose = pose * exp(-dx)
                double m[6];
                for (int i = 0; i < 6; ++i) m[i] = -dx[i];
                p = compose(p, se3_exp(m));
            };
            auto res = opt.optimize_lm<SE3>(cur.pose, resid, upd);
            st = res.first;
            err = res.second;
            opt.trace = nullptr;
        }
        if (status_out) *status_out = st;
        return err;
    }
};

// ------------------------------------------------------------------ FeatureAlignment (src/feature_alignment.cpp)
struct FlowParams { double x, y, z; };
struct FeatureAlignment {
    uint32_t half, area;
    Optimizer opt;
    std::vector<double> ref_patch;
    const Camera* cam;
    FeatureAlignment(uint32_t patch, const Camera* c)
        : half(patch / 2), area((2 * (patch / 2) + 1) * (2 * (patch / 2) + 1)), opt(3), cam(c) {}
    void compute_jacobian(const Image& g, V2 px) {  // :64-110
        std::fill(ref_patch.begin(), ref_patch.end(), 0.0);
        const double border = half + 2;
        if (!cam->is_in_frame(px, border)) return;
        uint32_t k = 0;
        const int32_t h = (int32_t)half;
        for (int32_t y = -h; y <= h; ++y)
            for (int32_t x = -h; x <= h; ++x, ++k) {
                const double row = px.y + y, col = px.x + x;
                ref_patch[k] = bilinear_f(g, col, row);
                const double dx = 0.5 * (bilinear_f(g, col + 1, row) - bilinear_f(g, col - 1, row));
                const double dy = 0.5 * (bilinear_f(g, col, row + 1) - bilinear_f(g, col, row - 1));
                opt.J[k * 3 + 0] = dx; opt.J[k * 3 + 1] = dy; opt.J[k * 3 + 2] = 1.0;
            }
    }
    uint32_t compute_residuals(const Image& g, const FlowParams& p) {  // :113-168
        const double border = half + 2;
        if (!cam->is_in_frame({p.x, p.y}, border)) return 0;
        uint32_t n = 0, k = 0;
        const int32_t h = (int32_t)half;
        for (int32_t y = -h; y <= h; ++y)
            for (int32_t x = -h; x <= h; ++x, ++k, ++n) {
                const double cur = bilinear_f(g, p.x + x, p.y + y);
                opt.r[k] = -(cur - ref_patch[k] + p.z);
                opt.vis[k] = 1;
            }
        return n;
    }
    double align(const Image& ref_grad, V2 ref_px, const Image& cur_grad, V2& px, int32_t* status_out) {  // :25-62
        ref_patch.assign(area, 0.0);
        opt.init_parameters(area);
        FlowParams flow{px.x, px.y, 0.0};
        compute_jacobian(ref_grad, ref_px);
        auto resid = [&](FlowParams& p) -> uint32_t { return compute_residuals(cur_grad, p); };
        auto upd = [&](FlowParams& p, const double* dx) { p.x += dx[0]; p.y += dx[1]; p.z += dx[2]; };
        auto res = opt.optimize_lm<FlowParams>(flow, resid, upd);
        px.x = flow.x;
        px.y = flow.y;
        if (status_out) *status_out = res.first;
        return res.second;
    }
};

// ------------------------------------------------------------------ depth filter (config 5)
// DepthEstimator::updateFilters (src/depth_estimator.cpp:192-309) with its helpers.  Seeds are the
// MixedGaussianFilter state (include/mixed_gaussian_filter.hpp:28-38) plus the feature they refine.
struct DepthSeed {
    double a, b, mu, sigma, var, max_depth;
    double px[2];
    double bearing[3];
    int32_t kf, valid;
};
enum DepthOutcome : int32_t {  // per seed, for the parity tests (no reference counterpart)
    kDepthRejected = 0,        // pointInCurCamera.z < 0 or outside the cur image (:229-237): invalid
    kDepthNoMatch = 1,         // matchEpipolarConstraint failed: b += 1 (:252-258)
    kDepthUpdated = 2,         // Vogiatzis update, still a seed (:261-266)
    kDepthConverged = 3,       // sqrt(var) * 10 < maxDepth: candidate point emitted, seed invalid (:281-291)
    kDepthNaN = 4              // inverse depth NaN (:292-297): invalid
};

// Frame::image2camera (src/frame.cpp:104-107): inverseProject2d(px) * depth
static V3 image2camera(const Camera& cam, V2 px, double depth) { return scl(cam.inverse_project2d(px.x, px.y), depth); }
// algorithm::computeRelativePose (src/algorithm.cpp:705-709): T_cur * T_ref^-1
static SE3 relative_pose(const SE3& ref, const SE3& cur) { return compose(cur, inverse(ref)); }

// algorithm::getAffineWarp (src/algorithm.cpp:335-367); A row-major: A[0] = (0,0), A[1] = (0,1) ...
static void affine_warp(const Camera& cam, const SE3& rel, V2 px, uint32_t patch, double depth, double A[4]) {
    const uint32_t half = patch / 2;
    const V3 c = image2camera(cam, px, depth);
    const V3 du = image2camera(cam, {px.x + (double)half, px.y + 0.0}, depth);
    const V3 dv = image2camera(cam, {px.x + 0.0, px.y + (double)half}, depth);
    const V2 cc = cam.project2d(act(rel, c)), uc = cam.project2d(act(rel, du)), vc = cam.project2d(act(rel, dv));
    A[0] = (uc.x - cc.x) / (double)half; A[2] = (uc.y - cc.y) / (double)half;  // column 0 = duDiff / h
    A[1] = (vc.x - cc.x) / (double)half; A[3] = (vc.y - cc.y) / (double)half;  // column 1 = dvDiff / h
}
// algorithm::applyAffineWarp (src/algorithm.cpp:369-394): samples only if the location is inside the
// frame by ceil(max |A (h, h)|) + 2 px; otherwise `data` keeps its previous contents
static void apply_affine_warp(const Camera& cam, const Image& im, V2 loc, int32_t half, const double A[4], uint8_t* data) {
    const double bx = A[0] * half + A[1] * half, by = A[2] * half + A[3] * half;
    const double maxb = std::ceil(std::max(std::fabs(bx), std::fabs(by))) + 2;
    if (!cam.is_in_frame(loc, maxb)) return;
    uint32_t idx = 0;
    for (int32_t i = -half; i <= half; ++i)
        for (int32_t j = -half; j <= half; ++j) {
            const double x = loc.x + (A[0] * j + A[1] * i), y = loc.y + (A[2] * j + A[3] * i);
            data[idx++] = (uint8_t)bilinear_f(im, x, y);
        }
}
// algorithm::computeScore (src/algorithm.cpp:396-410): ZSAD with Eigen's uint8 mean (sum wraps mod 256,
// then uint8 / uint8)
static double compute_score(const uint8_t* ref, const uint8_t* cur, int n) {
    uint8_t sr = 0, sc = 0;
    for (int i = 0; i < n; ++i) { sr = (uint8_t)(sr + ref[i]); sc = (uint8_t)(sc + cur[i]); }
    const double mr = (double)(uint8_t)(sr / (uint8_t)n), mc = (double)(uint8_t)(sc / (uint8_t)n);
    double sum = 0.0;
    for (int i = 0; i < n; ++i) sum += std::fabs((ref[i] - mr) - (cur[i] - mc));
    return sum;
}
// algorithm::depthFromTriangulation (src/algorithm.cpp:682-703), Eigen evaluation order
static bool depth_from_triangulation(const SE3& rel, V3 fr, V3 fc, double& depth) {
    double R[3][3];
    rotmat(rel.q, R);
    const V3 rf{R[0][0] * fr.x + R[0][1] * fr.y + R[0][2] * fr.z, R[1][0] * fr.x + R[1][1] * fr.y + R[1][2] * fr.z,
                R[2][0] * fr.x + R[2][1] * fr.y + R[2][2] * fr.z};
    const double A[3][2] = {{rf.x, -fc.x}, {rf.y, -fc.y}, {rf.z, -fc.z}};
    double M[2][2];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) M[i][j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j];
    const double det = M[0][0] * M[1][1] - M[1][0] * M[0][1];
    if (det < 0.000001) return false;
    const double invdet = 1.0 / det;
    const double Inv[2][2] = {{M[1][1] * invdet, -M[0][1] * invdet}, {-M[1][0] * invdet, M[0][0] * invdet}};
    const double t[3] = {rel.t.x, rel.t.y, rel.t.z};
    double tmp[2][3];  // (-Inv) * A^T
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 3; ++k) tmp[i][k] = (-Inv[i][0]) * A[k][0] + (-Inv[i][1]) * A[k][1];
    const double d0 = tmp[0][0] * t[0] + tmp[0][1] * t[1] + tmp[0][2] * t[2];
    depth = std::fabs(d0);
    return true;
}
static V2 clamp_to_image(V2 p, const Camera& cam) {  // src/algorithm.cpp:435-450
    p.x = p.x >= 0 ? p.x : 0.0;
    p.x = p.x < cam.width ? p.x : cam.width - 1;
    p.y = p.y >= 0 ? p.y : 0.0;
    p.y = p.y < cam.height ? p.y : cam.height - 1;
    return p;
}
// algorithm::matchEpipolarConstraint (src/algorithm.cpp:412-551) on the base (level-0) intensity images
static bool match_epipolar(const Camera& cam, const Image& ref_im, const SE3& ref_pose, const Image& cur_im,
                           const SE3& cur_pose, V2 px, V3 bearing, uint32_t patch, double d0, double dmin, double dmax,
                           double& depth) {
    const uint32_t half = patch / 2, area = patch * patch;
    const SE3 rel = relative_pose(ref_pose, cur_pose);
    const uint32_t thr = area * 128;
    V2 lc = cam.project2d(act(rel, image2camera(cam, px, d0)));
    V2 lmin = cam.project2d(act(rel, image2camera(cam, px, dmin)));
    V2 lmax = cam.project2d(act(rel, image2camera(cam, px, dmax)));
    lc = clamp_to_image(lc, cam);
    lmin = clamp_to_image(lmin, cam);
    lmax = clamp_to_image(lmax, cam);
    const V2 epi{lmax.x - lmin.x, lmax.y - lmin.y};
    double A[4];
    affine_warp(cam, rel, px, patch, d0, A);
    const double norm_epi = std::sqrt(epi.x * epi.x + epi.y * epi.y);
    std::vector<uint8_t> refp(area, 0), curp(area, 0);
    const double I[4] = {1.0, 0.0, 0.0, 1.0};
    apply_affine_warp(cam, ref_im, px, (int32_t)half, I, refp.data());
    if (norm_epi < 2.0) {
        const V2 center{(lmax.x + lmin.x) / 2.0, (lmax.y + lmin.y) / 2.0};
        return depth_from_triangulation(rel, bearing, cam.inverse_project2d(center.x, center.y), depth);
    }
    const uint32_t steps = (uint32_t)std::ceil(norm_epi);
    const V2 step{epi.x / norm_epi, epi.y / norm_epi};
    double best = std::numeric_limits<double>::max();
    V2 best_loc{0.0, 0.0};
    for (uint32_t i = 0; i < steps; ++i) {
        const V2 loc{lmin.x + i * step.x, lmin.y + i * step.y};
        apply_affine_warp(cam, cur_im, loc, (int32_t)half, A, curp.data());
        const double z = compute_score(refp.data(), curp.data(), (int)area);
        if (z < best) { best = z; best_loc = loc; }
    }
    if (best < thr) return depth_from_triangulation(rel, bearing, cam.inverse_project2d(best_loc.x, best_loc.y), depth);
    return false;
}
// DepthEstimator::computeTau (src/depth_estimator.cpp:342-357)
static double compute_tau(const SE3& rel, V3 f, double depth, double err_angle) {
    const V3 t = rel.t;
    const V3 diff = sub(scl(f, depth), t);
    const double nt = norm(t), nd = norm(diff);
    const double alpha = std::acos(dot(f, t) / nt);
    const double beta = std::acos(dot(diff, scl(t, -1.0)) / (nt * nd));
    const double beta_u = beta + err_angle;
    const double gamma_u = 3.141592653589793 - alpha - beta_u;
    const double depth_u = nt * std::sin(beta_u) / std::sin(gamma_u);
    return depth_u - depth;
}
// DepthEstimator::updateFilter (src/depth_estimator.cpp:311-340) + computeNormalDistribution
// (src/algorithm.cpp:907-911)
static void update_filter(double x, double tau2, DepthSeed& s) {
    const double norm_scale = std::sqrt(s.var + tau2);
    if (std::isnan(norm_scale)) return;
    const double s2 = 1.0 / (1.0 / s.var + 1.0 / tau2);
    const double m = s2 * (s.mu / s.var + x / tau2);
    const double p = (x - s.mu) / norm_scale;
    const double nd = 0.3989422804014327 / norm_scale * std::exp(-0.5 * p * p);
    double C1 = s.a / (s.a + s.b) * nd;
    double C2 = s.b / (s.a + s.b) * 1.00 / s.max_depth;
    const double nc = C1 + C2;
    C1 /= nc;
    C2 /= nc;
    const double f = C1 * (s.a + 1.0) / (s.a + s.b + 1.0) + C2 * s.a / (s.a + s.b + 1.0);
    const double e = C1 * (s.a + 1.0) * (s.a + 2.0) / ((s.a + s.b + 1.0) * (s.a + s.b + 2.0)) +
                     C2 * s.a * (s.a + 1.0) / ((s.a + s.b + 1.0) * (s.a + s.b + 2.0));
    const double new_mu = C1 * m + C2 * s.mu;
    s.var = C1 * (s2 + m * m) + C2 * (s.var + s.mu * s.mu) - new_mu * new_mu;
    s.sigma = std::sqrt(s.var);
    s.mu = new_mu;
    s.a = (e - f) / (f - e / f);
    s.b = s.a * (1.0 - f) / f;
}
// one seed of DepthEstimator::updateFilters (:213-297); returns the outcome, `point` for a candidate
static int32_t update_seed(const Camera& cam, const Image& kf_im, const SE3& kf_pose, const Image& cur_im,
                           const SE3& cur_pose, double err_angle, DepthSeed& s, V3& point) {
    const SE3 rel = relative_pose(kf_pose, cur_pose);
    const V3 f{s.bearing[0], s.bearing[1], s.bearing[2]};
    const V3 pc = act(rel, V3{f.x / s.mu, f.y / s.mu, f.z / s.mu});
    if (pc.z < 0 || !cam.is_in_frame(cam.project2d(pc), 0.0)) { s.valid = 0; return kDepthRejected; }
    const double inv_min = s.mu + s.var;
    const double inv_max = std::max(s.mu - s.var, 1e-7);
    double depth = 0.0;
    if (!match_epipolar(cam, kf_im, kf_pose, cur_im, cur_pose, {s.px[0], s.px[1]}, f, 7, 1.0 / s.mu, 1.0 / inv_min,
                        1.0 / inv_max, depth)) {
        s.b++;
        return kDepthNoMatch;
    }
    const double tau = compute_tau(rel, f, depth, err_angle);
    const double inv_tau = 0.5 * (1.0 / std::max(1e-7, depth - tau) - 1.0 / (depth + tau));
    update_filter(1.0 / depth, inv_tau * inv_tau, s);
    if (std::sqrt(s.var) * 10.0 < s.max_depth) {
        const V3 pcam = image2camera(cam, {s.px[0], s.px[1]}, 1.0 / s.mu);  // Frame::image2world (:109-113)
        point = act(inverse(kf_pose), pcam);
        s.valid = 0;
        return kDepthConverged;
    }
    if (std::isnan(inv_min)) { s.valid = 0; return kDepthNaN; }
    return kDepthUpdated;
}

// ------------------------------------------------------------------ pose-only bundle adjustment
// BundleAdjustment::optimizePose (src/bundle_adjustment.cpp:35-69) with computeJacobianPose (:71-98),
// computeResidualsPose (:101-134), computeImageJacPose (:136-160), updatePose (:162-166),
// resetParameters (:306-309).  ref_vis is the member m_refVisibility: the residual functor runs before
// the Jacobian functor in optimizeLM (src/optimizer.cpp:199 vs :242), so it reads the visibility the
// PREVIOUS call's Jacobian functor left (all false on a fresh object).  Returns -1 where the reference
// would dereference a null point (a stale visible flag on a feature without one).
struct PoseBA {
    Optimizer opt{6};
    int32_t optimize_pose(int32_t n, const double* bearing, const double* point, const uint8_t* has_point,
                          std::vector<uint8_t>& ref_vis, SE3& pose, double* err, int32_t* status) {
        if (n == 0) { *err = 0.0; *status = -1; return 0; }          // :37-38 (no optimisation run)
        opt.init_parameters((size_t)n * 3);                           // :45
        ref_vis.resize(n, 0);                                         // :46
        for (int32_t k = 0; k < n; ++k)
            if (ref_vis[k] && !has_point[k]) return -1;
        SE3 absolute = pose;
        auto resid = [&](SE3& T) -> uint32_t {
            uint32_t cnt = 0;
            for (int32_t k = 0; k < n; ++k) {
                if (!ref_vis[k]) continue;
                const V3 pc = act(T, {point[3 * k], point[3 * k + 1], point[3 * k + 2]});
                const double sq = pc.x * pc.x + pc.y * pc.y + pc.z * pc.z;  // Eigen normalized()
                const V3 u = sq > 0.0 ? V3{pc.x / std::sqrt(sq), pc.y / std::sqrt(sq), pc.z / std::sqrt(sq)} : pc;
                const V3 e{bearing[3 * k] - u.x, bearing[3 * k + 1] - u.y, bearing[3 * k + 2] - u.z};
                opt.r[cnt++] = std::fabs(e.x);
                opt.r[cnt++] = std::fabs(e.y);
                opt.r[cnt] = std::fabs(e.z);
                opt.vis[cnt] = 1;                                     // only the third row is visible (:127)
                cnt++;
            }
            return cnt;
        };
        auto jac = [&](SE3& T) {
            std::fill(ref_vis.begin(), ref_vis.end(), 0);             // resetParameters
            uint32_t cp = 0;
            for (int32_t k = 0; k < n; ++k) {
                if (!has_point[k]) continue;
                ref_vis[k] = 1;
                const V3 X = act(T, {point[3 * k], point[3 * k + 1], point[3 * k + 2]});
                const double Jr[3][6] = {{1.0, 0.0, 0.0, 0.0, X.z, -X.y},
                                         {0.0, 1.0, 0.0, -X.z, 0.0, X.x},
                                         {0.0, 0.0, 1.0, X.y, -X.x, 0.0}};
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 6; ++j) opt.J[(3 * cp + i) * 6 + j] = Jr[i][j];
                cp++;
            }
        };
        auto upd = [](SE3& T, const double* dx) { T = compose(se3_exp(dx), T); };  // exp(dx) * pose
        auto res = opt.optimize_lm<SE3>(absolute, resid, upd, jac);
        pose = absolute;                                              // :64 (unchanged on Non_Suff_Points)
        *err = res.second;
        *status = res.first;
        return 0;
    }
};

}  // namespace oracle

// =====================================================================================================
//  C ABI used by tests/ (ctypes) and bench.py's cpu_baseline leg.
// =====================================================================================================
using namespace oracle;

extern "C" {

typedef struct {
    double fx, fy, cx, cy;
    int32_t width, height;
} oc_camera;

typedef struct {
    const uint8_t* ref_pyr;
    const uint8_t* kf_pyr;
    const uint8_t* cur_pyr;
    double ref_pose[7];
    double kf_pose[7];
    int32_t n_ref, n_kf;
    const double* px;          // (n_ref+n_kf) x 2
    const double* bearing;     // x 3
    const double* point;       // x 3
    const uint8_t* has_point;  // (n_ref+n_kf)
} oc_pair;

int64_t oracle_pyramid_bytes(int32_t w, int32_t h, int32_t levels) { return level_dims(w, h, levels).total; }

void oracle_build_pyramid(const uint8_t* img, int32_t w, int32_t h, int32_t levels, uint8_t* out_img, uint8_t* out_grad) {
    build_pyramid(img, w, h, levels, out_img, out_grad);
}

void oracle_project2d(const oc_camera* c, const double* p3, double* out2) {
    Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    V2 uv = cam.project2d({p3[0], p3[1], p3[2]});
    out2[0] = uv.x;
    out2[1] = uv.y;
}

// PinholeCamera::inverseProject2d (src/pinhole_camera.cpp:81-101, no distortion): the unit bearing
void oracle_inverse_project2d(const oc_camera* c, const double* uv, double* out3) {
    Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    const V3 b = cam.inverse_project2d(uv[0], uv[1]);
    out3[0] = b.x;
    out3[1] = b.y;
    out3[2] = b.z;
}

void oracle_se3_exp(const double* tangent6, double* out7) {
    SE3 T = se3_exp(tangent6);
    out7[0] = T.q.x; out7[1] = T.q.y; out7[2] = T.q.z; out7[3] = T.q.w;
    out7[4] = T.t.x; out7[5] = T.t.y; out7[6] = T.t.z;
}

void oracle_se3_compose(const double* a7, const double* b7, double* out7) {
    SE3 a{{a7[0], a7[1], a7[2], a7[3]}, {a7[4], a7[5], a7[6]}};
    SE3 b{{b7[0], b7[1], b7[2], b7[3]}, {b7[4], b7[5], b7[6]}};
    SE3 T = compose(a, b);
    out7[0] = T.q.x; out7[1] = T.q.y; out7[2] = T.q.z; out7[3] = T.q.w;
    out7[4] = T.t.x; out7[5] = T.t.y; out7[6] = T.t.z;
}

void oracle_ldlt_solve(int32_t n, const double* H, const double* b, double* x) { ldlt_solve(n, H, b, x); }

double oracle_median(const double* v, int64_t len, uint32_t n_valid, int32_t mode) {
    std::vector<double> vec(v, v + len);
    return compute_median(vec, n_valid, mode);
}

double oracle_bilinear_d(const uint8_t* img, int32_t w, int32_t h, double x, double y) { return bilinear_d({img, w, h}, x, y); }
float oracle_bilinear_f(const uint8_t* img, int32_t w, int32_t h, double x, double y) { return bilinear_f({img, w, h}, x, y); }

static void load_frames(const oc_camera* c, int32_t levels, const oc_pair* P, Frame& ref, Frame& kf, Frame& cur) {
    LevelDims d = level_dims(c->width, c->height, levels);
    auto pose = [](const double* p) { return SE3{{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}}; };
    ref.pyr = P->ref_pyr; kf.pyr = P->kf_pyr; cur.pyr = P->cur_pyr;
    ref.grad = kf.grad = cur.grad = nullptr;
    ref.dims = kf.dims = cur.dims = d;
    ref.pose = pose(P->ref_pose);
    kf.pose = pose(P->kf_pose);
    ref.last_kf = &kf; kf.last_kf = nullptr; cur.last_kf = &kf;
    ref.features.clear(); kf.features.clear();
    for (int32_t i = 0; i < P->n_ref + P->n_kf; ++i) {
        Feature f;
        f.px = {P->px[2 * i], P->px[2 * i + 1]};
        f.bearing = {P->bearing[3 * i], P->bearing[3 * i + 1], P->bearing[3 * i + 2]};
        f.has_point = P->has_point[i] != 0;
        f.point = {P->point[3 * i], P->point[3 * i + 1], P->point[3 * i + 2]};
        if (i < P->n_ref) { f.frame = &ref; ref.features.push_back(f); }
        else { f.frame = &kf; kf.features.push_back(f); }
    }
}

// ImageAlignment::align on one frame pair.  cur_pose_inout: Sophus params (qx,qy,qz,qw,tx,ty,tz).
// traces (nullable): array of max_level+1 LevelTrace records, indexed by level.
double oracle_image_align(const oc_camera* c, int32_t patch, int32_t min_level, int32_t max_level, int32_t median_mode,
                          const oc_pair* P, double* cur_pose_inout, int32_t* status_out, void* traces) {
    Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    Frame ref, kf, cur;
    load_frames(c, max_level + 1, P, ref, kf, cur);
    const double* p = cur_pose_inout;
    cur.pose = SE3{{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}};
    ImageAlignment ia((uint32_t)patch, min_level, max_level, &cam);
    ia.opt.median_mode = median_mode;
    const double err = ia.align(ref, cur, status_out, (LevelTrace*)traces);
    cur_pose_inout[0] = cur.pose.q.x; cur_pose_inout[1] = cur.pose.q.y; cur_pose_inout[2] = cur.pose.q.z;
    cur_pose_inout[3] = cur.pose.q.w; cur_pose_inout[4] = cur.pose.t.x; cur_pose_inout[5] = cur.pose.t.y;
    cur_pose_inout[6] = cur.pose.t.z;
    return err;
}

int32_t oracle_level_trace_size(void) { return (int32_t)sizeof(LevelTrace); }

// oracle_image_align that also returns the residual vector of every level's robust scale, coarsest level first,
// back to back in `out` (cap doubles) with each level's n_valid in nvalid_out; returns the number of levels stored
// (tools/k2v_round_table.py: the block rounds of the reference's nth_element on real config-2 vectors)
int32_t oracle_image_align_vectors(const oc_camera* c, int32_t patch, int32_t min_level, int32_t max_level,
                                   int32_t median_mode, const oc_pair* P, double* cur_pose_inout, int32_t* status_out,
                                   double* out, int64_t cap, uint32_t* nvalid_out) {
    g_vec_dump = out;
    g_vec_cap = cap;
    g_vec_used = 0;
    g_vec_nvalid = nvalid_out;
    g_vec_levels = 0;
    oracle_image_align(c, patch, min_level, max_level, median_mode, P, cur_pose_inout, status_out, nullptr);
    g_vec_dump = nullptr;
    return g_vec_levels;
}

// ImageAlignment::computeImageJac (src/image_alignment.cpp:194-248): out = 2 x 6 row-major
void oracle_image_jac(const double* p3, double fx, double fy, double* out12) {
    double J[2][6];
    ImageAlignment::image_jac(J, {p3[0], p3[1], p3[2]}, fx, fy);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 6; ++j) out12[i * 6 + j] = J[i][j];
}

// Many independent alignments on nthreads host threads (one alignment per thread at a time, each
// single-threaded like the reference's main-thread call).  Used for the multi-core CPU baseline.
void oracle_image_align_batch(const oc_camera* c, int32_t patch, int32_t min_level, int32_t max_level, int32_t median_mode,
                              int32_t n_pairs, const oc_pair* pairs, double* poses_inout, double* err_out,
                              int32_t* status_out, int32_t nthreads) {
    std::atomic<int32_t> next{0};
    auto worker = [&]() {
        for (;;) {
            const int32_t i = next.fetch_add(1);
            if (i >= n_pairs) break;
            err_out[i] = oracle_image_align(c, patch, min_level, max_level, median_mode, &pairs[i], poses_inout + 7 * i,
                                            status_out + i, nullptr);
        }
    };
    if (nthreads <= 1) { worker(); return; }
    // one worker per CPU of the process's affinity mask, each pinned to its CPU (the CPU baseline's
    // "nproc pinned threads"); more threads than CPUs wrap around the mask
    cpu_set_t mask;
    CPU_ZERO(&mask);
    std::vector<int> cpus;
    if (sched_getaffinity(0, sizeof(mask), &mask) == 0)
        for (int cpu = 0; cpu < CPU_SETSIZE; ++cpu)
            if (CPU_ISSET(cpu, &mask)) cpus.push_back(cpu);
    std::vector<std::thread> th;
    for (int32_t t = 0; t < nthreads; ++t) {
        th.emplace_back(worker);
        if (!cpus.empty()) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(cpus[(size_t)t % cpus.size()], &one);
            (void)pthread_setaffinity_np(th.back().native_handle(), sizeof(one), &one);
        }
    }
    for (auto& t : th) t.join();
}

// FeatureAlignment::align for a batch of candidates sharing one ref / cur gradient L0 image.
// px_inout: n x 2 initial positions (updated in place); ref_px: n x 2 reference pixel positions.
void oracle_feature_align(const oc_camera* c, int32_t patch, const uint8_t* ref_grad, const uint8_t* cur_grad, int32_t n,
                          const double* ref_px, double* px_inout, double* err_out, int32_t* status_out) {
    Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    const Image rg{ref_grad, c->width, c->height}, cg{cur_grad, c->width, c->height};
    FeatureAlignment fa((uint32_t)patch, &cam);
    for (int32_t i = 0; i < n; ++i) {
        V2 px{px_inout[2 * i], px_inout[2 * i + 1]};
        int32_t st = 0;
        err_out[i] = fa.align(rg, {ref_px[2 * i], ref_px[2 * i + 1]}, cg, px, &st);
        px_inout[2 * i] = px.x;
        px_inout[2 * i + 1] = px.y;
        if (status_out) status_out[i] = st;
    }
}

// MixedGaussianFilter::MixedGaussianFilter (src/mixed_gaussian_filter.cpp:7-24)
void oracle_depth_seed_init(double depth_mean, double depth_min, double* a_b_mu_sigma_var_maxdepth) {
    double* o = a_b_mu_sigma_var_maxdepth;
    o[0] = 10; o[1] = 10; o[2] = 1.0 / depth_mean; o[5] = 1.0 / depth_min;
    o[3] = o[5] / 6; o[4] = o[3] * o[3];
}

// DepthEstimator::updateFilters (src/depth_estimator.cpp:192-309) for n seeds against one cur frame.
// kf_imgs[k] / kf_poses[7k]: level-0 intensity image and pose of keyframe k (seed.kf indexes them).
// seeds (n, in/out): updated in place, then compacted like the reference's remove_if (stable) to
// *n_out survivors.  outcome[n]: per input seed (DepthOutcome).  Candidates (m_map->addNewCandidate, in
// the reverse seed order of the update loop): cand_points[3 * c], cand_seed[c] (input index), *n_cand.
void oracle_depth_update(const oc_camera* c, int32_t n_kf, const uint8_t* const* kf_imgs, const double* kf_poses,
                         const uint8_t* cur_img, const double* cur_pose, int32_t n, void* seeds_v, int32_t* n_out,
                         int32_t* outcome, double* cand_points, int32_t* cand_seed, int32_t* n_cand) {
    (void)n_kf;
    Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    DepthSeed* seeds = (DepthSeed*)seeds_v;
    auto pose = [](const double* p) { return SE3{{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}}; };
    const SE3 cp = pose(cur_pose);
    const Image ci{cur_img, c->width, c->height};
    const double err_angle = std::atan(1.0 / (2.0 * c->fx)) * 2.0;  // :202-206 (pixel noise 1)
    int32_t nc = 0;
    for (int32_t i = n - 1; i >= 0; --i) {
        DepthSeed& s = seeds[i];
        const Image ki{kf_imgs[s.kf], c->width, c->height};
        V3 pt{0, 0, 0};
        outcome[i] = update_seed(cam, ki, pose(kf_poses + 7 * s.kf), ci, cp, err_angle, s, pt);
        if (outcome[i] == kDepthConverged) {
            cand_points[3 * nc] = pt.x; cand_points[3 * nc + 1] = pt.y; cand_points[3 * nc + 2] = pt.z;
            cand_seed[nc++] = i;
        }
    }
    int32_t k = 0;
    for (int32_t i = 0; i < n; ++i)
        if (seeds[i].valid) seeds[k++] = seeds[i];
    *n_out = k;
    *n_cand = nc;
}

int32_t oracle_depth_seed_size(void) { return (int32_t)sizeof(DepthSeed); }

// algorithm::computeScore (src/algorithm.cpp:396-410) on two n-byte patches
double oracle_zsad(const uint8_t* ref, const uint8_t* cur, int32_t n) { return compute_score(ref, cur, n); }

// algorithm::depthFromTriangulation (src/algorithm.cpp:682-703); returns 0 when rejected (det < 1e-6)
int32_t oracle_depth_triangulate(const double* rel7, const double* fref, const double* fcur, double* depth) {
    const SE3 rel{{rel7[0], rel7[1], rel7[2], rel7[3]}, {rel7[4], rel7[5], rel7[6]}};
    return depth_from_triangulation(rel, {fref[0], fref[1], fref[2]}, {fcur[0], fcur[1], fcur[2]}, *depth) ? 1 : 0;
}

// ---------------------------------------------------------------- Map reprojection (src/map.cpp)
// Map::reprojectMap (:260-478) with reprojectPoint (:481-492) and reprojectCell (:495-570), restated
// sequentially: one FeatureAlignment(7, 0, 3) call per accepted candidate, in the reference's order.
// Keyframe k (ref frame, then its last keyframe) owns features kf_feat_off[k] .. kf_feat_off[k+1]-1 at
// feat_px, observing point feat_point (-1: none).  Point state in/out: type (0 GOOD, 1 DELETED,
// 2 CANDIDATE, 3 UNKNOWN), succeeded projections, last projected frame id.  cell_visited (in/out) is the
// Map's m_cellVisited.  Out: overlap per keyframe, the new features of cur (aligned pixel, point,
// source feature) in creation order, m_matches, m_trials.
void oracle_reproject_map(const oc_camera* c, int32_t cell_size, const int32_t* cell_order, const double* cur_pose,
                          uint64_t cur_id, const uint8_t* cur_grad, int32_t n_kf, const uint8_t* const* kf_grad,
                          const int32_t* kf_feat_off, const double* feat_px, const int32_t* feat_point,
                          const double* point_pos, uint32_t* point_type, uint32_t* point_succ, uint64_t* point_last,
                          uint8_t* cell_visited, int32_t* overlap, int32_t* n_new, double* new_px, int32_t* new_point,
                          int32_t* new_feat, int32_t* matches, int32_t* trials) {
    const Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    const SE3 T{{cur_pose[0], cur_pose[1], cur_pose[2], cur_pose[3]}, {cur_pose[4], cur_pose[5], cur_pose[6]}};
    const uint32_t cols = (uint32_t)std::ceil((double)c->width / cell_size), rows = (uint32_t)std::ceil((double)c->height / cell_size);
    struct Cand { int32_t feat, kf, point; };
    std::vector<std::vector<Cand>> cells(cols * rows);  // resetGrid (:250-258)
    int32_t m = 0, t = 0, nn = 0;
    auto world2image = [&](int32_t p) { return cam.project2d(act(T, {point_pos[3 * p], point_pos[3 * p + 1], point_pos[3 * p + 2]})); };
    for (int32_t k = 0; k < n_kf; ++k) {
        overlap[k] = 0;
        for (int32_t f = kf_feat_off[k]; f < kf_feat_off[k + 1]; ++f) {
            const int32_t p = feat_point[f];
            if (p < 0) continue;                 // feature->m_point == nullptr
            if (point_last[p] == cur_id) continue;
            point_last[p] = cur_id;
            const V2 px = world2image(p);        // reprojectPoint
            if (!cam.is_in_frame(px, 3)) continue;
            const int32_t cell = (int32_t)((uint32_t)(int32_t)px.y / (uint32_t)cell_size * cols + (uint32_t)(int32_t)px.x / (uint32_t)cell_size);
            cells[cell].push_back({f, k, p});
            ++overlap[k];
        }
    }
    FeatureAlignment fa(7, &cam);
    const Image cg{cur_grad, c->width, c->height};
    for (uint32_t i = 0; i < cells.size(); ++i) {
        const int32_t idx = cell_order[i];
        std::vector<Cand>& cand = cells[idx];
        bool accepted = false;
        if (!cand.empty()) {  // reprojectCell
            std::sort(cand.begin(), cand.end(), [&](const Cand& a, const Cand& b) { return point_type[a.point] > point_type[b.point]; });
            for (const Cand& cd : cand) {
                ++t;
                if (point_type[cd.point] == 1u) continue;  // DELETED
                V2 px = world2image(cd.point);
                int32_t st = 0;
                (void)fa.align({kf_grad[cd.kf], c->width, c->height}, {feat_px[2 * cd.feat], feat_px[2 * cd.feat + 1]}, cg, px, &st);
                ++point_succ[cd.point];
                if (point_type[cd.point] == 3u && point_succ[cd.point] > 10) point_type[cd.point] = 0u;  // UNKNOWN -> GOOD
                new_px[2 * nn] = px.x; new_px[2 * nn + 1] = px.y;
                new_point[nn] = cd.point;
                new_feat[nn] = cd.feat;
                ++nn;
                accepted = true;
                break;
            }
        }
        if (accepted) {
            ++m;
            cell_visited[idx] = 1;
        }
        if (m > 150) break;
    }
    *n_new = nn;
    *matches = m;
    *trials = t;
}

// Map::addCandidateToFrame (src/map.cpp:595-627) restated sequentially over the candidate list:
// candidate i = (its feature: gradient of its frame cand_grad[i] at cand_px[i]; its point at
// cand_point_pos[i]).  matched[i] = 1 and new_px[i] = the aligned pixel when it was added.
void oracle_add_candidates(const oc_camera* c, int32_t cell_size, uint8_t* cell_visited, const double* cur_pose,
                           const uint8_t* cur_grad, int32_t n_cand, const uint8_t* const* cand_grad,
                           const double* cand_px, const double* cand_point_pos, uint8_t* matched, double* new_px) {
    const Camera cam{c->fx, c->fy, c->cx, c->cy, c->width, c->height};
    const SE3 T{{cur_pose[0], cur_pose[1], cur_pose[2], cur_pose[3]}, {cur_pose[4], cur_pose[5], cur_pose[6]}};
    const uint32_t cols = (uint32_t)std::ceil((double)c->width / cell_size);
    FeatureAlignment fa(7, &cam);
    const Image cg{cur_grad, c->width, c->height};
    for (int32_t i = 0; i < n_cand; ++i) {
        matched[i] = 0;
        V2 px = cam.project2d(act(T, {cand_point_pos[3 * i], cand_point_pos[3 * i + 1], cand_point_pos[3 * i + 2]}));
        if (!cam.is_in_frame(px, 3)) continue;
        const int32_t k = (int32_t)((uint32_t)(int32_t)px.y / (uint32_t)cell_size * cols + (uint32_t)(int32_t)px.x / (uint32_t)cell_size);
        if (cell_visited[k]) continue;
        int32_t st = 0;
        const double err = fa.align({cand_grad[i], c->width, c->height}, {cand_px[2 * i], cand_px[2 * i + 1]}, cg, px, &st);
        if (err < 50.0) {
            matched[i] = 1;
            new_px[2 * i] = px.x; new_px[2 * i + 1] = px.y;
            cell_visited[k] = 1;
        }
    }
}

// System::writeInFile (src/system.cpp:635-640): m_absPose.inverse().matrix3x4() streamed with
// std::setprecision(6) through Eigen's IOFormat(6, DontAlignCols, " ", " ", "", "", "", "")
// (src/utils.cpp:10-13): coefficients of a row joined by the coefficient separator, rows by the row
// separator, no prefixes.  Returns the line length (without newline), -1 if cap is short.
int32_t oracle_kitti_line(const double* pose, char* buf, int32_t cap) {
    const SE3 T{{pose[0], pose[1], pose[2], pose[3]}, {pose[4], pose[5], pose[6]}};
    const SE3 Ti = inverse(T);
    double R[3][3];
    rotmat(Ti.q, R);
    const double t[3] = {Ti.t.x, Ti.t.y, Ti.t.z};
    std::ostringstream os;
    os << std::setprecision(6);
    for (int r = 0; r < 3; ++r) {
        if (r) os << " ";                         // rowSeparator
        for (int c = 0; c < 4; ++c) {
            if (c) os << " ";                     // coeffSeparator
            os << (c < 3 ? R[r][c] : t[r]);
        }
    }
    const std::string line = os.str();
    if ((int32_t)line.size() + 1 > cap) return -1;
    std::memcpy(buf, line.c_str(), line.size() + 1);
    return (int32_t)line.size();
}

// one double as `stream << std::setprecision(6) << v` (utils::writeAllInfoFile, src/utils.cpp:62-70)
int32_t oracle_stream_g6(double v, char* buf, int32_t cap) {
    std::ostringstream os;
    os << std::setprecision(6) << v;
    const std::string s = os.str();
    if ((int32_t)s.size() + 1 > cap) return -1;
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int32_t)s.size();
}

// BundleAdjustment::optimizePose on one frame: n features (bearing n x 3, point n x 3, has_point n);
// vis_inout: m_refVisibility of the BundleAdjustment object (n_vis_in entries in, n out: the caller
// resizes like the member).  status -1: no optimisation ran (n == 0, return value 0).
int32_t oracle_optimize_pose(int32_t n, const double* bearing, const double* point, const uint8_t* has_point,
                             int32_t n_vis_in, uint8_t* vis_inout, double* pose_inout, int32_t median_mode,
                             double* err, int32_t* status) {
    PoseBA ba;
    ba.opt.median_mode = median_mode;
    std::vector<uint8_t> vis(vis_inout, vis_inout + n_vis_in);
    SE3 T{{pose_inout[0], pose_inout[1], pose_inout[2], pose_inout[3]}, {pose_inout[4], pose_inout[5], pose_inout[6]}};
    if (ba.optimize_pose(n, bearing, point, has_point, vis, T, err, status) != 0) return -1;
    if (n > 0) std::copy(vis.begin(), vis.end(), vis_inout);
    const double o[7] = {T.q.x, T.q.y, T.q.z, T.q.w, T.t.x, T.t.y, T.t.z};
    std::copy(o, o + 7, pose_inout);
    return 0;
}

}  // extern "C"
