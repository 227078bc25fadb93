// svo_math.h — SE(3), camera and bilinear arithmetic shared by the HIP kernels and the host shim.
//
// The operation order of every function below is the reference's (Sophus / Eigen / src/algorithm.cpp)
// evaluated left to right, and everything is compiled with -ffp-contract=off, so per-feature results
// are bit-identical to the CPU restatement in oracle/ (the checker).  Citations:
//   quaternion action  Eigen QuaternionBase::_transformVector (used by Sophus SO3 * point)
//   SE3 product/inverse/exp   Sophus se3.hpp / so3.hpp (src/image_alignment.cpp:379, src/frame.cpp:94-97)
//   cameraInWorld      src/frame.cpp:116-120          project2d  src/pinhole_camera.cpp:53-57
//   bilinear (double)  src/algorithm.cpp:896-905      bilinear (float) src/algorithm.cpp:885-894
//   image Jacobian     src/image_alignment.cpp:194-248
//   LDLT solve         Eigen LDLT<MatrixXd, Lower> (src/optimizer.cpp:306)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SVO_HD __host__ __device__ __forceinline__

namespace svo {

struct V3 { double x, y, z; };
struct Q { double x, y, z, w; };  // Eigen coefficient order
struct SE3 { Q q; V3 t; };         // world -> camera; Sophus params (qx,qy,qz,qw,tx,ty,tz)

SVO_HD V3 v3add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
SVO_HD V3 v3sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
SVO_HD V3 v3scl(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
SVO_HD V3 v3cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
SVO_HD double v3norm(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

SVO_HD V3 qrot(const Q& q, V3 v) {
    const V3 qv{q.x, q.y, q.z};
    V3 uv = v3cross(qv, v);
    uv = v3add(uv, uv);
    return v3add(v3add(v, v3scl(uv, q.w)), v3cross(qv, uv));
}
SVO_HD Q qconj(const Q& q) { return {-q.x, -q.y, -q.z, q.w}; }
SVO_HD Q qmul(const Q& a, const Q& b) {  // Sophus SO3 product + near-unit renormalisation
    Q r{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
        a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
    const double n2 = r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
    if (n2 != 1.0) {
        const double f = 2.0 / (1.0 + n2);
        r.x *= f; r.y *= f; r.z *= f; r.w *= f;
    }
    return r;
}
SVO_HD V3 se3_act(const SE3& T, V3 p) { return v3add(qrot(T.q, p), T.t); }
SVO_HD SE3 se3_inverse(const SE3& T) {
    const Q qi = qconj(T.q);
    return {qi, qrot(qi, v3scl(T.t, -1.0))};
}
SVO_HD SE3 se3_compose(const SE3& a, const SE3& b) { return {qmul(a.q, b.q), v3add(a.t, qrot(a.q, b.t))}; }
SVO_HD void rotmat(const Q& q, double R[3][3]) {  // Eigen toRotationMatrix
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1.0 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
    R[1][0] = txy + twz; R[1][1] = 1.0 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1.0 - (txx + tyy);
}
SVO_HD V3 camera_in_world(const SE3& T) {  // C = -R^T t
    double R[3][3];
    rotmat(T.q, R);
    V3 c;
    c.x = (-R[0][0]) * T.t.x + (-R[1][0]) * T.t.y + (-R[2][0]) * T.t.z;
    c.y = (-R[0][1]) * T.t.x + (-R[1][1]) * T.t.y + (-R[2][1]) * T.t.z;
    c.z = (-R[0][2]) * T.t.x + (-R[1][2]) * T.t.y + (-R[2][2]) * T.t.z;
    return c;
}
SVO_HD SE3 se3_exp(const double a[6]) {  // tangent (upsilon; omega), Sophus epsilon 1e-10
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
        theta = sqrt(theta_sq);
        const double half = 0.5 * theta;
        imag = sin(half) / theta;
        real = cos(half);
    }
    const Q q{imag * om.x, imag * om.y, imag * om.z, real};
    const double W[3][3] = {{0.0, -om.z, om.y}, {om.z, 0.0, -om.x}, {-om.y, om.x, 0.0}};
    double W2[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) W2[i][j] = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
    double V[3][3];
    if (theta < eps) {
        rotmat(q, V);
    } else {
        const double c1 = (1.0 - cos(theta)) / (theta_sq);
        const double c2 = (theta - sin(theta)) / (theta_sq * theta);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) V[i][j] = ((i == j ? 1.0 : 0.0) + c1 * W[i][j]) + c2 * W2[i][j];
    }
    const V3 t{V[0][0] * up.x + V[0][1] * up.y + V[0][2] * up.z, V[1][0] * up.x + V[1][1] * up.y + V[1][2] * up.z,
               V[2][0] * up.x + V[2][1] * up.y + V[2][2] * up.z};
    return {q, t};
}
SVO_HD SE3 se3_load(const double* p) { return {{p[0], p[1], p[2], p[3]}, {p[4], p[5], p[6]}}; }
SVO_HD void se3_store(const SE3& T, double* p) {
    p[0] = T.q.x; p[1] = T.q.y; p[2] = T.q.z; p[3] = T.q.w; p[4] = T.t.x; p[5] = T.t.y; p[6] = T.t.z;
}

// Eigen LDLT<.., Lower> factor + solve, n <= 6, row-major A (lower triangle read), factored in place.
// A / perm / tmp are caller workspace (registers, or LDS so that no thread keeps 36 doubles live).
template <typename Real, typename Int>
SVO_HD void ldlt_solve_ws(int n, Real* A, const double* b, double* x, Int* perm, Real* tmp) {
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double best = fabs(A[k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            const double v = fabs(A[i * n + i]);
            if (v > best) { best = v; piv = i; }
        }
        perm[k] = piv;
        if (piv != k) {
            for (int j = 0; j < k; ++j) { double t = A[k * n + j]; A[k * n + j] = A[piv * n + j]; A[piv * n + j] = t; }
            for (int i = piv + 1; i < n; ++i) { double t = A[i * n + k]; A[i * n + k] = A[i * n + piv]; A[i * n + piv] = t; }
            { double t = A[k * n + k]; A[k * n + k] = A[piv * n + piv]; A[piv * n + piv] = t; }
            for (int i = k + 1; i < piv; ++i) { double t = A[i * n + k]; A[i * n + k] = A[piv * n + i]; A[piv * n + i] = t; }
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
        const bool valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            for (int j = 0; j < n; ++j) perm[j] = j;
            break;
        }
        if (valid)
            for (int i = k + 1; i < n; ++i) A[i * n + k] /= akk;
    }
    for (int i = 0; i < n; ++i) x[i] = b[i];
    for (int k = 0; k < n; ++k) { double t = x[k]; x[k] = x[perm[k]]; x[perm[k]] = t; }
    for (int i = 0; i < n; ++i) {
        double s = x[i];
        for (int j = 0; j < i; ++j) s -= A[i * n + j] * x[j];
        x[i] = s;
    }
    for (int i = 0; i < n; ++i) {
        const double d = A[i * n + i];
        if (fabs(d) > 2.2250738585072014e-308) x[i] /= d;
        else x[i] = 0.0;
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = x[i];
        for (int j = i + 1; j < n; ++j) s -= A[j * n + i] * x[j];
        x[i] = s;
    }
    for (int k = n - 1; k >= 0; --k) { double t = x[k]; x[k] = x[perm[k]]; x[perm[k]] = t; }
}
SVO_HD void ldlt_solve(int n, const double* Hin, const double* b, double* x) {
    double A[36], tmp[6];
    int perm[6];
    for (int i = 0; i < n * n; ++i) A[i] = Hin[i];
    ldlt_solve_ws(n, A, b, x, perm, tmp);
}

// algorithm::bilinearInterpolationDouble — row-major u8 image with row pitch `w`
SVO_HD double bilinear_d(const uint8_t* img, int32_t w, double x, double y) {
    const int32_t x1 = (int32_t)x, y1 = (int32_t)y, x2 = x1 + 1, y2 = y1 + 1;
    const uint8_t* r1 = img + (int64_t)y1 * w;
    const uint8_t* r2 = r1 + w;
    const double a = (x2 - x) * r1[x1] + (x - x1) * r1[x2];
    const double b = (x2 - x) * r2[x1] + (x - x1) * r2[x2];
    return (y2 - y) * a + (y - y1) * b;
}
// algorithm::bilinearInterpolation (float result, float-rounded row blends)
SVO_HD float bilinear_f(const uint8_t* img, int32_t w, double x, double y) {
    const int32_t x1 = (int32_t)x, y1 = (int32_t)y, x2 = x1 + 1, y2 = y1 + 1;
    const uint8_t* r1 = img + (int64_t)y1 * w;
    const uint8_t* r2 = r1 + w;
    const float a = (float)((x2 - x) * r1[x1] + (x - x1) * r1[x2]);
    const float b = (float)((x2 - x) * r2[x1] + (x - x1) * r2[x2]);
    return (float)((y2 - y) * (double)a + (y - y1) * (double)b);
}

// ImageAlignment::computeImageJac, rows a (u) and b (v)
SVO_HD void image_jac(V3 p, double fx, double fy, double a[6], double b[6]) {
    const double x = p.x, y = p.y, z = p.z, x2 = x * x, y2 = y * y, z2 = z * z;
    a[0] = fx / z; a[1] = 0.0; a[2] = -(fx * x) / z2; a[3] = -(fx * x * y) / z2; a[4] = (fx * x2) / z2 + fx; a[5] = -(fx * y) / z;
    b[0] = 0.0; b[1] = fy / z; b[2] = -(fy * y) / z2; b[3] = -(fy * y2) / z2 - fy; b[4] = (fy * x * y) / z2; b[5] = (fy * x) / z;
}

// order-preserving map double -> uint64 (for exact radix selection)
SVO_HD uint64_t dkey(double d) {
    uint64_t u;
    __builtin_memcpy(&u, &d, 8);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
SVO_HD double dkey_inv(uint64_t k) {
    const uint64_t u = (k & 0x8000000000000000ull) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    double d;
    __builtin_memcpy(&d, &u, 8);
    return d;
}

// Optimizer::Status (include/optimizer.hpp:21-33)
enum Status : int32_t {
    kSuccess = 0, kMaxCoffDx = 1, kNonInDx = 2, kSmallStepSize = 3, kLambdaValue = 4, kNormInfDiff = 5,
    kNonSuffPoints = 6, kIncreaseChi = 7, kSmallChi = 8, kFailed = 9
};

}  // namespace svo
