// depth_filter.hip — DepthEstimator::updateFilters (src/depth_estimator.cpp:192-309) on gfx950.
//
// One 64-lane wave per seed (independent: the reference's loop carries no state between seeds except
// the order of the candidate list, restored by the compaction kernel).  Per seed, in the reference's
// order:
//   relative pose T_cur T_kf^-1 (src/algorithm.cpp:705-709), visibility of the mu point (:229-237),
//   inverse-depth range mu +- var (:240-241), matchEpipolarConstraint (src/algorithm.cpp:412-551):
//   three projections clamped to the image, affine warp (:335-367), 7x7 ref patch (identity warp),
//   then the epipolar scan: lane p < 49 samples patch pixel p of every step (float bilinear truncated to
//   uint8, :369-394) and the step's ZSAD with the uint8-wrapping means (:396-410) is a wave sum.  Every
//   term of the score is an integer, so the score is exact in any summation order and the strict-<
//   argmin over the steps (:509-522) matches the reference bit for bit.  A step outside the frame keeps
//   the previous patch, like the reference's untouched buffer.  Then triangulation (:682-703), tau
//   (src/depth_estimator.cpp:342-357) and the Gaussian x Beta update (:311-340).
// The compaction kernel then restores the reference's output order: survivors stable (remove_if,
// :302-307), candidates in the update loop's order (seed N-1 first).
#include "svo_internal.h"
#include "svo_math.h"

namespace svo {

namespace {

constexpr int kDfWaves = 4;
constexpr int kHalfP = 3, kSideP = 7, kAreaP = 49;  // patch 7 (src/depth_estimator.cpp:245)
constexpr double kPi = 3.141592653589793;            // utils::constants::pi (include/utils.hpp:45)

struct V2 { double x, y; };

struct Cam {
    double fx, fy, cx, cy;
    int W, H;
    __device__ V2 project(V3 p) const { return {fx * (p.x / p.z) + cx, fy * (p.y / p.z) + cy}; }  // :53-57
    __device__ V3 inverse_project(double u, double v) const {  // src/pinhole_camera.cpp:84-100
        const V3 p{(u - cx) / fx, (v - cy) / fy, 1.0};
        return v3scl(p, 1.0 / v3norm(p));
    }
    __device__ bool in_frame(V2 p, double b) const { return p.x >= b && p.y >= b && p.x < W - b && p.y < H - b; }
    __device__ V3 image2camera(V2 px, double depth) const { return v3scl(inverse_project(px.x, px.y), depth); }
    __device__ V2 clamp(V2 p) const {  // src/algorithm.cpp:435-450
        p.x = p.x >= 0 ? p.x : 0.0;
        p.x = p.x < W ? p.x : W - 1;
        p.y = p.y >= 0 ? p.y : 0.0;
        p.y = p.y < H ? p.y : H - 1;
        return p;
    }
};

__device__ __forceinline__ int wave_sum_i(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// algorithm::depthFromTriangulation (src/algorithm.cpp:682-703), Eigen evaluation order
__device__ bool triangulate(const SE3& rel, V3 fr, V3 fc, double& depth) {
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
    double tmp[3];  // row 0 of (-Inv) * A^T
    for (int k = 0; k < 3; ++k) tmp[k] = (-Inv[0][0]) * A[k][0] + (-Inv[0][1]) * A[k][1];
    depth = fabs(tmp[0] * t[0] + tmp[1] * t[1] + tmp[2] * t[2]);
    return true;
}

__device__ double compute_tau(const SE3& rel, V3 f, double depth, double err_angle) {  // :342-357
    const V3 t = rel.t;
    const V3 diff = v3sub(v3scl(f, depth), t);
    const double nt = v3norm(t), nd = v3norm(diff);
    const V3 mt = v3scl(t, -1.0);
    const double alpha = acos((f.x * t.x + f.y * t.y + f.z * t.z) / nt);
    const double beta = acos((diff.x * mt.x + diff.y * mt.y + diff.z * mt.z) / (nt * nd));
    const double beta_u = beta + err_angle;
    const double gamma_u = kPi - alpha - beta_u;
    const double depth_u = nt * sin(beta_u) / sin(gamma_u);
    return depth_u - depth;
}

__device__ void update_filter(double x, double tau2, svo_depth_seed& s) {  // :311-340, N(mu, s, x) :907-911
    const double norm_scale = sqrt(s.var + tau2);
    if (isnan(norm_scale)) return;
    const double s2 = 1.0 / (1.0 / s.var + 1.0 / tau2);
    const double m = s2 * (s.mu / s.var + x / tau2);
    const double p = (x - s.mu) / norm_scale;
    const double nd = 0.3989422804014327 / norm_scale * exp(-0.5 * p * p);
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
    s.sigma = sqrt(s.var);
    s.mu = new_mu;
    s.a = (e - f) / (f - e / f);
    s.b = s.a * (1.0 - f) / f;
}

}  // namespace

__global__ void __launch_bounds__(64 * kDfWaves) depth_update_kernel(DepthArgs a) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * kDfWaves + (int)(threadIdx.x >> 6);
    if (i >= a.n) return;  // whole waves
    const Cam cam{a.fx, a.fy, a.cx, a.cy, a.width, a.height};
    svo_depth_seed s = a.seeds[i];
    const SE3 kfp = se3_load(a.kf_poses + 7 * s.kf), curp = se3_load(a.cur_pose);
    const uint8_t* kimg = a.kf_imgs[s.kf];
    const uint8_t* cimg = a.cur_img;
    const SE3 rel = se3_compose(curp, se3_inverse(kfp));
    const V3 f{s.bearing[0], s.bearing[1], s.bearing[2]};
    const V2 px{s.px[0], s.px[1]};
    int32_t outcome;
    V3 point{0.0, 0.0, 0.0};
    const V3 pc = se3_act(rel, V3{f.x / s.mu, f.y / s.mu, f.z / s.mu});
    if (pc.z < 0 || !cam.in_frame(cam.project(pc), 0.0)) {
        s.valid = 0;
        outcome = SVO_DEPTH_REJECTED;
    } else {
        const double inv_min = s.mu + s.var;
        const double inv_max = fmax(s.mu - s.var, 1e-7);
        const double d0 = 1.0 / s.mu, dmin = 1.0 / inv_min, dmax = 1.0 / inv_max;
        // ---- matchEpipolarConstraint
        const V2 lmin = cam.clamp(cam.project(se3_act(rel, cam.image2camera(px, dmin))));
        const V2 lmax = cam.clamp(cam.project(se3_act(rel, cam.image2camera(px, dmax))));
        const V2 epi{lmax.x - lmin.x, lmax.y - lmin.y};
        double A[4];  // getAffineWarp (:335-367), row-major
        {
            const V3 c = cam.image2camera(px, d0);
            const V3 du = cam.image2camera({px.x + (double)kHalfP, px.y + 0.0}, d0);
            const V3 dv = cam.image2camera({px.x + 0.0, px.y + (double)kHalfP}, d0);
            const V2 cc = cam.project(se3_act(rel, c)), uc = cam.project(se3_act(rel, du)), vc = cam.project(se3_act(rel, dv));
            A[0] = (uc.x - cc.x) / (double)kHalfP; A[2] = (uc.y - cc.y) / (double)kHalfP;
            A[1] = (vc.x - cc.x) / (double)kHalfP; A[3] = (vc.y - cc.y) / (double)kHalfP;
        }
        const double norm_epi = sqrt(epi.x * epi.x + epi.y * epi.y);
        // ref patch with the identity warp (boundary ceil(3) + 2 = 5); lane p holds pixel p
        const int pi_ = lane / kSideP - kHalfP, pj = lane - (lane / kSideP) * kSideP - kHalfP;
        const bool pl = lane < kAreaP;
        int refv = 0;
        {
            const double bx = 1.0 * kHalfP + 0.0 * kHalfP, by = 0.0 * kHalfP + 1.0 * kHalfP;
            const double maxb = ceil(fmax(fabs(bx), fabs(by))) + 2;
            if (pl && cam.in_frame(px, maxb))
                refv = (uint8_t)bilinear_f(kimg, cam.W, px.x + (1.0 * pj + 0.0 * pi_), px.y + (0.0 * pj + 1.0 * pi_));
        }
        const int mr = (wave_sum_i(refv) & 255) / kAreaP;  // Eigen uint8 mean
        bool ok;
        double depth = 0.0;
        if (norm_epi < 2.0) {
            const V2 center{(lmax.x + lmin.x) / 2.0, (lmax.y + lmin.y) / 2.0};
            ok = triangulate(rel, f, cam.inverse_project(center.x, center.y), depth);
        } else {
            const uint32_t steps = (uint32_t)ceil(norm_epi);
            const V2 step{epi.x / norm_epi, epi.y / norm_epi};
            const double bx = A[0] * kHalfP + A[1] * kHalfP, by = A[2] * kHalfP + A[3] * kHalfP;
            const double maxb = ceil(fmax(fabs(bx), fabs(by))) + 2;
            const double ox = A[0] * pj + A[1] * pi_, oy = A[2] * pj + A[3] * pi_;  // A (j, i) of this lane
            int curv = 0;  // the patch buffer (zeroed once, kept across out-of-frame steps)
            double best = 1.7976931348623157e308;
            V2 best_loc{0.0, 0.0};
            for (uint32_t k = 0; k < steps; ++k) {
                const V2 loc{lmin.x + k * step.x, lmin.y + k * step.y};
                if (cam.in_frame(loc, maxb) && pl) curv = (uint8_t)bilinear_f(cimg, cam.W, loc.x + ox, loc.y + oy);
                const int mc = (wave_sum_i(curv) & 255) / kAreaP;
                const int err = pl ? abs((refv - mr) - (curv - mc)) : 0;
                const double z = (double)wave_sum_i(err);  // computeScore: integer terms, exact
                if (z < best) { best = z; best_loc = loc; }
            }
            ok = best < (double)(kAreaP * 128) &&
                 triangulate(rel, f, cam.inverse_project(best_loc.x, best_loc.y), depth);
        }
        if (!ok) {
            s.b++;
            outcome = SVO_DEPTH_NO_MATCH;
        } else {
            const double tau = compute_tau(rel, f, depth, a.err_angle);
            const double inv_tau = 0.5 * (1.0 / fmax(1e-7, depth - tau) - 1.0 / (depth + tau));
            update_filter(1.0 / depth, inv_tau * inv_tau, s);
            if (sqrt(s.var) * 10.0 < s.max_depth) {
                point = se3_act(se3_inverse(kfp), cam.image2camera(px, 1.0 / s.mu));  // Frame::image2world
                s.valid = 0;
                outcome = SVO_DEPTH_CONVERGED;
            } else if (isnan(inv_min)) {
                s.valid = 0;
                outcome = SVO_DEPTH_NAN;
            } else {
                outcome = SVO_DEPTH_UPDATED;
            }
        }
    }
    if (lane == 0) {
        a.seeds_new[i] = s;
        a.outcome[i] = outcome;
        a.points[3 * i] = point.x; a.points[3 * i + 1] = point.y; a.points[3 * i + 2] = point.z;
    }
}

// Stable compaction in one workgroup: survivors in seed order (remove_if, src/depth_estimator.cpp:302-307)
// and candidates in the update loop's order (seed n-1 first).  counts[0] = survivors, counts[1] = candidates.
__global__ void __launch_bounds__(1024) depth_compact_kernel(DepthArgs a) {
    __shared__ int wsum[2][16];
    __shared__ int base[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) { base[0] = 0; base[1] = 0; }
    __syncthreads();
    for (int c0 = 0; c0 < a.n; c0 += 1024) {
        const int i = c0 + tid, ir = a.n - 1 - i;  // survivors scan forward, candidates backward
        const bool keep = i < a.n && a.seeds_new[i].valid;
        const bool cand = i < a.n && a.outcome[ir] == SVO_DEPTH_CONVERGED;
        const uint64_t mk = __ballot(keep), mc = __ballot(cand);
        const uint64_t below = (1ull << lane) - 1ull;
        if (lane == 0) { wsum[0][wave] = __popcll(mk); wsum[1][wave] = __popcll(mc); }
        __syncthreads();
        int ok = base[0], oc = base[1];
        for (int w = 0; w < wave; ++w) { ok += wsum[0][w]; oc += wsum[1][w]; }
        if (keep) a.seeds_out[ok + __popcll(mk & below)] = a.seeds_new[i];
        if (cand) {
            const int k = oc + __popcll(mc & below);
            a.cand_points[3 * k] = a.points[3 * ir];
            a.cand_points[3 * k + 1] = a.points[3 * ir + 1];
            a.cand_points[3 * k + 2] = a.points[3 * ir + 2];
            a.cand_seed[k] = ir;
        }
        __syncthreads();
        if (tid == 0)
            for (int w = 0; w < 16; ++w) { base[0] += wsum[0][w]; base[1] += wsum[1][w]; }
        __syncthreads();
    }
    if (tid == 0) { a.counts[0] = base[0]; a.counts[1] = base[1]; }
}

void launch_depth_update(const DepthArgs& a, hipStream_t s) {
    if (a.n <= 0) return;
    hipLaunchKernelGGL(depth_update_kernel, dim3((a.n + kDfWaves - 1) / kDfWaves), dim3(64 * kDfWaves), 0, s, a);
    hipLaunchKernelGGL(depth_compact_kernel, dim3(1), dim3(1024), 0, s, a);
}

}  // namespace svo
