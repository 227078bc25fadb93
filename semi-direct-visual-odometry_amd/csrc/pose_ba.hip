// pose_ba.hip — BundleAdjustment::optimizePose (src/bundle_adjustment.cpp:35-166) for a batch of frames.
//
// One 512-thread workgroup per frame runs the reference's single LM step (Optimizer::optimizeLM<SE3d>,
// src/optimizer.cpp:162-370, which always leaves after the first damped step):
//   residuals  computeResidualsPose (:101-134) for the features the PREVIOUS call's Jacobian functor
//              marked visible (m_refVisibility, carried by the caller): |bearing - normalise(T P)| as
//              three rows per feature, only the third row visible; the other M - 3*nvis rows DBL_MAX;
//   scale      Tukey sigma from the median and MAD over all M = 3n rows (algorithm::computeMedian on
//              the full vector, src/algorithm.cpp:834-872): exact order statistics by an 8-pass radix
//              select over the doubles' bit patterns (all rows are >= 0) with LDS histograms;
//   weights    Tukey, chi^2 over the visible rows;
//   Jacobian   computeJacobianPose (:71-98): row block 3*cp of the cp-th feature with a point; rows and
//              residuals pair by index, as in the reference (J^T W J over rows);
//   step       H = J^T W J, g = J^T W r (only the visible third rows carry weight: J row (0,0,1,y,-x,0)),
//              Nielsen lambda = 1e-2 * max diag, Eigen LDLT, pose <- exp(dx) * pose (:162-166), status.
// Bound: latency of the dependent selection passes (one workgroup per frame); the frame's rows are
// read from L2-resident scratch 8 times per selection.
#include <cfloat>

#include "svo_internal.h"
#include "svo_math.h"

namespace svo {

namespace {

constexpr int kThreads = 512;

__device__ __forceinline__ uint64_t dbits(double v) { return (uint64_t)__double_as_longlong(v); }

// k-th smallest (0-based) of the m values v(i) >= 0 (mad: |rows[i] - med|), by their bit patterns
template <bool kMad>
__device__ double select_kth(const double* rows, int m, double med, uint32_t k, uint32_t* hist, uint64_t* sh) {
    uint64_t prefix = 0, mask = 0;
    const int lane = threadIdx.x & 63;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < m; i += kThreads) {
            const double v = kMad ? fabs(rows[i] - med) : rows[i];
            const uint64_t key = dbits(v);
            if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) {  // wave 0: which bin holds rank k
            const uint32_t c0 = hist[4 * lane], c1 = hist[4 * lane + 1], c2 = hist[4 * lane + 2], c3 = hist[4 * lane + 3];
            const uint32_t mine = c0 + c1 + c2 + c3;
            uint32_t inc = mine;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d, 64);
                if (lane >= d) inc += y;
            }
            const uint32_t before = inc - mine;
            if (k >= before && k < inc) {
                uint32_t r = k - before, bin = 4 * lane;
                if (r >= c0) { r -= c0; bin++;
                    if (r >= c1) { r -= c1; bin++;
                        if (r >= c2) { r -= c2; bin++; } } }
                sh[0] = prefix | ((uint64_t)bin << shift);
                sh[1] = r;
            }
        }
        __syncthreads();
        prefix = sh[0];
        k = (uint32_t)sh[1];
        mask |= (uint64_t)255 << shift;
        __syncthreads();
    }
    return __longlong_as_double((long long)prefix);
}

// algorithm::computeMedian over m rows with n_valid (odd / even by the total length; exact neighbour).
// The neighbour below rank mid is hi itself when fewer than mid rows are smaller, else the largest
// smaller row: one counting pass instead of a second selection.
template <bool kMad>
__device__ double median_rows(const double* rows, int m, double med, uint32_t n_valid, uint32_t* hist, uint64_t* sh) {
    const uint32_t mid = n_valid / 2;
    const double hi = select_kth<kMad>(rows, m, med, mid, hist, sh);
    if ((m & 1) || mid == 0) return hi;
    const uint64_t hk = dbits(hi);
    uint32_t less = 0;
    uint64_t below = 0;
    for (int i = threadIdx.x; i < m; i += kThreads) {
        const uint64_t key = dbits(kMad ? fabs(rows[i] - med) : rows[i]);
        if (key < hk) {
            ++less;
            below = key > below ? key : below;
        }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        less += __shfl_xor(less, d, 64);
        const uint64_t o = (uint64_t)__shfl_xor((long long)below, d, 64);
        below = o > below ? o : below;
    }
    if ((threadIdx.x & 63) == 0) {
        hist[threadIdx.x >> 6] = less;
        sh[0] = 0;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long*)&sh[0], (unsigned long long)below);
    __syncthreads();
    uint32_t cnt = 0;
    for (int w = 0; w < kThreads / 64; ++w) cnt += hist[w];
    const double lo = cnt == mid ? __longlong_as_double((long long)sh[0]) : hi;
    __syncthreads();
    return (lo + hi) / 2.0;
}

__global__ void __launch_bounds__(kThreads) pose_ba_kernel(PoseBAArgs a) {
    __shared__ uint32_t hist[256];
    __shared__ uint64_t sh[2];
    __shared__ int32_t scan_sh[kThreads / 64 + 1];
    __shared__ double red[kThreads / 64][28];
    const int f = blockIdx.x;
    const int32_t off = a.feat_off[f], n = a.feat_off[f + 1] - off;
    const int32_t m = 3 * n;
    double* rows = a.rows + 3 * (int64_t)off;  // M residual rows of this frame
    double* wts = a.wts + off;                 // weight of visible row 3j+2, by j
    const double* bearing = a.bearing + 3 * (int64_t)off;
    const double* point = a.point + 3 * (int64_t)off;
    const uint8_t* has_point = a.has_point + off;
    const uint8_t* vis_in = a.vis_in + off;
    const SE3 T = se3_load(a.poses + 7 * (int64_t)f);
    if (n == 0 || m < 6) {  // :37-38 (return 0, nothing run) / Non_Suff_Points (src/optimizer.cpp:173-174)
        for (int k = threadIdx.x; k < n; k += kThreads) a.vis_out[off + k] = vis_in[k];
        if (threadIdx.x == 0) {
            se3_store(T, a.poses_out + 7 * (int64_t)f);
            a.err[f] = n == 0 ? 0.0 : -1.0;
            a.status[f] = n == 0 ? -1 : SVO_STATUS_NON_SUFF_POINTS;
        }
        return;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // ---- residual rows of the stale-visible features, ranked in feature order
    int32_t nvis = 0;
    for (int base = 0; base < n; base += kThreads) {
        const int k = base + threadIdx.x;
        const int v = (k < n && vis_in[k]) ? 1 : 0;
        int inc = v;
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) scan_sh[wave] = inc;
        __syncthreads();
        int before = nvis;
        for (int w = 0; w < wave; ++w) before += scan_sh[w];
        int chunk = 0;
        for (int w = 0; w < kThreads / 64; ++w) chunk += scan_sh[w];
        if (v) {
            const int j = before + inc - 1;
            const V3 pc = se3_act(T, {point[3 * k], point[3 * k + 1], point[3 * k + 2]});
            const double sq = pc.x * pc.x + pc.y * pc.y + pc.z * pc.z;  // Eigen normalized()
            V3 u = pc;
            if (sq > 0.0) {
                const double s = sqrt(sq);
                u = {pc.x / s, pc.y / s, pc.z / s};
            }
            rows[3 * j] = fabs(bearing[3 * k] - u.x);
            rows[3 * j + 1] = fabs(bearing[3 * k + 1] - u.y);
            rows[3 * j + 2] = fabs(bearing[3 * k + 2] - u.z);
        }
        nvis += chunk;
        __syncthreads();
    }
    for (int i = 3 * nvis + threadIdx.x; i < m; i += kThreads) rows[i] = DBL_MAX;
    __syncthreads();
    const uint32_t n_proj = 3u * (uint32_t)nvis;
    // ---- Tukey scale (Optimizer::tukeyWeighting, src/optimizer.cpp:485-514)
    const double med = median_rows<false>(rows, m, 0.0, n_proj, hist, sh);
    const double mad = median_rows<true>(rows, m, med, n_proj, hist, sh);
    double sigma = 1.482602218505602 * mad;
    if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
    const double c = 4.6851 * sigma, c2 = c * c;
    // ---- weights of the visible rows; normal equations over the point features' Jacobian rows
    double acc[28];
#pragma unroll
    for (int i = 0; i < 28; ++i) acc[i] = 0.0;
    for (int j = threadIdx.x; j < nvis; j += kThreads) {
        const double r = rows[3 * j + 2];
        double w = 0.0;
        if (fabs(r) <= c) {
            const double t = 1.0 - (r * r) / c2;
            w = t * t;
        }
        wts[j] = w;
        acc[27] += r * r * w;  // chi^2
    }
    __syncthreads();
    int32_t cp_base = 0;
    for (int base = 0; base < n; base += kThreads) {
        const int k = base + threadIdx.x;
        const int v = (k < n && has_point[k]) ? 1 : 0;
        int inc = v;
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
        }
        if (lane == 63) scan_sh[wave] = inc;
        __syncthreads();
        int before = cp_base;
        for (int w = 0; w < wave; ++w) before += scan_sh[w];
        int chunk = 0;
        for (int w = 0; w < kThreads / 64; ++w) chunk += scan_sh[w];
        if (k < n) a.vis_out[off + k] = (uint8_t)v;  // resetParameters + the Jacobian functor's flags
        if (v) {
            const int cp = before + inc - 1;
            if (cp < nvis) {  // rows 3cp, 3cp+1 carry no weight; row 3cp+2 = (0, 0, 1, y, -x, 0)
                const double w = wts[cp];
                const double r = rows[3 * cp + 2];
                const V3 X = se3_act(T, {point[3 * k], point[3 * k + 1], point[3 * k + 2]});
                const double J[6] = {0.0, 0.0, 1.0, X.y, -X.x, 0.0};
                int t = 0;
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double jw = J[i] * w;
#pragma unroll
                    for (int jj = i; jj < 6; ++jj) acc[t++] += jw * J[jj];
                    acc[21 + i] += jw * r;
                }
            }
        }
        cp_base += chunk;
        __syncthreads();
    }
    // ---- block reduction of the 21 + 6 + 1 sums
#pragma unroll
    for (int i = 0; i < 28; ++i) {
        double v = acc[i];
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        if (lane == 0) red[wave][i] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double s[28];
    for (int i = 0; i < 28; ++i) {
        s[i] = red[0][i];
        for (int w = 1; w < kThreads / 64; ++w) s[i] += red[w][i];
    }
    double H[36], g[6], dx[6];
    int t = 0;
    for (int i = 0; i < 6; ++i)
        for (int jj = i; jj < 6; ++jj) { H[i * 6 + jj] = s[t]; H[jj * 6 + i] = s[t]; ++t; }
    for (int i = 0; i < 6; ++i) g[i] = s[21 + i];
    const double chi = s[27];
    double mx = H[0];
    for (int i = 1; i < 6; ++i) mx = fmax(mx, H[i * 6 + i]);
    const double lambda = 1e-2 * mx;  // Nielsen, first iteration (src/optimizer.cpp:296-301)
    for (int i = 0; i < 6; ++i) H[i * 6 + i] += lambda;
    ldlt_solve(6, H, g, dx);
    const SE3 Tn = se3_compose(se3_exp(dx), T);  // updatePose: exp(dx) * pose
    bool big = false, nan = false;
    double step = 0.0;
    for (int i = 0; i < 6; ++i) {
        big |= dx[i] > 1e3;
        nan |= isnan(dx[i]);
        step += dx[i] * dx[i];
    }
    int32_t st = SVO_STATUS_SUCCESS;
    if (big) st = SVO_STATUS_MAX_COFF_DX;
    else if (nan) st = SVO_STATUS_NON_IN_DX;
    else {
        st = step < 1e-16 ? SVO_STATUS_SMALL_STEP_SIZE : st;
        st = fabs(lambda) >= 1e14 ? SVO_STATUS_LAMBDA_VALUE : st;
    }
    se3_store(Tn, a.poses_out + 7 * (int64_t)f);
    a.err[f] = sqrt(chi / (double)n_proj);
    a.status[f] = st;
}

}  // namespace

void launch_pose_ba(const PoseBAArgs& a, hipStream_t s) {
    if (a.n_frames > 0) hipLaunchKernelGGL(pose_ba_kernel, dim3(a.n_frames), dim3(kThreads), 0, s, a);
}

}  // namespace svo
