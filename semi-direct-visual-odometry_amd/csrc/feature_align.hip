// feature_align.hip — FeatureAlignment::align (src/feature_alignment.cpp:25-62) for a batch of candidates.
//
// One 64-lane wave per candidate: the (2h+1)^2 patch (49 px at the reference's patch 7, src/map.cpp:18)
// maps onto the wave's lanes.  Everything a lane computes is the reference's per-pixel arithmetic on the
// level-0 GRADIENT images (float-rounded bilinear, src/algorithm.cpp:885-894); the order statistics for
// the Tukey scale are exact order statistics (a bitonic sort over the wave; the patch area is odd, so the
// reference's median is an exact order statistic too); chi2, J^T W J and J^T W r are then summed in row
// order, the reference's own order (src/optimizer.cpp:279-280), one accumulator per lane, so the 3x3
// system is bit-identical to the CPU restatement.  Solve: Nielsen damping + Eigen-LDLT; update flow += dx (:200-205).
#include "svo_internal.h"
#include "svo_math.h"

namespace svo {

namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kMaxArea = 128;

struct WaveLds {
    double r[kMaxArea];
    double v[kMaxArea];
    double w[kMaxArea];
    double jx[kMaxArea];
    double jy[kMaxArea];
    double med;
    double sel;
};

__device__ __forceinline__ bool in_frame(double x, double y, double b, int W, int H) {  // src/pinhole_camera.cpp:163-168
    return x >= b && y >= b && x < W - b && y < H - b;
}

// k-th smallest (0-based) of v[0..m) (m <= 128) held in LDS; every lane returns it.  Bitonic sort of
// the m values (padded with +inf) over the wave's 64 lanes x 2 registers: element e = 64 * reg + lane;
// partners 64 apart are in the same lane, the others one lane-xor away.
__device__ __forceinline__ double shfl_xor_d(double v, int m) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl_xor((int)(b & 0xffffffff), m, 64), hi = __shfl_xor((int)(b >> 32), m, 64);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ double wave_kth(WaveLds& L, int m, int k) {
    const int lane = threadIdx.x & 63;
    double x0 = lane < m ? L.v[lane] : __builtin_inf();
    double x1 = lane + 64 < m ? L.v[lane + 64] : __builtin_inf();
#pragma unroll
    for (int size = 2; size <= 128; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride == 64) {  // size 128: ascending, partner in the other register
                const double lo = fmin(x0, x1), hi = fmax(x0, x1);
                x0 = lo;
                x1 = hi;
            } else {
                const double p0 = shfl_xor_d(x0, stride), p1 = shfl_xor_d(x1, stride);
                const bool lower = (lane & stride) == 0;
                const bool asc0 = (lane & size) == 0, asc1 = ((lane + 64) & size) == 0;
                // keep the min where (lower == ascending), else the max
                x0 = (lower == asc0) ? fmin(x0, p0) : fmax(x0, p0);
                x1 = (lower == asc1) ? fmin(x1, p1) : fmax(x1, p1);
            }
        }
    }
    const double mine = k < 64 ? x0 : x1;
    return __shfl(mine, k & 63, 64);
}

}  // namespace

__global__ void __launch_bounds__(64 * kWavesPerBlock) feature_align_kernel(FeatureAlignArgs a) {
    __shared__ WaveLds lds[kWavesPerBlock];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = blockIdx.x * kWavesPerBlock + wv;
    WaveLds& L = lds[wv];
    const bool active = i < a.n;  // whole waves are active or not; all waves still reach every barrier
    const int A = a.area, h = a.half, side = 2 * a.half + 1;
    const int W = a.width, H = a.height;
    const double border = h + 2;
    const double DMAX = 1.7976931348623157e308;

    const uint8_t* gref = nullptr;
    const uint8_t* gcur = a.cur_grad;
    double rx = 0, ry = 0, fx = 0, fy = 0;
    if (active) {
        gref = a.ref_grad[i];
        rx = a.ref_px[2 * i]; ry = a.ref_px[2 * i + 1];
        fx = a.px[2 * i]; fy = a.px[2 * i + 1];
    }
    const bool ref_in = active && in_frame(rx, ry, border, W, H);
    const bool cur_in = active && in_frame(fx, fy, border, W, H);
    const int n = cur_in ? A : 0;

    // computeJacobian (:64-110) + computeResiduals (:113-168)
    for (int k = lane; k < A; k += 64) {
        const int ky = k / side - h, kx = k - (k / side) * side - h;
        double T = 0.0, jx = 0.0, jy = 0.0;
        if (ref_in) {
            const double row = ry + ky, col = rx + kx;
            T = (double)bilinear_f(gref, W, col, row);
            jx = 0.5 * (bilinear_f(gref, W, col + 1, row) - bilinear_f(gref, W, col - 1, row));
            jy = 0.5 * (bilinear_f(gref, W, col, row + 1) - bilinear_f(gref, W, col, row - 1));
        }
        double r = DMAX;
        if (cur_in) {
            const double cur = (double)bilinear_f(gcur, W, fx + kx, fy + ky);
            r = -(cur - T + 0.0);
        }
        L.r[k] = r;
        L.v[k] = r;
        L.jx[k] = jx;
        L.jy[k] = jy;
    }
    __syncthreads();
    // tukeyWeighting -> computeSigma(r, n) with the full-length vector (A entries, A odd)
    const int mid = n / 2;
    const double med = wave_kth(L, A, mid);
    for (int k = lane; k < A; k += 64) L.v[k] = fabs(L.r[k] - med);
    __syncthreads();
    const double mad = wave_kth(L, A, mid);
    double sigma = 1.482602218505602 * mad;
    if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
    const double c = 4.6851 * sigma, c2 = c * c;
    for (int k = lane; k < A; k += 64) {
        double w = 0.0;
        if (cur_in) {
            const double r = L.r[k];
            if (fabs(r) <= c) {
                const double t = 1.0 - (r * r) / c2;
                w = t * t;
            }
        }
        L.w[k] = w;
    }
    __syncthreads();
    // chi2, J^T W J and J^T W r in row order (src/optimizer.cpp:279-280, :470-483), one accumulator per
    // lane: lanes 0-8 H[p][q] += (J_p w) J_q, lanes 9-11 g[p] += (J_p w) r, lane 12 chi += r r w; rows
    // with w == 0 add nothing to H and g (as the CPU restatement skips them)
    double acc = 0.0;
    if (active && cur_in && lane < 13) {
        const int p = lane < 9 ? lane / 3 : lane - 9, q = lane < 9 ? lane % 3 : 0;
        const double J2 = ref_in ? 1.0 : 0.0;
        for (int k = 0; k < A; ++k) {
            const double r = L.r[k], w = L.w[k];
            if (lane == 12) {
                acc += r * r * w;
            } else if (w != 0.0) {
                const double jx = L.jx[k], jy = L.jy[k];
                const double jw = (p == 0 ? jx : (p == 1 ? jy : J2)) * w;
                acc += jw * (lane < 9 ? (q == 0 ? jx : (q == 1 ? jy : J2)) : r);
            }
        }
    }
    double sums[13];
#pragma unroll
    for (int t = 0; t < 13; ++t) sums[t] = __shfl(acc, t, 64);
    if (active && lane == 0) {
        double Hm[9], g[3];
        for (int t = 0; t < 9; ++t) Hm[t] = sums[t];
        for (int t = 0; t < 3; ++t) g[t] = sums[9 + t];
        const double chi = sums[12];
        double mx = Hm[0];
        mx = fmax(mx, Hm[4]);
        mx = fmax(mx, Hm[8]);
        const double lambda = 1e-2 * mx;
        for (int p = 0; p < 3; ++p) Hm[p * 4] += lambda;
        double dx[3];
        ldlt_solve(3, Hm, g, dx);
        const double nx = fx + dx[0], ny = fy + dx[1];
        bool big = false, nan = false;
        for (int p = 0; p < 3; ++p) { big |= dx[p] > 1e3; nan |= isnan(dx[p]); }
        int32_t st = kSuccess;
        if (big) st = kMaxCoffDx;
        else if (nan) st = kNonInDx;
        else {
            const double step = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
            st = step < 1e-16 ? kSmallStepSize : st;
            st = fabs(lambda) >= 1e14 ? kLambdaValue : st;
        }
        a.px[2 * i] = nx;
        a.px[2 * i + 1] = ny;
        a.err[i] = sqrt(chi / (double)n);
        a.status[i] = st;
    }
}

void launch_feature_align(const FeatureAlignArgs& a, hipStream_t s) {
    const int blocks = (a.n + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0) hipLaunchKernelGGL(feature_align_kernel, dim3(blocks), dim3(64 * kWavesPerBlock), 0, s, a);
}

}  // namespace svo
