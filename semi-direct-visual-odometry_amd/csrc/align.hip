// align.hip — sparse image alignment (ImageAlignment::align, src/image_alignment.cpp:25-67) on gfx950.
//
// One 512-thread workgroup owns one frame pair for the whole coarse-to-fine call.  Pairs are
// independent: no workgroup talks to another, a batch is one launch, and with
// <= 128 VGPRs and ~70 KB of LDS two pairs share a CU.  Per level:
//   P1  thread / feature : ref visibility (border rule :140-149), projection pose*X_w into cur (:320-340),
//                          image Jacobian at the WORLD point (:163, :194-248) -> per-feature scratch
//   S1  lane group / feature (32 lanes for the 25 px of patch 5, 64 for patch 7), kUnroll feature
//                          groups per wave iteration so their loads overlap: the feature's ref window
//                          ((2h+5)^2 px) and cur window ((2h+3)^2 px) are staged in LDS with a few byte
//                          loads, then every lane samples its pixel: r = I_cur - T_ref (:359); r goes to a
//                          per-pair scratch row (+inf = invisible slot), its value bin to an LDS histogram
//   S2  exact median (src/algorithm.cpp:834-853): the histogram names the bin of rank n/2; one sweep
//                          gathers that bin's values (plus the max below it) into LDS; exact rank there
//   S3/S4  the same for |r - median| -> MAD -> sigma = 1.482602218505602 * MAD (:855-872)
//   S5  lane group / feature : Tukey weight (src/optimizer.cpp:485-514), chi2, dx/dy re-sampled from the
//                          staged ref window, per-feature sums S_xx S_xy S_yy S_xr S_yr (shuffles in the
//                          lane group) -> per-feature scratch
//   P5b thread / feature : expand the 5 sums with the 2x6 image Jacobian into the lower triangle of
//                          J^T W J and J^T W r (factorised J row = dx*Jimg0 + dy*Jimg1); wave shuffles +
//                          fixed-order LDS tree -> deterministic, no atomics
//   P6  one lane          : Nielsen damping, Eigen-LDLT (LDS workspace), pose <- pose * exp(-dx),
//                          status, RMSE (src/optimizer.cpp:279-366, src/image_alignment.cpp:379)
// Exact order statistics: values are binned by a monotone map, so the bin of rank k and its
// population are exact; a bin with more than kCandCap values falls back to an 11-bit radix select
// on order-preserving uint64 keys restricted to that bin.
#include "svo_internal.h"
#include "svo_math.h"

namespace svo {

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kBins = 4096;
constexpr double kBinScale = 32.0;   // bins per grey level
constexpr double kBinOffset = 64.0;  // signed map covers [-64, 64); outliers clamp to the end bins
constexpr int kCandCap = 4096;
constexpr int kRankCap = 256;        // <= this many candidates: rank counting, else bitonic sort
constexpr int kWinBytes = 2048;      // per-wave staging buffer
constexpr int kUnroll = 4;           // feature groups in flight per wave iteration
constexpr int kRadixBits = 11;

struct Shared {
    uint32_t hist[kBins];
    double cand[kCandCap];
    uint8_t win[kWaves][kWinBytes];
    double red[kWaves][30];
    double accw[kWaves][28];  // per-wave J^T W J (21, lower) | J^T W r (6) | chi2
    double part[kThreads / 32][28];  // P5b partial sums per (feature chunk, term)
    double tot[28];
    uint32_t ired[kWaves][4];
    uint32_t scan[kThreads];
    double A[36];
    double tmp[6];
    int32_t perm[6];
    SE3 pose;
    uint64_t sel_prefix;
    uint32_t sel_k, sel_cnt, sel_bits, sel_bin, cand_n;
    double sel_hi, sel_lo;
};

__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_down(v, o, 64));
    return v;
}
__device__ __forceinline__ void wave_lds_sync() {  // this wave's LDS writes -> visible to its own lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// x / d for small x via a 32-bit magic multiplier (exact for x * d < 2^32)
__device__ __forceinline__ uint32_t magic_of(uint32_t d) { return (uint32_t)((0x100000000ull + d - 1) / d); }
__device__ __forceinline__ uint32_t udiv(uint32_t x, uint32_t m) { return __umulhi(x, m); }

// block-wide sums of 2 counters, valid in every thread
__device__ void block_sum_u2(Shared& sh, uint32_t& a, uint32_t& b) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    a = wave_sum_u(a);
    b = wave_sum_u(b);
    if (lane == 0) { sh.ired[wave][0] = a; sh.ired[wave][1] = b; }
    __syncthreads();
    a = 0; b = 0;
    for (int w = 0; w < kWaves; ++w) { a += sh.ired[w][0]; b += sh.ired[w][1]; }
    __syncthreads();
}

// selection value of a residual slot: kMad ? |r - med| : r   (monotone bin map per mode)
template <bool kMad>
__device__ __forceinline__ double sel_val(double r, double med) { return kMad ? fabs(r - med) : r; }
template <bool kMad>
__device__ __forceinline__ int sel_bin(double v) {
    const double t = kMad ? v * kBinScale : (v + kBinOffset) * kBinScale;
    return t < 0.0 ? 0 : (t >= (double)(kBins - 1) ? kBins - 1 : (int)t);
}

// Sweep the residual row with 4 x 16-B loads in flight per lane; fn(value, slot-valid) for each slot.
// res[M] is +inf when M is odd, so pairs never read past the row.
template <typename Fn>
__device__ __forceinline__ void sweep_res(const double* __restrict__ res, int M, Fn fn) {
    const int tid = threadIdx.x;
    for (int base = 2 * tid; base < M; base += 8 * kThreads) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int s2 = base + u * 2 * kThreads;
            v[u] = s2 < M ? *reinterpret_cast<const double2*>(res + s2) : make_double2(__builtin_inf(), __builtin_inf());
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (v[u].x != __builtin_inf()) fn(v[u].x);
            if (v[u].y != __builtin_inf()) fn(v[u].y);
        }
    }
}

// bin holding rank sh.sel_k of hist -> sh.sel_bin, sh.sel_k (rank inside the bin), sh.sel_cnt
__device__ void find_bin(Shared& sh, const uint32_t* hist, int bins) {
    const int tid = threadIdx.x;
    const uint32_t k = sh.sel_k;
    const int per = (bins + kThreads - 1) / kThreads;
    uint32_t local = 0;
    for (int i = 0; i < per; ++i) {
        const int b = tid * per + i;
        if (b < bins) local += hist[b];
    }
    // block exclusive scan of the per-thread counts: wave scan + wave totals
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t incl = local;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) sh.scan[wave] = incl;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; ++w) off += sh.scan[w];
    incl += off;
    const uint32_t excl = incl - local;
    if (k >= excl && k < incl) {
        uint32_t run = excl;
        for (int i = 0; i < per; ++i) {
            const int b = tid * per + i;
            const uint32_t c = b < bins ? hist[b] : 0;
            if (k < run + c) {
                sh.sel_bin = (uint32_t)b;
                sh.sel_k = k - run;
                sh.sel_cnt = c;
                break;
            }
            run += c;
        }
    }
    __syncthreads();
}

// k-th and (k-1)-th smallest of cand[0..n) (k-1 only if want_lo and k > 0)
__device__ void cand_select(Shared& sh, uint32_t n, uint32_t kk, bool want_lo) {
    const int tid = threadIdx.x;
    if (n <= (uint32_t)kRankCap) {
        for (uint32_t i = tid; i < n; i += kThreads) {
            const double vi = sh.cand[i];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < n; ++j) {
                const double vj = sh.cand[j];
                rank += (vj < vi) | ((vj == vi) & (j < i));
            }
            if (rank == kk) sh.sel_hi = vi;
            if (want_lo && rank + 1 == kk) sh.sel_lo = vi;
        }
        __syncthreads();
        return;
    }
    uint32_t p2 = 1;
    while (p2 < n) p2 <<= 1;
    for (uint32_t i = n + tid; i < p2; i += kThreads) sh.cand[i] = __builtin_inf();
    __syncthreads();
    for (uint32_t size = 2; size <= p2; size <<= 1)
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t i = tid; i < p2 / 2; i += kThreads) {
                const uint32_t lo = (i / stride) * stride * 2 + (i % stride), hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const double a = sh.cand[lo], b = sh.cand[hi];
                if ((a > b) == asc) { sh.cand[lo] = b; sh.cand[hi] = a; }
            }
            __syncthreads();
        }
    if (tid == 0) {
        sh.sel_hi = sh.cand[kk];
        if (want_lo && kk > 0) sh.sel_lo = sh.cand[kk - 1];
    }
    __syncthreads();
}

// radix fallback inside one overfull bin: exact k-th among values v with sel_bin(v) == bin
template <bool kMad>
__device__ double radix_in_bin(Shared& sh, const double* __restrict__ res, int M, uint32_t bin, uint32_t k, double med) {
    const int tid = threadIdx.x;
    if (tid == 0) { sh.sel_prefix = 0; sh.sel_bits = 0; sh.sel_k = k; }
    __syncthreads();
    while (sh.sel_bits < 64) {
        const int bits = sh.sel_bits;
        const int dbits = (64 - bits) < kRadixBits ? (64 - bits) : kRadixBits;
        const uint64_t prefix = sh.sel_prefix;
        const int shift = 64 - bits - dbits;
        for (int i = tid; i < (1 << dbits); i += kThreads) sh.hist[i] = 0;
        __syncthreads();
        sweep_res(res, M, [&](double r) {
            const double v = sel_val<kMad>(r, med);
            if ((uint32_t)sel_bin<kMad>(v) != bin) return;
            const uint64_t key = dkey(v);
            if (bits == 0 || (key >> (64 - bits)) == prefix)
                atomicAdd(&sh.hist[(key >> shift) & ((1u << dbits) - 1)], 1u);
        });
        __syncthreads();
        find_bin(sh, sh.hist, 1 << dbits);
        if (tid == 0) {
            sh.sel_prefix = (sh.sel_prefix << dbits) | sh.sel_bin;
            sh.sel_bits += dbits;
        }
        __syncthreads();
    }
    const double v = dkey_inv(sh.sel_prefix);
    __syncthreads();
    return v;
}

// (k-1)-th order statistic from the k-th (hi): hi itself if at most k-1 values are < hi, else max(<hi)
template <bool kMad>
__device__ double lower_neighbour_sweep(Shared& sh, const double* __restrict__ res, int M, uint32_t k, double hi,
                                        double med) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t less = 0;
    double mx = -__builtin_inf();
    sweep_res(res, M, [&](double r) {
        const double v = sel_val<kMad>(r, med);
        if (v < hi) { ++less; mx = fmax(mx, v); }
    });
    less = wave_sum_u(less);
    mx = wave_max(mx);
    if (lane == 0) { sh.ired[wave][0] = less; sh.red[wave][0] = mx; }
    __syncthreads();
    uint32_t tl = 0;
    double tm = -__builtin_inf();
    for (int w = 0; w < kWaves; ++w) { tl += sh.ired[w][0]; tm = fmax(tm, sh.red[w][0]); }
    __syncthreads();
    return (tl <= k - 1) ? hi : tm;
}

// computeMedian(v, n) with exact order statistics (odd/even decided by the TOTAL length M,
// src/algorithm.cpp:845-851; mid == 0 reads vec[mid]).  sh.hist holds the value-bin histogram.
template <bool kMad>
__device__ double block_median(Shared& sh, const double* __restrict__ res, int M, uint32_t n, double med) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t mid = n / 2;
    const bool want_lo = ((M & 1) == 0) && mid > 0;
    if (tid == 0) { sh.sel_k = mid; sh.cand_n = 0; }
    __syncthreads();
    find_bin(sh, sh.hist, kBins);
    const uint32_t bin = sh.sel_bin, kk = sh.sel_k, cnt = sh.sel_cnt;
    double hi, lo = 0.0;
    if (cnt <= (uint32_t)kCandCap) {
        double below = -__builtin_inf();
        sweep_res(res, M, [&](double r) {
            const double v = sel_val<kMad>(r, med);
            const uint32_t b = (uint32_t)sel_bin<kMad>(v);
            if (b == bin) sh.cand[atomicAdd(&sh.cand_n, 1u)] = v;
            else if (b < bin) below = fmax(below, v);
        });
        below = wave_max(below);
        if (lane == 0) sh.red[wave][0] = below;
        __syncthreads();
        double tb = -__builtin_inf();
        for (int w = 0; w < kWaves; ++w) tb = fmax(tb, sh.red[w][0]);
        cand_select(sh, cnt, kk, want_lo);
        hi = sh.sel_hi;
        if (want_lo) lo = kk > 0 ? sh.sel_lo : tb;
        __syncthreads();
    } else {
        hi = radix_in_bin<kMad>(sh, res, M, bin, kk, med);
        if (want_lo) lo = lower_neighbour_sweep<kMad>(sh, res, M, mid, hi, med);
    }
    return want_lo ? (lo + hi) / 2.0 : hi;
}

// bilinearInterpolationDouble (src/algorithm.cpp:896-905) reading a staged window whose top-left
// image pixel is (ox, oy); cells past the image edge hold 0 and only ever carry a zero weight.
__device__ __forceinline__ double bilerp_win(const uint8_t* win, int ww, int ox, int oy, double x, double y) {
    const int32_t x1 = (int32_t)x, y1 = (int32_t)y, x2 = x1 + 1, y2 = y1 + 1;
    const uint8_t* r1 = win + (y1 - oy) * ww - ox;
    const uint8_t* r2 = r1 + ww;
    const double a = (x2 - x) * r1[x1] + (x - x1) * r1[x2];
    const double b = (x2 - x) * r2[x1] + (x - x1) * r2[x2];
    return (y2 - y) * a + (y - y1) * b;
}

// ww x ww window of an image plane (row pitch W) starting at (ox, oy) -> dst, by the lpf lanes of a group
__device__ __forceinline__ void stage_window(uint8_t* dst, const uint8_t* img, int W, int H, int ox, int oy, int ww,
                                             uint32_t mww, int sub, int lpf) {
    const int64_t plane = (int64_t)W * H;
    for (int i = sub; i < ww * ww; i += lpf) {
        const int ry = (int)udiv((uint32_t)i, mww), rx = i - ry * ww;
        const int64_t lin = (int64_t)(oy + ry) * W + (ox + rx);
        dst[i] = (lin >= 0 && lin < plane) ? img[lin] : (uint8_t)0;
    }
}

// One damped Gauss-Newton step from the reduced sums in sh.tot (src/optimizer.cpp:279-334):
// lambda = 1e-2 * max diag(H); H_ii += lambda; dx = LDLT(H) \ g; pose <- pose * exp(-dx);
// status as the reference's single iteration leaves it; err = sqrt(chi2 / n) at the pre-update pose.
__device__ __attribute__((noinline)) void lm_step(Shared& sh, svo_level_trace& t, uint32_t n, double med, double mad,
                                                  double sigma) {
    double g[6], dx[6];
    int q = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j <= i; ++j) {
            const double v = sh.tot[q++];
            sh.A[i * 6 + j] = v;
            sh.A[j * 6 + i] = v;
        }
    for (int i = 0; i < 6; ++i) g[i] = sh.tot[21 + i];
    const double chi = sh.tot[27];
    double mx = sh.A[0];
    for (int i = 1; i < 6; ++i) mx = fmax(mx, sh.A[i * 7]);
    const double lambda = 1e-2 * mx;
    for (int i = 0; i < 6; ++i) sh.A[i * 7] += lambda;
    for (int i = 0; i < 36; ++i) t.H[i] = sh.A[i];
    ldlt_solve_ws(6, sh.A, g, dx, sh.perm, sh.tmp);
    double m[6];
    for (int i = 0; i < 6; ++i) m[i] = -dx[i];
    sh.pose = se3_compose(sh.pose, se3_exp(m));
    bool big = false, nan = false;
    for (int i = 0; i < 6; ++i) { big |= dx[i] > 1e3; nan |= isnan(dx[i]); }
    int32_t st = kSuccess;
    if (big) st = kMaxCoffDx;
    else if (nan) st = kNonInDx;
    else {
        double step = 0.0;
        for (int i = 0; i < 6; ++i) step += dx[i] * dx[i];
        st = step < 1e-16 ? kSmallStepSize : st;
        st = fabs(lambda) >= 1e14 ? kLambdaValue : st;
    }
    const double e = sqrt(chi / (double)n);
    t.n_vis = (int32_t)n; t.status = st;
    t.median = med; t.mad = mad; t.sigma = sigma; t.chi2 = chi; t.lambda = lambda; t.err = e;
    for (int i = 0; i < 6; ++i) { t.g[i] = g[i]; t.dx[i] = dx[i]; }
    sh.red[0][28] = e;
    sh.ired[0][3] = (uint32_t)st;
}

}  // namespace

// kStamps: diagnostic build (SVO_PHASE_STAMPS=1) — lane 0 writes s_memtime at each phase boundary to
// a.stamps[pair][level][8]; no stamp executes in the production instantiation.
#define SVO_STAMP(i) \
    if (kStamps && tid == 0) a.stamps[((int64_t)pair * (a.max_level + 1) + level) * 8 + (i)] = __builtin_amdgcn_s_memtime()

// kHalf: patch half size as a compile-time constant (the reference's patch p has h = p / 2 and a
// (2h+1)^2 footprint); the launcher instantiates h = 0..9.
template <int kHalf, bool kStamps>
__global__ void __launch_bounds__(kThreads, 4) align_pairs_kernel(AlignArgs a) {
    __shared__ Shared sh;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pair = blockIdx.x;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf;
    constexpr int h = kHalf, side = 2 * kHalf + 1, A = side * side;
    const int M = nf * A;
    // lane groups: lpf lanes per feature, fpw features per wave, U groups per wave iteration
    constexpr int lpf = A <= 16 ? 16 : (A <= 32 ? 32 : 64);
    constexpr int fpw = 64 / lpf;
    const int sub = lane & (lpf - 1), slotw = lane / lpf;
    constexpr int RW = 2 * h + 5, CW = 2 * h + 3, wbytes = RW * RW + CW * CW;
    constexpr int U = kUnroll < kWinBytes / (fpw * wbytes) ? kUnroll : kWinBytes / (fpw * wbytes);
    static_assert(U >= 1, "staging buffer too small for this patch size");
    const int ngroups = (nf + fpw - 1) / fpw;
    const uint32_t mside = magic_of((uint32_t)side), mrw = magic_of((uint32_t)RW), mcw = magic_of((uint32_t)CW);
    const int ky0 = sub / side - h, kx0 = sub % side - h;
    const int64_t fbase = (int64_t)pair * a.max_f;
    const double* __restrict__ px = a.px + 2 * fbase;
    const double* __restrict__ bearing = a.bearing + 3 * fbase;
    const double* __restrict__ point = a.point + 3 * fbase;
    const uint8_t* __restrict__ has_point = a.has_point + fbase;
    double* __restrict__ xw = a.xw + 3 * fbase;
    double* __restrict__ jimg = a.jimg + 12 * fbase;
    double* __restrict__ cuv = a.cuv + 2 * fbase;
    double* __restrict__ fsum = a.fsum + 5 * fbase;
    uint8_t* __restrict__ fvis = a.fvis + fbase;
    double* __restrict__ res = a.res + (int64_t)pair * a.res_stride;
    svo_level_trace* traces = a.traces + (int64_t)pair * (a.max_level + 1);

    if (tid == 0) sh.pose = se3_load(P.cur_pose);
    for (int l = tid; l <= a.max_level; l += kThreads) {
        svo_level_trace t = {};
        t.level = l;
        t.status = kFailed;
        traces[l] = t;
    }
    if (P.n_ref == 0 || M < 6) {  // align(): no ref features -> 0 (:27-28); optimizeLM: M < 6 (:173-174)
        if (tid == 0) {
            se3_store(sh.pose, a.pose_out + 7 * pair);
            a.err_out[pair] = P.n_ref == 0 ? 0.0 : -1.0;
            a.status_out[pair] = P.n_ref == 0 ? kFailed : kNonSuffPoints;
        }
        return;
    }

    // world point of every feature: X_w = T_f^-1 (bearing * |P - C_f|)   (src/image_alignment.cpp:153-155)
    {
        const SE3 Tr = se3_load(P.ref_pose), Tk = se3_load(P.kf_pose);
        const SE3 Tri = se3_inverse(Tr), Tki = se3_inverse(Tk);
        const V3 Cr = camera_in_world(Tr), Ck = camera_in_world(Tk);
        for (int f = tid; f < nf; f += kThreads) {
            if (!has_point[f]) continue;
            const bool is_ref = f < P.n_ref;
            const V3 Pw{point[3 * f], point[3 * f + 1], point[3 * f + 2]};
            const double depth = v3norm(v3sub(Pw, is_ref ? Cr : Ck));
            const V3 pc = v3scl(V3{bearing[3 * f], bearing[3 * f + 1], bearing[3 * f + 2]}, depth);
            const V3 pw = se3_act(is_ref ? Tri : Tki, pc);
            xw[3 * f] = pw.x; xw[3 * f + 1] = pw.y; xw[3 * f + 2] = pw.z;
        }
    }
    if (tid == 0 && (M & 1)) res[M] = __builtin_inf();  // pad for the 16-B sweeps
    __syncthreads();

    double err = 0.0;
    int32_t status = kFailed;
    for (int level = a.max_level; level >= a.min_level; --level) {
        SVO_STAMP(0);
        const int32_t W = a.geom.w[level], H = a.geom.h[level];
        const int64_t loff = a.geom.off[level];
        const uint8_t* __restrict__ ref_img = P.ref_pyr + loff;
        const uint8_t* __restrict__ kf_img = P.kf_pyr + loff;
        const uint8_t* __restrict__ cur_img = P.cur_pyr + loff;
        const double dom = (double)(1 << level), scale = 1.0 / dom;
        const double lfx = a.fx / dom, lfy = a.fy / dom;
        const int border = h + 2;

        // ---- P1: per-feature visibility, projection into cur, image Jacobian
        {
            const SE3 pose = sh.pose;
            uint32_t nrv = 0, ncv = 0;
            for (int f = tid; f < nf; f += kThreads) {
                uint8_t vis = 0;
                if (has_point[f]) {
                    const double u = px[2 * f] * scale, v = px[2 * f + 1] * scale;
                    const int ui = (int)floor(u), vi = (int)floor(v);
                    if (!((ui - border) < 0 || (vi - border) < 0 || (ui + border) >= W || (vi + border) >= H)) {
                        vis = 1;
                        const V3 pw{xw[3 * f], xw[3 * f + 1], xw[3 * f + 2]};
                        const V3 cp = se3_act(pose, pw);
                        const double cu = (a.fx * (cp.x / cp.z) + a.cx) * scale;
                        const double cv = (a.fy * (cp.y / cp.z) + a.cy) * scale;
                        const int cui = (int)floor(cu), cvi = (int)floor(cv);
                        if (!((cui - border) < 0 || (cvi - border) < 0 || (cui + border) >= W || (cvi + border) >= H)) {
                            vis = 3;
                            cuv[2 * f] = cu;
                            cuv[2 * f + 1] = cv;
                            double ja[6], jb[6];
                            image_jac(pw, lfx, lfy, ja, jb);
                            for (int j = 0; j < 6; ++j) { jimg[12 * f + j] = ja[j]; jimg[12 * f + 6 + j] = jb[j]; }
                        }
                    }
                }
                fvis[f] = vis;
                nrv += vis & 1;
                ncv += vis >> 1;
            }
            block_sum_u2(sh, nrv, ncv);
            if (tid == 0) {
                traces[level].n_ref_vis = (int32_t)nrv;
                sh.ired[0][2] = ncv;
            }
        }
        for (int i = tid; i < kBins; i += kThreads) sh.hist[i] = 0;
        __syncthreads();
        const uint32_t n = sh.ired[0][2] * (uint32_t)A;
        SVO_STAMP(1);

        // ---- S1: residuals through LDS-staged windows; value-bin histogram of r
        for (int g0 = wave * U; g0 < ngroups; g0 += kWaves * U) {
            int f[kUnroll], rox[kUnroll], roy[kUnroll], cox[kUnroll], coy[kUnroll];
            double ur[kUnroll], vr[kUnroll], cu[kUnroll], cv[kUnroll];
            bool fv[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                f[u] = (g0 + u) * fpw + slotw;
                fv[u] = u < U && g0 + u < ngroups && f[u] < nf && fvis[f[u]] == 3;
                if (fv[u]) {
                    ur[u] = px[2 * f[u]] * scale; vr[u] = px[2 * f[u] + 1] * scale;
                    cu[u] = cuv[2 * f[u]]; cv[u] = cuv[2 * f[u] + 1];
                    rox[u] = (int)floor(ur[u]) - h - 1; roy[u] = (int)floor(vr[u]) - h - 1;
                    cox[u] = (int)floor(cu[u]) - h; coy[u] = (int)floor(cv[u]) - h;
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
                if (fv[u]) {
                    uint8_t* wb = sh.win[wave] + (u * fpw + slotw) * wbytes;
                    stage_window(wb, f[u] < P.n_ref ? ref_img : kf_img, W, H, rox[u], roy[u], RW, mrw, sub, lpf);
                    stage_window(wb + RW * RW, cur_img, W, H, cox[u], coy[u], CW, mcw, sub, lpf);
                }
            wave_lds_sync();
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                if (!(u < U && g0 + u < ngroups && f[u] < nf)) continue;
                const uint8_t* wb = sh.win[wave] + (u * fpw + slotw) * wbytes;
                for (int k = sub, ky = ky0, kx = kx0; k < A; k += lpf) {
                    if (k != sub) { ky = (int)udiv((uint32_t)k, mside); kx = k - ky * side - h; ky -= h; }
                    double r = __builtin_inf();
                    if (fv[u]) {
                        const double T = bilerp_win(wb, RW, rox[u], roy[u], ur[u] + kx, vr[u] + ky);
                        const double I = bilerp_win(wb + RW * RW, CW, cox[u], coy[u], cu[u] + kx, cv[u] + ky);
                        r = I - T;
                        atomicAdd(&sh.hist[sel_bin<false>(r)], 1u);
                    }
                    res[f[u] * A + k] = r;
                }
            }
            wave_lds_sync();
        }
        __syncthreads();
        SVO_STAMP(2);

        // ---- S2-S4: robust scale  (Optimizer::tukeyWeighting -> algorithm::computeSigma)
        double med, mad;
        if (n == 0) {
            med = 1.7976931348623157e308;  // every slot is DBL_MAX in the reference
            mad = 0.0;
        } else {
            med = block_median<false>(sh, res, M, n, 0.0);
            SVO_STAMP(3);
            for (int i = tid; i < kBins; i += kThreads) sh.hist[i] = 0;
            __syncthreads();
            sweep_res(res, M, [&](double r) { atomicAdd(&sh.hist[sel_bin<true>(fabs(r - med))], 1u); });
            __syncthreads();
            mad = block_median<true>(sh, res, M, n, med);
        }
        double sigma = 1.482602218505602 * mad;
        if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
        const double c = 4.6851 * sigma, c2 = c * c;
        SVO_STAMP(4);

        // ---- S5: Tukey weights, chi2, per-feature factorised sums
        double chi_acc = 0.0;
        for (int g0 = wave * U; g0 < ngroups; g0 += kWaves * U) {
            int f[kUnroll], rox[kUnroll], roy[kUnroll];
            double ur[kUnroll], vr[kUnroll], r0[kUnroll];
            bool fv[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                f[u] = (g0 + u) * fpw + slotw;
                fv[u] = u < U && g0 + u < ngroups && f[u] < nf && fvis[f[u]] == 3;
                if (fv[u]) {
                    ur[u] = px[2 * f[u]] * scale; vr[u] = px[2 * f[u] + 1] * scale;
                    rox[u] = (int)floor(ur[u]) - h - 1; roy[u] = (int)floor(vr[u]) - h - 1;
                    r0[u] = sub < A ? res[f[u] * A + sub] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
                if (fv[u]) {
                    uint8_t* wb = sh.win[wave] + (u * fpw + slotw) * wbytes;
                    stage_window(wb, f[u] < P.n_ref ? ref_img : kf_img, W, H, rox[u], roy[u], RW, mrw, sub, lpf);
                }
            wave_lds_sync();
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                if (!(u < U && g0 + u < ngroups)) continue;  // wave-uniform: every lane joins the shuffles below
                const uint8_t* wb = sh.win[wave] + (u * fpw + slotw) * wbytes;
                double sxx = 0, sxy = 0, syy = 0, sxr = 0, syr = 0;
                if (fv[u]) {
                    for (int k = sub, ky = ky0, kx = kx0; k < A; k += lpf) {
                        double r = r0[u];
                        if (k != sub) {
                            ky = (int)udiv((uint32_t)k, mside); kx = k - ky * side - h; ky -= h;
                            r = res[f[u] * A + k];
                        }
                        double w = 0.0;
                        if (fabs(r) <= c) {
                            const double t = 1.0 - (r * r) / c2;
                            w = t * t;
                        }
                        chi_acc += r * r * w;
                        if (w == 0.0) continue;
                        const double row = vr[u] + ky, col = ur[u] + kx;
                        const double dx = 0.5 * (bilerp_win(wb, RW, rox[u], roy[u], col + 1, row) -
                                                 bilerp_win(wb, RW, rox[u], roy[u], col - 1, row));
                        const double dy = 0.5 * (bilerp_win(wb, RW, rox[u], roy[u], col, row + 1) -
                                                 bilerp_win(wb, RW, rox[u], roy[u], col, row - 1));
                        const double wdx = w * dx, wdy = w * dy;
                        sxx += wdx * dx; sxy += wdx * dy; syy += wdy * dy; sxr += wdx * r; syr += wdy * r;
                    }
                }
                for (int o = lpf >> 1; o > 0; o >>= 1) {
                    sxx += __shfl_down(sxx, o, lpf); sxy += __shfl_down(sxy, o, lpf); syy += __shfl_down(syy, o, lpf);
                    sxr += __shfl_down(sxr, o, lpf); syr += __shfl_down(syr, o, lpf);
                }
                if (fv[u] && sub == 0) {
                    double* fs = fsum + 5 * f[u];
                    fs[0] = sxx; fs[1] = sxy; fs[2] = syy; fs[3] = sxr; fs[4] = syr;
                }
            }
            wave_lds_sync();
        }
        chi_acc = wave_sum(chi_acc);
        if (lane == 0) sh.accw[wave][27] = chi_acc;
        __syncthreads();

        // ---- P5b: expand the per-feature sums into J^T W J (lower) and J^T W r.  Thread (term, chunk):
        // 27 terms x 16 feature chunks, one accumulator each; chunks summed in a fixed order below.
        {
            const int term = tid & 31, chunk = tid >> 5;
            if (term < 27) {
                int i, j;  // term -> (i, j) of the lower triangle, or g_i for term >= 21
                if (term < 21) {
                    i = 0;
                    while ((i + 1) * (i + 2) / 2 <= term) ++i;
                    j = term - i * (i + 1) / 2;
                } else {
                    i = term - 21;
                    j = 0;
                }
                double acc = 0.0;
                for (int f = chunk; f < nf; f += kThreads / 32) {
                    if (fvis[f] != 3) continue;
                    const double* fs = fsum + 5 * f;
                    const double* J = jimg + 12 * f;
                    const double ai = J[i], bi = J[6 + i];
                    if (term < 21) {
                        const double aj = J[j], bj = J[6 + j];
                        acc += ai * aj * fs[0] + (ai * bj + bi * aj) * fs[1] + bi * bj * fs[2];
                    } else {
                        acc += ai * fs[3] + bi * fs[4];
                    }
                }
                sh.part[chunk][term] = acc;
            }
        }
        __syncthreads();
        SVO_STAMP(5);

        // ---- P6: damped step, solve, update (one lane; LDS workspace)
        if (tid < 27) {  // chunk partials in a fixed order
            double s = 0.0;
            for (int c = 0; c < kThreads / 32; ++c) s += sh.part[c][tid];
            sh.tot[tid] = s;
        } else if (tid == 27) {
            double s = 0.0;
            for (int w = 0; w < kWaves; ++w) s += sh.accw[w][27];
            sh.tot[27] = s;
        }
        __syncthreads();
        if (tid == 0) lm_step(sh, traces[level], n, med, mad, sigma);
        __syncthreads();
        SVO_STAMP(6);
        err = sh.red[0][28];
        status = (int32_t)sh.ired[0][3];
        __syncthreads();
    }
    if (tid == 0) {
        se3_store(sh.pose, a.pose_out + 7 * pair);
        a.err_out[pair] = err;
        a.status_out[pair] = status;
    }
}

template <int kHalf>
static void launch_h(const AlignArgs& a, hipStream_t s) {
    if (a.stamps)
        hipLaunchKernelGGL((align_pairs_kernel<kHalf, true>), dim3(a.n_pairs), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((align_pairs_kernel<kHalf, false>), dim3(a.n_pairs), dim3(kThreads), 0, s, a);
}

void launch_align(const AlignArgs& a, hipStream_t s) {
    switch (a.half) {
        case 0: launch_h<0>(a, s); break;
        case 1: launch_h<1>(a, s); break;
        case 2: launch_h<2>(a, s); break;
        case 3: launch_h<3>(a, s); break;
        case 4: launch_h<4>(a, s); break;
        case 5: launch_h<5>(a, s); break;
        case 6: launch_h<6>(a, s); break;
        case 7: launch_h<7>(a, s); break;
        case 8: launch_h<8>(a, s); break;
        default: launch_h<9>(a, s); break;  // capi rejects larger patches (align_window_bytes)
    }
}

int align_window_bytes(int half) {
    const int A = (2 * half + 1) * (2 * half + 1);
    const int fpw = A <= 16 ? 4 : (A <= 32 ? 2 : 1);
    return fpw * ((2 * half + 5) * (2 * half + 5) + (2 * half + 3) * (2 * half + 3));
}
int align_window_capacity() { return kWinBytes; }

}  // namespace svo
