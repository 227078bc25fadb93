// align.hip — sparse image alignment (ImageAlignment::align, src/image_alignment.cpp:25-67) on gfx950.
//
// One 512-thread workgroup owns one frame pair for the whole coarse-to-fine call: pairs are independent
// (SURVEY.md §8(e)), so no workgroup ever talks to another and the batch needs one launch.  Per level:
//   P1  per feature : ref visibility (border rule :140-149), cur projection pose*X_w (:320-340),
//                     image Jacobian at the WORLD point (:163, :194-248)
//   P2  per pixel   : r = bilerp(I_cur) - bilerp(I_ref) (:359), +inf for invisible slots; first radix
//                     digit of the median histogrammed in LDS on the fly
//   P3  exact median of the visible residuals (radix select over order-preserving uint64 keys,
//                     11-bit digits, LDS histograms, candidate gather once a bucket is small)
//   P4  exact median of |r - median|  -> sigma = 1.482602218505602 * MAD   (src/algorithm.cpp:834-872)
//   P5  per pixel   : Tukey weight (src/optimizer.cpp:485-514), chi2, J row = dx*Jimg0 + dy*Jimg1 with
//                     dx, dy re-sampled from the ref image, lower-triangular J^T W J and J^T W r in
//                     registers; wave shuffles + fixed-order LDS tree (deterministic, no atomics)
//   P6  one lane    : Nielsen damping, Eigen-LDLT solve, pose <- pose * exp(-dx), status, RMSE
//                     (src/optimizer.cpp:279-366, src/image_alignment.cpp:379)
#include "svo_internal.h"
#include "svo_math.h"

namespace svo {

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kDigitBits = 11;
constexpr int kBins = 1 << kDigitBits;
constexpr int kCandCap = 1024;

struct Shared {
    uint32_t hist[kBins];
    uint64_t cand[kCandCap];
    double red[kWaves][32];
    uint32_t ired[kWaves][4];
    uint32_t scan[kThreads];
    SE3 pose;
    // selection state
    uint64_t sel_prefix;
    uint32_t sel_k, sel_cnt, sel_bits, cand_n;
    double sel_value;
    double med, mad;
    int32_t done;  // alignment ended early (status set)
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

// block-wide sums of up to 4 uint32 counters; result valid in every thread after return
__device__ void block_sum_u4(Shared& sh, uint32_t v[4]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = 0; i < 4; ++i) v[i] = wave_sum_u(v[i]);
    if (lane == 0)
        for (int i = 0; i < 4; ++i) sh.ired[wave][i] = v[i];
    __syncthreads();
    for (int i = 0; i < 4; ++i) {
        uint32_t s = 0;
        for (int w = 0; w < kWaves; ++w) s += sh.ired[w][i];
        v[i] = s;
    }
    __syncthreads();
}

// value of a residual slot for the current selection (median pass: r; MAD pass: |r - med|)
template <bool kMad>
__device__ __forceinline__ double sel_val(double r, double med) {
    return kMad ? fabs(r - med) : r;
}

// Find the bucket holding rank sh.sel_k in sh.hist; updates prefix/k/cnt.  All threads call.
__device__ void select_bucket(Shared& sh, int digit_bits) {
    const int tid = threadIdx.x;
    const uint32_t k = sh.sel_k;  // read before any thread can update it (the scan below syncs)
    const int bins = 1 << digit_bits;
    const int per = (bins + kThreads - 1) / kThreads;
    uint32_t local = 0;
    for (int i = 0; i < per; ++i) {
        const int b = tid * per + i;
        if (b < bins) local += sh.hist[b];
    }
    sh.scan[tid] = local;
    __syncthreads();
    // inclusive scan (Hillis-Steele on 512 entries)
    for (int o = 1; o < kThreads; o <<= 1) {
        const uint32_t add = tid >= o ? sh.scan[tid - o] : 0;
        __syncthreads();
        sh.scan[tid] += add;
        __syncthreads();
    }
    const uint32_t incl = sh.scan[tid];
    const uint32_t excl = incl - local;
    if (k >= excl && k < incl) {
        uint32_t run = excl;
        for (int i = 0; i < per; ++i) {
            const int b = tid * per + i;
            const uint32_t c = (b < bins) ? sh.hist[b] : 0;
            if (k < run + c) {
                sh.sel_prefix = (sh.sel_prefix << digit_bits) | (uint64_t)b;
                sh.sel_k = k - run;
                sh.sel_cnt = c;
                break;
            }
            run += c;
        }
    }
    __syncthreads();
    if (tid == 0) sh.sel_bits += digit_bits;
    __syncthreads();
}

// Exact k-th smallest (0-based) of the visible slot values.  hist must already hold the first-digit
// histogram (11 top bits of the key).  Returns the value in every thread.
template <bool kMad>
__device__ double block_select(Shared& sh, const double* __restrict__ res, int M, uint32_t k, double med) {
    const int tid = threadIdx.x;
    if (tid == 0) { sh.sel_prefix = 0; sh.sel_k = k; sh.sel_bits = 0; sh.cand_n = 0; }
    __syncthreads();
    select_bucket(sh, kDigitBits);
    while (sh.sel_cnt > kCandCap && sh.sel_bits < 64) {
        const int bits = sh.sel_bits;
        const int dbits = (64 - bits) < kDigitBits ? (64 - bits) : kDigitBits;
        const uint64_t prefix = sh.sel_prefix;
        for (int i = tid; i < (1 << dbits); i += kThreads) sh.hist[i] = 0;
        __syncthreads();
        const int shift = 64 - bits - dbits;
        for (int s = tid; s < M; s += kThreads) {
            const double r = res[s];
            if (r == __builtin_inf()) continue;
            const uint64_t key = dkey(sel_val<kMad>(r, med));
            if ((key >> (64 - bits)) == prefix) atomicAdd(&sh.hist[(key >> shift) & ((1u << dbits) - 1)], 1u);
        }
        __syncthreads();
        select_bucket(sh, dbits);
    }
    if (sh.sel_bits >= 64) {  // every bit fixed: the prefix is the key
        const double v = dkey_inv(sh.sel_prefix);
        __syncthreads();
        return v;
    }
    // gather the (few) candidates of the bucket and rank them exactly
    {
        const int bits = sh.sel_bits;
        const uint64_t prefix = sh.sel_prefix;
        for (int s = tid; s < M; s += kThreads) {
            const double r = res[s];
            if (r == __builtin_inf()) continue;
            const uint64_t key = dkey(sel_val<kMad>(r, med));
            if ((key >> (64 - bits)) == prefix) {
                const uint32_t slot = atomicAdd(&sh.cand_n, 1u);
                if (slot < kCandCap) sh.cand[slot] = key;
            }
        }
    }
    __syncthreads();
    const uint32_t n = sh.cand_n, kk = sh.sel_k;
    for (uint32_t i = tid; i < n; i += kThreads) {
        const uint64_t ki = sh.cand[i];
        uint32_t less = 0, eq_before = 0;
        for (uint32_t j = 0; j < n; ++j) {
            const uint64_t kj = sh.cand[j];
            less += kj < ki;
            eq_before += (kj == ki) & (j < i);
        }
        if (less + eq_before == kk) sh.sel_value = dkey_inv(ki);
    }
    __syncthreads();
    const double v = sh.sel_value;
    __syncthreads();
    return v;
}

// (mid-1)-th order statistic given hi = mid-th: hi itself if fewer than mid values are < hi,
// else the largest value < hi.
template <bool kMad>
__device__ double block_lower_neighbour(Shared& sh, const double* __restrict__ res, int M, uint32_t mid, double hi,
                                        double med) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t less = 0;
    double mx = -__builtin_inf();
    for (int s = tid; s < M; s += kThreads) {
        const double r = res[s];
        if (r == __builtin_inf()) continue;
        const double v = sel_val<kMad>(r, med);
        if (v < hi) { ++less; mx = fmax(mx, v); }
    }
    less = wave_sum_u(less);
    mx = wave_max(mx);
    if (lane == 0) { sh.ired[wave][0] = less; sh.red[wave][0] = mx; }
    __syncthreads();
    uint32_t tl = 0;
    double tm = -__builtin_inf();
    for (int w = 0; w < kWaves; ++w) { tl += sh.ired[w][0]; tm = fmax(tm, sh.red[w][0]); }
    __syncthreads();
    return (tl <= mid - 1) ? hi : tm;
}

// computeMedian(v, n) with exact order statistics: odd/even decided by the TOTAL length M
// (src/algorithm.cpp:845-851); mid == 0 reads vec[mid] (the reference's vec[-1] is UB).
template <bool kMad>
__device__ double block_median(Shared& sh, const double* __restrict__ res, int M, uint32_t n, double med) {
    const uint32_t mid = n / 2;
    const double hi = block_select<kMad>(sh, res, M, mid, med);
    if ((M & 1) || mid == 0) return hi;
    const double lo = block_lower_neighbour<kMad>(sh, res, M, mid, hi, med);
    return (lo + hi) / 2.0;
}

}  // namespace

__global__ void __launch_bounds__(kThreads) align_pairs_kernel(AlignArgs a) {
    __shared__ Shared sh;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pair = blockIdx.x;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf;
    const int A = a.area, h = a.half, side = 2 * a.half + 1;
    const int M = nf * A;
    const int64_t fbase = (int64_t)pair * a.max_f;
    const double* __restrict__ px = a.px + 2 * fbase;
    const double* __restrict__ bearing = a.bearing + 3 * fbase;
    const double* __restrict__ point = a.point + 3 * fbase;
    const uint8_t* __restrict__ has_point = a.has_point + fbase;
    double* __restrict__ xw = a.xw + 3 * fbase;
    double* __restrict__ jimg = a.jimg + 12 * fbase;
    double* __restrict__ cuv = a.cuv + 2 * fbase;
    uint8_t* __restrict__ fvis = a.fvis + fbase;
    double* __restrict__ res = a.res + fbase * A;
    svo_level_trace* traces = a.traces + (int64_t)pair * (a.max_level + 1);

    if (tid == 0) {
        sh.pose = se3_load(P.cur_pose);
        sh.done = 0;
    }
    for (int l = tid; l <= a.max_level; l += kThreads) {
        svo_level_trace t = {};
        t.level = l;
        t.status = kFailed;
        traces[l] = t;
    }
    if (P.n_ref == 0 || M < 6) {  // align(): no ref features -> return 0 (:27-28); optimizeLM: M < 6
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
            const V3 C = is_ref ? Cr : Ck;
            const V3 Pw{point[3 * f], point[3 * f + 1], point[3 * f + 2]};
            const double depth = v3norm(v3sub(Pw, C));
            const V3 pc = v3scl(V3{bearing[3 * f], bearing[3 * f + 1], bearing[3 * f + 2]}, depth);
            const V3 pw = se3_act(is_ref ? Tri : Tki, pc);
            xw[3 * f] = pw.x; xw[3 * f + 1] = pw.y; xw[3 * f + 2] = pw.z;
        }
    }
    __syncthreads();

    double err = 0.0;
    int32_t status = kFailed;
    for (int level = a.max_level; level >= a.min_level; --level) {
        const int32_t W = a.geom.w[level], H = a.geom.h[level];
        const int64_t loff = a.geom.off[level];
        const uint8_t* __restrict__ ref_img = P.ref_pyr + loff;
        const uint8_t* __restrict__ kf_img = P.kf_pyr + loff;
        const uint8_t* __restrict__ cur_img = P.cur_pyr + loff;
        const double dom = (double)(1 << level), scale = 1.0 / dom;
        const double lfx = a.fx / dom, lfy = a.fy / dom;
        const int border = h + 2;
        const SE3 pose = sh.pose;

        // ---- P1: per-feature visibility, projection and image Jacobian
        uint32_t cnt[4] = {0, 0, 0, 0};
        for (int f = tid; f < nf; f += kThreads) {
            uint8_t vis = 0;
            if (has_point[f]) {
                const double u = px[2 * f] * scale, v = px[2 * f + 1] * scale;
                const int ui = (int)floor(u), vi = (int)floor(v);
                if (!((ui - border) < 0 || (vi - border) < 0 || (ui + border) >= W || (vi + border) >= H)) {
                    vis = 1;
                    const V3 pw{xw[3 * f], xw[3 * f + 1], xw[3 * f + 2]};
                    double ja[6], jb[6];
                    image_jac(pw, lfx, lfy, ja, jb);
                    for (int j = 0; j < 6; ++j) { jimg[12 * f + j] = ja[j]; jimg[12 * f + 6 + j] = jb[j]; }
                    const V3 cp = se3_act(pose, pw);
                    const double cu = (a.fx * (cp.x / cp.z) + a.cx) * scale;
                    const double cv = (a.fy * (cp.y / cp.z) + a.cy) * scale;
                    const int cui = (int)floor(cu), cvi = (int)floor(cv);
                    if (!((cui - border) < 0 || (cvi - border) < 0 || (cui + border) >= W || (cvi + border) >= H)) {
                        vis = 3;
                        cuv[2 * f] = cu;
                        cuv[2 * f + 1] = cv;
                    }
                }
            }
            fvis[f] = vis;
            cnt[0] += vis & 1;
            cnt[1] += vis >> 1;
        }
        block_sum_u4(sh, cnt);
        const uint32_t n_ref_vis = cnt[0];
        const uint32_t n = cnt[1] * (uint32_t)A;

        // ---- P2: residuals (+inf for invisible slots) and first radix digit of the median
        for (int i = tid; i < kBins; i += kThreads) sh.hist[i] = 0;
        __syncthreads();
        for (int s = tid; s < M; s += kThreads) {
            const int f = s / A, k = s - f * A;
            double r = __builtin_inf();
            if (fvis[f] == 3) {
                const int ky = k / side - h, kx = k - (k / side) * side - h;
                const uint8_t* rimg = f < P.n_ref ? ref_img : kf_img;
                const double T = bilinear_d(rimg, W, px[2 * f] * scale + kx, px[2 * f + 1] * scale + ky);
                const double I = bilinear_d(cur_img, W, cuv[2 * f] + kx, cuv[2 * f + 1] + ky);
                r = I - T;
                atomicAdd(&sh.hist[dkey(r) >> (64 - kDigitBits)], 1u);
            }
            res[s] = r;
        }
        __syncthreads();

        // ---- P3/P4: robust scale  (Optimizer::tukeyWeighting -> algorithm::computeSigma)
        double med, mad;
        if (n == 0) {
            med = 1.7976931348623157e308;  // every slot is DBL_MAX in the reference
            mad = 0.0;
        } else {
            med = block_median<false>(sh, res, M, n, 0.0);
            for (int i = tid; i < kBins; i += kThreads) sh.hist[i] = 0;
            __syncthreads();
            for (int s = tid; s < M; s += kThreads) {
                const double r = res[s];
                if (r == __builtin_inf()) continue;
                atomicAdd(&sh.hist[dkey(fabs(r - med)) >> (64 - kDigitBits)], 1u);
            }
            __syncthreads();
            mad = block_median<true>(sh, res, M, n, med);
        }
        double sigma = 1.482602218505602 * mad;
        if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
        const double c = 4.6851 * sigma, c2 = c * c;

        // ---- P5: Tukey weights, chi2, normal equations (lower triangle, as the LDLT reads it)
        double acc[28];
        for (int i = 0; i < 28; ++i) acc[i] = 0.0;
        for (int s = tid; s < M; s += kThreads) {
            const double r = res[s];
            if (r == __builtin_inf()) continue;
            double w = 0.0;
            if (fabs(r) <= c) {
                const double t = 1.0 - (r * r) / c2;
                w = t * t;
            }
            acc[27] += r * r * w;
            if (w == 0.0) continue;
            const int f = s / A, k = s - f * A;
            const int ky = k / side - h, kx = k - (k / side) * side - h;
            const uint8_t* rimg = f < P.n_ref ? ref_img : kf_img;
            const double row = px[2 * f + 1] * scale + ky, col = px[2 * f] * scale + kx;
            const double dx = 0.5 * (bilinear_d(rimg, W, col + 1, row) - bilinear_d(rimg, W, col - 1, row));
            const double dy = 0.5 * (bilinear_d(rimg, W, col, row + 1) - bilinear_d(rimg, W, col, row - 1));
            double J[6];
            for (int j = 0; j < 6; ++j) J[j] = dx * jimg[12 * f + j] + dy * jimg[12 * f + 6 + j];
            int q = 0;
            for (int i = 0; i < 6; ++i) {
                const double jw = J[i] * w;
                for (int j = 0; j <= i; ++j) acc[q++] += jw * J[j];
                acc[21 + i] += jw * r;
            }
        }
        for (int i = 0; i < 28; ++i) {
            const double v = wave_sum(acc[i]);
            if (lane == 0) sh.red[wave][i] = v;
        }
        __syncthreads();

        // ---- P6: damped step, solve, update (one lane)
        if (tid == 0) {
            double tot[28];
            for (int i = 0; i < 28; ++i) {
                double s = 0.0;
                for (int w = 0; w < kWaves; ++w) s += sh.red[w][i];
                tot[i] = s;
            }
            double Hm[36], g[6], dx[6];
            int q = 0;
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j <= i; ++j) { Hm[i * 6 + j] = tot[q]; Hm[j * 6 + i] = tot[q]; ++q; }
            for (int i = 0; i < 6; ++i) g[i] = tot[21 + i];
            const double chi = tot[27];
            double mx = Hm[0];
            for (int i = 1; i < 6; ++i) mx = fmax(mx, Hm[i * 6 + i]);
            const double lambda = 1e-2 * mx;
            for (int i = 0; i < 6; ++i) Hm[i * 6 + i] += lambda;
            ldlt_solve(6, Hm, g, dx);
            double m[6];
            for (int i = 0; i < 6; ++i) m[i] = -dx[i];
            SE3 np = se3_compose(sh.pose, se3_exp(m));
            sh.pose = np;
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
            svo_level_trace t;
            t.level = level; t.n_ref_vis = (int32_t)n_ref_vis; t.n_vis = (int32_t)n; t.status = st;
            t.median = med; t.mad = mad; t.sigma = sigma; t.chi2 = chi; t.lambda = lambda; t.err = e;
            for (int i = 0; i < 36; ++i) t.H[i] = Hm[i];
            for (int i = 0; i < 6; ++i) { t.g[i] = g[i]; t.dx[i] = dx[i]; }
            traces[level] = t;
            sh.red[0][0] = e;
            sh.ired[0][0] = (uint32_t)st;
        }
        __syncthreads();
        err = sh.red[0][0];
        status = (int32_t)sh.ired[0][0];
        __syncthreads();
    }
    if (tid == 0) {
        se3_store(sh.pose, a.pose_out + 7 * pair);
        a.err_out[pair] = err;
        a.status_out[pair] = status;
    }
}

void launch_align(const AlignArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(align_pairs_kernel, dim3(a.n_pairs), dim3(kThreads), 0, s, a);
}

}  // namespace svo
