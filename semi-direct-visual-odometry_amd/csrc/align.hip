// align.hip — sparse image alignment (ImageAlignment::align, src/image_alignment.cpp:25-67) on gfx950.
//
// A batch holds n_pairs independent frame pairs.  The coarse-to-fine chain runs as
// stage kernels over all pairs of the batch, enqueued back to back on the context stream: each stage
// has its own register budget and launch shape (one persistent kernel spilled ~20 GB/launch).
//   K0 init      thread / feature : X_w = T_f^-1 (bearing * |P - C_f|) (:153-155); per-pair state
//   per level (max..min):
//   K1 residual  lane group / feature (32 lanes for the 25 px of patch 5, 64 for patch 7): ref
//                visibility (border rule :140-149), projection pose*X_w into cur (:320-340), image
//                Jacobian at the WORLD point (:163, :194-248).  The ref window ((2h+5)^2 px) and the
//                cur window ((2h+3)^2 px) are staged in LDS one row per lane with two aligned 16-B
//                loads; each lane then samples its pixel: r = I_cur - T_ref (:359) -> per-pair
//                residual row (+inf = invisible slot)
//   K2 scale     one workgroup / pair: exact median of the visible r (src/algorithm.cpp:834-853) and of
//                |r - median| (MAD, :855-865) -> sigma = 1.482602218505602 * MAD (:867-872).  Values
//                are binned by a monotone map into an LDS histogram; the bin of rank n/2 is exact; one
//                sweep gathers that bin's values into LDS and ranks them exactly; an overfull bin falls
//                back to an 11-bit radix select on order-preserving keys
//   K3 weights   lane group / feature: Tukey weight (src/optimizer.cpp:485-514), chi2 term, dx/dy
//                re-sampled from the staged ref window; per feature the 5 sums S_xx S_xy S_yy S_xr S_yr
//                are expanded with the 2x6 image Jacobian (factorised J row = dx*Jimg0 + dy*Jimg1),
//                one normal-equation term per lane, into per-workgroup partials (fixed order)
//   K4 solve     one workgroup / pair: partials summed in a fixed order (deterministic, no float
//                atomics); one lane: Nielsen damping, Eigen-LDLT, pose <- pose * exp(-dx), status,
//                RMSE (src/optimizer.cpp:279-366, src/image_alignment.cpp:379)
#include "svo_internal.h"
#include "svo_math.h"

namespace svo {

namespace {

constexpr int kFeatThreads = 256;    // K1 / K3 workgroup (4 waves)
constexpr int kFeatWaves = kFeatThreads / 64;
constexpr int kSelThreads = 512;     // K2 workgroup (two per CU)
constexpr int kSelWaves = kSelThreads / 64;
constexpr int kBins = 4096;
constexpr double kBinScale = 32.0;   // bins per grey level
constexpr double kBinOffset = 64.0;  // signed map covers [-64, 64); outliers clamp to the end bins
constexpr double kKeyScale = 512.0;  // K1's 16-bit residual key: 16 keys per value bin
constexpr uint32_t kKeyMax = 65534;  // largest key of a visible slot; 0xFFFF = invisible
constexpr int kCandCap = 2048;
constexpr int kRankCap = 256;        // <= this many candidates: rank counting, else bitonic sort
constexpr int kRadixBits = 11;
constexpr double kDblMax = 1.7976931348623157e308;

__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_down(v, o, 64));
    return __shfl(v, 0, 64);
}
__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_down(v, o, 64));
    return __shfl(v, 0, 64);
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

// features per K1/K3 workgroup: as many as fit ~40 KB of staged windows, at most 64
__host__ __device__ constexpr int feats_per_block(int half) {
    return half <= 3 ? 64 : (half <= 8 ? 32 : 16);
}

template <int kHalf>
struct Geo {
    static constexpr int h = kHalf, side = 2 * kHalf + 1, A = side * side;
    static constexpr int RW = 2 * h + 5, CW = 2 * h + 3;               // staged window sides (ref, cur)
    static constexpr int NB = (RW + 15 + 15) / 16;                     // 16-B blocks per staged row
    static constexpr int pitch = NB * 16;                              // LDS bytes per staged row
    static constexpr int FPB = feats_per_block(kHalf);                 // features per workgroup
    static constexpr int fstride1 = (RW + CW) * pitch + 16;            // K1 bytes per feature (ref + cur)
    static constexpr int fstride3 = RW * pitch + 16;                   // K3 bytes per feature (ref)
    static constexpr int pix_iters = (FPB * A + kFeatThreads - 1) / kFeatThreads;
};

// bilinearInterpolationDouble (src/algorithm.cpp:896-905) on a staged window.  Row r of the window
// (top-left pixel (ox, oy), image row pitch W) holds the aligned 16-B blocks that cover image bytes
// [lin, lin + width), lin = (oy + r) * W + ox = base + r * W, from byte lin & ~15 on.  Bytes past a row's
// end are the bytes the reference's unchecked Eigen map would read; they only ever carry a zero weight.
template <int kPitch>
__device__ __forceinline__ double bilerp_win(const uint8_t* win, uint32_t base, uint32_t W, int ox, int oy, double x,
                                             double y) {
    const int32_t x1 = (int32_t)x, y1 = (int32_t)y, x2 = x1 + 1, y2 = y1 + 1;
    const int ry = y1 - oy, cx = x1 - ox;
    const uint32_t l1 = base + (uint32_t)ry * W;
    const uint8_t* r1 = win + ry * kPitch + (int)(l1 & 15u) + cx;
    const uint8_t* r2 = win + (ry + 1) * kPitch + (int)((l1 + W) & 15u) + cx;
    const double a = (x2 - x) * r1[0] + (x - x1) * r1[1];
    const double b = (x2 - x) * r2[0] + (x - x1) * r2[1];
    return (y2 - y) * a + (y - y1) * b;
}

// 16-B load from an image plane.  The plane pointers come from the device-resident pair table, so the
// compiler only sees generic pointers; the explicit global address space keeps these loads off the flat
// path (a flat load also waits on LDS traffic, which serialises the staging loop).
__device__ __forceinline__ uint4 gload16(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(1))) const uint4 gu4;
    return *(gu4*)(p);
#else
    return *reinterpret_cast<const uint4*>(p);  // host pass only parses device code
#endif
}

// 16-bit monotone key of a residual for K2's sweeps: floor((r + 64) * 512) clamped to [0, kKeyMax];
// 0xFFFF marks an invisible slot.  key >> 4 is exactly the value bin floor((r + 64) * 32) of K2.
__device__ __forceinline__ uint16_t res_key(double r) {
    if (r == __builtin_inf()) return 0xFFFF;
    const double t = (r + kBinOffset) * kKeyScale;
    return (uint16_t)(t < 0.0 ? 0u : (t >= (double)kKeyMax ? kKeyMax : (uint32_t)t));
}

// Per-feature records of K1 / K3 (LDS)
struct ResRec {
    double ur, vr, cu, cv;     // feature pixel in the ref level, projection into the cur level
    int32_t rox, roy, cox, coy;  // staged window origins
    uint32_t rbase, cbase;     // roy * W + rox, coy * W + cox
    int32_t vis, isref;        // bit0 ref visible, bit1 cur visible; feature of the ref (else the lastKF)
};
struct WtRec {
    double fx, fy;             // fractional parts of the feature pixel at the level (bilinear weights)
    uint32_t rbase;            // roy * W + rox of the staged ref window
    int32_t vis, pad0, pad1;
    double ja[6], jb[6];       // computeImageJac at the world point, level-scaled focal lengths
};

// 4 consecutive bytes of a staged row starting at byte offset `off` (any alignment): two aligned
// dword reads and a byte-align funnel shift
__device__ __forceinline__ uint32_t lds_bytes4(const uint8_t* win, int off) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(win + (off & ~3));
    return __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)(off & 3));  // byte shift
}
__device__ __forceinline__ double byte_d(uint32_t v, int i) { return (double)((v >> (8 * i)) & 0xFFu); }

}  // namespace

int align_feat_iters() { return 1; }

int align_chunks(int max_f, int half, int feat_iters) {
    (void)feat_iters;
    const int fpb = feats_per_block(half);
    return (max_f + fpb - 1) / fpb;
}

// ------------------------------------------------------------------ K0: world points, pair state
__global__ void __launch_bounds__(256) align_init_kernel(AlignArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < a.n_pairs) {
        const PairDesc& P = a.pairs[gid];
        PairState& S = a.state[gid];
        for (int i = 0; i < 7; ++i) S.pose[i] = P.cur_pose[i];
        const int nf = P.n_ref + P.n_kf;
        S.active = (P.n_ref > 0 && (int64_t)nf * a.area >= 6) ? 1 : 0;
        S.err = P.n_ref == 0 ? 0.0 : -1.0;  // align() returns 0 (:27-28); optimizeLM returns -1 when M < 6
        S.status = P.n_ref == 0 ? kFailed : kNonSuffPoints;
        const int64_t M = (int64_t)nf * a.area;
        if (M & 1) a.res[gid * a.res_stride + M] = __builtin_inf();  // pad for the 16-B sweeps of K2
        for (int64_t s = M; s < ((M + 7) & ~(int64_t)7); ++s) a.keys[gid * a.key_stride + s] = 0xFFFF;
        svo_level_trace* tr = a.traces + gid * (a.max_level + 1);
        for (int l = 0; l <= a.max_level; ++l) {
            svo_level_trace t = {};
            t.level = l;
            t.status = kFailed;
            tr[l] = t;
        }
    }
    if (gid >= (int64_t)a.n_pairs * a.max_f) return;
    const int pair = (int)(gid / a.max_f), f = (int)(gid - (int64_t)pair * a.max_f);
    const PairDesc& P = a.pairs[pair];
    if (f >= P.n_ref + P.n_kf || !a.has_point[gid]) return;
    const bool is_ref = f < P.n_ref;
    const SE3 T = se3_load(is_ref ? P.ref_pose : P.kf_pose);
    const V3 C = camera_in_world(T);
    const V3 Pw{a.point[3 * gid], a.point[3 * gid + 1], a.point[3 * gid + 2]};
    const double depth = v3norm(v3sub(Pw, C));
    const V3 pc = v3scl(V3{a.bearing[3 * gid], a.bearing[3 * gid + 1], a.bearing[3 * gid + 2]}, depth);
    const V3 pw = se3_act(se3_inverse(T), pc);
    a.xw[3 * gid] = pw.x; a.xw[3 * gid + 1] = pw.y; a.xw[3 * gid + 2] = pw.z;
}

// ------------------------------------------------------------------ K1: visibility, projection, residuals
// grid.x = n_pairs * chunks; a workgroup owns FPB consecutive features of one pair.
//   1. one lane per feature: border tests, projection, window origins -> LDS record
//   2. one lane per window row: two aligned 16-B loads per row -> LDS (all rows' loads issued first)
//   3. one lane per pixel slot (flattened feature x pixel): r = I_cur - T_ref -> contiguous residual row
template <int kHalf>
__global__ void __launch_bounds__(kFeatThreads) align_residual_kernel(AlignArgs a, int level) {
    using G = Geo<kHalf>;
    constexpr int kRows = G::RW + G::CW;
    constexpr int kRowIters = (G::FPB * kRows + kFeatThreads - 1) / kFeatThreads;
    __shared__ __attribute__((aligned(16))) uint8_t win[G::FPB * G::fstride1];
    __shared__ ResRec rec[G::FPB];
    const int pair = blockIdx.x / a.chunks, chunk = blockIdx.x - pair * a.chunks;
    const PairState& S = a.state[pair];
    if (!S.active) return;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf, f0 = chunk * G::FPB;
    if (f0 >= nf) return;
    const int nb = nf - f0 < G::FPB ? nf - f0 : G::FPB;
    const int tid = threadIdx.x;
    const int W = a.geom.w[level], H = a.geom.h[level];
    const int64_t loff = a.geom.off[level];
    const double scale = 1.0 / (double)(1 << level);
    const int border = G::h + 2;
    const int64_t fbase = (int64_t)pair * a.max_f + f0;
    const uint8_t* const ref_plane = P.ref_pyr + loff;
    const uint8_t* const kf_plane = P.kf_pyr + loff;
    const uint8_t* const cur_plane = P.cur_pyr + loff;
    if (tid < G::FPB) {
        ResRec& R = rec[tid];
        int32_t vis = 0;
        // all of the feature's loads at once (one memory round trip); X_w is only used with a point
        const int64_t gf = fbase + (tid < nb ? tid : 0);
        const uint8_t hp = a.has_point[gf];
        const double pu = a.px[2 * gf], pv = a.px[2 * gf + 1];
        const V3 pw{a.xw[3 * gf], a.xw[3 * gf + 1], a.xw[3 * gf + 2]};
        if (tid < nb) {
            if (hp) {
                const double ur = pu * scale, vr = pv * scale;
                const int ui = (int)floor(ur), vi = (int)floor(vr);
                if (!((ui - border) < 0 || (vi - border) < 0 || (ui + border) >= W || (vi + border) >= H)) {
                    vis = 1;
                    const V3 cp = se3_act(se3_load(S.pose), pw);
                    const double cu = (a.fx * (cp.x / cp.z) + a.cx) * scale;
                    const double cv = (a.fy * (cp.y / cp.z) + a.cy) * scale;
                    const int cui = (int)floor(cu), cvi = (int)floor(cv);
                    if (!((cui - border) < 0 || (cvi - border) < 0 || (cui + border) >= W || (cvi + border) >= H)) {
                        vis = 3;
                        R.ur = ur; R.vr = vr; R.cu = cu; R.cv = cv;
                        R.rox = ui - G::h - 1; R.roy = vi - G::h - 1;
                        R.cox = cui - G::h; R.coy = cvi - G::h;
                        R.rbase = (uint32_t)((vi - G::h - 1) * W + ui - G::h - 1);
                        R.cbase = (uint32_t)((cvi - G::h) * W + cui - G::h);
                    }
                }
            }
            a.fvis[gf] = (uint8_t)vis;
            R.isref = f0 + tid < P.n_ref;
        }
        R.vis = vis;
    }
    __syncthreads();
    // every row's loads first (branch-free: rows of features without a window read a harmless in-plane
    // block), then the LDS stores
    uint4 blk[kRowIters][G::NB];
#pragma unroll
    for (int i = 0; i < kRowIters; ++i) {
        const int j = tid + i * kFeatThreads;
        const int fl = j / kRows < G::FPB ? j / kRows : G::FPB - 1, row = j - fl * kRows;
        const bool ok = rec[fl].vis == 3, isref = row < G::RW;
        const uint8_t* plane = isref ? (rec[fl].isref ? ref_plane : kf_plane) : cur_plane;
        const uint32_t lin = !ok ? 0u : (isref ? rec[fl].rbase + (uint32_t)(row * W)
                                              : rec[fl].cbase + (uint32_t)((row - G::RW) * W));
        const uint8_t* src = plane + (lin & ~15u);
#pragma unroll
        for (int b = 0; b < G::NB; ++b) blk[i][b] = gload16(src + 16 * b);
    }
#pragma unroll
    for (int i = 0; i < kRowIters; ++i) {
        const int j = tid + i * kFeatThreads, fl = j / kRows, row = j - fl * kRows;
        if (j < G::FPB * kRows) {
            uint4* d = reinterpret_cast<uint4*>(win + fl * G::fstride1 + row * G::pitch);
#pragma unroll
            for (int b = 0; b < G::NB; ++b) d[b] = blk[i][b];
        }
    }
    __syncthreads();
    double* __restrict__ res = a.res + (int64_t)pair * a.res_stride + (int64_t)f0 * G::A;
    uint16_t* __restrict__ keys = a.keys + (int64_t)pair * a.key_stride + (int64_t)f0 * G::A;
    const int ne = nb * G::A;
#pragma unroll 4
    for (int i = 0; i < G::pix_iters; ++i) {
        const int e = tid + i * kFeatThreads;
        if (e < ne) {
            const int fl = e / G::A, k = e - fl * G::A;
            const int ky = k / G::side - G::h, kx = k - (k / G::side) * G::side - G::h;
            const ResRec& R = rec[fl];
            double r = __builtin_inf();
            if (R.vis == 3) {
                const uint8_t* wr = win + fl * G::fstride1;
                const double T = bilerp_win<G::pitch>(wr, R.rbase, W, R.rox, R.roy, R.ur + kx, R.vr + ky);
                const double I = bilerp_win<G::pitch>(wr + G::RW * G::pitch, R.cbase, W, R.cox, R.coy, R.cu + kx,
                                                      R.cv + ky);
                r = I - T;
            }
            res[e] = r;
            keys[e] = res_key(r);
        }
    }
}

// ------------------------------------------------------------------ K2: exact robust scale
namespace {

struct SelShared {
    uint32_t hist[kBins];   // value bins of r (median), radix digits (exact fallback)
    uint32_t hlo[kBins];    // MAD bracket: bins of the lower / upper bound of |r - med| per value bin
    uint32_t hhi[kBins];    // (hhi is reused by cand_select's fine histogram)
    double cand[kCandCap];
    uint32_t mcand[kCandCap];  // MAD candidate slots
    double small[kRankCap];    // values of one fine bin (cand_select)
    uint32_t scan[kSelWaves];
    uint32_t ired[kSelWaves][2];
    double red[kSelWaves], red2[kSelWaves];
    uint64_t sel_prefix;
    uint32_t sel_k, sel_cnt, sel_bits, sel_bin, cand_n, mcand_n, small_n;
    uint32_t rngw[kSelWaves][4];
    double sel_hi, sel_lo;
};

template <bool kMad>
__device__ __forceinline__ double sel_val(double r, double med) { return kMad ? fabs(r - med) : r; }
template <bool kMad>
__device__ __forceinline__ int sel_bin(double v) {
    const double t = kMad ? v * kBinScale : (v + kBinOffset) * kBinScale;
    return t < 0.0 ? 0 : (t >= (double)(kBins - 1) ? kBins - 1 : (int)t);
}

// Sweep the residual row, 4 x 16-B loads in flight per lane; fn(value) for each visible slot.
// res[M] is +inf when M is odd, so 16-B pairs never read past the row.
template <typename Fn>
__device__ __forceinline__ void sweep_res(const double* __restrict__ res, int M, Fn fn) {
    const int tid = threadIdx.x;
    for (int base = 2 * tid; base < M; base += 8 * kSelThreads) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int s2 = base + u * 2 * kSelThreads;
            v[u] = s2 < M ? *reinterpret_cast<const double2*>(res + s2) : make_double2(__builtin_inf(), __builtin_inf());
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (v[u].x != __builtin_inf()) fn(v[u].x);
            if (v[u].y != __builtin_inf()) fn(v[u].y);
        }
    }
}

// Sweep the 16-bit residual keys of K1; fn(slot, key) for each visible slot.  A lane owns kKeyLoads
// 16-B groups of 8 keys per chunk and issues all of a chunk's loads before using any (one memory round
// trip per chunk; a config-2 pair, 50 000 slots, is one chunk).  Rows are padded with 0xFFFF to 8.
constexpr int kKeyLoads = 13;
template <typename Fn>
__device__ __forceinline__ void sweep_keys(const uint16_t* __restrict__ keys, int M8, Fn fn) {
    const int tid = threadIdx.x;
    for (int base = 8 * tid; base < M8; base += 8 * kSelThreads * kKeyLoads) {
        uint4 v[kKeyLoads];
#pragma unroll
        for (int u = 0; u < kKeyLoads; ++u) {
            const int s = base + u * 8 * kSelThreads;
            v[u] = s < M8 ? *reinterpret_cast<const uint4*>(keys + s) : make_uint4(~0u, ~0u, ~0u, ~0u);
        }
#pragma unroll
        for (int u = 0; u < kKeyLoads; ++u) {
            const int s = base + u * 8 * kSelThreads;
            const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((w[q] & 0xFFFFu) != 0xFFFFu) fn(s + 2 * q, w[q] & 0xFFFFu);
                if ((w[q] >> 16) != 0xFFFFu) fn(s + 2 * q + 1, w[q] >> 16);
            }
        }
    }
}

// distance bounds between the values of value bin j and a median known to lie in [mlo, mhi]
__device__ __forceinline__ void bin_dist(int j, double mlo, double mhi, double& dlo, double& dhi) {
    constexpr double eps = 1e-9;  // r + kBinOffset rounds by < 2^-45 before binning
    const double lo = j == 0 ? -__builtin_inf() : (double)j / kBinScale - kBinOffset - eps;
    const double hi = j == kBins - 1 ? __builtin_inf() : (double)(j + 1) / kBinScale - kBinOffset + eps;
    dlo = fmax(0.0, fmax(lo - mhi, mlo - hi));
    dhi = fmax(hi - mlo, mhi - lo);
}

// bin holding rank sh.sel_k of hist -> sh.sel_bin, sh.sel_k (rank inside the bin), sh.sel_cnt
__device__ void find_bin(SelShared& sh, const uint32_t* hist, int bins) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t k = sh.sel_k;
    const int per = (bins + kSelThreads - 1) / kSelThreads;
    uint32_t local = 0;
    for (int i = 0; i < per; ++i) {
        const int b = tid * per + i;
        if (b < bins) local += hist[b];
    }
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

// k-th and (k-1)-th smallest of v[0..n) (k-1 only if want_lo and k > 0): rank counting for small n,
// else a bitonic sort (v must then be sh.cand)
__device__ void select_direct(SelShared& sh, double* v, uint32_t n, uint32_t kk, bool want_lo) {
    const int tid = threadIdx.x;
    if (n <= (uint32_t)kRankCap) {
        for (uint32_t i = tid; i < n; i += kSelThreads) {
            const double vi = v[i];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < n; ++j) {
                const double vj = v[j];
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
    for (uint32_t i = n + tid; i < p2; i += kSelThreads) sh.cand[i] = __builtin_inf();
    __syncthreads();
    for (uint32_t size = 2; size <= p2; size <<= 1)
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t i = tid; i < p2 / 2; i += kSelThreads) {
                const uint32_t lo = (i / stride) * stride * 2 + (i % stride), hi = lo + stride;
                const bool asc = (lo & size) == 0;
                const double x = sh.cand[lo], y = sh.cand[hi];
                if ((x > y) == asc) { sh.cand[lo] = y; sh.cand[hi] = x; }
            }
            __syncthreads();
        }
    if (tid == 0) {
        sh.sel_hi = sh.cand[kk];
        if (want_lo && kk > 0) sh.sel_lo = sh.cand[kk - 1];
    }
    __syncthreads();
}

// append for the lanes with pred set: one LDS atomic per wave, slots in lane order
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred) {
    const uint64_t m = __ballot(pred);
    const int lane = threadIdx.x & 63;
    if (m == 0) return 0;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// k-th (and (k-1)-th) smallest of sh.cand[0..n).  Above kRankCap values, a 2048-bin histogram over
// the candidates' range narrows to one bin whose values are ranked directly (bitonic sort if that bin
// is still large).
__device__ void cand_select(SelShared& sh, uint32_t n, uint32_t kk, bool want_lo) {
    if (n <= (uint32_t)kRankCap) {
        select_direct(sh, sh.cand, n, kk, want_lo);
        return;
    }
    constexpr int kFine = 2048;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double vmin = __builtin_inf(), vmax = -__builtin_inf();
    for (uint32_t i = tid; i < n; i += kSelThreads) { vmin = fmin(vmin, sh.cand[i]); vmax = fmax(vmax, sh.cand[i]); }
    vmin = -wave_max(-vmin);
    vmax = wave_max(vmax);
    if (lane == 0) { sh.red[wave] = vmax; sh.red2[wave] = vmin; }
    for (int i = tid; i < kFine; i += kSelThreads) sh.hhi[i] = 0;
    if (tid == 0) sh.small_n = 0;
    __syncthreads();
    vmin = __builtin_inf(); vmax = -__builtin_inf();
    for (int w = 0; w < kSelWaves; ++w) { vmax = fmax(vmax, sh.red[w]); vmin = fmin(vmin, sh.red2[w]); }
    if (!(vmax > vmin) || !(vmax - vmin < __builtin_inf())) {
        select_direct(sh, sh.cand, n, kk, want_lo);
        return;
    }
    const double inv = (double)kFine / (vmax - vmin);
    auto fbin = [=](double v) { const int b = (int)((v - vmin) * inv); return b < kFine - 1 ? b : kFine - 1; };
    for (uint32_t i = tid; i < n; i += kSelThreads) atomicAdd(&sh.hhi[fbin(sh.cand[i])], 1u);
    if (tid == 0) sh.sel_k = kk;
    __syncthreads();
    find_bin(sh, sh.hhi, kFine);
    const uint32_t b2 = sh.sel_bin, kin = sh.sel_k, c2 = sh.sel_cnt;
    if (c2 > (uint32_t)kRankCap) {
        select_direct(sh, sh.cand, n, kk, want_lo);
        return;
    }
    double below_max = -__builtin_inf();
    for (uint32_t i = tid; i < n; i += kSelThreads) {
        const double v = sh.cand[i];
        const int b = fbin(v);
        const uint32_t s = wave_append(&sh.small_n, b == (int)b2);
        if (b == (int)b2) sh.small[s] = v;
        else if (b < (int)b2) below_max = fmax(below_max, v);
    }
    below_max = wave_max(below_max);
    if (lane == 0) sh.red[wave] = below_max;
    __syncthreads();
    below_max = -__builtin_inf();
    for (int w = 0; w < kSelWaves; ++w) below_max = fmax(below_max, sh.red[w]);
    select_direct(sh, sh.small, c2, kin, want_lo && kin > 0);
    if (want_lo && kin == 0 && tid == 0) sh.sel_lo = below_max;
    __syncthreads();
}

// radix fallback inside one overfull bin: exact k-th among values v with sel_bin(v) == bin
template <bool kMad>
__device__ double radix_in_bin(SelShared& sh, const double* __restrict__ res, int M, uint32_t bin, uint32_t k,
                               double med) {
    const int tid = threadIdx.x;
    if (tid == 0) { sh.sel_prefix = 0; sh.sel_bits = 0; sh.sel_k = k; }
    __syncthreads();
    while (sh.sel_bits < 64) {
        const int bits = sh.sel_bits;
        const int dbits = (64 - bits) < kRadixBits ? (64 - bits) : kRadixBits;
        const uint64_t prefix = sh.sel_prefix;
        const int shift = 64 - bits - dbits;
        for (int i = tid; i < (1 << dbits); i += kSelThreads) sh.hist[i] = 0;
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
__device__ double lower_neighbour_sweep(SelShared& sh, const double* __restrict__ res, int M, uint32_t k, double hi,
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
    if (lane == 0) { sh.ired[wave][0] = less; sh.red[wave] = mx; }
    __syncthreads();
    uint32_t tl = 0;
    double tm = -__builtin_inf();
    for (int w = 0; w < kSelWaves; ++w) { tl += sh.ired[w][0]; tm = fmax(tm, sh.red[w]); }
    __syncthreads();
    return (tl <= k - 1) ? hi : tm;
}

// computeMedian(v, n) with exact order statistics (odd/even decided by the TOTAL length M,
// src/algorithm.cpp:845-851; mid == 0 reads vec[mid]).  sh.hist holds the value-bin histogram.
template <bool kMad>
__device__ double block_median(SelShared& sh, const double* __restrict__ res, int M, uint32_t n, double med) {
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
        if (lane == 0) sh.red[wave] = below;
        __syncthreads();
        double tb = -__builtin_inf();
        for (int w = 0; w < kSelWaves; ++w) tb = fmax(tb, sh.red[w]);
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

}  // namespace

#if defined(SVO_STAMPS)
// diagnostic build only (make stamps): per (pair, level) cycle stamps of K2's phases
__device__ uint64_t g_stamps[4096 * 16];
#define K2_STAMP(i, v)                                                                      \
    do {                                                                                    \
        if (tid == 0 && pair * 5 + level < 4096) g_stamps[(pair * 5 + level) * 16 + (i)] = (v); \
    } while (0)
#else
#define K2_STAMP(i, v) \
    do {               \
    } while (0)
#endif

// One workgroup per pair (src/algorithm.cpp:834-872 on the level's residual vector).
//   1. value-bin histogram of the visible residuals from K1's 16-bit keys (key >> 4 = value bin);
//      the bin b holding rank n/2 and its count
//   2. MAD bracket without touching the slots again: every value bin j bounds |r - med| of its members
//      (med lies in bin b, or is exact on the slow path); the order statistic n/2 of those lower and
//      upper bounds brackets the MAD in [L0, U0).  Bins wholly below L0 are counted, bins meeting
//      [L0, U0) are MAD candidates, the rest lie above
//   3. one sweep over the keys gathers the slots of bin b (median candidates) and of the candidate
//      bins; only those slots' exact residuals are read
//   4. exact selection among the candidates (rank counting or bitonic sort in LDS)
// Cases the fast path cannot settle (overfull bins; the even-length neighbour below a bin's first
// element) take the exact path on the 8-B residuals.
__global__ void __launch_bounds__(kSelThreads) align_scale_kernel(AlignArgs a, int level) {
    __shared__ SelShared sh;
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    PairState& S = a.state[pair];
    if (!S.active) return;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf, M = nf * a.area, M8 = (M + 7) & ~7;
    const double* __restrict__ res = a.res + (int64_t)pair * a.res_stride;
    const uint16_t* __restrict__ keys = a.keys + (int64_t)pair * a.key_stride;
    const uint8_t* __restrict__ fvis = a.fvis + (int64_t)pair * a.max_f;
    K2_STAMP(0, clock64());
    uint32_t nrv = 0, ncv = 0;
    for (int f = tid; f < nf; f += kSelThreads) {
        const uint8_t v = fvis[f];
        nrv += v & 1;
        ncv += v >> 1;
    }
    for (int i = tid; i < kBins; i += kSelThreads) { sh.hist[i] = 0; sh.hlo[i] = 0; sh.hhi[i] = 0; }
    nrv = wave_sum_u(nrv);
    ncv = wave_sum_u(ncv);
    if (lane == 0) { sh.ired[wave][0] = nrv; sh.ired[wave][1] = ncv; }
    __syncthreads();
    nrv = 0; ncv = 0;
    for (int w = 0; w < kSelWaves; ++w) { nrv += sh.ired[w][0]; ncv += sh.ired[w][1]; }
    const uint32_t n = ncv * (uint32_t)a.area;
    const uint32_t mid = n / 2;
    const bool want_lo = ((M & 1) == 0) && mid > 0;
    double med = kDblMax, mad = 0.0;  // n == 0: every slot is DBL_MAX in the reference
    if (n > 0) {
        K2_STAMP(1, clock64());
        sweep_keys(keys, M8, [&](int, uint32_t q) { atomicAdd(&sh.hist[q >> 4], 1u); });
        if (tid == 0) { sh.sel_k = mid; sh.cand_n = 0; sh.mcand_n = 0; }
        __syncthreads();
        K2_STAMP(2, clock64());
        find_bin(sh, sh.hist, kBins);
        const uint32_t bin = sh.sel_bin, kk = sh.sel_k, cnt = sh.sel_cnt;
        const bool med_fast = cnt <= (uint32_t)kCandCap && !(want_lo && kk == 0);
        double mlo, mhi;
        if (med_fast) {
            const double eps = 1e-9;
            mlo = bin == 0 ? -__builtin_inf() : (double)bin / kBinScale - kBinOffset - eps;
            mhi = bin == kBins - 1 ? __builtin_inf() : (double)(bin + 1) / kBinScale - kBinOffset + eps;
        } else {
            med = block_median<false>(sh, res, M, n, 0.0);
            mlo = mhi = med;
            // the exact path may have reused sh.hist for radix digits: rebuild the value histogram
            for (int i = tid; i < kBins; i += kSelThreads) sh.hist[i] = 0;
            __syncthreads();
            sweep_keys(keys, M8, [&](int, uint32_t q) { atomicAdd(&sh.hist[q >> 4], 1u); });
            __syncthreads();
            K2_STAMP(10, 1000000 + cnt);
        }
        K2_STAMP(3, clock64());
        // ---- MAD bracket from the value histogram
        for (int j = tid; j < kBins; j += kSelThreads) {
            const uint32_t c = sh.hist[j];
            if (c) {
                double dlo, dhi;
                bin_dist(j, mlo, mhi, dlo, dhi);
                atomicAdd(&sh.hlo[sel_bin<true>(dlo)], c);
                atomicAdd(&sh.hhi[sel_bin<true>(dhi)], c);
            }
        }
        if (tid == 0) sh.sel_k = mid;
        __syncthreads();
        find_bin(sh, sh.hlo, kBins);
        const uint32_t blo = sh.sel_bin;
        if (tid == 0) sh.sel_k = mid;
        __syncthreads();
        find_bin(sh, sh.hhi, kBins);
        const uint32_t bhi = sh.sel_bin;
        const double L0 = (double)blo / kBinScale;
        const double U0 = bhi >= (uint32_t)(kBins - 1) ? __builtin_inf() : (double)(bhi + 1) / kBinScale;
        // bin classes: 0 below (dhi < L0), 1 candidate, 2 above (dlo >= U0).  dlo and dhi are V-shaped in
        // j around the median bin, so class 0 is one run of bins [C, D] inside the run [A, B] of classes
        // 0 and 1: candidate bins are [A, B] minus [C, D]
        uint32_t below = 0, ncand = 0, rA = kBins, rB = 0, rC = kBins, rD = 0;
        for (int j = tid; j < kBins; j += kSelThreads) {
            double dlo, dhi;
            bin_dist(j, mlo, mhi, dlo, dhi);
            const uint32_t cls = dhi < L0 ? 0u : (dlo < U0 ? 1u : 2u);
            if (cls != 2) { rA = min(rA, (uint32_t)j); rB = max(rB, (uint32_t)j); }
            if (cls == 0) { rC = min(rC, (uint32_t)j); rD = max(rD, (uint32_t)j); }
            below += cls == 0 ? sh.hist[j] : 0u;
            ncand += cls == 1 ? sh.hist[j] : 0u;
        }
        below = wave_sum_u(below);
        ncand = wave_sum_u(ncand);
        rA = wave_min_u(rA); rB = wave_max_u(rB); rC = wave_min_u(rC); rD = wave_max_u(rD);
        if (lane == 0) {
            sh.ired[wave][0] = below; sh.ired[wave][1] = ncand;
            sh.rngw[wave][0] = rA; sh.rngw[wave][1] = rB; sh.rngw[wave][2] = rC; sh.rngw[wave][3] = rD;
        }
        __syncthreads();
        below = 0; ncand = 0;
        for (int w = 0; w < kSelWaves; ++w) {
            below += sh.ired[w][0]; ncand += sh.ired[w][1];
            rA = min(rA, sh.rngw[w][0]); rB = max(rB, sh.rngw[w][1]);
            rC = min(rC, sh.rngw[w][2]); rD = max(rD, sh.rngw[w][3]);
        }
        const uint32_t kk2 = mid - below;
        bool mad_fast = ncand <= (uint32_t)kCandCap && mid >= below && kk2 < ncand;
        K2_STAMP(4, clock64());
        // ---- one sweep: median candidates (bin b) and MAD candidates (candidate bins)
        if (med_fast || mad_fast) {
            const uint32_t mbin = med_fast ? bin : kBins;  // kBins never matches
            const uint32_t cA = mad_fast ? rA : kBins;
            sweep_keys(keys, M8, [&](int s, uint32_t q) {
                const uint32_t j = q >> 4;
                if (j == mbin) sh.cand[atomicAdd(&sh.cand_n, 1u)] = __longlong_as_double((long long)s);
                if (j >= cA && j <= rB && !(j >= rC && j <= rD)) sh.mcand[atomicAdd(&sh.mcand_n, 1u)] = (uint32_t)s;
            });
            __syncthreads();
        }
        K2_STAMP(5, clock64());
        if (med_fast) {
            for (uint32_t i = tid; i < cnt; i += kSelThreads) sh.cand[i] = res[__double_as_longlong(sh.cand[i])];
            __syncthreads();
            cand_select(sh, cnt, kk, want_lo);
            med = want_lo ? (sh.sel_lo + sh.sel_hi) / 2.0 : sh.sel_hi;
            K2_STAMP(10, cnt);
            __syncthreads();
        }
        K2_STAMP(6, clock64());
        if (mad_fast) {
            for (uint32_t i = tid; i < ncand; i += kSelThreads) sh.cand[i] = fabs(res[sh.mcand[i]] - med);
            __syncthreads();
            cand_select(sh, ncand, kk2, want_lo);
            // the neighbour below the order statistic may be a counted (not gathered) slot unless it is >= L0
            if (want_lo && (kk2 == 0 || sh.sel_lo < L0)) mad_fast = false;
            else mad = want_lo ? (sh.sel_lo + sh.sel_hi) / 2.0 : sh.sel_hi;
            K2_STAMP(11, ncand);
            __syncthreads();
        }
        K2_STAMP(7, clock64());
        if (!mad_fast) {
            for (int i = tid; i < kBins; i += kSelThreads) sh.hist[i] = 0;
            __syncthreads();
            sweep_res(res, M, [&](double r) { atomicAdd(&sh.hist[sel_bin<true>(fabs(r - med))], 1u); });
            __syncthreads();
            mad = block_median<true>(sh, res, M, n, med);
            K2_STAMP(12, 1);
        }
        K2_STAMP(8, clock64());
        K2_STAMP(9, clock64());
    }
    if (tid == 0) {
        double sigma = 1.482602218505602 * mad;
        if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
        S.med = med;
        S.mad = mad;
        S.sigma = sigma;
        S.c = 4.6851 * sigma;
        S.n = n;
        S.n_ref_vis = nrv;
    }
}
// ------------------------------------------------------------------ K3: weights, normal-equation partials
// Same ownership and phases as K1 (ref windows only).  Per pixel slot: Tukey weight of r, dx/dy from the
// staged ref window, the Jacobian row J = dx * Jimg0 + dy * Jimg1 (src/image_alignment.cpp:186-188)
// and its weighted outer product accumulated in registers (21 H terms, 6 g terms, chi2).  A lane's
// accumulators are then combined by a halving exchange (32 shuffles for 28 terms) and per-wave sums are
// added in a fixed order: the partials of a workgroup are deterministic.
template <int kHalf>
__global__ void __launch_bounds__(kFeatThreads) align_weights_kernel(AlignArgs a, int level) {
    using G = Geo<kHalf>;
    constexpr int kRowIters = (G::FPB * G::RW + kFeatThreads - 1) / kFeatThreads;
    __shared__ __attribute__((aligned(16))) uint8_t win[G::FPB * G::fstride3];
    __shared__ WtRec rec[G::FPB];
    __shared__ double part[kFeatWaves][28];
    const int pair = blockIdx.x / a.chunks, chunk = blockIdx.x - pair * a.chunks;
    const PairState& S = a.state[pair];
    if (!S.active) return;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf, f0 = chunk * G::FPB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (f0 >= nf) {
        if (tid < 28) a.partials[((int64_t)pair * a.chunks + chunk) * 28 + tid] = 0.0;
        return;
    }
    const int nb = nf - f0 < G::FPB ? nf - f0 : G::FPB;
    const int W = a.geom.w[level];
    const int64_t loff = a.geom.off[level];
    const double dom = (double)(1 << level), scale = 1.0 / dom;
    const double c = S.c, c2 = c * c;
    const int64_t fbase = (int64_t)pair * a.max_f + f0;
    const double* __restrict__ res = a.res + (int64_t)pair * a.res_stride + (int64_t)f0 * G::A;
    const int ne = nb * G::A;
    const uint8_t* const ref_plane = P.ref_pyr + loff;
    const uint8_t* const kf_plane = P.kf_pyr + loff;
    // the first kPre residuals of this lane, loaded before the setup so their latency overlaps it
    constexpr int kPre = G::pix_iters < 8 ? G::pix_iters : 8;
    double rr[kPre];
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
        const int e = tid + i * kFeatThreads;
        rr[i] = e < ne ? res[e] : 0.0;
    }
    if (tid < G::FPB) {
        WtRec& R = rec[tid];
        int32_t vis = 0;
        const int64_t gf = fbase + (tid < nb ? tid : 0);  // all loads at once (see K1)
        const uint8_t fv = a.fvis[gf];
        const double pu = a.px[2 * gf], pv = a.px[2 * gf + 1];
        const V3 pw{a.xw[3 * gf], a.xw[3 * gf + 1], a.xw[3 * gf + 2]};
        if (tid < nb) {
            if (fv == 3) {
                vis = 3;
                const double ur = pu * scale, vr = pv * scale;
                const double fur = floor(ur), fvr = floor(vr);
                R.fx = ur - fur;
                R.fy = vr - fvr;
                R.rbase = (uint32_t)(((int)fvr - G::h - 1) * W + (int)fur - G::h - 1);
                image_jac(pw, a.fx / dom, a.fy / dom, R.ja, R.jb);
            }
        }
        R.vis = vis;
    }
    __syncthreads();
    uint4 blk[kRowIters][G::NB];  // all loads first, then the LDS stores (see K1)
#pragma unroll
    for (int i = 0; i < kRowIters; ++i) {
        const int j = tid + i * kFeatThreads;
        const int fl = j / G::RW < G::FPB ? j / G::RW : G::FPB - 1, row = j - fl * G::RW;
        const uint8_t* plane = f0 + fl < P.n_ref ? ref_plane : kf_plane;
        const uint32_t lin = rec[fl].vis == 3 ? rec[fl].rbase + (uint32_t)(row * W) : 0u;
        const uint8_t* src = plane + (lin & ~15u);
#pragma unroll
        for (int b = 0; b < G::NB; ++b) blk[i][b] = gload16(src + 16 * b);
    }
#pragma unroll
    for (int i = 0; i < kRowIters; ++i) {
        const int j = tid + i * kFeatThreads, fl = j / G::RW, row = j - fl * G::RW;
        if (j < G::FPB * G::RW) {
            uint4* d = reinterpret_cast<uint4*>(win + fl * G::fstride3 + row * G::pitch);
#pragma unroll
            for (int b = 0; b < G::NB; ++b) d[b] = blk[i][b];
        }
    }
    __syncthreads();
    double acc[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) acc[t] = 0.0;
    // Per pixel: Tukey weight, then dx/dy of the ref level at (u + x, v + y) (src/image_alignment.cpp:
    // 180-183).  The four bilinear samples share the feature's fractional weights, so they are formed
    // from 8 horizontal interpolants of the 12 window bytes around the pixel (same value as four
    // separate samples up to rounding).
    auto pixel = [&](int e, double r) {
        const int fl = e / G::A, k = e - fl * G::A;
        const WtRec& R = rec[fl];
        if (R.vis != 3 || !(fabs(r) <= c)) return;  // w = 0: no H, g or chi2 term (src/optimizer.cpp:502-511)
        const double tt = 1.0 - (r * r) / c2;
        const double w = tt * tt;
        acc[27] = fma(r * r, w, acc[27]);
        const int cy = k / G::side + 1, cx = k - (k / G::side) * G::side + 1;  // window cell of floor(u+x, v+y)
        const uint8_t* wr = win + fl * G::fstride3;
        uint32_t q[4];  // rows cy-1 .. cy+2, bytes at cols cx-1 .. cx+2
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = cy - 1 + i;
            q[i] = lds_bytes4(wr, row * G::pitch + (int)((R.rbase + (uint32_t)(row * W)) & 15u) + cx - 1);
        }
        const double fx = R.fx, gx = 1.0 - fx, fy = R.fy, gy = 1.0 - fy;
        auto hv = [&](int i, int c0) { return fma(fx, byte_d(q[i], c0 + 1), gx * byte_d(q[i], c0)); };
        const double dx = 0.5 * (gy * (hv(1, 2) - hv(1, 0)) + fy * (hv(2, 2) - hv(2, 0)));
        const double dy = 0.5 * ((gy * hv(2, 1) + fy * hv(3, 1)) - (gy * hv(0, 1) + fy * hv(1, 1)));
        double J[6], wJ[6];
#pragma unroll
        for (int q6 = 0; q6 < 6; ++q6) {
            J[q6] = fma(dx, R.ja[q6], dy * R.jb[q6]);
            wJ[q6] = w * J[q6];
        }
        // fused multiply-adds: the accumulation order already differs from the reference's GEMM
        int t = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) { acc[t] = fma(wJ[i], J[j], acc[t]); ++t; }
#pragma unroll
        for (int i = 0; i < 6; ++i) acc[21 + i] = fma(wJ[i], r, acc[21 + i]);
    };
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
        const int e = tid + i * kFeatThreads;
        if (e < ne) pixel(e, rr[i]);
    }
    for (int i = kPre; i < G::pix_iters; ++i) {
        const int e = tid + i * kFeatThreads;
        if (e < ne) pixel(e, res[e]);
    }
    // halving exchange: after the steps of offsets 32..2 lane L holds term L >> 1 (half of it)
#pragma unroll
    for (int o = 32, n = 32; o >= 2; o >>= 1, n >>= 1) {
        const bool up = (lane & o) != 0;
#pragma unroll
        for (int q = 0; q < n / 2; ++q) {
            const double keep = up ? acc[q + n / 2] : acc[q];
            const double send = up ? acc[q] : acc[q + n / 2];
            acc[q] = keep + __shfl_xor(send, o, 64);
        }
    }
    acc[0] += __shfl_xor(acc[0], 1, 64);
    if ((lane & 1) == 0 && (lane >> 1) < 28) part[wave][lane >> 1] = acc[0];
    __syncthreads();
    if (tid < 28) {
        double s = 0.0;
        for (int w = 0; w < kFeatWaves; ++w) s += part[w][tid];
        a.partials[((int64_t)pair * a.chunks + chunk) * 28 + tid] = s;
    }
}

// ------------------------------------------------------------------ K4: normal equations, LM step
namespace {
struct SolveShared {
    double tot[28];
    double A[36];
    double tmp[6];
    int32_t perm[6];
};
}  // namespace

__global__ void __launch_bounds__(64) align_solve_kernel(AlignArgs a, int level) {
    __shared__ SolveShared sh;
    const int pair = blockIdx.x, tid = threadIdx.x;
    PairState& S = a.state[pair];
    const bool last = level == a.min_level;
    if (S.active) {
        if (tid < 28) {  // chunk partials in a fixed order
            const double* p = a.partials + (int64_t)pair * a.chunks * 28 + tid;
            double s = 0.0;
            for (int c = 0; c < a.chunks; ++c) s += p[c * 28];
            sh.tot[tid] = s;
        }
        __syncthreads();
        if (tid == 0) {
            double g[6], dx[6];
            int q = 0;
            for (int r = 0; r < 6; ++r)
                for (int cidx = 0; cidx <= r; ++cidx) {
                    const double v = sh.tot[q++];
                    sh.A[r * 6 + cidx] = v;
                    sh.A[cidx * 6 + r] = v;
                }
            for (int r = 0; r < 6; ++r) g[r] = sh.tot[21 + r];
            const double chi = sh.tot[27];
            double mx = sh.A[0];
            for (int r = 1; r < 6; ++r) mx = fmax(mx, sh.A[r * 7]);
            const double lambda = 1e-2 * mx;
            for (int r = 0; r < 6; ++r) sh.A[r * 7] += lambda;
            svo_level_trace& t = a.traces[(int64_t)pair * (a.max_level + 1) + level];
            for (int r = 0; r < 36; ++r) t.H[r] = sh.A[r];
            ldlt_solve_ws(6, sh.A, g, dx, sh.perm, sh.tmp);
            double m[6];
            for (int r = 0; r < 6; ++r) m[r] = -dx[r];
            const SE3 np = se3_compose(se3_load(S.pose), se3_exp(m));
            se3_store(np, S.pose);
            bool big = false, nan = false;
            for (int r = 0; r < 6; ++r) { big |= dx[r] > 1e3; nan |= isnan(dx[r]); }
            int32_t st = kSuccess;
            if (big) st = kMaxCoffDx;
            else if (nan) st = kNonInDx;
            else {
                double step = 0.0;
                for (int r = 0; r < 6; ++r) step += dx[r] * dx[r];
                st = step < 1e-16 ? kSmallStepSize : st;
                st = fabs(lambda) >= 1e14 ? kLambdaValue : st;
            }
            const double e = sqrt(chi / (double)S.n);
            t.level = level; t.n_ref_vis = (int32_t)S.n_ref_vis; t.n_vis = (int32_t)S.n; t.status = st;
            t.median = S.med; t.mad = S.mad; t.sigma = S.sigma; t.chi2 = chi; t.lambda = lambda; t.err = e;
            for (int r = 0; r < 6; ++r) { t.g[r] = g[r]; t.dx[r] = dx[r]; }
            S.err = e;
            S.status = st;
        }
    }
    if (last && tid == 0) {
        for (int i = 0; i < 7; ++i) a.pose_out[7 * pair + i] = S.pose[i];
        a.err_out[pair] = S.err;
        a.status_out[pair] = S.status;
    }
}

// ------------------------------------------------------------------ launch
// marks (optional): an event recorded before every launch and after the last one, in launch order
// K0, then per level K1 K2 K3 K4 (1 + 4 * levels + 1 events)
template <int kHalf>
static void launch_all(const AlignArgs& a, hipStream_t s, hipEvent_t* marks) {
    int m = 0;
    auto mark = [&]() {
        if (marks) (void)hipEventRecord(marks[m++], s);
    };
    const int64_t nthreads = (int64_t)a.n_pairs * a.max_f;
    const int64_t blocks = (nthreads > a.n_pairs ? nthreads : a.n_pairs) / 256 + 1;
    mark();
    hipLaunchKernelGGL(align_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
    const unsigned fgrid = (unsigned)((int64_t)a.n_pairs * a.chunks);
    for (int level = a.max_level; level >= a.min_level; --level) {
        mark();
        hipLaunchKernelGGL(align_residual_kernel<kHalf>, dim3(fgrid), dim3(kFeatThreads), 0, s, a, level);
        mark();
        hipLaunchKernelGGL(align_scale_kernel, dim3(a.n_pairs), dim3(kSelThreads), 0, s, a, level);
        mark();
        hipLaunchKernelGGL(align_weights_kernel<kHalf>, dim3(fgrid), dim3(kFeatThreads), 0, s, a, level);
        mark();
        hipLaunchKernelGGL(align_solve_kernel, dim3(a.n_pairs), dim3(64), 0, s, a, level);
    }
    mark();
}

void launch_align(const AlignArgs& a, hipStream_t s, hipEvent_t* marks) {
    switch (a.half) {
        case 0: launch_all<0>(a, s, marks); break;
        case 1: launch_all<1>(a, s, marks); break;
        case 2: launch_all<2>(a, s, marks); break;
        case 3: launch_all<3>(a, s, marks); break;
        case 4: launch_all<4>(a, s, marks); break;
        case 5: launch_all<5>(a, s, marks); break;
        case 6: launch_all<6>(a, s, marks); break;
        case 7: launch_all<7>(a, s, marks); break;
        case 8: launch_all<8>(a, s, marks); break;
        default: launch_all<9>(a, s, marks); break;  // the C ABI rejects larger patches
    }
}

int align_max_half() { return 9; }

#if defined(SVO_STAMPS)
extern "C" int svo_debug_stamps(void* out, size_t bytes) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps)) == hipSuccess ? 0 : -2;
}
#endif

}  // namespace svo
