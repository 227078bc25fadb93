// align.hip — sparse image alignment (ImageAlignment::align, src/image_alignment.cpp:25-67) on gfx950.
//
// A batch holds n_pairs independent frame pairs.  The coarse-to-fine chain runs as
// stage kernels over all pairs of the batch, enqueued back to back on the context stream:
//   per level (max..min):
//   K1 residual  lane / feature (256-lane workgroups); at the first level it also forms the world points
//                X_w = T_f^-1 (bearing * |P - C_f|) (:153-155) and the pair state (init_pair)
//                ref visibility (border rule :140-149), projection
//                pose * X_w into cur (:320-340); the feature's ref and cur windows are loaded into
//                registers, one 16-B load per window row, and r = I_cur - T_ref (:359) is formed with the
//                reference's own bilinear arithmetic in separable form: each window row's horizontal
//                blends are computed once and shared by the two patch rows that use them (same values,
//                same rounding as algorithm::bilinearInterpolationDouble, src/algorithm.cpp:896-905)
//   K2 scale     one workgroup / pair: exact median of the visible r (src/algorithm.cpp:834-853) and of
//                |r - median| (MAD, :855-865) -> sigma = 1.482602218505602 * MAD (:867-872).  Values
//                are binned by a monotone map into an LDS histogram; the bin of rank n/2 is exact; one
//                sweep gathers that bin's values into LDS and ranks them exactly; an overfull bin falls
//                back to an 11-bit radix select on order-preserving keys
//   K3 weights   lane / feature: Tukey weight (src/optimizer.cpp:485-514), chi2 term, dx/dy of the ref
//                level from the register-resident window (:180-183); the lane accumulates the 5 sums
//                S_xx S_xy S_yy S_xr S_yr of its feature and expands them with the 2x6 image Jacobian
//                (J row = dx * Jimg0 + dy * Jimg1, :186-188) into the 21 + 6 normal-equation terms; a
//                halving exchange sums the wave's features into per-workgroup partials.  The last
//                workgroup of a pair to publish (device-scope arrival counter) sums the partials in a
//                fixed order (deterministic, no float atomics) and takes the LM step: Nielsen damping,
//                Eigen-LDLT, pose <- pose * exp(-dx), status, RMSE (src/optimizer.cpp:279-366,
//                src/image_alignment.cpp:379)
#include <type_traits>

#include "svo_internal.h"
#include "svo_math.h"
#include "svo_wave.h"

namespace svo {
#if defined(SVO_TIMELINE)
SVO_TL_DEFINE(k13)
SVO_TL_READER(k13)
#endif


namespace {

constexpr int kLaneFeats = 256;      // K1 / K3 workgroup: 4 waves, one feature per lane
constexpr int kLaneWaves = kLaneFeats / 64;
constexpr int kSelThreads = 512;     // K2 workgroup (two per CU)
constexpr int kSelWaves = kSelThreads / 64;
constexpr int kBins = 4096;
constexpr double kBinScale = 32.0;   // bins per grey level
constexpr double kBinOffset = 64.0;  // signed map covers [-64, 64); outliers clamp to the end bins
constexpr double kKeyScale = 512.0;  // K1's 16-bit residual key: 16 keys per value bin
constexpr uint32_t kKeyMax = 65534;  // largest key of a visible slot; 0xFFFF = invisible
constexpr int kCandCap = 2048;
constexpr int kRankCap = 256;        // <= this many candidates: rank counting, else bitonic sort
constexpr int kPrevCap = 256;        // slots of the bin below the median's gathered for its lower neighbour
constexpr int kRadixBits = 11;
constexpr double kDblMax = 1.7976931348623157e308;

// Window geometry of one feature at one level (patch half size kHalf), in image cells relative to
// (floor(u), floor(v)) of the feature at that level.
template <int kHalf>
struct Win {
    static constexpr int h = kHalf, side = 2 * kHalf + 1, A = side * side;
    static constexpr int RB = 2 * h + 2;           // K1: rows and bytes -h .. h+1 (bilinear corners)
    static constexpr int WB = 2 * h + 4;           // K3: rows and bytes -h-1 .. h+2 (corners of the +-1 samples)
    static constexpr int RW = (RB + 3) / 4;        // dwords kept per K1 row
    static constexpr int WW = (WB + 3) / 4;        // dwords kept per K3 row
    static constexpr int RD = (RB + 3 + 3) / 4;    // dwords loaded per K1 row (dword-aligned start)
    static constexpr int WD = (WB + 3 + 3) / 4;    // dwords loaded per K3 row
};

// 16-B load from an image plane.  The plane pointers come from the device-resident pair table, so the
// compiler only sees generic pointers; the explicit global address space keeps these loads off the flat
// path.  Only 4-B alignment is required (and given).
__device__ __forceinline__ uint4 gload16(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(1))) const uint4 gu4;
    return *(gu4*)(p);
#else
    return *reinterpret_cast<const uint4*>(p);  // host pass only parses device code
#endif
}

// One window row: image bytes [lin, lin + 4 NW) of `plane` -> out (little-endian dwords), loaded as the
// ND dwords from the dword below `lin` (16-, 12-, 8- or 4-B global loads) and re-aligned with byte funnel
// shifts.  Bytes past the row's window are don't-care (the pyramid planes are padded, so the loads stay
// inside the allocation).
template <int ND, int NW>
__device__ __forceinline__ void load_row(const uint8_t* plane, uint32_t lin, uint32_t (&out)[NW]) {
    uint32_t d[ND + 1];
    const uint8_t* p = plane + (lin & ~3u);
#pragma unroll
    for (int q = 0; q + 4 <= ND; q += 4) {
        const uint4 v = gload16(p + 4 * q);
        d[q] = v.x; d[q + 1] = v.y; d[q + 2] = v.z; d[q + 3] = v.w;
    }
    constexpr int q0 = ND & ~3;
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int rem = ND & 3;
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    typedef __attribute__((address_space(1))) const u32x3 g3;
    typedef __attribute__((address_space(1))) const uint2 g2;
    typedef __attribute__((address_space(1))) const uint32_t g1;
    if constexpr (rem == 3) { const u32x3 v = *(g3*)(p + 4 * q0); d[q0] = v.x; d[q0 + 1] = v.y; d[q0 + 2] = v.z; }
    if constexpr (rem == 2) { const uint2 v = *(g2*)(p + 4 * q0); d[q0] = v.x; d[q0 + 1] = v.y; }
    if constexpr (rem == 1) { d[q0] = *(g1*)(p + 4 * q0); }
#else
    for (int q = q0; q < ND; ++q) d[q] = reinterpret_cast<const uint32_t*>(p)[q];
#endif
    d[ND] = 0u;
    const uint32_t sh = lin & 3u;
#pragma unroll
    for (int i = 0; i < NW; ++i) out[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
}
template <int NW>
__device__ __forceinline__ double wbyte(const uint32_t (&w)[NW], int j) {  // byte j of a row, as double
    return (double)((w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
}

// Raw buffer access to one pair's residual / key rows: the resource (base, size) is wave-uniform, the
// slot row offset k * fstride goes in the scalar offset and the lane's feature in a 32-bit vector offset,
// so a slot store / load is one instruction with no per-lane 64-bit address arithmetic.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(const void* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void slot_store(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rs, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ void slot_store16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint16_t v) {
    __builtin_amdgcn_raw_buffer_store_b16(v, rs, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ double slot_load(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)voff, (int)soff, 0));
}

// Feature windows of a window level (AlignArgs::win): per pair, the ref section (WB rows of WW dwords) then
// the cur section (RB rows of RW dwords), each row a [feature][N dwords] plane of fstride features, so a
// wave's access to one row is one contiguous run.  voff = the lane's feature * 4N, soff = the row's base.
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int N>
__device__ __forceinline__ void win_store(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, const uint32_t (&v)[N]) {
    int i = 0;
#pragma unroll
    for (; i + 4 <= N; i += 4)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[i], v[i + 1], v[i + 2], v[i + 3]}, rs, (int)(voff + 4 * i), (int)soff, 0);
    if constexpr (N % 4 == 3) __builtin_amdgcn_raw_buffer_store_b96(u32x3{v[i], v[i + 1], v[i + 2]}, rs, (int)(voff + 4 * i), (int)soff, 0);
    if constexpr (N % 4 == 2) __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[i], v[i + 1]}, rs, (int)(voff + 4 * i), (int)soff, 0);
    if constexpr (N % 4 == 1) __builtin_amdgcn_raw_buffer_store_b32(v[i], rs, (int)(voff + 4 * i), (int)soff, 0);
}
template <int N>
__device__ __forceinline__ void win_load(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint32_t (&v)[N]) {
    int i = 0;
#pragma unroll
    for (; i + 4 <= N; i += 4) {
        const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(voff + 4 * i), (int)soff, 0);
        v[i] = t.x; v[i + 1] = t.y; v[i + 2] = t.z; v[i + 3] = t.w;
    }
    if constexpr (N % 4 == 3) {
        const u32x3 t = __builtin_amdgcn_raw_buffer_load_b96(rs, (int)(voff + 4 * i), (int)soff, 0);
        v[i] = t.x; v[i + 1] = t.y; v[i + 2] = t.z;
    }
    if constexpr (N % 4 == 2) {
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(voff + 4 * i), (int)soff, 0);
        v[i] = t.x; v[i + 1] = t.y;
    }
    if constexpr (N % 4 == 1) v[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(voff + 4 * i), (int)soff, 0);
}

// (x, y) -> (x with its upper kSpan-lane blocks replaced by y's lower ones, y with its lower blocks replaced
// by x's upper ones): v_permlane32_swap / v_permlane16_swap on both 32-bit halves.  x + y then holds
// x's pair sums in the blocks with lane bit log2(kSpan) clear and y's where it is set.
template <int kSpan>
__device__ __forceinline__ void lane_swap(double& x, double& y) {
    const uint2 a = __builtin_bit_cast(uint2, x), b = __builtin_bit_cast(uint2, y);
    uint2 na, nb;
    if constexpr (kSpan == 32) {
        const auto lo = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
        na = make_uint2(lo[0], hi[0]); nb = make_uint2(lo[1], hi[1]);
    } else {
        const auto lo = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
        na = make_uint2(lo[0], hi[0]); nb = make_uint2(lo[1], hi[1]);
    }
    x = __builtin_bit_cast(double, na);
    y = __builtin_bit_cast(double, nb);
}

// 16-bit monotone key of a residual for K2's sweeps: floor((r + 64) * 512) clamped to [0, kKeyMax];
// 0xFFFF marks an invisible slot.  key >> 4 is exactly the value bin floor((r + 64) * 32) of K2.
// (r finite.)  fma(r, 512, 32768) rounds exactly like (r + 64) * 512 (scaling by a power of two commutes
// with rounding): one fma, a clamp at 0, the conversion and a min per pixel.
__device__ __forceinline__ uint16_t res_key(double r) {
    const double t = fmax(fma(r, kKeyScale, kBinOffset * kKeyScale), 0.0);
    const uint32_t k = (uint32_t)t;
    return (uint16_t)(k < kKeyMax ? k : kKeyMax);
}

// XCD-aware workgroup -> (pair, chunk) map for K1 / K3.  Workgroups are dealt round-robin over the
// 8 XCDs (b and b + 8 share one), so the workgroups b = 8 s + x of XCD x take pair 8 (s / chunks) + x,
// chunk s % chunks: every chunk of a pair runs on one XCD, back to back, and the pair's image lines
// are fetched into one L2 instead of eight.  K2 (one workgroup per pair) lands on the same XCD.  The
// grid is rounded up to whole groups of 8 pairs; workgroups of pairs >= n_pairs exit.  Placement only
// affects speed, never results.
__device__ __forceinline__ void xcd_pair_chunk(int chunks, int& pair, int& chunk) {
    const int b = (int)blockIdx.x, x = b & 7, s = b >> 3, grp = s / chunks;
    chunk = s - grp * chunks;
    pair = grp * 8 + x;
}

// Slot rows of a pair are fstride = n_features rounded up to 64 wide: a wave's 64 keys of one patch pixel
// are one whole aligned 128-B line.
__device__ __forceinline__ int slot_stride(int nf) { return (nf + 63) & ~63; }

}  // namespace

int align_feat_iters() { return 1; }
int align_win_dwords(int half) {
    const int RB = 2 * half + 2, WB = 2 * half + 4;
    return WB * ((WB + 3) / 4) + RB * ((RB + 3) / 4);
}

int align_chunks(int max_f, int half, int feat_iters) {
    (void)half;
    (void)feat_iters;
    return (max_f + kLaneFeats - 1) / kLaneFeats;
}

// ------------------------------------------------------------------ pair state, world points
// Done by the first (coarsest) level's K1 rather than a launch of its own: one pass over the batch's
// feature records instead of two, and one launch less per chain.
__device__ __forceinline__ bool pair_active(const PairDesc& P, int area) {
    return P.n_ref > 0 && (int64_t)(P.n_ref + P.n_kf) * area >= 6;
}

// the pair's optimizer state before the first level (src/image_alignment.cpp:25-60): pose, status, the
// per-level traces; one lane
__device__ void init_pair(const AlignArgs& a, const PairDesc& P, int pair) {
    PairState& S = a.state[pair];
    for (int i = 0; i < 7; ++i) S.pose[i] = P.cur_pose[i];
    S.active = pair_active(P, a.area) ? 1 : 0;
    S.err = P.n_ref == 0 ? 0.0 : -1.0;  // align() returns 0 (:27-28); optimizeLM returns -1 when M < 6
    S.status = P.n_ref == 0 ? kFailed : kNonSuffPoints;
    a.arrive[pair] = 0u;
    svo_level_trace* tr = a.traces + pair * (a.max_level + 1);
    for (int l = 0; l <= a.max_level; ++l) {
        svo_level_trace t = {};
        t.level = l;
        t.status = kFailed;
        tr[l] = t;
    }
}

// world point of feature f (src/image_alignment.cpp:153-155): the frame's inverse pose applied to the
// bearing scaled by the distance of the feature's point from the camera centre
__device__ __forceinline__ V3 world_point(const AlignArgs& a, const PairDesc& P, int64_t gf, bool is_ref) {
    const SE3 T = se3_load(is_ref ? P.ref_pose : P.kf_pose);
    const V3 C = camera_in_world(T);
    const V3 Pw{a.point[3 * gf], a.point[3 * gf + 1], a.point[3 * gf + 2]};
    const double depth = v3norm(v3sub(Pw, C));
    const V3 pc = v3scl(V3{a.bearing[3 * gf], a.bearing[3 * gf + 1], a.bearing[3 * gf + 2]}, depth);
    return se3_act(se3_inverse(T), pc);
}

// ------------------------------------------------------------------ K1: visibility, projection, residuals
// One lane per feature slot f of the pair (f < fstride; slots past n_features are written invisible).
// Per pixel (kx, ky) the reference computes T = bilerpD(I_ref, u + kx, v + ky) and I = bilerpD(I_cur,
// cu + kx, cv + ky) (src/image_alignment.cpp:169-176, :351-359).  With x = u + kx, x1 = (int)x, the
// column weights x - x1 and x2 - x = 1 - (x - x1) (both exact for x >= 1) depend on kx only and the row
// blends a = (x2 - x) I(y, x1) + (x - x1) I(y, x2) on (image row, kx) only, so every window row's blends
// are formed once and shared by the two patch rows that read them: bit-identical to the per-sample
// formula whenever x1 = floor(u) + kx and y1 = floor(v) + ky.  A feature where u + kx rounds up to the
// next integer (x1 = floor(u) + kx + 1) takes the per-pixel path instead.
// kRef (median_mode SVO_MEDIAN_REFERENCE): the exact residuals (doubles, DBL_MAX for an invisible slot) in
// the reference's feature-major slot order (slot f * area + k, the vector K2R's introselect runs over)
// instead of 16-bit pixel-major keys.
template <int kHalf, bool kWin, bool kRef>  // kWin: a window level (AlignArgs::win_levels)
__global__ void __launch_bounds__(kLaneFeats, kHalf <= 2 ? 3 : 2) align_residual_kernel(AlignArgs a, int level) {
    using G = Win<kHalf>;
    using KeyT = typename std::conditional<kRef, double, uint16_t>::type;
    constexpr int h = G::h, side = G::side, RB = G::RB, NW = G::RW;
    constexpr KeyT kInvis = kRef ? (KeyT)1.7976931348623157e308 : (KeyT)0xFFFF;
    // keys are staged in LDS ([pixel][feature], or [feature][pixel] for kRef) and written as whole 16-B
    // pieces of the slot rows (one 2-B store per lane and pixel wrote each 128-B line in many partial
    // requests: 2.8x the key bytes)
    // (kRef: the residual doubles are staged too, up to 64 KB: one 8-B store per lane and pixel at a
    // 200-B lane stride touched 64 lines per instruction)
    constexpr bool kLds = G::A * kLaneFeats * (int)sizeof(KeyT) <= (kRef ? 65536 : 32768);
    __shared__ __attribute__((aligned(16))) KeyT kbuf[kLds ? G::A * kLaneFeats : 1];
    SVO_TL_SCOPE(k13, kTlK1, level, a.pair_base);
    int pair, chunk;
    xcd_pair_chunk(a.chunks, pair, chunk);
    if (pair >= a.n_pairs) return;
    const PairDesc& P = a.pairs[pair];
    // the first level initialises the pair (one lane) and forms the world points; its other lanes take
    // the initial pose and the active flag from the pair record, not from the state being written
    const bool first = level == a.max_level;
    if (first && chunk == 0 && threadIdx.x == 0) init_pair(a, P, pair);
    if (!(first ? pair_active(P, a.area) : a.state[pair].active != 0)) return;
    const double* const pose = first ? P.cur_pose : a.state[pair].pose;
    const int nf = P.n_ref + P.n_kf, fstride = slot_stride(nf);
    const int tid = (int)threadIdx.x, f0 = chunk * kLaneFeats, f = f0 + tid;
    if (f0 >= fstride) return;  // whole workgroup
    const int W = a.geom.w[level], H = a.geom.h[level];
    const int64_t loff = a.geom.off[level];
    const double scale = ldexp(1.0, -level);  // = 1 / 2^level exactly, no division
    const int border = h + 2;
    // key of slot (k, f) at keys[k * fstride + f] (kRef: keys32[f * area + k])
    const __amdgpu_buffer_rsrc_t keys = slot_rsrc(a.keys + (int64_t)pair * a.key_stride, a.key_stride * 2);
    const uint32_t fo = (uint32_t)f;
    auto put = [&](int k, KeyT key) {
        if constexpr (kLds) {
            if constexpr (kRef) kbuf[tid * G::A + k] = key;
            else kbuf[k * kLaneFeats + tid] = key;
        } else if constexpr (kRef) {
            a.scratch[(int64_t)pair * a.key_stride + (int64_t)f * G::A + k] = key;
        } else {
            slot_store16(keys, 2 * fo, 2 * (uint32_t)(k * fstride), key);
        }
    };
    auto rkey = [](double r) -> KeyT {
        if constexpr (kRef) return r;
        else return res_key(r);
    };
    int vis = 0;
    double ur = 0.0, vr = 0.0, cu = 0.0, cv = 0.0;
    if (f < nf) {
        const int64_t gf = (int64_t)pair * a.max_f + f;
        const uint8_t hp = a.has_point[gf];  // all of the feature's loads at once (one memory round trip)
        const double pu = a.px[2 * gf], pv = a.px[2 * gf + 1];
        V3 pw{0.0, 0.0, 0.0};
        if (!first) {
            pw = V3{a.xw[3 * gf], a.xw[3 * gf + 1], a.xw[3 * gf + 2]};
        } else if (hp) {
            pw = world_point(a, P, gf, f < P.n_ref);
            a.xw[3 * gf] = pw.x; a.xw[3 * gf + 1] = pw.y; a.xw[3 * gf + 2] = pw.z;
        }
        if (hp) {
            ur = pu * scale;
            vr = pv * scale;
            const int ui = (int)floor(ur), vi = (int)floor(vr);
            if (!((ui - border) < 0 || (vi - border) < 0 || (ui + border) >= W || (vi + border) >= H)) {
                vis = 1;
                const V3 cp = se3_act(se3_load(pose), pw);
                cu = (a.fx * (cp.x / cp.z) + a.cx) * scale;
                cv = (a.fy * (cp.y / cp.z) + a.cy) * scale;
                const int cui = (int)floor(cu), cvi = (int)floor(cv);
                if (!((cui - border) < 0 || (cvi - border) < 0 || (cui + border) >= W || (cvi + border) >= H)) {
                    vis = 3;
                    reinterpret_cast<double2*>(a.cproj)[gf] = make_double2(cu, cv);
                }
            }
        }
        a.fvis[gf] = (uint8_t)vis;
    }
    if (vis != 3) {
        if (f < fstride) {
#pragma unroll
            for (int k = 0; k < G::A; ++k) put(k, kInvis);
        }
    } else {
        const uint8_t* const rplane = (f < P.n_ref ? P.ref_pyr : P.kf_pyr) + loff;
        const uint8_t* const cplane = P.cur_pyr + loff;
        const int ru = (int)floor(ur), rv = (int)floor(vr), qu = (int)floor(cu), qv = (int)floor(cv);
        double rwx[side], cwx[side];  // x - x1 per patch column (y - y1 per patch row: formed in the row loop)
        bool fast = true;
#pragma unroll
        for (int k = 0; k < side; ++k) {
            const double d = (double)(k - h);
            const double xr = ur + d, xc = cu + d;
            const int xr1 = (int)xr, xc1 = (int)xc;
            fast = fast && xr1 == ru + k - h && xc1 == qu + k - h && (int)(vr + d) == rv + k - h &&
                   (int)(cv + d) == qv + k - h;
            rwx[k] = xr - (double)xr1;
            cwx[k] = xc - (double)xc1;
        }
        uint32_t rrow[RB][NW], crow[RB][NW];
        if constexpr (kWin) {  // window level: K3's ref window (rows / bytes -h-1 .. h+2) and the cur window, handed on
            uint32_t wrow[G::WB][G::WW];
#pragma unroll
            for (int R = 0; R < G::WB; ++R) load_row<G::WD>(rplane, (uint32_t)((rv - h - 1 + R) * W + (ru - h - 1)), wrow[R]);
#pragma unroll
            for (int r = 0; r < RB; ++r) load_row<G::RD>(cplane, (uint32_t)((qv - h + r) * W + (qu - h)), crow[r]);
            const __amdgpu_buffer_rsrc_t ws = slot_rsrc(a.win + (int64_t)pair * a.win_stride, a.win_stride * 4);
#pragma unroll
            for (int R = 0; R < G::WB; ++R) win_store<G::WW>(ws, fo * (4 * G::WW), (uint32_t)(R * fstride * 4 * G::WW), wrow[R]);
            const uint32_t cbase = (uint32_t)(G::WB * G::WW * fstride * 4);
#pragma unroll
            for (int r = 0; r < RB; ++r) win_store<NW>(ws, fo * (4 * NW), cbase + (uint32_t)(r * fstride * 4 * NW), crow[r]);
#pragma unroll
            for (int r = 0; r < RB; ++r)  // K1's rows: window rows 1.., shifted by one byte
#pragma unroll
                for (int i = 0; i < NW; ++i)
                    rrow[r][i] = __builtin_amdgcn_alignbyte(i + 1 < G::WW ? wrow[r + 1][i + 1] : 0u, wrow[r + 1][i], 1);
        } else {
            if (fast) {
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    load_row<G::RD>(rplane, (uint32_t)((rv - h + r) * W + (ru - h)), rrow[r]);
                    load_row<G::RD>(cplane, (uint32_t)((qv - h + r) * W + (qu - h)), crow[r]);
                }
            }
        }
        if (fast) {
            double rprev[side], cprev[side];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                double rcur[side], ccur[side];
#pragma unroll
                for (int kx = 0; kx < side; ++kx) {  // (x2 - x) I(y, x1) + (x - x1) I(y, x2)
                    rcur[kx] = (1.0 - rwx[kx]) * wbyte(rrow[r], kx) + rwx[kx] * wbyte(rrow[r], kx + 1);
                    ccur[kx] = (1.0 - cwx[kx]) * wbyte(crow[r], kx) + cwx[kx] * wbyte(crow[r], kx + 1);
                }
                if (r > 0) {
                    const int ky = r - 1;
                    const double d = (double)(ky - h), yr = vr + d, yc = cv + d;
                    const double rwy = yr - (double)(rv + ky - h), cwy = yc - (double)(qv + ky - h);  // y - y1
#pragma unroll
                    for (int kx = 0; kx < side; ++kx) {  // (y2 - y) a + (y - y1) b
                        const double T = (1.0 - rwy) * rprev[kx] + rwy * rcur[kx];
                        const double I = (1.0 - cwy) * cprev[kx] + cwy * ccur[kx];
                        put(ky * side + kx, rkey(I - T));
                    }
                }
#pragma unroll
                for (int kx = 0; kx < side; ++kx) { rprev[kx] = rcur[kx]; cprev[kx] = ccur[kx]; }
            }
        } else {
            for (int ky = 0; ky < side; ++ky)
                for (int kx = 0; kx < side; ++kx) {
                    const double T = bilinear_d(rplane, W, ur + (double)(kx - h), vr + (double)(ky - h));
                    const double I = bilinear_d(cplane, W, cu + (double)(kx - h), cv + (double)(ky - h));
                    put(ky * side + kx, rkey(I - T));
                }
        }
    }
    if constexpr (kLds && kRef) {  // the workgroup's features are one contiguous run of slots
        __syncthreads();
        const int nfe = fstride - f0 < kLaneFeats ? fstride - f0 : kLaneFeats;  // a multiple of 64
        double* const kp = a.scratch + (int64_t)pair * a.key_stride + (int64_t)f0 * G::A;
        for (int idx = tid; idx < nfe * G::A / 2; idx += kLaneFeats)
            *reinterpret_cast<uint4*>(kp + 2 * idx) = *reinterpret_cast<const uint4*>(&kbuf[2 * idx]);
    } else if constexpr (kLds) {
        __syncthreads();
        const int per_row = (fstride - f0 < kLaneFeats ? fstride - f0 : kLaneFeats) / 8;  // 16-B pieces
        uint16_t* const kp = a.keys + (int64_t)pair * a.key_stride + f0;
        for (int idx = tid; idx < G::A * per_row; idx += kLaneFeats) {
            const int k = idx / per_row, c8 = idx - k * per_row;
            *reinterpret_cast<uint4*>(kp + (int64_t)k * fstride + 8 * c8) =
                *reinterpret_cast<const uint4*>(&kbuf[k * kLaneFeats + 8 * c8]);
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
    uint32_t pcand[kPrevCap];  // slots of the highest non-empty bin below the median's (even length, rank 0)
    double small[kRankCap];    // values of one fine bin (cand_select)
    uint32_t scan[kSelWaves];
    uint32_t ired[kSelWaves][2];
    double red[kSelWaves], red2[kSelWaves];
    uint64_t sel_prefix;
    uint32_t sel_k, sel_cnt, sel_bits, sel_bin, cand_n, mcand_n, pcand_n, small_n;
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

// The exact residual of one slot, recomputed from the images: K1 keeps only the 16-bit keys and the
// projection of each visible feature, so K2 evaluates r = bilerpD(I_cur, cu + kx, cv + ky) -
// bilerpD(I_ref, u + kx, v + ky) (src/image_alignment.cpp:351-359) for the few slots it must rank
// exactly; the per-sample formula is the one K1's separable form reproduces bit for bit.
struct SlotSrc {
    const uint16_t* keys;
    double* scratch;        // pair's slot row for the exact paths (materialize())
    const double* px;       // pair's feature pixels (level 0)
    const double* cproj;    // pair's projections into the cur level (K1)
    const uint8_t *rplane, *kplane, *cplane;
    int W, fstride, n_ref, side, half;
    double scale;
    __device__ __forceinline__ double r(uint32_t s) const {
        const int k = (int)(s / (uint32_t)fstride), f = (int)(s - (uint32_t)k * (uint32_t)fstride);
        const int ky = k / side, kx = k - ky * side;
        const double ur = px[2 * f] * scale, vr = px[2 * f + 1] * scale;
        const double cu = cproj[2 * f], cv = cproj[2 * f + 1];
        const double T = bilinear_d(f < n_ref ? rplane : kplane, W, ur + (double)(kx - half), vr + (double)(ky - half));
        const double I = bilinear_d(cplane, W, cu + (double)(kx - half), cv + (double)(ky - half));
        return I - T;
    }
};

// Exact residual of every slot (+inf = invisible) into the pair's scratch row, for the exact paths of K2
// (overfull bins; a neighbour the bin bracket cannot settle): four slots in flight per lane.
__device__ __forceinline__ void materialize(const SlotSrc& res, int Ms) {
    for (int s0 = threadIdx.x; s0 < Ms; s0 += 4 * kSelThreads) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int s = s0 + u * kSelThreads;
            v[u] = (s < Ms && res.keys[s] != 0xFFFF) ? res.r((uint32_t)s) : __builtin_inf();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int s = s0 + u * kSelThreads;
            if (s < Ms) res.scratch[s] = v[u];
        }
    }
    __syncthreads();
}

// Sweep the materialized residual row (Ms slots, a multiple of 8), 4 x 16-B loads in flight per lane;
// fn(value) for each visible slot.
template <typename Fn>
__device__ __forceinline__ void sweep_res(const SlotSrc& src, int M, Fn fn) {
    const double* __restrict__ res = src.scratch;
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
// trip per chunk; a config-2 pair, 50 000 slots, is one chunk).  M8 (slots) is a multiple of 8.
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

// The gather's key filter: three inclusive 16-bit key ranges whose union holds every key of the wanted
// bins (it may hold more: the exact bin tests follow).  miss(w) for a dword of two keys: a zero half
// means that key lies in some range (v_pk_max_u16 / v_pk_min_u16 clamp, xor, v_pk_min_u16).
using u16x2 = unsigned short __attribute__((ext_vector_type(2)));
struct KeyRanges {
    u16x2 lo[3], hi[3];
    __device__ __forceinline__ uint32_t miss(uint32_t w) const {
        const u16x2 v = __builtin_bit_cast(u16x2, w);
        u16x2 m;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const u16x2 c = __builtin_elementwise_min(__builtin_elementwise_max(v, lo[r]), hi[r]);
            const u16x2 x = __builtin_bit_cast(u16x2, __builtin_bit_cast(uint32_t, c) ^ w);
            m = r == 0 ? x : __builtin_elementwise_min(m, x);
        }
        return __builtin_bit_cast(uint32_t, m);
    }
};
constexpr int kGatherLoads = 4;

// Ranges for the median bin (and pb, the highest non-empty bin below it: the bins between are empty) and
// the MAD candidate bins [A, B] minus the class-0 run [C, D] (two bands).  An empty range repeats another
// one; 0xFFFF (an invisible slot, in bin 4095) is never inside a range.
__device__ __forceinline__ KeyRanges gather_ranges(bool med_fast, uint32_t pb, uint32_t mbin, bool mad_fast,
                                                   uint32_t A, uint32_t B, uint32_t C, uint32_t D) {
    uint32_t lo[3], hi[3];
    bool ok[3];
    ok[0] = med_fast;
    lo[0] = 16u * (pb < mbin ? pb : mbin);
    hi[0] = 16u * mbin + 15u;
    if (C <= D) {
        ok[1] = mad_fast && A < C; lo[1] = 16u * A; hi[1] = 16u * C - 1u;
        ok[2] = mad_fast && D < B; lo[2] = 16u * (D + 1u); hi[2] = 16u * B + 15u;
    } else {
        ok[1] = ok[2] = mad_fast; lo[1] = lo[2] = 16u * A; hi[1] = hi[2] = 16u * B + 15u;
    }
    const int any = ok[0] ? 0 : (ok[1] ? 1 : 2);
    KeyRanges R;
    for (int r = 0; r < 3; ++r) {
        const int t = ok[r] ? r : any;
        const unsigned short l = (unsigned short)lo[t], h = (unsigned short)(hi[t] > 0xFFFEu ? 0xFFFEu : hi[t]);
        R.lo[r] = u16x2{l, l};
        R.hi[r] = u16x2{h, h};
    }
    return R;
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
    uint32_t incl = wave_incl_scan(local);
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
    base = lane_read(base, leader);
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
__device__ __forceinline__ double radix_in_bin(SelShared& sh, const SlotSrc& res, int Ms, uint32_t bin, uint32_t k,
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
        sweep_res(res, Ms, [&](double r) {
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
__device__ __forceinline__ double lower_neighbour_sweep(SelShared& sh, const SlotSrc& res, int Ms, uint32_t k, double hi,
                                        double med) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t less = 0;
    double mx = -__builtin_inf();
    sweep_res(res, Ms, [&](double r) {
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
// src/algorithm.cpp:845-851; mid == 0 reads vec[mid]); Ms = slots swept.  sh.hist holds the value-bin
// histogram.
template <bool kMad>
__device__ __forceinline__ double block_median(SelShared& sh, const SlotSrc& res, int M, int Ms, uint32_t n, double med) {
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
        sweep_res(res, Ms, [&](double r) {
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
        hi = radix_in_bin<kMad>(sh, res, Ms, bin, kk, med);
        if (want_lo) lo = lower_neighbour_sweep<kMad>(sh, res, Ms, mid, hi, med);
    }
    return want_lo ? (lo + hi) / 2.0 : hi;
}

}  // namespace

#if defined(SVO_STAMPS)
// diagnostic build only (make stamps): per (pair, level) cycle stamps of K2's phases
__device__ uint64_t g_stamps[4096 * 16];
#define K2_STAMP(i, v)                                                                      \
    do {                                                                                    \
        if (tid == 0 && (a.pair_base + pair) * 5 + level < 4096)                                \
            g_stamps[((a.pair_base + pair) * 5 + level) * 16 + (i)] = (v);                      \
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
// element) take the exact path over every visible slot's recomputed residual.
__global__ void __launch_bounds__(kSelThreads, 4) align_scale_kernel(AlignArgs a, int level) {
    __shared__ SelShared sh;
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    PairState& S = a.state[pair];
    if (!S.active) return;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf, M = nf * a.area, M8 = slot_stride(nf) * a.area;  // M: reference length
    const uint16_t* __restrict__ keys = a.keys + (int64_t)pair * a.key_stride;
    SlotSrc res;
    res.keys = keys;
    res.scratch = a.scratch + (int64_t)pair * a.key_stride;
    res.px = a.px + (int64_t)pair * a.max_f * 2;
    res.cproj = a.cproj + (int64_t)pair * a.max_f * 2;
    res.rplane = P.ref_pyr + a.geom.off[level];
    res.kplane = P.kf_pyr + a.geom.off[level];
    res.cplane = P.cur_pyr + a.geom.off[level];
    res.W = a.geom.w[level];
    res.fstride = slot_stride(nf);
    res.n_ref = P.n_ref;
    res.half = a.half;
    res.side = 2 * a.half + 1;
    res.scale = ldexp(1.0, -level);
    const uint8_t* __restrict__ fvis = a.fvis + (int64_t)pair * a.max_f;
    K2_STAMP(0, clock64());
    K2_STAMP(14, __builtin_amdgcn_s_memrealtime());  // 100 MHz, chip-wide: workgroup start / end spread
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
        if (tid == 0) { sh.sel_k = mid; sh.cand_n = 0; sh.mcand_n = 0; sh.pcand_n = 0; }
        __syncthreads();
        K2_STAMP(2, clock64());
        find_bin(sh, sh.hist, kBins);
        const uint32_t bin = sh.sel_bin, kk = sh.sel_k, cnt = sh.sel_cnt;
        // even length with rank n/2 first in its bin: the lower neighbour is the largest value of the
        // highest non-empty bin below (gathered too)
        const bool need_prev = want_lo && kk == 0;
        uint32_t pbin = kBins;
        if (need_prev) {
            uint32_t jm = 0;
            for (int j = tid; j < (int)bin; j += kSelThreads)
                if (sh.hist[j]) jm = max(jm, (uint32_t)j + 1u);
            jm = wave_max_u(jm);
            if (lane == 0) sh.rngw[wave][0] = jm;
            __syncthreads();
            jm = 0;
            for (int w = 0; w < kSelWaves; ++w) jm = max(jm, sh.rngw[w][0]);
            pbin = jm - 1u;  // mid > 0 values lie below the bin
        }
        const bool med_fast = cnt <= (uint32_t)kCandCap && (!need_prev || sh.hist[pbin] <= (uint32_t)kPrevCap);
        bool mat = false;  // scratch row materialized (block-uniform)
        double mlo, mhi;
        if (med_fast) {
            const double eps = 1e-9;
            // need_prev: med = (largest value of bin pbin + smallest of bin) / 2 may lie below the bin,
            // down to the midpoint of the two bins' lower edges
            const uint32_t lob = need_prev ? pbin : bin;
            mlo = lob == 0 ? -__builtin_inf() : ((double)lob + (double)bin) / (2.0 * kBinScale) - kBinOffset - eps;
            mhi = bin == kBins - 1 ? __builtin_inf() : (double)(bin + 1) / kBinScale - kBinOffset + eps;
        } else {
            materialize(res, M8);
            mat = true;
            med = block_median<false>(sh, res, M, M8, n, 0.0);
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
#if defined(SVO_K2_DUP)  // diagnostic: a second histogram-style sweep of the keys, timed on its own
        sweep_keys(keys, M8, [&](int, uint32_t q) { atomicAdd(&sh.hhi[q >> 4], 1u); });
        __syncthreads();
        K2_STAMP(13, clock64());
#endif
        // ---- one sweep: median candidates (bin b) and MAD candidates (candidate bins)
        if (med_fast || mad_fast) {
            const uint32_t mbin = med_fast ? bin : kBins;  // kBins never matches
            const uint32_t pb = med_fast ? pbin : kBins;
            const uint32_t cA = mad_fast ? rA : kBins;
            // A branch-free packed filter passes each 16-B group of 8 keys through three key ranges that
            // cover every wanted bin (gather_ranges); only the lanes' hits (a few per group) run the exact
            // bin tests and the LDS appends.  (Testing each key against the three lists directly costs
            // ~60 instructions a key: the sweep was issue bound at ~4x a plain histogram sweep.)
            const KeyRanges R = gather_ranges(med_fast, pb, mbin, mad_fast, rA, rB, rC, rD);
            for (int base = 8 * tid; base < M8; base += 8 * kSelThreads * kGatherLoads) {
                uint4 v[kGatherLoads];
#pragma unroll
                for (int u = 0; u < kGatherLoads; ++u) {
                    const int s = base + u * 8 * kSelThreads;
                    v[u] = s < M8 ? *reinterpret_cast<const uint4*>(keys + s) : make_uint4(~0u, ~0u, ~0u, ~0u);
                }
#pragma unroll
                for (int u = 0; u < kGatherLoads; ++u) {
                    const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                    uint32_t hits = 0;
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const uint32_t m = R.miss(w[d]);
                        hits |= ((m & 0xFFFFu) == 0 ? 1u : 0u) << (2 * d);
                        hits |= ((m >> 16) == 0 ? 1u : 0u) << (2 * d + 1);
                    }
                    const uint32_t s0 = (uint32_t)(base + u * 8 * kSelThreads);
                    while (hits) {
                        const int q = __builtin_ctz(hits);
                        hits &= hits - 1u;
                        const uint32_t wq = q < 4 ? (q < 2 ? w[0] : w[1]) : (q < 6 ? w[2] : w[3]);
                        const uint32_t k = (wq >> (16 * (q & 1))) & 0xFFFFu, j = k >> 4, sl = s0 + (uint32_t)q;
                        if (j == mbin) sh.cand[atomicAdd(&sh.cand_n, 1u)] = __longlong_as_double((long long)sl);
                        if (j == pb) sh.pcand[atomicAdd(&sh.pcand_n, 1u)] = sl;
                        if (j >= cA && j <= rB && !(j >= rC && j <= rD)) sh.mcand[atomicAdd(&sh.mcand_n, 1u)] = sl;
                    }
                }
            }
            __syncthreads();
        }
        K2_STAMP(5, clock64());
        if (med_fast) {
            for (uint32_t i = tid; i < cnt; i += kSelThreads) sh.cand[i] = res.r((uint32_t)__double_as_longlong(sh.cand[i]));
            double lo_prev = -__builtin_inf();
            if (need_prev) {
                const uint32_t pc = sh.hist[pbin];
                for (uint32_t i = tid; i < pc; i += kSelThreads) lo_prev = fmax(lo_prev, res.r(sh.pcand[i]));
                lo_prev = wave_max(lo_prev);
                if (lane == 0) sh.red2[wave] = lo_prev;
            }
            __syncthreads();
            if (need_prev)
                for (int w = 0; w < kSelWaves; ++w) lo_prev = fmax(lo_prev, sh.red2[w]);
            cand_select(sh, cnt, kk, want_lo && !need_prev);
            med = want_lo ? ((need_prev ? lo_prev : sh.sel_lo) + sh.sel_hi) / 2.0 : sh.sel_hi;
            K2_STAMP(10, cnt);
            __syncthreads();
        }
        K2_STAMP(6, clock64());
        if (mad_fast) {
            for (uint32_t i = tid; i < ncand; i += kSelThreads) sh.cand[i] = fabs(res.r(sh.mcand[i]) - med);
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
            if (!mat) materialize(res, M8);
            for (int i = tid; i < kBins; i += kSelThreads) sh.hist[i] = 0;
            __syncthreads();
            sweep_res(res, M8, [&](double r) { atomicAdd(&sh.hist[sel_bin<true>(fabs(r - med))], 1u); });
            __syncthreads();
            mad = block_median<true>(sh, res, M, M8, n, med);
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
        S.scale_kernel = SVO_SCALE_K2;
    }
    K2_STAMP(15, __builtin_amdgcn_s_memrealtime());
}
// ------------------------------------------------------------------ K3: weights, normal equations, LM step
namespace {
// image_jac (src/image_alignment.cpp:194-248) with one reciprocal of z instead of ten divisions: K3's
// sums are compared within tolerance, and the ulp-level differences are far inside it
__device__ __forceinline__ void image_jac_rcp(V3 p, double fx, double fy, double a[6], double b[6]) {
    const double iz = 1.0 / p.z, x = p.x * iz, y = p.y * iz;  // normalised coordinates
    const double fxi = fx * iz, fyi = fy * iz;
    a[0] = fxi; a[1] = 0.0; a[2] = -fxi * x; a[3] = -fx * x * y; a[4] = fx * x * x + fx; a[5] = -fx * y;
    b[0] = 0.0; b[1] = fyi; b[2] = -fyi * y; b[3] = -fy * y * y - fy; b[4] = fy * x * y; b[5] = fy * x;
}

struct SolveShared {
    double tot[28];
    double A[36];
    double tmp[6];
    int32_t perm[6];
};

// Per-pair LM step of one level (src/optimizer.cpp:279-366) from the chunk partials, summed in a fixed
// order: lanes 0..27 one term each, then lane 0 solves.  Called by the one workgroup (one wave) of the
// pair that published last.
__device__ void pair_step(const AlignArgs& a, PairState& S, int level, int pair, SolveShared& sh) {
    const int lane = threadIdx.x;
    if (lane < 28) {
        const double* p = a.partials + (int64_t)pair * a.chunks * 28 + lane;
        double s = 0.0;
        for (int c = 0; c < a.chunks; ++c) s += p[c * 28];
        sh.tot[lane] = s;
    }
    __syncthreads();
    if (lane != 0) return;
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
    const double lambda = 1e-2 * mx;  // Nielsen initial damping, first (only) iteration (:294-302)
    for (int r = 0; r < 6; ++r) sh.A[r * 7] += lambda;
    svo_level_trace& t = a.traces[(int64_t)pair * (a.max_level + 1) + level];
    for (int r = 0; r < 36; ++r) t.H[r] = sh.A[r];
    ldlt_solve_ws(6, sh.A, g, dx, sh.perm, sh.tmp);
    double m[6];
    for (int r = 0; r < 6; ++r) m[r] = -dx[r];
    const SE3 np = se3_compose(se3_load(S.pose), se3_exp(m));  // pose * exp(-dx) (src/image_alignment.cpp:379)
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
    const double e = sqrt(chi / (double)S.n);  // RMSE before the update (:366)
    t.level = level; t.n_ref_vis = (int32_t)S.n_ref_vis; t.n_vis = (int32_t)S.n; t.status = st;
    t.median = S.med; t.mad = S.mad; t.sigma = S.sigma; t.chi2 = chi; t.lambda = lambda; t.err = e;
    t.scale_kernel = S.scale_kernel;
    for (int r = 0; r < 6; ++r) { t.g[r] = g[r]; t.dx[r] = dx[r]; }
    S.err = e;
    S.status = st;
    if (level == a.min_level) {
        for (int i = 0; i < 7; ++i) a.pose_out[7 * pair + i] = S.pose[i];
        a.err_out[pair] = S.err;
        a.status_out[pair] = S.status;
    }
    a.arrive[pair] = 0u;  // next level's K3 (after the kernel boundary) counts from 0 again
}
}  // namespace

// One lane per feature slot, 64-lane workgroups (same map as K1).  dx / dy at (u + kx, v + ky) of the
// ref level are the reference's central differences of bilinear samples (:180-183) formed with the
// feature's fractional weights shared by all samples (fx = u - floor(u)): the blends hv(R, c) of every
// window row R are computed once, and D(R) = hv(R, c+1) - hv(R, c-1), P(R) = hv(R, c) give
//   dx = (gy D(R0) + fy D(R0+1)) / 2,   dy = (gy (P(R0+1) - P(R0-1)) + fy (P(R0+2) - P(R0))) / 2
// for the pixel's cell (R0, c) (equal to the per-sample formula up to rounding); pixel row ky (R0 = ky + 1)
// is emitted once row R0 + 2 has been blended.  The Tukey weight uses
// r^2 / c^2 as r^2 * (1 / c^2) (rounding only); H, g and chi2 match the reference within the tolerances of
// tests/test_gpu_parity.py.
template <int kHalf, bool kWin>  // kWin: a window level (AlignArgs::win_levels)
__global__ void __launch_bounds__(kLaneFeats, kHalf <= 2 ? 4 : 3) align_weights_kernel(AlignArgs a, int level) {
    using G = Win<kHalf>;
    constexpr int h = G::h, side = G::side, WB = G::WB, NW = G::WW;
    // the wave partials and the LM step's workspace share their LDS (the step starts after the last read of the
    // partials, two barriers later): ~0.9 KB per workgroup, so that up to three K3 workgroups fit beside a K2V
    // workgroup whose waves 1-7 have ended (K2V leaves 3.4 KB of the CU's LDS unallocated)
    __shared__ union {
        SolveShared ssh;
        double part[kLaneWaves][28];
    } lds;
    SolveShared& ssh = lds.ssh;
    double (&part)[kLaneWaves][28] = lds.part;
    __shared__ uint32_t last_flag;
    SVO_TL_SCOPE(k13, kTlK3, level, a.pair_base);
    int pair, chunk;
    xcd_pair_chunk(a.chunks, pair, chunk);
    if (pair >= a.n_pairs) return;
    PairState& S = a.state[pair];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (!S.active) {  // nothing to align: the outputs are the initial state (init_pair)
        if (level == a.min_level && chunk == 0 && tid == 0) {
            for (int i = 0; i < 7; ++i) a.pose_out[7 * pair + i] = S.pose[i];
            a.err_out[pair] = S.err;
            a.status_out[pair] = S.status;
        }
        return;
    }
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf;
    const int f = chunk * kLaneFeats + tid;
    const int W = a.geom.w[level];
    const int64_t loff = a.geom.off[level];
    const double scale = ldexp(1.0, -level);  // exact, no division
    const double c = S.c, inv_c2 = 1.0 / (c * c);
    double acc[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) acc[t] = 0.0;
    const int64_t gf = (int64_t)pair * a.max_f + (f < nf ? f : 0);
    const uint8_t fvis = f < nf ? a.fvis[gf] : 0;
    if (fvis == 3) {
        const double pu = a.px[2 * gf], pv = a.px[2 * gf + 1];
        const V3 pw{a.xw[3 * gf], a.xw[3 * gf + 1], a.xw[3 * gf + 2]};
        const double2 cp = reinterpret_cast<const double2*>(a.cproj)[gf];  // projection into cur (K1)
        const double ur = pu * scale, vr = pv * scale, fur = floor(ur), fvr = floor(vr);
        const double fx = ur - fur, gx = 1.0 - fx, fy = vr - fvr, gy = 1.0 - fy;
        const double fcu = floor(cp.x), fcv = floor(cp.y);
        const double cfx = cp.x - fcu, cgx = 1.0 - cfx, cfy = cp.y - fcv, cgy = 1.0 - cfy;
        const int ru = (int)fur, rv = (int)fvr, qu = (int)fcu, qv = (int)fcv;
        const uint8_t* const plane = (f < P.n_ref ? P.ref_pyr : P.kf_pyr) + loff;
        const uint8_t* const cplane = P.cur_pyr + loff;
        uint32_t row[WB][NW], crow[G::RB][G::RW];
        if constexpr (kWin) {  // the windows K1 wrote (one contiguous run per row and wave)
            const int fstride = slot_stride(nf);
            const __amdgpu_buffer_rsrc_t ws = slot_rsrc(a.win + (int64_t)pair * a.win_stride, a.win_stride * 4);
            const uint32_t fo = (uint32_t)f, cbase = (uint32_t)(WB * NW * fstride * 4);
#pragma unroll
            for (int R = 0; R < WB; ++R) win_load<NW>(ws, fo * (4 * NW), (uint32_t)(R * fstride * 4 * NW), row[R]);
#pragma unroll
            for (int r = 0; r < G::RB; ++r)
                win_load<G::RW>(ws, fo * (4 * G::RW), cbase + (uint32_t)(r * fstride * 4 * G::RW), crow[r]);
        } else {
#pragma unroll
            for (int R = 0; R < WB; ++R) load_row<G::WD>(plane, (uint32_t)((rv - h - 1 + R) * W + (ru - h - 1)), row[R]);
#pragma unroll
            for (int r = 0; r < G::RB; ++r) load_row<G::RD>(cplane, (uint32_t)((qv - h + r) * W + (qu - h)), crow[r]);
        }
        double sxx = 0.0, sxy = 0.0, syy = 0.0, sxr = 0.0, syr = 0.0, chi = 0.0;
        // rolling row state: P(R-2), P(R-1) at the pixel columns, E(R-1) = P(R) - P(R-2), D(R-2), D(R-1)
        double P2[side], P1[side], E1[side], D2[side], D1[side];
        double cprev[side];  // cur row blends of patch row ky (window row ky)
        const double hgy = 0.5 * gy, hfy = 0.5 * fy;  // the 1/2 of the central differences, folded
#pragma unroll
        for (int kx = 0; kx < side; ++kx) cprev[kx] = fma(cfx, wbyte(crow[0], kx + 1), cgx * wbyte(crow[0], kx));
#pragma unroll
        for (int R = 0; R < WB; ++R) {
            double hv[2 * h + 3];
#pragma unroll
            for (int cc = 0; cc < 2 * h + 3; ++cc) hv[cc] = fma(fx, wbyte(row[R], cc + 1), gx * wbyte(row[R], cc));
            if (R >= 3) {  // pixel row ky: cell row R0 = ky + 1 = R - 2
                const int ky = R - 3;
#pragma unroll
                for (int kx = 0; kx < side; ++kx) {
                    const double P0 = hv[kx + 1];     // window column of cell floor(u) + kx - h
                    const double E0 = P0 - P2[kx];    // E(R0 + 1); E1 = E(R0)
                    const double ccur = fma(cfx, wbyte(crow[ky + 1], kx + 1), cgx * wbyte(crow[ky + 1], kx));
                    const double I = fma(cfy, ccur, cgy * cprev[kx]);
                    cprev[kx] = ccur;
                    const double T = fma(fy, P1[kx], gy * P2[kx]);
                    const double r = I - T;  // the residual of K1 up to rounding (shared weights)
                    const double dx = fma(hfy, D1[kx], hgy * D2[kx]);
                    const double dy = fma(hfy, E0, hgy * E1[kx]);
                    const double r2 = r * r;
                    // Tukey (src/optimizer.cpp:502-511): (1 - r^2/c^2)^2 for |r| <= c, else 0, as a clamp
                    // of the base at 0 (the two forms differ only at |r| = c, by a rounding-sized weight)
                    const double tt = fmax(fma(-r2, inv_c2, 1.0), 0.0);
                    const double w = tt * tt;
                    const double wdx = w * dx, wdy = w * dy;
                    sxx = fma(wdx, dx, sxx);
                    sxy = fma(wdx, dy, sxy);
                    syy = fma(wdy, dy, syy);
                    sxr = fma(wdx, r, sxr);
                    syr = fma(wdy, r, syr);
                    chi = fma(r2, w, chi);
                }
            }
#pragma unroll
            for (int kx = 0; kx < side; ++kx) {
                const double P0 = hv[kx + 1];
                if (R >= 2) E1[kx] = P0 - P2[kx];
                P2[kx] = P1[kx];
                P1[kx] = P0;
                D2[kx] = D1[kx];
                D1[kx] = hv[kx + 2] - hv[kx];
            }
        }
        // J row = dx * a + dy * b with the image Jacobian rows a, b at the WORLD point (:163, :194-248;
        // a[1] = b[0] = 0).  Per feature sum_px w J J^T = a u^T + b v^T with u = Sxx a + Sxy b,
        // v = Sxy a + Syy b: the 21 lower H terms (row-major lower triangle), the 6 g terms and chi2
        double ja[6], jb[6];
        image_jac_rcp(pw, a.fx * scale, a.fy * scale, ja, jb);
        double u[6], v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            u[i] = i == 0 ? sxx * ja[0] : (i == 1 ? sxy * jb[1] : fma(sxx, ja[i], sxy * jb[i]));
            v[i] = i == 0 ? sxy * ja[0] : (i == 1 ? syy * jb[1] : fma(sxy, ja[i], syy * jb[i]));
        }
        int t = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j)
                acc[t++] = i == 0 ? ja[0] * u[j] : (i == 1 ? jb[1] * v[j] : fma(ja[i], u[j], jb[i] * v[j]));
#pragma unroll
        for (int i = 0; i < 6; ++i)
            acc[21 + i] = i == 0 ? ja[0] * sxr : (i == 1 ? jb[1] * syr : fma(ja[i], sxr, jb[i] * syr));
        acc[27] = chi;
    }
    // halving exchange: after the steps of offsets 32..2 lane L holds term L >> 1 (half of it).  The
    // steps across 32 and 16 lanes are CDNA4 permlane swaps (two terms per swap pair, no selects)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        lane_swap<32>(acc[q], acc[q + 16]);
        acc[q] += acc[q + 16];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        lane_swap<16>(acc[q], acc[q + 8]);
        acc[q] += acc[q + 8];
    }
#pragma unroll
    for (int o = 8, n = 8; o >= 2; o >>= 1, n >>= 1) {
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
    // publish (MI355X_MICROARCH.md, inter-workgroup visibility): the partials are stored write-through
    // (agent-scope stores: sc1, they leave the XCD's L2) by wave 0, drained by its vmcnt(0), then one lane
    // adds to the pair's arrival counter; the workgroup whose add returns a.chunks - 1 is the last,
    // acquires (invalidates its CU's L1) and takes the LM step.  No per-workgroup L2 write-back.
    if (wave == 0) {
        if (lane < 28) {
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < kLaneWaves; ++w) t += part[w][lane];
            __hip_atomic_store(a.partials + ((int64_t)pair * a.chunks + chunk) * 28 + lane, t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
            last_flag = __hip_atomic_fetch_add(a.arrive + pair, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        (uint32_t)a.chunks - 1;
    }
    __syncthreads();
    if (!last_flag) return;
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    pair_step(a, S, level, pair, ssh);
}

// ------------------------------------------------------------------ launch
// marks (optional): an event recorded before every launch and after the last one, in launch order
// start, then per level K1 K2 K3 (1 + 3 * levels + 1 events)
template <int kHalf>
static void launch_all(const AlignArgs& a, hipStream_t s, hipEvent_t* marks) {
    int m = 0;
    auto mark = [&]() {
        if (marks) (void)hipEventRecord(marks[m++], s);
    };
    mark();  // (the pair init runs inside the first K1: the "init" interval is empty)
    const unsigned fgrid = (unsigned)((int64_t)((a.n_pairs + 7) / 8) * 8 * a.chunks);
    for (int level = a.max_level; level >= a.min_level; --level) {
        mark();
        const bool win = (a.win_levels >> level) & 1u;
        if (a.median_mode == 1) {
            if (win) hipLaunchKernelGGL((align_residual_kernel<kHalf, true, true>), dim3(fgrid), dim3(kLaneFeats), 0, s, a, level);
            else hipLaunchKernelGGL((align_residual_kernel<kHalf, false, true>), dim3(fgrid), dim3(kLaneFeats), 0, s, a, level);
            mark();
            launch_scale_ref(a, level, s);
        } else {
            if (win) hipLaunchKernelGGL((align_residual_kernel<kHalf, true, false>), dim3(fgrid), dim3(kLaneFeats), 0, s, a, level);
            else hipLaunchKernelGGL((align_residual_kernel<kHalf, false, false>), dim3(fgrid), dim3(kLaneFeats), 0, s, a, level);
            mark();
            hipLaunchKernelGGL(align_scale_kernel, dim3(a.n_pairs), dim3(kSelThreads), 0, s, a, level);
        }
        mark();
        if (win) hipLaunchKernelGGL((align_weights_kernel<kHalf, true>), dim3(fgrid), dim3(kLaneFeats), 0, s, a, level);
        else hipLaunchKernelGGL((align_weights_kernel<kHalf, false>), dim3(fgrid), dim3(kLaneFeats), 0, s, a, level);
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
