// svo_wave.h — wave64 reductions / scans and the residual keys shared by the alignment kernels
// (align.hip, align_ref.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace svo {

// Wave reductions and scans with DPP row operations (GFX9 encodings) instead of shfl (ds_bpermute, an
// LDS round trip per step): quad_perm / row_half_mirror / row_mirror reduce inside each 16-lane row,
// readlane combines the four rows.  DPP reads every lane's register regardless of EXEC, so all 64 lanes
// must be active: every caller is block-uniform code.
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
template <int kCtrl>
__device__ __forceinline__ double dpp_mov(double v) {
    const uint2 u = __builtin_bit_cast(uint2, v);
    return __builtin_bit_cast(double, make_uint2(dpp_mov<kCtrl>(u.x), dpp_mov<kCtrl>(u.y)));
}
__device__ __forceinline__ uint32_t lane_read(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
// v_writelane_b32 (no clang builtin on this toolchain: the LLVM intrinsic by name): lane l of `old` := v
__device__ int svo_writelane_i32(int v, int l, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t lane_write(uint32_t old, uint32_t v, uint32_t l) {
    return (uint32_t)svo_writelane_i32((int)v, (int)l, (int)old);
}
__device__ __forceinline__ double lane_read(double v, int l) {
    const uint2 u = __builtin_bit_cast(uint2, v);
    return __builtin_bit_cast(double, make_uint2(lane_read(u.x, l), lane_read(u.y, l)));
}
template <typename T, typename F>
__device__ __forceinline__ T wave_allreduce(T v, F op) {
    v = op(v, dpp_mov<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp_mov<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp_mov<0x141>(v));  // row_half_mirror
    v = op(v, dpp_mov<0x140>(v));  // row_mirror: every lane of a row holds the row's result
    return op(op(lane_read(v, 0), lane_read(v, 16)), op(lane_read(v, 32), lane_read(v, 48)));
}
__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v) {
    return wave_allreduce(v, [](uint32_t x, uint32_t y) { return x + y; });
}
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
    return wave_allreduce(v, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
}
__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
    return wave_allreduce(v, [](uint32_t x, uint32_t y) { return x > y ? x : y; });
}
__device__ __forceinline__ double wave_max(double v) {
    return wave_allreduce(v, [](double x, double y) { return fmax(x, y); });
}
// inclusive prefix sum over the wave: row_shr 1..3 (bound_ctrl zero-fills across the row start), row_shr
// 4 / 8 into banks 1-3 / 2-3, then row_bcast 15 / 31 carry the row totals into rows 1, 3 / 2, 3
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    uint32_t s = v;
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xF, 0xF, true);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x114, 0xF, 0xE, true);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x118, 0xF, 0xC, true);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x142, 0xA, 0xF, false);
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x143, 0xC, 0xF, false);
    return s;
}
// lanes below this one with their bit set in m
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// 32-bit residual key of the reference-semantics robust scale (K1 in median_mode SVO_MEDIAN_REFERENCE,
// K2R): with g = floor(r * 2^22) + 2^30 (exact: r * 2^22 only rescales, |r| <= 255 keeps g in 31 bits),
//   key = g << 1 | (r * 2^22 != floor(r * 2^22))
// i.e. the residual on a 2^-22 grid plus a bit telling whether it lies ON the grid point.  key is
// monotone non-decreasing in r, so key_a < key_b proves r_a < r_b; equal keys with the bit clear are
// equal residuals (integer / dyadic ones: flat patches); only equal keys with the bit set need the exact
// residuals.  0xFFFFFFFF marks an invisible slot (the reference's DBL_MAX, above every visible key).
constexpr uint32_t kKeyInvisible = 0xFFFFFFFFu;
constexpr double kKeyGrid = 4194304.0;            // 2^22
constexpr double kKeyStep = 2.384185791015625e-07;  // 2^-22
constexpr int64_t kKeyBias = 1ll << 30;
__host__ __device__ __forceinline__ int64_t key_grid(double x) { return (int64_t)floor(x * kKeyGrid) + kKeyBias; }
__host__ __device__ __forceinline__ uint32_t res_key32(double r) {
    const double t = r * kKeyGrid, fl = floor(t);
    int64_t g = (int64_t)fl + kKeyBias;
    g = g < 0 ? 0 : (g > 0x7FFFFFFE ? 0x7FFFFFFE : g);  // never binds for |r| <= 255
    return ((uint32_t)g << 1) | (t != fl ? 1u : 0u);
}
// the grid point of a key (its residual when the low bit is clear; the open interval's lower end else)
__host__ __device__ __forceinline__ double key_r(uint32_t k) { return (double)((int64_t)(k >> 1) - kKeyBias) * kKeyStep; }

}  // namespace svo
