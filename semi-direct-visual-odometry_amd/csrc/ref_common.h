// ref_common.h — pieces of libstdc++'s introselect shared by the two device forms of the reference's robust
// scale: K2R (align_ref.hip, segments in LDS / global scratch) and K2V (align_refv.hip, the residual vector
// resident in registers).  Both restate std::nth_element as tests/cpp/introselect_model.cpp derives it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "svo_wave.h"

namespace svo {
namespace refsel {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr double kDblMax = 1.7976931348623157e308;

enum { kSrc = 0, kGlb = 1, kLds = 2 };  // where a segment lives

__device__ __forceinline__ int lg2(uint32_t n) { return 31 - __builtin_clz(n); }
__device__ __forceinline__ uint64_t low_mask(uint32_t b) { return b >= 64 ? ~0ull : ((1ull << b) - 1ull); }
__device__ __forceinline__ uint32_t popc(uint64_t m) { return (uint32_t)__popcll(m); }
// position of the j-th (0-based) set bit of m
__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t j) {
    uint32_t pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint32_t c = popc(m & ((1ull << w) - 1ull));
        if (j >= c) { j -= c; m >>= w; pos += (uint32_t)w; }
    }
    return pos;
}
// block-uniform values loaded or computed in vector registers, moved to scalar registers (control flow on
// them stays scalar)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni(uint64_t v) { return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v); }
__device__ __forceinline__ double uni(double v) { return __builtin_bit_cast(double, uni(__builtin_bit_cast(uint64_t, v))); }
__device__ __forceinline__ uint64_t lane_read64(uint64_t v, int l) {
    return ((uint64_t)lane_read((uint32_t)(v >> 32), l) << 32) | lane_read((uint32_t)v, l);
}

// libstdc++ __move_median_to_first(result, a, b, c): the chosen position and value
__device__ __forceinline__ void median3(double a, double b, double c, uint32_t A, uint32_t B, uint32_t C, uint32_t& ch,
                                        double& p) {
    if (a < b) {
        if (b < c) { ch = B; p = b; }
        else if (a < c) { ch = C; p = c; }
        else { ch = A; p = a; }
    } else if (a < c) { ch = A; p = a; }
    else if (b < c) { ch = C; p = c; }
    else { ch = B; p = b; }
}

// Ks of a Hoare round from the step that holds the crossing: t* is the first split point with
// G(t) >= Lc(t) (G = #GE before t, Lc = #LE from t on); the step starts at a split point where G < Lc, with
// carries gcar = G and lcar = Lc there, and masks ge / le.  Ks = max(G(t* - 1), Lc(t*)).
__device__ __forceinline__ uint32_t crossing_ks(uint32_t gcar, uint32_t lcar, uint64_t ge, uint64_t le) {
    uint32_t lo = 1, hi = 64;  // smallest bit split b with G(b) >= Lc(b) inside the step
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        const uint64_t lm = low_mask(mid);
        if (gcar + popc(ge & lm) >= lcar - popc(le & lm)) hi = mid;
        else lo = mid + 1;
    }
    const uint32_t g1 = gcar + popc(ge & low_mask(lo - 1));
    const uint32_t l2 = lcar - popc(le & low_mask(lo));
    return g1 > l2 ? g1 : l2;
}

// ---- heap select (depth limit), one lane: stl_heap.h __adjust_heap / __push_heap / __make_heap /
// __pop_heap and stl_algo.h __heap_select restated over a[i] = position first + i, then the swap of first and
// nth (tests/cpp/introselect_model.cpp checks the restatement).  Only adversarial inputs reach it.
__device__ __forceinline__ void heap_select_at(double* a, uint32_t len, uint32_t middle, uint32_t nth_rel) {
    auto push_heap = [&](uint32_t hole, uint32_t top, double value) {
        uint32_t parent = (hole - 1) / 2;
        while (hole > top && a[parent] < value) {
            a[hole] = a[parent];
            hole = parent;
            parent = (hole - 1) / 2;
        }
        a[hole] = value;
    };
    auto adjust_heap = [&](uint32_t hole, uint32_t n, double value) {
        const uint32_t top = hole;
        uint32_t second = hole;
        while (n >= 1 && second < (n - 1) / 2) {
            second = 2 * (second + 1);
            if (a[second] < a[second - 1]) second--;
            a[hole] = a[second];
            hole = second;
        }
        if ((n & 1u) == 0 && second == (n - 2) / 2) {
            second = 2 * (second + 1);
            a[hole] = a[second - 1];
            hole = second - 1;
        }
        push_heap(hole, top, value);
    };
    if (middle >= 2) {
        uint32_t parent = (middle - 2) / 2;
        while (true) {
            adjust_heap(parent, middle, a[parent]);
            if (parent == 0) break;
            parent--;
        }
    }
    for (uint32_t i = middle; i < len; ++i)
        if (a[i] < a[0]) {
            const double v = a[i];
            a[i] = a[0];
            adjust_heap(0, middle, v);
        }
    const double f0 = a[0], n0 = a[nth_rel];  // std::iter_swap(first, nth)
    a[0] = n0;
    a[nth_rel] = f0;
}
// the same as a free function of plain values (K2R: the selection state never needs an address); the
// segment lives in LDS (seg, from position base) or in global scratch (gseg, absolute positions)
__device__ __attribute__((noinline)) inline void heap_select_fn(double* seg, uint32_t base, double* gseg, int where,
                                                                uint32_t first, uint32_t len, uint32_t middle,
                                                                uint32_t nth_rel) {
    if (where == kLds) heap_select_at(seg + (first - base), len, middle, nth_rel);
    else heap_select_at(gseg + first, len, middle, nth_rel);
}

// std::__insertion_sort of the last <= 3 values of a segment: (vec[nth - 1], vec[nth]) where they lie inside
__device__ __forceinline__ void sort3(double (&v)[3], uint32_t n) {
    for (uint32_t i = 1; i < n; ++i) {
        const double x = v[i];
        uint32_t j = i;
        while (j > 0 && x < v[j - 1]) { v[j] = v[j - 1]; --j; }
        v[j] = x;
    }
}

}  // namespace refsel
}  // namespace svo
