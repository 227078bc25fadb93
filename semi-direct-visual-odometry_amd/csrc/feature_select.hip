// feature_select.hip — FeatureSelection (src/feature_selection.cpp:19-287) on gfx950 + its host half.
//
// gradientMagnitudeWithSSC (:27-89) is three steps: (1) every level-0 pixel whose gradient magnitude
// (the pyramid's own Simd::AbsGradientSaturatedSum plane, :250-266) exceeds the threshold becomes a
// keypoint, in row-major order (:38-50); (2) std::sort by response, descending (:53-54); (3) SSC's
// binary search over a covering radius (:166-248) and the per-cell bucketing (:60-75).
//   Step 1 is the pixel stream and runs on the device: an ordered stream compaction of the gradient
//   plane into 32-bit keys (response << 24 | y * W + x), two launches (per-segment counts, then
//   scan + write).  Steps 2-3 are order dependent: std::sort is not stable, so which of the many equal
//   responses (they are 8-bit) comes first is decided by libstdc++'s introsort, and SSC's greedy sweep
//   and the bucketing depend on that order.  They run on the host over the keys with the reference's
//   comparator; std::sort's permutation depends only on the comparison results, so sorting the keys
//   gives the reference's keypoint order exactly.
// gradientMagnitudeByValue (:91-143, bucketing branch) is fully parallel: one workgroup per grid cell
// takes the cell's first maximum in row-major order (strict >, as the reference's scan).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>
#include <thread>
#include <vector>

#include "svo_internal.h"

namespace svo {

namespace {

constexpr int kSegPx = 4096;  // pixels per compaction workgroup: 256 threads x 16 (one 16-B load each)

__device__ __forceinline__ int count16(const uint8_t* plane, int64_t p0, int64_t npx, int thr, uint8_t v[16]) {
    if (p0 + 16 <= npx) {
        const uint4 q = *reinterpret_cast<const uint4*>(plane + p0);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = (p0 + i < npx) ? plane[p0 + i] : 0;
    }
    int n = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) n += (int)v[i] > thr;
    return n;
}

// exclusive scan of one int per thread over a 256-thread workgroup; returns the prefix, *total the sum
__device__ __forceinline__ int block_scan256(int x, int* total) {
    __shared__ int wsum[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int before = 0;
    for (int i = 0; i < wave; ++i) before += wsum[i];
    *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    return before + inc - x;
}

__global__ void __launch_bounds__(256) fs_count_kernel(const uint8_t* plane, int64_t npx, int thr, int* seg_counts) {
    uint8_t v[16];
    const int64_t p0 = (int64_t)blockIdx.x * kSegPx + threadIdx.x * 16;
    int total;
    (void)block_scan256(count16(plane, p0, npx, thr, v), &total);
    if (threadIdx.x == 0) seg_counts[blockIdx.x] = total;
}

__global__ void __launch_bounds__(256) fs_write_kernel(const uint8_t* plane, int64_t npx, int width, int thr,
                                                       const int* seg_counts, uint32_t* keys, int* n_keys) {
    __shared__ int base_sh;
    // keys before this segment
    int b = 0;
    for (int i = threadIdx.x; i < (int)blockIdx.x; i += 256) b += seg_counts[i];
    int btot;
    (void)block_scan256(b, &btot);
    if (threadIdx.x == 0) base_sh = btot;
    __syncthreads();
    const int base = base_sh;
    uint8_t v[16];
    const int64_t p0 = (int64_t)blockIdx.x * kSegPx + threadIdx.x * 16;
    int seg_total;
    __syncthreads();  // block_scan256's LDS is reused
    int o = base + block_scan256(count16(plane, p0, npx, thr, v), &seg_total);
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((int)v[i] > thr) keys[o++] = ((uint32_t)v[i] << 24) | (uint32_t)(p0 + i);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_keys = base + seg_total;
    (void)width;
}

// one workgroup per cell (blockIdx.x = col, blockIdx.y = row): first maximum in row-major order;
// cell_px = value << 24 | pixel index, or ~0 for none
__global__ void __launch_bounds__(256) fs_cell_max_kernel(const uint8_t* plane, int width, int height, int cell,
                                                          const uint8_t* occupancy, int thr, uint32_t* cell_px) {
    const int c = blockIdx.x, r = blockIdx.y, cols = gridDim.x;
    const int cidx = r * cols + c;
    if (occupancy[cidx]) {
        if (threadIdx.x == 0) cell_px[cidx] = 0xFFFFFFFFu;
        return;
    }
    const int mc = (c + 1) * cell < width ? cell : width - c * cell;
    const int mr = (r + 1) * cell < height ? cell : height - r * cell;
    // key = value << 20 | (0xFFFFF - position in the cell's row-major scan): the max key is the first max
    uint32_t best = 0;
    const int area = mc > 0 && mr > 0 ? mc * mr : 0;
    for (int k = threadIdx.x; k < area; k += 256) {
        const int i = k / mc, j = k - i * mc;
        const uint32_t val = plane[(int64_t)(r * cell + i) * width + c * cell + j];
        const uint32_t key = (val << 20) | (uint32_t)(0xFFFFF - k);
        best = key > best ? key : best;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(best, d, 64);
        best = o > best ? o : best;
    }
    __shared__ uint32_t wbest[4];
    if ((threadIdx.x & 63) == 0) wbest[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        best = max(max(wbest[0], wbest[1]), max(wbest[2], wbest[3]));
        const int val = (int)(best >> 20);
        // the reference's max starts at 0 with a strict >, so an all-zero cell keeps (0, 0): never above thr
        if (val > thr) {
            const int k = 0xFFFFF - (int)(best & 0xFFFFF);
            const int i = k / mc, j = k - i * mc;
            cell_px[cidx] = ((uint32_t)val << 24) | (uint32_t)((r * cell + i) * width + c * cell + j);
        } else {
            cell_px[cidx] = 0xFFFFFFFFu;
        }
    }
}

}  // namespace

int feature_detect_segments(int64_t npx) { return (int)((npx + kSegPx - 1) / kSegPx); }

void launch_feature_detect(const uint8_t* plane, int width, int height, int thr, int* seg_counts, uint32_t* keys,
                           int* n_keys, hipStream_t s) {
    const int64_t npx = (int64_t)width * height;
    const int nseg = feature_detect_segments(npx);
    hipLaunchKernelGGL(fs_count_kernel, dim3(nseg), dim3(256), 0, s, plane, npx, thr, seg_counts);
    hipLaunchKernelGGL(fs_write_kernel, dim3(nseg), dim3(256), 0, s, plane, npx, width, thr, seg_counts, keys, n_keys);
}

void launch_feature_cell_max(const uint8_t* plane, int width, int height, int cell, int grid_rows, int grid_cols,
                             const uint8_t* occupancy, int thr, uint32_t* cell_px, hipStream_t s) {
    hipLaunchKernelGGL(fs_cell_max_kernel, dim3(grid_cols, grid_rows), dim3(256), 0, s, plane, width, height, cell,
                       occupancy, thr, cell_px);
}

// ---------------------------------------------------------------------------------------------- host
// std::sort with the reference's comparator (lhs.response > rhs.response, :53-54) over the keys, giving
// libstdc++'s exact permutation faster.  libstdc++'s std::sort is __introsort_loop (Hoare partitions
// around a median-of-three moved to the front, recursion on the right part, depth limit 2 floor(log2 n),
// heap sort past it, segments of <= 16 left alone) followed by __final_insertion_sort.  Insertion sort is
// stable, so that last pass yields the stable order by key of the partitioned array: one counting sort
// over the 8-bit responses here.  The partition phase is restated step for step; segments at the same
// depth are disjoint, so large ones run on their own threads (up to 7) without changing any step.
namespace {
inline bool before(uint32_t a, uint32_t b) { return (a >> 24) > (b >> 24); }

inline void median_to_first(uint32_t* r, uint32_t* a, uint32_t* b, uint32_t* c) {
    if (before(*a, *b)) {
        if (before(*b, *c)) std::swap(*r, *b);
        else if (before(*a, *c)) std::swap(*r, *c);
        else std::swap(*r, *a);
    } else if (before(*a, *c)) {
        std::swap(*r, *a);
    } else if (before(*b, *c)) {
        std::swap(*r, *c);
    } else {
        std::swap(*r, *b);
    }
}

inline uint32_t* partition_pivot(uint32_t* first, uint32_t* last) {
    median_to_first(first, first + 1, first + (last - first) / 2, last - 1);
    uint32_t* lo = first + 1;
    uint32_t* hi = last;
    const uint32_t pv = *first;
    for (;;) {
        while (before(*lo, pv)) ++lo;
        --hi;
        while (before(pv, *hi)) --hi;
        if (!(lo < hi)) return lo;
        std::swap(*lo, *hi);
        ++lo;
    }
}

// segments above kSpawnMin take a thread of their own while the budget lasts
constexpr ptrdiff_t kSpawnMin = 8192;

void introsort_loop(uint32_t* first, uint32_t* last, int depth, std::atomic<int>* budget) {
    std::vector<std::thread> sides;
    while (last - first > 16) {
        if (depth == 0) {
            std::partial_sort(first, last, last, before);  // libstdc++ __partial_sort(first, last, last)
            break;
        }
        --depth;
        uint32_t* cut = partition_pivot(first, last);
        if (budget && last - cut > kSpawnMin && budget->fetch_sub(1) > 0) {
            sides.emplace_back(introsort_loop, cut, last, depth, budget);
        } else {
            if (budget && last - cut > kSpawnMin) budget->fetch_add(1);
            introsort_loop(cut, last, depth, budget);
        }
        last = cut;
    }
    for (std::thread& t : sides) t.join();
}
}  // namespace

void feature_sort_keys(uint32_t* keys, int32_t n) {
    if (n < 2) return;
    int lg = 0;
    while ((2 << lg) <= n) ++lg;  // floor(log2 n)
    std::atomic<int> budget(7);  // extra threads
    introsort_loop(keys, keys + n, 2 * lg, n >= 32768 ? &budget : nullptr);
    // __final_insertion_sort == stable order by response (descending)
    uint32_t count[257] = {0};
    for (int32_t i = 0; i < n; ++i) ++count[256 - (keys[i] >> 24)];
    for (int v = 1; v < 257; ++v) count[v] += count[v - 1];
    std::vector<uint32_t> tmp(keys, keys + n);
    for (int32_t i = 0; i < n; ++i) keys[count[255 - (tmp[i] >> 24)]++] = tmp[i];
}

// SSC (src/feature_selection.cpp:166-248) over keypoints given by their (x, y) in sorted order.  Same
// arithmetic as the reference (int / long long / double / float exactly where it has them); the covered
// grid is one flat byte plane instead of vector<vector<bool>>.  Width 0 (fewer than Kmin keypoints: the
// reference divides by zero there) ends the search with the previous result, like its low > high exit.
void feature_ssc(const int32_t* xs, const int32_t* ys, int32_t n, int32_t num_ret, float tolerance, int32_t cols,
                 int32_t rows, std::vector<int32_t>& out) {
    const int32_t e1 = rows + cols + 2 * num_ret;
    const long long e2 = 4LL * cols + 4LL * num_ret + 4LL * rows * num_ret + (long long)rows * rows +
                         (long long)cols * cols - 2LL * rows * cols + 4LL * rows * cols * num_ret;
    const double e3 = std::sqrt((double)e2), e4 = 2 * (num_ret - 1);
    const double s1 = -std::round((e1 + e3) / e4), s2 = -std::round((e1 - e3) / e4);
    int high = s1 > s2 ? (int)s1 : (int)s2;
    int low = (int)std::sqrt((double)n / num_ret);
    const float K = (float)num_ret;
    const uint32_t kmin = (uint32_t)std::round(K - K * tolerance), kmax = (uint32_t)std::round(K + K * tolerance);
    std::vector<int32_t> cur, prev;
    std::vector<uint8_t> covered;
    int prev_w = -1;
    for (;;) {
        const int wdt = low + (high - low) / 2;
        if (wdt == prev_w || low > high || wdt <= 0) {
            out.swap(prev);
            return;
        }
        const double c = wdt / 2.0;
        const int32_t ncc = (int32_t)(cols / c), ncr = (int32_t)(rows / c);
        const int32_t gc = ncc + 1;
        const int32_t reach = (int32_t)(wdt / c);
        covered.assign((size_t)(ncr + 1) * gc, 0);
        cur.clear();
        for (int32_t i = 0; i < n; ++i) {
            const int32_t row = (int32_t)((double)(float)ys[i] / c), col = (int32_t)((double)(float)xs[i] / c);
            if (covered[(size_t)row * gc + col]) continue;
            cur.push_back(i);
            const int32_t r0 = row >= reach ? row - reach : 0, r1 = row + reach <= ncr ? row + reach : ncr;
            const int32_t c0 = col >= reach ? col - reach : 0, c1 = col + reach <= ncc ? col + reach : ncc;
            for (int32_t r = r0; r <= r1; ++r) std::memset(&covered[(size_t)r * gc + c0], 1, (size_t)(c1 - c0 + 1));
        }
        if (cur.size() >= kmin && cur.size() <= kmax) {
            out.swap(cur);
            return;
        }
        if (cur.size() < kmin) high = wdt - 1;
        else low = wdt + 1;
        prev_w = wdt;
        prev.swap(cur);
    }
}

}  // namespace svo
