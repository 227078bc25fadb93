// pyramid.hip — ImagePyramid::createImagePyramid (src/image_pyramid.cpp:36-52) on gfx950.
//
//   gradient L0 : Simd::AbsGradientSaturatedSum (3rd_party/simd/include/Simd/SimdLib.h:856-884):
//                 min(|I(x+1,y)-I(x-1,y)| + |I(x,y+1)-I(x,y-1)|, 255), border pixels 0
//   level l > 0 : cv::pyrDown of level l-1 for BOTH stacks (the gradient stack is pyrDown of the
//                 gradient, not the gradient of the downsampled image): 5x5 [1 4 6 4 1]^2 kernel,
//                 BORDER_REFLECT_101, (sum + 128) >> 8, dst size ((w+1)/2, (h+1)/2).
// Integer arithmetic only, so the result is bit-exact by construction.  One launch per level for any number of frames
// (DESIGN 18.4):
//   pyr_l01_kernel   level-0 gradient + level 1 of both stacks, one register-streaming pass over the base image;
//   pyr_dn_kernel    each later level of both stacks, register-streaming pyrDown.
// The round-4 kernels stay behind SVO_PYR=0 for A/B measurement: abs_grad_kernel (flat 8192-px runs staged with
// 16-B loads, 16 pixels and one 16-B store per thread) and pyr_down_kernel (8x256 destination tiles, vertical pass
// from global memory into LDS, then the horizontal pass), one launch per level.
#include "svo_internal.h"

namespace svo {

namespace {

// BORDER_REFLECT_101 for i in [-2, n + 1] (the 5-tap footprint of a valid output); rows / columns that
// no output reads are clamped into the image so that every load stays in bounds.
__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    i = i < 0 ? -i : i;
    i = i >= n ? 2 * n - 2 - i : i;
    return min(max(i, 0), n - 1);
}

// frames [first, first+count) x {intensity, gradient}; grid.z = 2*count.  A workgroup makes an
// 8-row x 256-column destination tile: vertical [1 4 6 4 1] pass first, one thread per source column
// reading its 20 source rows straight from global memory (consecutive threads, consecutive bytes),
// 16-bit column sums into LDS, then the horizontal pass from LDS.
#ifndef SVO_DNH
#define SVO_DNH 8
#endif
constexpr int kDnW = 256, kDnH = SVO_DNH;
constexpr int kDnCols = 2 * kDnW + 4, kDnRows = 2 * kDnH + 4;

__global__ void __launch_bounds__(256) pyr_down_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off,
                                                       int64_t src_off, int sw, int sh, int64_t dst_off, int dw,
                                                       int dh, int first) {
    __shared__ uint16_t vs[kDnH][kDnCols];
    const int frame = first + (blockIdx.z >> 1);
    uint8_t* base = stacks + frame * frame_stride + ((blockIdx.z & 1) ? grad_off : 0);
    const uint8_t* src = base + src_off;
    uint8_t* dst = base + dst_off;
    const int dx0 = blockIdx.x * kDnW, dy0 = blockIdx.y * kDnH;
    const int sx0 = 2 * dx0 - 2, sy0 = 2 * dy0 - 2;
    const int nrows = min(kDnH, dh - dy0);                 // destination rows of this tile
    const int ncols = min(2 * min(kDnW, dw - dx0) + 4, kDnCols);  // source columns the tile reads
    int64_t roff[kDnRows];
#pragma unroll
    for (int r = 0; r < kDnRows; ++r) roff[r] = (int64_t)reflect101(sy0 + r, sh) * sw;
    for (int c = threadIdx.x; c < ncols; c += 256) {
        const int x = reflect101(sx0 + c, sw);
        uint32_t v[kDnRows];
#pragma unroll
        for (int r = 0; r < kDnRows; ++r) v[r] = src[roff[r] + x];
#pragma unroll
        for (int t = 0; t < kDnH; ++t)
            if (t < nrows)
                vs[t][c] = (uint16_t)(v[2 * t] + 4 * v[2 * t + 1] + 6 * v[2 * t + 2] + 4 * v[2 * t + 3] + v[2 * t + 4]);
    }
    __syncthreads();
    const int x = dx0 + threadIdx.x;
    if (x >= dw) return;
    const int c = 2 * threadIdx.x;
    for (int t = 0; t < nrows; ++t) {
        const uint16_t* r = vs[t] + c;
        const int s = r[0] + 4 * r[1] + 6 * r[2] + 4 * r[3] + r[4];
        dst[(int64_t)(dy0 + t) * dw + x] = (uint8_t)((s + 128) >> 8);
    }
}

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ uint32_t grad4(uint32_t l, uint32_t r, uint32_t u, uint32_t d) {
    uint32_t res = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const u16x2 L = as_u16x2((l >> (8 * half)) & 0x00FF00FFu), R = as_u16x2((r >> (8 * half)) & 0x00FF00FFu);
        const u16x2 Up = as_u16x2((u >> (8 * half)) & 0x00FF00FFu), Dn = as_u16x2((d >> (8 * half)) & 0x00FF00FFu);
        const u16x2 gx = __builtin_elementwise_max(L, R) - __builtin_elementwise_min(L, R);
        const u16x2 gy = __builtin_elementwise_max(Up, Dn) - __builtin_elementwise_min(Up, Dn);
        const u16x2 g = __builtin_elementwise_min(gx + gy, (u16x2){255, 255});
        res |= as_u32(g) << (8 * half);
    }
    return res;
}

// Simd::AbsGradientSaturatedSum over a flat run of kGradRun (8192) pixels per workgroup: the run plus one row
// (and one pixel) either side is staged in LDS with 16-B loads, each thread forms 16 consecutive pixels
// and writes them with one 16-B store.  Plane bases are 256-B aligned (make_geom), so the run is too.
// Interior runs read aligned dwords and realign them with v_alignbyte; the four neighbours are combined
// byte-parallel in 16-bit lanes.  Runs touching the border take a per-pixel path.
constexpr int kGradThreads = 512;
constexpr int kGradRun = kGradThreads * 16;
constexpr int kGradMaxW = 4096;  // staged rows: the run + 2 rows + 2 px (+ 16-B rounding)
constexpr int kGradStage = kGradRun + 2 * kGradMaxW + 64;

__global__ void __launch_bounds__(kGradThreads) abs_grad_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off, int w,
                                                       int h, int first) {
    __shared__ __attribute__((aligned(16))) uint8_t st[kGradStage];
    const int frame = first + blockIdx.y;
    const uint8_t* src = stacks + frame * frame_stride;
    uint8_t* dst = stacks + frame * frame_stride + grad_off;
    const int64_t npx = (int64_t)w * h;
    const int64_t p0 = (int64_t)blockIdx.x * kGradRun;
    // staged range [s0, s1): 16-B aligned, covering [p0 - w - 1, p0 + kGradRun + w + 1) within the plane
    const int64_t lo = p0 - w - 1 < 0 ? 0 : p0 - w - 1;
    const int64_t s0 = lo & ~(int64_t)15;
    int64_t s1 = p0 + kGradRun + w + 1;
    s1 = s1 > npx ? npx : s1;
    const int64_t full = (s1 - s0) & ~(int64_t)15;  // 16-B chunks entirely inside the plane
    for (int64_t o = (int64_t)threadIdx.x * 16; o < full; o += kGradThreads * 16)
        *reinterpret_cast<uint4*>(st + o) = *reinterpret_cast<const uint4*>(src + s0 + o);
    for (int64_t o = full + threadIdx.x; o < s1 - s0; o += kGradThreads) st[o] = src[s0 + o];
    __syncthreads();
    // 32-bit index math (planes are < 2^31 px; 64-bit divisions were a large part of the kernel)
    const uint32_t q0 = (uint32_t)p0 + (uint32_t)threadIdx.x * 16u, NPX = (uint32_t)npx, W = (uint32_t)w;
    if (q0 >= NPX) return;
    const uint32_t y = q0 / W, x = q0 - y * W;
    const int n = NPX - q0 < 16u ? (int)(NPX - q0) : 16;
    const int c0 = (int)(q0 - (uint32_t)s0);  // 16-B aligned LDS offset of the run
    uint32_t out[4];
    if (n == 16 && w >= 32 && c0 >= w) {  // (c0 < w: the plane's first row; up-neighbours unstaged)
        // every full group on the byte-parallel path (aligned dword LDS reads realigned with v_alignbyte),
        // including groups that wrap onto the next row (the flat layout keeps every non-border pixel's four
        // neighbours right); pixels on the image border (Simd leaves them 0) are cleared afterwards.
        // Reads past the staged bytes (the last row's down-neighbours) stay inside the array and only feed
        // cleared pixels.
        const uint32_t* sd = reinterpret_cast<const uint32_t*>(st);
        uint32_t C[6], U[5], D[5];
#pragma unroll
        for (int i = 0; i < 6; ++i) C[i] = sd[c0 / 4 - 1 + i];
        const int cu = c0 - w, cd = c0 + w;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            U[i] = sd[(cu >> 2) + i];
            D[i] = sd[(cd >> 2) + i];
        }
        const uint32_t su = (uint32_t)(cu & 3), sdn = (uint32_t)(cd & 3);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            out[i] = grad4(__builtin_amdgcn_alignbyte(C[i + 1], C[i], 3), __builtin_amdgcn_alignbyte(C[i + 2], C[i + 1], 1),
                           __builtin_amdgcn_alignbyte(U[i + 1], U[i], su), __builtin_amdgcn_alignbyte(D[i + 1], D[i], sdn));
        // border pixels of the group: bit i for pixel q0 + i (w >= 32: at most one row end inside)
        const uint32_t rem = W - x;  // pixels of row y from q0 on
        const uint32_t in_y = rem >= 16u ? 0xFFFFu : (1u << rem) - 1u;
        uint32_t z = 0;
        if (y == 0 || y == (uint32_t)h - 1) z |= in_y;
        if (rem < 16u && y + 1 == (uint32_t)h - 1) z |= 0xFFFFu & ~in_y;
        if (x == 0) z |= 1u;
        if (rem <= 16u) z |= 1u << (rem - 1);  // column w - 1
        if (rem < 16u) z |= 1u << rem;         // column 0 of row y + 1
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t zb = (z >> (4 * i)) & 0xFu;
            const uint32_t m = ((zb & 1u) ? 0xFFu : 0u) | ((zb & 2u) ? 0xFF00u : 0u) | ((zb & 4u) ? 0xFF0000u : 0u) |
                               ((zb & 8u) ? 0xFF000000u : 0u);
            out[i] &= ~m;
        }
    } else {
        int yy = (int)y, xx = (int)x;
        out[0] = out[1] = out[2] = out[3] = 0;
        for (int i = 0; i < n; ++i) {
            uint32_t g = 0;
            if (xx > 0 && yy > 0 && xx < w - 1 && yy < h - 1) {
                const uint8_t* c = st + (c0 + i);
                const int gx = abs((int)c[1] - (int)c[-1]);
                const int gy = abs((int)c[w] - (int)c[-w]);
                g = (uint32_t)min(gx + gy, 255);
            }
            out[i >> 2] |= g << (8 * (i & 3));
            if (++xx == w) { xx = 0; ++yy; }
        }
    }
    if (n == 16) {
        *reinterpret_cast<uint4*>(dst + q0) = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
        for (int i = 0; i < n; ++i) dst[q0 + i] = (uint8_t)(out[i >> 2] >> (8 * (i & 3)));
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Level-0 gradient + level 1 of BOTH stacks in one pass over the base image (pyr_l01_kernel).
//
// One wave streams a vertical strip of the base image down a band of level-1 rows, entirely in registers: lane l
// holds four source columns c0 = 4 (own * strip + l - 1) .. c0 + 3 of each row as one dword (an aligned dword buffer
// load realigned with the right neighbour lane's dword through DPP), lanes 0 and 63 are halo lanes (their values
// feed their neighbours' taps; they store nothing).  Every row is kept as two u16 pairs, columns (0, 2) and (1, 3),
// and all arithmetic runs on packed u16 pairs (every sum of this pyramid stays below 2^16):
//  * the gradient (Simd::AbsGradientSaturatedSum) in the pair domain: the left / right neighbours of columns (0, 2)
//    are (-1, 1) / (1, 3) and of (1, 3) are (0, 2) / (2, 4), one DPP and one alignbyte per parity;
//  * the vertical [1 4 6 4 1] pass as running sums: source row 2m + 1 adds 4x to level-1 rows m and m + 1, row 2m
//    adds 1x / 6x / 1x to rows m - 1, m, m + 1, so a lane carries two partial sums per stack and the four base rows
//    the gradient needs, and every role alternates between two register sets from one step to the next (the loop,
//    unrolled by two, moves no register); the 4x / 6x terms are v_pk_mad_u16;
//  * the horizontal pass takes the neighbour lanes' sums by DPP, the rounding shift folded into the final byte
//    permute (the high bytes of sum + 128);
//  * BORDER_REFLECT_101: rows through the reflected row index of each tap (every tap of a valid output is one
//    reflection away; bands that touch neither the first nor the last base rows carry no reflection and no border-row
//    test), columns by substituting the reflected sums in the edge strips.
// The outputs leave straight from the lanes: a dword per lane per gradient row, a 16-bit pair per lane per level-1
// row, at their (unaligned) addresses; the lanes at the right edge store byte by byte.  Integer arithmetic only:
// bit-exact.  (Round 5 history, DESIGN 18.4: the same pass with a window of unpacked rows (v2), with the running
// sums but per-pixel neighbour permutes (v3), with aligned-dword gradient stores or paired level-1 stores, each
// measured slower on the same box.)
constexpr int kL01Waves = 4;                  // independent waves per workgroup (strip x band each)
constexpr int kL01Band = 32;                  // level-1 rows per band
constexpr int kStripOwn = 61;                 // owner lanes per strip at most (lanes 0 and own + 1 <= 62 are halo)

// (bound_ctrl: the lane without a source reads 0; no "old" operand to materialize)
__device__ __forceinline__ uint32_t from_left(uint32_t v) {   // lane i <- lane i - 1 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {  // lane i <- lane i + 1 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xF, 0xF, true);
}
__device__ __forceinline__ int refl101(int i, int n) {  // one reflection (valid taps never need two) + clamp
    i = i < 0 ? -i : i;
    i = i >= n ? 2 * n - 2 - i : i;
    return min(max(i, 0), n - 1);
}

typedef uint16_t u16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pe(uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0C020C00u); }  // b0, b2
__device__ __forceinline__ uint32_t po(uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0x0C030C01u); }  // b1, b3
__device__ __forceinline__ uint32_t pk_absdiff(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_max(as_u16x2(a), as_u16x2(b)) - __builtin_elementwise_min(as_u16x2(a), as_u16x2(b)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return as_u32(as_u16x2(a) + as_u16x2(b)); }
struct Acc {
    uint32_t ie, io, ge, go;  // intensity / gradient partial sums, columns (0, 2) and (1, 3)
};
__device__ __forceinline__ uint32_t pk_mad4(uint32_t a, uint32_t c) {  // a * 4 + c on u16 pairs, one instruction
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, 4, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t pk_mad6(uint32_t a, uint32_t c) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, 6, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(c));
    return r;
}
struct Px2 {
    uint32_t e, o;  // columns (0, 2) and (1, 3) as u16 pairs
};

template <bool kLE, bool kRE, bool kIn>
__device__ __forceinline__ void l01_strip(uint8_t* ibase, uint8_t* gbase, int32_t stack_bytes, int W, int H, int64_t off1,
                                            int W1, int own, int col0, int r0, int r1, int lane) {
    const int c0 = col0 + 4 * (lane - 1);
    const int cl = (c0 >= 0 && c0 <= W + 3) ? c0 : 0;
    const bool owner = lane >= 1 && lane <= own;
    uint32_t me = 0xFFFFFFFFu, mo = 0xFFFFFFFFu;
    if (kLE && c0 == 0) me &= 0xFFFF0000u;
    if (kRE) {
        if (c0 == W - 1) me &= 0xFFFF0000u;
        if (c0 + 2 == W - 1) me &= 0x0000FFFFu;
        if (c0 + 1 == W - 1) mo &= 0xFFFF0000u;
        if (c0 + 3 == W - 1) mo &= 0x0000FFFFu;
    }
    // (buffer accesses: the stack in a descriptor, the row offset a scalar, the lane's column the vector offset; no
    // 64-bit address arithmetic per lane and access)
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(ibase, 0, stack_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(gbase, 0, stack_bytes, 0x00020000);
    const uint32_t ucl = (uint32_t)cl, uc0 = (uint32_t)c0, ux = (uint32_t)(c0 >> 1);
    auto prow = [&](int y) -> int64_t {  // (uniform) the base offset of image row y
        return kIn ? (int64_t)__builtin_amdgcn_readfirstlane(y) * W
                   : (int64_t)__builtin_amdgcn_readfirstlane(refl101(y, H)) * W;
    };
    auto raw = [&](int y) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(ri, ucl, (uint32_t)(prow(y) & ~(int64_t)3), 0);
    };
    auto cook = [&](uint32_t lo, int y) -> Px2 {
        const uint32_t v = __builtin_amdgcn_alignbyte(from_right(lo), lo, (uint32_t)(prow(y) & 3));
        return Px2{pe(v), po(v)};
    };
    auto grad = [&](const Px2& up, const Px2& mid, const Px2& dn, int y, uint32_t& ge, uint32_t& go) {
        const uint32_t le = __builtin_amdgcn_alignbyte(mid.o, from_left(mid.o), 2);   // columns (-1, 1)
        const uint32_t ro = __builtin_amdgcn_alignbyte(from_right(mid.e), mid.e, 2);  // columns (2, 4)
        const u16x2v lim = {255, 255};
        ge = as_u32(__builtin_elementwise_min(as_u16x2(pk_add(pk_absdiff(le, mid.o), pk_absdiff(up.e, dn.e))), lim));
        go = as_u32(__builtin_elementwise_min(as_u16x2(pk_add(pk_absdiff(mid.e, ro), pk_absdiff(up.o, dn.o))), lim));
        if (!kIn) {
            const int py = __builtin_amdgcn_readfirstlane(refl101(y, H));
            if (py == 0 || py == H - 1) {  // (uniform)
                ge = 0u;
                go = 0u;
            }
        }
        if (kLE || kRE) {
            ge &= me;
            go &= mo;
        }
    };
    auto hpass2 = [&](uint32_t ev, uint32_t od) -> uint32_t {
        const uint32_t lev = from_left(ev), lod = from_left(od), rev = from_right(ev);
        uint32_t A = __builtin_amdgcn_alignbyte(ev, lev, 2), B = __builtin_amdgcn_alignbyte(od, lod, 2);
        uint32_t C = ev, D = od, E = __builtin_amdgcn_alignbyte(rev, ev, 2);
        if (kLE && c0 == 0) {
            A = (A & 0xFFFF0000u) | (C >> 16);
            B = (B & 0xFFFF0000u) | (D & 0xFFFFu);
        }
        if (kRE) {
            const int d = W - 1 - c0;
            if (d == 0) {
                D = (D & 0xFFFF0000u) | (B & 0xFFFFu);
                E = (E & 0xFFFF0000u) | (A & 0xFFFFu);
            } else if (d == 1) {
                E = (E & 0xFFFF0000u) | (C & 0xFFFFu);
            } else if (d == 2) {
                D = (D & 0xFFFFu) | (B & 0xFFFF0000u);
                E = (E & 0xFFFFu) | (A & 0xFFFF0000u);
            } else if (d == 3) {
                E = (E & 0xFFFFu) | (C & 0xFFFF0000u);
            }
        }
        // (A + E) + 4 (B + D) + 6 C + 128, every partial below 2^16; the outputs are the pairs' high bytes
        const uint32_t t = pk_mad6(C, pk_mad4(pk_add(B, D), pk_add(A, E)));
        const uint32_t q = as_u32(as_u16x2(t) + (u16x2v){128, 128});
        return __builtin_amdgcn_perm(0u, q, 0x0C0C0301u);  // x0 | x1 << 8
    };
    const bool full_g = owner && (!kRE || c0 + 3 < W), part_g = kRE && owner && c0 < W && c0 + 3 >= W;
    const int x = c0 >> 1;
    const bool full_1 = owner && (!kRE || x + 1 < W1), part_1 = kRE && owner && x == W1 - 1;
    const int ylim = min(2 * r1, H);
    auto store_grad = [&](int y, uint32_t ge, uint32_t go) {
        if (y >= ylim) return;  // (uniform)
        const uint32_t v = ge | (go << 8);
        const int64_t ro = (int64_t)__builtin_amdgcn_readfirstlane(y * W);
        if (full_g) __builtin_amdgcn_raw_buffer_store_b32(v, rg, uc0, (uint32_t)ro, 0);
        if (kRE && part_g)
            for (int i = 0; i < 4; ++i)
                if (c0 + i < W) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> (8 * i)), rg, uc0 + (uint32_t)i, (uint32_t)ro, 0);
    };
    auto store_l1 = [&](const __amdgpu_buffer_rsrc_t& rs, int r, uint32_t v) {
        const uint32_t so = (uint32_t)off1 + (uint32_t)__builtin_amdgcn_readfirstlane(r * W1);
        if (full_1) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs, ux, so, 0);
        if (kRE && part_1) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, rs, ux, so, 0);
    };
    auto step = [&](int r, const Px2& I0, const Px2& I1, Px2& I2, Px2& I3, uint32_t& Pa, uint32_t& Pb, Acc& X, Acc& Y) {
        I2 = cook(Pa, 2 * r + 2);
        I3 = cook(Pb, 2 * r + 3);
        Pa = raw(2 * r + 6);
        Pb = raw(2 * r + 7);
        uint32_t g1e, g1o, g2e, g2o;
        grad(I0, I1, I2, 2 * r + 1, g1e, g1o);
        grad(I1, I2, I3, 2 * r + 2, g2e, g2o);
        store_grad(2 * r + 1, g1e, g1o);
        store_grad(2 * r + 2, g2e, g2o);
        X.ie = pk_add(pk_mad4(I1.e, X.ie), I2.e);
        X.io = pk_add(pk_mad4(I1.o, X.io), I2.o);
        X.ge = pk_add(pk_mad4(g1e, X.ge), g2e);
        X.go = pk_add(pk_mad4(g1o, X.go), g2o);
        Y.ie = pk_mad6(I2.e, pk_mad4(I1.e, Y.ie));
        Y.io = pk_mad6(I2.o, pk_mad4(I1.o, Y.io));
        Y.ge = pk_mad6(g2e, pk_mad4(g1e, Y.ge));
        Y.go = pk_mad6(g2o, pk_mad4(g1o, Y.go));
        store_l1(ri, r, hpass2(X.ie, X.io));
        store_l1(rg, r, hpass2(X.ge, X.go));
        X = Acc{I2.e, I2.o, g2e, g2o};
    };
    Px2 Ia, Ib, Ic, Id;
    Acc X, Y;
    {
        const Px2 Jm3 = cook(raw(2 * r0 - 3), 2 * r0 - 3), Jm2 = cook(raw(2 * r0 - 2), 2 * r0 - 2);
        const Px2 Jm1 = cook(raw(2 * r0 - 1), 2 * r0 - 1);
        Ia = cook(raw(2 * r0), 2 * r0);
        Ib = cook(raw(2 * r0 + 1), 2 * r0 + 1);
        uint32_t hm2e, hm2o, hm1e, hm1o, h0e, h0o;
        grad(Jm3, Jm2, Jm1, 2 * r0 - 2, hm2e, hm2o);
        grad(Jm2, Jm1, Ia, 2 * r0 - 1, hm1e, hm1o);
        grad(Jm1, Ia, Ib, 2 * r0, h0e, h0o);
        store_grad(2 * r0, h0e, h0o);
        X.ie = pk_mad6(Ia.e, pk_mad4(Jm1.e, Jm2.e));
        X.io = pk_mad6(Ia.o, pk_mad4(Jm1.o, Jm2.o));
        X.ge = pk_mad6(h0e, pk_mad4(hm1e, hm2e));
        X.go = pk_mad6(h0o, pk_mad4(hm1o, hm2o));
        Y = Acc{Ia.e, Ia.o, h0e, h0o};
    }
    uint32_t P0 = raw(2 * r0 + 2), P1 = raw(2 * r0 + 3), P2 = raw(2 * r0 + 4), P3 = raw(2 * r0 + 5);
    int r = r0;
    for (; r + 1 < r1; r += 2) {
        step(r, Ia, Ib, Ic, Id, P0, P1, X, Y);
        step(r + 1, Ic, Id, Ia, Ib, P2, P3, Y, X);
    }
    if (r < r1) step(r, Ia, Ib, Ic, Id, P0, P1, X, Y);
}

__global__ void __launch_bounds__(64 * kL01Waves) pyr_l01_kernel(uint8_t* stacks, int64_t frame_stride,
                                                                   int64_t grad_off, int W, int H, int64_t off1, int W1,
                                                                   int H1, int own, int nstrip, int nband, int first) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = blockIdx.x * kL01Waves + wv;
    if (gw >= nstrip * nband) return;  // (wave-uniform)
    const int strip = gw % nstrip, band = gw / nstrip;
    uint8_t* const ibase = stacks + (first + (int64_t)blockIdx.y) * frame_stride;
    uint8_t* const gbase = ibase + grad_off;
    const int col0 = 4 * own * strip;
    const int r0 = band * kL01Band, r1 = min(r0 + kL01Band, H1);
    const bool le = strip == 0, re = col0 + 4 * own >= W;
    // the band's rows 2 r0 - 3 .. 2 r1 + 7 (reads, the prefetch included) and its gradient rows 2 r0 - 2 .. 2 r1 all
    // inside [1, H - 2]: no reflection, no border row
    const bool in = 2 * r0 - 3 >= 1 && 2 * r1 + 7 <= H - 2;
    const int32_t sb = (int32_t)grad_off;  // (each stack's bytes fit below the gradient stack's offset)
#define SVO_L01(LE, RE)                                                                                     \
    if (in) l01_strip<LE, RE, true>(ibase, gbase, sb, W, H, off1, W1, own, col0, r0, r1, lane);               \
    else l01_strip<LE, RE, false>(ibase, gbase, sb, W, H, off1, W1, own, col0, r0, r1, lane);
    if (le && re) { SVO_L01(true, true) }
    else if (le) { SVO_L01(true, false) }
    else if (re) { SVO_L01(false, true) }
    else { SVO_L01(false, false) }
#undef SVO_L01
}

// ---------------------------------------------------------------------------------------------------------------
// pyr_dn_kernel: cv::pyrDown of one level of either stack (levels >= 2),
// the register-streaming form of pyr_l01_kernel without the gradient: lane l takes four source columns as two u16
// pairs, two running sums per lane, two output pixels per lane and output row, unrolled by two so that no register
// moves; buffer accesses, v_pk_mad_u16 for the 4x / 6x terms, the rounding shift in the final permute, interior bands
// without reflection.  grid.y = 2 * frames (stack, frame).
template <bool kLE, bool kRE, bool kIn>
__device__ __forceinline__ void dn_strip(uint8_t* base, int32_t stack_bytes, uint32_t src_off, uint32_t dst_off, int W,
                                          int H, int W1, int own, int col0, int r0, int r1, int lane) {
    const int c0 = col0 + 4 * (lane - 1);
    const int cl = (c0 >= 0 && c0 <= W + 3) ? c0 : 0;
    const bool owner = lane >= 1 && lane <= own;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, stack_bytes, 0x00020000);
    const uint32_t ucl = (uint32_t)cl, ux = (uint32_t)(c0 >> 1);
    auto prow = [&](int y) -> uint32_t {
        return kIn ? (uint32_t)__builtin_amdgcn_readfirstlane(y) * (uint32_t)W
                   : (uint32_t)__builtin_amdgcn_readfirstlane(refl101(y, H)) * (uint32_t)W;
    };
    auto raw = [&](int y) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(rs, ucl, src_off + (prow(y) & ~3u), 0);
    };
    auto cook = [&](uint32_t lo, int y, uint32_t& e, uint32_t& o) {
        const uint32_t v = __builtin_amdgcn_alignbyte(from_right(lo), lo, prow(y) & 3u);
        e = pe(v);
        o = po(v);
    };
    auto hpass2 = [&](uint32_t ev, uint32_t od) -> uint32_t {
        const uint32_t lev = from_left(ev), lod = from_left(od), rev = from_right(ev);
        uint32_t A = __builtin_amdgcn_alignbyte(ev, lev, 2), B = __builtin_amdgcn_alignbyte(od, lod, 2);
        uint32_t C = ev, D = od, E = __builtin_amdgcn_alignbyte(rev, ev, 2);
        if (kLE && c0 == 0) {
            A = (A & 0xFFFF0000u) | (C >> 16);
            B = (B & 0xFFFF0000u) | (D & 0xFFFFu);
        }
        if (kLE && kRE && W <= 2) {  // one or two columns: every tap reflects back into them (x0 only: W1 = 1)
            const uint32_t v0 = C & 0xFFFFu, v1 = W == 2 ? (D & 0xFFFFu) : v0;
            A = v0;
            B = v1;
            C = v0;
            D = v1;
            E = v0;
        } else if (kRE) {
            const int d = W - 1 - c0;
            if (d == 0) {
                D = (D & 0xFFFF0000u) | (B & 0xFFFFu);
                E = (E & 0xFFFF0000u) | (A & 0xFFFFu);
            } else if (d == 1) {
                E = (E & 0xFFFF0000u) | (C & 0xFFFFu);
            } else if (d == 2) {
                D = (D & 0xFFFFu) | (B & 0xFFFF0000u);
                E = (E & 0xFFFFu) | (A & 0xFFFF0000u);
            } else if (d == 3) {
                E = (E & 0xFFFFu) | (C & 0xFFFF0000u);
            }
        }
        const uint32_t t = pk_mad6(C, pk_mad4(pk_add(B, D), pk_add(A, E)));
        const uint32_t q = as_u32(as_u16x2(t) + (u16x2v){128, 128});
        return __builtin_amdgcn_perm(0u, q, 0x0C0C0301u);
    };
    const bool full_1 = owner && (!kRE || (int)ux + 1 < W1), part_1 = kRE && owner && (int)ux == W1 - 1;
    auto store = [&](int r, uint32_t v) {
        const uint32_t so = dst_off + (uint32_t)__builtin_amdgcn_readfirstlane(r * W1);
        if (full_1) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs, ux, so, 0);
        if (kRE && part_1) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, rs, ux, so, 0);
    };
    auto step = [&](int r, uint32_t& Pa, uint32_t& Pb, uint32_t& Xe, uint32_t& Xo, uint32_t& Ye, uint32_t& Yo) {
        uint32_t e1, o1, e2, o2;
        cook(Pa, 2 * r + 1, e1, o1);
        cook(Pb, 2 * r + 2, e2, o2);
        Pa = raw(2 * r + 5);
        Pb = raw(2 * r + 6);
        Xe = pk_add(pk_mad4(e1, Xe), e2);
        Xo = pk_add(pk_mad4(o1, Xo), o2);
        Ye = pk_mad6(e2, pk_mad4(e1, Ye));
        Yo = pk_mad6(o2, pk_mad4(o1, Yo));
        store(r, hpass2(Xe, Xo));
        Xe = e2;
        Xo = o2;
    };
    uint32_t Xe, Xo, Ye, Yo;
    {
        uint32_t e0, o0, e1, o1, e2, o2;
        cook(raw(2 * r0 - 2), 2 * r0 - 2, e0, o0);
        cook(raw(2 * r0 - 1), 2 * r0 - 1, e1, o1);
        cook(raw(2 * r0), 2 * r0, e2, o2);
        Xe = pk_mad6(e2, pk_mad4(e1, e0));
        Xo = pk_mad6(o2, pk_mad4(o1, o0));
        Ye = e2;
        Yo = o2;
    }
    uint32_t P0 = raw(2 * r0 + 1), P1 = raw(2 * r0 + 2), P2 = raw(2 * r0 + 3), P3 = raw(2 * r0 + 4);
    int r = r0;
    for (; r + 1 < r1; r += 2) {
        step(r, P0, P1, Xe, Xo, Ye, Yo);
        step(r + 1, P2, P3, Ye, Yo, Xe, Xo);
    }
    if (r < r1) step(r, P0, P1, Xe, Xo, Ye, Yo);
}

__global__ void __launch_bounds__(64 * kL01Waves) pyr_dn_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off,
                                                                 int64_t src_off, int W, int H, int64_t dst_off, int W1,
                                                                 int H1, int own, int nstrip, int nband, int band_rows,
                                                                 int first) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = blockIdx.x * kL01Waves + wv;
    if (gw >= nstrip * nband) return;  // (wave-uniform)
    const int strip = gw % nstrip, band = gw / nstrip;
    uint8_t* const base = stacks + (first + (int64_t)(blockIdx.y >> 1)) * frame_stride + ((blockIdx.y & 1) ? grad_off : 0);
    const int col0 = 4 * own * strip;
    const int r0 = band * band_rows, r1 = min(r0 + band_rows, H1);
    const bool le = strip == 0, re = col0 + 4 * own >= W;
    // source rows 2 r0 - 2 .. 2 r1 + 4 (the prefetch included) inside the plane: no reflection
    const bool in = 2 * r0 - 2 >= 0 && 2 * r1 + 4 <= H - 1;
    const int32_t sb = (int32_t)grad_off;
    const uint32_t so = (uint32_t)src_off, dso = (uint32_t)dst_off;
#define SVO_DN(LE, RE)                                                                                      \
    if (in) dn_strip<LE, RE, true>(base, sb, so, dso, W, H, W1, own, col0, r0, r1, lane);                      \
    else dn_strip<LE, RE, false>(base, sb, so, dso, W, H, W1, own, col0, r0, r1, lane);
    if (le && re) { SVO_DN(true, true) }
    else if (le) { SVO_DN(true, false) }
    else if (re) { SVO_DN(false, true) }
    else { SVO_DN(false, false) }
#undef SVO_DN
}
int pyr_mode() {  // SVO_PYR (measurement knob, read once): 0 the round-4 kernels (abs_grad_kernel, pyr_down_kernel per
                  // level), 1 (default) pyr_l01_kernel + pyr_dn_kernel per level
    static const int m = getenv("SVO_PYR") ? atoi(getenv("SVO_PYR")) : 1;
    return m;
}

}  // namespace

// stacks: device base of the pyramid set; frame i occupies [i*stride, i*stride + 2*frame_bytes):
// intensity stack at +0, gradient stack at +grad_off.  Level 0 of the intensity stack must be filled.
void launch_pyramid(uint8_t* stacks, const LevelGeom& g, int32_t first, int32_t count, hipStream_t s) {
    const int64_t grad_off = (g.frame_bytes + 255) / 256 * 256;
    const int64_t stride = (grad_off + g.frame_bytes + 255) / 256 * 256;
    const int64_t npx = (int64_t)g.w[0] * g.h[0];
    int l = 1;
    if (g.levels >= 2 && pyr_mode() != 0) {
        // strips of `own` lanes x 4 columns, as few strips as the width needs.  own <= kStripOwn (61): lane 0 is the left
        // halo, lane own + 1 the right halo, and the right halo's realigned dword takes its high bytes from lane own + 2
        // (from_right), which must be a real lane; with own = 62 the halo lane 63 would read 0 from a lane 64 that does
        // not exist and the last owner's level-1 gradient tap at the strip seam would be wrong.
        const int nstrip = (g.w[0] + 4 * kStripOwn - 1) / (4 * kStripOwn);
        const int own = (g.w[0] + 4 * nstrip - 1) / (4 * nstrip);
        const int nband = (g.h[1] + kL01Band - 1) / kL01Band;
        const int waves = nstrip * nband;
        hipLaunchKernelGGL(pyr_l01_kernel, dim3((unsigned)((waves + kL01Waves - 1) / kL01Waves), count), dim3(64 * kL01Waves),
                           0, s, stacks, stride, grad_off, g.w[0], g.h[0], g.off[1], g.w[1], g.h[1], own, nstrip, nband, first);
        l = 2;
        for (; l < g.levels; ++l) {
            const int w = g.w[l - 1];
            const int ns = (w + 4 * kStripOwn - 1) / (4 * kStripOwn);
            const int ow = (w + 4 * ns - 1) / (4 * ns);
            const int band_rows = max(8, (g.h[l] + 7) / 8);  // bands of >= 8 output rows, ~8 waves per frame-stack
            const int nb = (g.h[l] + band_rows - 1) / band_rows;
            const int wv = ns * nb;
            hipLaunchKernelGGL(pyr_dn_kernel, dim3((unsigned)((wv + kL01Waves - 1) / kL01Waves), 2 * count),
                               dim3(64 * kL01Waves), 0, s, stacks, stride, grad_off, g.off[l - 1], w, g.h[l - 1], g.off[l],
                               g.w[l], g.h[l], ow, ns, nb, band_rows, first);
        }
    } else {
        hipLaunchKernelGGL(abs_grad_kernel, dim3((unsigned)((npx + kGradRun - 1) / kGradRun), count), dim3(kGradThreads), 0,
                           s, stacks, stride, grad_off, g.w[0], g.h[0], first);
    }
    for (; l < g.levels; ++l) {
        dim3 grid((g.w[l] + kDnW - 1) / kDnW, (g.h[l] + kDnH - 1) / kDnH, 2 * count);
        hipLaunchKernelGGL(pyr_down_kernel, grid, dim3(256), 0, s, stacks, stride, grad_off, g.off[l - 1], g.w[l - 1],
                           g.h[l - 1], g.off[l], g.w[l], g.h[l], first);
    }
}

}  // namespace svo