// pyramid.hip — ImagePyramid::createImagePyramid (src/image_pyramid.cpp:36-52) on gfx950.
//
//   gradient L0 : Simd::AbsGradientSaturatedSum (3rd_party/simd/include/Simd/SimdLib.h:856-884):
//                 min(|I(x+1,y)-I(x-1,y)| + |I(x,y+1)-I(x,y-1)|, 255), border pixels 0
//   level l > 0 : cv::pyrDown of level l-1 for BOTH stacks (the gradient stack is pyrDown of the
//                 gradient, not the gradient of the downsampled image): 5x5 [1 4 6 4 1]^2 kernel,
//                 BORDER_REFLECT_101, (sum + 128) >> 8, dst size ((w+1)/2, (h+1)/2).
// Integer arithmetic only, so the result is bit-exact by construction.  pyrDown: each 256-thread
// workgroup computes a 64x16 destination tile from a (2*16+4)x(2*64+4) source tile staged in LDS
// (reflection only for border tiles), separable horizontal then vertical pass.  Gradient: flat 4096-pixel
// runs staged with 16-B loads, 16 pixels and one 16-B store per thread.
#include "svo_internal.h"

namespace svo {

namespace {

constexpr int kTileW = 64, kTileH = 16;
constexpr int kSrcW = 2 * kTileW + 4, kSrcH = 2 * kTileH + 4;

// BORDER_REFLECT_101 for i in [-2, n + 1] (the 5-tap footprint of a valid output); staged halo cells
// that no output reads are clamped into the image so that every staged load stays in bounds.
__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    i = i < 0 ? -i : i;
    i = i >= n ? 2 * n - 2 - i : i;
    return min(max(i, 0), n - 1);
}

// frames [first, first+count) x {intensity, gradient}; grid.z = 2*count.  Separable: the horizontal
// [1 4 6 4 1] pass over the staged rows into LDS (16-bit sums), then the vertical pass.
__global__ void __launch_bounds__(256) pyr_down_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off,
                                                       int64_t src_off, int sw, int sh, int64_t dst_off, int dw,
                                                       int dh, int first) {
    __shared__ uint8_t tile[kSrcH][kSrcW];
    __shared__ uint16_t hs[kSrcH][kTileW];
    const int frame = first + (blockIdx.z >> 1);
    uint8_t* base = stacks + frame * frame_stride + ((blockIdx.z & 1) ? grad_off : 0);
    const uint8_t* src = base + src_off;
    uint8_t* dst = base + dst_off;
    const int dx0 = blockIdx.x * kTileW, dy0 = blockIdx.y * kTileH;
    const int sx0 = 2 * dx0 - 2, sy0 = 2 * dy0 - 2;
    const bool interior = sx0 >= 0 && sy0 >= 0 && sx0 + kSrcW <= sw && sy0 + kSrcH <= sh;
    for (int i = threadIdx.x; i < kSrcH * kSrcW; i += 256) {
        const int ty = i / kSrcW, tx = i - ty * kSrcW;
        const int y = interior ? sy0 + ty : reflect101(sy0 + ty, sh);
        const int x = interior ? sx0 + tx : reflect101(sx0 + tx, sw);
        tile[ty][tx] = src[(int64_t)y * sw + x];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kSrcH * kTileW; i += 256) {
        const int ty = i / kTileW, tx = i - ty * kTileW;
        const uint8_t* r = tile[ty] + 2 * tx;
        hs[ty][tx] = (uint16_t)(r[0] + 4 * r[1] + 6 * r[2] + 4 * r[3] + r[4]);
    }
    __syncthreads();
    const int tx = threadIdx.x & (kTileW - 1);
    for (int ty = threadIdx.x >> 6; ty < kTileH; ty += 4) {
        const int x = dx0 + tx, y = dy0 + ty;
        if (x >= dw || y >= dh) continue;
        const int s = hs[2 * ty][tx] + 4 * hs[2 * ty + 1][tx] + 6 * hs[2 * ty + 2][tx] + 4 * hs[2 * ty + 3][tx] +
                      hs[2 * ty + 4][tx];
        dst[(int64_t)y * dw + x] = (uint8_t)((s + 128) >> 8);
    }
}

// Simd::AbsGradientSaturatedSum over a flat run of kGradRun pixels per workgroup: the run plus one row
// (and one pixel) either side is staged in LDS with 16-B loads, each thread forms 16 consecutive pixels
// and writes them with one 16-B store.  Plane bases are 256-B aligned (make_geom), so the run is too.
constexpr int kGradRun = 256 * 16;
constexpr int kGradMaxW = 4096;  // staged rows: the run + 2 rows + 2 px (+ 16-B rounding)
constexpr int kGradStage = kGradRun + 2 * kGradMaxW + 64;

__global__ void __launch_bounds__(256) abs_grad_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off, int w,
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
    for (int64_t o = (int64_t)threadIdx.x * 16; o < full; o += 256 * 16)
        *reinterpret_cast<uint4*>(st + o) = *reinterpret_cast<const uint4*>(src + s0 + o);
    for (int64_t o = full + threadIdx.x; o < s1 - s0; o += 256) st[o] = src[s0 + o];
    __syncthreads();
    const int64_t q0 = p0 + (int64_t)threadIdx.x * 16;
    if (q0 >= npx) return;
    int y = (int)(q0 / w), x = (int)(q0 - (int64_t)y * w);
    uint32_t out[4] = {0, 0, 0, 0};
    const int n = npx - q0 < 16 ? (int)(npx - q0) : 16;
    for (int i = 0; i < n; ++i) {
        uint32_t g = 0;
        if (x > 0 && y > 0 && x < w - 1 && y < h - 1) {
            const uint8_t* c = st + (q0 + i - s0);
            const int gx = abs((int)c[1] - (int)c[-1]);
            const int gy = abs((int)c[w] - (int)c[-w]);
            g = (uint32_t)min(gx + gy, 255);
        }
        out[i >> 2] |= g << (8 * (i & 3));
        if (++x == w) { x = 0; ++y; }
    }
    if (n == 16) {
        *reinterpret_cast<uint4*>(dst + q0) = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
        for (int i = 0; i < n; ++i) dst[q0 + i] = (uint8_t)(out[i >> 2] >> (8 * (i & 3)));
    }
}

}  // namespace

// stacks: device base of the pyramid set; frame i occupies [i*stride, i*stride + 2*frame_bytes):
// intensity stack at +0, gradient stack at +grad_off.  Level 0 of the intensity stack must be filled.
void launch_pyramid(uint8_t* stacks, const LevelGeom& g, int32_t first, int32_t count, hipStream_t s) {
    const int64_t grad_off = (g.frame_bytes + 255) / 256 * 256;
    const int64_t stride = (grad_off + g.frame_bytes + 255) / 256 * 256;
    const int64_t npx = (int64_t)g.w[0] * g.h[0];
    hipLaunchKernelGGL(abs_grad_kernel, dim3((unsigned)((npx + kGradRun - 1) / kGradRun), count), dim3(256), 0, s,
                       stacks, stride, grad_off, g.w[0], g.h[0], first);
    for (int l = 1; l < g.levels; ++l) {
        dim3 grid((g.w[l] + kTileW - 1) / kTileW, (g.h[l] + kTileH - 1) / kTileH, 2 * count);
        hipLaunchKernelGGL(pyr_down_kernel, grid, dim3(256), 0, s, stacks, stride, grad_off, g.off[l - 1], g.w[l - 1],
                           g.h[l - 1], g.off[l], g.w[l], g.h[l], first);
    }
}

}  // namespace svo
