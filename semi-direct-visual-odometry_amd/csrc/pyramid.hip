// pyramid.hip — ImagePyramid::createImagePyramid (src/image_pyramid.cpp:36-52) on gfx950.
//
//   gradient L0 : Simd::AbsGradientSaturatedSum (3rd_party/simd/include/Simd/SimdLib.h:856-884):
//                 min(|I(x+1,y)-I(x-1,y)| + |I(x,y+1)-I(x,y-1)|, 255), border pixels 0
//   level l > 0 : cv::pyrDown of level l-1 for BOTH stacks (the gradient stack is pyrDown of the
//                 gradient, not the gradient of the downsampled image): 5x5 [1 4 6 4 1]^2 kernel,
//                 BORDER_REFLECT_101, (sum + 128) >> 8, dst size ((w+1)/2, (h+1)/2).
// Integer arithmetic only, so the result is bit-exact by construction.  Each 256-thread workgroup
// computes a 64x16 destination tile from a (2*16+3)x(2*64+3) source tile staged in LDS with
// coalesced row reads; the vertical pass runs on the staged rows.
#include "svo_internal.h"

namespace svo {

namespace {

constexpr int kTileW = 64, kTileH = 16;
constexpr int kSrcW = 2 * kTileW + 4, kSrcH = 2 * kTileH + 4;

// BORDER_REFLECT_101 for any i (periodic form; staged halo cells that no output uses stay in range)
__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    const int period = 2 * n - 2;
    i %= period;
    if (i < 0) i += period;
    return i >= n ? period - i : i;
}

// frames [first, first+count) x {intensity, gradient}; grid.z = 2*count
__global__ void __launch_bounds__(256) pyr_down_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off,
                                                       int64_t src_off, int sw, int sh, int64_t dst_off, int dw,
                                                       int dh, int first) {
    __shared__ uint8_t tile[kSrcH][kSrcW];
    const int frame = first + (blockIdx.z >> 1);
    uint8_t* base = stacks + frame * frame_stride + ((blockIdx.z & 1) ? grad_off : 0);
    const uint8_t* src = base + src_off;
    uint8_t* dst = base + dst_off;
    const int dx0 = blockIdx.x * kTileW, dy0 = blockIdx.y * kTileH;
    const int sx0 = 2 * dx0 - 2, sy0 = 2 * dy0 - 2;
    for (int i = threadIdx.x; i < kSrcH * kSrcW; i += 256) {
        const int ty = i / kSrcW, tx = i - ty * kSrcW;
        const int y = reflect101(sy0 + ty, sh);
        const int x = reflect101(sx0 + tx, sw);
        tile[ty][tx] = src[(int64_t)y * sw + x];
    }
    __syncthreads();
    const int tx = threadIdx.x & (kTileW - 1);
    for (int ty = threadIdx.x >> 6; ty < kTileH; ty += 4) {
        const int x = dx0 + tx, y = dy0 + ty;
        if (x >= dw || y >= dh) continue;
        int s = 0;
        const int k[5] = {1, 4, 6, 4, 1};
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint8_t* row = tile[2 * ty + i] + 2 * tx;
            const int rs = row[0] + 4 * row[1] + 6 * row[2] + 4 * row[3] + row[4];
            s += k[i] * rs;
        }
        dst[(int64_t)y * dw + x] = (uint8_t)((s + 128) >> 8);
    }
}

__global__ void __launch_bounds__(256) abs_grad_kernel(uint8_t* stacks, int64_t frame_stride, int64_t grad_off, int w,
                                                       int h, int first) {
    const int frame = first + blockIdx.z;
    const uint8_t* src = stacks + frame * frame_stride;
    uint8_t* dst = stacks + frame * frame_stride + grad_off;
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= w || y >= h) return;
    uint8_t out = 0;
    if (x > 0 && y > 0 && x < w - 1 && y < h - 1) {
        const int64_t o = (int64_t)y * w + x;
        const int dx = abs((int)src[o + 1] - (int)src[o - 1]);
        const int dy = abs((int)src[o + w] - (int)src[o - w]);
        out = (uint8_t)min(dx + dy, 255);
    }
    dst[(int64_t)y * w + x] = out;
}

}  // namespace

// stacks: device base of the pyramid set; frame i occupies [i*stride, i*stride + 2*frame_bytes):
// intensity stack at +0, gradient stack at +grad_off.  Level 0 of the intensity stack must be filled.
void launch_pyramid(uint8_t* stacks, const LevelGeom& g, int32_t first, int32_t count, hipStream_t s) {
    const int64_t grad_off = (g.frame_bytes + 255) / 256 * 256;
    const int64_t stride = (grad_off + g.frame_bytes + 255) / 256 * 256;
    hipLaunchKernelGGL(abs_grad_kernel, dim3((g.w[0] + 63) / 64, (g.h[0] + 3) / 4, count), dim3(256), 0, s, stacks,
                       stride, grad_off, g.w[0], g.h[0], first);
    for (int l = 1; l < g.levels; ++l) {
        dim3 grid((g.w[l] + kTileW - 1) / kTileW, (g.h[l] + kTileH - 1) / kTileH, 2 * count);
        hipLaunchKernelGGL(pyr_down_kernel, grid, dim3(256), 0, s, stacks, stride, grad_off, g.off[l - 1], g.w[l - 1],
                           g.h[l - 1], g.off[l], g.w[l], g.h[l], first);
    }
}

}  // namespace svo
