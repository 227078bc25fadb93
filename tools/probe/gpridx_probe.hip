// Cost of VGPR indexing mode (s_set_gpr_idx_on / off around v_mov) against plain v_mov, one workgroup of
// 512 threads (two waves per SIMD), cycles per iteration on thread 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(512, 1) k_idx(uint64_t* out, int n, int stride) {
    uint32_t lo = threadIdx.x, hi = 0;
    asm volatile("v_mov_b32 v200, %0\n\tv_mov_b32 v201, %0" :: "v"(lo) : "v200", "v201", "v255");
    const uint64_t t0 = clock64();
    for (int i = 0; i < n; ++i) {
        const int idx = __builtin_amdgcn_readfirstlane((i * stride) & 31);
        asm volatile("s_set_gpr_idx_on %2, gpr_idx(SRC0)\n\tv_mov_b32 %0, v200\n\tv_mov_b32 %1, v201\n\ts_set_gpr_idx_off"
                     : "=v"(lo), "=v"(hi) : "s"(idx));
        lo += hi;
    }
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = lo; }
}
__global__ void __launch_bounds__(512, 1) k_plain(uint64_t* out, int n, int stride) {
    uint32_t lo = threadIdx.x, hi = 0;
    asm volatile("v_mov_b32 v200, %0\n\tv_mov_b32 v201, %0" :: "v"(lo) : "v200", "v201", "v255");
    const uint64_t t0 = clock64();
    for (int i = 0; i < n; ++i) {
        const int idx = __builtin_amdgcn_readfirstlane((i * stride) & 31);
        asm volatile("s_mov_b32 m0, %2\n\tv_mov_b32 %0, v200\n\tv_mov_b32 %1, v201"
                     : "=v"(lo), "=v"(hi) : "s"(idx));
        lo += hi;
    }
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = lo; }
}
__global__ void __launch_bounds__(512, 1) k_cmp(uint64_t* out, int n, int stride) {
    uint32_t lo = threadIdx.x;
    double p = 1.5;
    uint64_t acc = 0;
    asm volatile("v_mov_b32 v200, %0\n\tv_mov_b32 v201, %0" :: "v"(lo) : "v200", "v201", "v255");
    const uint64_t t0 = clock64();
    for (int i = 0; i < n; ++i) {
        const int idx = __builtin_amdgcn_readfirstlane((i * stride) & 31);
        uint64_t m;
        asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_cmp_nlt_f64 %0, v[200:201], %2\n\ts_set_gpr_idx_off"
                     : "=s"(m) : "s"(idx), "s"(p));
        acc += m;
    }
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}

int main() {
    uint64_t* d;
    hipMalloc(&d, 64);
    uint64_t h[2];
    const int n = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_idx, dim3(1), dim3(512), 0, 0, d, n, 2);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("gpr_idx v_mov pair: %.1f cycles / iteration\n", (double)h[0] / n);
        hipLaunchKernelGGL(k_plain, dim3(1), dim3(512), 0, 0, d, n, 2);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("plain  v_mov pair: %.1f cycles / iteration\n", (double)h[0] / n);
        hipLaunchKernelGGL(k_cmp, dim3(1), dim3(512), 0, 0, d, n, 2);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("gpr_idx v_cmp_f64: %.1f cycles / iteration\n", (double)h[0] / n);
    }
    return 0;
}
