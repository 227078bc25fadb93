// Probe: raw buffer stores/loads with a scalar row offset + lane offset (gfx950 descriptor word 3).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__global__ void k(double* p, double* out, int stride, int flags) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, stride * 8 * 25, flags);
    for (int kk = 0; kk < 25; ++kk) {
        double v = threadIdx.x + 1000.0 * kk;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, threadIdx.x * 8, kk * stride * 8, 0);
    }
    __syncthreads();
    double s = 0;
    for (int kk = 0; kk < 25; ++kk)
        s += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, threadIdx.x * 8, kk * stride * 8, 0));
    out[threadIdx.x] = s;
}
int main() {
    const int stride = 72;
    double *p, *o;
    hipMalloc(&p, 8 * stride * 25); hipMalloc(&o, 8 * 64);
    for (int flags : {0x00020000, 0x00027000, 0x00024000}) {
        hipMemset(p, 0, 8 * stride * 25);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, p, o, stride, flags);
        double h[64], hp[72 * 25];
        hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
        hipMemcpy(hp, p, sizeof(hp), hipMemcpyDeviceToHost);
        printf("flags %#x: lane5 sum %.1f (expect %.1f), p[3*72+5]=%.1f (expect 3005)\n", flags, h[5], 25 * 5 + 1000.0 * 300, hp[3 * 72 + 5]);
    }
    return 0;
}
