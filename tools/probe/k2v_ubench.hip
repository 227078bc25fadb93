// k2v_ubench.hip — cycle costs of K2V's per-row primitives on gfx950 (diagnostic, not part of the product).
// One workgroup of 64 / 256 / 512 / 1024 threads (1, 4, 8, 16 waves: 2 waves share a SIMD from 8 on, 4 at 16) runs each
// variant's loop of kIters x 4 rows on register-resident doubles; thread 0 of every wave reports clock64 cycles per
// row, and the workgroup's aggregate rows per 1000 cycles (waves x rows / the slowest wave's cycles).  Variants: the classification quad (round-4 serial form through VCC / the compares-first form), the
// compares alone, the exchange-source quad (round-4 serial form / independent per-row chains), a v_readlane ->
// SALU -> v_readlane ping-pong, an LDS write -> read round trip.
//   hipcc -O3 --offload-arch=gfx950 -o tools/probe_bin/k2v_ubench tools/probe/k2v_ubench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kIters = 2000;

__device__ int ub_writelane(int v, int l, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wl(uint32_t old, uint32_t v, int l) { return (uint32_t)ub_writelane((int)v, l, (int)old); }

template <int V>
__global__ void __launch_bounds__(1024) ubench(double* io, uint64_t* cyc, uint32_t* sink) {
    __shared__ double mb[4096];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double x0 = io[tid], x1 = io[tid + 512], x2 = io[tid + 1024], x3 = io[tid + 1536];
    const double p = io[4096];
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, acc = 0;
    const uint32_t pb = (uint32_t)(uintptr_t)mb + 8u * (uint32_t)lane;
    __syncthreads();
    const uint64_t t0 = clock64();
    for (int it = 0; it < kIters; ++it) {
        if constexpr (V == 0) {  // round-4 cls4: GE into VCC, LE into an SGPR pair moved through VCC
            uint64_t m;
            asm volatile(
                "v_cmp_ngt_f64 vcc, %[p], %[x0]\n\tv_cmp_nlt_f64_e64 %[m], %[p], %[x0]\n\tv_writelane_b32 %[a0], vcc_lo, 0\n\t"
                "v_writelane_b32 %[a1], vcc_hi, 0\n\ts_mov_b64 vcc, %[m]\n\tv_writelane_b32 %[a2], vcc_lo, 0\n\t"
                "v_writelane_b32 %[a3], vcc_hi, 0\n\t"
                "v_cmp_ngt_f64 vcc, %[p], %[x1]\n\tv_cmp_nlt_f64_e64 %[m], %[p], %[x1]\n\tv_writelane_b32 %[a0], vcc_lo, 1\n\t"
                "v_writelane_b32 %[a1], vcc_hi, 1\n\ts_mov_b64 vcc, %[m]\n\tv_writelane_b32 %[a2], vcc_lo, 1\n\t"
                "v_writelane_b32 %[a3], vcc_hi, 1\n\t"
                "v_cmp_ngt_f64 vcc, %[p], %[x2]\n\tv_cmp_nlt_f64_e64 %[m], %[p], %[x2]\n\tv_writelane_b32 %[a0], vcc_lo, 2\n\t"
                "v_writelane_b32 %[a1], vcc_hi, 2\n\ts_mov_b64 vcc, %[m]\n\tv_writelane_b32 %[a2], vcc_lo, 2\n\t"
                "v_writelane_b32 %[a3], vcc_hi, 2\n\t"
                "v_cmp_ngt_f64 vcc, %[p], %[x3]\n\tv_cmp_nlt_f64_e64 %[m], %[p], %[x3]\n\tv_writelane_b32 %[a0], vcc_lo, 3\n\t"
                "v_writelane_b32 %[a1], vcc_hi, 3\n\ts_mov_b64 vcc, %[m]\n\tv_writelane_b32 %[a2], vcc_lo, 3\n\t"
                "v_writelane_b32 %[a3], vcc_hi, 3"
                : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [m] "=&s"(m)
                : [p] "s"(p), [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3)
                : "vcc");
        } else if constexpr (V == 1 || V == 2) {  // compares first (e64 into SGPR pairs), then the writelanes
            uint64_t g0, g1, g2, g3, l0, l1, l2, l3;
            asm volatile(
                "v_cmp_ngt_f64_e64 %[g0], %[p], %[x0]\n\tv_cmp_nlt_f64_e64 %[l0], %[p], %[x0]\n\t"
                "v_cmp_ngt_f64_e64 %[g1], %[p], %[x1]\n\tv_cmp_nlt_f64_e64 %[l1], %[p], %[x1]\n\t"
                "v_cmp_ngt_f64_e64 %[g2], %[p], %[x2]\n\tv_cmp_nlt_f64_e64 %[l2], %[p], %[x2]\n\t"
                "v_cmp_ngt_f64_e64 %[g3], %[p], %[x3]\n\tv_cmp_nlt_f64_e64 %[l3], %[p], %[x3]"
                : [g0] "=&s"(g0), [g1] "=&s"(g1), [g2] "=&s"(g2), [g3] "=&s"(g3), [l0] "=&s"(l0), [l1] "=&s"(l1),
                  [l2] "=&s"(l2), [l3] "=&s"(l3)
                : [p] "s"(p), [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3));
            if (V == 1) {
                a0 = wl(a0, (uint32_t)g0, 0); a1 = wl(a1, (uint32_t)(g0 >> 32), 0);
                a2 = wl(a2, (uint32_t)l0, 0); a3 = wl(a3, (uint32_t)(l0 >> 32), 0);
                a0 = wl(a0, (uint32_t)g1, 1); a1 = wl(a1, (uint32_t)(g1 >> 32), 1);
                a2 = wl(a2, (uint32_t)l1, 1); a3 = wl(a3, (uint32_t)(l1 >> 32), 1);
                a0 = wl(a0, (uint32_t)g2, 2); a1 = wl(a1, (uint32_t)(g2 >> 32), 2);
                a2 = wl(a2, (uint32_t)l2, 2); a3 = wl(a3, (uint32_t)(l2 >> 32), 2);
                a0 = wl(a0, (uint32_t)g3, 3); a1 = wl(a1, (uint32_t)(g3 >> 32), 3);
                a2 = wl(a2, (uint32_t)l3, 3); a3 = wl(a3, (uint32_t)(l3 >> 32), 3);
            } else {
                acc += (uint32_t)(g0 ^ g1 ^ g2 ^ g3 ^ l0 ^ l1 ^ l2 ^ l3);  // (keeps the compares; one SALU xor chain)
            }
        } else if constexpr (V == 3) {  // round-4 src4: per row readlane / exec / mbcnt x2 / address / ds_write
            uint64_t m0, m1, m2, m3, sv;
            uint32_t t, k, a;
            asm volatile(
                "s_mov_b64 %[sv], exec\n\tv_cmp_nlt_f64 %[m0], %[x0], %[p]\n\tv_cmp_nlt_f64 %[m1], %[x1], %[p]\n\t"
                "v_cmp_nlt_f64 %[m2], %[x2], %[p]\n\tv_cmp_nlt_f64 %[m3], %[x3], %[p]\n\t"
                "v_readlane_b32 %[t], %[pb], 0\n\ts_mov_b64 exec, %[m0]\n\tv_mbcnt_lo_u32_b32 %[k], exec_lo, 0\n\t"
                "v_mbcnt_hi_u32_b32 %[k], exec_hi, %[k]\n\tv_lshl_add_u32 %[a], %[k], 3, %[t]\n\tds_write_b64 %[a], %[x0]\n\t"
                "v_readlane_b32 %[t], %[pb], 1\n\ts_mov_b64 exec, %[m1]\n\tv_mbcnt_lo_u32_b32 %[k], exec_lo, 0\n\t"
                "v_mbcnt_hi_u32_b32 %[k], exec_hi, %[k]\n\tv_lshl_add_u32 %[a], %[k], 3, %[t]\n\tds_write_b64 %[a], %[x1]\n\t"
                "v_readlane_b32 %[t], %[pb], 2\n\ts_mov_b64 exec, %[m2]\n\tv_mbcnt_lo_u32_b32 %[k], exec_lo, 0\n\t"
                "v_mbcnt_hi_u32_b32 %[k], exec_hi, %[k]\n\tv_lshl_add_u32 %[a], %[k], 3, %[t]\n\tds_write_b64 %[a], %[x2]\n\t"
                "v_readlane_b32 %[t], %[pb], 3\n\ts_mov_b64 exec, %[m3]\n\tv_mbcnt_lo_u32_b32 %[k], exec_lo, 0\n\t"
                "v_mbcnt_hi_u32_b32 %[k], exec_hi, %[k]\n\tv_lshl_add_u32 %[a], %[k], 3, %[t]\n\tds_write_b64 %[a], %[x3]\n\t"
                "s_mov_b64 exec, %[sv]"
                : [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [sv] "=&s"(sv), [t] "=&s"(t),
                  [k] "=&v"(k), [a] "=&v"(a)
                : [p] "s"(p), [pb] "v"(pb), [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3)
                : "memory", "scc");
        } else if constexpr (V == 4) {  // round-5 src4: compares, then four independent slot chains, then the writes
            uint64_t m0, m1, m2, m3, sv;
            asm volatile("v_cmp_nlt_f64 %[m0], %[x0], %[p]\n\tv_cmp_nlt_f64 %[m1], %[x1], %[p]\n\t"
                         "v_cmp_nlt_f64 %[m2], %[x2], %[p]\n\tv_cmp_nlt_f64 %[m3], %[x3], %[p]"
                         : [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3)
                         : [p] "s"(p), [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3));
            uint32_t t0, t1, t2, t3, k0, k1, k2, k3;
            asm volatile(
                "s_nop 0\n\tv_readlane_b32 %[t0], %[pb], 0\n\tv_readlane_b32 %[t1], %[pb], 1\n\t"
                "v_readlane_b32 %[t2], %[pb], 2\n\tv_readlane_b32 %[t3], %[pb], 3\n\t"
                "v_mbcnt_lo_u32_b32 %[k0], %[l0], 0\n\tv_mbcnt_lo_u32_b32 %[k1], %[l1], 0\n\t"
                "v_mbcnt_lo_u32_b32 %[k2], %[l2], 0\n\tv_mbcnt_lo_u32_b32 %[k3], %[l3], 0\n\t"
                "v_mbcnt_hi_u32_b32 %[k0], %[h0], %[k0]\n\tv_mbcnt_hi_u32_b32 %[k1], %[h1], %[k1]\n\t"
                "v_mbcnt_hi_u32_b32 %[k2], %[h2], %[k2]\n\tv_mbcnt_hi_u32_b32 %[k3], %[h3], %[k3]\n\t"
                "v_lshl_add_u32 %[k0], %[k0], 3, %[t0]\n\tv_lshl_add_u32 %[k1], %[k1], 3, %[t1]\n\t"
                "v_lshl_add_u32 %[k2], %[k2], 3, %[t2]\n\tv_lshl_add_u32 %[k3], %[k3], 3, %[t3]\n\t"
                "s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m0]\n\tds_write_b64 %[k0], %[x0]\n\t"
                "s_mov_b64 exec, %[m1]\n\tds_write_b64 %[k1], %[x1]\n\ts_mov_b64 exec, %[m2]\n\tds_write_b64 %[k2], %[x2]\n\t"
                "s_mov_b64 exec, %[m3]\n\tds_write_b64 %[k3], %[x3]\n\ts_mov_b64 exec, %[sv]"
                : [sv] "=&s"(sv), [t0] "=&s"(t0), [t1] "=&s"(t1), [t2] "=&s"(t2), [t3] "=&s"(t3), [k0] "=&v"(k0),
                  [k1] "=&v"(k1), [k2] "=&v"(k2), [k3] "=&v"(k3)
                : [pb] "v"(pb), [m0] "s"(m0), [m1] "s"(m1), [m2] "s"(m2), [m3] "s"(m3), [l0] "s"((uint32_t)m0),
                  [l1] "s"((uint32_t)m1), [l2] "s"((uint32_t)m2), [l3] "s"((uint32_t)m3), [h0] "s"((uint32_t)(m0 >> 32)),
                  [h1] "s"((uint32_t)(m1 >> 32)), [h2] "s"((uint32_t)(m2 >> 32)), [h3] "s"((uint32_t)(m3 >> 32)),
                  [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3)
                : "memory", "scc");
        } else if constexpr (V == 5) {  // readlane -> SALU -> readlane ping-pong (the search chains' pattern)
            uint32_t s = acc;
#pragma unroll
            for (int i = 0; i < 4; ++i) s = (uint32_t)__builtin_amdgcn_readlane((int)(a0 + s), (int)(s & 63)) + 1u;
            acc = s;
        } else if constexpr (V == 7) {  // four indexed-register reads (s_set_gpr_idx_on SRC0 / v_mov / off), K2V's vget
            uint32_t lo0, lo1, lo2, lo3;
            const uint32_t i0 = (acc & 3u) * 2u, i1 = ((acc + 1u) & 3u) * 2u, i2 = ((acc + 2u) & 3u) * 2u, i3 = ((acc + 3u) & 3u) * 2u;
            asm volatile("s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\tv_mov_b32 %0, %8\n\ts_set_gpr_idx_off\n\t"
                         "s_set_gpr_idx_on %5, gpr_idx(SRC0)\n\tv_mov_b32 %1, %8\n\ts_set_gpr_idx_off\n\t"
                         "s_set_gpr_idx_on %6, gpr_idx(SRC0)\n\tv_mov_b32 %2, %8\n\ts_set_gpr_idx_off\n\t"
                         "s_set_gpr_idx_on %7, gpr_idx(SRC0)\n\tv_mov_b32 %3, %8\n\ts_set_gpr_idx_off"
                         : "=&v"(lo0), "=&v"(lo1), "=&v"(lo2), "=&v"(lo3)
                         : "s"(__builtin_amdgcn_readfirstlane(i0)), "s"(__builtin_amdgcn_readfirstlane(i1)),
                           "s"(__builtin_amdgcn_readfirstlane(i2)), "s"(__builtin_amdgcn_readfirstlane(i3)),
                           "v"((uint32_t)__builtin_bit_cast(uint64_t, x0)));
            acc += lo0 ^ lo1 ^ lo2 ^ lo3;
        } else if constexpr (V == 8) {  // the same four reads on fixed registers (plain v_mov)
            uint32_t lo0, lo1, lo2, lo3;
            asm volatile("v_mov_b32 %0, %4\n\tv_mov_b32 %1, %5\n\tv_mov_b32 %2, %6\n\tv_mov_b32 %3, %7"
                         : "=&v"(lo0), "=&v"(lo1), "=&v"(lo2), "=&v"(lo3)
                         : "v"((uint32_t)__builtin_bit_cast(uint64_t, x0)), "v"((uint32_t)__builtin_bit_cast(uint64_t, x1)),
                           "v"((uint32_t)__builtin_bit_cast(uint64_t, x2)), "v"((uint32_t)__builtin_bit_cast(uint64_t, x3)));
            acc += lo0 ^ lo1 ^ lo2 ^ lo3;
        } else if constexpr (V == 6) {  // LDS write -> read round trip (uniform address)
            mb[(acc & 1023u) + 64u * wave] = x0;
            asm volatile("" ::: "memory");
            const double y = mb[((acc + 1u) & 1023u) + 64u * wave];
            acc += (uint32_t)(y > p) + 1u;
        }
    }
    const uint64_t t1 = clock64();
    if (lane == 0) cyc[wave] = t1 - t0;
    sink[tid] = a0 ^ a1 ^ a2 ^ a3 ^ acc;
}

int main() {
    (void)hipSetDevice(0);
    double *io;
    uint64_t* cyc;
    uint32_t* sink;
    (void)hipMalloc(&io, 8 * 5000);
    (void)hipMalloc(&cyc, 8 * 16);
    (void)hipMalloc(&sink, 4 * 1024);
    double h[5000];
    for (int i = 0; i < 5000; ++i) h[i] = (i * 37 % 101) - 50.0;
    h[4096] = 0.5;
    (void)hipMemcpy(io, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[] = {"cls quad, round-4 serial (VCC)", "cls quad, compares first + writelanes",
                           "8 compares only", "src quad, round-4 serial", "src quad, independent chains",
                           "readlane->SALU->readlane", "LDS write->read", "4 indexed reads (gpr_idx)", "4 fixed v_mov"};
    void (*ks[])(double*, uint64_t*, uint32_t*) = {ubench<0>, ubench<1>, ubench<2>, ubench<3>, ubench<4>, ubench<5>,
                                                   ubench<6>, ubench<7>, ubench<8>};
    for (int v = 0; v < 9; ++v) {
        for (int nw : {1, 4, 8, 16}) {
            hipLaunchKernelGGL(ks[v], dim3(1), dim3(64 * nw), 0, 0, io, cyc, sink);  // warm
            hipLaunchKernelGGL(ks[v], dim3(1), dim3(64 * nw), 0, 0, io, cyc, sink);
            uint64_t c[16] = {};
            (void)hipMemcpy(c, cyc, 8 * nw, hipMemcpyDeviceToHost);
            const double per = v == 6 ? 1.0 : 4.0;  // (rows per iteration: 4; V5: 4 ping-pongs; V6: 1 round trip)
            uint64_t cmax = 0;
            for (int w = 0; w < nw; ++w) cmax = c[w] > cmax ? c[w] : cmax;
            printf("%-42s waves %2d: cycles per row  w0 %.1f  w%d %.1f   aggregate rows per 1000 cycles %.1f\n", names[v], nw,
                   c[0] / (double)kIters / per, nw - 1, c[nw - 1] / (double)kIters / per,
                   1000.0 * nw * kIters * per / (double)cmax);
        }
    }
    hipError_t e = hipDeviceSynchronize();
    printf("done: %s\n", hipGetErrorString(e));
    return 0;
}
