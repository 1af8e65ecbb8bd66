// VALU issue rate on gfx950 by instruction class: 8 independent chains per lane, 4 waves
// per SIMD (1024-thread blocks, one per CU... grid = 4 x CUs of 256 threads), timed with
// hipEvents.  Prints wave64 instructions per SIMD-cycle for each class (at the nominal
// 2.4 GHz; the clock is reported from the kernel's s_memtime span too).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(256) void k_rate(float* out, double* outd, int iters, unsigned long long* clk) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
    unsigned long long smask = 0x5555555555555555ull ^ (unsigned long long)iters;
    asm volatile("" : "+s"(smask));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (KIND == 0) {  // v_mul_f32
                asm volatile("v_mul_f32 %0, %0, %0\n v_mul_f32 %1, %1, %1\n v_mul_f32 %2, %2, %2\n v_mul_f32 %3, %3, %3\n"
                             "v_mul_f32 %4, %4, %4\n v_mul_f32 %5, %5, %5\n v_mul_f32 %6, %6, %6\n v_mul_f32 %7, %7, %7"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if (KIND == 1) {  // v_mul_f64
                asm volatile("v_mul_f64 %0, %0, %0\n v_mul_f64 %1, %1, %1\n v_mul_f64 %2, %2, %2\n v_mul_f64 %3, %3, %3\n"
                             "v_mul_f64 %4, %4, %4\n v_mul_f64 %5, %5, %5\n v_mul_f64 %6, %6, %6\n v_mul_f64 %7, %7, %7"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
            } else if (KIND == 2) {  // v_add_f64
                asm volatile("v_add_f64 %0, %0, %0\n v_add_f64 %1, %1, %1\n v_add_f64 %2, %2, %2\n v_add_f64 %3, %3, %3\n"
                             "v_add_f64 %4, %4, %4\n v_add_f64 %5, %5, %5\n v_add_f64 %6, %6, %6\n v_add_f64 %7, %7, %7"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
            } else if (KIND == 3) {  // v_pk_mul_f32 on pairs
                asm volatile("v_pk_mul_f32 %0, %0, %0\n v_pk_mul_f32 %1, %1, %1\n v_pk_mul_f32 %2, %2, %2\n v_pk_mul_f32 %3, %3, %3\n"
                             "v_pk_mul_f32 %4, %4, %4\n v_pk_mul_f32 %5, %5, %5\n v_pk_mul_f32 %6, %6, %6\n v_pk_mul_f32 %7, %7, %7"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
            } else if (KIND == 4) {  // v_fma_f64
                asm volatile("v_fma_f64 %0, %0, %0, %0\n v_fma_f64 %1, %1, %1, %1\n v_fma_f64 %2, %2, %2, %2\n v_fma_f64 %3, %3, %3, %3\n"
                             "v_fma_f64 %4, %4, %4, %4\n v_fma_f64 %5, %5, %5, %5\n v_fma_f64 %6, %6, %6, %6\n v_fma_f64 %7, %7, %7, %7"
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
            } else if (KIND == 5) {  // v_cmp_gt_f64 (into SGPR pairs) — compare cost
                unsigned long long m0, m1, m2, m3;
                asm volatile("v_cmp_gt_f64 %0, %4, %5\n v_cmp_gt_f64 %1, %5, %6\n v_cmp_gt_f64 %2, %6, %7\n v_cmp_gt_f64 %3, %7, %4\n"
                             "v_cmp_gt_f64 %0, %4, %5\n v_cmp_gt_f64 %1, %5, %6\n v_cmp_gt_f64 %2, %6, %7\n v_cmp_gt_f64 %3, %7, %4"
                             : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(d0), "v"(d1), "v"(d2), "v"(d3));
            } else if (KIND == 6) {  // v_max_f32
                asm volatile("v_max_f32 %0, %0, %1\n v_max_f32 %1, %1, %2\n v_max_f32 %2, %2, %3\n v_max_f32 %3, %3, %4\n"
                             "v_max_f32 %4, %4, %5\n v_max_f32 %5, %5, %6\n v_max_f32 %6, %6, %7\n v_max_f32 %7, %7, %0"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if (KIND == 8) {  // v_cndmask_b32_e64 with an SGPR pair set by SALU outside the loop
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %8\n v_cndmask_b32_e64 %1, %1, %2, %8\n v_cndmask_b32_e64 %2, %2, %3, %8\n v_cndmask_b32_e64 %3, %3, %4, %8\n"
                             "v_cndmask_b32_e64 %4, %4, %5, %8\n v_cndmask_b32_e64 %5, %5, %6, %8\n v_cndmask_b32_e64 %6, %6, %7, %8\n v_cndmask_b32_e64 %7, %7, %0, %8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(smask));
            } else if (KIND == 9) {  // v_cmp_gt_f32 into SGPR pairs, 8 per block (no cndmask)
                unsigned long long m0, m1, m2, m3;
                asm volatile("v_cmp_gt_f32 %0, %4, %5\n v_cmp_gt_f32 %1, %5, %6\n v_cmp_gt_f32 %2, %6, %7\n v_cmp_gt_f32 %3, %7, %4\n"
                             "v_cmp_gt_f32 %0, %4, %5\n v_cmp_gt_f32 %1, %5, %6\n v_cmp_gt_f32 %2, %6, %7\n v_cmp_gt_f32 %3, %7, %4"
                             : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
            } else if (KIND == 10) {  // v_add_u32 (integer)
                asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %1, %1, %2\n v_add_u32 %2, %2, %3\n v_add_u32 %3, %3, %4\n"
                             "v_add_u32 %4, %4, %5\n v_add_u32 %5, %5, %6\n v_add_u32 %6, %6, %7\n v_add_u32 %7, %7, %0"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if (KIND == 11) {  // v_fma_f32 independent
                asm volatile("v_fma_f32 %0, %0, %0, %1\n v_fma_f32 %1, %1, %1, %2\n v_fma_f32 %2, %2, %2, %3\n v_fma_f32 %3, %3, %3, %4\n"
                             "v_fma_f32 %4, %4, %4, %5\n v_fma_f32 %5, %5, %5, %6\n v_fma_f32 %6, %6, %6, %7\n v_fma_f32 %7, %7, %7, %0"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if (KIND == 12) {  // v_max3_f32
                asm volatile("v_max3_f32 %0, %0, %1, %2\n v_max3_f32 %1, %1, %2, %3\n v_max3_f32 %2, %2, %3, %4\n v_max3_f32 %3, %3, %4, %5\n"
                             "v_max3_f32 %4, %4, %5, %6\n v_max3_f32 %5, %5, %6, %7\n v_max3_f32 %6, %6, %7, %0\n v_max3_f32 %7, %7, %0, %1"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            } else if (KIND == 13) {  // v_writelane_b32 (register stack push)
                asm volatile("v_writelane_b32 %0, %8, 1\n v_writelane_b32 %1, %8, 2\n v_writelane_b32 %2, %8, 3\n v_writelane_b32 %3, %8, 4\n"
                             "v_writelane_b32 %4, %8, 5\n v_writelane_b32 %5, %8, 6\n v_writelane_b32 %6, %8, 7\n v_writelane_b32 %7, %8, 8"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"((unsigned)smask));
            } else if (KIND == 14) {  // (A) cmp vcc -> 1 cndmask vcc -> 6 independent v_mul_f32
                asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_mul_f32 %2, %2, %2\n v_mul_f32 %3, %3, %3\n"
                             "v_mul_f32 %4, %4, %4\n v_mul_f32 %5, %5, %5\n v_mul_f32 %6, %6, %6\n v_mul_f32 %7, %7, %7"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
            } else if (KIND == 15) {  // (B) cmp -> SGPR pair, cndmask_e64 reading it, x4
                unsigned long long m0, m1;
                asm volatile("v_cmp_gt_f32 %8, %0, %1\n v_cndmask_b32_e64 %0, %0, %1, %8\n v_cmp_gt_f32 %9, %2, %3\n v_cndmask_b32_e64 %2, %2, %3, %9\n"
                             "v_cmp_gt_f32 %8, %4, %5\n v_cndmask_b32_e64 %4, %4, %5, %8\n v_cmp_gt_f32 %9, %6, %7\n v_cndmask_b32_e64 %6, %6, %7, %9"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=&s"(m0), "=&s"(m1));
            } else if (KIND == 16) {  // (C) 8 cndmask reading vcc set by SALU outside
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n"
                             "v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %5, %5, %6, vcc\n v_cndmask_b32 %6, %6, %7, vcc\n v_cndmask_b32 %7, %7, %0, vcc"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
            } else if (KIND == 17) {  // (D) cmp vcc followed by cmp vcc (no cndmask): cmp into vcc x8
                asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cmp_gt_f32 vcc, %1, %2\n v_cmp_gt_f32 vcc, %2, %3\n v_cmp_gt_f32 vcc, %3, %4\n"
                             "v_cmp_gt_f32 vcc, %4, %5\n v_cmp_gt_f32 vcc, %5, %6\n v_cmp_gt_f32 vcc, %6, %7\n v_cmp_gt_f32 vcc, %7, %0"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
            } else if (KIND == 18) {  // (E) cmp vcc -> 2 consecutive cndmask vcc (a 64-bit select) -> 5 mul
                asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_mul_f32 %3, %3, %3\n"
                             "v_mul_f32 %4, %4, %4\n v_mul_f32 %5, %5, %5\n v_mul_f32 %6, %6, %6\n v_mul_f32 %7, %7, %7"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
            } else if (KIND == 19) {  // (F) 8 cndmask e32 reading vcc written by ONE v_cmp at the block start, each separated by a mul
                asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_mul_f32 %2, %2, %2\n v_cndmask_b32 %3, %3, %4, vcc\n"
                             "v_mul_f32 %4, %4, %4\n v_cndmask_b32 %5, %5, %6, vcc\n v_mul_f32 %6, %6, %6\n v_cndmask_b32 %7, %7, %0, vcc"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
            } else if (KIND == 7) {  // v_cndmask_b32 (vcc)
                asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n"
                             "v_cndmask_b32 %3, %3, %4, vcc\n v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %5, %5, %6, vcc\n v_cndmask_b32 %6, %6, %7, vcc"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    outd[blockIdx.x * 256 + threadIdx.x] = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const char* names[] = {"v_mul_f32", "v_mul_f64", "v_add_f64", "v_pk_mul_f32", "v_fma_f64", "v_cmp_gt_f64", "v_max_f32",
                           "v_cndmask_b32(+1 cmp/8)", "v_cndmask_e64 sgpr", "v_cmp_gt_f32", "v_add_u32", "v_fma_f32",
                           "v_max3_f32", "v_writelane_b32", "(A) cmp>cnd(vcc)+6mul", "(B) cmp>sgpr>cnd x4", "(C) cnd vcc(salu)", "(D) cmp vcc x8", "(E) cmp>2cnd+5mul", "(F) cmp>(cnd,mul)x4"};
    float* o;
    double* od;
    unsigned long long* clk;
    (void)hipMalloc(&o, sizeof(float) * 256 * cus * 64);
    (void)hipMalloc(&od, sizeof(double) * 256 * cus * 64);
    (void)hipMalloc(&clk, 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 4096;
    for (int wps = 2; wps <= 4; wps *= 2) {  // waves per SIMD: blocks of 256 threads = 4 waves (one per SIMD)
        const int grid = cus * wps;
        for (int kind = 0; kind < 20; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0);
                switch (kind) {
#define L(K) case K: hipLaunchKernelGGL(k_rate<K>, dim3(grid), dim3(256), 0, 0, o, od, iters, clk); break;
                    L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19)
#undef L
                }
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                unsigned long long c = 0;
                (void)hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
                const double insts_per_simd = (double)iters * 64 * wps;  // wave-instructions per SIMD
                const double cyc = ms * 1e-3 * 2.4e9;
                if (rep) printf("waves/SIMD %d  %-24s  %.3f ms  SIMD-cycles per wave64 instr %.2f  (wave's own s_memtime span %.0f ticks: %.2f per instr)\n",
                                wps, names[kind], ms, cyc / insts_per_simd, (double)c, (double)c / (iters * 64));
            }
        }
    }
    return 0;
}
