// Micro-benchmark: issue cost and dependent latency of the fp64 VALU forms the
// LFT sweep is built from (one wave, s_memtime around unrolled asm sequences).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_f64.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void ub(long long* out, double seed) {
  double a = seed, b = seed * 0.5, c0 = seed + 1, c1 = c0 + 1, c2 = c1 + 1, c3 = c2 + 1,
         c4 = c3 + 1, c5 = c4 + 1, c6 = c5 + 1, c7 = c6 + 1;
  long long t0, t1;
  int k = 0;
#define TIME(body, ...)                                                   \
  __builtin_amdgcn_s_waitcnt(0);                                        \
  t0 = __builtin_amdgcn_s_memtime();                                    \
  asm volatile(body : __VA_ARGS__);                                     \
  t1 = __builtin_amdgcn_s_memtime();                                    \
  if (threadIdx.x == 0) out[k] = t1 - t0;                               \
  ++k;
  // 0: empty
  TIME("s_nop 0", "+v"(a));
  // 1: dependent v_fma_f64 chain (64)
  TIME(REP64("v_fma_f64 %0, %0, %1, %1\n"), "+v"(a) : "v"(b));
  // 2: independent v_fma_f64 (8 accumulators x 8)
  TIME(REP8("v_fma_f64 %0, %8, %9, %0\nv_fma_f64 %1, %8, %9, %1\nv_fma_f64 %2, %8, %9, %2\n"
            "v_fma_f64 %3, %8, %9, %3\nv_fma_f64 %4, %8, %9, %4\nv_fma_f64 %5, %8, %9, %5\n"
            "v_fma_f64 %6, %8, %9, %6\nv_fma_f64 %7, %8, %9, %7\n"),
       "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
       : "v"(a), "v"(b));
  // 3: independent v_fmac_f64_dpp row_newbcast (8 accumulators x 8)
  TIME("s_nop 4\n" REP8("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"),
       "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
       : "v"(a), "v"(b));
  // 4: dependent v_rcp_f64 chain (64)
  TIME(REP64("v_rcp_f64 %0, %0\n"), "+v"(a));
  // 5: independent v_rcp_f64 (8 x 8)
  TIME(REP8("v_rcp_f64 %0, %8\nv_rcp_f64 %1, %8\nv_rcp_f64 %2, %8\nv_rcp_f64 %3, %8\n"
            "v_rcp_f64 %4, %8\nv_rcp_f64 %5, %8\nv_rcp_f64 %6, %8\nv_rcp_f64 %7, %8\n"),
       "=v"(c0), "=v"(c1), "=v"(c2), "=v"(c3), "=v"(c4), "=v"(c5), "=v"(c6), "=v"(c7)
       : "v"(a));
  // 6: dependent v_add_f64 chain (64)
  TIME(REP64("v_add_f64 %0, %0, %1\n"), "+v"(a) : "v"(b));
  // 7: dependent VALU -> DPP-mov chain: v_mov_b64_dpp then v_add (32 pairs, s_nop 1 between)
  TIME(REP8(REP8("v_mov_b64_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                 "v_add_f64 %1, %0, %2\ns_nop 1\n")),
       "+v"(c0), "+v"(a) : "v"(b));
  // 8: 64 x v_cndmask_b32 independent
  {
    int x0 = 1, x1 = 2, x2 = 3, x3 = 4;
    TIME(REP8(REP8("v_cndmask_b32_e64 %0, %4, %5, vcc\n") ), "=v"(x0), "=v"(x1), "=v"(x2),
         "=v"(x3) : "v"(x0), "v"(x1));
  }
  // 9: dependent v_fmac_f64_dpp chain through the accumulator (64)
  TIME("s_nop 4\n" REP64("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"),
       "+v"(c0) : "v"(a), "v"(b));
  // 10: v_cmp_lt_f64 + s_and (64 pairs)
  TIME(REP64("v_cmp_lt_f64 vcc, 0, %0\ns_and_b64 s[4:5], s[4:5], vcc\n"), "+v"(a) : : "vcc", "s4", "s5");
  // 11: 64 s_nop 0
  TIME(REP64("s_nop 0\n"), "+v"(a));
  // 12: v_mul_f64 dependent chain (64)
  TIME(REP64("v_mul_f64 %0, %0, %1\n"), "+v"(a) : "v"(b));
  // 13: ds_read_b64 x 64 independent + one wait
  {
    __shared__ double sm[64 * 64];
    sm[threadIdx.x] = a;
    __syncthreads();
    unsigned ad = (unsigned)(uintptr_t)(&sm[threadIdx.x]);
    TIME(REP64("ds_read_b64 %0, %1\n") "s_waitcnt lgkmcnt(0)\n", "=v"(c0) : "v"(ad));
  }

  // 14: sweep pattern: independent fmac_dpp with src0 == acc (8 regs x 8)
  TIME("s_nop 4\n" REP8("v_fmac_f64_dpp %0, %0, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %1, %1, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %2, %2, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %3, %3, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %4, %4, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %5, %5, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %6, %6, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %7, %7, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"),
       "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
       : "v"(a));
  // 15: i-outer GEMM chain: acc += bcast_J(x) * y_J, y_J = 8 different regs, same acc (x8)
  TIME("s_nop 4\n" REP8("v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %1, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"),
       "+v"(a) : "v"(b), "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(c4), "v"(c5), "v"(c6), "v"(c7));
  // 16: XtY i-outer chain: acc += bcast_i(x_J) * y_J with x_J, y_J different regs (x8)
  {
    double d0 = a + 3, d1 = d0 + 1, d2 = d1 + 1, d3 = d2 + 1;
    TIME("s_nop 4\n" REP8("v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %2, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %3, %7 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %1, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %2, %10 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %3, %11 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                          "v_fmac_f64_dpp %0, %4, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"),
         "+v"(b) : "v"(d0), "v"(d1), "v"(d2), "v"(d3), "v"(c0), "v"(c1), "v"(c2), "v"(c3),
         "v"(c4), "v"(c5), "v"(c6), "v"(c7));
  }
  // 17: two interleaved i-outer chains (acc a, b alternating), y_J different regs
  TIME("s_nop 4\n" REP8("v_fmac_f64_dpp %0, %2, %3 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %1, %2, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %2, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %1, %2, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %2, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %1, %2, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %0, %2, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
                        "v_fmac_f64_dpp %1, %2, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"),
       "+v"(a), "+v"(b) : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(c4), "v"(c5), "v"(c6), "v"(c7), "v"(seed));
  // 18: rcp -> dependent fma latency: (rcp, fma) pairs x 32
  TIME(REP8("v_rcp_f64 %1, %0\nv_fma_f64 %0, %1, %2, %2\nv_rcp_f64 %1, %0\nv_fma_f64 %0, %1, %2, %2\n"
            "v_rcp_f64 %1, %0\nv_fma_f64 %0, %1, %2, %2\nv_rcp_f64 %1, %0\nv_fma_f64 %0, %1, %2, %2\n"),
       "+v"(a), "=&v"(c0) : "v"(b));
  // 19: dependent v_fma_f64 chain where every fma reads 3 distinct regs (acc forwarded)
  TIME(REP8("v_fma_f64 %0, %1, %2, %0\nv_fma_f64 %0, %3, %4, %0\nv_fma_f64 %0, %5, %6, %0\n"
            "v_fma_f64 %0, %7, %8, %0\nv_fma_f64 %0, %1, %3, %0\nv_fma_f64 %0, %5, %7, %0\n"
            "v_fma_f64 %0, %2, %4, %0\nv_fma_f64 %0, %6, %8, %0\n"),
       "+v"(a) : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(c4), "v"(c5), "v"(c6), "v"(c7));

  // 20..23: independent add / mul / min / mov_b64 (8 x 8)
#define IND8(OP) REP8(OP " %0, %8, %9\n" OP " %1, %8, %9\n" OP " %2, %8, %9\n" OP " %3, %8, %9\n" \
                      OP " %4, %8, %9\n" OP " %5, %8, %9\n" OP " %6, %8, %9\n" OP " %7, %8, %9\n")
  TIME(IND8("v_add_f64"), "=v"(c0), "=v"(c1), "=v"(c2), "=v"(c3), "=v"(c4), "=v"(c5), "=v"(c6), "=v"(c7) : "v"(a), "v"(b));
  TIME(IND8("v_mul_f64"), "=v"(c0), "=v"(c1), "=v"(c2), "=v"(c3), "=v"(c4), "=v"(c5), "=v"(c6), "=v"(c7) : "v"(a), "v"(b));
  TIME(IND8("v_min_f64"), "=v"(c0), "=v"(c1), "=v"(c2), "=v"(c3), "=v"(c4), "=v"(c5), "=v"(c6), "=v"(c7) : "v"(a), "v"(b));
  TIME(REP8("v_mov_b64 %0, 1.0\nv_mov_b64 %1, 1.0\nv_mov_b64 %2, 1.0\nv_mov_b64 %3, 1.0\n"
            "v_mov_b64 %4, 1.0\nv_mov_b64 %5, 1.0\nv_mov_b64 %6, 1.0\nv_mov_b64 %7, 1.0\n"),
       "=v"(c0), "=v"(c1), "=v"(c2), "=v"(c3), "=v"(c4), "=v"(c5), "=v"(c6), "=v"(c7));
  // 24: independent v_fma_f64 with 2 distinct sources + own acc (GEMM-like, non-DPP)
  TIME(REP8("v_fma_f64 %0, %8, %9, %0\nv_fma_f64 %1, %8, %9, %1\nv_fma_f64 %2, %8, %9, %2\n"
            "v_fma_f64 %3, %8, %9, %3\nv_fma_f64 %4, %8, %9, %4\nv_fma_f64 %5, %8, %9, %5\n"
            "v_fma_f64 %6, %8, %9, %6\nv_fma_f64 %7, %8, %9, %7\n"),
       "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) : "v"(a), "v"(b));
  if (threadIdx.x == 0) out[63] = (long long)(a + b + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7);
}

int main() {
  long long* d;
  hipMalloc(&d, 64 * sizeof(long long));
  long long h[64];
  const char* names[] = {"empty",       "fma_f64 dep x64",  "fma_f64 indep x64", "fmac_dpp indep x64",
                         "rcp_f64 dep x64", "rcp_f64 indep x64", "add_f64 dep x64",
                         "movdpp+add dep x64 pairs", "cndmask_b32 x64", "fmac_dpp dep x64",
                         "cmp_f64+s_and x64", "s_nop0 x64", "mul_f64 dep x64", "ds_read_b64 x64",
                         "sweep-pattern dpp x64", "XY i-outer dep chain x64", "XtY i-outer dep chain x64",
                         "2 interleaved chains x64", "rcp->fma pairs x32 (per pair/2)", "fma dep 3-reg x64",
                         "add_f64 indep x64", "mul_f64 indep x64", "min_f64 indep x64", "mov_b64 imm x64",
                         "fma_f64 indep (repeat)"};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, 1.0000001);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  }
  for (int i = 0; i < 25; ++i)
    printf("%-28s %6lld ticks  -> %.2f per instr (minus empty)\n", names[i], h[i],
           (double)(h[i] - h[0]) / 64.0);
  return 0;
}
