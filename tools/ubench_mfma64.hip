// Micro-benchmark: does the fp64 matrix pipe run beside the fp64 VALU on gfx950?
// One wave, s_memtime around unrolled asm: v_mfma_f64_16x16x4_f64 and
// v_mfma_f64_4x4x4_4b_f64 issue rates alone, v_fmac_f64_dpp (the LFT sweep's
// product form) alone, and the two interleaved in one stream.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma64.hip -o /tmp/ubm && /tmp/ubm
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

#define REP2(x) x x
#define REP4(x) REP2(x) REP2(x)
#define REP8(x) REP4(x) REP4(x)
#define REP16(x) REP8(x) REP8(x)

// 8 independent DPP FMAs (the sweep's pattern: acc is also the multiplicand)
#define DPP8                                                                   \
  "v_fmac_f64_dpp %4, %4, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %5, %5, %16 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %6, %6, %16 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %7, %7, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %8, %8, %16 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %9, %9, %16 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %10, %10, %16 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"   \
  "v_fmac_f64_dpp %11, %11, %16 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
#define DPP4                                                                   \
  "v_fmac_f64_dpp %4, %4, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %5, %5, %16 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %6, %6, %16 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %7, %7, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
#define M16(acc) "v_mfma_f64_16x16x4_f64 " acc ", %17, %18, " acc "\n"
#define M4(acc) "v_mfma_f64_4x4x4_4b_f64 " acc ", %17, %18, " acc "\n"
#define MROT16 M16("%0") M16("%1") M16("%2") M16("%3")

__global__ void ub(long long* out, double seed) {
  d4 a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3;
  double c0 = seed + 1, c1 = c0 + 1, c2 = c1 + 1, c3 = c2 + 1, c4 = c3 + 1, c5 = c4 + 1,
         c6 = c5 + 1, c7 = c6 + 1;
  double x = seed * 0.5, y = seed * 0.25;
  double e0 = seed, e1 = seed + 1, e2 = seed + 2, e3 = seed + 3;
  long long t0, t1;
  int k = 0;
#define TIME(body)                                                            \
  __builtin_amdgcn_s_waitcnt(0);                                             \
  asm volatile("s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7" ::: "memory");            \
  t0 = __builtin_amdgcn_s_memtime();                                         \
  asm volatile(body "s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\n"  \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2),      \
                 "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7), "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3) \
               : "v"(x), "v"(x), "v"(y));                                   \
  t1 = __builtin_amdgcn_s_memtime();                                         \
  if (threadIdx.x == 0) out[k] = t1 - t0;                                    \
  ++k;
  TIME("")                                       // 0 empty (incl. 8 trailing nops)
  TIME(REP4(MROT16))                             // 1 16 MFMA16, 4 accs
  TIME(REP16(M16("%0")))                         // 2 16 MFMA16 dependent
  TIME("s_nop 4\n" REP8(DPP8))                   // 3 64 DPP
  TIME("s_nop 4\n" REP16(DPP8))                  // 4 128 DPP
  TIME("s_nop 4\n" REP16(DPP8 DPP4))             // 5 192 DPP
  TIME(REP4(M16("%0") DPP4 M16("%1") DPP4 M16("%2") DPP4 M16("%3") DPP4))  // 6 16 MFMA + 64 DPP
  TIME(REP4(M16("%0") DPP8 M16("%1") DPP8 M16("%2") DPP8 M16("%3") DPP8))  // 7 16 MFMA + 128 DPP
  TIME(REP4(M16("%0") DPP8 DPP4 M16("%1") DPP8 DPP4 M16("%2") DPP8 DPP4 M16("%3") DPP8 DPP4))  // 8 +192
  TIME(REP16(M4("%12") M4("%13") M4("%14") M4("%15")))  // 9 64 MFMA4x4 (4b), 4 accs
  TIME(REP16(M4("%12") DPP4 M4("%13") DPP4 M4("%14") DPP4 M4("%15") DPP4))  // 10 64 MFMA4 + 256 DPP
  TIME(REP16(M4("%12") DPP4 M4("%13") DPP4))  // 11 32 MFMA4 + 128 DPP
  TIME("s_nop 4\n" REP16(DPP8 DPP8))             // 12 256 DPP
  if (threadIdx.x == 0)
    out[63] = (long long)(a0.x + a1.y + a2.z + a3.w + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 +
                          e0 + e1 + e2 + e3);
}

int main() {
  long long* d;
  hipMalloc(&d, 64 * sizeof(long long));
  long long h[64];
  const char* names[] = {"empty", "mfma16x16x4 indep x16", "mfma16x16x4 dep x16", "dpp x64",
                         "dpp x128", "dpp x192", "16 mfma16 + 64 dpp", "16 mfma16 + 128 dpp",
                         "16 mfma16 + 192 dpp", "mfma4x4x4_4b indep x64", "64 mfma4 + 256 dpp",
                         "32 mfma4 + 128 dpp", "dpp x256"};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, 1.0000001);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  }
  for (int i = 0; i < 13; ++i)
    printf("%-26s %6lld ticks (minus empty: %lld)\n", names[i], h[i], h[i] - h[0]);
  return 0;
}
