// Micro-benchmark: does the f32 matrix pipe (v_mfma_f32_16x16x4_f32) run beside
// the fp64 VALU (v_fmac_f64_dpp, the conditioned kernel's product form) on gfx950?
// One wave, s_memtime around unrolled asm: MFMA alone, DPP alone, interleaved.
// (the fp32-block s = 13 kernel of config 5.)
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma32.hip -o /tmp/ubm32 && /tmp/ubm32
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

#define REP2(x) x x
#define REP4(x) REP2(x) REP2(x)
#define REP8(x) REP4(x) REP4(x)
#define REP16(x) REP8(x) REP8(x)

#define DPP8                                                                   \
  "v_fmac_f64_dpp %4, %4, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %5, %5, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %6, %6, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %7, %7, %12 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %8, %8, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %9, %9, %12 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %10, %10, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"   \
  "v_fmac_f64_dpp %11, %11, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
#define DPP4                                                                   \
  "v_fmac_f64_dpp %4, %4, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %5, %5, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %6, %6, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %7, %7, %12 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
#define M16(acc) "v_mfma_f32_16x16x4_f32 " acc ", %13, %14, " acc "\n"
#define MROT16 M16("%0") M16("%1") M16("%2") M16("%3")

__global__ void ub(long long* out, float seed) {
  f4 a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3;
  double c0 = seed + 1, c1 = c0 + 1, c2 = c1 + 1, c3 = c2 + 1, c4 = c3 + 1, c5 = c4 + 1,
         c6 = c5 + 1, c7 = c6 + 1;
  double x = seed * 0.5;
  float fa = seed * 0.25f, fb = seed * 0.125f;
  long long t0, t1;
  int k = 0;
#define TIME(body)                                                            \
  __builtin_amdgcn_s_waitcnt(0);                                             \
  asm volatile("s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7" ::: "memory");            \
  t0 = __builtin_amdgcn_s_memtime();                                         \
  asm volatile(body "s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\n"  \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2),      \
                 "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)                           \
               : "v"(x), "v"(fa), "v"(fb));                                 \
  t1 = __builtin_amdgcn_s_memtime();                                         \
  if (threadIdx.x == 0) out[k] = t1 - t0;                                    \
  ++k;
  TIME("")                                                                     // 0
  TIME(REP4(MROT16))                                                           // 1 16 MFMA, 4 accs
  TIME(REP8(MROT16))                                                           // 2 32 MFMA
  TIME("s_nop 4\n" REP8(DPP8))                                                 // 3 64 DPP
  TIME("s_nop 4\n" REP16(DPP8))                                                // 4 128 DPP
  TIME("s_nop 4\n" REP16(DPP8 DPP8))                                           // 5 256 DPP
  TIME(REP4(M16("%0") DPP4 M16("%1") DPP4 M16("%2") DPP4 M16("%3") DPP4))      // 6 16 + 64
  TIME(REP4(M16("%0") DPP8 M16("%1") DPP8 M16("%2") DPP8 M16("%3") DPP8))      // 7 16 + 128
  TIME(REP8(M16("%0") DPP8 M16("%1") DPP8 M16("%2") DPP8 M16("%3") DPP8))      // 8 32 + 256
  TIME(REP4(M16("%0") DPP8 DPP8 M16("%1") DPP8 DPP8 M16("%2") DPP8 DPP8 M16("%3") DPP8 DPP8))  // 9 16 + 256
  if (threadIdx.x == 0)
    out[63] = (long long)(a0.x + a1.y + a2.z + a3.w + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7);
}

int main() {
  long long* d;
  hipMalloc(&d, 64 * sizeof(long long));
  long long h[64];
  const char* names[] = {"empty", "mfma_f32_16x16x4 x16", "mfma_f32_16x16x4 x32", "dpp f64 x64",
                         "dpp f64 x128", "dpp f64 x256", "16 mfma + 64 dpp", "16 mfma + 128 dpp",
                         "32 mfma + 256 dpp", "16 mfma + 256 dpp"};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, 1.0000001f);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  }
  for (int i = 0; i < 10; ++i)
    printf("%-26s %6lld ticks (minus empty: %lld)\n", names[i], h[i], h[i] - h[0]);
  return 0;
}
