// Micro-benchmark: does an fp64 MFMA stream in one wave overlap an fp64 DPP-FMA
// stream in ANOTHER wave on the same SIMD (gfx950)?  (tools/ubench_mfma64.hip
// answers the one-wave, interleaved case: no.)
// One workgroup of 512 threads = 8 waves, two per SIMD (wave w on SIMD w % 4).
// Waves 0..3 ("M") run 32 independent v_mfma_f64_16x16x4_f64 (4 accumulators);
// waves 4..7 ("D") run 384 independent v_fmac_f64_dpp row_newbcast (8 chains,
// the LFT/Riccati product form).  Modes: 0 = M waves only, 1 = D waves only,
// 2 = both at once.  Every wave stamps s_memtime around its stream after a
// workgroup barrier; the span per SIMD pair is max(end) - min(start).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma2w.hip -o /tmp/ub2m && /tmp/ub2m
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

#define REP2(x) x x
#define REP4(x) REP2(x) REP2(x)
#define REP8(x) REP4(x) REP4(x)
#define REP16(x) REP8(x) REP8(x)
#define DPP8                                                                  \
  "v_fmac_f64_dpp %0, %0, %8 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %1, %1, %8 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %2, %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %3, %3, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %4, %4, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %5, %5, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %6, %6, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"     \
  "v_fmac_f64_dpp %7, %7, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
#define M16(acc) "v_mfma_f64_16x16x4_f64 " acc ", %4, %5, " acc "\n"
#define MROT16 M16("%0") M16("%1") M16("%2") M16("%3")

template <int MODE>
__global__ __launch_bounds__(512) void ub(long long* out, double seed) {
  const int w = threadIdx.x >> 6;
  const bool mw = w < 4;
  const bool run = MODE == 2 || (MODE == 0 && mw) || (MODE == 1 && !mw);
  d4 a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3;
  double c0 = seed + 1, c1 = c0 + 1, c2 = c1 + 1, c3 = c2 + 1, c4 = c3 + 1, c5 = c4 + 1,
         c6 = c5 + 1, c7 = c6 + 1, x = seed * 0.5;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (run) {
    if (mw) {
      asm volatile(REP8(MROT16) "s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
                   : "v"(x), "v"(x));
    } else {
      asm volatile("s_nop 4\n" REP16(REP2(DPP8)) REP8(DPP8)
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                   : "v"(x));
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    out[2 * w] = t0;
    out[2 * w + 1] = t1;
  }
  if (threadIdx.x == 0)
    out[31] = (long long)(a0.x + a1.y + a2.z + a3.w + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7);
}

int main() {
  long long* d;
  hipMalloc(&d, 32 * sizeof(long long));
  long long h[32];
  const char* names[] = {"M waves alone (32 mfma16x16x4 f64 each)",
                         "D waves alone (384 dpp fma f64 each)", "M and D waves together"};
  for (int mode = 0; mode < 3; ++mode) {
    double best[4] = {1e30, 1e30, 1e30, 1e30}, mdur = 1e30, ddur = 1e30;
    for (int rep = 0; rep < 5; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(ub<0>, dim3(1), dim3(512), 0, 0, d, 1.0000001);
      if (mode == 1) hipLaunchKernelGGL(ub<1>, dim3(1), dim3(512), 0, 0, d, 1.0000001);
      if (mode == 2) hipLaunchKernelGGL(ub<2>, dim3(1), dim3(512), 0, 0, d, 1.0000001);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      for (int s = 0; s < 4; ++s) {  // SIMD s: waves s (M) and s + 4 (D)
        const long long st = h[2 * s] < h[2 * (s + 4)] ? h[2 * s] : h[2 * (s + 4)];
        const long long en = h[2 * s + 1] > h[2 * (s + 4) + 1] ? h[2 * s + 1] : h[2 * (s + 4) + 1];
        if (en - st < best[s]) best[s] = (double)(en - st);
      }
      double m = 0, dd = 0;
      for (int s = 0; s < 4; ++s) {
        m += (double)(h[2 * s + 1] - h[2 * s]) / 4;
        dd += (double)(h[2 * (s + 4) + 1] - h[2 * (s + 4)]) / 4;
      }
      if (m < mdur) mdur = m;
      if (dd < ddur) ddur = dd;
    }
    printf("%-42s span per SIMD %6.0f %6.0f %6.0f %6.0f ticks; M wave %6.0f, D wave %6.0f\n",
           names[mode], best[0], best[1], best[2], best[3], mdur, ddur);
  }
  return 0;
}
