// Micro-benchmark: fp64 VALU issue with one vs two waves per SIMD.
// A workgroup of 256 threads puts one wave on each SIMD of a CU, 512 threads two.
// Every wave runs the same stream (independent v_fmac_f64_dpp row_newbcast, the
// LFT kernels' form, or plain v_fma_f64); s_memtime per wave around it.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_2wave.hip -o /tmp/ub2 && /tmp/ub2
#include <hip/hip_runtime.h>
#include <stdio.h>

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
#define FMA8                                                                  \
  "v_fma_f64 %0, %8, %9, %0\nv_fma_f64 %1, %8, %9, %1\nv_fma_f64 %2, %8, %9, %2\n" \
  "v_fma_f64 %3, %8, %9, %3\nv_fma_f64 %4, %8, %9, %4\nv_fma_f64 %5, %8, %9, %5\n" \
  "v_fma_f64 %6, %8, %9, %6\nv_fma_f64 %7, %8, %9, %7\n"

template <int MODE>
__global__ void ub(long long* out, double seed) {
  double c0 = seed + 1, c1 = c0 + 1, c2 = c1 + 1, c3 = c2 + 1, c4 = c3 + 1, c5 = c4 + 1,
         c6 = c5 + 1, c7 = c6 + 1, x = seed * 0.5, y = seed * 0.25;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 8; ++it) {
    if constexpr (MODE == 0)
      asm volatile("s_nop 4\n" REP16(REP2(DPP8))
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                   : "v"(x), "v"(y));
    else
      asm volatile(REP16(REP2(FMA8))
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                   : "v"(x), "v"(y));
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
  if (threadIdx.x == 1) out[1023] = (long long)(c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7);
}

int main() {
  long long* d;
  (void)hipMalloc(&d, 1024 * sizeof(long long));
  long long h[1024];
  const char* nm[2] = {"fmac_f64_dpp", "fma_f64"};
  for (int mode = 0; mode < 2; ++mode)
    for (int thr : {256, 512}) {
      for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(ub<0>, dim3(1), dim3(thr), 0, 0, d, 1.0000001);
        else hipLaunchKernelGGL(ub<1>, dim3(1), dim3(thr), 0, 0, d, 1.0000001);
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      }
      long long mx = 0;
      for (int w = 0; w < thr / 64; ++w) mx = h[w] > mx ? h[w] : mx;
      printf("%-14s %3d threads (%d wave/SIMD): max wave %lld ticks for 2048 instr -> %.2f per instr per wave, %.2f per SIMD-instr\n",
             nm[mode], thr, thr / 256, mx, mx / 2048.0, mx / 2048.0 / (thr / 256));
    }
  return 0;
}
