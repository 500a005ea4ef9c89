// Micro-benchmark: does a wave whose EXEC covers only part of its 64 lanes issue
// fp64 / fp32 VALU faster?  (The line search runs 24,576 lanes = 384 full waves on
// 1,024 SIMDs; if a half-empty wave issued in half the cycles, spreading the lanes
// over more, partly filled waves would shorten the per-wave stream.)  One wave,
// s_memtime around 64 independent FMAs, EXEC = lanes [0, active).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_exec.hip -o /tmp/ubx && /tmp/ubx
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x

__global__ void ub(long long* out, double seed, int active) {
  const int lane = threadIdx.x;
  double c0 = seed + 1, c1 = c0 + 1, c2 = c1 + 1, c3 = c2 + 1, c4 = c3 + 1, c5 = c4 + 1,
         c6 = c5 + 1, c7 = c6 + 1, a = seed, b = seed * 0.5;
  float f0 = c0, f1 = c1, f2 = c2, f3 = c3, f4 = c4, f5 = c5, f6 = c6, f7 = c7, fa = a, fb = b;
  long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
  if (lane < active) {
    __builtin_amdgcn_s_waitcnt(0);
    t0 = __builtin_amdgcn_s_memtime();
    asm volatile(REP8(REP8("v_fma_f64 %0, %8, %9, %0\nv_fma_f64 %1, %8, %9, %1\nv_fma_f64 %2, %8, %9, %2\n"
                           "v_fma_f64 %3, %8, %9, %3\nv_fma_f64 %4, %8, %9, %4\nv_fma_f64 %5, %8, %9, %5\n"
                           "v_fma_f64 %6, %8, %9, %6\nv_fma_f64 %7, %8, %9, %7\n"))
                 : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                 : "v"(a), "v"(b));
    t1 = __builtin_amdgcn_s_memtime();
    asm volatile(REP8(REP8("v_fma_f32 %0, %8, %9, %0\nv_fma_f32 %1, %8, %9, %1\nv_fma_f32 %2, %8, %9, %2\n"
                           "v_fma_f32 %3, %8, %9, %3\nv_fma_f32 %4, %8, %9, %4\nv_fma_f32 %5, %8, %9, %5\n"
                           "v_fma_f32 %6, %8, %9, %6\nv_fma_f32 %7, %8, %9, %7\n"))
                 : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                 : "v"(fa), "v"(fb));
    t2 = __builtin_amdgcn_s_memtime();
    // dependent v_fma_f64 chain (512)
    asm volatile(REP8(REP8(REP8("v_fma_f64 %0, %0, %1, %1\n"))) : "+v"(a) : "v"(b));
    t3 = __builtin_amdgcn_s_memtime();
    // independent v_mul_f64 + v_add_f64 pairs (the libm polynomial shape)
    asm volatile(REP8(REP8("v_mul_f64 %0, %0, %8\nv_add_f64 %1, %1, %8\nv_mul_f64 %2, %2, %8\n"
                           "v_add_f64 %3, %3, %8\nv_mul_f64 %4, %4, %8\nv_add_f64 %5, %5, %8\n"
                           "v_mul_f64 %6, %6, %8\nv_add_f64 %7, %7, %8\n"))
                 : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                 : "v"(b));
    t4 = __builtin_amdgcn_s_memtime();
  }
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = t2 - t1;
    out[2] = t3 - t2;
    out[3] = t4 - t3;
  }
  if (lane == 1 && active == 0) out[4] = (long long)(c0 + c7 + f0 + f7 + a);
}

int main() {
  long long* d;
  hipMalloc(&d, 8 * sizeof(long long));
  const int acts[] = {64, 48, 33, 32, 24, 16, 8, 1};
  printf("active  fma_f64(512 indep)  fma_f32(512 indep)  fma_f64(512 dep)  mul/add_f64(512 indep)  [cycles per instruction]\n");
  for (int rep = 0; rep < 2; ++rep)
    for (int act : acts) {
      long long h[8] = {};
      for (int it = 0; it < 3; ++it) {
        hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, 1.0 + 1e-9 * act, act);
        hipMemcpy(h, d, 8 * sizeof(long long), hipMemcpyDeviceToHost);
      }
      if (rep == 1)
        printf("%6d  %8.2f  %8.2f  %8.2f  %8.2f\n", act, h[0] / 512.0, h[1] / 512.0, h[2] / 512.0,
               h[3] / 512.0);
    }
  hipFree(d);
  return 0;
}
