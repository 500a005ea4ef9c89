// Cycles of the generated sweep / elimination / product blocks in isolation
// (one wave; s_memtime around REPS calls of each block on register data).
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -I time_opt_ilqr_amd/csrc tools/ubench_sweep.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "hop_device.hpp"

using namespace hop;
constexpr int S = 13, REPS = 64;

__global__ void ub(long long* out, const double* seed) {
  const int c = threadIdx.x & 15;
  double r[S], q[S], x[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    r[i] = seed[i] + (i == c ? 4.0 : 0.0);
    q[i] = seed[i] * 0.5 + (i == c ? 3.0 : 0.0);
    x[i] = seed[i] * 0.25 + (i == c ? 2.0 : 0.0);
  }
  long long t0, t1;
  int k = 0;
  double dmin = 1.0, dmin2 = 1.0, acc = 0.0;
#define TIME(body)                                \
  __builtin_amdgcn_s_waitcnt(0);                  \
  t0 = __builtin_amdgcn_s_memtime();              \
  for (int it = 0; it < REPS; ++it) { body; }     \
  t1 = __builtin_amdgcn_s_memtime();              \
  if (threadIdx.x == 0) out[k] = (t1 - t0);       \
  ++k;
  TIME(SweepQ<S>::run(r, dmin));                                   // 0: one sweep
  TIME(SweepQ<S>::run(r, dmin); SweepQ<S>::run(q, dmin2));        // 1: two sweeps, sequential
  TIME(ElimQ<S>::run(x, acc, dmin2, 1e-9));                       // 2: bordered elimination
  TIME(SweepElimQ<S>::run(r, dmin, x, acc, dmin2, 1e-9));         // 3: sweep + elim merged
  TIME({                                                           // 4: X*Y product, row chains
    static_for<S>([&](auto I) { LaneDot<S>::fmaq(q[I], r[I], x); });
  });
  TIME({                                                           // 5: X^T*Y product (LaneB)
    static_for<S>([&](auto J) { LaneB<S>::fma(q, r[J], x[J]); });
  });
  if (threadIdx.x == 0) out[15] = (long long)(r[0] + q[0] + x[0] + acc + dmin + dmin2);
}

int main() {
  long long* d;
  double* sd;
  (void)hipMalloc(&d, 16 * sizeof(long long));
  (void)hipMalloc(&sd, 16 * sizeof(double));
  double hs[16];
  for (int i = 0; i < 16; ++i) hs[i] = 0.01 * (i + 1);
  (void)hipMemcpy(sd, hs, sizeof(hs), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, sd);
  hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, sd);
  long long h[16];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  // s_memtime ticks at 100 MHz; the shader clock is ~2.4 GHz: report ticks and
  // an estimate of shader cycles per block call
  const char* names[] = {"SweepQ<13>", "2 x SweepQ<13> sequential", "ElimQ<13>",
                         "SweepElimQ<13> (merged)", "X*Y product (13 row chains)",
                         "X^T*Y product (LaneB)"};
  const int instrs[] = {261, 522, 184, 445, 169, 169};
  for (int i = 0; i < 6; ++i) {
    const double per = (double)h[i] / REPS;
    printf("%-32s %8.2f ticks/call  (%d instrs)\n", names[i], per, instrs[i]);
  }
  return 0;
}
