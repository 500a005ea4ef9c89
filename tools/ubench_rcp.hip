// Accuracy of v_rcp_f64 (no Newton step) vs IEEE 1/d over a sweep of inputs:
// prints the max relative error and max ulp distance.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__global__ void k(const double* in, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_rcp(in[i]);
}

int main() {
  const int n = 1 << 22;
  double* h = (double*)malloc(n * sizeof(double));
  double* r = (double*)malloc(n * sizeof(double));
  srand(7);
  for (int i = 0; i < n; ++i) {
    double m = 1.0 + (double)rand() / RAND_MAX;                 // mantissa in [1, 2)
    int e = (rand() % 60) - 30;
    h[i] = ldexp(m, e) * ((rand() & 1) ? 1.0 : -1.0);
  }
  double *di, *dout;
  hipMalloc(&di, n * sizeof(double));
  hipMalloc(&dout, n * sizeof(double));
  hipMemcpy(di, h, n * sizeof(double), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, di, dout, n);
  hipMemcpy(r, dout, n * sizeof(double), hipMemcpyDeviceToHost);
  double maxrel = 0;
  long long maxulp = 0;
  for (int i = 0; i < n; ++i) {
    const double ref = 1.0 / h[i];
    const double rel = fabs(r[i] - ref) / fabs(ref);
    if (rel > maxrel) maxrel = rel;
    long long a, b;
    memcpy(&a, &r[i], 8);
    memcpy(&b, &ref, 8);
    long long u = a > b ? a - b : b - a;
    if (u > maxulp) maxulp = u;
  }
  printf("v_rcp_f64: max rel err %.3e, max ulp %lld over %d inputs\n", maxrel, maxulp, n);
  return 0;
}
