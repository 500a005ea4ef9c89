// Where does buffer_load_dwordx4 ... offen offset:N lds put its data, and from where
// does it read?  (LDS-DMA addressing with an instruction offset, gfx950.)  One wave:
// global src[i] = i (floats); LDS cleared to -1; M0 = 0; each lane's voffset =
// lane * 16 + vbias; then one load with offset:1024.  The LDS image is copied out.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(const float* src, int nrec_bytes, int vbias, float* out) {
  __shared__ float lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = -1.0f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0,
                                                               nrec_bytes, 0x00020000);
  unsigned voff = threadIdx.x * 16u + (unsigned)vbias;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen offset:1024 lds\n\t"
      "s_waitcnt vmcnt(0)\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds))
      : "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 4096; i += 64) out[i] = lds[i];
}

int main() {
  const int n = 1 << 16;
  float* h = new float[n];
  for (int i = 0; i < n; ++i) h[i] = (float)i;
  float *d, *o;
  hipMalloc(&d, n * 4);
  hipMalloc(&o, 4096 * 4);
  hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
  float res[4096];
  const int biases[3] = {0, 4096, -1024};  // -1024: the wrapped voffset (+ offset:1024 = lane*16)
  for (int b = 0; b < 3; ++b) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, n * 4, biases[b], o);
    hipMemcpy(res, o, sizeof(res), hipMemcpyDeviceToHost);
    int first = -1, last = -1;
    for (int i = 0; i < 4096; ++i)
      if (res[i] != -1.0f) { if (first < 0) first = i; last = i; }
    printf("vbias %6d: LDS floats written [%d, %d]; lds[first] = %g (global float index), lds[first+4] = %g, lds[last] = %g\n",
           biases[b], first, last, first >= 0 ? res[first] : -1.0, first >= 0 ? res[first + 4] : -1.0,
           last >= 0 ? res[last] : -1.0);
  }
  hipFree(d);
  hipFree(o);
  return 0;
}
