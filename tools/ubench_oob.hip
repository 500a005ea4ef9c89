// Buffer range-check granularity: a buffer_load_dwordx4 straddling num_records.
// Prints which of the 4 dwords come back (per-dword check) or all zero (per-load).
// Out-of-range buffer loads return 0; they never fault.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(const float* src, float* out) {
  // num_records = 20 bytes: dwords 0..4 in range; load 16 bytes at offset 12 -> dwords 3..6
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 20,
                                                               0x00020000);
  float4 v;
  unsigned off = 12;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen\n s_waitcnt vmcnt(0)"
               : "=v"(v) : "v"(off), "s"(r) : "memory");
  if (threadIdx.x == 0) {
    out[0] = v.x;
    out[1] = v.y;
    out[2] = v.z;
    out[3] = v.w;
  }
}

int main() {
  float h[16], *d, *o;
  for (int i = 0; i < 16; ++i) h[i] = 100.0f + i;
  (void)hipMalloc(&d, sizeof(h));
  (void)hipMalloc(&o, 16);
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  float r[4];
  (void)hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
  printf("dwords 3..6 (3,4 in range; 5,6 out): %g %g %g %g  -> %s\n", r[0], r[1], r[2], r[3],
         (r[0] == 103.0f && r[1] == 104.0f) ? "per-dword check" : "whole load dropped");
  return 0;
}
