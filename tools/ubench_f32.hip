// Issue cost of fp32 VALU forms vs fp64 at one wave (s_memtime, shader cycles):
// decides whether an fp32 port of the DPP sweep kernel can beat the fp64 one.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_f32.hip -o tools/ubench_f32.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void ub(long long* out, float seed) {
  float c0 = seed, c1 = seed + 1, c2 = seed + 2, c3 = seed + 3, c4 = seed + 4, c5 = seed + 5,
        c6 = seed + 6, c7 = seed + 7, a = seed * 0.5f, b = seed * 0.25f;
  double d0 = c0, d1 = c1, d2 = c2, d3 = c3, d4 = c4, d5 = c5, d6 = c6, d7 = c7, da = a, db = b;
  long long t0, t1;
  int k = 0;
#define TIME(body, ...)                      \
  __builtin_amdgcn_s_waitcnt(0);           \
  t0 = __builtin_amdgcn_s_memtime();       \
  asm volatile(body : __VA_ARGS__);        \
  t1 = __builtin_amdgcn_s_memtime();       \
  if (threadIdx.x == 0) out[k] = t1 - t0;  \
  ++k;
#define F32DPP(i, L) "v_fmac_f32_dpp %" #i ", %8, %9 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
#define F64DPP(i, L) "v_fmac_f64_dpp %" #i ", %8, %9 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
  TIME("s_nop 4\n" REP8(F32DPP(0, 1) F32DPP(1, 2) F32DPP(2, 3) F32DPP(3, 4) F32DPP(4, 5)
                        F32DPP(5, 6) F32DPP(6, 7) F32DPP(7, 8)),
       "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
       : "v"(a), "v"(b));
  TIME(REP8("v_fmac_f32 %0, %8, %9\nv_fmac_f32 %1, %8, %9\nv_fmac_f32 %2, %8, %9\n"
            "v_fmac_f32 %3, %8, %9\nv_fmac_f32 %4, %8, %9\nv_fmac_f32 %5, %8, %9\n"
            "v_fmac_f32 %6, %8, %9\nv_fmac_f32 %7, %8, %9\n"),
       "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
       : "v"(a), "v"(b));
  TIME("s_nop 4\n" REP8(F64DPP(0, 1) F64DPP(1, 2) F64DPP(2, 3) F64DPP(3, 4) F64DPP(4, 5)
                        F64DPP(5, 6) F64DPP(6, 7) F64DPP(7, 8)),
       "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
       : "v"(da), "v"(db));
  TIME(REP64("v_fmac_f32 %0, %1, %2\n"), "+v"(c0) : "v"(a), "v"(b));  // dependent chain
  TIME(REP64("v_rcp_f32 %0, %0\n"), "+v"(c1));
  if (threadIdx.x == 0) out[15] = (long long)(c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
}

int main() {
  long long* d;
  (void)hipMalloc(&d, 16 * sizeof(long long));
  hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, 1.0f);
  hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d, 1.0f);
  long long h[16];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"64 x v_fmac_f32_dpp row_newbcast (8 acc)", "64 x v_fmac_f32 (8 acc)",
                         "64 x v_fmac_f64_dpp row_newbcast (8 acc)", "64 x v_fmac_f32 dependent",
                         "64 x v_rcp_f32 dependent"};
  for (int i = 0; i < 5; ++i) printf("%-44s %6lld cycles = %.2f / instr\n", names[i], h[i], h[i] / 64.0);
  return 0;
}
