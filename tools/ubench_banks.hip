// Micro-benchmark: does VGPR bank placement decide the cost of a DPP fp64 FMA?
// Explicit physical registers (clobbered), LaneB pattern: 8 accumulators, the
// same DPP source and multiplier.  v[2k:2k+1] occupies banks (2k%4, 2k%4+1).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_banks.hip -o tools/ubench_banks.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(x) x x x x x x x x
#define DPP " row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
#define CLOB                                                                                    \
  "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", \
      "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27",  \
      "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40",  \
      "v41", "v42", "v43"

__global__ void ub(long long* out) {
  long long t0, t1;
  int k = 0;
#define TIME(body)                                  \
  __builtin_amdgcn_s_waitcnt(0);                    \
  t0 = __builtin_amdgcn_s_memtime();                \
  asm volatile(body ::: CLOB);                      \
  t1 = __builtin_amdgcn_s_memtime();                \
  if (threadIdx.x == 0) out[k] = t1 - t0;           \
  ++k;
  asm volatile("v_mov_b32 v0, 0\nv_mov_b32 v1, 0x3ff00000\nv_mov_b32 v2, 0\nv_mov_b32 v3, 0x3ff00000\nv_mov_b32 v4, 0\nv_mov_b32 v5, 0x3ff00000\nv_mov_b32 v6, 0\nv_mov_b32 v7, 0x3ff00000\nv_mov_b32 v8, 0\nv_mov_b32 v9, 0x3ff00000\nv_mov_b32 v10, 0\nv_mov_b32 v11, 0x3ff00000\nv_mov_b32 v12, 0\nv_mov_b32 v13, 0x3ff00000\nv_mov_b32 v14, 0\nv_mov_b32 v15, 0x3ff00000\nv_mov_b32 v16, 0\nv_mov_b32 v17, 0x3ff00000\nv_mov_b32 v18, 0\nv_mov_b32 v19, 0x3ff00000\nv_mov_b32 v20, 0\nv_mov_b32 v21, 0x3ff00000\nv_mov_b32 v22, 0\nv_mov_b32 v23, 0x3ff00000\nv_mov_b32 v24, 0\nv_mov_b32 v25, 0x3ff00000\nv_mov_b32 v26, 0\nv_mov_b32 v27, 0x3ff00000\nv_mov_b32 v28, 0\nv_mov_b32 v29, 0x3ff00000\nv_mov_b32 v30, 0\nv_mov_b32 v31, 0x3ff00000\nv_mov_b32 v32, 0\nv_mov_b32 v33, 0x3ff00000\nv_mov_b32 v34, 0\nv_mov_b32 v35, 0x3ff00000\nv_mov_b32 v36, 0\nv_mov_b32 v37, 0x3ff00000\nv_mov_b32 v38, 0\nv_mov_b32 v39, 0x3ff00000\nv_mov_b32 v40, 0\nv_mov_b32 v41, 0x3ff00000\nv_mov_b32 v42, 0\nv_mov_b32 v43, 0x3ff00000\n" ::: CLOB);
  TIME("s_nop 0");
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[4:5], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[8:9], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[12:13], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[16:17], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[20:21], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[24:25], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[28:29], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[4:5], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[8:9], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[12:13], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[16:17], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[20:21], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[24:25], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[28:29], v[32:33], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[4:5], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[8:9], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[12:13], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[16:17], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[20:21], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[24:25], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[28:29], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[4:5], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[8:9], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[12:13], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[16:17], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[20:21], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[24:25], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[28:29], v[34:35], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[6:7], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[10:11], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[14:15], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[18:19], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[22:23], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[26:27], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[30:31], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[6:7], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[10:11], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[14:15], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[18:19], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[22:23], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[26:27], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[30:31], v[32:33], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[6:7], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[10:11], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[14:15], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[18:19], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[22:23], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[26:27], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[30:31], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[6:7], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[10:11], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[14:15], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[18:19], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[22:23], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[26:27], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[30:31], v[34:35], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP ));
}

__global__ void ub2(long long* out) {
  long long t0, t1;
  int k = 0;
#define TIME(body)                                  \
  __builtin_amdgcn_s_waitcnt(0);                    \
  t0 = __builtin_amdgcn_s_memtime();                \
  asm volatile(body ::: CLOB);                      \
  t1 = __builtin_amdgcn_s_memtime();                \
  if (threadIdx.x == 0) out[k] = t1 - t0;           \
  ++k;
  asm volatile("v_mov_b32 v0, 0\nv_mov_b32 v1, 0x3ff00000\nv_mov_b32 v2, 0\nv_mov_b32 v3, 0x3ff00000\nv_mov_b32 v4, 0\nv_mov_b32 v5, 0x3ff00000\nv_mov_b32 v6, 0\nv_mov_b32 v7, 0x3ff00000\nv_mov_b32 v8, 0\nv_mov_b32 v9, 0x3ff00000\nv_mov_b32 v10, 0\nv_mov_b32 v11, 0x3ff00000\nv_mov_b32 v12, 0\nv_mov_b32 v13, 0x3ff00000\nv_mov_b32 v14, 0\nv_mov_b32 v15, 0x3ff00000\nv_mov_b32 v16, 0\nv_mov_b32 v17, 0x3ff00000\nv_mov_b32 v18, 0\nv_mov_b32 v19, 0x3ff00000\nv_mov_b32 v20, 0\nv_mov_b32 v21, 0x3ff00000\nv_mov_b32 v22, 0\nv_mov_b32 v23, 0x3ff00000\nv_mov_b32 v24, 0\nv_mov_b32 v25, 0x3ff00000\nv_mov_b32 v26, 0\nv_mov_b32 v27, 0x3ff00000\nv_mov_b32 v28, 0\nv_mov_b32 v29, 0x3ff00000\nv_mov_b32 v30, 0\nv_mov_b32 v31, 0x3ff00000\nv_mov_b32 v32, 0\nv_mov_b32 v33, 0x3ff00000\nv_mov_b32 v34, 0\nv_mov_b32 v35, 0x3ff00000\nv_mov_b32 v36, 0\nv_mov_b32 v37, 0x3ff00000\nv_mov_b32 v38, 0\nv_mov_b32 v39, 0x3ff00000\nv_mov_b32 v40, 0\nv_mov_b32 v41, 0x3ff00000\nv_mov_b32 v42, 0\nv_mov_b32 v43, 0x3ff00000\n" ::: CLOB);
  TIME("s_nop 0");
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[42:43], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[40:41], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[6:7], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[10:11], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[14:15], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[18:19], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[22:23], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[26:27], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[30:31], v[34:35], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[6:7], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[10:11], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[14:15], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[18:19], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[22:23], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[26:27], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[30:31], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[6:7], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[10:11], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[14:15], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[18:19], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[22:23], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[26:27], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[30:31], v[32:33], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[2:3], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[6:7], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[10:11], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[14:15], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[18:19], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[22:23], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[26:27], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[30:31], v[32:33], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[4:5], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[8:9], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[12:13], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[16:17], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[20:21], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[24:25], v[34:35], v[38:39]" DPP "v_fmac_f64_dpp v[28:29], v[34:35], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[4:5], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[8:9], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[12:13], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[16:17], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[20:21], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[24:25], v[34:35], v[36:37]" DPP "v_fmac_f64_dpp v[28:29], v[34:35], v[36:37]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[4:5], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[8:9], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[12:13], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[16:17], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[20:21], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[24:25], v[32:33], v[38:39]" DPP "v_fmac_f64_dpp v[28:29], v[32:33], v[38:39]" DPP ));
  TIME("s_nop 4\n" R8("v_fmac_f64_dpp v[0:1], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[4:5], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[8:9], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[12:13], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[16:17], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[20:21], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[24:25], v[32:33], v[36:37]" DPP "v_fmac_f64_dpp v[28:29], v[32:33], v[36:37]" DPP ));
}

int main() {
  long long* d;
  (void)hipMalloc(&d, 64 * sizeof(long long));
  long long h[64];
  const char* names[] = {"empty",
"acc{0,1} x{0,1} y{0,1}",
"acc{0,1} x{0,1} y{2,3}",
"acc{0,1} x{2,3} y{0,1}",
"acc{0,1} x{2,3} y{2,3}",
"acc{2,3} x{0,1} y{0,1}",
"acc{2,3} x{0,1} y{2,3}",
"acc{2,3} x{2,3} y{0,1}",
"acc{2,3} x{2,3} y{2,3}",
"chain acc{0,1} x{0,1} y{0,1}",
"chain acc{0,1} x{2,3} y{0,1}",
"chain acc{2,3} x{0,1} y{0,1}",
"chain acc{2,3} x{2,3} y{0,1}"};
  const int n = 13;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(ub, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  }
  for (int i = 0; i < n; ++i)
    printf("%-40s %6lld ticks -> %.2f per instr\n", names[i], h[i], (double)(h[i] - h[0]) / 64.0);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(ub2, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  }
  printf("reversed order:\n");
  for (int i = 0; i < n; ++i) {
    const int j = i == 0 ? 0 : n - i;  // case i ran at position j
    printf("%-40s %6lld ticks -> %.2f per instr\n", names[i], h[j], (double)(h[j] - h[0]) / 64.0);
  }
  return 0;
}
