// Batched Riccati passes, exact-size fp64 kernel for the Quadrotor shape
// (n = 12, m = 4): the gains at each problem's T* (backward_pass_truncated,
// solver.py:156-230, mode 0) and the value expansions
// (value_expansions_and_gains_prefix, horizon_selection.py:97-212, mode 1).
// Same arithmetic, association and failure semantics as riccati.hip (the
// generic kernel, which keeps every other shape, fp32 and the extra-cost
// terms); built for a wave alone on its SIMD (B = 4096 -> 1024 waves):
//
//  * one problem per 16-lane DPP row; [A_k | B_k] fills all 16 lanes of 12
//    registers (lane c < 12: column c of A_k, lanes 12..15: the columns of B_k),
//    so V [A|B] and [A|B]^T V [A|B] are two full-width products;
//  * step k-1's A_k, B_k, x_k, u_k stream into a per-wave LDS image by LDS-DMA
//    (9 one-KiB pieces per wave-step, bounds-checked buffer descriptors) while
//    step k computes; no VGPR holds prefetch data and no address arithmetic is
//    done per step (loop-invariant per-lane LDS addresses, the two image
//    buffers selected by an immediate offset in a 2-step unrolled loop);
//  * K, k (and Vxx, Vx, V0 in mode 1) leave by buffer stores whose per-step
//    displacement is a scalar offset;
//  * the loop-invariant Q, R columns/rows and the terminal data live in registers.
#include <math.h>

#include "hop_device.hpp"
#include "hop_kernels.hpp"

namespace hop {
namespace ricf {

constexpr int NX = 12, MU = 4;          // n, m
constexpr int CH_A = NX * NX * 8 / 16;  // 72 16-B chunks of A_k per problem
constexpr int CH_B = NX * MU * 8 / 16;  // 24 of B_k
constexpr int CH_X = NX * 8 / 16;       // 6 of x_k
constexpr int CH_U = MU * 8 / 16;       // 2 of u_k
// per-wave image of one step (4 problems): [A 5 KiB][B 2 KiB][x 1 KiB][u 1 KiB]
constexpr int OFF_A = 0, OFF_B = 5 * 1024, OFF_X = 7 * 1024, OFF_U = 8 * 1024;
constexpr int BUF = 9 * 1024;               // second image at +BUF
constexpr int OFF_T = 2 * BUF;              // transpose tiles
constexpr int OFF_Q = OFF_T + kProbPerWave * kLdsTile * 8;  // Q rows: problem g, row r, lane c
constexpr int Q_PROB = NX * 16 * 8;                         // at OFF_Q + 1536 g + 128 r + 8 c
constexpr int WAVE_BYTES = OFF_Q + kProbPerWave * Q_PROB;
// the two-waves-per-SIMD J-curve layout (OCC2): ONE step image (its DMA is issued
// after the step's reads, still one step ahead), the tiles, and one Q image shared by
// the wave's problems (a batch-shared Q): 19,456 B, so two 4-wave workgroups fit a CU
constexpr int OFF_T2 = BUF;
constexpr int OFF_Q2 = OFF_T2 + kProbPerWave * kLdsTile * 8;
constexpr int WAVE_BYTES2 = OFF_Q2 + Q_PROB;
static_assert(2 * kWavesPerBlock * WAVE_BYTES2 <= 160 * 1024, "OCC2 needs two workgroups per CU");

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32x2 as_u2(double v) { return __builtin_bit_cast(u32x2, v); }

// per-lane source offset of piece j (lane q = 64 j + lane carries chunk q % CH of
// problem q / CH of the wave); lanes past the wave's data point out of range
template <int CH>
__device__ __forceinline__ unsigned voff(int j, int lane, long long wave_prob0, long long pb0,
                                         long long batch, long long pstr) {
  const int q = 64 * j + lane;
  const int p = q / CH, r = q % CH;
  const long long pe = wave_prob0 + p < batch ? wave_prob0 + p : batch - 1;
  return (q < kProbPerWave * CH) ? (unsigned)((pe - pb0) * pstr + r * 16) : 0x7FFFFFFFu;
}

// the step's 9 LDS-DMA pieces (A 5, B 2, x, u, contiguous 1-KiB pieces of the image) in
// one asm block: the LDS-DMA instruction offset is added to both the LDS destination
// (M0 + offset + 16 lane) and the memory address (tools/ubench/lds_dma_offset.hip), so
// piece j goes to M0 = IMG + 4096 (j / 4) with offset 1024 (j % 4) and its voffset is
// lowered by that offset once at kernel start (dma9_voff): 3 M0 writes (each with the
// wait state an M0 write needs before an LDS-DMA) instead of 9
static_assert(OFF_B == OFF_A + 5 * 1024 && OFF_X == OFF_A + 7 * 1024 && OFF_U == OFF_A + 8 * 1024,
              "dma9: contiguous 1-KiB pieces");
__device__ __forceinline__ unsigned dma9_voff(unsigned voff, int piece) {
  return voff - 1024u * (unsigned)(piece % 4);
}
template <int IMG>
__device__ __forceinline__ void dma9(const unsigned (&va)[5], const unsigned (&vb)[2], unsigned vx,
                                     unsigned vu, __amdgpu_buffer_rsrc_t rA,
                                     __amdgpu_buffer_rsrc_t rB, __amdgpu_buffer_rsrc_t rX,
                                     __amdgpu_buffer_rsrc_t rU, unsigned wlds, unsigned sA,
                                     unsigned sB, unsigned sX, unsigned sU) {
  unsigned keep;
#define HOP_M0(OFF) "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\t"
#define HOP_PO(R, V, SO, IO) "buffer_load_dwordx4 %[" #V "], %[" #R "], %[" #SO "] offen offset:" #IO " lds\n\t"
  asm volatile(
      HOP_VMNOP
      "s_mov_b32 %[keep], m0\n\t"
      HOP_M0(%[m0]) HOP_PO(ra, a0, sa, 0) HOP_PO(ra, a1, sa, 1024) HOP_PO(ra, a2, sa, 2048)
      HOP_PO(ra, a3, sa, 3072)
      HOP_M0(%[m1]) HOP_PO(ra, a4, sa, 0) HOP_PO(rb, b0, sb, 1024) HOP_PO(rb, b1, sb, 2048)
      HOP_PO(rx, x0, sx, 3072)
      HOP_M0(%[m2]) HOP_PO(ru, x1, su, 0)
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [w] "s"(wlds), [sa] "s"(sA), [sb] "s"(sB), [sx] "s"(sX), [su] "s"(sU),
        [ra] "s"(rA), [rb] "s"(rB), [rx] "s"(rX), [ru] "s"(rU),
        [a0] "v"(va[0]), [a1] "v"(va[1]), [a2] "v"(va[2]), [a3] "v"(va[3]), [a4] "v"(va[4]),
        [b0] "v"(vb[0]), [b1] "v"(vb[1]), [x0] "v"(vx), [x1] "v"(vu),
        [m0] "i"(IMG + OFF_A), [m1] "i"(IMG + OFF_A + 4096), [m2] "i"(IMG + OFF_A + 8192)
      : "memory", "scc");
#undef HOP_PO
#undef HOP_M0
}

// [A|B] rows (12 registers, column c per lane), x_c and u_c from image IMG, and
// (VT) the transpose of the previous step's value update parked in the tile:
// every read in flight, one wait, one asm statement (early-clobber outputs)
template <int IMG>
__device__ __forceinline__ void read_step(const unsigned (&ad)[NX], unsigned xa, unsigned ua,
                                          double (&ab)[NX], double& x, double& u) {
  asm volatile(
      "ds_read_b64 %0, %14 offset:%c28\n\t"
      "ds_read_b64 %1, %15 offset:%c28\n\t"
      "ds_read_b64 %2, %16 offset:%c28\n\t"
      "ds_read_b64 %3, %17 offset:%c28\n\t"
      "ds_read_b64 %4, %18 offset:%c28\n\t"
      "ds_read_b64 %5, %19 offset:%c28\n\t"
      "ds_read_b64 %6, %20 offset:%c28\n\t"
      "ds_read_b64 %7, %21 offset:%c28\n\t"
      "ds_read_b64 %8, %22 offset:%c28\n\t"
      "ds_read_b64 %9, %23 offset:%c28\n\t"
      "ds_read_b64 %10, %24 offset:%c28\n\t"
      "ds_read_b64 %11, %25 offset:%c28\n\t"
      "ds_read_b64 %12, %26 offset:%c28\n\t"
      "ds_read_b64 %13, %27 offset:%c28\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(ab[0]), "=&v"(ab[1]), "=&v"(ab[2]), "=&v"(ab[3]), "=&v"(ab[4]), "=&v"(ab[5]),
        "=&v"(ab[6]), "=&v"(ab[7]), "=&v"(ab[8]), "=&v"(ab[9]), "=&v"(ab[10]), "=&v"(ab[11]),
        "=&v"(x), "=&v"(u)
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]),
        "v"(ad[7]), "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(xa), "v"(ua),
        "i"(IMG)
      : "memory");
}
// ... and (Q) the step's Qxx accumulator start, Q row r on lane c, from the Q image
template <int IMG>
__device__ __forceinline__ void read_q12(unsigned qa, double (&q)[NX]) {
  asm volatile(
      "ds_read_b64 %0, %12 offset:0\n\t"
      "ds_read_b64 %1, %12 offset:128\n\t"
      "ds_read_b64 %2, %12 offset:256\n\t"
      "ds_read_b64 %3, %12 offset:384\n\t"
      "ds_read_b64 %4, %12 offset:512\n\t"
      "ds_read_b64 %5, %12 offset:640\n\t"
      "ds_read_b64 %6, %12 offset:768\n\t"
      "ds_read_b64 %7, %12 offset:896\n\t"
      "ds_read_b64 %8, %12 offset:1024\n\t"
      "ds_read_b64 %9, %12 offset:1152\n\t"
      "ds_read_b64 %10, %12 offset:1280\n\t"
      "ds_read_b64 %11, %12 offset:1408\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]),
        "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11])
      : "v"(qa)
      : "memory");
}
template <int IMG>
__device__ __forceinline__ void read_step_vt(const unsigned (&ad)[NX], unsigned xa, unsigned ua,
                                             unsigned ra, double (&ab)[NX], double& x, double& u,
                                             double (&t)[NX]) {
  asm volatile(
      "ds_read_b64 %0, %26 offset:%c41\n\t"
      "ds_read_b64 %1, %27 offset:%c41\n\t"
      "ds_read_b64 %2, %28 offset:%c41\n\t"
      "ds_read_b64 %3, %29 offset:%c41\n\t"
      "ds_read_b64 %4, %30 offset:%c41\n\t"
      "ds_read_b64 %5, %31 offset:%c41\n\t"
      "ds_read_b64 %6, %32 offset:%c41\n\t"
      "ds_read_b64 %7, %33 offset:%c41\n\t"
      "ds_read_b64 %8, %34 offset:%c41\n\t"
      "ds_read_b64 %9, %35 offset:%c41\n\t"
      "ds_read_b64 %10, %36 offset:%c41\n\t"
      "ds_read_b64 %11, %37 offset:%c41\n\t"
      "ds_read_b64 %12, %38 offset:%c41\n\t"
      "ds_read_b64 %13, %39 offset:%c41\n\t"
      "ds_read_b64 %14, %40 offset:0\n\t"
      "ds_read_b64 %15, %40 offset:8\n\t"
      "ds_read_b64 %16, %40 offset:16\n\t"
      "ds_read_b64 %17, %40 offset:24\n\t"
      "ds_read_b64 %18, %40 offset:32\n\t"
      "ds_read_b64 %19, %40 offset:40\n\t"
      "ds_read_b64 %20, %40 offset:48\n\t"
      "ds_read_b64 %21, %40 offset:56\n\t"
      "ds_read_b64 %22, %40 offset:64\n\t"
      "ds_read_b64 %23, %40 offset:72\n\t"
      "ds_read_b64 %24, %40 offset:80\n\t"
      "ds_read_b64 %25, %40 offset:88\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(ab[0]), "=&v"(ab[1]), "=&v"(ab[2]), "=&v"(ab[3]), "=&v"(ab[4]), "=&v"(ab[5]),
        "=&v"(ab[6]), "=&v"(ab[7]), "=&v"(ab[8]), "=&v"(ab[9]), "=&v"(ab[10]), "=&v"(ab[11]),
        "=&v"(x), "=&v"(u), "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]),
        "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]), "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]),
        "=&v"(t[11])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]),
        "v"(ad[7]), "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(xa), "v"(ua),
        "v"(ra), "i"(IMG)
      : "memory");
}

// read_step / read_step_vt plus the step's Qxx accumulator start (Q row r on lane c,
// from the per-wave Q image) under the same wait
template <int IMG>
__device__ __forceinline__ void read_step_q(const unsigned (&ad)[NX], unsigned xa, unsigned ua, unsigned qa, double (&ab)[NX], double& x, double& u, double (&q)[NX]) {
  asm volatile(
      "ds_read_b64 %0, %26 offset:%c41\n\t"
      "ds_read_b64 %1, %27 offset:%c41\n\t"
      "ds_read_b64 %2, %28 offset:%c41\n\t"
      "ds_read_b64 %3, %29 offset:%c41\n\t"
      "ds_read_b64 %4, %30 offset:%c41\n\t"
      "ds_read_b64 %5, %31 offset:%c41\n\t"
      "ds_read_b64 %6, %32 offset:%c41\n\t"
      "ds_read_b64 %7, %33 offset:%c41\n\t"
      "ds_read_b64 %8, %34 offset:%c41\n\t"
      "ds_read_b64 %9, %35 offset:%c41\n\t"
      "ds_read_b64 %10, %36 offset:%c41\n\t"
      "ds_read_b64 %11, %37 offset:%c41\n\t"
      "ds_read_b64 %12, %38 offset:%c41\n\t"
      "ds_read_b64 %13, %39 offset:%c41\n\t"
      "ds_read_b64 %14, %40 offset:0\n\t"
      "ds_read_b64 %15, %40 offset:128\n\t"
      "ds_read_b64 %16, %40 offset:256\n\t"
      "ds_read_b64 %17, %40 offset:384\n\t"
      "ds_read_b64 %18, %40 offset:512\n\t"
      "ds_read_b64 %19, %40 offset:640\n\t"
      "ds_read_b64 %20, %40 offset:768\n\t"
      "ds_read_b64 %21, %40 offset:896\n\t"
      "ds_read_b64 %22, %40 offset:1024\n\t"
      "ds_read_b64 %23, %40 offset:1152\n\t"
      "ds_read_b64 %24, %40 offset:1280\n\t"
      "ds_read_b64 %25, %40 offset:1408\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(ab[0]), "=&v"(ab[1]), "=&v"(ab[2]), "=&v"(ab[3]), "=&v"(ab[4]), "=&v"(ab[5]), "=&v"(ab[6]), "=&v"(ab[7]), "=&v"(ab[8]), "=&v"(ab[9]), "=&v"(ab[10]), "=&v"(ab[11]), "=&v"(x), "=&v"(u), "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]), "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(xa), "v"(ua), "v"(qa), "i"(IMG)
      : "memory");
}
template <int IMG>
__device__ __forceinline__ void read_step_vt_q(const unsigned (&ad)[NX], unsigned xa, unsigned ua, unsigned ra, unsigned qa, double (&ab)[NX], double& x, double& u, double (&t)[NX], double (&q)[NX]) {
  asm volatile(
      "ds_read_b64 %0, %38 offset:%c54\n\t"
      "ds_read_b64 %1, %39 offset:%c54\n\t"
      "ds_read_b64 %2, %40 offset:%c54\n\t"
      "ds_read_b64 %3, %41 offset:%c54\n\t"
      "ds_read_b64 %4, %42 offset:%c54\n\t"
      "ds_read_b64 %5, %43 offset:%c54\n\t"
      "ds_read_b64 %6, %44 offset:%c54\n\t"
      "ds_read_b64 %7, %45 offset:%c54\n\t"
      "ds_read_b64 %8, %46 offset:%c54\n\t"
      "ds_read_b64 %9, %47 offset:%c54\n\t"
      "ds_read_b64 %10, %48 offset:%c54\n\t"
      "ds_read_b64 %11, %49 offset:%c54\n\t"
      "ds_read_b64 %12, %50 offset:%c54\n\t"
      "ds_read_b64 %13, %51 offset:%c54\n\t"
      "ds_read_b64 %14, %52 offset:0\n\t"
      "ds_read_b64 %15, %52 offset:8\n\t"
      "ds_read_b64 %16, %52 offset:16\n\t"
      "ds_read_b64 %17, %52 offset:24\n\t"
      "ds_read_b64 %18, %52 offset:32\n\t"
      "ds_read_b64 %19, %52 offset:40\n\t"
      "ds_read_b64 %20, %52 offset:48\n\t"
      "ds_read_b64 %21, %52 offset:56\n\t"
      "ds_read_b64 %22, %52 offset:64\n\t"
      "ds_read_b64 %23, %52 offset:72\n\t"
      "ds_read_b64 %24, %52 offset:80\n\t"
      "ds_read_b64 %25, %52 offset:88\n\t"
      "ds_read_b64 %26, %53 offset:0\n\t"
      "ds_read_b64 %27, %53 offset:128\n\t"
      "ds_read_b64 %28, %53 offset:256\n\t"
      "ds_read_b64 %29, %53 offset:384\n\t"
      "ds_read_b64 %30, %53 offset:512\n\t"
      "ds_read_b64 %31, %53 offset:640\n\t"
      "ds_read_b64 %32, %53 offset:768\n\t"
      "ds_read_b64 %33, %53 offset:896\n\t"
      "ds_read_b64 %34, %53 offset:1024\n\t"
      "ds_read_b64 %35, %53 offset:1152\n\t"
      "ds_read_b64 %36, %53 offset:1280\n\t"
      "ds_read_b64 %37, %53 offset:1408\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(ab[0]), "=&v"(ab[1]), "=&v"(ab[2]), "=&v"(ab[3]), "=&v"(ab[4]), "=&v"(ab[5]), "=&v"(ab[6]), "=&v"(ab[7]), "=&v"(ab[8]), "=&v"(ab[9]), "=&v"(ab[10]), "=&v"(ab[11]), "=&v"(x), "=&v"(u), "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]), "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11]), "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]), "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(xa), "v"(ua), "v"(ra), "v"(qa), "i"(IMG)
      : "memory");
}

// OCC2: ... and Q's rows for lx = Q e (row c on lane c at qra + 8 i), re-read each step
// instead of held in 24 VGPRs
template <int IMG>
__device__ __forceinline__ void read_step_q_qr(const unsigned (&ad)[NX], unsigned xa, unsigned ua, unsigned qa, unsigned qra, double (&ab)[NX], double& x, double& u, double (&q)[NX], double (&qr)[NX]) {
  asm volatile(
      "ds_read_b64 %0, %38 offset:%c54\n\t"
      "ds_read_b64 %1, %39 offset:%c54\n\t"
      "ds_read_b64 %2, %40 offset:%c54\n\t"
      "ds_read_b64 %3, %41 offset:%c54\n\t"
      "ds_read_b64 %4, %42 offset:%c54\n\t"
      "ds_read_b64 %5, %43 offset:%c54\n\t"
      "ds_read_b64 %6, %44 offset:%c54\n\t"
      "ds_read_b64 %7, %45 offset:%c54\n\t"
      "ds_read_b64 %8, %46 offset:%c54\n\t"
      "ds_read_b64 %9, %47 offset:%c54\n\t"
      "ds_read_b64 %10, %48 offset:%c54\n\t"
      "ds_read_b64 %11, %49 offset:%c54\n\t"
      "ds_read_b64 %12, %50 offset:%c54\n\t"
      "ds_read_b64 %13, %51 offset:%c54\n\t"
      "ds_read_b64 %14, %52 offset:0\n\t"
      "ds_read_b64 %15, %52 offset:128\n\t"
      "ds_read_b64 %16, %52 offset:256\n\t"
      "ds_read_b64 %17, %52 offset:384\n\t"
      "ds_read_b64 %18, %52 offset:512\n\t"
      "ds_read_b64 %19, %52 offset:640\n\t"
      "ds_read_b64 %20, %52 offset:768\n\t"
      "ds_read_b64 %21, %52 offset:896\n\t"
      "ds_read_b64 %22, %52 offset:1024\n\t"
      "ds_read_b64 %23, %52 offset:1152\n\t"
      "ds_read_b64 %24, %52 offset:1280\n\t"
      "ds_read_b64 %25, %52 offset:1408\n\t"
      "ds_read_b64 %26, %53 offset:0\n\t"
      "ds_read_b64 %27, %53 offset:8\n\t"
      "ds_read_b64 %28, %53 offset:16\n\t"
      "ds_read_b64 %29, %53 offset:24\n\t"
      "ds_read_b64 %30, %53 offset:32\n\t"
      "ds_read_b64 %31, %53 offset:40\n\t"
      "ds_read_b64 %32, %53 offset:48\n\t"
      "ds_read_b64 %33, %53 offset:56\n\t"
      "ds_read_b64 %34, %53 offset:64\n\t"
      "ds_read_b64 %35, %53 offset:72\n\t"
      "ds_read_b64 %36, %53 offset:80\n\t"
      "ds_read_b64 %37, %53 offset:88\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(ab[0]), "=&v"(ab[1]), "=&v"(ab[2]), "=&v"(ab[3]), "=&v"(ab[4]), "=&v"(ab[5]), "=&v"(ab[6]), "=&v"(ab[7]), "=&v"(ab[8]), "=&v"(ab[9]), "=&v"(ab[10]), "=&v"(ab[11]), "=&v"(x), "=&v"(u), "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]), "=&v"(qr[0]), "=&v"(qr[1]), "=&v"(qr[2]), "=&v"(qr[3]), "=&v"(qr[4]), "=&v"(qr[5]), "=&v"(qr[6]), "=&v"(qr[7]), "=&v"(qr[8]), "=&v"(qr[9]), "=&v"(qr[10]), "=&v"(qr[11])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]), "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(xa), "v"(ua), "v"(qa), "v"(qra), "i"(IMG)
      : "memory");
}
template <int IMG>
__device__ __forceinline__ void read_step_vt_q_qr(const unsigned (&ad)[NX], unsigned xa, unsigned ua, unsigned ra, unsigned qa, unsigned qra, double (&ab)[NX], double& x, double& u, double (&t)[NX], double (&q)[NX], double (&qr)[NX]) {
  asm volatile(
      "ds_read_b64 %0, %50 offset:%c67\n\t"
      "ds_read_b64 %1, %51 offset:%c67\n\t"
      "ds_read_b64 %2, %52 offset:%c67\n\t"
      "ds_read_b64 %3, %53 offset:%c67\n\t"
      "ds_read_b64 %4, %54 offset:%c67\n\t"
      "ds_read_b64 %5, %55 offset:%c67\n\t"
      "ds_read_b64 %6, %56 offset:%c67\n\t"
      "ds_read_b64 %7, %57 offset:%c67\n\t"
      "ds_read_b64 %8, %58 offset:%c67\n\t"
      "ds_read_b64 %9, %59 offset:%c67\n\t"
      "ds_read_b64 %10, %60 offset:%c67\n\t"
      "ds_read_b64 %11, %61 offset:%c67\n\t"
      "ds_read_b64 %12, %62 offset:%c67\n\t"
      "ds_read_b64 %13, %63 offset:%c67\n\t"
      "ds_read_b64 %14, %64 offset:0\n\t"
      "ds_read_b64 %15, %64 offset:8\n\t"
      "ds_read_b64 %16, %64 offset:16\n\t"
      "ds_read_b64 %17, %64 offset:24\n\t"
      "ds_read_b64 %18, %64 offset:32\n\t"
      "ds_read_b64 %19, %64 offset:40\n\t"
      "ds_read_b64 %20, %64 offset:48\n\t"
      "ds_read_b64 %21, %64 offset:56\n\t"
      "ds_read_b64 %22, %64 offset:64\n\t"
      "ds_read_b64 %23, %64 offset:72\n\t"
      "ds_read_b64 %24, %64 offset:80\n\t"
      "ds_read_b64 %25, %64 offset:88\n\t"
      "ds_read_b64 %26, %65 offset:0\n\t"
      "ds_read_b64 %27, %65 offset:128\n\t"
      "ds_read_b64 %28, %65 offset:256\n\t"
      "ds_read_b64 %29, %65 offset:384\n\t"
      "ds_read_b64 %30, %65 offset:512\n\t"
      "ds_read_b64 %31, %65 offset:640\n\t"
      "ds_read_b64 %32, %65 offset:768\n\t"
      "ds_read_b64 %33, %65 offset:896\n\t"
      "ds_read_b64 %34, %65 offset:1024\n\t"
      "ds_read_b64 %35, %65 offset:1152\n\t"
      "ds_read_b64 %36, %65 offset:1280\n\t"
      "ds_read_b64 %37, %65 offset:1408\n\t"
      "ds_read_b64 %38, %66 offset:0\n\t"
      "ds_read_b64 %39, %66 offset:8\n\t"
      "ds_read_b64 %40, %66 offset:16\n\t"
      "ds_read_b64 %41, %66 offset:24\n\t"
      "ds_read_b64 %42, %66 offset:32\n\t"
      "ds_read_b64 %43, %66 offset:40\n\t"
      "ds_read_b64 %44, %66 offset:48\n\t"
      "ds_read_b64 %45, %66 offset:56\n\t"
      "ds_read_b64 %46, %66 offset:64\n\t"
      "ds_read_b64 %47, %66 offset:72\n\t"
      "ds_read_b64 %48, %66 offset:80\n\t"
      "ds_read_b64 %49, %66 offset:88\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(ab[0]), "=&v"(ab[1]), "=&v"(ab[2]), "=&v"(ab[3]), "=&v"(ab[4]), "=&v"(ab[5]), "=&v"(ab[6]), "=&v"(ab[7]), "=&v"(ab[8]), "=&v"(ab[9]), "=&v"(ab[10]), "=&v"(ab[11]), "=&v"(x), "=&v"(u), "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]), "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11]), "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]), "=&v"(qr[0]), "=&v"(qr[1]), "=&v"(qr[2]), "=&v"(qr[3]), "=&v"(qr[4]), "=&v"(qr[5]), "=&v"(qr[6]), "=&v"(qr[7]), "=&v"(qr[8]), "=&v"(qr[9]), "=&v"(qr[10]), "=&v"(qr[11])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]), "v"(ad[8]), "v"(ad[9]), "v"(ad[10]), "v"(ad[11]), "v"(xa), "v"(ua), "v"(ra), "v"(qa), "v"(qra), "i"(IMG)
      : "memory");
}

// park x (column c per lane) in the problem's tile: row i at wa + 136 i (no wait:
// the wave's LDS operations execute in order, the next reads see these writes)
__device__ __forceinline__ void lds_park12(const double (&x)[NX], unsigned wa) {
  asm volatile(
      "ds_write_b64 %12, %0 offset:0\n\t"
      "ds_write_b64 %12, %1 offset:136\n\t"
      "ds_write_b64 %12, %2 offset:272\n\t"
      "ds_write_b64 %12, %3 offset:408\n\t"
      "ds_write_b64 %12, %4 offset:544\n\t"
      "ds_write_b64 %12, %5 offset:680\n\t"
      "ds_write_b64 %12, %6 offset:816\n\t"
      "ds_write_b64 %12, %7 offset:952\n\t"
      "ds_write_b64 %12, %8 offset:1088\n\t"
      "ds_write_b64 %12, %9 offset:1224\n\t"
      "ds_write_b64 %12, %10 offset:1360\n\t"
      "ds_write_b64 %12, %11 offset:1496"
      :
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]),
        "v"(x[8]), "v"(x[9]), "v"(x[10]), "v"(x[11]), "v"(wa)
      : "memory");
}

// the 12 transposed reads of a parked matrix and their wait (epilogue)
__device__ __forceinline__ void lds_read_t12(double (&t)[NX], unsigned ra) {
  asm volatile(
      "ds_read_b64 %0, %12 offset:0\n\t"
      "ds_read_b64 %1, %12 offset:8\n\t"
      "ds_read_b64 %2, %12 offset:16\n\t"
      "ds_read_b64 %3, %12 offset:24\n\t"
      "ds_read_b64 %4, %12 offset:32\n\t"
      "ds_read_b64 %5, %12 offset:40\n\t"
      "ds_read_b64 %6, %12 offset:48\n\t"
      "ds_read_b64 %7, %12 offset:56\n\t"
      "ds_read_b64 %8, %12 offset:64\n\t"
      "ds_read_b64 %9, %12 offset:72\n\t"
      "ds_read_b64 %10, %12 offset:80\n\t"
      "ds_read_b64 %11, %12 offset:88\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]),
        "=&v"(t[6]), "=&v"(t[7]), "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11])
      : "v"(ra)
      : "memory");
}

__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// all but the N youngest vector-memory operations done (loads, stores and
// LDS-DMA count together in issue order)
template <int N>
__device__ __forceinline__ void vm_wait_n() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

// x <- 0.5 (x + x^T) through the problem's LDS tile in ONE asm statement: the
// wave's LDS operations execute in order, so the transposed reads follow the
// writes without a wait in between; one lgkmcnt wait at the end
template <int S>
__device__ __forceinline__ void lds_transpose(const double (&x)[S], double (&t)[S], unsigned wa,
                                              unsigned ra);
template <>
__device__ __forceinline__ void lds_transpose<12>(const double (&x)[12], double (&t)[12],
                                                  unsigned wa, unsigned ra) {
  asm volatile(
      "ds_write_b64 %24, %12 offset:0\n\t"
      "ds_write_b64 %24, %13 offset:136\n\t"
      "ds_write_b64 %24, %14 offset:272\n\t"
      "ds_write_b64 %24, %15 offset:408\n\t"
      "ds_write_b64 %24, %16 offset:544\n\t"
      "ds_write_b64 %24, %17 offset:680\n\t"
      "ds_write_b64 %24, %18 offset:816\n\t"
      "ds_write_b64 %24, %19 offset:952\n\t"
      "ds_write_b64 %24, %20 offset:1088\n\t"
      "ds_write_b64 %24, %21 offset:1224\n\t"
      "ds_write_b64 %24, %22 offset:1360\n\t"
      "ds_write_b64 %24, %23 offset:1496\n\t"
      "ds_read_b64 %0, %25 offset:0\n\t"
      "ds_read_b64 %1, %25 offset:8\n\t"
      "ds_read_b64 %2, %25 offset:16\n\t"
      "ds_read_b64 %3, %25 offset:24\n\t"
      "ds_read_b64 %4, %25 offset:32\n\t"
      "ds_read_b64 %5, %25 offset:40\n\t"
      "ds_read_b64 %6, %25 offset:48\n\t"
      "ds_read_b64 %7, %25 offset:56\n\t"
      "ds_read_b64 %8, %25 offset:64\n\t"
      "ds_read_b64 %9, %25 offset:72\n\t"
      "ds_read_b64 %10, %25 offset:80\n\t"
      "ds_read_b64 %11, %25 offset:88\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]),
        "=&v"(t[6]), "=&v"(t[7]), "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11])
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]),
        "v"(x[8]), "v"(x[9]), "v"(x[10]), "v"(x[11]), "v"(wa), "v"(ra)
      : "memory");
}
template <>
__device__ __forceinline__ void lds_transpose<4>(const double (&x)[4], double (&t)[4], unsigned wa,
                                                 unsigned ra) {
  asm volatile(
      "ds_write_b64 %8, %4 offset:0\n\t"
      "ds_write_b64 %8, %5 offset:136\n\t"
      "ds_write_b64 %8, %6 offset:272\n\t"
      "ds_write_b64 %8, %7 offset:408\n\t"
      "ds_read_b64 %0, %9 offset:0\n\t"
      "ds_read_b64 %1, %9 offset:8\n\t"
      "ds_read_b64 %2, %9 offset:16\n\t"
      "ds_read_b64 %3, %9 offset:24\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3])
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(wa), "v"(ra)
      : "memory");
}

// sum_r x[r] at lane r (the trace of a row-per-register 4 x 4 block), on every lane
__device__ __forceinline__ double diag_sum4(const double (&x)[4]) {
  double acc = 0.0;
  const double one = 1.0;
  asm(HOP_NOP2
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:0" HOP_DPP_TAIL
      "v_fmac_f64_dpp %0, %2, %5 row_newbcast:1" HOP_DPP_TAIL
      "v_fmac_f64_dpp %0, %3, %5 row_newbcast:2" HOP_DPP_TAIL
      "v_fmac_f64_dpp %0, %4, %5 row_newbcast:3" HOP_DPP_TAIL
      : "+&v"(acc)
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(one));
  return acc;
}

// Packed rows (PK): P[r] = [Qux row r (lanes 0..11) | Quu row r (lanes 12..15)].  The
// transpose of the 4 x 4 block for _sym(Quu), in ONE asm statement: the rows are
// written a second time with lane 12 + x's entries at row 12 + x, column r (an
// immediate stride of 8; lanes < 12 write into row 0, which the plain row writes that
// follow overwrite), then read back with a stride of 136: lanes < 12 see their own
// Qux entries, lanes 12 + j see P[j][12 + r], the transpose.
__device__ __forceinline__ void lds_sym_packed4(const double (&x)[4], double (&t)[4], unsigned wa,
                                                unsigned wt, unsigned rt) {
  asm volatile(
      "ds_write_b64 %5, %7 offset:0\n\t"
      "ds_write_b64 %5, %8 offset:8\n\t"
      "ds_write_b64 %5, %9 offset:16\n\t"
      "ds_write_b64 %5, %10 offset:24\n\t"
      "ds_write_b64 %4, %7 offset:0\n\t"
      "ds_write_b64 %4, %8 offset:136\n\t"
      "ds_write_b64 %4, %9 offset:272\n\t"
      "ds_write_b64 %4, %10 offset:408\n\t"
      "ds_read_b64 %0, %6 offset:0\n\t"
      "ds_read_b64 %1, %6 offset:136\n\t"
      "ds_read_b64 %2, %6 offset:272\n\t"
      "ds_read_b64 %3, %6 offset:408\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3])
      : "v"(wa), "v"(wt), "v"(rt), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3])
      : "memory");
}
// sum of lanes [OFF, OFF + N) of x on every lane of the row
template <int N, int OFF>
__device__ __forceinline__ double lane_sum_off(double x) {
  double acc = 0.0, one[N];
#pragma unroll
  for (int j = 0; j < N; ++j) one[j] = 1.0;
  LaneDotOff<N, OFF>::fma(acc, x, one);
  return acc;
}
// sum_r x[r] at lane 12 + r (the trace of the packed 4 x 4 block)
__device__ __forceinline__ double diag_sum4_off12(const double (&x)[4]) {
  double acc = 0.0;
  const double one = 1.0;
  asm(HOP_NOP2
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:12" HOP_DPP_TAIL
      "v_fmac_f64_dpp %0, %2, %5 row_newbcast:13" HOP_DPP_TAIL
      "v_fmac_f64_dpp %0, %3, %5 row_newbcast:14" HOP_DPP_TAIL
      "v_fmac_f64_dpp %0, %4, %5 row_newbcast:15" HOP_DPP_TAIL
      : "+&v"(acc)
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(one));
  return acc;
}

// acc[r] += bcast_{12 + r}(d) * y[r], r < 4: rows of the packed [Qux | Quu] block scaled
// by a per-row factor that lives on lanes 12..15 (the equilibration below)
__device__ __forceinline__ void row_scale12(double (&acc)[4], double d, const double (&y)[4]) {
  asm(HOP_NOP2
      "v_fmac_f64_dpp %0, %4, %5 row_newbcast:12" HOP_DPP_TAIL
      "v_fmac_f64_dpp %1, %4, %6 row_newbcast:13" HOP_DPP_TAIL
      "v_fmac_f64_dpp %2, %4, %7 row_newbcast:14" HOP_DPP_TAIL
      "v_fmac_f64_dpp %3, %4, %8 row_newbcast:15" HOP_DPP_TAIL
      : "+&v"(acc[0]), "+&v"(acc[1]), "+&v"(acc[2]), "+&v"(acc[3])
      : "v"(d), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  const unsigned nrec = bytes > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (unsigned)(bytes > 0 ? bytes : 0);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nrec,
                                           0x00020000);
}

__device__ __forceinline__ void st64(double v, __amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
  __builtin_amdgcn_raw_buffer_store_b64(as_u2(v), r, vo, so, 0);
}

// section stamps of the diagnostic instantiation (developer builds,
// tools/stamps_riccati.py --fast): per-wave shader-clock totals per section
__device__ unsigned long long g_ricf_stamp[16];

// EXP (developer builds, timing experiments only -- results are wrong): 1 drops
// the stores, 2 the per-step LDS-DMA.  JC: the J-curve form (mode 1 at horizon jl for
// the whole wave, no K / k / V stores; RiccatiArgs::jc_J).  blk: the workgroup's
// problem block.
// PK (packed rows, default): [Qux | Quu] of row r of B^T V [A|B] + R share one 16-lane
// register (Quu on lanes 12..15), so the offset-form 4 x 4 sweep leaves
// (Quu_reg + eps I)^-1 Qux = -K on lanes 0..11 directly: no K product, no lane
// rotations of Quu, no inverse rebuilt from the sweep's offset form; Qu, k and R du
// live on lanes 12..15 likewise.  PK = false keeps the round-2 form (developer A/B).
// QL (default): the one-wave layout reads the step's Qxx accumulator start (the Q
// image) inside the V [A|B] product's asm block (LaneRowsQ) instead of with the
// step's other reads, so its LDS latency hides under the 144 FMAs
template <int MODE, bool WANTV, bool STAMP, int EXP, bool JC, bool PK = true, bool OCC2 = false,
          bool QL = true>
__device__ __forceinline__ void ric_body(const RiccatiArgs<double>& a, long long blk, int jl) {
  constexpr int S = NX, MM = MU;
  unsigned long long sec[12] = {};
  unsigned long long tprev = 0;
  auto stamp = [&](int j) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long tt = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (j >= 0) sec[j] += tt - tprev;
      tprev = tt;
    }
  };
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned char* wbase = smem_raw + w * (OCC2 ? WAVE_BYTES2 : WAVE_BYTES);
  const unsigned wlds = (unsigned)(uintptr_t)wbase;
  double* tile = reinterpret_cast<double*>(wbase + (OCC2 ? OFF_T2 : OFF_T)) + g * kLdsTile;
#pragma unroll 1
  for (int i = c; i < kLdsTile; i += kRowLanes) tile[i] = 0.0;

  const long long wave_prob0 = (blk * kWavesPerBlock + w) * kProbPerWave;
  const long long prob = wave_prob0 + g;
  const bool valid = prob < a.batch;
  const long long pb = valid ? prob : a.batch - 1;
  if (wave_prob0 >= a.batch) return;  // wave-uniform; no workgroup barrier in this kernel
  const long long pb0 = wave_prob0;
  const int NA = a.nalloc;
  // descriptors cover only the wave's problems: an out-of-range offset then
  // always means "dropped" (the commit mask of the stores below relies on it)
  const long long left = a.batch - pb0 < kProbPerWave ? a.batch - pb0 : kProbPerWave;

  // buffer descriptors based at the wave's first problem (exact bounds: OOB reads 0,
  // OOB writes dropped)
  const long long pA = (long long)NA * S * S * 8, pB = (long long)NA * S * MM * 8;
  const long long pX = (long long)(NA + 1) * S * 8, pU = (long long)NA * MM * 8;
  const __amdgpu_buffer_rsrc_t rA = rsrc(a.A + pb0 * (pA / 8), left * pA),
                               rB = rsrc(a.Bm + pb0 * (pB / 8), left * pB),
                               rX = rsrc(a.X + pb0 * (pX / 8), left * pX),
                               rU = rsrc(a.U + pb0 * (pU / 8), left * pU);
  const long long pK = (long long)NA * MM * S * 8, pk = (long long)NA * MM * 8;
  const __amdgpu_buffer_rsrc_t rK = rsrc(JC ? a.X : a.K + pb0 * (pK / 8), JC ? 0 : left * pK),
                               rk = rsrc(JC ? a.X : a.k + pb0 * (pk / 8), JC ? 0 : left * pk);
  const long long pVxx = (long long)(NA + 1) * S * S * 8, pVx = (long long)(NA + 1) * S * 8,
                  pV0 = (long long)(NA + 1) * 8;
  constexpr bool wantv = WANTV;
  // stores per step, all issued unconditionally (non-committing lanes write out of
  // range): K 4, k 1 [+ Vxx 12 (of the step before), Vx 1, V0 1].  (Row c of the
  // exactly symmetric V is also lane c's 12 registers, but 6 16-B stores of those
  // rows scatter 48 16-B pieces per instruction and measured 5 % slower in mode 1.)
  constexpr int NST = JC ? 0 : 5 + (WANTV ? 14 : 0);
  unsigned va[5], vb[2], vx_, vu_;
#pragma unroll
  for (int j = 0; j < 5; ++j)  // image pieces 0 .. 4
    va[j] = dma9_voff(voff<CH_A>(j, lane, wave_prob0, pb0, a.batch, pA), j);
#pragma unroll
  for (int j = 0; j < 2; ++j)  // pieces 5, 6
    vb[j] = dma9_voff(voff<CH_B>(j, lane, wave_prob0, pb0, a.batch, pB), 5 + j);
  vx_ = dma9_voff(voff<CH_X>(0, lane, wave_prob0, pb0, a.batch, pX), 7);
  vu_ = dma9_voff(voff<CH_U>(0, lane, wave_prob0, pb0, a.batch, pU), 8);
  // per-lane image addresses of [A|B] row j, x_c and u_c
  unsigned ad[S];
#pragma unroll
  for (int j = 0; j < S; ++j)
    ad[j] = wlds + (c < S ? OFF_A + 1152 * g + 8 * c + 96 * j
                          : OFF_B + 384 * g + 8 * (c - S) + 32 * j);
  const unsigned xa = wlds + OFF_X + 96 * g + 8 * (c < S ? c : 0);
  const unsigned ua = wlds + OFF_U + 32 * g + 8 * (c < MM ? c : ((PK && c >= S) ? c - S : 0));
  // per-lane store offsets (problem part; the step part is the scalar offset)
  const unsigned pofs = (unsigned)(pb - pb0);
  const unsigned voK = pofs * (unsigned)pK + 8u * (c < S ? c : 0);
  const unsigned vok = pofs * (unsigned)pk + 8u * (c < MM ? c : ((PK && c >= S) ? c - S : 0));

  const double* xgp = a.xg + pb * a.xg_bstride;
  const double* urp = a.u_ref + pb * a.uref_bstride;
  const double* Qp = a.Q + pb * a.q_bstride;
  const double* Rp = a.R + pb * a.r_bstride;
  const double* Qfp = a.Qf + pb * a.qf_bstride;
  const int L = valid ? (JC ? jl : a.horizon[pb]) : 0;
  int Lw = L;
  Lw = max(Lw, __shfl_xor(Lw, 16));
  Lw = max(Lw, __shfl_xor(Lw, 32));
  Lw = __builtin_amdgcn_readfirstlane(Lw);
  Lw = Lw < NA ? Lw : NA;
  const double lam0 = JC ? a.lm_value : a.lm[pb];

  // loop-invariant cost blocks in registers: Q column c / row c, R column / row
  const int cq = c < S ? c : 0, cr = c < MM ? c : 0;
  // Q row r on lane c (the Qxx accumulator start) lives in the wave's Q image and
  // is re-read each step with the step's [A|B]; only Q's rows (for lx) stay in VGPRs
  double qrow_r[S], rcol[MM], rrow[MM];
  // (OCC2: one image for the wave; its 4 problems write the same batch-shared Q; Q's
  // rows are read from it per step, lanes 12..15 reading row 0: their lx is never used)
  const unsigned qa = wlds + (OCC2 ? OFF_Q2 : OFF_Q + Q_PROB * g) + 8 * c;
  const unsigned qra = wlds + OFF_Q2 + 128 * cq;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const double qv = c < S ? Qp[i * S + cq] : 0.0;
    asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(qa), "v"(qv), "i"(128 * i) : "memory");
    if constexpr (!OCC2) qrow_r[i] = c < S ? Qp[cq * S + i] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < MM; ++i) {
    rcol[i] = c < MM ? Rp[i * MM + cr] : ((i == c) ? 1.0 : 0.0);
    rrow[i] = c < MM ? Rp[cr * MM + i] : ((i == c) ? 1.0 : 0.0);
  }
  const double xg_c = c < S ? xgp[cq] : 0.0;
  // PK: u and u_ref ride on lanes 12..15 as well (du, R du, Qu, k of the packed rows)
  const double ur_c = c < MM ? urp[cr] : ((PK && c >= S) ? urp[c - S] : 0.0);
  double rpk[PK ? MM : 1], rrow12[PK ? MM : 1], dgc[PK ? MM : 1], ohr[PK ? MM : 1],
      nd[PK ? MM : 1];
  if constexpr (PK) {
    const double lam1 = MODE == 0 ? lam0 : (lam0 > 1e-12 ? lam0 : 1e-12);
    const int cs = c >= S ? c - S : 0;
#pragma unroll
    for (int r = 0; r < MM; ++r) {
      rpk[r] = c >= S ? Rp[r * MM + cs] : 0.0;     // lanes 12..15: row r of R
      rrow12[r] = c >= S ? Rp[cs * MM + r] : 0.0;  // lanes 12..15: column r of R
      // lane 12 + r of register r (the packed block's diagonal): lam + eps (chol_solve's
      // first try), a one-hot and the offset form's -1
      dgc[r] = (c == S + r) ? lam1 + 1e-9 : 0.0;
      ohr[r] = (c == S + r) ? 1.0 : 0.0;
      nd[r] = -ohr[r];
    }
  }
  const bool wrap_c = (c < S) && ((a.wrap_mask >> c) & 1u);

  unsigned st = 0;
  bool alive = valid && L > 0 && L <= NA;
  if (valid && !(L > 0 && L <= NA)) st |= ST_FAIL;

  // terminal: Vxx = sym(Qf), Vx = Qf eT, V0 = 1/2 eT' Qf eT
  double V[S], vx, v0;
  {
    double qfrow[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      V[i] = c < S ? Qfp[i * S + cq] : 0.0;
      qfrow[i] = c < S ? Qfp[cq * S + i] : 0.0;
    }
    const int iT = (L > 0 && L <= NA) ? L : 0;
    double eT = c < S ? a.X[pb * (NA + 1) * S + (long long)iT * S + cq] - xg_c : 0.0;
    if (wrap_c) eT = wrap_angle(eT);
    const bool fin = ((__ballot(!finite_val(eT)) >> (16 * g)) & 0xffffull) == 0ull;
    if (!fin) {
      st |= ST_NONFINITE | ST_FAIL;
      alive = false;
    }
    vx = 0.0;
    LaneDot<S>::fma(vx, eT, qfrow);
    v0 = 0.5 * lane_sum<S>(eT * vx);
    symmetrize(V, tile, c);
    if (alive && wantv) {  // the terminal expansion (plain stores, before the loop)
      double* o = a.Vxx + (pb * (NA + 1) + L) * (long long)(S * S);
      if (c < S) {
#pragma unroll
        for (int i = 0; i < S; ++i) o[i * S + c] = V[i];
        a.Vx[pb * (NA + 1) * S + (long long)L * S + c] = vx;
      }
      if (c == 0) a.V0[pb * (NA + 1) + L] = v0;
    }
  }
  const __amdgpu_buffer_rsrc_t rVxx = rsrc(wantv ? a.Vxx + pb0 * (pVxx / 8) : a.K,
                                           wantv ? left * pVxx : 0),
                               rVx = rsrc(wantv ? a.Vx + pb0 * (pVx / 8) : a.K,
                                          wantv ? left * pVx : 0),
                               rV0 = rsrc(wantv ? a.V0 + pb0 * (pV0 / 8) : a.K,
                                          wantv ? left * pV0 : 0);
  const unsigned voVxx = pofs * (unsigned)pVxx + 8u * (c < S ? c : 0);
  const unsigned voVx = pofs * (unsigned)pVx + 8u * (c < S ? c : 0);
  const unsigned voV0 = pofs * (unsigned)pV0;
  const unsigned twa = (unsigned)(uintptr_t)tile + 8u * c;         // (i, c): + 136 i
  const unsigned tra = (unsigned)(uintptr_t)tile + 8u * kLdsRow * c;  // (c, i): + 8 i
  // PK: the packed 4 x 4 block's transpose through tile rows 12..15 (lds_sym_packed4)
  const unsigned tbase = (unsigned)(uintptr_t)tile;
  const unsigned tw2 = c < S ? twa : tbase + 136u * c;
  const unsigned tr2 = c < S ? twa : tbase + 136u * S + 8u * (c - S);
  constexpr unsigned OOB = 0x80000000u;

  // Deferred symmetrisation: step i parks its value update Vn in the tile and
  // carries it (Vp, with its commit flag) into step i-1, whose LDS read of the
  // step's [A|B] image also reads Vn^T; V = sym(Vn) is formed there, so the
  // transpose's LDS latency hides under the stores and the next step's DMA issue.
  double Vp[S];
  bool cprev = false;
  zero(Vp);

  // one step (index i) reading image IMG; issues the DMA of step i-1 into the
  // other image first
  auto step = [&](int i, auto IMGc, auto FIRSTc) {
    constexpr int IMG = decltype(IMGc)::value;
    constexpr bool FIRST = decltype(FIRSTc)::value;
    constexpr int NEXT = OCC2 ? 0 : (IMG == 0 ? BUF : 0);
    // this step's pieces landed; the previous step's NST stores may still be in flight
    stamp(-1);
    if constexpr (FIRST) vm_wait();
    else vm_wait_n<EXP == 1 ? 0 : NST>();
    stamp(0);
    auto dma_prev = [&]() {
      if (EXP != 2 && i > 0)
        dma9<NEXT>(va, vb, vx_, vu_, rA, rB, rX, rU, wlds, (unsigned)(i - 1) * (S * S * 8),
                   (unsigned)(i - 1) * (S * MM * 8), (unsigned)(i - 1) * (S * 8),
                   (unsigned)(i - 1) * (MM * 8));
    };
    if constexpr (!OCC2) dma_prev();
    stamp(1);
    double ab[S], xi, ui;
    double Qxx[S];  // Q (the accumulator start of Qxx = Q + A^T V A)
    double qrow[S];  // Q row c (lx = Q e): loop-invariant registers, or (OCC2) LDS
    if constexpr (!OCC2) copy(qrow, qrow_r);
    constexpr bool QLATE = QL && !OCC2;
    if constexpr (FIRST) {
      if constexpr (OCC2) read_step_q_qr<IMG>(ad, xa, ua, qa, qra, ab, xi, ui, Qxx, qrow);
      else if constexpr (QLATE) read_step<IMG>(ad, xa, ua, ab, xi, ui);
      else read_step_q<IMG>(ad, xa, ua, qa, ab, xi, ui, Qxx);
    } else {
      double t[S];
      if constexpr (OCC2) read_step_vt_q_qr<IMG>(ad, xa, ua, tra, qa, qra, ab, xi, ui, t, Qxx, qrow);
      else if constexpr (QLATE) read_step_vt<IMG>(ad, xa, ua, tra, ab, xi, ui, t);
      else read_step_vt_q<IMG>(ad, xa, ua, tra, qa, ab, xi, ui, t, Qxx);
      // _sym of step i+1's Vxx; a row that did not commit carried (and parked) its
      // old, exactly symmetric V, for which this is V itself
#pragma unroll
      for (int r = 0; r < S; ++r) V[r] = 0.5 * (Vp[r] + t[r]);
    }
    // OCC2: the single image is free once its reads have waited (lgkmcnt(0) above)
    if constexpr (OCC2) dma_prev();
    // Vxx of step i+1 (mode 1 / requested): NST counts 12 stores here every step
    // (the first step's are out of range) so vm_wait_n stays exact
    if constexpr (WANTV && EXP != 1) {
      const bool wr = !FIRST && cprev && c < S;
      const unsigned sv = (unsigned)(i + 1) * (S * S * 8), vo = wr ? voVxx : OOB;
#pragma unroll
      for (int r = 0; r < S; ++r) st64(V[r], rVxx, vo + 8u * S * r, sv);
    }
    stamp(2);
    const bool act = alive && (i < L);
    double e = c < S ? xi - xg_c : 0.0;
    if (wrap_c) e = wrap_angle(e);
    const double du = (c < MM || (PK && c >= S)) ? ui - ur_c : 0.0;
    // the brute-force curve (solver.py:326-356) checks nothing itself: only its
    // chol_solve raises, so a non-finite e at t = 0 only feeds V_0 (inf/NaN in J)
    const bool e_ok = (JC && i == 0) || finite_val(e);
    const unsigned long long badm = __ballot(!(e_ok && finite_val(du)));
    const bool bad = ((badm >> (16 * g)) & 0xffffull) != 0ull;

    // lx = Q e, lu = R du (lanes < n / < m)
    double lx = 0.0, lu = 0.0;
    LaneDot<S>::fma(lx, e, qrow);
    if constexpr (PK) LaneDotOff<MM, S>::fma(lu, du, rrow12);  // R du on lanes 12..15
    else LaneDot<MM>::fma(lu, du, rrow);
    double l0 = 0.0;
    if constexpr (MODE == 1) {
      if constexpr (PK)
        l0 = 0.5 * lane_sum<S>(e * lx) + 0.5 * lane_sum_off<MM, S>(du * lu) + a.w_stage;
      else
        l0 = 0.5 * lane_sum<S>(e * lx) + 0.5 * lane_sum<MM>(du * lu) + a.w_stage;
    }
    // Q-function: qab = [A|B]^T Vx; VA = V [A|B]; [A|B]^T V [A|B]
    double qab = 0.0;
    LaneDot<S>::fma(qab, vx, ab);
    const double qx = lx + qab;  // Qx = lx + A^T Vx (lanes < n)
    // Qu = lu + B^T Vx: lanes < m, or (PK) lanes 12..15 where B^T Vx already is
    const double qu = PK ? lu + qab : lu + ror_row<kRowLanes - S>(qab);
    stamp(3);
    // products as one dependent DPP chain per output row (accumulator forwarded)
    double VA[S];
    zero(VA);
    if constexpr (QLATE) LaneRowsQ<S>::run(VA, Qxx, V, ab, qa);  // V [A|B], Q's rows
    else static_for<S>([&](auto I) { LaneDot<S>::fma(VA[I], V[I], ab); });  // V [A|B]
    stamp(4);
    // Q + A^T V A is accumulated into Qxx under the Quu^-1 sweep below
    double Uq[MM];  // Qux rows (lanes < n): P under PK
    double Kq[MM];  // K rows (lanes < n); under PK -K (the sweep's lanes 0..11)
    double kvq;     // k (lanes < m; under PK lanes 12..15)
    bool fail_row;
    double(&Vn)[S] = Qxx;  // the value update accumulates into Qxx in place
    double vxn = qx, v0n = v0;
    if constexpr (PK) {
      // P[R] = R row R (lanes 12..15) + B^T V [A|B] row R: [Qux | Quu] on one register
      double P[MM], PT[MM];
#pragma unroll
      for (int r = 0; r < MM; ++r) P[r] = rpk[r];
      static_for<MM>([&](auto R) { ColChain<S>::template fmaq<S + R>(P[R], ab, VA); });
      stamp(5);
      lds_sym_packed4(P, PT, twa, tw2, tr2);  // lanes 12..15 of PT: Quu^T; lanes < 12: Qux
      stamp(6);
      bool solved;
      // rj: the sweep's rows, scaled (see below); rk: (Quu_reg + eps I)^-1 Qux = -K on
      // lanes 0..11; dq: the row scale D_c on lanes 12..15 (1 elsewhere)
      double rj[MM], rk[MM], dq;
      {
        // Equilibrated solve (round 6).  The offset-form sweep keeps -(M)^-1 + I: an
        // entry of M^-1 ~ 1/d next to the 1 loses u d of its relative accuracy, and so
        // does row p of the Qux lanes at a pivot d.  On a real quadrotor linearisation
        // near the pitch singularity Vxx reaches 3e10 and Quu's diagonal 2e11, which
        // left mode 1's Vxx 5e-6 off the reference where NumPy's Cholesky solve stays
        // at 2e-9 of the 40-digit value (tests/test_gpu_gains.py).  So the sweep runs on
        // M' = D M D, D = diag(M)^-1/2 (unit diagonal: every pivot of the SPD case is
        // <= 1, and M'^-1 has entries >= 1 on its diagonal), with the Qux lanes scaled
        // by the same D_r: the sweep leaves M'^-1 D Qux there, and M^-1 Qux = D (that),
        // M^-1 = D M'^-1 D.  The pivots keep their signs (the PD test is unchanged);
        // a non-positive or non-finite diagonal gives D = NaN, a failed first attempt
        // and the ladder, as before.  M = _sym(Quu) + (lam + 1e-9) I.  Cost: +8 % on
        // mode 0 and the J curve with 1/sqrt and exact-zero diagonals, less with the
        // rsq form below (profiles/r06_ab_riccati_equilibration.jsonl).
        const double lam1 = MODE == 0 ? lam0 : (lam0 > 1e-12 ? lam0 : 1e-12);
        // M = _sym(Quu) + (lam + eps) I on lanes 12..15 (Qux on lanes < 12, exactly)
        double qs[MM];
#pragma unroll
        for (int r = 0; r < MM; ++r) qs[r] = __builtin_fma(0.5, P[r] + PT[r], dgc[r]);
        // D_c = diag(M)^-1/2 on lanes 12..15 (1 elsewhere).  Any positive D is exact
        // algebra (the same D scales and unscales), so one v_rsq_f64 serves; the offset
        // diagonal below is D_c^2 M_cc - 1 as computed, not an assumed 0.  A non-positive
        // diagonal gives NaN, +inf gives D = 0 and a NaN diagonal: a failed first try.
        double mdg = qs[0] * ohr[0];
#pragma unroll
        for (int r = 1; r < MM; ++r) mdg = __builtin_fma(qs[r], ohr[r], mdg);
        dq = c >= S ? __builtin_amdgcn_rsq(mdg) : 1.0;
#pragma unroll
        for (int r = 0; r < MM; ++r) {
          qs[r] *= dq;  // column scale (lanes 12..15)
          rj[r] = nd[r];
        }
        row_scale12(rj, dq, qs);  // row scale, minus I: M' - I
        double dj = 1.0;
        SweepQColChainOff<MM, S, S>::run(rj, dj, Qxx, ab, VA);
        const bool okj = (dj > 0.0) && (bcast<S>(rj[0]) == bcast<S>(rj[0]));
#pragma unroll
        for (int r = 0; r < MM; ++r) rk[r] = 0.0;
        row_scale12(rk, dq, rj);  // lanes < 12: D_r (M'^-1 D Qux)_r = (M^-1 Qux)_r
        bool ok0 = true;
        if constexpr (MODE == 0) {
          // trace((M + eps I)^-1) = sum_c D_c^2 (1 - rj[c]_cc)
          const double d2 = dq * dq;
          double wt[MM];
#pragma unroll
          for (int r = 0; r < MM; ++r) wt[r] = __builtin_fma(-rj[r], d2, d2);
          const double tr = diag_sum4_off12(wt);
          const bool sure = okj && (tr < 1e6);
          if (__any(!sure && act)) {  // the exact jitter-free check (rows that step)
            double rc[MM];
#pragma unroll
            for (int r = 0; r < MM; ++r)
              rc[r] = ror_row<kRowLanes - S>(0.5 * (P[r] + PT[r])) + ((c == r) ? lam1 - 1.0 : 0.0);
            double dc = 1.0;
            SweepQ<MM>::run(rc, dc);
            const bool okc = (dc > 0.0) && (bcast<0>(rc[0]) == bcast<0>(rc[0]));
            ok0 = sure || okc;
          }
        }
        solved = okj && ok0;
        if (__any(!okj && ok0 && act)) {  // the jitter / lambda ladders (rare), on lanes 0..3
          const bool ladder = !okj && ok0;
          double Qs[MM], Ql[MM];
#pragma unroll
          for (int r = 0; r < MM; ++r) Qs[r] = ror_row<kRowLanes - S>(0.5 * (P[r] + PT[r]));
          bool good;
          if constexpr (MODE == 0) {
#pragma unroll
            for (int r = 0; r < MM; ++r) Ql[r] = Qs[r] + ((c == r) ? lam0 : 0.0);
            bool okc = true;
            good = spd_inverse_nofallback_chk(Ql, tile, c, 8, st, okc) && okc;
          } else {
            double lam = lam1;
            int tries = 0;
#pragma unroll 1
            while (true) {
#pragma unroll
              for (int r = 0; r < MM; ++r) Ql[r] = Qs[r] + ((c == r) ? lam : 0.0);
              good = spd_inverse_nofallback(Ql, tile, c, 8, st);
              ++tries;
              const bool done = good || tries >= a.reg_max_tries;
              if (!__any(!done && act && ladder)) break;
              if (!done) lam *= 10.0;
            }
          }
          // back to the packed form (unscaled, D = 1): lanes 0..11 Ql Qux, lanes
          // 12..15 I - Ql
#pragma unroll
          for (int r = 0; r < MM; ++r) {
            double y = 0.0;
            LaneDot<MM>::fma(y, Ql[r], P);
            const double il = ror_row<S>(Ql[r]);
            const double rl = c < S ? y : (((c == S + r) ? 1.0 : 0.0) - il);
            rj[r] = ladder ? rl : rj[r];
            rk[r] = ladder ? rl : rk[r];
          }
          dq = ladder ? 1.0 : dq;
          solved = ladder ? good : solved;
        }
      }
      fail_row = act && (bad || !solved);
      stamp(7);
      // gains: K = -rk (lanes < 12); k = -(M + eps I)^-1 Qu = -D M'^-1 (D Qu) on lanes
      // 12..15, with M'^-1 y = y - sum_j y_j rj[j] (M' has unit diagonal, so |M'^-1 y|
      // >= |y| / 4: no cancellation)
      const double yq = dq * qu;
      double kv = -yq;
      LaneDotOff<MM, S>::fma(kv, yq, rj);
      kv *= dq;
      stamp(8);
      if constexpr (MODE == 0) {
        LaneDotOff<MM, S>::fma_neg(vxn, qu, rk);  // + K^T Qu
        LaneDotOff<MM, S>::fma(vxn, kv, P);       // + Qux^T k
        double qk = 0.0;
        LaneDotOff<MM, S>::fma(qk, kv, PT);       // (Quu k) on lanes 12..15
        LaneDotOff<MM, S>::fma_neg(vxn, qk, rk);  // + K^T Quu k
        double QK[MM];
        copy(QK, P);
        static_for<MM>([&](auto R) { LaneDotOff<MM, S>::fma_neg(QK[R], P[R], rk); });  // Qux + Quu K
        static_for<S>([&](auto R) {
          ColChain<MM>::template fma_negq<R>(Vn[R], rk, QK);  // + K^T (Qux + Quu K)
          ColChain<MM>::template fma_negq<R>(Vn[R], P, rk);   // + Qux^T K
        });
      } else {
        static_for<S>([&](auto R) {  // Qxx - Qux^T Quu^-1 Qux
          ColChain<MM>::template fma_negq<R>(Vn[R], P, rk);
        });
        LaneDotOff<MM, S>::fma(vxn, kv, P);  // Qx - Qux^T Quu^-1 Qu
        v0n = l0 + v0 + 0.5 * lane_sum_off<MM, S>(qu * kv);
      }
#pragma unroll
      for (int r = 0; r < MM; ++r) {
        Uq[r] = P[r];
        Kq[r] = rk[r];
      }
      kvq = kv;
    } else {
      // Q + A^T V A is accumulated into Qxx under the Quu^-1 sweep below
      double QB[MM];
      zero(QB);
      static_for<MM>([&](auto R) {  // B^T V [A|B]
        ColChain<S>::template fmaq<S + R>(QB[R], ab, VA);
      });
      double Qux[MM], Quu[MM];
#pragma unroll
      for (int r = 0; r < MM; ++r) {
        Qux[r] = QB[r];                                    // B^T V A   (lanes < n)
        Quu[r] = rcol[r] + ror_row<kRowLanes - S>(QB[r]);  // R + B^T V B (lanes < m)
      }
      // regularised solve
      stamp(5);
      double QuuT[MM];
      lds_transpose<MM>(Quu, QuuT, twa, tra);
      stamp(6);
      // First attempt as one offset-form asm sweep (SweepQ, the hot LFT kernel's
      // block): the diagonal carries (value - 1), the sweep returns -(M+eps I)^-1 + I
      // and its minimum pivot -- chol_solve's first try (eps = 1e-9; mode 1 at
      // lam = max(lm, 1e-12)).  Mode 0's jitter-free cholesky(Quu_reg) check
      // (solver.py:211-219) follows from the same sweep whenever
      // trace((M + eps I)^-1) < 1e6: then lambda_min(M) > 1e-6 - eps > 0.  Rows
      // outside that bound get the exact check (a second sweep without jitter), rows
      // whose first try fails the generic jitter / lambda ladders (hop_device.hpp);
      // both rare, wave-uniform branches.
      double Qi[MM], Qs[MM];
      bool solved;
      {
        const double lam1 = MODE == 0 ? lam0 : (lam0 > 1e-12 ? lam0 : 1e-12);
        double rj[MM];
#pragma unroll
        for (int r = 0; r < MM; ++r) {
          Qs[r] = 0.5 * (Quu[r] + QuuT[r]);
          rj[r] = Qs[r] + ((c == r) ? lam1 + (1e-9 - 1.0) : 0.0);
        }
        double dj = 1.0;
        // the sweep fused with Qxx = Q + A^T V A (lanes < n; A^T V B on lanes n..):
        // the 144 chain FMAs fill the pivots' rcp / Newton latency
        SweepQColChain<MM, S>::run(rj, dj, Qxx, ab, VA);
        const bool okj = (dj > 0.0) && (bcast<0>(rj[0]) == bcast<0>(rj[0]));
#pragma unroll
        for (int r = 0; r < MM; ++r) Qi[r] = ((c == r) ? 1.0 : 0.0) - rj[r];  // +(M+eps I)^-1
        bool ok0 = true;
        if constexpr (MODE == 0) {
          const double tr = diag_sum4(Qi);  // trace((M + eps I)^-1)
          const bool sure = okj && (tr < 1e6);
          if (__any(!sure && act)) {  // the exact jitter-free check (rows that step)
            double rc[MM];
#pragma unroll
            for (int r = 0; r < MM; ++r) rc[r] = Qs[r] + ((c == r) ? lam1 - 1.0 : 0.0);
            double dc = 1.0;
            SweepQ<MM>::run(rc, dc);
            const bool okc = (dc > 0.0) && (bcast<0>(rc[0]) == bcast<0>(rc[0]));
            ok0 = sure || okc;
          }
        }
        solved = okj && ok0;
        if (__any(!okj && ok0 && act)) {  // the jitter / lambda ladders for the rows that need them
          const bool ladder = !okj && ok0;
          if constexpr (MODE == 0) {
            double Ql[MM];
#pragma unroll
            for (int r = 0; r < MM; ++r) Ql[r] = Qs[r] + ((c == r) ? lam0 : 0.0);
            bool okc = true;
            const bool good = spd_inverse_nofallback_chk(Ql, tile, c, 8, st, okc) && okc;
#pragma unroll
            for (int r = 0; r < MM; ++r) Qi[r] = ladder ? Ql[r] : Qi[r];
            solved = ladder ? good : solved;
          } else {
            double lam = lam1;
            int tries = 0;
            bool okr = false;
            double Ql[MM];
#pragma unroll 1
            while (true) {
#pragma unroll
              for (int r = 0; r < MM; ++r) Ql[r] = Qs[r] + ((c == r) ? lam : 0.0);
              okr = spd_inverse_nofallback(Ql, tile, c, 8, st);
              ++tries;
              const bool done = okr || tries >= a.reg_max_tries;
              if (!__any(!done && act && ladder)) break;
              if (!done) lam *= 10.0;
            }
#pragma unroll
            for (int r = 0; r < MM; ++r) Qi[r] = ladder ? Ql[r] : Qi[r];
            solved = ladder ? okr : solved;
          }
        }
      }
      fail_row = act && (bad || !solved);
      stamp(7);
      // gains
      double K[MM];
      zero(K);
      static_for<MM>([&](auto R) { LaneDot<MM>::fma_neg(K[R], Qi[R], Qux); });  // -Quu_reg^-1 Qux
      double kv = 0.0;
      LaneDot<MM>::fma_neg(kv, qu, Qi);          // k = -Quu_reg^-1 Qu  (lanes < m)
      stamp(8);
      // value update
      if constexpr (MODE == 0) {
        LaneDot<MM>::fma(vxn, qu, K);    // + K^T Qu
        LaneDot<MM>::fma(vxn, kv, Qux);  // + Qux^T k
        double qk = 0.0;
        LaneDot<MM>::fma(qk, kv, QuuT);  // (Quu k)[c]
        LaneDot<MM>::fma(vxn, qk, K);    // + K^T Quu k
        double QK[MM];
        copy(QK, Qux);
        static_for<MM>([&](auto R) { LaneDot<MM>::fma(QK[R], Quu[R], K); });  // Qux + Quu K
        static_for<S>([&](auto R) {
          ColChain<MM>::template fmaq<R>(Vn[R], K, QK);    // + K^T (Qux + Quu K)
          ColChain<MM>::template fmaq<R>(Vn[R], Qux, K);   // + Qux^T K
        });
      } else {
        static_for<S>([&](auto R) {  // Qxx - Qux^T Quu^-1 Qux
          ColChain<MM>::template fmaq<R>(Vn[R], Qux, K);
        });
        LaneDot<MM>::fma(vxn, kv, Qux);             // Qx - Qux^T Quu^-1 Qu
        v0n = l0 + v0 + 0.5 * lane_sum<MM>(qu * kv);
      }

#pragma unroll
      for (int r = 0; r < MM; ++r) {
        Uq[r] = Qux[r];
        Kq[r] = K[r];
      }
      kvq = kv;
    }
    stamp(9);
    lds_park12(Vn, twa);  // its transpose is read with the next step's image
    stamp(10);
    // finiteness of the update: x * 0 is 0 for finite x, NaN otherwise.
    // value_expansions (horizon_selection.py:209-210) raises on any non-finite V;
    // the brute-force curve only through the next step's chol_solve (Vxx, Vx: never
    // V_0), and at t = 0 only through chol_solve(Quu_reg, Qux) itself
    double z = __builtin_fma(vxn, 0.0, JC ? 0.0 : v0n * 0.0);
#pragma unroll
    for (int r = 0; r < S; ++r) z = __builtin_fma(Vn[r], 0.0, z);
    if (JC && i == 0) {
      z = 0.0;
#pragma unroll
      for (int r = 0; r < MM; ++r) z = __builtin_fma(Uq[r], 0.0, z);
    }
    const unsigned long long vbm = __ballot(!(z == z) && c < S);
    const bool vfail = act && (((vbm >> (16 * g)) & 0xffffull) != 0ull);
    const bool commit = act && !fail_row && !vfail;
    if (act && (fail_row || vfail)) {
      st |= ST_FAIL;
      if (bad || vfail) st |= ST_NONFINITE;
      alive = false;
    }
    if (__any(!commit)) {  // a row keeps its V: carry and park that instead (rare but
                           // for rows waiting for their horizon to start)
#pragma unroll
      for (int r = 0; r < S; ++r) Vp[r] = commit ? Vn[r] : V[r];
      lds_park12(Vp, twa);
    } else {
#pragma unroll
      for (int r = 0; r < S; ++r) Vp[r] = Vn[r];
    }
    cprev = commit;
    vx = commit ? vxn : vx;
    v0 = commit ? v0n : v0;
    stamp(11);
    // stores: every lane issues them (fixed count for vm_wait_n), lanes that do
    // not commit address out of range (dropped by the descriptor's range check)
    if constexpr (EXP != 1 && !JC) {
      const bool wr = commit && c < S;
      const unsigned so = (unsigned)i * (MM * S * 8), vo = wr ? voK : OOB;
#pragma unroll
      for (int r = 0; r < MM; ++r) st64(PK ? -Kq[r] : Kq[r], rK, vo + 8u * S * r, so);
      st64(kvq, rk, (commit && (PK ? c >= S : c < MM)) ? vok : OOB, (unsigned)i * (MM * 8));
      if constexpr (WANTV) {
        st64(vxn, rVx, wr ? voVx : OOB, (unsigned)i * (S * 8));
        st64(v0n, rV0, (commit && c == 0) ? voV0 : OOB, (unsigned)i * 8);
      }
    }
    stamp(1);  // section 1 = stores (closed here), reopened at the step top
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, OCC2 ? 0 : BUF>;
  if (Lw > 0) {
    const int i0 = Lw - 1;
    dma9<0>(va, vb, vx_, vu_, rA, rB, rX, rU, wlds, (unsigned)i0 * (S * S * 8),
            (unsigned)i0 * (S * MM * 8), (unsigned)i0 * (S * 8), (unsigned)i0 * (MM * 8));
    using T1 = std::true_type;
    using F0 = std::false_type;
    step(i0, I0{}, T1{});
    int i = i0 - 1;
#pragma unroll 1
    while (i >= 1) {
      step(i, I1{}, F0{});
      step(i - 1, I0{}, F0{});
      i -= 2;
    }
    if (i == 0) step(0, I1{}, F0{});
    if constexpr (WANTV) {  // Vxx of step 0
      double t[S];
      lds_read_t12(t, tra);
      const bool wr = cprev && c < S;
#pragma unroll
      for (int r = 0; r < S; ++r) st64(0.5 * (Vp[r] + t[r]), rVxx, wr ? voVxx + 8u * S * r : OOB, 0u);
    }
  }
  vm_wait();
  if constexpr (STAMP) {
    if (lane == 0) {
      for (int j = 0; j < 12; ++j) atomicAdd(&g_ricf_stamp[j], sec[j]);
      atomicAdd(&g_ricf_stamp[15], 1ull);
    }
  }
  if (valid && c == 0) {
    if constexpr (JC) {  // V_0 of this horizon's sweep (the reference raises on failure: NaN)
      const long long o = prob * a.jc_tmax + (L - 1);
      a.jc_J[o] = alive ? v0 : NAN;
      a.jc_status[o] = (int)st;
    } else {
      a.status[prob] = (int)st;
    }
  }
}

// OCC2: the two-waves-per-SIMD layout of the J curve (below) for batches that give a
// SIMD more than one wave (a batch-shared Q; launch() picks it)
template <int MODE, bool WANTV, bool STAMP = false, int EXP = 0, bool PK = true, bool OCC2 = false,
          bool QL = true>
__global__ __launch_bounds__(256, OCC2 ? 2 : 1) void riccati_fast_kernel(RiccatiArgs<double> a) {
  ric_body<MODE, WANTV, STAMP, EXP, false, PK, OCC2, QL>(a, (long long)blockIdx.x, 0);
}

// The J-curve form: workgroups [b * P, (b+1) * P), P = ceil(jc_tmax / 2), run problem
// block b; workgroup h sweeps horizon jc_tmax - h and then h + 1, so every wave runs
// the same jc_tmax + 1 steps (11 % faster than one horizon per workgroup, longest
// first) and a block's horizons sit in adjacent workgroups (its A, B, x, u re-reads
// meet in the caches)
// XCD: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup
// dispatch), so consecutive ids -- one problem block's horizons -- land on 8 different
// L2s and each re-reads the block's A, B, x, u from HBM.  The remap gives the ids an
// XCD receives (w = x, x + 8, x + 16, ...) consecutive logical ids, so a block's
// horizons share one L2.
// OCC2 (the default for a batch-shared Q): 247 VGPRs and 19,456 B of LDS per wave
// (one step image, one Q image, Q's rows re-read from it per step), so two 4-wave
// workgroups share a CU and each SIMD interleaves two waves' dependent DPP chains:
// 1.31x the one-wave layout at the bench shape, bit-identical (round 3).  With the HBM
// stream now at 4 TB/s (27.9 GB per launch: every XCD's L2 re-reads each block), the
// XCD grouping above pays: 0.75 GB per launch and 6.8 % faster (default with OCC2).
template <bool XCD, bool PK = true, bool OCC2 = false>
__global__ __launch_bounds__(256, OCC2 ? 2 : 1) void riccati_fast_jcurve_kernel(RiccatiArgs<double> a) {
  const unsigned P = (unsigned)((a.jc_tmax + 1) / 2);
  unsigned w = blockIdx.x;
  if constexpr (XCD) {
    const unsigned G8 = gridDim.x / 8u * 8u;  // a remainder keeps its ids
    if (w < G8) w = (w % 8u) * (G8 / 8u) + w / 8u;
  }
  const int h = (int)(w % P);
  const long long blk = (long long)(w / P);
  ric_body<1, false, false, 0, true, PK, OCC2>(a, blk, a.jc_tmax - h);
  if (h + 1 < a.jc_tmax - h) ric_body<1, false, false, 0, true, PK, OCC2>(a, blk, h + 1);
}

template <int MODE, bool WANTV>
hipError_t launch(const RiccatiArgs<double>& a, hipStream_t stream) {
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  const size_t lds = (size_t)kWavesPerBlock * WAVE_BYTES;
#ifdef HOP_DEV
  if (opt(HOP_OPT_STAMPS)) {
    hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV, true>), dim3((unsigned)blocks),
                       dim3(256), lds, stream, a);
    return hipGetLastError();
  }
  if (g_opt_variant == 81 || g_opt_variant == 82) {
    if (g_opt_variant == 81)
      hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV, false, 1>), dim3((unsigned)blocks),
                         dim3(256), lds, stream, a);
    else
      hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV, false, 2>), dim3((unsigned)blocks),
                         dim3(256), lds, stream, a);
    return hipGetLastError();
  }
  if (g_opt_variant == 84) {  // separate Qux / Quu rows (the round-3 schedule, A/B)
    hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV, false, 0, false>), dim3((unsigned)blocks),
                       dim3(256), lds, stream, a);
    return hipGetLastError();
  }
  if (g_opt_variant == 96) {  // Q image read with the step's other reads (A/B)
    hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV, false, 0, true, false, false>),
                       dim3((unsigned)blocks), dim3(256), lds, stream, a);
    return hipGetLastError();
  }
  const bool force1 = g_opt_variant == 89, force2 = g_opt_variant == 90;  // layouts (A/B)
#else
  constexpr bool force1 = false, force2 = false;
#endif
  // mode 0 (K, k only), more waves than SIMDs and a batch-shared Q: two waves per SIMD
  // (OCC2), which hides the dependent chains' latency the one-wave layout exposes (B =
  // 32,768: 1.818 -> 1.540 ms).  Mode 1 streams Vxx and is HBM-bound: two waves were
  // 4 % slower there (2.376 -> 2.476 ms), so it keeps one wave per SIMD.
  constexpr bool occ2_mode = MODE == 0 && !WANTV;
  if (occ2_mode && a.q_bstride == 0 && !force1 &&
      (force2 || (a.batch + kProbPerWave - 1) / kProbPerWave > 4ll * cu_count(stream))) {
    hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV, false, 0, true, occ2_mode>),
                       dim3((unsigned)blocks), dim3(256),
                       (size_t)kWavesPerBlock * (occ2_mode ? WAVE_BYTES2 : WAVE_BYTES), stream, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((riccati_fast_kernel<MODE, WANTV>), dim3((unsigned)blocks), dim3(256), lds,
                     stream, a);
  return hipGetLastError();
}

}  // namespace ricf

// n = 12, m = 4 fp64 without the extra stage-cost terms -> the exact-size kernel;
// anything else -> hipErrorNotSupported (the caller runs the generic kernel)
hipError_t dispatch_riccati_fast(const RiccatiArgs<double>& a, hipStream_t stream) {
  if (a.n != ricf::NX || a.m != ricf::MU || a.qxx_extra || a.qx_extra || a.c_extra)
    return hipErrorNotSupported;
  // 32-bit buffer offsets: the per-wave tensors must stay below 4 GiB
  // 32-bit buffer offsets: a wave's 4 problems must stay below 2 GiB per tensor
  // (out-of-range store offsets start at 2 GiB)
  const long long NA = a.nalloc;
  if (4 * (NA + 1) * ricf::NX * ricf::NX * 8 >= 0x7FFF0000ll) return hipErrorNotSupported;
  if (a.jc_J) {  // the J-curve form: one launch, ceil(jc_tmax / 2) workgroups per block
    const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
    const dim3 grid((unsigned)(blocks * ((a.jc_tmax + 1) / 2)));
    const size_t lds = (size_t)kWavesPerBlock * ricf::WAVE_BYTES;
#ifdef HOP_DEV
    if (g_opt_variant == 83) {  // XCD-grouped horizons (A/B)
      hipLaunchKernelGGL(ricf::riccati_fast_jcurve_kernel<true>, grid, dim3(256), lds, stream, a);
      return hipGetLastError();
    }
    if (g_opt_variant == 84) {  // separate Qux / Quu rows (A/B)
      hipLaunchKernelGGL((ricf::riccati_fast_jcurve_kernel<false, false>), grid, dim3(256), lds,
                         stream, a);
      return hipGetLastError();
    }
    if (g_opt_variant == 88 && a.q_bstride == 0) {  // two waves per SIMD, round-robin XCDs (A/B)
      hipLaunchKernelGGL((ricf::riccati_fast_jcurve_kernel<false, true, true>), grid, dim3(256),
                         (size_t)kWavesPerBlock * ricf::WAVE_BYTES2, stream, a);
      return hipGetLastError();
    }
    if (g_opt_variant == 86) {  // one wave per SIMD with a batch-shared Q (A/B)
      hipLaunchKernelGGL(ricf::riccati_fast_jcurve_kernel<false>, grid, dim3(256), lds, stream, a);
      return hipGetLastError();
    }
#endif
    if (a.q_bstride == 0) {  // a batch-shared Q: two waves per SIMD (OCC2), XCD-grouped horizons
      hipLaunchKernelGGL((ricf::riccati_fast_jcurve_kernel<true, true, true>), grid, dim3(256),
                         (size_t)kWavesPerBlock * ricf::WAVE_BYTES2, stream, a);
      return hipGetLastError();
    }
    hipLaunchKernelGGL(ricf::riccati_fast_jcurve_kernel<false>, grid, dim3(256), lds, stream, a);
    return hipGetLastError();
  }
  if (a.mode == 1) return ricf::launch<1, true>(a, stream);
  return a.Vxx ? ricf::launch<0, true>(a, stream) : ricf::launch<0, false>(a, stream);
}

}  // namespace hop

// Diagnostic (not part of include/hop.h): read (and optionally reset) the section
// stamps of the exact-size Riccati kernel (HOP_OPT_STAMPS, developer builds).
extern "C" int hop_debug_ricf_stamps(unsigned long long* host16, int reset) {
  if (hipMemcpyFromSymbol(host16, HIP_SYMBOL(hop::ricf::g_ricf_stamp),
                          16 * sizeof(unsigned long long)) != hipSuccess)
    return -3;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hop::ricf::g_ricf_stamp), z, sizeof(z)) != hipSuccess)
      return -3;
  }
  return 0;
}
