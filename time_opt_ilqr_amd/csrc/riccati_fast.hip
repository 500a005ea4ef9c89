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
constexpr int WAVE_BYTES = OFF_T + kProbPerWave * kLdsTile * 8;

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

// the step's 9 LDS-DMA pieces (A 5, B 2, x, u) in one asm block; M0 saved once
// and set per piece from the wave's LDS base plus an immediate
template <int IMG>
__device__ __forceinline__ void dma9(const unsigned (&va)[5], const unsigned (&vb)[2], unsigned vx,
                                     unsigned vu, __amdgpu_buffer_rsrc_t rA,
                                     __amdgpu_buffer_rsrc_t rB, __amdgpu_buffer_rsrc_t rX,
                                     __amdgpu_buffer_rsrc_t rU, unsigned wlds, unsigned sA,
                                     unsigned sB, unsigned sX, unsigned sU) {
  unsigned keep;
#define HOP_P(R, V, OFF, SO)                                                  \
  "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\tbuffer_load_dwordx4 %[" #V "], %[" #R \
  "], %[" #SO "] offen lds\n\t"
  asm volatile(
      "s_mov_b32 %[keep], m0\n\t"
      HOP_P(ra, a0, %[o0], sa) HOP_P(ra, a1, %[o1], sa) HOP_P(ra, a2, %[o2], sa)
      HOP_P(ra, a3, %[o3], sa) HOP_P(ra, a4, %[o4], sa)
      HOP_P(rb, b0, %[p0], sb) HOP_P(rb, b1, %[p1], sb)
      HOP_P(rx, x0, %[ox], sx) HOP_P(ru, x1, %[ou], su)
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [w] "s"(wlds), [sa] "s"(sA), [sb] "s"(sB), [sx] "s"(sX), [su] "s"(sU),
        [ra] "s"(rA), [rb] "s"(rB), [rx] "s"(rX), [ru] "s"(rU),
        [a0] "v"(va[0]), [a1] "v"(va[1]), [a2] "v"(va[2]), [a3] "v"(va[3]), [a4] "v"(va[4]),
        [b0] "v"(vb[0]), [b1] "v"(vb[1]), [x0] "v"(vx), [x1] "v"(vu),
        [o0] "i"(IMG + OFF_A), [o1] "i"(IMG + OFF_A + 1024), [o2] "i"(IMG + OFF_A + 2048),
        [o3] "i"(IMG + OFF_A + 3072), [o4] "i"(IMG + OFF_A + 4096), [p0] "i"(IMG + OFF_B),
        [p1] "i"(IMG + OFF_B + 1024), [ox] "i"(IMG + OFF_X), [ou] "i"(IMG + OFF_U)
      : "memory", "scc");
#undef HOP_P
}

// [A|B] rows (12 registers, column c per lane), x_c and u_c from image IMG:
// 14 ds_read_b64 in flight, one wait, one asm statement (early-clobber outputs)
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

__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  const unsigned nrec = bytes > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (unsigned)(bytes > 0 ? bytes : 0);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nrec,
                                           0x00020000);
}

__device__ __forceinline__ void st64(double v, __amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
  __builtin_amdgcn_raw_buffer_store_b64(as_u2(v), r, vo, so, 0);
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void riccati_fast_kernel(RiccatiArgs<double> a) {
  constexpr int S = NX, MM = MU;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned char* wbase = smem_raw + w * WAVE_BYTES;
  const unsigned wlds = (unsigned)(uintptr_t)wbase;
  double* tile = reinterpret_cast<double*>(wbase + OFF_T) + g * kLdsTile;
#pragma unroll 1
  for (int i = c; i < kLdsTile; i += kRowLanes) tile[i] = 0.0;

  const long long wave_prob0 = ((long long)blockIdx.x * kWavesPerBlock + w) * kProbPerWave;
  const long long prob = wave_prob0 + g;
  const bool valid = prob < a.batch;
  const long long pb = valid ? prob : a.batch - 1;
  if (wave_prob0 >= a.batch) return;  // wave-uniform; no workgroup barrier in this kernel
  const long long pb0 = wave_prob0;
  const int NA = a.nalloc;
  const long long left = a.batch - pb0;

  // buffer descriptors based at the wave's first problem (exact bounds: OOB reads 0,
  // OOB writes dropped)
  const long long pA = (long long)NA * S * S * 8, pB = (long long)NA * S * MM * 8;
  const long long pX = (long long)(NA + 1) * S * 8, pU = (long long)NA * MM * 8;
  const __amdgpu_buffer_rsrc_t rA = rsrc(a.A + pb0 * (pA / 8), left * pA),
                               rB = rsrc(a.Bm + pb0 * (pB / 8), left * pB),
                               rX = rsrc(a.X + pb0 * (pX / 8), left * pX),
                               rU = rsrc(a.U + pb0 * (pU / 8), left * pU);
  const long long pK = (long long)NA * MM * S * 8, pk = (long long)NA * MM * 8;
  const __amdgpu_buffer_rsrc_t rK = rsrc(a.K + pb0 * (pK / 8), left * pK),
                               rk = rsrc(a.k + pb0 * (pk / 8), left * pk);
  const long long pVxx = (long long)(NA + 1) * S * S * 8, pVx = (long long)(NA + 1) * S * 8,
                  pV0 = (long long)(NA + 1) * 8;
  const bool wantv = MODE == 1 || a.Vxx;
  unsigned va[5], vb[2], vx_, vu_;
#pragma unroll
  for (int j = 0; j < 5; ++j) va[j] = voff<CH_A>(j, lane, wave_prob0, pb0, a.batch, pA);
#pragma unroll
  for (int j = 0; j < 2; ++j) vb[j] = voff<CH_B>(j, lane, wave_prob0, pb0, a.batch, pB);
  vx_ = voff<CH_X>(0, lane, wave_prob0, pb0, a.batch, pX);
  vu_ = voff<CH_U>(0, lane, wave_prob0, pb0, a.batch, pU);
  // per-lane image addresses of [A|B] row j, x_c and u_c
  unsigned ad[S];
#pragma unroll
  for (int j = 0; j < S; ++j)
    ad[j] = wlds + (c < S ? OFF_A + 1152 * g + 8 * c + 96 * j
                          : OFF_B + 384 * g + 8 * (c - S) + 32 * j);
  const unsigned xa = wlds + OFF_X + 96 * g + 8 * (c < S ? c : 0);
  const unsigned ua = wlds + OFF_U + 32 * g + 8 * (c < MM ? c : 0);
  // per-lane store offsets (problem part; the step part is the scalar offset)
  const unsigned pofs = (unsigned)(pb - pb0);
  const unsigned voK = pofs * (unsigned)pK + 8u * (c < S ? c : 0);
  const unsigned vok = pofs * (unsigned)pk + 8u * (c < MM ? c : 0);

  const double* xgp = a.xg + pb * a.xg_bstride;
  const double* urp = a.u_ref + pb * a.uref_bstride;
  const double* Qp = a.Q + pb * a.q_bstride;
  const double* Rp = a.R + pb * a.r_bstride;
  const double* Qfp = a.Qf + pb * a.qf_bstride;
  const int L = valid ? a.horizon[pb] : 0;
  int Lw = L;
  Lw = max(Lw, __shfl_xor(Lw, 16));
  Lw = max(Lw, __shfl_xor(Lw, 32));
  Lw = __builtin_amdgcn_readfirstlane(Lw);
  Lw = Lw < NA ? Lw : NA;
  const double lam0 = a.lm[pb];

  // loop-invariant cost blocks in registers: Q column c / row c, R column / row
  const int cq = c < S ? c : 0, cr = c < MM ? c : 0;
  double qcol[S], qrow[S], rcol[MM], rrow[MM];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    qcol[i] = c < S ? Qp[i * S + cq] : 0.0;
    qrow[i] = c < S ? Qp[cq * S + i] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < MM; ++i) {
    rcol[i] = c < MM ? Rp[i * MM + cr] : ((i == c) ? 1.0 : 0.0);
    rrow[i] = c < MM ? Rp[cr * MM + i] : ((i == c) ? 1.0 : 0.0);
  }
  const double xg_c = c < S ? xgp[cq] : 0.0;
  const double ur_c = c < MM ? urp[cr] : 0.0;
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
    v0 = 0.5 * row_sum_dpp(c < S ? eT * vx : 0.0);
    symmetrize(V, tile, c);
    if (alive && wantv) {
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

  // one step (index i) reading image IMG; issues the DMA of step i-1 into the
  // other image first
  auto step = [&](int i, auto IMGc) {
    constexpr int IMG = decltype(IMGc)::value;
    constexpr int NEXT = IMG == 0 ? BUF : 0;
    vm_wait();  // this step's pieces landed (and the previous step's stores left)
    if (i > 0)
      dma9<NEXT>(va, vb, vx_, vu_, rA, rB, rX, rU, wlds, (unsigned)(i - 1) * (S * S * 8),
                 (unsigned)(i - 1) * (S * MM * 8), (unsigned)(i - 1) * (S * 8),
                 (unsigned)(i - 1) * (MM * 8));
    double ab[S], xi, ui;
    read_step<IMG>(ad, xa, ua, ab, xi, ui);
    const bool act = alive && (i < L);
    double e = c < S ? xi - xg_c : 0.0;
    if (wrap_c) e = wrap_angle(e);
    const double du = c < MM ? ui - ur_c : 0.0;
    const unsigned long long badm = __ballot(!(finite_val(e) && finite_val(du)));
    const bool bad = ((badm >> (16 * g)) & 0xffffull) != 0ull;

    // lx = Q e, lu = R du (lanes < n / < m)
    double lx = 0.0, lu = 0.0;
    LaneDot<S>::fma(lx, e, qrow);
    LaneDot<MM>::fma(lu, du, rrow);
    double l0 = 0.0;
    if constexpr (MODE == 1)
      l0 = 0.5 * row_sum_dpp(c < S ? e * lx : 0.0) + 0.5 * row_sum_dpp(c < MM ? du * lu : 0.0) +
           a.w_stage;
    // Q-function: qab = [A|B]^T Vx; VA = V [A|B]; [A|B]^T V [A|B]
    double qab = 0.0;
    LaneDot<S>::fma(qab, vx, ab);
    const double qx = lx + qab;                          // Qx = lx + A^T Vx (lanes < n)
    const double qu = lu + ror_row<kRowLanes - S>(qab);  // Qu = lu + B^T Vx (lanes < m)
    double VA[S];
    zero(VA);
    acc_xy<false>(VA, V, ab);
    double Qxx[S];
    copy(Qxx, qcol);
    acc_xty<false>(Qxx, ab, VA);  // Q + A^T V A (lanes < n)
    double QB[MM];
    zero(QB);
    static_for<S>([&](auto J) { LaneBOff<MM, S>::fma(QB, ab[J], VA[J]); });  // B^T V [A|B]
    double Qux[MM], Quu[MM];
#pragma unroll
    for (int r = 0; r < MM; ++r) {
      Qux[r] = QB[r];                                    // B^T V A   (lanes < n)
      Quu[r] = rcol[r] + ror_row<kRowLanes - S>(QB[r]);  // R + B^T V B (lanes < m)
    }
    // regularised solve
    double QuuT[MM];
    transpose(QuuT, Quu, tile, c);
    double Qi[MM];
    bool solved;
    if constexpr (MODE == 0) {
#pragma unroll
      for (int r = 0; r < MM; ++r) Qi[r] = 0.5 * (Quu[r] + QuuT[r]) + ((c == r) ? lam0 : 0.0);
      bool ok = true;
      solved = spd_inverse_nofallback_chk(Qi, tile, c, 8, st, ok) && ok;
    } else {
      double lam = lam0 > 1e-12 ? lam0 : 1e-12;
      int tries = 0;
#pragma unroll 1
      while (true) {
#pragma unroll
        for (int r = 0; r < MM; ++r) Qi[r] = 0.5 * (Quu[r] + QuuT[r]) + ((c == r) ? lam : 0.0);
        const bool okr = spd_inverse_nofallback(Qi, tile, c, 8, st);
        ++tries;
        solved = okr;
        const bool done = okr || tries >= a.reg_max_tries;
        if (!__any(!done && act)) break;
        if (!done) lam *= 10.0;
      }
    }
    const bool fail_row = act && (bad || !solved);
    // gains
    double K[MM];
    zero(K);
    acc_xy<true, double, MM, MM>(K, Qi, Qux);  // K = -Quu_reg^-1 Qux (column c)
    double kv = 0.0;
    LaneDot<MM>::fma_neg(kv, qu, Qi);          // k = -Quu_reg^-1 Qu  (lanes < m)
    // value update
    double Vn[S];
    copy(Vn, Qxx);
    double vxn = qx, v0n = v0;
    if constexpr (MODE == 0) {
      LaneDot<MM>::fma(vxn, qu, K);    // + K^T Qu
      LaneDot<MM>::fma(vxn, kv, Qux);  // + Qux^T k
      double qk = 0.0;
      LaneDot<MM>::fma(qk, kv, QuuT);  // (Quu k)[c]
      LaneDot<MM>::fma(vxn, qk, K);    // + K^T Quu k
      double QK[MM];
      copy(QK, Qux);
      acc_xy<false, double, MM, MM>(QK, Quu, K);  // Qux + Quu K
      acc_xty<false, double, S, MM>(Vn, K, QK);   // + K^T (Qux + Quu K)
      acc_xty<false, double, S, MM>(Vn, Qux, K);  // + Qux^T K
    } else {
      acc_xty<false, double, S, MM>(Vn, Qux, K);  // Qxx - Qux^T Quu^-1 Qux
      LaneDot<MM>::fma(vxn, kv, Qux);             // Qx - Qux^T Quu^-1 Qu
      v0n = l0 + v0 + 0.5 * row_sum_dpp(c < MM ? qu * kv : 0.0);
    }
    symmetrize(Vn, tile, c);
    bool vbad = !finite_val(vxn) || !finite_val(v0n);
#pragma unroll
    for (int r = 0; r < S; ++r) vbad = vbad || !finite_val(Vn[r]);
    const unsigned long long vbm = __ballot(vbad && c < S);
    const bool vfail = act && (((vbm >> (16 * g)) & 0xffffull) != 0ull);
    const bool commit = act && !fail_row && !vfail;
    if (act && (fail_row || vfail)) {
      st |= ST_FAIL;
      if (bad || vfail) st |= ST_NONFINITE;
      alive = false;
    }
    if (commit) {
#pragma unroll
      for (int r = 0; r < S; ++r) V[r] = Vn[r];
      vx = vxn;
      v0 = v0n;
    }
    if (commit && c < S) {
      const unsigned so = (unsigned)i * (MM * S * 8);
#pragma unroll
      for (int r = 0; r < MM; ++r) st64(K[r], rK, voK + 8u * S * r, so);
      if (wantv) {
        const unsigned sv = (unsigned)i * (S * S * 8);
#pragma unroll
        for (int r = 0; r < S; ++r) st64(Vn[r], rVxx, voVxx + 8u * S * r, sv);
        st64(vxn, rVx, voVx, (unsigned)i * (S * 8));
      }
    }
    if (commit && c < MM) st64(kv, rk, vok, (unsigned)i * (MM * 8));
    if (wantv && commit && c == 0) st64(v0n, rV0, voV0, (unsigned)i * 8);
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, BUF>;
  if (Lw > 0) {
    const int i0 = Lw - 1;
    dma9<0>(va, vb, vx_, vu_, rA, rB, rX, rU, wlds, (unsigned)i0 * (S * S * 8),
            (unsigned)i0 * (S * MM * 8), (unsigned)i0 * (S * 8), (unsigned)i0 * (MM * 8));
    int i = i0;
#pragma unroll 1
    while (i >= 1) {
      step(i, I0{});
      step(i - 1, I1{});
      i -= 2;
    }
    if (i == 0) step(0, I0{});
  }
  vm_wait();
  if (valid && c == 0) a.status[prob] = (int)st;
}

template <int MODE>
hipError_t launch(const RiccatiArgs<double>& a, hipStream_t stream) {
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  const size_t lds = (size_t)kWavesPerBlock * WAVE_BYTES;
  hipLaunchKernelGGL((riccati_fast_kernel<MODE>), dim3((unsigned)blocks), dim3(256), lds, stream,
                     a);
  return hipGetLastError();
}

}  // namespace ricf

// n = 12, m = 4 fp64 without the extra stage-cost terms -> the exact-size kernel;
// anything else -> hipErrorNotSupported (the caller runs the generic kernel)
hipError_t dispatch_riccati_fast(const RiccatiArgs<double>& a, hipStream_t stream) {
  if (a.n != ricf::NX || a.m != ricf::MU || a.qxx_extra || a.qx_extra || a.c_extra)
    return hipErrorNotSupported;
  // 32-bit buffer offsets: the per-wave tensors must stay below 4 GiB
  const long long NA = a.nalloc;
  if (4 * (NA + 1) * ricf::NX * ricf::NX * 8 >= 0xFFFFFFF0ll) return hipErrorNotSupported;
  return a.mode == 0 ? ricf::launch<0>(a, stream) : ricf::launch<1>(a, stream);
}

}  // namespace hop
