// LFT horizon sweep, exact-size fp64 specialisation (s == S, m == MM) -- the
// hot kernel for the Quadrotor shape (s = 13, m = 4).  Same algorithm and
// outputs as lft_sweep.hip (horizon_selection.py:36-86), restructured for a
// wave that is alone on its SIMD (B = 4096 -> 1024 waves = 1 per SIMD):
//
//  * inputs of step k+1 (Q, A, B, QT) stream into per-wave LDS images by
//    LDS-DMA (buffer_load_dwordx4 ... lds, bounds-checked) while step k
//    computes; no VGPRs are held for prefetch.  Rows/columns of Q, QT, A^T and
//    B come straight from the image, so symmetrising inverse inputs and
//    forming A^T cost no extra transposes.
//  * every inverse is kept NEGATED (the sweep's native output, -M^-1) and the
//    sign is folded into the consuming broadcast-FMAs (fma_neg).
//  * offset form (Chain / Sched schedules): diagonals carry -1 + eps, applied
//    by one LDS atomic per lane on the parked input, so a Gauss-Jordan pivot
//    needs no lane-p fix-ups; inverses come out as -M^-1 + I and the +I is
//    absorbed by starting the consuming products from Y instead of 0.
//  * the query of horizon t needs only z0^T (X0 + eps I)^-1 z0, answered by a
//    bordered forward elimination with z0 as column S (lane S is free when
//    s < 16) -- no third inverse.
//  * Sched / SchedRow: each sweep is one hand-scheduled asm block in which the
//    dependent chain of pivot p+1 (broadcast, v_rcp_f64, Newton-folded scale)
//    is interleaved into the 13 broadcast-FMAs of pivot p.
//
// This file also holds the conditioned-prefix kernels (lft_cond_kernel,
// lft_cond_cf_kernel), the default for s = 13, m = 4, which hand
// the problems they cannot take to lft_sweep_v2_kernel in rerun mode.
//
// Schedules other than the defaults are compiled only in developer builds
// (HOP_DEV, build.py --dev) and selected by hop_set_options' variant number:
//   2  Select : compiler-scheduled pivots with lane-p selects (first v2)
//   8  Chain  : offset form, short C++ pivot chain, pad-free DPP blocks
//   10 Sched  : offset form, whole-sweep asm blocks
//   12 SchedRow: Sched + X*Y products as one dependent DPP chain per output
//      row (accumulator forwarded: 4.0 vs 4.9 cycles per FMA)
//   14 SchedLdl: SchedRow + the query's Wt = (QT^-1 + Gbar)^-1 and its two
//      products replaced by one LDL^T elimination that streams X0
//   30 SchedLdlDma: SchedLdl with the step's LDS-DMA pieces from one asm block
//      (the reference association; the rerun path of the conditioned kernels)
//   20 / 32 stamped SchedLdl / SchedLdlDma (diagnostic, tools/stamps.py)
//   40 (default) conditioned prefix SchedCondL + rerun; 41 without the rerun;
//   42 its stamps (tools/stamps.py --cond); 43 SchedCond (no LDS reads inside
//   the sweep blocks).  Trajectory form: 53 (default) closed-form stage
//   inverses + rerun, 54 without; 40 / 41 Gauss-Jordan stage inverses; 24
//   stamped SchedLdlTraj.
#include <stdlib.h>

#include "hop_device.hpp"
#include "hop_kernels.hpp"

namespace hop {
namespace v2 {

// v_rcp_f64 + NR Newton steps (NR = 1 checked against the IEEE-division
// generic kernel at 1e-10 in tests)
template <int NR>
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
  }
  return r;
}

// lanes whose row-local index equals P: bits P, P+16, P+32, P+48 (an SGPR constant)
template <int P>
__device__ __forceinline__ double sel_lane(double a, double b) {
  constexpr unsigned long long mask = 0x0001000100010001ull << P;
  const int2 x = __builtin_bit_cast(int2, a), y = __builtin_bit_cast(int2, b);
  int2 r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.x) : "v"(x.x), "v"(y.x), "s"(mask));
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r.y) : "v"(x.y), "v"(y.y), "s"(mask));
  return __builtin_bit_cast(double, r);
}

// Schedules.  PIV: 0 select pivots, 4 short C++ chain, 5 whole-sweep asm.
struct Select {
  static constexpr int PIV = 0, NR = 1, LDSASM = 0, ELIM = 0, STAMP = 0, XYROW = 0, DMA1 = 0;
};
struct Chain {
  static constexpr int PIV = 4, NR = 1, LDSASM = 1, ELIM = 1, STAMP = 0, XYROW = 0, DMA1 = 0;
};
struct Sched {
  static constexpr int PIV = 5, NR = 1, LDSASM = 1, ELIM = 1, STAMP = 0, XYROW = 0, DMA1 = 0;
};
struct SchedRow : Sched {  // X*Y products as one dependent chain per output row
  static constexpr int XYROW = 1;
};

struct SchedLdl : SchedRow {  // + query by LDL^T elimination with row ops and rank-1 streams
  static constexpr int QLDL = 1;
};
template <class C>
constexpr bool has_qldl() {
  if constexpr (requires { C::QLDL; }) return C::QLDL != 0;
  return false;
}
struct SchedStamped : SchedLdl {
  static constexpr int STAMP = 1;
};
// trajectory form: the augmented blocks are built in LDS from the raw
// linearisation each step (augmented.py:10-87), see the TRAJ paths below
struct SchedLdlTraj : SchedLdl {
  static constexpr int TRAJ = 1;
  static constexpr int SCALE = 1;  // equilibrated Gauss-Jordan inverses (see sweep)
};
struct SchedLdlTrajStamped : SchedLdlTraj {
  static constexpr int STAMP = 1;
};
// the step's 20 LDS-DMA pieces issued from one asm block (dma_step20)
struct SchedLdlDma : SchedLdl {
  static constexpr int DMA1 = 1;
  static constexpr int SCALE = 1;  // equilibrated Gauss-Jordan inverses (see sweep)
};
struct SchedLdlDmaStamped : SchedLdlDma {
  static constexpr int STAMP = 1;
};
// conditioned-prefix kernel, augmented form (default): Sigma_{k+1} = A T as one
// dependent DPP chain per output row, rows of A_k read from the image with A^T's
struct SchedCond : SchedLdlDma {
  static constexpr int AROW = 1;
  static constexpr int SCALE = 0;  // first attempts only: its own sweeps (rerun on doubt)
};
#ifndef HOP_COND_DMAI
#define HOP_COND_DMAI 0  // A/B builds (tools/exp_build.py): the DMA pieces inside the update
#endif
constexpr bool kCondDmai = HOP_COND_DMAI != 0;
#ifndef HOP_FMA3
#define HOP_FMA3 0  // A/B builds: the congruence query's row offsets as inline-asm v_fma_f64
#endif
constexpr bool kFma3 = HOP_FMA3 != 0;
#ifndef HOP_COND_SWEEP2
#define HOP_COND_SWEEP2 0  // A/B: the s = 13 kernel's two sweeps as one interleaved block
#endif
constexpr bool kCondSweep2 = HOP_COND_SWEEP2 != 0;
#ifndef HOP_COND_MFMA64
#define HOP_COND_MFMA64 0  // A/B: the s = 13 fp64 predict on v_mfma_f64_16x16x4_f64
#endif
constexpr bool kCondMfma64 = HOP_COND_MFMA64 != 0;
#ifndef HOP_SMALL_SWEEP2
#define HOP_SMALL_SWEEP2 1  // small-s row groups: the two stage sweeps as one interleaved block
#endif
constexpr bool kSmallSweep2 = HOP_SMALL_SWEEP2 != 0;
// + the QT image reads under the E sweep, the A/B reads under the X sweep
#ifndef HOP_COND_WQ
#define HOP_COND_WQ 1  // developer A/B builds (tools/exp_build.py): 0 = round 3's query
#endif
struct SchedCondL : SchedCond {
  static constexpr int LDSPIPE = 1;
  static constexpr int WQ = HOP_COND_WQ;
};
template <class C>
constexpr bool has_ldspipe() {
  if constexpr (requires { C::LDSPIPE; }) return C::LDSPIPE != 0;
  return false;
}
struct SchedCondLStamped : SchedCondL {
  static constexpr int STAMP = 1;
};
// SYM2: the stage / terminal inverses of the UNHALVED symmetric sums (M + M^T:
// inverse (2M)^-1 = M^-1 / 2, exact), consumed as fma(-2, NE, X) by the update and
// the query with their diagonal offset at 2 (no 0.5 multiplies); the update's
// Newton step on the reciprocal (CondLdl2); and the predict as one block whose
// eps I rows come from LDS instead of lane selects (PredictEps)
struct SchedCondL2 : SchedCondL {
  static constexpr int SYM2 = 1, NEWT = 1, PEPS = 1;
};
struct SchedCondL2Stamped : SchedCondL2 {
  static constexpr int STAMP = 1;
};
// the three parts of SchedCondL2 alone (developer A/B)
struct SchedCondLSym : SchedCondL {  // the default since round 3
  static constexpr int SYM2 = 1, NEWT = 0, PEPS = 0;
};
// round 4: the query by congruence (the X sweep stops one pivot short; see the
// query below): the default of SchedCondL and its descendants; WQ = 0 keeps the
// round-3 query (developer variant 99, A/B)
template <class C>
constexpr bool has_wq() {
  if constexpr (requires { C::WQ; }) return C::WQ != 0;
  return false;
}
struct SchedCondLSymG : SchedCondLSym {
  static constexpr int WQ = 0;
};
// the default without the periodic Sigma symmetrisation (developer variant 96, A/B)
struct SchedCondLSymNS : SchedCondLSym {
  static constexpr int NOSYM = 1;
};
// the symmetrisation after the step's DMA issue, through its own LDS scratch past the
// four waves' areas (developer variant 93, A/B)
struct SchedCondLSymL : SchedCondLSym {
  static constexpr int SYMLATE = 1;
};
template <class C>
constexpr bool has_symlate() {
  if constexpr (requires { C::SYMLATE; }) return C::SYMLATE != 0;
  return false;
}
template <class C>
constexpr bool has_sym_every() {
  if constexpr (requires { C::NOSYM; }) return C::NOSYM == 0;
  return true;
}
// the default at two waves per SIMD: packed images (Geo PACK), 2 workgroups per CU
// (batches above one wave per SIMD)
struct SchedCondLSymP : SchedCondLSym {
  static constexpr int PACK = 1;
};
template <class C>
constexpr bool has_pack() {
  if constexpr (requires { C::PACK; }) return C::PACK != 0;
  return false;
}
struct SchedCondLSymStamped : SchedCondLSym {
  static constexpr int STAMP = 1;
};
// stamps of the round-4 default (the symmetrisation after the DMA issue)
struct SchedCondLSymLStamped : SchedCondLSymL {
  static constexpr int STAMP = 1;
};
struct SchedCondLNewt : SchedCondL {
  static constexpr int SYM2 = 0, NEWT = 1, PEPS = 0;
};
struct SchedCondLPeps : SchedCondL {
  static constexpr int SYM2 = 0, NEWT = 0, PEPS = 1;
};
// SYM2 + the reciprocal Newton without the one-block predict (49 measured slower)
struct SchedCondLSN : SchedCondL {
  static constexpr int SYM2 = 1, NEWT = 1, PEPS = 0;
};
// DMA placement A/B: DSTAG 1 = odd waves issue the step's pieces after the update
// (the CU's waves no longer burst together); 2 = Q/QT pieces after the E sweep
// (their images are read by then), A/B after the X sweep
struct SchedCondLStag1 : SchedCondL {
  static constexpr int DSTAG = 1;
};
struct SchedCondLStag2 : SchedCondL {
  static constexpr int DSTAG = 2;
};
template <class C>
constexpr int dstag() {
  if constexpr (requires { C::DSTAG; }) return C::DSTAG;
  return 0;
}
template <class C>
constexpr bool has_sym2() {
  if constexpr (requires { C::SYM2; }) return C::SYM2 != 0;
  return false;
}
template <class C>
constexpr bool has_newt() {
  if constexpr (requires { C::NEWT; }) return C::NEWT != 0;
  return false;
}
template <class C>
constexpr bool has_peps() {
  if constexpr (requires { C::PEPS; }) return C::PEPS != 0;
  return false;
}

// small-s row groups (s <= 5 fp64 augmented blocks at batches that leave the
// one-problem-per-lane kernel most SIMDs idle): the
// conditioned kernel's own layout -- four problems per wave, one per 16-lane DPP row,
// s of its lanes busy -- so B = 4,096 runs 1,024 waves instead of 64.  Unhalved
// symmetric sums (SYM2) and the congruence query (WQ, the terminal block's X sweep
// stopped one pivot short: SweepQP) like the s = 13 default; the image reads are
// plain (no LDS-pipelined sweeps: SweepQSym / SweepQAB exist for s = 13 only).
#ifndef HOP_SMALL_QPIPE
#define HOP_SMALL_QPIPE 0  // small-s row groups: step k's query under step k+1's sweeps (A/B)
#endif
constexpr bool kSmallQPipe = HOP_SMALL_QPIPE != 0;
#ifndef HOP_SMALL_STAMP
#define HOP_SMALL_STAMP 0  // diagnostic builds: section stamps (tools/stamps_small.py)
#endif
struct SchedCondSmall : SchedCond {
  static constexpr int SYM2 = 1, NEWT = 0, PEPS = 0, WQ = 1, SMALLS = 1;
  static constexpr int STAMP = HOP_SMALL_STAMP;
};
template <class C>
constexpr bool has_smalls() {
  if constexpr (requires { C::SMALLS; }) return C::SMALLS != 0;
  return false;
}

// fp32 blocks (config 5): the predict's two products A~ and A T on the f32 matrix
// cores, one problem per v_mfma_f32_16x16x4_f32 tile
struct SchedCondMfma : SchedCond {
  static constexpr int MFMA = 1;
};
template <class C>
constexpr bool has_mfma() {
  if constexpr (requires { C::MFMA; }) return C::MFMA != 0;
  return false;
}

template <class C>
constexpr bool has_arow() {
  if constexpr (requires { C::AROW; }) return C::AROW != 0;
  return false;
}
// conditioned-prefix kernel on the trajectory form (lft_cond_kernel)
struct SchedCondTraj : SchedLdlDma {
  static constexpr int SCALE = 0;
  static constexpr int TRAJ = 1;
};
// fused hand-over: a wave whose problems the conditioned kernel flagged recomputes
// them with the reference association (lft_v2_body) at the end of the same launch,
// instead of a second (rerun) launch that every wave enters to read its status
struct SchedCondLSymF : SchedCondLSym {
  static constexpr int FUSE = 1;
};
struct SchedCondTrajF : SchedCondTraj {
  static constexpr int FUSE = 1;
};
// lft_cond_cf_kernel with the round-3 query: the elimination of Sigma_eps + X_t with
// X_t's 1/sigma ~ 1e9 rank-1 part formed (A/B, developer variant 97); the default
// eliminates the congruent W^-T Sigma_eps W^-1 + diag(Pi, 1/sigma) instead
struct SchedCondTrajG : SchedCondTraj {
  static constexpr int GJQ = 1;
};
// without the periodic Sigma symmetrisation (developer A/B: 95; 94 = with the
// round-3 query too, i.e. round 3's kernel)
struct SchedCondTrajNS : SchedCondTraj {
  static constexpr int NOSYM = 1;
};
struct SchedCondTrajGNS : SchedCondTrajG {
  static constexpr int NOSYM = 1;
};
template <class C>
constexpr bool has_gjq() {
  if constexpr (requires { C::GJQ; }) return C::GJQ != 0;
  return false;
}
template <class C>
constexpr bool has_fuse() {
  if constexpr (requires { C::FUSE; }) return C::FUSE != 0;
  return false;
}
template <class C>
constexpr bool has_traj() {
  if constexpr (requires { C::TRAJ; }) return C::TRAJ != 0;
  return false;
}
template <class C>
constexpr bool offset_form() {
  return C::PIV == 4 || C::PIV == 5;
}

// One Gauss-Jordan pivot of a column-per-lane matrix (Select schedule),
// d = M_pp + eps broadcast from lane p.  Result after all pivots: -(M+eps)^-1.
// Column p minus e_p: lane p broadcasts d-1; all rows in one block; fix lane p after.
template <class C, int S, int p>
__device__ __forceinline__ void pivot(double (&r)[S], double eps, bool& ok) {
  const double d = bcast<p>(r[p]) + eps;
  ok = ok && (d > 0.0);
  const double rd = rcp_nr<C::NR>(d);
  const double t = sel_lane<p>(r[p], d - 1.0);
  r[p] = t;
  RowB<S>::template sweep<p>(r, -t * rd);
  r[p] = sel_lane<p>(r[p], r[p] - 1.0);
}

// Offset-form pivot with the shortest dependent chain (Chain schedule):
//   d = 1 + bcast_p(r_p)       one DPP FMA (no v_mov_dpp + s_nop + v_add)
//   rd0 = rcp(d); sc = sc0 + sc0 e with sc0 = -r_p rd0, e = 1 - d rd0 (one Newton
//   step folded into the scale: rcp -> fma -> fma instead of rcp -> fma -> fma -> mul)
//   pivot test: min(d) in a VGPR (no v_cmp -> s_and VCC round trip per pivot);
//   NaN pivots are caught once per sweep (they turn every entry NaN).
// The block writes r[p+1] first and carries no s_nop: its DPP sources were last
// written by the previous block, the chain lies in between (checked at build).
template <class C, int S, int p>
__device__ __forceinline__ void pivot4(double (&r)[S], double& dmin) {
  double d = 1.0;
  fmac_bcast<p, p == 0>(d, r[p], 1.0);
  const double rd0 = __builtin_amdgcn_rcp(d);
  const double e = __builtin_fma(-d, rd0, 1.0);
  const double sc0 = -r[p] * rd0;
  dmin = __builtin_fmin(dmin, d);
  const double sc = __builtin_fma(sc0, e, sc0);
  if constexpr (p == 0) RowB<S>::template sweep<p>(r, sc);
  else RowB<S>::template sweepq<p>(r, sc);
}

// every pivot > 0 and none NaN (a NaN pivot makes every entry NaN, lane 0 included)
template <int S>
__device__ __forceinline__ bool pivots_ok(const double (&r)[S], double dmin) {
  const double x = bcast<0>(r[0]);
  return (dmin > 0.0) && (x == x);
}

template <class C>
constexpr bool has_scale() {
  if constexpr (requires { C::SCALE; }) return C::SCALE != 0;
  return false;
}

// The offset-form Gauss-Jordan sweep updates column p at pivot p as x (1 - (d-1)/d):
// that cancels to an absolute error of u in the factor, u d relative, so a pivot
// d >> 1 costs its column u d of accuracy, and every later step carries it.  The
// reference-association kernel (the rerun of the conditioned kernels' hand-overs and
// HOP_OPT_REFERENCE_ASSOC) meets such pivots after an escalated stage: E_k ~ 1e6 puts
// pivots of that size into W = (E_k + Gbar)^-1, and J drifted 0.12 away from the
// 50-digit value within 20 steps where NumPy's Cholesky inverses stay at 3e-4
// (round 5, tools/dump_escalation_case.py; a NumPy model of the sweep reproduces the
// 0.12).  SCALE schedules invert the equilibrated D (M + eps I) D, D = diag(M + eps
// I)^-1/2, instead: unit diagonal, so every pivot of the SPD case is <= 1, and
// (M + eps I)^-1 = D M'^-1 D.  The pivots keep their signs (Cholesky's test is
// unchanged) and the rows stay independent (the retry ladder's bitwise property).
template <int S>
__device__ __forceinline__ void sweep_equilibrated(double (&r)[S], double& dmin, int c) {
  double dg = 0.0;  // lane c: the offset diagonal entry r[c][c] = M_cc + eps - 1
  static_for<S>([&](auto I) { dg = (c == (int)I) ? r[I] : dg; });
  const double dd = 1.0 + dg;
  const double Dc = c < S ? 1.0 / __builtin_sqrt(dd) : 0.0;  // NaN when not positive
  // the diagonal of M' - I is 0, or NaN for an infinite M_cc (its D_c = 0 would
  // otherwise turn the +inf into an identity row the sweep accepts, where Cholesky
  // and the unscaled sweep fail: the ladder and the LU slot, as utils.py:69-93)
  const double z = 0.0 * dd;
  static_for<S>([&](auto I) {
    const double v = (r[I] * Dc) * bcast<I>(Dc);
    r[I] = (c == (int)I) ? z : v;  // M' - I: unit diagonal
  });
  SweepQ<S>::run(r, dmin);
  static_for<S>([&](auto I) {  // -M^-1 + I = D (R' - I) D + I
    const double v = ((r[I] - ((c == (int)I) ? 1.0 : 0.0)) * Dc) * bcast<I>(Dc);
    r[I] = (c == (int)I) ? v + 1.0 : v;
  });
}

template <class C, int S>
__device__ __forceinline__ void sweep(double (&r)[S], double eps, bool& ok) {
  if constexpr (C::PIV == 5 && has_scale<C>()) {
    double dmin = 1.0;
    sweep_equilibrated<S>(r, dmin, (int)(threadIdx.x & 15));
    ok = ok && pivots_ok(r, dmin);
  } else if constexpr (C::PIV == 5) {
    double dmin = 1.0;
    SweepQ<S>::run(r, dmin);
    ok = ok && pivots_ok(r, dmin);
  } else if constexpr (C::PIV == 4) {
    double dmin = 1.0;
    static_for<S>([&](auto P) { pivot4<C, S, P>(r, dmin); });
    ok = ok && pivots_ok(r, dmin);
  } else {
    static_for<S>([&](auto P) { pivot<C, S, P>(r, eps, ok); });
  }
}

// Two independent sweeps; the C++ schedules interleave their pivots so the
// reciprocal chains overlap (the asm sweep hides its own chain).
template <class C, int S>
__device__ __forceinline__ void sweep2(double (&r)[S], double epsr, bool& okr, double (&q)[S],
                                       double epsq, bool& okq) {
  if constexpr (C::PIV == 5) {
    sweep<C, S>(r, epsr, okr);
    sweep<C, S>(q, epsq, okq);
  } else if constexpr (C::PIV == 4) {
    double dr = 1.0, dq = 1.0;
    static_for<S>([&](auto P) {
      pivot4<C, S, P>(r, dr);
      pivot4<C, S, P>(q, dq);
    });
    okr = okr && pivots_ok(r, dr);
    okq = okq && pivots_ok(q, dq);
  } else {
    static_for<S>([&](auto P) {
      pivot<C, S, P>(r, epsr, okr);
      pivot<C, S, P>(q, epsq, okq);
    });
  }
}

// Read column c and row c of a row-major LD-strided S x S LDS matrix with all
// 2S ds_read_b64 in flight and a single lgkmcnt wait (hipcc, short of VGPRs,
// otherwise interleaves ~10 read/wait round trips per matrix)
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)p;
}

// (loads and their wait are ONE asm statement with early-clobber outputs: a
// separate wait statement lets hipcc copy a destination before its data lands)
template <int S, int LD>
__device__ __forceinline__ void lds_col_row(const double* img, int c, double (&col)[S],
                                            double (&row)[S]) {
  const unsigned bc = lds_addr(img) + 8u * c;        // (i, c): + 8 LD i
  const unsigned br = lds_addr(img) + 8u * LD * c;   // (c, i): + 8 i
  LdsSym<S, LD>::run(bc, br, col, row);
}

// sym(M) from a row-major S x S image (LDS) or a padded tile
template <class C, int S, int LD>
__device__ __forceinline__ void sym_from(const double* img, int c, double (&r)[S]) {
  if constexpr (C::LDSASM) {
    double t[S];
    lds_col_row<S, LD>(img, c, r, t);
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = 0.5 * (r[i] + t[i]);
  } else {
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = 0.5 * (img[i * LD + c] + img[c * LD + i]);
  }
}

// m[c][c] += delta on lanes c < S of a row-major LDS matrix (one LDS atomic per
// lane, no VALU): applies the (eps - 1) diagonal offset of the offset form.
template <int S, int LD>
__device__ __forceinline__ void diag_add(const double* img, int c, double delta) {
  if (c < S) {
    const unsigned a = lds_addr(img) + 8u * (LD + 1) * c;
    asm volatile("ds_add_f64 %0, %1" ::"v"(a), "v"(delta) : "memory");
  }
}

// chol_inv's _assert_finite (utils.py:77): a non-finite input raises in the
// reference and can never factor, so its row runs no jitter ladder; the
// inverse (or quadratic form) is NaN and the row gets ST_NONFINITE alone, as
// the oracle's spd_inverse.  Checked only after a failed first attempt (rare
// path): the input image at img (row-major, row stride LD: S rows, NC columns,
// NC = S + 1 with the bordered column z0 of the query), one ballot.
template <int S, int LD, int NC = S>
__device__ __forceinline__ bool row_input_nonfinite(const double* img, int c) {
  double z = 0.0;
  if (c < NC) {
#pragma unroll
    for (int i = 0; i < S; ++i) z = __builtin_fma(img[i * LD + c], 0.0, z);
  }
  const unsigned long long m = __ballot(!(z == z));
  return ((m >> (16 * ((threadIdx.x & 63) >> 4))) & 0xffffull) != 0ull;
}

// Retry ladder shared by all inverses (utils.py:69-93 semantics): rows that
// failed re-form their input with eps x 10; after max_tries the last sweep is
// kept (LU slot) and flagged.  Rows that already succeeded recompute bitwise
// the same result.  Rare path.
template <class C, int S, int LD>
__device__ __forceinline__ void retry_inverse(double (&r)[S], const double* img, int c, bool ok0,
                                              int max_tries, unsigned& st) {
  double eps = ok0 ? 1e-9 : 1e-8;  // rows that succeeded keep their jitter
  double cur = 1e-9;               // offset form: jitter currently in the LDS diagonal
  int tries = ok0 ? 0 : 1;
  const bool nf = !ok0 && row_input_nonfinite<S, LD>(img, c);
  bool done = ok0 || nf, lu = false;
  if (!ok0) st |= nf ? ST_NONFINITE : ST_JITTER;
#pragma unroll 1
  while (__any(!done)) {
    if constexpr (offset_form<C>()) {
      diag_add<S, LD>(img, c, eps - cur);  // +0 for rows that keep their jitter
      cur = eps;
    }
    sym_from<C, S, LD>(img, c, r);
    bool ok = true;
    sweep<C, S>(r, eps, ok);
    const bool last = tries >= max_tries;
    if (!done && !ok && last) {
      st |= ST_LU;
      lu = true;
    }
    done = done || ok || last;
    if (!__any(!done)) break;
    if (!done) {
      eps *= 10.0;
      ++tries;
    }
  }
  if (__any(lu)) {  // the LU slot (utils.py:88-93): solve(sym(A) + eps I, I), pivoted
    wave_sync();
    if (lu) {
      constexpr bool OFFF = offset_form<C>();  // offset form: the image diagonal is value - 1 + eps
      double x[S];
#pragma unroll
      for (int i = 0; i < S; ++i) x[i] = (i == c) ? 1.0 : 0.0;
      const bool okl = lu_lds_solve<double>(img, LD, S, OFFF ? 1.0 : 0.0, OFFF ? 0.0 : eps, x) == 0;
#pragma unroll
      for (int i = 0; i < S; ++i)
        r[i] = okl ? ((OFFF && i == c) ? 1.0 : 0.0) - x[i] : __builtin_nan("");
    }
  }
  if (nf) {
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = __builtin_nan("");
  }
}

// Bordered forward elimination: r holds [M | b] column-per-lane (b on lane S,
// which is free when s < 16).  Gaussian elimination without pivoting (its
// pivots are the Cholesky squares, so d > 0 is the potrf test) leaves
// b^T (M + eps I)^-1 b = sum_p b_p^2 / d_p, returned broadcast to the row.
template <class C, int S>
__device__ __forceinline__ double elim_quad(double (&r)[S], double eps, bool& ok) {
  double acc = 0.0;
  if constexpr (C::PIV == 5) {
    double dmin = 1.0;
    ElimQ<S>::run(r, acc, dmin, eps);
    const double q = bcast<S>(acc);
    ok = ok && (dmin > 0.0) && (q == q);
    return q;
  } else if constexpr (C::PIV == 4) {
    double dmin = 1.0;
    static_for<S>([&](auto P) {
      constexpr int p = P;
      double d = eps;
      // block p-1 wrote S-p rows, r[p] first: fewer than 3 leave < 2 wait states
      fmac_bcast<p, p == 0 || (S - p) <= 2>(d, r[p], 1.0);
      const double rd0 = __builtin_amdgcn_rcp(d);
      const double e = __builtin_fma(-d, rd0, 1.0);
      const double sc0 = -r[p] * rd0;
      dmin = __builtin_fmin(dmin, d);
      const double sc = __builtin_fma(sc0, e, sc0);
      acc = __builtin_fma(-r[p], sc, acc);
      if constexpr (p == 0) TailB<S>::template elim<p>(r, sc);
      else TailB<S>::template elimq<p>(r, sc);
    });
    const double q = bcast<S>(acc);
    ok = ok && (dmin > 0.0) && (q == q);
    return q;
  } else {
    static_for<S>([&](auto P) {
      constexpr int p = P;
      const double d = bcast<p>(r[p]) + eps;
      ok = ok && (d > 0.0);
      const double sc = -r[p] * rcp_nr<C::NR>(d);
      acc = __builtin_fma(-r[p], sc, acc);
      TailB<S>::template elim<p>(r, sc);
    });
    return bcast<S>(acc);
  }
}

// z0^T (sym(X0) + eps I)^-1 z0 with the chol_inv retry ladder; X0 parked in the
// tile whose row S holds z0 (so that sym() keeps lane S = z0).
template <class C, int S>
__device__ __forceinline__ double quad_retry(double (&r)[S], double* tile, int c, bool ok0,
                                             double q, int mt, unsigned& st);
template <class C, int S>
__device__ __forceinline__ double quad_inverse(double (&r)[S], double* tile, int c, int mt,
                                               unsigned& st) {
  lds_put(tile, c, r);
  wave_sync();
  sym_from<C, S, kLdsRow>(tile, c, r);
  bool ok = true;
  double q = elim_quad<C, S>(r, 1e-9, ok);
  if (__any(!ok)) q = quad_retry<C, S>(r, tile, c, ok, q, mt, st);
  wave_sync();
  return q;
}

// chol_inv ladder of quad_inverse (rare path): re-form sym(X0) from the tile
template <class C, int S>
__device__ __forceinline__ double quad_retry(double (&r)[S], double* tile, int c, bool ok0,
                                             double q, int mt, unsigned& st) {
  {
    double eps = ok0 ? 1e-9 : 1e-8;
    int tries = ok0 ? 0 : 1;
    const bool nf = !ok0 && row_input_nonfinite<S, kLdsRow, S + 1>(tile, c);
    bool done = ok0 || nf, lu = false;
    if (!ok0) st |= nf ? ST_NONFINITE : ST_JITTER;
#pragma unroll 1
    while (__any(!done)) {
      sym_from<C, S, kLdsRow>(tile, c, r);
      bool ok2 = true;
      q = elim_quad<C, S>(r, eps, ok2);
      const bool last = tries >= mt;
      if (!done && !ok2 && last) {
        st |= ST_LU;
        lu = true;
      }
      done = done || ok2 || last;
      if (!__any(!done)) break;
      if (!done) {
        eps *= 10.0;
        ++tries;
      }
    }
    if (lu) {  // the LU slot: z0^T solve(sym(X0) + eps I, z0), pivoted (z0 in the tile's row S)
      double y[S];
#pragma unroll
      for (int i = 0; i < S; ++i) y[i] = tile[S * kLdsRow + i];
      const bool okl = lu_lds_solve<double>(tile, kLdsRow, S, 0.0, eps, y) == 0;
      double qq = 0.0;
#pragma unroll
      for (int i = 0; i < S; ++i) qq += tile[S * kLdsRow + i] * y[i];
      q = okl ? qq : __builtin_nan("");
    }
    if (nf) q = __builtin_nan("");
  }
  return q;
}

// Query without the Wt inverse (has_qldl): r = Xt + Gbar - I (offset form) is
// parked, symmetrised and eliminated (QueryLdl); the same row operations turn a
// copy of H = Fbar^T into L^-1 H and X0 = Ebar - sum_p Ht_p (x) Ht_p / d_p is
// streamed.  chol_inv ladder on failure: re-form from the tile with eps x 10
// (Ht and X0 restart from H and Ebar, which are untouched).
template <class C, int S>
__device__ __forceinline__ void query_x0_ldl(double (&r)[S], const double (&H)[S],
                                             const double (&Eb)[S], double (&X0)[S], double* tile,
                                             int c, int mt, unsigned& st) {
  lds_put(tile, c, r);
  diag_add<S, kLdsRow>(tile, c, 1e-9);  // r carries -I: diagonal = value - 1 + eps
  wave_sync();
  sym_from<C, S, kLdsRow>(tile, c, r);
  double Ht[S];
  copy(Ht, H);
  copy(X0, Eb);
  double dmin = 1.0;
  QueryLdl<S>::run(r, Ht, X0, dmin);
  const bool ok0 = pivots_ok(X0, dmin);
  if (__any(!ok0)) {
    double eps = ok0 ? 1e-9 : 1e-8, cur = 1e-9;
    int tries = ok0 ? 0 : 1;
    // Xt + Gbar non-finite (or H, Ebar: X0 = Ebar - Fbar Wt Fbar^T is then NaN too)
    bool nf = !ok0 && row_input_nonfinite<S, kLdsRow>(tile, c);
    {
      double z = 0.0;
#pragma unroll
      for (int i = 0; i < S; ++i) z = __builtin_fma(H[i], 0.0, __builtin_fma(Eb[i], 0.0, z));
      const unsigned long long m = __ballot(c < S && !(z == z));
      nf = nf || (!ok0 && ((m >> (16 * ((threadIdx.x & 63) >> 4))) & 0xffffull) != 0ull);
    }
    bool done = ok0 || nf, lu = false;
    if (!ok0) st |= nf ? ST_NONFINITE : ST_JITTER;
#pragma unroll 1
    while (__any(!done)) {
      diag_add<S, kLdsRow>(tile, c, eps - cur);
      cur = eps;
      sym_from<C, S, kLdsRow>(tile, c, r);
      copy(Ht, H);
      copy(X0, Eb);
      dmin = 1.0;
      QueryLdl<S>::run(r, Ht, X0, dmin);
      const bool ok = pivots_ok(X0, dmin);
      const bool last = tries >= mt;
      if (!done && !ok && last) {
        st |= ST_LU;
        lu = true;
      }
      done = done || ok || last;
      if (!__any(!done)) break;
      if (!done) {
        eps *= 10.0;
        ++tries;
      }
    }
    if (__any(lu)) {
      // the LU slot of Wt = chol_inv(Xt + Gbar) (utils.py:88-93, pivoted): lane c
      // solves (Mt + eps I) v = (column c of Fbar^T), then X0 = Ebar - Fbar Wt Fbar^T
      // = Ebar - sum_j H_j (x) v_j (the tile holds Mt in offset form: diag - 1 + eps)
      wave_sync();
      double v[S];
#pragma unroll
      for (int i = 0; i < S; ++i) v[i] = H[i];
      bool okl = true;
      if (lu) okl = lu_lds_solve<double>(tile, kLdsRow, S, 1.0, 0.0, v) == 0;
      double Xl[S];
      copy(Xl, Eb);
      acc_xty<true>(Xl, H, v);  // Ebar - Fbar (Mt + eps I)^-1 Fbar^T
#pragma unroll
      for (int i = 0; i < S; ++i) X0[i] = lu ? (okl ? Xl[i] : __builtin_nan("")) : X0[i];
    }
    if (nf) {
#pragma unroll
      for (int i = 0; i < S; ++i) X0[i] = __builtin_nan("");
    }
  }
  wave_sync();
}


// Negated inverse of sym(img): r <- -(sym(M) + eps I)^-1  (+ I in offset form)
template <class C, int S, int LD>
__device__ __forceinline__ void neg_inverse(double (&r)[S], const double* img, int c, int mt,
                                            unsigned& st) {
  sym_from<C, S, LD>(img, c, r);
  bool ok = true;
  sweep<C, S>(r, 1e-9, ok);
  if (__any(!ok)) retry_inverse<C, S, LD>(r, img, c, ok, mt, st);
}

template <class C, int S, int LD1, int LD2>
__device__ __forceinline__ void neg_inverse2(double (&r)[S], const double* img1, double (&q)[S],
                                             const double* img2, int c, int mt, unsigned& st) {
  sym_from<C, S, LD1>(img1, c, r);
  sym_from<C, S, LD2>(img2, c, q);
  bool okr = true, okq = true;
  sweep2<C, S>(r, 1e-9, okr, q, 1e-9, okq);
  if (__any(!okr)) retry_inverse<C, S, LD1>(r, img1, c, okr, mt, st);
  if (__any(!okq)) retry_inverse<C, S, LD2>(q, img2, c, okq, mt, st);
}

// Negated inverse of sym(x) for a register matrix: x is parked in the tile.
// Offset form: `off` is the diagonal offset already in r (-1 when r was formed
// from offset-form inverses), so the tile diagonal gets eps - 1 - off.
template <class C, int S>
__device__ __forceinline__ void neg_inverse_reg(double (&r)[S], double* tile, int c, int mt,
                                                unsigned& st, double off = 0.0) {
  lds_put(tile, c, r);
  if constexpr (offset_form<C>()) diag_add<S, kLdsRow>(tile, c, 1e-9 - 1.0 - off);
  wave_sync();
  neg_inverse<C, S, kLdsRow>(r, tile, c, mt, st);
  wave_sync();
}

// Products: with the pad-free schedules only the first broadcast block of a
// product is padded (its source may have just been written); later blocks
// read the same, unchanged source registers.  The SCALE schedules (the
// reference-association kernels) run near the register limit, where the
// compiler may reload a later block's source from an AGPR right before it:
// every block is padded there (the build's hazard check found one).
template <class C, bool NEG, int S, int K>
__device__ __forceinline__ void gxy(double (&out)[S], const double (&x)[S], const double (&y)[K]) {
  if constexpr (C::XYROW) {
    // out[i] += sum_j bcast_j(x_i) y_j: the accumulator is forwarded between
    // consecutive FMAs (4.0 cycles each vs 4.9 for 13 independent accumulators)
    static_for<S>([&](auto I) {
      if constexpr (I == 0 || has_scale<C>()) {
        if constexpr (NEG) LaneDot<K>::fma_neg(out[I], x[I], y);
        else LaneDot<K>::fma(out[I], x[I], y);
      } else {
        if constexpr (NEG) LaneDot<K>::fma_negq(out[I], x[I], y);
        else LaneDot<K>::fmaq(out[I], x[I], y);
      }
    });
  } else if constexpr (offset_form<C>()) {
    static_for<K>([&](auto J) {
      if constexpr (J == 0 || has_scale<C>()) {
        if constexpr (NEG) RowB<S>::template fma_neg<J>(out, x, y[J]);
        else RowB<S>::template fma<J>(out, x, y[J]);
      } else {
        if constexpr (NEG) RowB<S>::template fma_negq<J>(out, x, y[J]);
        else RowB<S>::template fmaq<J>(out, x, y[J]);
      }
    });
  } else {
    acc_xy<NEG>(out, x, y);
  }
}
template <class C, bool NEG, int S, int K>
__device__ __forceinline__ void gxty(double (&out)[S], const double (&x)[K], const double (&y)[K]) {
  if constexpr (offset_form<C>()) {
    static_for<K>([&](auto J) {
      if constexpr (J == 0 || has_scale<C>()) {
        if constexpr (NEG) LaneB<S>::fma_neg(out, x[J], y[J]);
        else LaneB<S>::fma(out, x[J], y[J]);
      } else {
        if constexpr (NEG) LaneB<S>::fma_negq(out, x[J], y[J]);
        else LaneB<S>::fmaq(out, x[J], y[J]);
      }
    });
  } else {
    acc_xty<NEG>(out, x, y);
  }
}

// Diagnostic section stamps: per-wave shader-clock totals per section, summed
// over waves into g_hop_stamp (read by hop_debug_stamps; slot 15 counts waves).
__device__ unsigned long long g_hop_stamp[16];

// ---------------------------------------------------------------------------
// LDS-DMA streaming of one step's blocks into the wave's images
// ---------------------------------------------------------------------------
// Every LDS-DMA statement opens with HOP_VMNOP: three wait states, so that with the
// M0 write and its own s_nop 0 no buffer_load reads a descriptor or soffset SGPR within
// five wait states of a VALU write of it (the compiler reloads spilled SGPRs with
// v_readlane right before the statement; it pads only its own instruction pairs).
// The build drops every such pad the compiled code around it makes unnecessary
// (tools/nop_elide.py) and checks the result (tools/check_dpp_hazards.py).
__device__ __forceinline__ void dma16(unsigned voff, __amdgpu_buffer_rsrc_t rsrc, unsigned lds,
                                      unsigned soff) {
  unsigned keep;
  asm volatile(
      HOP_VMNOP         // VALU SGPR write -> VMEM read (tools/check_dpp_hazards.py)
      ".p2align 3\n\t"  // the 8-byte buffer_load at 0 mod 8 (code placement)
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds), "s"(soff)
      : "memory");
}

__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The LDS-DMA instruction offset is added to both addresses: the LDS destination is
// M0 + offset + 16 lane and the memory address voffset + soffset + offset (measured,
// tools/ubench/lds_dma_offset.hip, a wrapped voffset included).  So one M0 serves the
// pieces of an image that lie within the 12-bit offset field: piece j of an image at
// M0 = image + 4096 (j / 4), offset 1024 (j % 4), its voffset lowered by that offset
// once at kernel start (dma_voff_lowered).  Two M0 writes per 6-piece image instead of
// six, each with the wait state an M0 write needs before an LDS-DMA.
__device__ __forceinline__ unsigned dma_voff_lowered(unsigned voff, int j) {
  return voff - 1024u * (unsigned)(j % 4);
}

// Trajectory form: the step's 10 raw pieces (A 5, B 2, x, a, u) in one asm block;
// va / vb lowered (dma_voff_lowered)
template <int OA, int OB, int OX, int OV, int OU>
__device__ __forceinline__ void dma_traj10(const unsigned (&va)[5], const unsigned (&vb)[2],
                                           unsigned vx, unsigned vv, unsigned vu,
                                           __amdgpu_buffer_rsrc_t rA, __amdgpu_buffer_rsrc_t rB,
                                           __amdgpu_buffer_rsrc_t rX, __amdgpu_buffer_rsrc_t rV,
                                           __amdgpu_buffer_rsrc_t rU, unsigned wlds, unsigned sA,
                                           unsigned sB, unsigned sX, unsigned sV, unsigned sU) {
  unsigned keep;
#define HOP_M0(OFF) "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\t"
#define HOP_PO(R, V, SO, IO) "buffer_load_dwordx4 %[" #V "], %[" #R "], %[" #SO "] offen offset:" #IO " lds\n\t"
  asm volatile(
      HOP_VMNOP
      ".p2align 3\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      HOP_M0(%[o0]) HOP_PO(ra, a0, sa, 0) HOP_PO(ra, a1, sa, 1024) HOP_PO(ra, a2, sa, 2048)
      HOP_PO(ra, a3, sa, 3072)
      HOP_M0(%[o4]) HOP_PO(ra, a4, sa, 0)
      HOP_M0(%[p0]) HOP_PO(rb, b0, sb, 0) HOP_PO(rb, b1, sb, 1024)
      HOP_M0(%[ox]) HOP_PO(rx, x0, sx, 0)
      HOP_M0(%[ov]) HOP_PO(rv, x1, sv, 0)
      HOP_M0(%[ou]) HOP_PO(ru, x2, su, 0)
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [w] "s"(wlds), [sa] "s"(sA), [sb] "s"(sB), [sx] "s"(sX), [sv] "s"(sV), [su] "s"(sU),
        [ra] "s"(rA), [rb] "s"(rB), [rx] "s"(rX), [rv] "s"(rV), [ru] "s"(rU),
        [a0] "v"(va[0]), [a1] "v"(va[1]), [a2] "v"(va[2]), [a3] "v"(va[3]), [a4] "v"(va[4]),
        [b0] "v"(vb[0]), [b1] "v"(vb[1]), [x0] "v"(vx), [x1] "v"(vv), [x2] "v"(vu),
        [o0] "i"(OA), [o4] "i"(OA + 4096), [p0] "i"(OB), [ox] "i"(OX), [ov] "i"(OV), [ou] "i"(OU)
      : "memory", "scc");
#undef HOP_PO
#undef HOP_M0
}

// One step's 20 LDS-DMA pieces (Q, A, B, QT images of s = 13, m = 4) in one asm
// block: M0 saved once and set per piece from the wave's LDS base plus an
// immediate (no per-piece SGPR, no readlane of spilled addresses, no save /
// restore pair per piece).
// PACK: dma_step20 with the images back to back.  The full pieces first, then the
// last piece of Q, A, QT (LM lanes) and of B (LB lanes) under a narrowed EXEC, so no
// lane past an image's data writes into the next image; EXEC restored at the end.
// The narrowed masks are ANDed with the caller's EXEC, so a lane the caller turned
// off stays off (the kernel calls this with full EXEC; the AND keeps it safe if not).
template <int OQ, int OA, int OB, int OT, int LM, int LB>
__device__ __forceinline__ void dma_step20p(const unsigned (&vm)[6], const unsigned (&vb)[2],
                                            __amdgpu_buffer_rsrc_t rQ, __amdgpu_buffer_rsrc_t rA,
                                            __amdgpu_buffer_rsrc_t rB, __amdgpu_buffer_rsrc_t rT,
                                            unsigned wlds, unsigned soM, unsigned soB) {
  static_assert(LM > 0 && LM <= 32 && LB > 32 && LB <= 64, "partial-piece masks");
  unsigned keep, elo, ehi;
#define HOP_P(R, V, OFF, SO)                                                  \
  "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\tbuffer_load_dwordx4 %[" #V "], %[" #R \
  "], %[" #SO "] offen lds\n\t"
  asm volatile(
      HOP_VMNOP
      ".p2align 3\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      "s_mov_b32 %[elo], exec_lo\n\t"
      "s_mov_b32 %[ehi], exec_hi\n\t"
      HOP_P(rq, v0, %[q0], sm) HOP_P(rq, v1, %[q1], sm) HOP_P(rq, v2, %[q2], sm)
      HOP_P(rq, v3, %[q3], sm) HOP_P(rq, v4, %[q4], sm)
      HOP_P(ra, v0, %[a0], sm) HOP_P(ra, v1, %[a1], sm) HOP_P(ra, v2, %[a2], sm)
      HOP_P(ra, v3, %[a3], sm) HOP_P(ra, v4, %[a4], sm)
      HOP_P(rb, u0, %[b0], sb)
      HOP_P(rt, v0, %[t0], sm) HOP_P(rt, v1, %[t1], sm) HOP_P(rt, v2, %[t2], sm)
      HOP_P(rt, v3, %[t3], sm) HOP_P(rt, v4, %[t4], sm)
      "s_and_b32 exec_lo, %[elo], %[mlo]\n\t"
      "s_mov_b32 exec_hi, 0\n\t"
      HOP_P(rq, v5, %[q5], sm) HOP_P(ra, v5, %[a5], sm) HOP_P(rt, v5, %[t5], sm)
      "s_mov_b32 exec_lo, %[elo]\n\t"
      "s_and_b32 exec_hi, %[ehi], %[bhi]\n\t"
      HOP_P(rb, u1, %[b1], sb)
      "s_mov_b32 exec_lo, %[elo]\n\t"
      "s_mov_b32 exec_hi, %[ehi]\n\t"
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep), [elo] "=&s"(elo), [ehi] "=&s"(ehi)
      : [w] "s"(wlds), [sm] "s"(soM), [sb] "s"(soB), [rq] "s"(rQ), [ra] "s"(rA), [rb] "s"(rB),
        [rt] "s"(rT), [v0] "v"(vm[0]), [v1] "v"(vm[1]), [v2] "v"(vm[2]), [v3] "v"(vm[3]),
        [v4] "v"(vm[4]), [v5] "v"(vm[5]), [u0] "v"(vb[0]), [u1] "v"(vb[1]),
        [q0] "i"(OQ), [q1] "i"(OQ + 1024), [q2] "i"(OQ + 2048), [q3] "i"(OQ + 3072),
        [q4] "i"(OQ + 4096), [q5] "i"(OQ + 5120), [a0] "i"(OA), [a1] "i"(OA + 1024),
        [a2] "i"(OA + 2048), [a3] "i"(OA + 3072), [a4] "i"(OA + 4096), [a5] "i"(OA + 5120),
        [b0] "i"(OB), [b1] "i"(OB + 1024), [t0] "i"(OT), [t1] "i"(OT + 1024),
        [t2] "i"(OT + 2048), [t3] "i"(OT + 3072), [t4] "i"(OT + 4096), [t5] "i"(OT + 5120),
        [mlo] "i"((int)((1ull << LM) - 1ull)), [bhi] "i"((int)((1ull << (LB - 32)) - 1ull))
      : "memory", "scc");
#undef HOP_P
}
// vm / vb lowered (dma_voff_lowered): 7 M0 writes instead of 20
template <int OQ, int OA, int OB, int OT>
__device__ __forceinline__ void dma_step20(const unsigned (&vm)[6], const unsigned (&vb)[2],
                                           __amdgpu_buffer_rsrc_t rQ, __amdgpu_buffer_rsrc_t rA,
                                           __amdgpu_buffer_rsrc_t rB, __amdgpu_buffer_rsrc_t rT,
                                           unsigned wlds, unsigned soM, unsigned soB) {
  unsigned keep;
#define HOP_M0(OFF) "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\t"
#define HOP_PO(R, V, SO, IO) "buffer_load_dwordx4 %[" #V "], %[" #R "], %[" #SO "] offen offset:" #IO " lds\n\t"
#define HOP_IMG(R, O0, O4)                                                                   \
  HOP_M0(O0) HOP_PO(R, v0, sm, 0) HOP_PO(R, v1, sm, 1024) HOP_PO(R, v2, sm, 2048)            \
  HOP_PO(R, v3, sm, 3072) HOP_M0(O4) HOP_PO(R, v4, sm, 0) HOP_PO(R, v5, sm, 1024)
  asm volatile(
      HOP_VMNOP
      ".p2align 3\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      HOP_IMG(rq, %[q0], %[q4]) HOP_IMG(ra, %[a0], %[a4])
      HOP_M0(%[b0]) HOP_PO(rb, u0, sb, 0) HOP_PO(rb, u1, sb, 1024)
      HOP_IMG(rt, %[t0], %[t4])
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [w] "s"(wlds), [sm] "s"(soM), [sb] "s"(soB), [rq] "s"(rQ), [ra] "s"(rA), [rb] "s"(rB),
        [rt] "s"(rT), [v0] "v"(vm[0]), [v1] "v"(vm[1]), [v2] "v"(vm[2]), [v3] "v"(vm[3]),
        [v4] "v"(vm[4]), [v5] "v"(vm[5]), [u0] "v"(vb[0]), [u1] "v"(vb[1]),
        [q0] "i"(OQ), [q4] "i"(OQ + 4096), [a0] "i"(OA), [a4] "i"(OA + 4096), [b0] "i"(OB),
        [t0] "i"(OT), [t4] "i"(OT + 4096)
      : "memory", "scc");
#undef HOP_IMG
#undef HOP_PO
#undef HOP_M0
}


// The same 20 pieces in two groups (DSTAG 2): Q and QT (12) as soon as their
// images are read, A and B (8) after the X sweep's reads
template <int OQ, int OT>
__device__ __forceinline__ void dma_stepQT(const unsigned (&vm)[6], __amdgpu_buffer_rsrc_t rQ,
                                           __amdgpu_buffer_rsrc_t rT, unsigned wlds, unsigned soM) {
  unsigned keep;
#define HOP_P(R, V, OFF, SO)                                                  \
  "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\tbuffer_load_dwordx4 %[" #V "], %[" #R \
  "], %[" #SO "] offen lds\n\t"
  asm volatile(
      HOP_VMNOP
      ".p2align 3\n\t"  // every piece's 8-byte buffer_load at 0 mod 8 (code placement)
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      HOP_P(rq, v0, %[q0], sm) HOP_P(rq, v1, %[q1], sm) HOP_P(rq, v2, %[q2], sm)
      HOP_P(rq, v3, %[q3], sm) HOP_P(rq, v4, %[q4], sm) HOP_P(rq, v5, %[q5], sm)
      HOP_P(rt, v0, %[t0], sm) HOP_P(rt, v1, %[t1], sm) HOP_P(rt, v2, %[t2], sm)
      HOP_P(rt, v3, %[t3], sm) HOP_P(rt, v4, %[t4], sm) HOP_P(rt, v5, %[t5], sm)
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [w] "s"(wlds), [sm] "s"(soM), [rq] "s"(rQ), [rt] "s"(rT), [v0] "v"(vm[0]),
        [v1] "v"(vm[1]), [v2] "v"(vm[2]), [v3] "v"(vm[3]), [v4] "v"(vm[4]), [v5] "v"(vm[5]),
        [q0] "i"(OQ), [q1] "i"(OQ + 1024), [q2] "i"(OQ + 2048), [q3] "i"(OQ + 3072),
        [q4] "i"(OQ + 4096), [q5] "i"(OQ + 5120), [t0] "i"(OT), [t1] "i"(OT + 1024),
        [t2] "i"(OT + 2048), [t3] "i"(OT + 3072), [t4] "i"(OT + 4096), [t5] "i"(OT + 5120)
      : "memory", "scc");
#undef HOP_P
}
template <int OA, int OB>
__device__ __forceinline__ void dma_stepAB(const unsigned (&vm)[6], const unsigned (&vb)[2],
                                           __amdgpu_buffer_rsrc_t rA, __amdgpu_buffer_rsrc_t rB,
                                           unsigned wlds, unsigned soM, unsigned soB) {
  unsigned keep;
#define HOP_P(R, V, OFF, SO)                                                  \
  "s_add_u32 m0, %[w], " #OFF "\n\ts_nop 0\n\tbuffer_load_dwordx4 %[" #V "], %[" #R \
  "], %[" #SO "] offen lds\n\t"
  asm volatile(
      HOP_VMNOP
      ".p2align 3\n\t"  // every piece's 8-byte buffer_load at 0 mod 8 (code placement)
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 %[keep], m0\n\t"
      HOP_P(ra, v0, %[a0], sm) HOP_P(ra, v1, %[a1], sm) HOP_P(ra, v2, %[a2], sm)
      HOP_P(ra, v3, %[a3], sm) HOP_P(ra, v4, %[a4], sm) HOP_P(ra, v5, %[a5], sm)
      HOP_P(rb, u0, %[b0], sb) HOP_P(rb, u1, %[b1], sb)
      "s_mov_b32 m0, %[keep]"
      : [keep] "=&s"(keep)
      : [w] "s"(wlds), [sm] "s"(soM), [sb] "s"(soB), [ra] "s"(rA), [rb] "s"(rB),
        [v0] "v"(vm[0]), [v1] "v"(vm[1]), [v2] "v"(vm[2]), [v3] "v"(vm[3]), [v4] "v"(vm[4]),
        [v5] "v"(vm[5]), [u0] "v"(vb[0]), [u1] "v"(vb[1]), [a0] "i"(OA), [a1] "i"(OA + 1024),
        [a2] "i"(OA + 2048), [a3] "i"(OA + 3072), [a4] "i"(OA + 4096), [a5] "i"(OA + 5120),
        [b0] "i"(OB), [b1] "i"(OB + 1024)
      : "memory", "scc");
#undef HOP_P
}

// PACK (the conditioned kernel at two waves per SIMD, SchedCondLSymP): the images
// packed back to back (the last DMA piece of each block type runs on the lanes that
// carry data only, so nothing is written past an image) and the tile slot cut to the
// zero area the lanes past s - 1 read: 19,400 B per wave at s = 13 fp64, so two 4-wave
// workgroups fit a CU's 160 KiB
// SMALLT (the small-s row-group schedule): the tile slot cut to the zero area, as
// PACK's (the conditioned kernel reads nothing else from it)
template <int S, int MM, int ES = 8, bool PACK = false, bool SMALLT = false>  // ES: bytes per element
struct Geo {
  static constexpr int SS = S * S;
  static constexpr int CHM = (SS * ES + 15) / 16;     // 16-B chunks per S x S block
  static constexpr int IMGM = CHM * 16;               // bytes per problem image (16-aligned)
  static constexpr int NJM = (kProbPerWave * CHM + 63) / 64;  // DMA instrs per block type
  // bytes per wave image (a full DMA piece writes 1 KiB)
  static constexpr int IMGM_W = PACK ? kProbPerWave * IMGM : NJM * 1024;
  static constexpr int SM = S * MM;
  static constexpr int CHB = (SM * ES + 15) / 16;
  static constexpr int IMGB = CHB * 16;
  static constexpr int NJB = (kProbPerWave * CHB + 63) / 64;
  static constexpr int IMGB_W = PACK ? kProbPerWave * IMGB : NJB * 1024;
  // lanes of the last piece that carry data (PACK masks the rest)
  static constexpr int LASTM = kProbPerWave * CHM - 64 * (NJM - 1);
  static constexpr int LASTB = kProbPerWave * CHB - 64 * (NJB - 1);
  static constexpr int TILE_W = (PACK || SMALLT) ? 8 * (SS + 8) : kProbPerWave * kLdsTile * 8;
  // per-wave layout: [Q][A][QT][B][tiles]
  static constexpr int OFF_Q = 0, OFF_A = IMGM_W, OFF_QT = 2 * IMGM_W, OFF_B = 3 * IMGM_W;
  static constexpr int OFF_T = 3 * IMGM_W + IMGB_W;
  static constexpr int WAVE_BYTES = OFF_T + TILE_W;
  // trajectory form (n = S-1): raw A_k staged in the A image area, raw B_k in
  // the B area, then x_{k+1}, a_k and u_k after the tiles.  Per problem the
  // staged block of a piece type is CH 16-B chunks at 16 CH g.
  static constexpr int NN = S - 1;
  static constexpr int CHA = (NN * NN * 8 + 15) / 16, NJA = (kProbPerWave * CHA + 63) / 64;
  static constexpr int CHR = (NN * MM * 8 + 15) / 16, NJR = (kProbPerWave * CHR + 63) / 64;
  static constexpr int CHX = (NN * 8 + 15) / 16, NJX = (kProbPerWave * CHX + 63) / 64;
  static constexpr int CHV = (NN * 8 + 15) / 16, NJV = (kProbPerWave * CHV + 63) / 64;
  static constexpr int CHU = (MM * 8 + 15) / 16, NJU = (kProbPerWave * CHU + 63) / 64;
  static_assert(ES != 8 || (NJA <= NJM && NJR <= NJB),
                "raw blocks must fit the augmented image areas");
  static constexpr int OFF_VX = OFF_T + TILE_W, OFF_VA = OFF_VX + 1024 * NJX,
                       OFF_VU = OFF_VA + 1024 * NJV;
  // raw Q of the wave's problems, transposed (lane c reads its row as a column); the
  // closed-form kernel uses the area as its S x S symmetrisation scratch
  static constexpr int OFF_CQ = OFF_VU + 1024 * NJU;
  static constexpr int CQ_BYTES = kProbPerWave * 8 * (NN * NN > SS ? NN * NN : SS);
  static constexpr int WAVE_BYTES_T = OFF_CQ + CQ_BYTES;
};

// Sigma symmetrised, (Sigma + Sigma^T) / 2 (lanes >= S, m and gamma, untouched),
// through a wave-private S x S scratch t of this lane's problem.  The conditioned
// update Sigma' = Sigma_eps - Sigma_eps S^-1 Sigma_eps passes Sigma_eps's
// antisymmetric rounding through unchanged while it contracts the symmetric part, so
// without this the antisymmetric part accumulates over the horizon: on a real
// quadrotor linearisation (tests/golden/real_lin_hp.npz) J ends 0.5 off the 50-digit
// value.  Every 8 steps (round 4) was not enough where A_k grows large (a quadrotor
// rollout near its pitch singularity: the asymmetry injected between two
// symmetrisations is amplified by |A_k|^2 per step, then survives the next update's
// contraction): problem 1492 of the round-5 50-digit fixture
// (tests/golden/real_lin_batch_hp.npz, |A_k| ~ 4e3) ended 3.3e-4 off at horizons
// 92-100, and problem 4068 (|A_k| ~ 9.5e3) still 1.3e-6 with every 4 steps.  Every 2
// steps the NumPy model of the kernel's arithmetic holds both within 3e-8 of the
// 50-digit curves, and 788 CPU-generated quadrotor problems within 4e-8 of
// symmetrising every step (every 4: 7e-8, 8: 2e-5, 16: 7e-2).
#ifndef HOP_SYM_EVERY
#define HOP_SYM_EVERY 2
#endif
constexpr int kSymEvery = HOP_SYM_EVERY;
static_assert(kSymEvery >= 1, "a symmetrisation interval");
// the steps that symmetrise Sigma before their update (step 0's Sigma_eps = eps I is
// symmetric)
__device__ __forceinline__ bool sym_step(int k) { return k > 0 && k % kSymEvery == kSymEvery - 1; }
// split form (the one-wave layouts, whose scratch is their own): the rows are stored
// right after the predict of the step before (the query, which only reads Sigma, and
// the next step's top then hide the LDS round trip) and read back transposed and
// averaged where sym_average would run
#ifndef HOP_SYM_SPLIT
#define HOP_SYM_SPLIT 1
#endif
constexpr bool kSymSplit = HOP_SYM_SPLIT != 0;
template <int S>
__device__ __forceinline__ void sym_store(const double (&X)[S], double* t, int c) {
  if (c < S) {
#pragma unroll
    for (int i = 0; i < S; ++i) t[i * S + c] = X[i];
  }
}
template <int S>
__device__ __forceinline__ void sym_load_average(double (&X)[S], const double* t, int c) {
  const int cr = c < S ? c : 0;
  const double hs = c < S ? 0.5 : 0.0;
  double y[S];
  LdsRow<S>::run(lds_addr(t) + 8u * S * cr, y);  // "memory" clobber: after the stores
#pragma unroll
  for (int i = 0; i < S; ++i) X[i] = __builtin_fma(hs, y[i] - X[i], X[i]);
}
// sym_load_average in two halves (the closed-form kernel): the transposed reads issued
// with no wait, other work, then the wait and the average.  The two statements are
// marked (hop_ldissue / hop_ldwait): the build's hazard check fails any code object in
// which an instruction between them reads or writes a destination of the reads (a
// copy, spill or reuse of a register whose data has not landed, which hipcc cannot
// see: the loads are inside an asm statement; tools/check_dpp_hazards.py).  The compiler's own LDS
// waits in between also wait for these reads (LDS operations complete in order), so
// the round trip is shared with the next reads instead of paid alone.
__device__ __forceinline__ void sym_issue13(const double* t, int c, double (&y)[13]) {
  const int cr = c < 13 ? c : 0;
  asm volatile(
      "ds_read_b64 %0, %13 offset:0\n\tds_read_b64 %1, %13 offset:8\n\t"
      "ds_read_b64 %2, %13 offset:16\n\tds_read_b64 %3, %13 offset:24\n\t"
      "ds_read_b64 %4, %13 offset:32\n\tds_read_b64 %5, %13 offset:40\n\t"
      "ds_read_b64 %6, %13 offset:48\n\tds_read_b64 %7, %13 offset:56\n\t"
      "ds_read_b64 %8, %13 offset:64\n\tds_read_b64 %9, %13 offset:72\n\t"
      "ds_read_b64 %10, %13 offset:80\n\tds_read_b64 %11, %13 offset:88\n\t"
      "ds_read_b64 %12, %13 offset:96 ; hop_ldissue"
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "=&v"(y[4]), "=&v"(y[5]),
        "=&v"(y[6]), "=&v"(y[7]), "=&v"(y[8]), "=&v"(y[9]), "=&v"(y[10]), "=&v"(y[11]),
        "=&v"(y[12])
      : "v"(lds_addr(t) + 8u * 13 * cr)
      : "memory");
}
__device__ __forceinline__ void sym_wait_average13(double (&X)[13], double (&y)[13], int c) {
  asm volatile("s_waitcnt lgkmcnt(0) ; hop_ldwait"
               : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]),
                 "+v"(y[6]), "+v"(y[7]), "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]),
                 "+v"(y[12])
               :
               : "memory");
  const double hs = c < 13 ? 0.5 : 0.0;
#pragma unroll
  for (int i = 0; i < 13; ++i) X[i] = __builtin_fma(hs, y[i] - X[i], X[i]);
}
// the step whose predict stores the rows for the symmetrisation at step k + 1
__device__ __forceinline__ bool sym_store_step(int k, int N) { return k + 1 < N && sym_step(k + 1); }
template <int S>
__device__ __forceinline__ void sym_average(double (&X)[S], double* t, int c) {
  if (c < S) {
#pragma unroll
    for (int i = 0; i < S; ++i) t[i * S + c] = X[i];
  }
  wave_sync();
  // row c of the scratch (column c of Sigma) in one asm block: plain C++ reads here
  // were sunk one by one under the lane condition (13 branches, each waiting alone);
  // then Sigma <- (Sigma + Sigma^T) / 2 on lanes < S by one FMA per row (a per-row
  // lane mask "c < i" would hold 13 loop-invariant SGPR pairs: the closed-form
  // kernel spilled 63 SGPRs with it)
  const int cr = c < S ? c : 0;
  const double hs = c < S ? 0.5 : 0.0;
  double y[S];
  LdsRow<S>::run(lds_addr(t) + 8u * S * cr, y);
#pragma unroll
  for (int i = 0; i < S; ++i) X[i] = __builtin_fma(hs, y[i] - X[i], X[i]);
  wave_sync();
}

// per-lane DMA source offset of piece j: lane q = 64 j + lane carries chunk
// q % CH of problem q / CH of the wave (OOB sentinel for unused lanes)
template <int CH>
__device__ __forceinline__ unsigned chunk_voff(int j, int lane, long long wave_prob0,
                                               long long pb0, long long batch, long long pstr) {
  const int q = 64 * j + lane;
  const int p = q / CH, r = q % CH;
  const long long pe = wave_prob0 + p < batch ? wave_prob0 + p : batch - 1;
  return (q < kProbPerWave * CH) ? (unsigned)((pe - pb0) * pstr + r * 16) : 0x7FFFFFFFu;
}

// First index < cnt of a non-finite element of p (INT_MAX if none), scanned by the
// whole wave in chunks of 64 x 64 elements (64 loads in flight per lane: the scan is
// latency-bound, one round trip per chunk); stops after the first chunk that holds
// one.  Wave-uniform result.
__device__ __forceinline__ int wave_first_nonfinite(const double* p, long long cnt, int lane) {
  constexpr int U = 64;
  int found = INT_MAX;
#pragma unroll 1
  for (long long base = 0; base < cnt; base += 64 * U) {
    // unconditional loads (a clamped index past the end): a load under "i < cnt"
    // became a branch with its own vmcnt(0) wait, 64 serial round trips per chunk
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + u * 64 + lane;
      v[u] = p[i < cnt ? i : cnt - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + u * 64 + lane;
      if (i < cnt && !finite_val(v[u]) && (int)i < found) found = (int)i;
    }
    if (__any(found != INT_MAX)) break;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int x = __shfl_xor(found, o);
    found = x < found ? x : found;
  }
  return found;
}
// Any non-finite element in K small arrays (each at most 256 elements), all loads in
// flight at once (one round trip).  Wave-uniform.
template <int K>
__device__ __forceinline__ bool wave_any_nonfinite(const double* const (&p)[K],
                                                   const int (&cnt)[K], int lane) {
  double v[K][4];
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 64 * r + lane;
      v[s][r] = p[s][i < cnt[s] ? i : cnt[s] - 1];  // unconditional (see above)
    }
  bool bad = false;
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) bad = bad || (64 * r + lane < cnt[s] && !finite_val(v[s][r]));
  return __any(bad);
}
__device__ __forceinline__ int step_of(int idx, int per) { return idx == INT_MAX ? INT_MAX : idx / per; }

// Non-finite triage of the conditioned kernels' hand-overs (rerun launch).  The
// reference turns a non-finite input into a NaN inverse with ST_NONFINITE and no
// ladder (utils.py:77; the oracle's and every kernel's semantics), so
// with h_poison = 1 + the first stage whose inputs are non-finite (1 for shared
// inputs: R^-1, z0 / xg, u_ref, Q, P, w) and h_qt = the first horizon whose
// terminal block is non-finite, J(t) is NaN for every t >= h_nf = min(h_poison,
// h_qt) as soon as h_poison <= h_qt + 1 (the usual shape: a rollout that leaves
// the finite range at x_k poisons stage k and horizon k's terminal block at once).
// When the conditioned kernel's first flag came at or after h_nf, its J(t < h_nf)
// were computed from finite inputs before any flag: the problem's outcome is that
// curve, NaN from h_nf on, status ST_NONFINITE and the fused argmin replayed over
// it -- what the reference association computes, without the sequential rerun
// (0.8 ms of latency for one wave).  Returns this lane's "resolved".
template <int S, int MM, bool TRAJ>
__device__ __forceinline__ bool nonfinite_resolve(const LftArgs<double>& a, int lane, int g,
                                               long long wave_prob0, bool need_me, int st_me) {
  const unsigned long long nb = __ballot(need_me);
  const int N = a.n;
  const int INF = N + 1;
  bool resolved = false;
#pragma unroll 1
  for (int gg = 0; gg < kProbPerWave; ++gg) {
    if (((nb >> (16 * gg)) & 0xffffull) == 0ull) continue;  // wave-uniform
    const long long pb = wave_prob0 + gg;
    const int kf = HOP_HANDOVER_HORIZON(__shfl(st_me, 16 * gg));  // 0: prologue / forced
    int kS = INT_MAX, h_qt = INF;
    bool shared;
    if constexpr (TRAJ) {
      constexpr int NN = S - 1;
      static_assert(NN * NN <= 256 && MM * MM <= 256, "shared arrays of one scan round trip");
      const TrajArgs<double>& t = a.tr;
      const double* const sp[6] = {a.R + pb * a.r_bstride, t.xg + pb * t.xg_bs,
                                   t.u_ref + pb * t.ur_bs, t.Q + pb * t.q_bs, t.P + pb * t.p_bs,
                                   t.w + pb * t.w_bs};
      const int sc[6] = {MM * MM, NN, MM, NN * NN, NN * NN, 1};
      shared = wave_any_nonfinite<6>(sp, sc, lane);
      // x_k feeds stage k and horizon k's terminal block
      const int kX = step_of(wave_first_nonfinite(t.X + pb * (long long)(a.nalloc + 1) * NN,
                                                  (long long)(N + 1) * NN, lane), NN);
      if (kX != INT_MAX && kX >= 1) h_qt = kX;
      if (kX != INT_MAX && kX < N) kS = kX;
      // the other stage inputs matter only before kX (h_poison <= kX + 1 already)
      const long long steps = kX < N ? kX : N;
      const long long na = a.nalloc;
      kS = min(kS, step_of(wave_first_nonfinite(t.A + pb * na * NN * NN, steps * NN * NN, lane), NN * NN));
      kS = min(kS, step_of(wave_first_nonfinite(t.Bm + pb * na * NN * MM, steps * NN * MM, lane), NN * MM));
      kS = min(kS, step_of(wave_first_nonfinite(t.ares + pb * na * NN, steps * NN, lane), NN));
      kS = min(kS, step_of(wave_first_nonfinite(t.U + pb * na * MM, steps * MM, lane), MM));
      if (t.qxx_extra)
        kS = min(kS, step_of(wave_first_nonfinite(t.qxx_extra + pb * na * NN * NN, steps * NN * NN, lane), NN * NN));
      if (t.qx_extra)
        kS = min(kS, step_of(wave_first_nonfinite(t.qx_extra + pb * na * NN, steps * NN, lane), NN));
      if (t.c_extra) kS = min(kS, step_of(wave_first_nonfinite(t.c_extra + pb * na, steps, lane), 1));
    } else {
      constexpr int SS = S * S, SM = S * MM;
      const long long na = a.nalloc;
      const double* const sp[2] = {a.R + pb * a.r_bstride, a.z0 + pb * a.z_bstride};
      const int sc[2] = {MM * MM, S};
      shared = wave_any_nonfinite<2>(sp, sc, lane);
      const int kq = step_of(wave_first_nonfinite(a.QT + pb * na * SS, (long long)N * SS, lane), SS);
      if (kq != INT_MAX) h_qt = kq + 1;
      // stages 0 .. h_qt decide h_poison <= h_qt + 1
      const long long steps = h_qt < N ? h_qt + 1 : N;
      kS = min(kS, step_of(wave_first_nonfinite(a.Q + pb * na * SS, steps * SS, lane), SS));
      kS = min(kS, step_of(wave_first_nonfinite(a.A + pb * na * SS, steps * SS, lane), SS));
      kS = min(kS, step_of(wave_first_nonfinite(a.B + pb * na * SM, steps * SM, lane), SM));
    }
    const int h_poison = shared ? 1 : (kS != INT_MAX ? kS + 1 : INF);
    const int h_nf = h_poison < h_qt ? h_poison : h_qt;
    const bool ok = HOP_TRIAGE_ACCEPTS(kf, h_poison, h_qt, N);
    if (ok) {  // wave-uniform
      double* J = a.J + pb * N;
      const double qnan = __builtin_nan("");
#pragma unroll 1
      for (int t = h_nf + lane; t <= N; t += 64) J[t - 1] = qnan;
      if (a.t_max > 0 && a.t_star != nullptr) {
        // the fused argmin, replayed over the stored curve in one pass: its sequential
        // rule (the first horizon t_min initialises, a NaN wins and sticks, a strictly
        // smaller value replaces) is "the first NaN of the window, else the first
        // minimiser", with a virtual (0, 0.0) first when t_min < 1
        const int t_hi = a.t_max < N ? a.t_max : N;
        int nan_t = INT_MAX, min_t = INT_MAX;
        double min_v = 0.0;
#pragma unroll 1
        for (int t = 1 + lane; t <= N; t += 64) {
          const bool in = t >= a.t_min && (t == a.t_min || t <= t_hi);
          const double jk = t < h_nf ? J[t - 1] : qnan;  // (at most 2 per lane at N = 100)
          if (in) {
            if (jk != jk) {
              nan_t = t < nan_t ? t : nan_t;
            } else if (min_t == INT_MAX || jk < min_v) {
              min_v = jk;
              min_t = t;
            }
          }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          const int xn = __shfl_xor(nan_t, o);
          nan_t = xn < nan_t ? xn : nan_t;
          const int xt = __shfl_xor(min_t, o);
          const double xv = __shfl_xor(min_v, o);
          if (xt != INT_MAX && (min_t == INT_MAX || xv < min_v || (xv == min_v && xt < min_t))) {
            min_v = xv;
            min_t = xt;
          }
        }
        if (lane == 0) {
          int tbest = 0;
          double best = 0.0;
          if (a.t_min < 1) {  // the virtual (0, 0.0): only a NaN or a negative value replaces it
            if (nan_t != INT_MAX) {
              tbest = nan_t;
              best = qnan;
            } else if (min_t != INT_MAX && min_v < 0.0) {
              tbest = min_t;
              best = min_v;
            }
          } else if (nan_t != INT_MAX) {
            tbest = nan_t;
            best = qnan;
          } else if (min_t != INT_MAX) {
            tbest = min_t;
            best = min_v;
          }
          a.t_star[pb] = tbest;
          a.j_star[pb] = best;
        }
      }
      if (lane == 0) a.status[pb] = (int)ST_NONFINITE;
    }
    if (gg == g) resolved = ok;
  }
  return resolved;
}

// The exact-size LFT sweep of one wave's 4 problems (the kernel below).  need: -1 =
// a.cond's semantics (rerun launch: the problems whose status carries ST_RERUN);
// 0 / 1 = this lane's problem is (not) recomputed -- the conditioned kernel's fused
// hand-over passes its own flags here instead of a second launch.
template <class C, int S, int MM>
__device__ __forceinline__ void lft_v2_body(LftArgs<double> a, int need_in) {
  using G = Geo<S, MM>;
  constexpr bool OFF = offset_form<C>();
  constexpr bool TRAJ = has_traj<C>();
  static_assert(!TRAJ || (OFF && C::ELIM), "trajectory form: SchedLdl family");
  constexpr int NN = G::NN;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int WB = TRAJ ? G::WAVE_BYTES_T : G::WAVE_BYTES;
  unsigned char* wbase = smem_raw + w * WB;
  const unsigned wlds = (unsigned)(uintptr_t)wbase;  // LDS byte address (wave-uniform)
  double* tile = reinterpret_cast<double*>(wbase + G::OFF_T) + g * kLdsTile;
  const double* imQ = reinterpret_cast<const double*>(wbase + G::OFF_Q + g * G::IMGM);
  const double* imA = reinterpret_cast<const double*>(wbase + G::OFF_A + g * G::IMGM);
  const double* imT = reinterpret_cast<const double*>(wbase + G::OFF_QT + g * G::IMGM);
  const double* imB = reinterpret_cast<const double*>(wbase + G::OFF_B + g * G::IMGB);
#pragma unroll 1
  for (int i = c; i < kLdsTile; i += kRowLanes) tile[i] = 0.0;

  const long long wave_prob0 = ((long long)blockIdx.x * kWavesPerBlock + w) * kProbPerWave;
  const long long prob = wave_prob0 + g;
  bool valid = prob < a.batch;
  if (need_in >= 0) {  // fused hand-over: the caller's flags
    valid = valid && need_in != 0;
    if (!__any(valid)) return;
  } else if (a.cond & 1) {  // rerun launch after SchedCond: only the problems it handed over
    const int st_in = valid ? a.status[prob] : 0;
    bool need = valid && (st_in & (int)ST_RERUN);
    // hand-overs explained by non-finite inputs take the reference's outcome here
    // instead of a recompute (bit 4: a forced hand-over, never triaged)
    if (!(a.cond & 16) && __any(need)) {  // called by the whole wave (lane-0 writes, shuffles)
      const bool resolved = nonfinite_resolve<S, MM, TRAJ>(a, lane, g, wave_prob0, need, st_in);
      need = need && !resolved;
    }
    if (a.cond & 8) return;  // triage only (HOP_OPT_NO_RERUN): the rest keep their hand-over word
    if (!__any(need)) return;  // wave-uniform; no workgroup barrier in this kernel
    valid = need;
  }
  const long long pb0 = wave_prob0 < a.batch ? wave_prob0 : a.batch - 1;  // wave-uniform
  const int N = a.n, mt = a.max_tries;
  constexpr int SS = S * S, SM = S * MM;
  const long long pstrM = (long long)a.nalloc * SS * 8;  // bytes per problem (Q/A/QT)
  const long long pstrB = (long long)a.nalloc * SM * 8;

  // buffer descriptors for the wave's 4 problems (bounds-checked: OOB -> 0)
  auto mk = [&](const double* base, long long pstr) {
    // exact bounds: range checking is per dword (tools/ubench_oob.hip), so the
    // last 16-B chunk of the tensor returns its valid dwords and zeros -- no
    // read past the allocation (which can end on an unmapped page)
    const long long left = (a.batch - pb0) * pstr;
    const unsigned nrec = left > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (unsigned)left;
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double*>(base) + pb0 * (pstr / 8), (short)0, (int)nrec, 0x00020000);
  };
  // augmented form: Q, A, QT, B images; trajectory form: A, B, x, a, u pieces
  const long long pstA = (long long)a.nalloc * NN * NN * 8, pstR = (long long)a.nalloc * NN * MM * 8;
  const long long pstX = (long long)(a.nalloc + 1) * NN * 8, pstV = (long long)a.nalloc * NN * 8;
  const long long pstU = (long long)a.nalloc * MM * 8;
  const __amdgpu_buffer_rsrc_t rQ = TRAJ ? mk(a.tr.A, pstA) : mk(a.Q, pstrM),
                               rA = TRAJ ? mk(a.tr.Bm, pstR) : mk(a.A, pstrM),
                               rT = TRAJ ? mk(a.tr.X, pstX) : mk(a.QT, pstrM),
                               rB = TRAJ ? mk(a.tr.ares, pstV) : mk(a.B, pstrB),
                               rU = TRAJ ? mk(a.tr.U, pstU) : rB;
  // per-lane chunk offsets (static over steps)
  unsigned voM[G::NJM], voB[G::NJB];
#pragma unroll
  for (int j = 0; j < G::NJM; ++j) {
    const int q = 64 * j + lane;
    const int p = q / G::CHM, r = q % G::CHM;
    long long pe = wave_prob0 + p < a.batch ? wave_prob0 + p : a.batch - 1;
    voM[j] = (q < kProbPerWave * G::CHM) ? (unsigned)((pe - pb0) * pstrM + r * 16) : 0x7FFFFFFFu;
  }
#pragma unroll
  for (int j = 0; j < G::NJB; ++j) {
    const int q = 64 * j + lane;
    const int p = q / G::CHB, r = q % G::CHB;
    long long pe = wave_prob0 + p < a.batch ? wave_prob0 + p : a.batch - 1;
    voB[j] = (q < kProbPerWave * G::CHB) ? (unsigned)((pe - pb0) * pstrB + r * 16) : 0x7FFFFFFFu;
  }
  unsigned voTA[G::NJA], voTR[G::NJR], voTX[G::NJX], voTV[G::NJV], voTU[G::NJU];
  if constexpr (TRAJ) {
#pragma unroll
    for (int j = 0; j < G::NJA; ++j)
      voTA[j] = chunk_voff<G::CHA>(j, lane, wave_prob0, pb0, a.batch, pstA);
#pragma unroll
    for (int j = 0; j < G::NJR; ++j)
      voTR[j] = chunk_voff<G::CHR>(j, lane, wave_prob0, pb0, a.batch, pstR);
#pragma unroll
    for (int j = 0; j < G::NJX; ++j)
      voTX[j] = chunk_voff<G::CHX>(j, lane, wave_prob0, pb0, a.batch, pstX);
#pragma unroll
    for (int j = 0; j < G::NJV; ++j)
      voTV[j] = chunk_voff<G::CHV>(j, lane, wave_prob0, pb0, a.batch, pstV);
#pragma unroll
    for (int j = 0; j < G::NJU; ++j)
      voTU[j] = chunk_voff<G::CHU>(j, lane, wave_prob0, pb0, a.batch, pstU);
  }
  // dma_step20 / dma_traj10 take the voffsets lowered by their pieces' instruction offsets
  unsigned voMl[G::NJM], voBl[G::NJB], voTAl[G::NJA], voTRl[G::NJR];
#pragma unroll
  for (int j = 0; j < G::NJM; ++j) voMl[j] = dma_voff_lowered(voM[j], j);
#pragma unroll
  for (int j = 0; j < G::NJB; ++j) voBl[j] = dma_voff_lowered(voB[j], j);
#pragma unroll
  for (int j = 0; j < G::NJA; ++j) voTAl[j] = TRAJ ? dma_voff_lowered(voTA[j], j) : 0u;
#pragma unroll
  for (int j = 0; j < G::NJR; ++j) voTRl[j] = TRAJ ? dma_voff_lowered(voTR[j], j) : 0u;
  auto dma_step = [&](int k) {  // Q, A, B, QT of step k
    if constexpr (TRAJ) {  // A_k, B_k, x_{k+1}, a_k, u_k
      const unsigned soA = (unsigned)(k * NN * NN * 8), soR = (unsigned)(k * NN * MM * 8),
                     soV = (unsigned)(k * NN * 8), soU = (unsigned)(k * MM * 8);
      const unsigned soX = soV + NN * 8;
      if constexpr (G::NJA == 5 && G::NJR == 2 && G::NJX == 1 && G::NJV == 1 && G::NJU == 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        dma_traj10<G::OFF_A, G::OFF_B, G::OFF_VX, G::OFF_VA, G::OFF_VU>(
            voTAl, voTRl, voTX[0], voTV[0], voTU[0], rQ, rA, rT, rB, rU, wlds, soA, soR, soX, soV,
            soU);
        return;
      }
#pragma unroll
      for (int j = 0; j < G::NJA; ++j) dma16(voTA[j], rQ, wlds + G::OFF_A + 1024 * j, soA);
#pragma unroll
      for (int j = 0; j < G::NJR; ++j) dma16(voTR[j], rA, wlds + G::OFF_B + 1024 * j, soR);
#pragma unroll
      for (int j = 0; j < G::NJX; ++j) dma16(voTX[j], rT, wlds + G::OFF_VX + 1024 * j, soX);
#pragma unroll
      for (int j = 0; j < G::NJV; ++j) dma16(voTV[j], rB, wlds + G::OFF_VA + 1024 * j, soV);
#pragma unroll
      for (int j = 0; j < G::NJU; ++j) dma16(voTU[j], rU, wlds + G::OFF_VU + 1024 * j, soU);
      return;
    }
    const unsigned soM = (unsigned)(k * SS * 8), soB = (unsigned)(k * SM * 8);
    if constexpr (C::DMA1 && G::NJM == 6 && G::NJB == 2) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_step20<G::OFF_Q, G::OFF_A, G::OFF_B, G::OFF_QT>(voMl, voBl, rQ, rA, rB, rT, wlds, soM,
                                                         soB);
      return;
    }
#pragma unroll
    for (int j = 0; j < G::NJM; ++j) dma16(voM[j], rQ, wlds + G::OFF_Q + 1024 * j, soM);
#pragma unroll
    for (int j = 0; j < G::NJM; ++j) dma16(voM[j], rA, wlds + G::OFF_A + 1024 * j, soM);
#pragma unroll
    for (int j = 0; j < G::NJB; ++j) dma16(voB[j], rB, wlds + G::OFF_B + 1024 * j, soB);
#pragma unroll
    for (int j = 0; j < G::NJM; ++j) dma16(voM[j], rT, wlds + G::OFF_QT + 1024 * j, soM);
  };

  const long long pb = valid ? prob : a.batch - 1;
  const double* zp = a.z0 + pb * a.z_bstride;
  const double zc = (!C::ELIM && c < S) ? zp[c < S ? c : 0] : 0.0;
  if constexpr (C::ELIM) {  // tile row S holds z0 (lane S of Ebar / X0, see quad_inverse)
    static_assert(S < kRowLanes, "bordered elimination needs a free lane");
    wave_sync();  // the zeroing loop wrote these words from other lanes
    if (c < S) tile[S * kLdsRow + c] = TRAJ ? (c == NN ? 1.0 : 0.0) : zp[c];  // z0 = e_s
  }
  // trajectory form: per-lane constants and the constant parts of the Q / QT images
  double xg_c = 0.0, ur_c = 0.0, w2 = 0.0, qdiag = 0.0, pdiag = 0.0, pcc = 0.0;
  double qe_k = 0.0, eqe_k = 0.0;  // Q e_k and e_k^T Q e_k (carried from step k-1)
  bool wrap_c = false;
  double* cq = reinterpret_cast<double*>(wbase + G::OFF_CQ) + g * NN * NN;
  double qr_n[NN], pr_n[NN];       // rows c of Q and P for the next step's build
  auto load_rows = [&]() {
    if constexpr (TRAJ) {
      const int cc = c < NN ? c : 0;
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        qr_n[j] = cq[j * NN + cc];
        pr_n[j] = imT[j * S + cc];
      }
    }
  };
  if constexpr (TRAJ) {
    const TrajArgs<double>& t = a.tr;
    const double* Qg = t.Q + pb * t.q_bs;
    const double* Pg = t.P + pb * t.p_bs;
    const int cc = c < NN ? c : 0;
    if (c < NN) {  // raw Q (Q e, augmented.py:35), transposed
#pragma unroll
      for (int j = 0; j < NN; ++j) cq[j * NN + c] = Qg[c * NN + j];
    }
    pcc = Pg[cc * NN + cc];
    xg_c = c < NN ? t.xg[pb * t.xg_bs + cc] : 0.0;
    ur_c = c < MM ? t.u_ref[pb * t.ur_bs + (c < MM ? c : 0)] : 0.0;
    w2 = 2.0 * t.w[pb * t.w_bs];
    wrap_c = c < NN && ((t.wrap_mask >> c) & 1u);
    // diagonals with chol_inv's first jitter and the offset form folded in
    // (the value the augmented path reaches with diag_add)
    qdiag = (0.5 * (Qg[cc * NN + cc] + Qg[cc * NN + cc]) + t.q_reg) + (1e-9 - 1.0);
    pdiag = Pg[cc * NN + cc] + (1e-9 - 1.0);
    double* wq = const_cast<double*>(imQ);
    double* wt = const_cast<double*>(imT);
    // step 0's Q e_0 and e_0^T Q e_0; later steps carry Q e_{k+1} from step k
    {
      const double* X0 = t.X + pb * (long long)(a.nalloc + 1) * NN;
      double e0 = c < NN ? X0[cc] - xg_c : 0.0;
      if (t.wrap_mask != 0u) {
        const double w0 = wrap_angle(e0);
        e0 = wrap_c ? w0 : e0;
      }
      double q4[4] = {0.0, 0.0, 0.0, 0.0};
      double qr0[NN];
#pragma unroll
      for (int j = 0; j < NN; ++j) qr0[j] = c < NN ? Qg[cc * NN + j] : 0.0;
      LaneDot4<NN>::fma(q4, e0, qr0);
      qe_k = (q4[0] + q4[1]) + (q4[2] + q4[3]);
      eqe_k = lane_sum<NN>(e0 * qe_k);
    }
    if (c < NN) {  // column c: _sym(Q) + q_reg I, and P (augmented.py:33, 82)
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        wq[i * S + c] = 0.5 * (Qg[i * NN + c] + Qg[c * NN + i]) + (i == c ? t.q_reg : 0.0);
        wt[i * S + c] = Pg[i * NN + c];
      }
    }
    load_rows();
  }
  unsigned st = 0;
  // R^-1 (cached, shared or per problem) as columns on lanes 0..MM-1
  double rinv[MM];
  {
    const double* Rp = a.R + pb * a.r_bstride;
#pragma unroll
    for (int i = 0; i < MM; ++i) rinv[i] = (c < MM) ? Rp[i * MM + (c < MM ? c : 0)] : 0.0;
  }

  dma_step(0);
  double Eb[S], H[S], Gb[S];
  double best = 0.0;
  int tbest = 0;
  const bool fuse_argmin = a.t_max > 0;

  double jprev = 0.0;
  // J(t) bookkeeping: non-finite status and the fused argmin (np.argmin: the
  // first minimiser wins, a NaN wins)
  auto take_j = [&](int t, double jk) {
    if (!finite_val(jk)) st |= ST_NONFINITE;
    if (fuse_argmin) {
      if (t == a.t_min) {
        best = jk;
        tbest = t;
      } else if (t > a.t_min && t <= a.t_max) {
        const bool bnan = best != best, jnan = jk != jk;
        if (!bnan && (jnan || jk < best)) {
          best = jk;
          tbest = t;
        }
      }
    }
  };
  unsigned long long sec[15] = {};
  unsigned long long tprev = 0;
  auto stamp = [&](int j) {
    if constexpr (C::STAMP) {
      __builtin_amdgcn_sched_barrier(0);  // keep the sections' code on their side
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (j >= 0) sec[j] += t - tprev;
      tprev = t;
    }
  };
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    stamp(-1);
    dma_wait();
    wave_sync();
    // J of the previous step is stored only now, so that the vmcnt(0) above
    // never waits on a store issued at the end of the previous step
    if (k > 0 && valid && c == 0) a.J[prob * N + k - 1] = jprev;
    double atil = 0.0;  // trajectory form: a~_k = a_k - B_k du_k (augmented.py:50)
    if constexpr (TRAJ) {
      // build the last row / column and the diagonal of Q_aug[k] (augmented.py:31-47)
      // and QT_aug[k] (augmented.py:77-86) in the images; the rest is constant
      const double* sX = reinterpret_cast<const double*>(wbase + G::OFF_VX) + g * 2 * G::CHX;
      const double* sV = reinterpret_cast<const double*>(wbase + G::OFF_VA) + g * 2 * G::CHV;
      const double* sU = reinterpret_cast<const double*>(wbase + G::OFF_VU) + g * 2 * G::CHU;
      const double* sR = reinterpret_cast<const double*>(wbase + G::OFF_B) + g * 2 * G::CHR;
      const int cc = c < NN ? c : 0, cm = c < MM ? c : 0;
      // Per step only e_{k+1} is new: Q e_k and e_k^T Q e_k were formed at step
      // k-1 from the same e (carried), P e_{k+1} and Q e_{k+1} are formed now.
      // Every LDS load first, unconditionally at clamped addresses (a load under
      // a lane condition becomes an exec-masked branch with its own wait), then
      // the lane selects.  Row c of Q comes from the constant area, row c of P
      // is column c of the QT image (P symmetric; its diagonal kept in pcc).
      stamp(9);
      double x1 = sX[cc], av = sV[cc], uu = sU[cm];
      double rb[MM], qr[NN], pr[NN];
#pragma unroll
      for (int q = 0; q < MM; ++q) rb[q] = sR[cc * MM + q];
#pragma unroll
      for (int j = 0; j < NN; ++j) {  // loaded at the end of the previous step
        qr[j] = qr_n[j];
        pr[j] = pr_n[j];
      }
      const bool in = c < NN;
#pragma unroll
      for (int j = 0; j < NN; ++j) {
        qr[j] = in ? qr[j] : 0.0;
        pr[j] = in ? (j == c ? pcc : pr[j]) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < MM; ++q) rb[q] = in ? rb[q] : 0.0;
      double e1 = in ? x1 - xg_c : 0.0;
      stamp(10);
      if (a.tr.wrap_mask != 0u) {  // wave-uniform: no wrap work without wrapped states
        const double we1 = wrap_angle(e1);  // branch-free
        e1 = wrap_c ? we1 : e1;
      }
      const double du = c < MM ? uu - ur_c : 0.0;
      av = in ? av : 0.0;
      stamp(11);
      // Q e_{k+1}, P e_{k+1} as 4 interleaved partial sums each (a single
      // 12-deep dependent DPP chain exposes the fp64 latency at 1 wave/SIMD)
      double q4[4] = {0.0, 0.0, 0.0, 0.0}, p4[4] = {0.0, 0.0, 0.0, 0.0}, bd = 0.0;
      LaneDot4<NN>::fma(q4, e1, qr);
      LaneDot4<NN>::fma(p4, e1, pr);
      LaneDot<MM>::fma(bd, du, rb);  // (B du)[c]
      const double qe1 = (q4[0] + q4[1]) + (q4[2] + q4[3]);
      const double pe = (p4[0] + p4[1]) + (p4[2] + p4[3]);
      atil = av - bd;
      stamp(12);
      // e^T Q e and e^T P e: row sums (lane NN's value is the one stored)
      const double eqe1 = lane_sum<NN>(e1 * qe1);
      const double epe = lane_sum<NN>(e1 * pe);
      stamp(13);
      double* wq = const_cast<double*>(imQ);
      double* wt = const_cast<double*>(imT);
      if (c < NN) {
        wq[c * S + NN] = qe_k;
        wq[NN * S + c] = qe_k;
        wq[c * S + c] = qdiag;
        wt[c * S + NN] = pe;
        wt[NN * S + c] = pe;
        wt[c * S + c] = pdiag;
      } else if (c == NN) {
        wq[NN * S + NN] = ((eqe_k + w2) + a.tr.rho_reg) + (1e-9 - 1.0);
        wt[NN * S + NN] = (epe + a.tr.rho_reg) + (1e-9 - 1.0);
      }
      qe_k = qe1;
      eqe_k = eqe1;
      // no wave_sync: the image reads (LdsSym) are asm with a memory clobber and
      // one wave's LDS operations execute in order
      stamp(14);
    } else if constexpr (OFF) {
      diag_add<S, S>(imQ, c, 1e-9 - 1.0);
      diag_add<S, S>(imT, c, 1e-9 - 1.0);
    }
    // ---- stage: NE = -(Q_k)^-1 and NX = -(QT_k)^-1 together
    double NE[S], NX[S];
    stamp(0);
    neg_inverse2<C, S, S, S>(NE, imQ, NX, imT, c, mt, st);
    stamp(1);
    double at[S], brow[MM];
    if constexpr (TRAJ) {  // row c of A_aug = [[A_k, a~],[0, 1]], B_aug = [[B_k],[0]]
      const double* sA = reinterpret_cast<const double*>(wbase + G::OFF_A) + g * 2 * G::CHA;
      const double* sR = reinterpret_cast<const double*>(wbase + G::OFF_B) + g * 2 * G::CHR;
      const int cc = c < NN ? c : 0;
#pragma unroll
      for (int j = 0; j < NN; ++j) at[j] = c < NN ? sA[cc * NN + j] : 0.0;
      at[NN] = c < NN ? atil : (c == NN ? 1.0 : 0.0);
#pragma unroll
      for (int j = 0; j < MM; ++j) brow[j] = c < NN ? sR[cc * MM + j] : 0.0;
    } else {
#pragma unroll
      for (int j = 0; j < S; ++j) at[j] = imA[c * S + j];   // row c of A
#pragma unroll
      for (int j = 0; j < MM; ++j) brow[j] = imB[c * MM + j];
    }
    wave_sync();
    if (k + 1 < N) dma_step(k + 1);
    stamp(2);
    // offset form: NE, NX, NW carry +I; a product -(N + I) Y = (-N) Y - Y starts from Y
    double F[S];
    if constexpr (OFF) copy(F, at); else zero(F);
    gxy<C, true>(F, NE, at);    // F = E A^T
    double Gk[S];
    zero(Gk);
    gxty<C, false>(Gk, at, F);  // A F
    double y[MM];
    zero(y);
    acc_xy<false, double, MM, MM>(y, rinv, brow);
    acc_xty<false, double, S, MM>(Gk, brow, y);  // + B R^-1 B^T
    stamp(3);

    if (k == 0) {
#pragma unroll
      for (int i = 0; i < S; ++i) Eb[i] = -NE[i];
      if constexpr (OFF) {
#pragma unroll
        for (int i = 0; i < S; ++i) Eb[i] = (c == i) ? Eb[i] + 1.0 : Eb[i];
      }
      transpose(H, F, tile, c);
      if constexpr (C::ELIM) {  // lane S: Ebar column = z0, Fbar^T column = 0 (invariant)
#pragma unroll
        for (int i = 0; i < S; ++i) {
          Eb[i] = (c == S) ? tile[S * kLdsRow + i] : Eb[i];
          H[i] = (c == S) ? 0.0 : H[i];
        }
      }
      copy(Gb, Gk);
    } else {
      double NW[S];
#pragma unroll
      for (int i = 0; i < S; ++i) NW[i] = Gb[i] - NE[i];  // E_k + Gbar
      neg_inverse_reg<C, S>(NW, tile, c, mt, st, -1.0);     // NW = -W
      stamp(4);
      double Z[S];
      if constexpr (OFF) copy(Z, H); else zero(Z);
      gxy<C, true>(Z, NW, H);     // Z = W Fbar^T
      gxty<C, true>(Eb, H, Z);    // Ebar -= Fbar W Fbar^T
      zero(H);
      gxty<C, false>(H, F, Z);    // H' = F^T W Fbar^T
      if constexpr (OFF) copy(Z, F); else zero(Z);
      gxy<C, true>(Z, NW, F);     // W F
      copy(Gb, Gk);
      gxty<C, true>(Gb, F, Z);    // Gbar = G - F^T W F
    }
    stamp(5);

    // ---- query horizon t = k + 1
#pragma unroll
    for (int i = 0; i < S; ++i) NX[i] = Gb[i] - NX[i];   // QT^-1 + Gbar
    if constexpr (has_qldl<C>()) {
      double X0[S];
      query_x0_ldl<C, S>(NX, H, Eb, X0, tile, c, mt, st);  // X0 = Ebar - Fbar Wt Fbar^T
      copy(NX, X0);
      stamp(6);
    } else {
      neg_inverse_reg<C, S>(NX, tile, c, mt, st, -1.0);     // NX = -Wt
      stamp(6);
      double V[S];
      if constexpr (OFF) copy(V, H); else zero(V);
      gxy<C, true>(V, NX, H);      // Wt Fbar^T
      copy(NX, Eb);
      gxty<C, true>(NX, H, V);     // X0 = Ebar - Fbar Wt Fbar^T
    }
    stamp(7);
    double jk;
    if constexpr (C::ELIM) {
      jk = 0.5 * quad_inverse<C, S>(NX, tile, c, mt, st);
    } else {
      neg_inverse_reg<C, S>(NX, tile, c, mt, st);             // NX = -P0
      double u = 0.0;
      LaneDot<S>::fma_neg(u, zc, NX);  // (z0^T P0)[c]
      jk = 0.5 * row_sum((c < S) ? u * zc : 0.0);
    }
    stamp(8);
    load_rows();  // trajectory form: next step's Q / P rows (constant LDS data)
    take_j(k + 1, jk);
    jprev = jk;
  }
  dma_wait();
  if constexpr (C::STAMP) {
    if (lane == 0) {
      for (int j = 0; j < 15; ++j) atomicAdd(&g_hop_stamp[j], sec[j]);
      atomicAdd(&g_hop_stamp[15], 1ull);
    }
  }
  if (valid && c == 0) {
    if (N > 0) a.J[prob * N + N - 1] = jprev;
    a.status[prob] = (int)st;
    if (fuse_argmin && a.t_star != nullptr) {
      a.t_star[prob] = tbest;
      a.j_star[prob] = best;
    }
  }
}

template <class C, int S, int MM>
__global__ __launch_bounds__(256, 1) void lft_sweep_v2_kernel(LftArgs<double> a) {
  lft_v2_body<C, S, MM>(a, -1);
}

// ===========================================================================
// The rerun as a pipeline over the workgroup's waves (round 5)
//
// A problem the conditioned kernel hands over (a genuine chol_inv escalation, not
// explained by non-finite inputs) is recomputed with the reference association,
// horizon_selection.py:36-86.  Its per-step work splits into
//   stage  E_k = chol_inv(Q_k), F_k = E_k A_k^T, G_k = A_k F_k + B_k R^-1 B_k^T
//          (:57-64)                                          independent per k
//   chain  W_k = chol_inv(E_k + Gbar), Gbar = G_k - F_k^T W_k F_k           sequential
//          Ebar -= Fbar W_k Fbar^T, Fbar^T <- F_k^T W_k Fbar^T      sequential, behind it
//   query  X_t = chol_inv(QT_t), X0 = Ebar - Fbar (X_t + Gbar)^-1 Fbar^T,
//          J = 1/2 z0^T chol_inv(X0) z0 (:77-85)                     independent per t
// and the one-wave LFT kernel runs all of it in sequence (about 0.8 ms at N = 100).
// Here the workgroup's four waves run it as a pipeline with one barrier per beat of
// BS steps: wave 2 computes the stage blocks of beat b (its four rows, four steps),
// wave 0 the Gbar chain of beat b - 1, wave 1 the Ebar / Fbar^T chain of beat b - 2
// (from the W_k wave 0 left), wave 3 the queries of beat b - 3 (four rows, four
// horizons); the blocks pass through LDS rings.  Every row runs the LFT kernel's own
// code on the same values (sweeps, ladders, products, the LDL^T query), so J, the
// status word and the argmin are bitwise those of lft_sweep_v2_kernel<SchedLdlDma>
// (tests/test_gpu_parity.py test_pipelined_rerun_*).  A workgroup with more than
// kPipeMax problems left after the triage runs the LFT body on them instead (one
// wave per four problems in parallel beats a sequence of pipelines there).
// ===========================================================================
constexpr int kPipeMax = 4;  // problems per workgroup the pipeline takes (above: the LFT body)
constexpr int kPipeBS = 4;   // steps per beat
// The chains' products split over the four rows of the wave (HOP_PIPE_SPLIT=0: every
// row computes the whole product, as the LFT kernel does).  Row g forms output rows
// g, 4 + g, 8 + g (and 12 for g = 0): the i-th of them is the i-th register of a
// four-register slice.  out[r] += sum_j bcast_j(x[r]) y[j] needs x's rows of the slice
// and all of y; out[r] += sum_j x[j][r] y[j] is the same with x's columns of the slice
// (read transposed from LDS).  Each output element is the same FMA chain in the same
// order as in the whole product, so the values are bitwise the same; the slices meet
// again through LDS where the next product needs every row.
#ifndef HOP_PIPE_SPLIT
#define HOP_PIPE_SPLIT 1
#endif
constexpr bool kPipeSplit = HOP_PIPE_SPLIT != 0;

// rows 4 i + g of a matrix in LDS (row stride RS doubles; rows past S - 1 read row S - 1)
template <int S, int RS>
__device__ __forceinline__ void get_slice(const double* m, int g, int c, double (&x)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * i + g < S ? 4 * i + g : S - 1;
    x[i] = m[r * RS + c];
  }
}
// columns 4 i + g, transposed: x[i] on lane c = M[c][4 i + g] (clamped to the matrix)
template <int S, int RS>
__device__ __forceinline__ void get_slice_t(const double* m, int g, int c, double (&x)[4]) {
  const int cr = c < S ? c : S - 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = 4 * i + g < S ? 4 * i + g : S - 1;
    x[i] = m[cr * RS + col];
  }
}
template <int S, int RS>
__device__ __forceinline__ void put_slice(double* m, int g, int c, const double (&x)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * i + g < S) m[(4 * i + g) * RS + c] = x[i];
}
// the slice of a matrix held whole in registers (three lane selects per register)
template <int S>
__device__ __forceinline__ void sel_slice(const double (&x)[S], int g, double (&o)[4]) {
  auto at = [&](int r) { return x[r < S ? r : S - 1]; };
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double a = (g & 1) ? at(4 * i + 1) : at(4 * i);
    const double b = (g & 1) ? at(4 * i + 3) : at(4 * i + 2);
    o[i] = (g & 2) ? b : a;
  }
}

template <int S, int MM, int BS>
struct PipeGeo {
  using G = Geo<S, MM>;
  static constexpr int MAT = S * 16 * 8;  // one S-row register matrix, all 16 lanes of a row
  // ring depths in beats (production beat j -> last consumption beat)
  static constexpr int D_NE = 3, D_F = 3, D_GK = 2, D_NW = 2, D_GB = 3, D_EB = 2, D_H = 2;
  static constexpr int OFF_NE = 0;
  static constexpr int OFF_F = OFF_NE + D_NE * BS * MAT;
  static constexpr int OFF_GK = OFF_F + D_F * BS * MAT;
  static constexpr int OFF_NW = OFF_GK + D_GK * BS * MAT;
  static constexpr int OFF_GB = OFF_NW + D_NW * BS * MAT;
  static constexpr int OFF_EB = OFF_GB + D_GB * BS * MAT;
  static constexpr int OFF_H = OFF_EB + D_EB * BS * MAT;
  // row images of the stage wave (Q, A, B) and the query wave (QT), then a zero pad
  // for the lanes past S - 1 that read past an image (their values are never used)
  static constexpr int OFF_IQ = OFF_H + D_H * BS * MAT;
  static constexpr int OFF_IA = OFF_IQ + 4 * G::IMGM;
  static constexpr int OFF_IB = OFF_IA + 4 * G::IMGM;
  static constexpr int OFF_IT = OFF_IB + 4 * G::IMGB;
  static constexpr int OFF_PAD = OFF_IT + 4 * G::IMGM;
  static constexpr int OFF_TILE = OFF_PAD + 512;      // waves 0, 1, 3: a tile per row
  static constexpr int OFF_MISC = OFF_TILE + 12 * kLdsTile * 8;
  static constexpr int BYTES = OFF_MISC + 256;       // need flags, status word
  static constexpr int ZERO_FROM = OFF_IQ;           // zeroed per problem: images .. tiles
};

template <int S>
__device__ __forceinline__ void ring_put(unsigned char* base, int off, int slot, int c,
                                         const double (&x)[S]) {
  double* m = reinterpret_cast<double*>(base + off) + slot * S * 16;
#pragma unroll
  for (int i = 0; i < S; ++i) m[i * 16 + c] = x[i];
}
template <int S>
__device__ __forceinline__ void ring_get(const unsigned char* base, int off, int slot, int c,
                                         double (&x)[S]) {
  const double* m = reinterpret_cast<const double*>(base + off) + slot * S * 16;
#pragma unroll
  for (int i = 0; i < S; ++i) x[i] = m[i * 16 + c];
}

// The fused argmin's sequential rule (horizon t = t_min initialises; a NaN wins and
// sticks; a strictly smaller value replaces) applied to one more horizon.
__device__ __forceinline__ void argmin_take(int t, double jk, int t_min, int t_max, double& best,
                                            int& tbest) {
  if (t == t_min) {
    best = jk;
    tbest = t;
  } else if (t > t_min && t <= t_max) {
    const bool bnan = best != best, jnan = jk != jk;
    if (!bnan && (jnan || jk < best)) {
      best = jk;
      tbest = t;
    }
  }
}

template <class C, int S, int MM, int BS>
__device__ __forceinline__ void pipe_problem(const LftArgs<double>& a, long long p) {
  using PG = PipeGeo<S, MM, BS>;
  using G = Geo<S, MM>;
  constexpr bool TRAJ = has_traj<C>();
  static_assert(C::ELIM && has_qldl<C>() && offset_form<C>(),
                "the LFT kernel's schedules (SchedLdlDma, SchedLdlTraj)");
  constexpr int NN = S - 1;
  static_assert(PG::BYTES <= 160 * 1024, "one workgroup's LDS");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  unsigned char* base = smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = a.n, mt = a.max_tries;
  constexpr int SS = S * S, SM = S * MM;
  // zero the images, the pad and the tiles; z0 into row S of every tile
  {
    double* z = reinterpret_cast<double*>(base + PG::ZERO_FROM);
    constexpr int nz = (PG::OFF_MISC - PG::ZERO_FROM) / 8;
#pragma unroll 1
    for (int i = tid; i < nz; i += 256) z[i] = 0.0;
    __syncthreads();
    if (tid < 12 * S) {  // the trajectory form's z0 is e_s (augmented.py:57)
      double* t = reinterpret_cast<double*>(base + PG::OFF_TILE) + (tid / S) * kLdsTile;
      t[S * kLdsRow + tid % S] = TRAJ ? (tid % S == NN ? 1.0 : 0.0) : a.z0[p * a.z_bstride + tid % S];
    }
    if (tid == 0) *reinterpret_cast<int*>(base + PG::OFF_MISC + 64) = 0;  // status word
    __syncthreads();
  }
  // R^-1 (cached): columns on lanes 0 .. MM-1
  double rinv[MM];
  {
    const double* Rp = a.R + p * a.r_bstride;
#pragma unroll
    for (int i = 0; i < MM; ++i) rinv[i] = (c < MM) ? Rp[i * MM + (c < MM ? c : 0)] : 0.0;
  }
  // trajectory form (the LFT kernel's TRAJ path, lft_v2_body): per-lane constants of
  // the in-kernel builders (augmented.py:31-56, 77-86); each row builds its step's
  // Q_aug / QT_aug image from them and the raw x_k, A_k, B_k, a_k, u_k
  const bool in = c < NN;
  const int cc = in ? c : 0, cm = c < MM ? c : 0;
  double xg_c = 0.0, ur_c = 0.0, w2 = 0.0, qdiag = 0.0, pdiag = 0.0;
  bool wrap_c = false;
  const double* Qg = nullptr;
  const double* Pg = nullptr;
  const double* Xp = nullptr;
  if constexpr (TRAJ) {
    const TrajArgs<double>& t = a.tr;
    Qg = t.Q + p * t.q_bs;
    Pg = t.P + p * t.p_bs;
    Xp = t.X + p * (long long)(a.nalloc + 1) * NN;
    xg_c = in ? t.xg[p * t.xg_bs + cc] : 0.0;
    ur_c = c < MM ? t.u_ref[p * t.ur_bs + cm] : 0.0;
    w2 = 2.0 * t.w[p * t.w_bs];
    wrap_c = in && ((t.wrap_mask >> c) & 1u);
    qdiag = (0.5 * (Qg[cc * NN + cc] + Qg[cc * NN + cc]) + t.q_reg) + (1e-9 - 1.0);
    pdiag = Pg[cc * NN + cc] + (1e-9 - 1.0);
  }
  auto err = [&](double x) {  // wrap_error(x - xg) on lane c (utils.py:131-137)
    double e = in ? x - xg_c : 0.0;
    if (a.tr.wrap_mask != 0u) {
      const double we = wrap_angle(e);
      e = wrap_c ? we : e;
    }
    return e;
  };
  const int tw = w == 3 ? 2 : w;  // tile set of waves 0, 1, 3
  double* tile = reinterpret_cast<double*>(base + PG::OFF_TILE) + (tw * 4 + g) * kLdsTile;
  double* imQ = reinterpret_cast<double*>(base + PG::OFF_IQ + g * G::IMGM);
  double* imA = reinterpret_cast<double*>(base + PG::OFF_IA + g * G::IMGM);
  double* imB = reinterpret_cast<double*>(base + PG::OFF_IB + g * G::IMGB);
  double* imT = reinterpret_cast<double*>(base + PG::OFF_IT + g * G::IMGM);
  const long long pk0 = p * (long long)a.nalloc;  // step 0 of problem p
  unsigned st = 0;
  double Gb[S], Eb[S], H[S];  // the chains' carried prefix (waves 0 and 1)
  double Gbd[4], Ebd[4], Hd[4];  // their slices (kPipeSplit)
  double best = 0.0;
  int tbest = 0;
  const int nb = (N + BS - 1) / BS;
#ifdef HOP_PIPE_STAMP  // developer timing (tools/pipe_stamps.py): per wave, the clocks busy
  // and waiting at the beat barrier; wave 0's sliced step by section
  unsigned long long t_busy = 0, t_wait = 0, t_sec[3] = {0, 0, 0};
#endif
#pragma unroll 1
  for (int b = 0; b < nb + 3; ++b) {
#ifdef HOP_PIPE_STAMP
    const unsigned long long t_b0 = __builtin_amdgcn_s_memtime();
#endif
    if (w == 2) {  // ---- stage blocks of beat b, one step per row
      const int k = BS * b + g % BS, kc = k < N ? k : N - 1;
      if (b < nb && TRAJ) {
        // Q_aug[k]: _sym(Q) + q_reg I, its bordered row / column Q e_k, corner
        // e_k^T Q e_k + 2w + rho (the LFT kernel's values: Q e_k by the same 4-way split
        // LaneDot4, the diagonal with the offset form's eps - 1 folded in); A~ row c
        const TrajArgs<double>& t = a.tr;
        const double* ar = t.A + (pk0 + kc) * NN * NN;
        const double* br = t.Bm + (pk0 + kc) * NN * MM;
        double qr[NN], qs[NN], at[S], brow[MM], rb[MM];
#pragma unroll
        for (int j = 0; j < NN; ++j) {
          qr[j] = in ? Qg[cc * NN + j] : 0.0;
          qs[j] = 0.5 * (Qg[j * NN + cc] + Qg[cc * NN + j]) + (j == c ? t.q_reg : 0.0);
          at[j] = in ? ar[cc * NN + j] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < MM; ++q) {
          rb[q] = in ? br[cc * MM + q] : 0.0;
          brow[q] = rb[q];
        }
        const double e0 = err(Xp[(long long)kc * NN + cc]);
        const double uu = t.U[(pk0 + kc) * MM + cm];
        const double av = in ? t.ares[(pk0 + kc) * NN + cc] : 0.0;
        double q4[4] = {0.0, 0.0, 0.0, 0.0};
        LaneDot4<NN>::fma(q4, e0, qr);
        const double qe = (q4[0] + q4[1]) + (q4[2] + q4[3]);
        const double eqe = lane_sum<NN>(e0 * qe);
        const double du = c < MM ? uu - ur_c : 0.0;
        double bd = 0.0;
        LaneDot<MM>::fma(bd, du, rb);  // (B du)[c]
        const double atil = av - bd;
        at[NN] = in ? atil : (c == NN ? 1.0 : 0.0);
        if (in) {
#pragma unroll
          for (int i = 0; i < NN; ++i) imQ[i * S + c] = qs[i];
          imQ[c * S + NN] = qe;
          imQ[NN * S + c] = qe;
          imQ[c * S + c] = qdiag;
        } else if (c == NN) {
          imQ[NN * S + NN] = ((eqe + w2) + t.rho_reg) + (1e-9 - 1.0);
        }
        wave_sync();
        double NE[S];
        neg_inverse<C, S, S>(NE, imQ, c, mt, st);
        double F[S];
        copy(F, at);
        gxy<C, true>(F, NE, at);    // F = E A^T
        double Gk[S];
        zero(Gk);
        gxty<C, false>(Gk, at, F);  // A F
        double y[MM];
        zero(y);
        acc_xy<false, double, MM, MM>(y, rinv, brow);
        acc_xty<false, double, S, MM>(Gk, brow, y);  // + B R^-1 B^T
        if (k < N && g < BS) {
          ring_put<S>(base, PG::OFF_NE, k % (PG::D_NE * BS), c, NE);
          ring_put<S>(base, PG::OFF_F, k % (PG::D_F * BS), c, F);
          ring_put<S>(base, PG::OFF_GK, k % (PG::D_GK * BS), c, Gk);
        }
        wave_sync();
      } else if (b < nb) {
        const double* q = a.Q + (pk0 + kc) * SS;
        const double* am = a.A + (pk0 + kc) * SS;
        const double* bm = a.B + (pk0 + kc) * SM;
        // every load in flight before the first LDS store (clamped, unconditional)
        constexpr int NQ = (SS + 15) / 16, NB = (SM + 15) / 16;
        double vq[NQ], va[NQ], vb[NB];
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
          const int e = c + 16 * u < SS ? c + 16 * u : SS - 1;
          vq[u] = q[e];
          va[u] = am[e];
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) vb[u] = bm[c + 16 * u < SM ? c + 16 * u : SM - 1];
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
          if (c + 16 * u < SS) {
            imQ[c + 16 * u] = vq[u];
            imA[c + 16 * u] = va[u];
          }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u)
          if (c + 16 * u < SM) imB[c + 16 * u] = vb[u];
        wave_sync();
        diag_add<S, S>(imQ, c, 1e-9 - 1.0);
        double NE[S];
        neg_inverse<C, S, S>(NE, imQ, c, mt, st);
        double at[S], brow[MM];
#pragma unroll
        for (int j = 0; j < S; ++j) at[j] = imA[c * S + j];
#pragma unroll
        for (int j = 0; j < MM; ++j) brow[j] = imB[c * MM + j];
        double F[S];
        copy(F, at);
        gxy<C, true>(F, NE, at);    // F = E A^T
        double Gk[S];
        zero(Gk);
        gxty<C, false>(Gk, at, F);  // A F
        double y[MM];
        zero(y);
        acc_xy<false, double, MM, MM>(y, rinv, brow);
        acc_xty<false, double, S, MM>(Gk, brow, y);  // + B R^-1 B^T
        if (k < N && g < BS) {
          ring_put<S>(base, PG::OFF_NE, k % (PG::D_NE * BS), c, NE);
          ring_put<S>(base, PG::OFF_F, k % (PG::D_F * BS), c, F);
          ring_put<S>(base, PG::OFF_GK, k % (PG::D_GK * BS), c, Gk);
        }
        wave_sync();
      }
    } else if (w == 0 && kPipeSplit) {  // ---- the Gbar chain of beat b - 1, sliced products
      const int jb = b - 1;
      if (jb >= 0 && jb < nb) {
        double* tiles = reinterpret_cast<double*>(base + PG::OFF_TILE);  // wave 0: tiles 0 .. 3
#pragma unroll 1
        for (int kk = 0; kk < BS; ++kk) {
          const int k = BS * jb + kk;
          if (k >= N) break;
          const double* mF = reinterpret_cast<const double*>(base + PG::OFF_F) +
                             (k % (PG::D_F * BS)) * S * 16;
          const double* mG = reinterpret_cast<const double*>(base + PG::OFF_GK) +
                             (k % (PG::D_GK * BS)) * S * 16;
          double Gkd[4];
          get_slice<S, 16>(mG, g, c, Gkd);
          if (k == 0) {
            copy(Gbd, Gkd);
          } else {
#ifdef HOP_PIPE_STAMP
            const unsigned long long s0 = __builtin_amdgcn_s_memtime();
#endif
            const double* mE = reinterpret_cast<const double*>(base + PG::OFF_NE) +
                               (k % (PG::D_NE * BS)) * S * 16;
            double F[S], Fd[4], Ftd[4], NEd[4], NWd[4];
            ring_get<S>(base, PG::OFF_F, k % (PG::D_F * BS), c, F);
            get_slice<S, 16>(mF, g, c, Fd);
            get_slice_t<S, 16>(mF, g, c, Ftd);
            get_slice<S, 16>(mE, g, c, NEd);
#pragma unroll
            for (int i = 0; i < 4; ++i) NWd[i] = Gbd[i] - NEd[i];  // E_k + Gbar, this row's slice
            // every row's tile gets the whole matrix (the inverse and its ladder run per row)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) put_slice<S, kLdsRow>(tiles + gg * kLdsTile, g, c, NWd);
            diag_add<S, kLdsRow>(tile, c, 1e-9 - 1.0 - (-1.0));
            wave_sync();
#ifdef HOP_PIPE_STAMP
            const unsigned long long s1 = __builtin_amdgcn_s_memtime();
#endif
            double NW[S];
            neg_inverse<C, S, kLdsRow>(NW, tile, c, mt, st);  // NW = -W
            wave_sync();
#ifdef HOP_PIPE_STAMP
            const unsigned long long s2 = __builtin_amdgcn_s_memtime();
#endif
            if (g == 0) ring_put<S>(base, PG::OFF_NW, k % (PG::D_NW * BS), c, NW);
            double Wd[4], Zd[4], Z[S];
            sel_slice<S>(NW, g, Wd);
            copy(Zd, Fd);
            gxy<C, true>(Zd, Wd, F);  // W F, this row's slice
            put_slice<S, kLdsRow>(tiles, g, c, Zd);
            wave_sync();
            lds_get<double, S>(tiles, c, Z);
            copy(Gbd, Gkd);
            gxy<C, true>(Gbd, Ftd, Z);  // Gbar = G - F^T W F, this row's slice
#ifdef HOP_PIPE_STAMP
            __builtin_amdgcn_sched_barrier(0);
            const unsigned long long s3 = __builtin_amdgcn_s_memtime();
            t_sec[0] += s1 - s0;
            t_sec[1] += s2 - s1;
            t_sec[2] += s3 - s2;
#endif
          }
          double* mB = reinterpret_cast<double*>(base + PG::OFF_GB) + (k % (PG::D_GB * BS)) * S * 16;
          put_slice<S, 16>(mB, g, c, Gbd);
        }
        wave_sync();
      }
    } else if (w == 0) {  // ---- the Gbar chain of beat b - 1 (all rows: the same step)
      const int jb = b - 1;
      if (jb >= 0 && jb < nb) {
#pragma unroll 1
        for (int kk = 0; kk < BS; ++kk) {
          const int k = BS * jb + kk;
          if (k >= N) break;
          double F[S], Gk[S];
          ring_get<S>(base, PG::OFF_F, k % (PG::D_F * BS), c, F);
          ring_get<S>(base, PG::OFF_GK, k % (PG::D_GK * BS), c, Gk);
          if (k == 0) {
            copy(Gb, Gk);
          } else {
            double NE[S], NW[S];
            ring_get<S>(base, PG::OFF_NE, k % (PG::D_NE * BS), c, NE);
#pragma unroll
            for (int i = 0; i < S; ++i) NW[i] = Gb[i] - NE[i];  // E_k + Gbar
            neg_inverse_reg<C, S>(NW, tile, c, mt, st, -1.0);     // NW = -W
            if (g == 0) ring_put<S>(base, PG::OFF_NW, k % (PG::D_NW * BS), c, NW);
            double Z[S];
            copy(Z, F);
            gxy<C, true>(Z, NW, F);     // W F
            copy(Gb, Gk);
            gxty<C, true>(Gb, F, Z);    // Gbar = G - F^T W F
          }
          if (g == 0) ring_put<S>(base, PG::OFF_GB, k % (PG::D_GB * BS), c, Gb);
        }
        wave_sync();
      }
    } else if (w == 1 && kPipeSplit) {  // ---- the Ebar / Fbar^T chain of beat b - 2, sliced
      const int jb = b - 2;
      if (jb >= 0 && jb < nb) {
        // rows 0 .. S-1 of wave 1's third and fourth tiles: the exchanges of W Fbar^T and
        // of Fbar^T (row S of every tile keeps z0)
        double* tZ = reinterpret_cast<double*>(base + PG::OFF_TILE) + 6 * kLdsTile;
        double* tH = reinterpret_cast<double*>(base + PG::OFF_TILE) + 7 * kLdsTile;
#pragma unroll 1
        for (int kk = 0; kk < BS; ++kk) {
          const int k = BS * jb + kk;
          if (k >= N) break;
          if (k == 0) {
            double F[S], NE[S];
            ring_get<S>(base, PG::OFF_F, 0, c, F);
            ring_get<S>(base, PG::OFF_NE, 0, c, NE);
#pragma unroll
            for (int i = 0; i < S; ++i) Eb[i] = -NE[i];
#pragma unroll
            for (int i = 0; i < S; ++i) Eb[i] = (c == i) ? Eb[i] + 1.0 : Eb[i];
            transpose(H, F, tile, c);
#pragma unroll
            for (int i = 0; i < S; ++i) {  // lane S: Ebar column = z0, Fbar^T column = 0
              Eb[i] = (c == S) ? tile[S * kLdsRow + i] : Eb[i];
              H[i] = (c == S) ? 0.0 : H[i];
            }
            sel_slice<S>(Eb, g, Ebd);
            sel_slice<S>(H, g, Hd);
            if (g == 0) lds_put(tH, c, H);
            wave_sync();
          } else {
            const double* mF = reinterpret_cast<const double*>(base + PG::OFF_F) +
                               (k % (PG::D_F * BS)) * S * 16;
            const double* mW = reinterpret_cast<const double*>(base + PG::OFF_NW) +
                               (k % (PG::D_NW * BS)) * S * 16;
            double NWd[4], Ftd[4], Htd[4], Zd[4], Z[S];
            get_slice<S, 16>(mW, g, c, NWd);
            get_slice_t<S, 16>(mF, g, c, Ftd);
            get_slice_t<S, kLdsRow>(tH, g, c, Htd);  // Fbar^T of the previous step, transposed
            copy(Zd, Hd);
            gxy<C, true>(Zd, NWd, H);   // Z = W Fbar^T, this row's slice
            put_slice<S, kLdsRow>(tZ, g, c, Zd);
            wave_sync();
            lds_get<double, S>(tZ, c, Z);
            gxy<C, true>(Ebd, Htd, Z);  // Ebar -= Fbar W Fbar^T
            zero(Hd);
            gxy<C, false>(Hd, Ftd, Z);  // H' = F^T W Fbar^T
            put_slice<S, kLdsRow>(tH, g, c, Hd);
            wave_sync();
            lds_get<double, S>(tH, c, H);
          }
          double* mEb = reinterpret_cast<double*>(base + PG::OFF_EB) + (k % (PG::D_EB * BS)) * S * 16;
          double* mH = reinterpret_cast<double*>(base + PG::OFF_H) + (k % (PG::D_H * BS)) * S * 16;
          put_slice<S, 16>(mEb, g, c, Ebd);
          put_slice<S, 16>(mH, g, c, Hd);
        }
        wave_sync();
      }
    } else if (w == 1) {  // ---- the Ebar / Fbar^T chain of beat b - 2
      const int jb = b - 2;
      if (jb >= 0 && jb < nb) {
#pragma unroll 1
        for (int kk = 0; kk < BS; ++kk) {
          const int k = BS * jb + kk;
          if (k >= N) break;
          double F[S];
          ring_get<S>(base, PG::OFF_F, k % (PG::D_F * BS), c, F);
          if (k == 0) {
            double NE[S];
            ring_get<S>(base, PG::OFF_NE, 0, c, NE);
#pragma unroll
            for (int i = 0; i < S; ++i) Eb[i] = -NE[i];
#pragma unroll
            for (int i = 0; i < S; ++i) Eb[i] = (c == i) ? Eb[i] + 1.0 : Eb[i];
            transpose(H, F, tile, c);
#pragma unroll
            for (int i = 0; i < S; ++i) {  // lane S: Ebar column = z0, Fbar^T column = 0
              Eb[i] = (c == S) ? tile[S * kLdsRow + i] : Eb[i];
              H[i] = (c == S) ? 0.0 : H[i];
            }
          } else {
            double NW[S], Z[S];
            ring_get<S>(base, PG::OFF_NW, k % (PG::D_NW * BS), c, NW);
            copy(Z, H);
            gxy<C, true>(Z, NW, H);     // Z = W Fbar^T
            gxty<C, true>(Eb, H, Z);    // Ebar -= Fbar W Fbar^T
            zero(H);
            gxty<C, false>(H, F, Z);    // H' = F^T W Fbar^T
          }
          if (g == 0) {
            ring_put<S>(base, PG::OFF_EB, k % (PG::D_EB * BS), c, Eb);
            ring_put<S>(base, PG::OFF_H, k % (PG::D_H * BS), c, H);
          }
        }
        wave_sync();
      }
    } else {  // ---- wave 3: the queries of beat b - 3, one horizon per row
      const int jb = b - 3;
      if (jb >= 0 && jb < nb) {
        const int k = BS * jb + g % BS, kc = k < N ? k : N - 1;
        if constexpr (TRAJ) {
          // QT_aug[k] (horizon k + 1, e_{k+1}): P, its border P e, corner e^T P e + rho
          const TrajArgs<double>& t = a.tr;
          double pr[NN], ps[NN];
#pragma unroll
          for (int j = 0; j < NN; ++j) {
            pr[j] = in ? Pg[j * NN + cc] : 0.0;  // column c of P (the LFT kernel's image reads)
            ps[j] = Pg[j * NN + cc];
          }
          const double e1 = err(Xp[(long long)(kc + 1) * NN + cc]);
          double p4[4] = {0.0, 0.0, 0.0, 0.0};
          LaneDot4<NN>::fma(p4, e1, pr);
          const double pe = (p4[0] + p4[1]) + (p4[2] + p4[3]);
          const double epe = lane_sum<NN>(e1 * pe);
          if (in) {
#pragma unroll
            for (int i = 0; i < NN; ++i) imT[i * S + c] = ps[i];
            imT[c * S + NN] = pe;
            imT[NN * S + c] = pe;
            imT[c * S + c] = pdiag;
          } else if (c == NN) {
            imT[NN * S + NN] = (epe + t.rho_reg) + (1e-9 - 1.0);
          }
          wave_sync();
        } else {
          const double* qt = a.QT + (pk0 + kc) * SS;
          constexpr int NQ = (SS + 15) / 16;
          double vt[NQ];
#pragma unroll
          for (int u = 0; u < NQ; ++u) vt[u] = qt[c + 16 * u < SS ? c + 16 * u : SS - 1];
#pragma unroll
          for (int u = 0; u < NQ; ++u)
            if (c + 16 * u < SS) imT[c + 16 * u] = vt[u];
          wave_sync();
          diag_add<S, S>(imT, c, 1e-9 - 1.0);
        }
        double NX[S], Gq[S], Eq[S], Hq[S];
        neg_inverse<C, S, S>(NX, imT, c, mt, st);
        ring_get<S>(base, PG::OFF_GB, kc % (PG::D_GB * BS), c, Gq);
        ring_get<S>(base, PG::OFF_EB, kc % (PG::D_EB * BS), c, Eq);
        ring_get<S>(base, PG::OFF_H, kc % (PG::D_H * BS), c, Hq);
#pragma unroll
        for (int i = 0; i < S; ++i) NX[i] = Gq[i] - NX[i];   // QT^-1 + Gbar
        double X0[S];
        query_x0_ldl<C, S>(NX, Hq, Eq, X0, tile, c, mt, st);  // X0 = Ebar - Fbar Wt Fbar^T
        copy(NX, X0);
        const double jk = 0.5 * quad_inverse<C, S>(NX, tile, c, mt, st);
        if (k < N && g < BS) {
          if (!finite_val(jk)) st |= ST_NONFINITE;
          if (c == 0) a.J[p * N + k] = jk;
        }
        // the fused argmin, in horizon order (rows = consecutive horizons)
        if (a.t_max > 0) {
#pragma unroll
          for (int r = 0; r < BS; ++r) {
            const double jr = __shfl(jk, 16 * r);
            if (BS * jb + r < N) argmin_take(BS * jb + r + 1, jr, a.t_min, a.t_max, best, tbest);
          }
        }
        wave_sync();
      }
    }
#ifdef HOP_PIPE_STAMP
    const unsigned long long t_b1 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();  // one beat: every ring slot written this beat is read after it
#ifdef HOP_PIPE_STAMP
    t_busy += t_b1 - t_b0;
    t_wait += __builtin_amdgcn_s_memtime() - t_b1;
#endif
  }
#ifdef HOP_PIPE_STAMP
  if (lane == 0) {
    atomicAdd(&g_hop_stamp[w], t_busy);
    atomicAdd(&g_hop_stamp[4 + w], t_wait);
    if (w == 0)
      for (int j = 0; j < 3; ++j) atomicAdd(&g_hop_stamp[8 + j], t_sec[j]);
    atomicAdd(&g_hop_stamp[15], 1ull);
  }
#endif
  // status: the OR of every row's ladder bits (the chains' rows repeat row 0)
  unsigned* stw = reinterpret_cast<unsigned*>(base + PG::OFF_MISC + 64);
  const bool contrib = (w == 0 || w == 1) ? g == 0 : g < BS;
  if (c == 0 && contrib && st != 0u) atomicOr(stw, st);
  __syncthreads();
  if (tid == 0) a.status[p] = (int)*stw;
  if (w == 3 && lane == 0 && a.t_max > 0 && a.t_star != nullptr) {
    a.t_star[p] = tbest;
    a.j_star[p] = best;
  }
}

// The rerun launch after the s = 13 conditioned kernel (augmented blocks): the
// non-finite triage of every handed-over problem (as lft_v2_body's rerun mode), then
// the pipelined recompute of what is left (kPipeMax problems or fewer per workgroup)
// or, above that, the LFT body on every wave (a.cond as in lft_v2_body: bit 0 rerun,
// 4 developer reason bits, 8 triage only, 16 forced hand-over: no triage).
template <class C, int S, int MM, int BS>
__global__ __launch_bounds__(256, 1) void lft_rerun_pipe_kernel(LftArgs<double> a) {
  using PG = PipeGeo<S, MM, BS>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long wave_prob0 = ((long long)blockIdx.x * kWavesPerBlock + w) * kProbPerWave;
  const long long prob = wave_prob0 + g;
  const bool valid = prob < a.batch;
  const int st_in = valid ? a.status[prob] : 0;
  bool need = valid && (st_in & (int)ST_RERUN);
  if (!(a.cond & 16) && __any(need)) {  // the whole wave (lane-0 writes, shuffles)
    const bool resolved =
        nonfinite_resolve<S, MM, has_traj<C>()>(a, lane, g, wave_prob0, need, st_in);
    need = need && !resolved;
  }
  int* flags = reinterpret_cast<int*>(smem_raw + PG::OFF_MISC);
  if (c == 0) flags[w * 4 + g] = need ? 1 : 0;
  __syncthreads();
  if (a.cond & 8) return;  // triage only (HOP_OPT_NO_RERUN): the rest keep their hand-over word
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < kProbPerBlock; ++i) cnt += flags[i];
  if (cnt == 0) return;  // workgroup-uniform
  if (cnt > kPipeMax) {
    lft_v2_body<C, S, MM>(a, need ? 1 : 0);
    return;
  }
  int mine[kProbPerBlock];
#pragma unroll
  for (int i = 0; i < kProbPerBlock; ++i) mine[i] = flags[i];
  __syncthreads();  // the flags live in the misc area the pipeline reuses
#pragma unroll 1
  for (int i = 0; i < kProbPerBlock; ++i) {
    if (!mine[i]) continue;  // uniform
    pipe_problem<C, S, MM, BS>(a, (long long)blockIdx.x * kProbPerBlock + i);
    __syncthreads();
  }
}


// ===========================================================================
// SchedCond: the same J(t) by the conditioned prefix (z0 eliminated first).
//
// The LFT composition is associative.  The reference
// composes the stages 0..t-1 into (Ebar, Fbar, Gbar) and applies both
// boundaries, z0 and QT_t, at the query.  Folding z0 into the prefix first
// leaves the Schur complement of Ebar, a "vector" LFT element:
//   Sigma_t = Gbar - Fbar^T Ebar^-1 Fbar,  m_t = Fbar^T Ebar^-1 z0,
//   gamma_t = -z0^T Ebar^-1 z0,
// and J(t) = 1/2 z0^T (X0 + eps I)^-1 z0 (horizon_selection.py:77-85) becomes
//   J(t) = 1/2 (m_t^T (Sigma_t + X_t + eps I)^-1 m_t - gamma_t)     (Woodbury).
// Per stage (E_k = (Q_k + eps I)^-1, A_k, B_k):
//   Sigma_eps = Sigma + eps I          (the reference's jitter of W = (E_k + Gbar + eps I)^-1,
//                                       and at k = 0 the jitter of X0 + eps I)
//   S = Sigma_eps + E_k = L D L^T
//   Sigma' = Sigma_eps - Sigma_eps S^-1 Sigma_eps,  m' = m - Sigma_eps S^-1 m,
//   gamma' = gamma - m^T S^-1 m                    (CondLdl: one elimination + rank-1 streams)
//   Sigma_{k+1} = A_k Sigma' A_k^T + B_k R^-1 B_k^T,  m_{k+1} = A_k m'
// and the query of horizon k+1 is one bordered elimination of
// [Sigma_{k+1} + eps I + X_{k+1} | m_{k+1}] (ElimQ).  No W, Wt or X0 inverse and
// none of the compose's products: ~1,700 instead of ~3,000 VALU instructions
// per wave-step.  With the jitters placed as above the J curves agree with the
// reference to 1e-12 on well-conditioned inputs (tests/test_host_cpu.py model,
// tests/test_gpu_parity.py).
//
// Register state per problem (lane c = column c): X[0..S-1] = Sigma_eps with m
// on lane S, X[S] = gamma on lane S.  Lanes > S-1 of every image read (Q, QT,
// A, B) come from a zero area, so NE / NX are exactly zero there and lane S of
// Sigma is never disturbed by them.
//
// Anything unusual -- a first-attempt Cholesky failure of Q_k or QT_k (the
// reference's jitter ladder), a non-positive pivot of S or of the query, a
// non-finite J -- sets ST_RERUN, and the launch that follows (the SchedLdlDma
// kernel in rerun mode) recomputes exactly those problems with the reference's
// own association and every chol_inv ladder, so status bits and the failure
// semantics stay the reference's.
// ===========================================================================
template <class C, int S>
__device__ __forceinline__ void sym_from_z(const double* img, unsigned zaddr, int c,
                                           double (&r)[S]) {
  const bool in = c < S;
  const unsigned bc = in ? lds_addr(img) + 8u * c : zaddr;
  const unsigned br = in ? lds_addr(img) + 8u * S * c : zaddr;
  double t[S];
  LdsSym<S, S>::run(bc, br, r, t);
#pragma unroll
  for (int i = 0; i < S; ++i) r[i] = has_sym2<C>() ? r[i] + t[i] : 0.5 * (r[i] + t[i]);
}

// Trajectory form of the conditioned-prefix kernel (SchedCondTraj): the
// augmented Q / QT images are built in LDS from the raw linearisation exactly
// as in lft_sweep_v2_kernel's TRAJ path (augmented.py:10-87): constant parts
// once, per step only the last row / column and the diagonal, Q e_k carried.
template <int S, int MM>
struct CondTraj {
  static constexpr int NN = S - 1;
  double xg_c = 0.0, ur_c = 0.0, w2 = 0.0, qdiag = 0.0, pdiag = 0.0, pcc = 0.0;
  double qe_k = 0.0, eqe_k = 0.0;
  bool wrap_c = false;
  double qr_n[NN], pr_n[NN];

  __device__ __forceinline__ void load_rows(const double* cq, const double* imT, int c) {
    const int cc = c < NN ? c : 0;
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      qr_n[j] = cq[j * NN + cc];
      pr_n[j] = imT[j * S + cc];
    }
  }

  __device__ __forceinline__ void init(const LftArgs<double>& a, long long pb, int c, double* cq,
                                       double* wq, double* wt) {
    const TrajArgs<double>& t = a.tr;
    const double* Qg = t.Q + pb * t.q_bs;
    const double* Pg = t.P + pb * t.p_bs;
    const int cc = c < NN ? c : 0;
    if (c < NN) {  // raw Q (Q e, augmented.py:35), transposed
#pragma unroll
      for (int j = 0; j < NN; ++j) cq[j * NN + c] = Qg[c * NN + j];
    }
    pcc = Pg[cc * NN + cc];
    xg_c = c < NN ? t.xg[pb * t.xg_bs + cc] : 0.0;
    ur_c = c < MM ? t.u_ref[pb * t.ur_bs + (c < MM ? c : 0)] : 0.0;
    w2 = 2.0 * t.w[pb * t.w_bs];
    wrap_c = c < NN && ((t.wrap_mask >> c) & 1u);
    qdiag = (0.5 * (Qg[cc * NN + cc] + Qg[cc * NN + cc]) + t.q_reg) + (1e-9 - 1.0);
    pdiag = Pg[cc * NN + cc] + (1e-9 - 1.0);
    {
      const double* X0 = t.X + pb * (long long)(a.nalloc + 1) * NN;
      double e0 = c < NN ? X0[cc] - xg_c : 0.0;
      if (t.wrap_mask != 0u) {
        const double w0 = wrap_angle(e0);
        e0 = wrap_c ? w0 : e0;
      }
      double q4[4] = {0.0, 0.0, 0.0, 0.0};
      double qr0[NN];
#pragma unroll
      for (int j = 0; j < NN; ++j) qr0[j] = c < NN ? Qg[cc * NN + j] : 0.0;
      LaneDot4<NN>::fma(q4, e0, qr0);
      qe_k = (q4[0] + q4[1]) + (q4[2] + q4[3]);
      eqe_k = lane_sum<NN>(e0 * qe_k);
    }
    if (c < NN) {  // column c: _sym(Q) + q_reg I, and P (augmented.py:33, 82)
#pragma unroll
      for (int i = 0; i < NN; ++i) {
        wq[i * S + c] = 0.5 * (Qg[i * NN + c] + Qg[c * NN + i]) + (i == c ? t.q_reg : 0.0);
        wt[i * S + c] = Pg[i * NN + c];
      }
    }
  }

  // last row / column and diagonal of Q_aug[k], QT_aug[k]; returns a~_k[c]
  __device__ __forceinline__ double step(const LftArgs<double>& a, int c, const double* sX,
                                         const double* sV, const double* sU, const double* sR,
                                         double* wq, double* wt) {
    const int cc = c < NN ? c : 0, cm = c < MM ? c : 0;
    double x1 = sX[cc], av = sV[cc], uu = sU[cm];
    double rb[MM], qr[NN], pr[NN];
#pragma unroll
    for (int q = 0; q < MM; ++q) rb[q] = sR[cc * MM + q];
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      qr[j] = qr_n[j];
      pr[j] = pr_n[j];
    }
    const bool in = c < NN;
#pragma unroll
    for (int j = 0; j < NN; ++j) {
      qr[j] = in ? qr[j] : 0.0;
      pr[j] = in ? (j == c ? pcc : pr[j]) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < MM; ++q) rb[q] = in ? rb[q] : 0.0;
    double e1 = in ? x1 - xg_c : 0.0;
    if (a.tr.wrap_mask != 0u) {
      const double we1 = wrap_angle(e1);
      e1 = wrap_c ? we1 : e1;
    }
    const double du = c < MM ? uu - ur_c : 0.0;
    av = in ? av : 0.0;
    double q4[4] = {0.0, 0.0, 0.0, 0.0}, p4[4] = {0.0, 0.0, 0.0, 0.0}, bd = 0.0;
    LaneDot4<NN>::fma(q4, e1, qr);
    LaneDot4<NN>::fma(p4, e1, pr);
    LaneDot<MM>::fma(bd, du, rb);
    const double qe1 = (q4[0] + q4[1]) + (q4[2] + q4[3]);
    const double pe = (p4[0] + p4[1]) + (p4[2] + p4[3]);
    const double atil = av - bd;
    const double eqe1 = lane_sum<NN>(e1 * qe1);
    const double epe = lane_sum<NN>(e1 * pe);
    if (c < NN) {
      wq[c * S + NN] = qe_k;
      wq[NN * S + c] = qe_k;
      wq[c * S + c] = qdiag;
      wt[c * S + NN] = pe;
      wt[NN * S + c] = pe;
      wt[c * S + c] = pdiag;
    } else if (c == NN) {
      wq[NN * S + NN] = ((eqe_k + w2) + a.tr.rho_reg) + (1e-9 - 1.0);
      wt[NN * S + NN] = (epe + a.tr.rho_reg) + (1e-9 - 1.0);
    }
    qe_k = qe1;
    eqe_k = eqe1;
    return atil;
  }
};

// T = float: fp32 blocks in HBM / LDS (half the bytes), converted on the LDS
// reads; the arithmetic stays fp64 (fp32 DPP FMAs issue no faster at one wave
// per SIMD) and J / J* are rounded to fp32 on the store.
template <class C, int S, int MM, class T = double>
__global__ __launch_bounds__(256, has_pack<C>() ? 2 : 1) void lft_cond_kernel(LftArgs<T> a) {
  constexpr int ES = (int)sizeof(T);
  constexpr bool F32 = ES == 4;
  using G = Geo<S, MM, ES, has_pack<C>(), has_smalls<C>()>;
  static_assert(!has_pack<C>() || (!F32 && !has_traj<C>() && G::NJM == 6 && G::NJB == 2 &&
                                   2 * kWavesPerBlock * G::WAVE_BYTES <= 160 * 1024),
                "packed images: s = 13 fp64 blocks, two workgroups per CU");
  constexpr bool TRAJ = has_traj<C>();
  static_assert(!F32 || (!TRAJ && dstag<C>() == 0 && !has_sym2<C>() && !has_peps<C>()),
                "fp32 blocks: augmented form, halved sums");
  constexpr int NN = G::NN;
  static_assert(S < kRowLanes, "m rides on lane S");
  static_assert(G::TILE_W >= 8 * S * S + 64, "zero area in the tile slot");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int WB = TRAJ ? G::WAVE_BYTES_T : G::WAVE_BYTES;
  unsigned char* wbase = smem_raw + w * WB;
  const unsigned wlds = (unsigned)(uintptr_t)wbase;
  double* zarea = reinterpret_cast<double*>(wbase + G::OFF_T);
  const unsigned zaddr = wlds + G::OFF_T;
  constexpr bool MF = has_mfma<C>();
  static_assert(!MF || (F32 && S == 13 && MM == 4), "MFMA predict: fp32 blocks, s = 13");
  // MFMA: the zero area grows to 2,880 B (a zero and a 1.0f for every problem's
  // image offset p * IMGM, p < 4) and the f32 staging region follows it
  // MF64 (HOP_COND_MFMA64, A/B): the fp64 predict's two products on v_mfma_f64_16x16x4_f64,
  // one problem per 16 x 16 tile; [Sigma' | m'] staged through the Q image and the result
  // through the QT image (both read by then), so the step's DMA moves after the predict.
  // Zero area: zeros at every p * 1360 (image offsets) and p * 1472 (staging offsets),
  // a 1.0 at 1416 + p * 1360 (A~'s (13, 13), the m' pass-through), p < 4.
  constexpr bool MF64 = kCondMfma64 && has_symlate<C>() && has_sym2<C>() && !has_newt<C>() &&
                        !has_peps<C>() && !TRAJ && !F32 && !has_pack<C>() && S == 13 && MM == 4 &&
                        dstag<C>() == 0;
  constexpr int M6XP = 1472, M6ONE = 1416;  // staging stride per problem, 1.0 offset (bytes)
  static_assert(!MF64 || (G::IMGM == 1360 && M6ONE + 3 * G::IMGM + 8 <= G::TILE_W &&
                          4 * M6XP <= G::IMGM_W && 8 * (S * S + 8) <= M6ONE),
                "fp64 MFMA staging: Q / QT image areas, ones past the sym zero area");
  constexpr int ZB = MF ? 2880 : (MF64 ? 3 * M6XP + 8 : 8 * (S * S + 8));
  constexpr int MFB = 2880, MFP = 1152;  // staging region offset, bytes per problem
  static_assert(!MF || (MFB + 4 * MFP <= G::TILE_W && 800 + 3 * G::IMGM + 4 <= ZB &&
                        G::IMGM == 688),
                "MFMA staging in the tile slot");
#pragma unroll 1
  for (int i = lane; i < ZB / 8; i += 64) zarea[i] = 0.0;
  if constexpr (MF64) {
    if (lane < 4) zarea[(M6ONE + lane * G::IMGM) / 8] = 1.0;
  }
  if constexpr (MF) {
    float* mz = reinterpret_cast<float*>(wbase + G::OFF_T + MFB);
#pragma unroll 1
    for (int i = lane; i < 4 * MFP / 4; i += 64) mz[i] = 0.0f;
    // A~[13][13] = 1 (the row carrying m'): one 1.0f per problem image offset, at a
    // float index no other zero-area read uses (13 i and i, i < 13)
    if (lane < 4) reinterpret_cast<float*>(zarea)[200 + lane * (G::IMGM / 4)] = 1.0f;
  }
  // SYM2: eps I rows for the predict, read as element 15 + I - c of a zero-padded
  // vector holding eps at element 15 (after the zero area)
  constexpr int EPSV = 192;  // doubles from the zero area's start
  static_assert(!has_peps<C>() || G::TILE_W >= 8 * (EPSV + 32), "eps vector in the tile slot");
  if constexpr (has_peps<C>()) {
    if (lane < 32) zarea[EPSV + lane] = lane == 15 ? 1e-9 : 0.0;
  }
  const unsigned eps_addr = zaddr + 8u * (EPSV + 15 - c);
  constexpr double DOFF = has_sym2<C>() ? 1e-9 - 0.5 : 1e-9 - 1.0;  // image diagonal offset
  constexpr double KOFF = has_sym2<C>() ? 2.0 : 1.0;  // update / query diagonal offset
  // the congruence query (has_wq): the ldspipe schedules on augmented images only
  constexpr bool WQ = has_wq<C>() && (has_ldspipe<C>() || has_smalls<C>()) && !TRAJ && !MF;
  const double kmask = c < S - 1 ? -KOFF : 0.0;     // P11^-1 - KOFF I on lanes < S-1
  const double e_last = c == S - 1 ? 1.0 : 0.0;
  const T* imQ = reinterpret_cast<const T*>(wbase + G::OFF_Q + g * G::IMGM);
  const T* imA = reinterpret_cast<const T*>(wbase + G::OFF_A + g * G::IMGM);
  const T* imT = reinterpret_cast<const T*>(wbase + G::OFF_QT + g * G::IMGM);
  const T* imB = reinterpret_cast<const T*>(wbase + G::OFF_B + g * G::IMGB);
  const T* zareaT = reinterpret_cast<const T*>(zarea);

  const long long wave_prob0 = ((long long)blockIdx.x * kWavesPerBlock + w) * kProbPerWave;
  const long long prob = wave_prob0 + g;
  const bool valid = prob < a.batch;
  const long long pb0 = wave_prob0 < a.batch ? wave_prob0 : a.batch - 1;
  const int N = a.n;
  constexpr int SS = S * S, SM = S * MM;
  const long long pstrM = (long long)a.nalloc * SS * ES;
  const long long pstrB = (long long)a.nalloc * SM * ES;
  auto mk = [&](const T* base, long long pstr) {
    const long long left = (a.batch - pb0) * pstr;
    const unsigned nrec = left > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (unsigned)left;
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(base) + pb0 * (pstr / ES), (short)0, (int)nrec, 0x00020000);
  };
  const long long pstA = (long long)a.nalloc * NN * NN * 8, pstR = (long long)a.nalloc * NN * MM * 8;
  const long long pstX = (long long)(a.nalloc + 1) * NN * 8, pstV = (long long)a.nalloc * NN * 8;
  const long long pstU = (long long)a.nalloc * MM * 8;
  const __amdgpu_buffer_rsrc_t rQ = TRAJ ? mk(a.tr.A, pstA) : mk(a.Q, pstrM),
                               rA = TRAJ ? mk(a.tr.Bm, pstR) : mk(a.A, pstrM),
                               rT = TRAJ ? mk(a.tr.X, pstX) : mk(a.QT, pstrM),
                               rB = TRAJ ? mk(a.tr.ares, pstV) : mk(a.B, pstrB),
                               rU = TRAJ ? mk(a.tr.U, pstU) : rB;
  unsigned voM[G::NJM], voB[G::NJB];
  unsigned voTA[G::NJA], voTR[G::NJR], voTX[G::NJX], voTV[G::NJV], voTU[G::NJU];
  if constexpr (TRAJ) {
    static_assert(G::NJA == 5 && G::NJR == 2 && G::NJX == 1 && G::NJV == 1 && G::NJU == 1,
                  "trajectory pieces of the s = 13, m = 4 shape");
#pragma unroll
    for (int j = 0; j < G::NJA; ++j)
      voTA[j] = chunk_voff<G::CHA>(j, lane, wave_prob0, pb0, a.batch, pstA);
#pragma unroll
    for (int j = 0; j < G::NJR; ++j)
      voTR[j] = chunk_voff<G::CHR>(j, lane, wave_prob0, pb0, a.batch, pstR);
    voTX[0] = chunk_voff<G::CHX>(0, lane, wave_prob0, pb0, a.batch, pstX);
    voTV[0] = chunk_voff<G::CHV>(0, lane, wave_prob0, pb0, a.batch, pstV);
    voTU[0] = chunk_voff<G::CHU>(0, lane, wave_prob0, pb0, a.batch, pstU);
  } else {
#pragma unroll
    for (int j = 0; j < G::NJM; ++j)
      voM[j] = chunk_voff<G::CHM>(j, lane, wave_prob0, pb0, a.batch, pstrM);
#pragma unroll
    for (int j = 0; j < G::NJB; ++j)
      voB[j] = chunk_voff<G::CHB>(j, lane, wave_prob0, pb0, a.batch, pstrB);
  }
  // dma_step20 / dma_traj10 take the voffsets lowered by their pieces' instruction offsets
  unsigned voMl[G::NJM], voBl[G::NJB], voTAl[G::NJA], voTRl[G::NJR];
#pragma unroll
  for (int j = 0; j < G::NJM; ++j) voMl[j] = TRAJ ? 0u : dma_voff_lowered(voM[j], j);
#pragma unroll
  for (int j = 0; j < G::NJB; ++j) voBl[j] = TRAJ ? 0u : dma_voff_lowered(voB[j], j);
#pragma unroll
  for (int j = 0; j < G::NJA; ++j) voTAl[j] = TRAJ ? dma_voff_lowered(voTA[j], j) : 0u;
#pragma unroll
  for (int j = 0; j < G::NJR; ++j) voTRl[j] = TRAJ ? dma_voff_lowered(voTR[j], j) : 0u;
  auto dma_step = [&](int k) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (TRAJ) {  // A_k, B_k, x_{k+1}, a_k, u_k
      const unsigned soA = (unsigned)(k * NN * NN * 8), soR = (unsigned)(k * NN * MM * 8),
                     soV = (unsigned)(k * NN * 8), soU = (unsigned)(k * MM * 8);
      dma_traj10<G::OFF_A, G::OFF_B, G::OFF_VX, G::OFF_VA, G::OFF_VU>(
          voTAl, voTRl, voTX[0], voTV[0], voTU[0], rQ, rA, rT, rB, rU, wlds, soA, soR,
          soV + NN * 8, soV, soU);
    } else if constexpr (G::NJM == 6 && G::NJB == 2) {
      const unsigned soM = (unsigned)(k * SS * ES), soB = (unsigned)(k * SM * ES);
      if constexpr (has_pack<C>())
        dma_step20p<G::OFF_Q, G::OFF_A, G::OFF_B, G::OFF_QT, G::LASTM, G::LASTB>(
            voM, voB, rQ, rA, rB, rT, wlds, soM, soB);
      else
        dma_step20<G::OFF_Q, G::OFF_A, G::OFF_B, G::OFF_QT>(voMl, voBl, rQ, rA, rB, rT, wlds,
                                                           soM, soB);
    } else {
      const unsigned soM = (unsigned)(k * SS * ES), soB = (unsigned)(k * SM * ES);
#pragma unroll
      for (int j = 0; j < G::NJM; ++j) dma16(voM[j], rQ, wlds + G::OFF_Q + 1024 * j, soM);
#pragma unroll
      for (int j = 0; j < G::NJM; ++j) dma16(voM[j], rA, wlds + G::OFF_A + 1024 * j, soM);
#pragma unroll
      for (int j = 0; j < G::NJB; ++j) dma16(voB[j], rB, wlds + G::OFF_B + 1024 * j, soB);
#pragma unroll
      for (int j = 0; j < G::NJM; ++j) dma16(voM[j], rT, wlds + G::OFF_QT + 1024 * j, soM);
    }
  };

  const long long pb = valid ? prob : a.batch - 1;
  double rinv[MM];
  {
    const T* Rp = a.R + pb * a.r_bstride;
#pragma unroll
    for (int i = 0; i < MM; ++i)
      rinv[i] = (c < MM) ? (double)Rp[i * MM + (c < MM ? c : 0)] : 0.0;
  }
  double* cq = reinterpret_cast<double*>(wbase + G::OFF_CQ) + g * NN * NN;
  CondTraj<S, MM> tb;
  if constexpr (TRAJ && !F32) {
    tb.init(a, pb, c, cq, const_cast<double*>(imQ), const_cast<double*>(imT));
    wave_sync();
    tb.load_rows(cq, imT, c);
  }
  // X = [Sigma_0 + eps I | z0], gamma_0 = 0 (Sigma_0 = 0: z0 known exactly);
  // the trajectory form's z0 is e_s (augmented.py:57)
  const T* zp = a.z0 + pb * a.z_bstride;
  double X[S + 1];
  static_for<S>([&](auto I) {
    const double z = TRAJ ? (I == NN ? 1.0 : 0.0) : (double)zp[I];
    X[I] = (c == S) ? z : sel_lane<I>(0.0, 1e-9);
  });
  X[S] = 0.0;
  const double e_s = (c == S) ? 1.0 : 0.0;  // row S of A~^T: carries m through the first product
  bool bad = (a.cond & 2) != 0;
  // the first flagged horizon + 1 (0: none; 1: the prologue or a forced hand-over),
  // left in status bits 13.. for the rerun launch's non-finite triage
  int kf1 = bad ? 1 : 0;
  // developer builds: first failing test and horizon (see lft_cond_cf_kernel); stored
  // at HOP_HANDOVER_REASON_SHIFT, which puts the horizon where the hand-over word has it
  static_assert(HOP_HANDOVER_REASON_SHIFT + 8 == HOP_HANDOVER_SHIFT, "why = reason | t << 8");
  static_assert(ST_RERUN == HOP_ST_HANDOVER, "the hand-over bit");
  int why = 0;
  auto flag = [&](bool f, int bit, int t) {
    if constexpr (kDevBuild) why = (f && why == 0) ? (bit | (t << 8)) : why;
  };
  unsigned long long sec[8] = {};
  unsigned long long tprev = 0;
  auto stamp = [&](int j) {
    if constexpr (C::STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (j >= 0) sec[j] += t - tprev;
      tprev = t;
    }
  };

  // MFMA operand addresses (loop-invariant; problem p at an immediate offset):
  //   X staged as [p][row][17] f32 (row i of [Sigma' | m'] written by lane c = column);
  //   prod 1 (T = X A~^T) k-slice kk: lane (g, c) carries k = 4 g + kk, A operand
  //   X[c][k], B operand A~[c][k] (the A image; (13, 13): 1; else the zero area);
  //   prod 2 (A T): A operand A[c][4 g + kk], B operand = register kk of T's
  //   accumulator (row 4 g + kk, column c): the same k, no lane movement;
  //   the result (row 4 g + r, column c) goes back as [p][column][18] f32.
  unsigned mx_w = 0, mx_a = 0, ma_b[4] = {}, ma_a[4] = {}, ms_w = 0, ms_r = 0;
  const unsigned lds0 = (unsigned)(uintptr_t)smem_raw;
  auto lds_ptr = [&](unsigned ad) { return smem_raw + (ad - lds0); };
  if constexpr (MF) {
    const unsigned mfb = zaddr + MFB;
    mx_w = mfb + g * MFP + 4u * c;
    mx_a = mfb + 4u * (17 * c + 4 * g);
    ms_w = mfb + 4u * (18 * c + 4 * g);
    ms_r = mfb + g * MFP + 4u * 18 * c;
    const unsigned ia = lds_addr(imA) - (unsigned)(g * G::IMGM);  // problem 0's image
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kx = 4 * g + kk;
      const bool in = c < S && kx < S;
      ma_b[kk] = in ? ia + 4u * (S * c + kx) : (c == S && kx == S ? zaddr + 800u : zaddr);
      ma_a[kk] = in ? ia + 4u * (S * c + kx) : zaddr;
    }
  }

  // MF64 operand addresses (problem p at an immediate offset: p * M6XP in the staging,
  // p * IMGM in the A image; invalid lanes read the zero area at the same offsets):
  //   f64 MFMA C/D map (cdna_hip_programming.md): lane (g, c) holds row g + 4 r, column c
  //   of register r; A / B as the f32 16x16x4 form (A[c][k], B[k][c], k = lane group).
  //   product 1 (T = [Sigma' | m'] A~^T), slice kk: lane (g, c) carries k = 4 g + kk:
  //     A operand X[c][k] (staged [p][row][14]), B operand A~^T[k][c] = A[c][k] (+ the 1.0);
  //   product 2 (A T), slice kk: k = g + 4 kk, so the B operand is register kk of T's
  //     accumulator (row g + 4 kk, column c) and the A operand A[c][g + 4 kk];
  //   the result (row g + 4 r, column c) goes to the QT image as [p][column][13].
  unsigned m6_xw = 0, m6_xa[4] = {}, m6_aa[4] = {}, m6_ab[4] = {}, m6_dw = 0, m6_xr = 0;
  if constexpr (MF64) {
    const unsigned qb = lds_addr(imQ) - (unsigned)(g * G::IMGM);  // the wave's Q image area
    const unsigned tb = lds_addr(imT) - (unsigned)(g * G::IMGM);
    const unsigned ab = lds_addr(imA) - (unsigned)(g * G::IMGM);
    m6_xw = qb + (unsigned)(g * M6XP) + 8u * c;
    m6_dw = tb + 8u * (S * c + g);
    m6_xr = c < S + 1 ? tb + (unsigned)(g * M6XP) + 8u * S * c : zaddr;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kx = 4 * g + kk;
      m6_xa[kk] = (c < S && kx < S + 1) ? qb + 8u * ((S + 1) * c + kx) : zaddr;
      const bool in = c < S && kx < S;
      m6_ab[kk] = in ? ab + 8u * (S * c + kx) : (c == S && kx == S ? zaddr + M6ONE : zaddr);
      const int k2 = g + 4 * kk;  // product 2's k (the accumulator's row map)
      m6_aa[kk] = (c < S && k2 < S) ? ab + 8u * (S * c + k2) : zaddr;
    }
  }

  dma_step(0);
  double best = 0.0, jprev = 0.0;
  int tbest = 0;
  const bool fuse_argmin = a.t_max > 0;
  // QPIPE (small-s row groups): the query of horizon k + 1 runs in step k + 1, its
  // ElimQ interleaved with that step's two sweeps (SweepQ2ElimQ): at s <= 5 each of
  // them is a chain of short pivot blocks.  Same operations on the same values (the
  // query reads Sigma before the next step's symmetrisation and update, as before), so
  // J and T* are bitwise the in-step query's; flags keep their horizons.
  constexpr bool QPIPE = WQ && has_smalls<C>() && kSmallSweep2 && kSmallQPipe;
  double NXp[S];  // the terminal block's sweep of the pending query
#pragma unroll
  for (int i = 0; i < S; ++i) NXp[i] = 0.0;
  // the query's congruence prelude (see the in-step query below) and its tail
  auto query_prelude = [&](const double (&nx)[S], double (&rq)[S], double& gam, int kq) {
    const double ub = c < S - 1 ? nx[S - 1] : 0.0;
    const double sg = (bcast<S - 1>(nx[S - 1]) + 1.0) * (1.0 / KOFF);
    bad = bad || !(sg > 0.0);
    flag(!(sg > 0.0), 1, kq + 1);
#pragma unroll
    for (int i = 0; i < S - 1; ++i) rq[i] = __builtin_fma(kmask, nx[i], X[i]);
    rq[S - 1] = X[S - 1];
    RowB<S>::template sweep<S - 1>(rq, ub);
    LaneB<S - 1>::fma(reinterpret_cast<double (&)[S - 1]>(rq), ub, rq[S - 1]);
    rq[S - 1] = __builtin_fma(e_last, recip_nr(sg) - KOFF, rq[S - 1]);
    gam = bcast<S>(X[S]);
  };
  auto query_tail = [&](double acc, double dmin, double gam, int kq) {
    const double q = bcast<S>(acc);
    bad = bad || !(dmin > 0.0) || (q != q);
    flag(!(dmin > 0.0) || (q != q), 16, kq + 1);
    const double jk = 0.5 * (q - gam);
    bad = bad || !finite_val(jk);
    flag(!finite_val(jk), 32, kq + 1);
    kf1 = (bad && kf1 == 0) ? kq + 2 : kf1;
    if (valid && c == 0) a.J[prob * N + kq] = (T)jk;
    if (fuse_argmin) {
      const int t = kq + 1;
      if (t == a.t_min) {
        best = jk;
        tbest = t;
      } else if (t > a.t_min && t <= a.t_max) {
        const bool bnan = best != best, jnan = jk != jk;
        if (!bnan && (jnan || jk < best)) {
          best = jk;
          tbest = t;
        }
      }
    }
  };
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    stamp(-1);
    dma_wait();
    wave_sync();
    stamp(0);
    if (!QPIPE && k > 0 && valid && c == 0) a.J[prob * N + k - 1] = (T)jprev;
    double atil = 0.0;
    if constexpr (F32) {
    } else if constexpr (TRAJ) {
      const double* sX = reinterpret_cast<const double*>(wbase + G::OFF_VX) + g * 2 * G::CHX;
      const double* sV = reinterpret_cast<const double*>(wbase + G::OFF_VA) + g * 2 * G::CHV;
      const double* sU = reinterpret_cast<const double*>(wbase + G::OFF_VU) + g * 2 * G::CHU;
      const double* sR = reinterpret_cast<const double*>(wbase + G::OFF_B) + g * 2 * G::CHR;
      atil = tb.step(a, c, sX, sV, sU, sR, const_cast<double*>(imQ), const_cast<double*>(imT));
    } else {
      diag_add<S, S>(imQ, c, DOFF);
      diag_add<S, S>(imT, c, DOFF);
    }
    // ---- NE = -(Q_k + eps I)^-1 + I, NX = -(QT_k + eps I)^-1 + I (first attempt only)
    double NE[S], NX[S];
    double at[S + 1], brow[MM];  // at[j] = column j of A~ (lanes > S-1: 0), at[S] = e_S
    double ar[has_arow<C>() ? S : 1];  // AROW: rows of A_k, read before the image is refilled
    float mb[MF ? 4 : 1][4], ma[MF ? 4 : 1][4];  // MFMA predict operands (likewise)
    stamp(1);
    if constexpr (has_ldspipe<C>() && !TRAJ && F32) {
      // fp32 images: Q's converting reads, then QT's 4-byte reads under the E sweep
      // and A_k / B_k's under the X sweep, converted after (the offset form in fp64)
      const bool in = c < S;
      const T* qc = in ? imQ + c : zareaT;
      const T* qr = in ? imQ + S * c : zareaT;
#pragma unroll
      for (int i = 0; i < S; ++i) NE[i] = 0.5 * ((double)qc[S * i] + (double)qr[i]);
      static_for<S>([&](auto I) { NE[I] += sel_lane<I>(0.0, 1e-9 - 1.0); });
      stamp(2);
      float o[2 * S];
      const unsigned aq[2] = {in ? lds_addr(imT) + 4u * c : zaddr,
                              in ? lds_addr(imT) + 4u * S * c : zaddr};
      double d1 = 1.0, d2 = 1.0;
      SweepQSymF<S>::run(NE, d1, o, aq);
#pragma unroll
      for (int i = 0; i < S; ++i) NX[i] = 0.5 * ((double)o[i] + (double)o[S + i]);
      static_for<S>([&](auto I) { NX[I] += sel_lane<I>(0.0, 1e-9 - 1.0); });
      float o2[2 * S + MM];
      const unsigned ab[3] = {in ? lds_addr(imA) + 4u * S * c : zaddr, lds_addr(imA) + 4u * c,
                              in ? lds_addr(imB) + 4u * MM * c : zaddr};
      if constexpr (WQ) SweepQABFP<S>::run(NX, d2, o2, ab);  // pivots 0 .. S-2 (the query)
      else SweepQABF<S>::run(NX, d2, o2, ab);
      bad = bad || !pivots_ok(NE, d1) || !pivots_ok(NX, d2);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        at[j] = (double)o2[j];
        if constexpr (has_arow<C>()) ar[j] = (double)o2[S + j];
      }
#pragma unroll
      for (int q = 0; q < MM; ++q) brow[q] = (double)o2[2 * S + q];
      stamp(3);
    } else if constexpr (has_ldspipe<C>() && !TRAJ && kCondSweep2 && WQ && has_sym2<C>() &&
                         S == 13 && MM == 4 && dstag<C>() == 0) {
      // Q's and QT's symmetric sums behind one LDS round trip, then the two independent
      // sweeps as one interleaved block (each sweep's pivot chains hide behind the
      // other's FMAs) with A_k's / B_k's reads underneath
      const bool in = c < S;
      const unsigned iq = lds_addr(imQ), it = lds_addr(imT);
      const unsigned a4[4] = {in ? iq + 8u * c : zaddr, in ? iq + 8u * S * c : zaddr,
                              in ? it + 8u * c : zaddr, in ? it + 8u * S * c : zaddr};
      double qq[4 * S];
      LdsSym2<S, S>::run(a4, qq);
#pragma unroll
      for (int i = 0; i < S; ++i) {
        NE[i] = qq[i] + qq[S + i];
        NX[i] = qq[2 * S + i] + qq[3 * S + i];
      }
      stamp(2);
      double d1 = 1.0, d2 = 1.0;
      double o2[2 * S + MM];
      const unsigned ab[3] = {in ? lds_addr(imA) + 8u * S * c : zaddr, lds_addr(imA) + 8u * c,
                              in ? lds_addr(imB) + 8u * MM * c : zaddr};
      SweepQ2AB<S>::run(NE, d1, NX, d2, o2, ab);  // X: pivots 0 .. S-2 (the congruence query)
      bad = bad || !pivots_ok(NE, d1) || !pivots_ok(NX, d2);
      flag(!pivots_ok(NE, d1) || !pivots_ok(NX, d2), 1, k + 1);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        at[j] = o2[j];
        if constexpr (has_arow<C>()) ar[j] = o2[S + j];
      }
#pragma unroll
      for (int q = 0; q < MM; ++q) brow[q] = o2[2 * S + q];
      stamp(3);
    } else if constexpr (has_ldspipe<C>() && !TRAJ) {
      // QT's sym reads ride under the E sweep, A_k / B_k's under the X sweep
      sym_from_z<C, S>(imQ, zaddr, c, NE);
      stamp(2);
      const bool in = c < S;
      double o[2 * S];
      const unsigned aq[2] = {in ? lds_addr(imT) + 8u * c : zaddr,
                              in ? lds_addr(imT) + 8u * S * c : zaddr};
      double d1 = 1.0, d2 = 1.0;
      SweepQSym<S>::run(NE, d1, o, aq);
      if constexpr (dstag<C>() == 2) {  // the Q and QT images are read: refill them now
        wave_sync();
        if (k + 1 < N)
          dma_stepQT<G::OFF_Q, G::OFF_QT>(voM, rQ, rT, wlds, (unsigned)((k + 1) * SS * ES));
      }
#pragma unroll
      for (int i = 0; i < S; ++i) NX[i] = has_sym2<C>() ? o[i] + o[S + i] : 0.5 * (o[i] + o[S + i]);
      double o2[2 * S + MM];
      const unsigned ab[3] = {in ? lds_addr(imA) + 8u * S * c : zaddr, lds_addr(imA) + 8u * c,
                              in ? lds_addr(imB) + 8u * MM * c : zaddr};
      if constexpr (WQ) SweepQABP<S>::run(NX, d2, o2, ab);  // pivots 0 .. S-2 (the query)
      else SweepQAB<S>::run(NX, d2, o2, ab);
      bad = bad || !pivots_ok(NE, d1) || !pivots_ok(NX, d2);
      flag(!pivots_ok(NE, d1) || !pivots_ok(NX, d2), 1, k + 1);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        at[j] = o2[j];
        if constexpr (has_arow<C>()) ar[j] = o2[S + j];
      }
#pragma unroll
      for (int q = 0; q < MM; ++q) brow[q] = o2[2 * S + q];
      stamp(3);
    } else {
    if constexpr (F32) {  // fp32 images: converting reads, offset form applied in fp64
      const bool in = c < S;
      const T* qc = in ? imQ + c : zareaT;
      const T* qr = in ? imQ + S * c : zareaT;
      const T* tc = in ? imT + c : zareaT;
      const T* tr = in ? imT + S * c : zareaT;
#pragma unroll
      for (int i = 0; i < S; ++i) {
        NE[i] = 0.5 * ((double)qc[S * i] + (double)qr[i]);
        NX[i] = 0.5 * ((double)tc[S * i] + (double)tr[i]);
      }
      static_for<S>([&](auto I) {
        NE[I] += sel_lane<I>(0.0, 1e-9 - 1.0);
        NX[I] += sel_lane<I>(0.0, 1e-9 - 1.0);
      });
    } else {
      sym_from_z<C, S>(imQ, zaddr, c, NE);
      sym_from_z<C, S>(imT, zaddr, c, NX);
    }
    stamp(2);
    {
      double d1 = 1.0, d2 = 1.0;
      if constexpr (QPIPE) {
        if (k > 0) {  // step k - 1's query under this step's sweeps
          double rq[S], gam, accq = 0.0, dminq = 1.0;
          query_prelude(NXp, rq, gam, k - 1);
          SweepQ2ElimQ<S>::run(NE, d1, NX, d2, rq, accq, dminq, KOFF);
          query_tail(accq, dminq, gam, k - 1);
        } else {
          SweepQ2<S>::run(NE, d1, NX, d2);
        }
      } else if constexpr (WQ && has_smalls<C>() && kSmallSweep2) {
        SweepQ2<S>::run(NE, d1, NX, d2);  // both sweeps, pivot blocks interleaved
      } else {
        SweepQ<S>::run(NE, d1);
        if constexpr (WQ) SweepQP<S>::run(NX, d2);  // pivots 0 .. S-2 (the congruence query)
        else SweepQ<S>::run(NX, d2);
      }
      bad = bad || !pivots_ok(NE, d1) || !pivots_ok(NX, d2);
      flag(!pivots_ok(NE, d1) || !pivots_ok(NX, d2), 1, k + 1);
    }
    stamp(3);
    // MFMA: the A~ / A operands of the predict's two products, read here because the
    // step's DMA (issued below, before the update) refills the A image
    if constexpr (MF) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          mb[kk][p] = *reinterpret_cast<const float*>(lds_ptr(ma_b[kk] + p * G::IMGM));
          ma[kk][p] = *reinterpret_cast<const float*>(lds_ptr(ma_a[kk] + p * G::IMGM));
        }
    } else if constexpr (has_arow<C>()) {
      const T* pr = imA + c;  // lanes > S-1 read the next row: unused (bcast_j, j < S)
#pragma unroll
      for (int i = 0; i < S; ++i) ar[i] = (double)pr[i * S];
    }
    if constexpr (TRAJ && !F32) {  // row c of A_aug = [[A_k, a~],[0, 1]], B_aug = [[B_k],[0]]
      const double* sA = reinterpret_cast<const double*>(wbase + G::OFF_A) + g * 2 * G::CHA;
      const double* sR = reinterpret_cast<const double*>(wbase + G::OFF_B) + g * 2 * G::CHR;
      const int cc = c < NN ? c : 0;
#pragma unroll
      for (int j = 0; j < NN; ++j) at[j] = c < NN ? sA[cc * NN + j] : 0.0;
      at[NN] = c < NN ? atil : (c == NN ? 1.0 : 0.0);
#pragma unroll
      for (int j = 0; j < MM; ++j) brow[j] = c < NN ? sR[cc * MM + j] : 0.0;
    } else {
      const bool in = c < S;
      const T* pa = in ? imA + S * c : zareaT;  // branch-free: lanes > S-1 read zeros
      const T* pbm = in ? imB + MM * c : zareaT;
#pragma unroll
      for (int j = 0; j < S; ++j) at[j] = (double)pa[j];
#pragma unroll
      for (int j = 0; j < MM; ++j) brow[j] = (double)pbm[j];
    }
    }
    at[S] = e_s;
    const bool dma_late = dstag<C>() == 1 && (w & 1);
    // the step's DMA pieces spread through the update block instead of one burst
    // before it (HOP_COND_DMAI, SchedCondLSymL only)
    constexpr bool dmai = kCondDmai && has_symlate<C>() && has_sym2<C>() && !has_newt<C>() &&
                          !TRAJ && !F32 && !has_pack<C>() && S == 13 && MM == 4;
    if constexpr (dstag<C>() == 2) {
      wave_sync();
      if (k + 1 < N)
        dma_stepAB<G::OFF_A, G::OFF_B>(voM, voB, rA, rB, wlds, (unsigned)((k + 1) * SS * ES),
                                       (unsigned)((k + 1) * SM * ES));
    } else {
      // the step's images are consumed: the Q and A image areas are the symmetrisation
      // scratch (the four problems' S x S doubles: 5,408 B, more than one fp32 image)
      if constexpr (!TRAJ && has_sym_every<C>() && !has_symlate<C>()) {
        static_assert(kProbPerWave * S * S * 8 <= G::OFF_QT, "scratch within the Q and A images");
        if (sym_step(k))
          sym_average<S>(reinterpret_cast<double (&)[S]>(X),
                            reinterpret_cast<double*>(wbase + G::OFF_Q) + g * S * S, c);
      }
    }
    if (dstag<C>() != 2 && !dma_late) {
      wave_sync();
      if (k + 1 < N && !dmai && !MF64) dma_step(k + 1);
      if constexpr (has_symlate<C>()) {
        static_assert(!TRAJ && !has_pack<C>(), "own scratch: the one-wave layout");
        if (sym_step(k)) {
          double* scr = reinterpret_cast<double*>(smem_raw + kWavesPerBlock * WB) +
                        (w * kProbPerWave + g) * S * S;
          if constexpr (kSymSplit)
            sym_load_average<S>(reinterpret_cast<double (&)[S]>(X), scr, c);
          else
            sym_average<S>(reinterpret_cast<double (&)[S]>(X), scr, c);
        }
      }
    }
    stamp(4);
    // ---- update: condition the prefix on stage k's cost
    {
      double r[S], Ht[S];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        // Sigma_eps + E_k - I (offset form); SYM2: NE = -E_k/2 + I, so - 2I
        r[i] = has_sym2<C>() ? __builtin_fma(-2.0, NE[i], X[i]) : X[i] - NE[i];
        if constexpr (has_peps<C>())  // an opaque copy: X keeps its loop registers
          asm("v_mov_b64 %0, %1" : "=v"(Ht[i]) : "v"(X[i]));
        else
          Ht[i] = X[i];
      }
      double dmin = 1.0;
      if constexpr (dmai) {  // the next step's pieces issued inside the update block
        {
          // the last step re-reads its own blocks (in L2 / MALL), so the update has
          // one form (two copies of the block spilled 40 VGPRs)
          const int kn = k + 1 < N ? k + 1 : k;
          DmaStep20 q;
#pragma unroll
          for (int j = 0; j < 6; ++j) q.v[j] = voMl[j];
          q.u[0] = voBl[0];
          q.u[1] = voBl[1];
          q.rq = rQ;
          q.ra = rA;
          q.rb = rB;
          q.rt = rT;
          q.so_m = (unsigned)(kn * SS * ES);
          q.so_b = (unsigned)(kn * SM * ES);
          q.m0[0] = wlds + G::OFF_Q;
          q.m0[1] = wlds + G::OFF_Q + 4096;
          q.m0[2] = wlds + G::OFF_A;
          q.m0[3] = wlds + G::OFF_A + 4096;
          q.m0[4] = wlds + G::OFF_B;
          q.m0[5] = wlds + G::OFF_QT;
          q.m0[6] = wlds + G::OFF_QT + 4096;
          CondLdlO2R0D<S>::run(r, Ht, X, dmin, q);
        }
      } else if constexpr (has_sym2<C>() && has_newt<C>()) CondLdl2<S>::run(r, Ht, X, dmin);
      else if constexpr (has_sym2<C>()) CondLdlO2R0<S>::run(r, Ht, X, dmin);
      else if constexpr (has_newt<C>()) CondLdlO1R1<S>::run(r, Ht, X, dmin);
      else CondLdl<S>::run(r, Ht, X, dmin);
      const double x = bcast<S - 1>(r[S - 1]);
      bad = bad || !(dmin > 0.0) || (x != x);
      flag(!(dmin > 0.0) || (x != x), 4, k + 1);
    }
    if (dma_late) {  // DSTAG 1: the odd waves' pieces, half a step after the even waves'
      wave_sync();
      if (k + 1 < N) dma_step(k + 1);
    }
    stamp(5);
    // ---- predict: Sigma_{k+1} = A Sigma' A^T + B R^-1 B^T + eps I, m_{k+1} = A m'
    {
      double Tm[S];
      double (&Xs)[S] = reinterpret_cast<double (&)[S]>(X);
      if constexpr (MF) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        typedef float f2 __attribute__((ext_vector_type(2)));
        // stage [Sigma' | m'] as f32 rows
#pragma unroll
        for (int i = 0; i < S; ++i)
          *reinterpret_cast<float*>(lds_ptr(mx_w + 68u * i)) = (float)X[i];
        f4 D1[4], D2[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) D1[p] = D2[p] = (f4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const float xa = *reinterpret_cast<const float*>(lds_ptr(mx_a + p * MFP + 4u * kk));
            D1[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, mb[kk][p], D1[p], 0, 0, 0);
          }
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            D2[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(ma[kk][p], D1[p][kk], D2[p], 0, 0, 0);
          }
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          *reinterpret_cast<f2*>(lds_ptr(ms_w + p * MFP)) = (f2){D2[p][0], D2[p][1]};
          *reinterpret_cast<f2*>(lds_ptr(ms_w + p * MFP + 8u)) = (f2){D2[p][2], D2[p][3]};
        }
        static_for<S>([&](auto I) {
          X[I] = (double)*reinterpret_cast<const float*>(lds_ptr(ms_r + 4u * I)) +
                 sel_lane<I>(0.0, 1e-9);
        });
      } else if constexpr (MF64) {
        typedef double d4 __attribute__((ext_vector_type(4)));
        if (c < S + 1) {  // stage [Sigma' | m'] rows: [p][row][14] doubles in the Q image
#pragma unroll
          for (int i = 0; i < S; ++i)
            *reinterpret_cast<double*>(lds_ptr(m6_xw + 8u * (S + 1) * i)) = X[i];
        }
        wave_sync();
        double xa[4][4], aa[4][4], bb[4][4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            xa[kk][q] = *reinterpret_cast<const double*>(lds_ptr(m6_xa[kk] + q * M6XP));
            aa[kk][q] = *reinterpret_cast<const double*>(lds_ptr(m6_aa[kk] + q * G::IMGM));
            bb[kk][q] = *reinterpret_cast<const double*>(lds_ptr(m6_ab[kk] + q * G::IMGM));
          }
        d4 D1[4], D2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) D1[q] = D2[q] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            D1[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[kk][q], bb[kk][q], D1[q], 0, 0, 0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            D2[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(aa[kk][q], D1[q][kk], D2[q], 0, 0, 0);
        wave_sync();  // the staging reads are done: the QT image takes the result
        if (c < S + 1) {  // rows g + 4 r < S of column c, as [p][column][13]
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (g + 4 * r < S)
                *reinterpret_cast<double*>(lds_ptr(m6_dw + q * M6XP + 32u * r)) = D2[q][r];
        }
        wave_sync();
        static_for<S>([&](auto I) {
          X[I] = *reinterpret_cast<const double*>(lds_ptr(m6_xr + 8u * I)) + sel_lane<I>(0.0, 1e-9);
        });
      } else if constexpr (has_peps<C>()) {
        PredictEps<S>::run(Xs, Tm, at, ar, eps_addr);  // eps I + A [Sigma' | m'] A~^T
      } else {
      // T = [Sigma' | m'] A~^T; A~^T's row S is e_S, so its term is X masked to lane S
#pragma unroll
      for (int i = 0; i < S; ++i) Tm[i] = X[i] * e_s;
      double (&atS)[S] = reinterpret_cast<double (&)[S]>(at);
      gxy<C, false, S, S>(Tm, Xs, atS);
      static_for<S>([&](auto I) { X[I] = sel_lane<I>(0.0, 1e-9); });
      if constexpr (has_arow<C>()) {
        gxy<C, false, S, S>(Xs, ar, Tm);  // + A T, one chain per row
      } else {
        double (&at13)[S] = reinterpret_cast<double (&)[S]>(at);
        gxty<C, false>(Xs, at13, Tm);  // + A T
      }
      }
      double y[MM];
      zero(y);
      acc_xy<false, double, MM, MM>(y, rinv, brow);
      acc_xty<false, double, S, MM>(Xs, brow, y);  // + B R^-1 B^T
      if constexpr (has_symlate<C>() && kSymSplit) {
        if (sym_store_step(k, N))
          sym_store<S>(Xs, reinterpret_cast<double*>(smem_raw + kWavesPerBlock * WB) +
                               (w * kProbPerWave + g) * S * S,
                       c);
      }
    }
    if constexpr (MF64) {  // the Q / QT / A images are read: the next step's pieces
      wave_sync();
      if (k + 1 < N) dma_step(k + 1);
    }
    stamp(6);
    if constexpr (QPIPE) {  // the query runs in the next step (or after the loop)
#pragma unroll
      for (int i = 0; i < S; ++i) NXp[i] = NX[i];
      kf1 = (bad && kf1 == 0) ? k + 2 : kf1;  // this step's stage flags: horizon k + 1
      continue;
    }
    // ---- query horizon t = k + 1: [Sigma_eps + X_t - I | m] by bordered elimination
    double jk;
    if constexpr (WQ) {
      // QT + eps I = [[P11, b], [b^T, cc]] swept on pivots 0 .. S-2 only (offset form,
      // x KOFF for SYM2): NX = I - P11^-1 / KOFF on rows / lanes < S-1, u = P11^-1 b
      // on lane S-1 of those rows and on row S-1, KOFF sigma - 1 at (S-1, S-1),
      // sigma = cc - b^T P11^-1 b.  X_t = W^T diag(P11^-1, 1/sigma) W with W = [[I, 0],
      // [-u^T, 1]], so the query eliminates W^-T Sigma_eps W^-1 + D with m~ = W^-T m:
      // the augmented terminal block's 1/sigma ~ 1e9 (rho_reg = 1e-12) then sits alone
      // on the last pivot instead of cancelling in every pivot (lft_cond_cf_kernel
      // and small_math.hpp cond_query do the same)
      const double ub = c < S - 1 ? NX[S - 1] : 0.0;
      const double sg = (bcast<S - 1>(NX[S - 1]) + 1.0) * (1.0 / KOFF);
      bad = bad || !(sg > 0.0);
      flag(!(sg > 0.0), 1, k + 1);
      // P = diag(P11^-1 - KOFF I, 0) has a zero last row and column, so W^-T P W^-1 = P:
      // it is added before the congruence (no copy of Sigma's rows needed)
      double rq[S];
#pragma unroll
      for (int i = 0; i < S - 1; ++i) {
        // one three-address v_fma_f64 (hipcc emitted a copy of X[i] + v_fmac: 12 moves)
        if constexpr (kFma3)
          asm("v_fma_f64 %0, %1, %2, %3" : "=v"(rq[i]) : "v"(kmask), "v"(NX[i]), "v"(X[i]));
        else
          rq[i] = __builtin_fma(kmask, NX[i], X[i]);
      }
      rq[S - 1] = X[S - 1];
      RowB<S>::template sweep<S - 1>(rq, ub);  // (.) W^-1
      LaneB<S - 1>::fma(reinterpret_cast<double (&)[S - 1]>(rq), ub, rq[S - 1]);  // W^-T (.)
      rq[S - 1] = __builtin_fma(e_last, recip_nr(sg) - KOFF, rq[S - 1]);  // + 1/sigma - KOFF
      double acc = 0.0, dmin = 1.0;
      ElimQ<S>::run(rq, acc, dmin, KOFF);
      const double q = bcast<S>(acc);
      const double gam = bcast<S>(X[S]);
      bad = bad || !(dmin > 0.0) || (q != q);
      flag(!(dmin > 0.0) || (q != q), 16, k + 1);
      jk = 0.5 * (q - gam);
    } else {
      double rq[S];
#pragma unroll
      for (int i = 0; i < S; ++i)
        rq[i] = has_sym2<C>() ? __builtin_fma(-2.0, NX[i], X[i]) : X[i] - NX[i];
      double acc = 0.0, dmin = 1.0;
      ElimQ<S>::run(rq, acc, dmin, KOFF);
      const double q = bcast<S>(acc);
      const double gam = bcast<S>(X[S]);
      bad = bad || !(dmin > 0.0) || (q != q);
      flag(!(dmin > 0.0) || (q != q), 16, k + 1);
      jk = 0.5 * (q - gam);
    }
    stamp(7);
    if constexpr (TRAJ && !F32) tb.load_rows(cq, imT, c);
    bad = bad || !finite_val(jk);
    flag(!finite_val(jk), 32, k + 1);
    kf1 = (bad && kf1 == 0) ? k + 2 : kf1;  // first flagged horizon + 1
    if (fuse_argmin) {
      const int t = k + 1;
      if (t == a.t_min) {
        best = jk;
        tbest = t;
      } else if (t > a.t_min && t <= a.t_max) {
        const bool bnan = best != best, jnan = jk != jk;
        if (!bnan && (jnan || jk < best)) {
          best = jk;
          tbest = t;
        }
      }
    }
    jprev = jk;
  }
  if constexpr (QPIPE) {  // the last step's query
    if (N > 0) {
      double rq[S], gam, acc = 0.0, dmin = 1.0;
      query_prelude(NXp, rq, gam, N - 1);
      ElimQ<S>::run(rq, acc, dmin, KOFF);
      query_tail(acc, dmin, gam, N - 1);
    }
  }
  dma_wait();
  if constexpr (C::STAMP) {
    if (lane == 0) {
      for (int j = 0; j < 8; ++j) atomicAdd(&g_hop_stamp[j], sec[j]);
      atomicAdd(&g_hop_stamp[15], 1ull);
    }
  }
  if (valid && c == 0) {
    if (!QPIPE && N > 0) a.J[prob * N + N - 1] = (T)jprev;
    // the hand-over word (include/hop.h); the developer reason field under cond & 4
    a.status[prob] = bad ? ((a.cond & 4) ? (int)ST_RERUN | why << HOP_HANDOVER_REASON_SHIFT
                                         : HOP_HANDOVER_WORD(kf1 - 1))
                         : 0;
    if (fuse_argmin && a.t_star != nullptr) {
      a.t_star[prob] = tbest;
      a.j_star[prob] = (T)best;
    }
  }
  if constexpr (has_fuse<C>()) {
    static_assert(!F32, "fused hand-over: fp64 blocks");
    const bool hand = valid && bad;
    if (__any(hand)) {  // wave-uniform; the rerun body uses this wave's LDS only
      LftArgs<double> r = a;
      r.cond = 1;
      using RC = std::conditional_t<TRAJ, SchedLdlTraj, SchedLdlDma>;
      lft_v2_body<RC, S, MM>(r, hand ? 1 : 0);
    }
  }
}



// ===========================================================================
// SchedCondCF: trajectory form of the conditioned kernel with CLOSED-FORM stage
// inverses (Q and P are time-invariant).
//   Q_aug,k + eps I = [[Qs + eps I, q],[q^T, c]],  q = Q e_k, c = e_k^T Q e_k + 2w + rho + eps
//   (Qs = _sym(Q) + q_reg I, augmented.py:31-47) has the inverse
//   Qi_ext + w' v'^T with Qi = (Qs + eps I)^-1 (once per problem), v = Qi q,
//   v' = [v; -1], sigma = c - q.v, w' = v' / sigma.
//   QT_aug,t + eps I = [[P + eps I, P e],[e^T P, e^T P e + rho + eps]] likewise, with
//   u = Pi P e = e - eps Pi e and the Schur complement in its cancellation-free
//   form sigma_T = rho + eps + eps e.u (augmented.py:63-87).
// So each step needs two matrix-vector products and two rank-1 updates instead
// of two 13 x 13 Gauss-Jordan sweeps, and S = Sigma_eps + E_k comes out
// directly (non-offset: CondLdlN).  Qs + eps I or P + eps I not PD, sigma <= 0,
// a bad pivot or a non-finite J hand the problem to the rerun launch.
// ===========================================================================
template <int NN>
__device__ __forceinline__ void lane_matvec(double& out, double x, const double (&rows)[NN]) {
  double q4[4] = {0.0, 0.0, 0.0, 0.0};
  LaneDot4<NN>::fma(q4, x, rows);  // sum_j bcast_j(x) rows[j]
  out = (q4[0] + q4[1]) + (q4[2] + q4[3]);
}

template <class C, int S, int MM>
__global__ __launch_bounds__(256, 1) void lft_cond_cf_kernel(LftArgs<double> a) {
  using G = Geo<S, MM>;
  constexpr int NN = G::NN;
  static_assert(S < kRowLanes && G::NJA == 5 && G::NJR == 2 && G::NJX == 1 && G::NJV == 1 &&
                    G::NJU == 1,
                "trajectory pieces of the s = 13, m = 4 shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned char* wbase = smem_raw + w * G::WAVE_BYTES_T;
  const unsigned wlds = (unsigned)(uintptr_t)wbase;
  const long long wave_prob0 = ((long long)blockIdx.x * kWavesPerBlock + w) * kProbPerWave;
  const long long prob = wave_prob0 + g;
  const bool valid = prob < a.batch;
  const long long pb0 = wave_prob0 < a.batch ? wave_prob0 : a.batch - 1;
  const long long pb = valid ? prob : a.batch - 1;
  const int N = a.n;
  const TrajArgs<double>& t = a.tr;
  auto mk = [&](const double* base, long long pstr) {
    const long long left = (a.batch - pb0) * pstr;
    const unsigned nrec = left > 0xFFFFFFF0ll ? 0xFFFFFFF0u : (unsigned)left;
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double*>(base) + pb0 * (pstr / 8), (short)0, (int)nrec, 0x00020000);
  };
  const long long pstA = (long long)a.nalloc * NN * NN * 8, pstR = (long long)a.nalloc * NN * MM * 8;
  const long long pstX = (long long)(a.nalloc + 1) * NN * 8, pstV = (long long)a.nalloc * NN * 8;
  const long long pstU = (long long)a.nalloc * MM * 8;
  const __amdgpu_buffer_rsrc_t rA = mk(t.A, pstA), rB = mk(t.Bm, pstR), rX = mk(t.X, pstX),
                               rV = mk(t.ares, pstV), rU = mk(t.U, pstU);
  unsigned voTA[G::NJA], voTR[G::NJR], voTX[1], voTV[1], voTU[1];
#pragma unroll
  for (int j = 0; j < G::NJA; ++j)
    voTA[j] = chunk_voff<G::CHA>(j, lane, wave_prob0, pb0, a.batch, pstA);
#pragma unroll
  for (int j = 0; j < G::NJR; ++j)
    voTR[j] = chunk_voff<G::CHR>(j, lane, wave_prob0, pb0, a.batch, pstR);
  voTX[0] = chunk_voff<G::CHX>(0, lane, wave_prob0, pb0, a.batch, pstX);
  voTV[0] = chunk_voff<G::CHV>(0, lane, wave_prob0, pb0, a.batch, pstV);
  voTU[0] = chunk_voff<G::CHU>(0, lane, wave_prob0, pb0, a.batch, pstU);
  unsigned voTAl[G::NJA], voTRl[G::NJR];  // lowered by the pieces' instruction offsets
#pragma unroll
  for (int j = 0; j < G::NJA; ++j) voTAl[j] = dma_voff_lowered(voTA[j], j);
#pragma unroll
  for (int j = 0; j < G::NJR; ++j) voTRl[j] = dma_voff_lowered(voTR[j], j);
  auto dma_step = [&](int k) {  // A_k, B_k, x_{k+1}, a_k, u_k
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned soA = (unsigned)(k * NN * NN * 8), soR = (unsigned)(k * NN * MM * 8),
                   soV = (unsigned)(k * NN * 8), soU = (unsigned)(k * MM * 8);
    dma_traj10<G::OFF_A, G::OFF_B, G::OFF_VX, G::OFF_VA, G::OFF_VU>(
        voTAl, voTRl, voTX[0], voTV[0], voTU[0], rA, rB, rX, rV, rU, wlds, soA, soR, soV + NN * 8,
        soV, soU);
  };
  dma_step(0);

  // ---- per-problem constants (lane c = column c; lanes > NN-1 zero)
  const double* Qg = t.Q + pb * t.q_bs;
  const double* Pg = t.P + pb * t.p_bs;
  const bool in = c < NN;
  const int cc = in ? c : 0;
  const double eps = 1e-9;
  bool bad = (a.cond & 2) != 0;
  // the first flagged horizon + 1 (0: none; 1: the prologue or a forced hand-over),
  // left in status bits 13.. for the rerun launch's non-finite triage
  int kf1 = bad ? 1 : 0;
  // developer builds: the first failing test and its horizon (hand-over diagnosis,
  // reported in status bits 5.. under a.cond & 4); product builds compile none of it
  int why = 0;
  auto flag = [&](bool f, int bit, int t) {
    if constexpr (kDevBuild) why = (f && why == 0) ? (bit | (t << 8)) : why;
  };
  // raw Q rows (Q e), (Qs + eps I)^-1 and (P + eps I)^-1 rows, parked per wave in
  // LDS as register images (row i of lane l at [i][l]; the Q / QT image areas
  // and the tile slot are free in this kernel) and re-read each step
  double* lq = reinterpret_cast<double*>(wbase + G::OFF_T);
  double* csym = reinterpret_cast<double*>(wbase + G::OFF_CQ) + g * S * S;  // sym scratch
  double* lqi = reinterpret_cast<double*>(wbase + G::OFF_Q);
  double* lpi = reinterpret_cast<double*>(wbase + G::OFF_QT);
  static_assert(G::TILE_W >= NN * 512 && G::IMGM_W >= NN * 512, "constant images");
  {
    double qr[NN], Qi[NN], Pi[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      qr[i] = in ? Qg[cc * NN + i] : 0.0;  // lane c: Q[c][i], so sum_i bcast_i(e) qr[i] = (Q e)[c]
      const double qs = 0.5 * (Qg[i * NN + cc] + Qg[cc * NN + i]) + (i == c ? t.q_reg : 0.0);
      Qi[i] = in ? qs : 0.0;
      Pi[i] = in ? Pg[i * NN + cc] : 0.0;
    }
    // offset form (diag - 1 + eps), swept: -M^-1 + I; back to M^-1 with the lane selects
    static_for<NN>([&](auto I) {
      Qi[I] = Qi[I] + sel_lane<I>(0.0, eps - 1.0);
      Pi[I] = Pi[I] + sel_lane<I>(0.0, eps - 1.0);
    });
    double d1 = 1.0, d2 = 1.0;
    SweepQ<NN>::run(Qi, d1);
    SweepQ<NN>::run(Pi, d2);
    bad = bad || !pivots_ok(Qi, d1) || !pivots_ok(Pi, d2);
    flag(bad, 1, 0);
    kf1 = bad ? 1 : 0;
    static_for<NN>([&](auto I) {
      Qi[I] = sel_lane<I>(0.0, 1.0) - Qi[I];
      Pi[I] = sel_lane<I>(0.0, 1.0) - Pi[I];
    });
#pragma unroll
    for (int i = 0; i < NN; ++i) {
      lq[i * 64 + lane] = qr[i];
      lqi[i * 64 + lane] = Qi[i];
      lpi[i * 64 + lane] = Pi[i];
    }
  }
  auto rows = [&](const double* img, double (&o)[NN]) {
#pragma unroll
    for (int i = 0; i < NN; ++i) o[i] = img[i * 64 + lane];
  };
  const double xg_c = in ? t.xg[pb * t.xg_bs + cc] : 0.0;
  const double ur_c = c < MM ? t.u_ref[pb * t.ur_bs + (c < MM ? c : 0)] : 0.0;
  const double w2 = 2.0 * t.w[pb * t.w_bs];
  const bool wrap_c = in && ((t.wrap_mask >> c) & 1u);
  auto err = [&](double x) {  // wrap_error(x - xg) on lane c (utils.py:131-137)
    double e = in ? x - xg_c : 0.0;
    if (t.wrap_mask != 0u) {
      const double we = wrap_angle(e);
      e = wrap_c ? we : e;
    }
    return e;
  };
  // e_0, Q e_0, e_0^T Q e_0 (carried: step k's stage block uses e_k)
  double qe_k, eqe_k;
  {
    const double e0 = err(t.X[pb * (long long)(a.nalloc + 1) * NN + cc]);
    double qr[NN];
    rows(lq, qr);
    lane_matvec<NN>(qe_k, e0, qr);
    eqe_k = lane_sum<NN>(e0 * qe_k);
  }
  double rinv[MM];
  {
    const double* Rp = a.R + pb * a.r_bstride;
#pragma unroll
    for (int i = 0; i < MM; ++i) rinv[i] = (c < MM) ? Rp[i * MM + (c < MM ? c : 0)] : 0.0;
  }
  double X[S + 1];  // [Sigma_eps | m], gamma on lane S of X[S]; z0 = e_s (augmented.py:57)
  static_for<S>([&](auto I) { X[I] = (c == S) ? (I == NN ? 1.0 : 0.0) : sel_lane<I>(0.0, eps); });
  X[S] = 0.0;
  const double e_s = (c == S) ? 1.0 : 0.0;
  const double e_nn = (c == NN) ? 1.0 : 0.0;  // the query's 1/sigma entry
  const double m1 = (c == NN) ? -1.0 : 0.0;  // lane NN of v' / u'

  double best = 0.0, jprev = 0.0;
  int tbest = 0;
  const bool fuse_argmin = a.t_max > 0;
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    dma_wait();
    wave_sync();
    if (k > 0 && valid && c == 0) a.J[prob * N + k - 1] = jprev;
    const double* sX = reinterpret_cast<const double*>(wbase + G::OFF_VX) + g * 2 * G::CHX;
    const double* sV = reinterpret_cast<const double*>(wbase + G::OFF_VA) + g * 2 * G::CHV;
    const double* sU = reinterpret_cast<const double*>(wbase + G::OFF_VU) + g * 2 * G::CHU;
    const double* sR = reinterpret_cast<const double*>(wbase + G::OFF_B) + g * 2 * G::CHR;
    const double* sA = reinterpret_cast<const double*>(wbase + G::OFF_A) + g * 2 * G::CHA;
    // raw pieces of step k: x_{k+1}, a_k, u_k, row c of A_k and B_k
    const int cm = c < MM ? c : 0;
    const double x1 = sX[cc], av = in ? sV[cc] : 0.0, uu = sU[cm];
    double at[S + 1], brow[MM];
#pragma unroll
    for (int j = 0; j < NN; ++j) at[j] = in ? sA[cc * NN + j] : 0.0;
#pragma unroll
    for (int j = 0; j < MM; ++j) brow[j] = in ? sR[cc * MM + j] : 0.0;
    wave_sync();
    if (k + 1 < N) dma_step(k + 1);
    // a~_k = a_k - B_k du_k (augmented.py:50); A~ = [[A_k, a~],[0, 1]]
    const double du = c < MM ? uu - ur_c : 0.0;
    double bd;
    {
      double rb[MM];
#pragma unroll
      for (int q = 0; q < MM; ++q) rb[q] = brow[q];
      bd = 0.0;
      LaneDot<MM>::fma(bd, du, rb);
    }
    const double atil = av - bd;
    at[NN] = in ? atil : (c == NN ? 1.0 : 0.0);
    at[S] = e_s;
    // the periodic symmetrisation (split: the rows were stored after the last predict);
    // its reads share their round trip with e_{k+1}'s below (X is first needed after)
    constexpr bool SYMI = kSymSplit && has_sym_every<C>() && S == 13;
    double ysym[S];
    const bool sy = sym_step(k);
    if constexpr (SYMI) {
      if (sy) sym_issue13(csym, c, reinterpret_cast<double (&)[13]>(ysym));
    } else if constexpr (kSymSplit && has_sym_every<C>()) {
      if (sy) sym_load_average<S>(reinterpret_cast<double (&)[S]>(X), csym, c);
    }
    // ---- e_{k+1}: the terminal block of horizon k+1 and the next stage block
    const double e1 = err(x1);
    double qe1;
    {
      double qr[NN];
      rows(lq, qr);
      lane_matvec<NN>(qe1, e1, qr);
    }
    const double eqe1 = lane_sum<NN>(e1 * qe1);
    if constexpr (SYMI) {
      if (sy)
        sym_wait_average13(reinterpret_cast<double (&)[13]>(X),
                           reinterpret_cast<double (&)[13]>(ysym), c);
    }
    // ---- stage inverse E_k in closed form, S = Sigma_eps + E_k (non-offset)
    double r[S];
    {
      double Qi[NN];
      rows(lqi, Qi);
      double v;
      lane_matvec<NN>(v, qe_k, Qi);  // Qi q
      const double qv = lane_sum<NN>(qe_k * v);
      const double sig = (((eqe_k + w2) + t.rho_reg) + eps) - qv;
      bad = bad || !(sig > 0.0);
      flag(!(sig > 0.0), 2, k + 1);
      const double vp = in ? v : m1;
      const double wp = vp * recip_nr(sig);
#pragma unroll
      for (int i = 0; i < NN; ++i) r[i] = X[i] + Qi[i];
      r[NN] = X[NN];
      LaneB<S>::fma(r, wp, vp);  // + w' v'^T
    }
    // ---- update: condition the prefix on stage k's cost
    if (!kSymSplit && has_sym_every<C>() && sym_step(k))
      sym_average<S>(reinterpret_cast<double (&)[S]>(X), csym, c);
    {
      double Ht[S];
      copy(Ht, reinterpret_cast<double (&)[S]>(X));
      double dmin = 1.0;
      CondLdlN<S>::run(r, Ht, X, dmin);
      const double x = bcast<S - 1>(r[S - 1]);
      bad = bad || !(dmin > 0.0) || (x != x);
      flag(!(dmin > 0.0) || (x != x), 4, k + 1);
    }
    // ---- predict
    {
      double T[S];
      zero(T);
      double (&Xs)[S] = reinterpret_cast<double (&)[S]>(X);
      gxy<C, false, S, S + 1>(T, Xs, at);  // T = [Sigma' | m'] A~^T
      static_for<S>([&](auto I) { X[I] = sel_lane<I>(0.0, eps); });
      double (&at13)[S] = reinterpret_cast<double (&)[S]>(at);
      gxty<C, false>(Xs, at13, T);  // + A~ T
      double y[MM];
      zero(y);
      acc_xy<false, double, MM, MM>(y, rinv, brow);
      acc_xty<false, double, S, MM>(Xs, brow, y);  // + B R^-1 B^T
      if constexpr (kSymSplit && has_sym_every<C>()) {
        if (sym_store_step(k, N)) sym_store<S>(Xs, csym, c);
      }
    }
    // ---- query of horizon k+1 with QT_aug[k] (e_{k+1}) in closed form
    double jk;
    {
      double Pi[NN];
      rows(lpi, Pi);
      double z;
      lane_matvec<NN>(z, e1, Pi);  // Pi e
      const double u = in ? e1 - eps * z : m1;  // Pi P e = e - eps Pi e
      const double eu = lane_sum<NN>(e1 * u);
      const double sig = (t.rho_reg + eps) + eps * eu;
      bad = bad || !(sig > 0.0);
      flag(!(sig > 0.0), 8, k + 1);
      double rq[S];
      if constexpr (has_gjq<C>()) {
#pragma unroll
        for (int i = 0; i < NN; ++i) rq[i] = X[i] + Pi[i];
        rq[NN] = X[NN];
      }
      double q;
      if constexpr (has_gjq<C>()) {  // round 3: eliminate Sigma_eps + X_t itself
        const double wq = u * recip_nr(sig);
        LaneB<S>::fma(rq, wq, u);
        double acc = 0.0, dmin = 1.0;
        ElimQ<S>::run(rq, acc, dmin, 0.0);
        q = bcast<S>(acc);
        bad = bad || !(dmin > 0.0) || (q != q);
        flag(!(dmin > 0.0) || (q != q), 16, k + 1);
      } else {
        // X_t = W^T D W with D = diag(Pi, 1/sigma), W = [[I, 0], [-u^T, 1]] (u here the
        // first NN lanes of u), so m^T (Sigma_eps + X_t)^-1 m = m~^T (Sigma~ + D)^-1 m~
        // with Sigma~ = W^-T Sigma_eps W^-1, m~ = W^-T m, W^-1 = I + e_NN [u; 0]^T.  The
        // 1/sigma ~ 1e9 of the terminal block then sits alone on the last diagonal
        // entry: no pivot cancels it (the round-3 form, eliminating Sigma_eps + X_t,
        // lost 1e-7 .. 1e-5 of q on real quadrotor linearisations and handed problems
        // the reference solves cleanly to the rerun; this form holds ~1e-16, measured
        // against exact rational arithmetic)
        // Pi_ext has a zero last row and column: W^-T Pi_ext W^-1 = Pi_ext, so it is
        // added before the congruence
        const double ub = in ? e1 - eps * z : 0.0;
#pragma unroll
        for (int i = 0; i < NN; ++i) rq[i] = X[i] + Pi[i];
        rq[NN] = X[NN];
        RowB<S>::template sweep<NN>(rq, ub);  // (.) W^-1: row i += (.)_i,NN [u; 0]
        LaneB<NN>::fma(reinterpret_cast<double (&)[NN]>(rq), ub, rq[NN]);  // W^-T (.): + u_i row NN
        rq[NN] = __builtin_fma(e_nn, recip_nr(sig), rq[NN]);  // D's 1/sigma
        double acc = 0.0, dmin = 1.0;
        ElimQ<S>::run(rq, acc, dmin, 0.0);
        q = bcast<S>(acc);
        bad = bad || !(dmin > 0.0) || (q != q);
        flag(!(dmin > 0.0) || (q != q), 16, k + 1);
      }
      const double gam = bcast<S>(X[S]);
      jk = 0.5 * (q - gam);
    }
    qe_k = qe1;
    eqe_k = eqe1;
    bad = bad || !finite_val(jk);
    flag(!finite_val(jk), 32, k + 1);
    kf1 = (bad && kf1 == 0) ? k + 2 : kf1;
    if (fuse_argmin) {
      const int tt = k + 1;
      if (tt == a.t_min) {
        best = jk;
        tbest = tt;
      } else if (tt > a.t_min && tt <= a.t_max) {
        const bool bnan = best != best, jnan = jk != jk;
        if (!bnan && (jnan || jk < best)) {
          best = jk;
          tbest = tt;
        }
      }
    }
    jprev = jk;
  }
  dma_wait();
  if (valid && c == 0) {
    if (N > 0) a.J[prob * N + N - 1] = jprev;
    a.status[prob] = bad ? ((a.cond & 4) ? (int)ST_RERUN | why << HOP_HANDOVER_REASON_SHIFT
                                         : HOP_HANDOVER_WORD(kf1 - 1))
                         : 0;
    if (fuse_argmin && a.t_star != nullptr) {
      a.t_star[prob] = tbest;
      a.j_star[prob] = best;
    }
  }
  if constexpr (has_fuse<C>()) {  // the fused hand-over (see SchedCondTrajF)
    const bool hand = valid && bad;
    if (__any(hand)) {
      LftArgs<double> r = a;
      r.cond = 1;
      lft_v2_body<SchedLdlTraj, S, MM>(r, hand ? 1 : 0);
    }
  }
}

}  // namespace v2

// Small-s row groups (SchedCondSmall): fp64 augmented blocks at s <= 5, batch-major,
// when the batch leaves lft_small.hip's one-problem-per-lane kernel most SIMDs idle
// (B / 64 waves).  Four problems per wave (one per DPP row),
// so B = 4,096 runs 1,024 waves.  Its hand-overs go to lft_small.hip's LFT
// instantiation (the rerun launch alone: cond = 1 | kCondRerunOnly), whose chol_inv
// ladders and status bits are the reference's.  Larger batches (and tile64 blocks, the
// trajectory form, per-step R, debug outputs) stay on lft_small.hip.
// The crossover batch (kSmallRowGroupMax, hop_kernels.hpp): tools/bench_small_rg.py.
namespace v2 {
template <int S, int MM>
hipError_t launch_cond_small(const LftArgs<double>& a, hipStream_t stream) {
  using G = Geo<S, MM, 8, false, true>;
  static_assert(G::WAVE_BYTES * kWavesPerBlock <= 64 * 1024, "several workgroups per CU");
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  const bool force = opt(HOP_OPT_FORCE_HANDOVER);
  LftArgs<double> c = a;
  c.cond = (force ? 2 : 0) | ((kDevBuild && opt(HOP_OPT_NO_RERUN)) ? 4 : 0);
  hipLaunchKernelGGL((lft_cond_kernel<SchedCondSmall, S, MM>), dim3((unsigned)blocks), dim3(256),
                     (size_t)(G::WAVE_BYTES * kWavesPerBlock), stream, c);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess || opt(HOP_OPT_NO_RERUN)) return e;  // hand-over words left in status
  LftArgs<double> r = a;
  r.cond = 1 | kCondRerunOnly;
  return dispatch_lft_small<double>(r, stream);
}
}  // namespace v2
hipError_t dispatch_cond_small(const LftArgs<double>& a, hipStream_t stream) {
  if (a.traj || a.tile64 || !cond_small_takes(a.s, a.m, a.batch)) return hipErrorNotSupported;
#ifdef HOP_DEV
  if (g_opt_variant == 80) return hipErrorNotSupported;  // A/B: the lane-per-problem kernel
#endif
  if (a.s == 2 && a.m == 1) return v2::launch_cond_small<2, 1>(a, stream);
  if (a.s == 3 && a.m == 1) return v2::launch_cond_small<3, 1>(a, stream);
  if (a.s == 4 && a.m == 1) return v2::launch_cond_small<4, 1>(a, stream);
  if (a.s == 4 && a.m == 2) return v2::launch_cond_small<4, 2>(a, stream);
  if (a.s == 5 && a.m == 1) return v2::launch_cond_small<5, 1>(a, stream);
  if (a.s == 5 && a.m == 2) return v2::launch_cond_small<5, 2>(a, stream);
  return hipErrorNotSupported;
}

// exact-size fast path: returns hipErrorNotSupported when the shape has none.
// Product builds: the conditioned-prefix kernel + the rerun launch of the
// reference association for the problems it flagged (HOP_OPT_REFERENCE_ASSOC:
// the reference association alone; HOP_OPT_FORCE_HANDOVER: every problem handed
// over).  Developer builds (HOP_DEV) add the A/B schedules of DESIGN.md 3.2 by
// number (hop_set_options variant).
hipError_t dispatch_lft_v2(const LftArgs<double>& a, hipStream_t stream) {
  if (a.dbg_efg || a.dbg_pre || a.r_kstride != 0 || !a.r_is_inv) return hipErrorNotSupported;
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  const int variant = g_opt_variant;
  auto launch = [&](auto kern, size_t bytes, const LftArgs<double>& args) {
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), bytes, stream, args);
    return hipGetLastError();
  };
  // conditioned kernel, then the rerun launch (cond = 1) of the flagged problems
  // developer builds under HOP_OPT_NO_RERUN: the flagged problems' status also
  // carries the first failing test and horizon (bits 5.., lft_cond_cf_kernel)
  const int why_bit = (kDevBuild && opt(HOP_OPT_NO_RERUN)) ? 4 : 0;
  auto cond_rerun = [&](auto kc, auto kr, size_t bytes, bool rerun) {
    LftArgs<double> c = a;
    const bool force = opt(HOP_OPT_FORCE_HANDOVER);
    c.cond = (force ? 2 : 0) | why_bit;
    hipError_t e = launch(kc, bytes, c);
    if (e != hipSuccess || !rerun) return e;
    // the rerun launch: non-finite triage, then the recompute of the rest
    // (HOP_OPT_NO_RERUN: the triage alone, the rest keep HOP_ST_HANDOVER)
    LftArgs<double> r = a;
    r.cond = 1 | (force ? 16 : 0) | (opt(HOP_OPT_NO_RERUN) ? 8 | why_bit : 0);
    return launch(kr, bytes, r);
  };
  // augmented blocks: the rerun launch is the pipelined recompute (lft_rerun_pipe_kernel;
  // its LDS also holds the LFT body's layout for the fallback)
  using PipeG = v2::PipeGeo<13, 4, v2::kPipeBS>;
  constexpr size_t bytes_pipe =
      (size_t)PipeG::BYTES > (size_t)v2::Geo<13, 4>::WAVE_BYTES * kWavesPerBlock
          ? (size_t)PipeG::BYTES
          : (size_t)v2::Geo<13, 4>::WAVE_BYTES * kWavesPerBlock;
  static_assert(bytes_pipe <= 160 * 1024, "one workgroup per CU");
  auto cond_pipe = [&](auto kc, size_t bytes) {
    LftArgs<double> c = a;
    const bool force = opt(HOP_OPT_FORCE_HANDOVER);
    c.cond = (force ? 2 : 0) | why_bit;
    hipError_t e = launch(kc, bytes, c);
    if (e != hipSuccess) return e;
    LftArgs<double> r = a;
    r.cond = 1 | (force ? 16 : 0) | (opt(HOP_OPT_NO_RERUN) ? 8 | why_bit : 0);
    return launch(v2::lft_rerun_pipe_kernel<v2::SchedLdlDma, 13, 4, v2::kPipeBS>, bytes_pipe, r);
  };
  if (a.traj) {  // in-kernel augmentation (capi routes only s = 13, m = 4 here)
    if (a.s != 13 || a.m != 4 || a.tr.n != 12 || a.tr.m != 4) return hipErrorNotSupported;
    const size_t bytes = (size_t)(v2::Geo<13, 4>::WAVE_BYTES_T * kWavesPerBlock);
    if (opt(HOP_OPT_REFERENCE_ASSOC))
      return launch(v2::lft_sweep_v2_kernel<v2::SchedLdlTraj, 13, 4>, bytes, a);
#ifdef HOP_DEV
    if (variant == 54)  // closed-form stage inverses without the rerun launch
      return cond_rerun(v2::lft_cond_cf_kernel<v2::SchedCondTraj, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlTraj, 13, 4>, bytes, false);
    if (variant == 95)
      return cond_rerun(v2::lft_cond_cf_kernel<v2::SchedCondTrajNS, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlTraj, 13, 4>, bytes, true);
    if (variant == 94)
      return cond_rerun(v2::lft_cond_cf_kernel<v2::SchedCondTrajGNS, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlTraj, 13, 4>, bytes, true);
    if (variant == 97 || variant == 98)  // the round-3 query (+ rerun unless 98)
      return cond_rerun(v2::lft_cond_cf_kernel<v2::SchedCondTrajG, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlTraj, 13, 4>, bytes, variant == 97);
    if (variant == 40 || variant == 41)  // Gauss-Jordan stage inverses (+ rerun unless 41)
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondTraj, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlTraj, 13, 4>, bytes, variant == 40);
    if (variant == 24 || opt(HOP_OPT_STAMPS))  // section stamps (tools/stamps.py --traj)
      return launch(v2::lft_sweep_v2_kernel<v2::SchedLdlTrajStamped, 13, 4>, bytes, a);
    if (variant == 61) {  // the fused hand-over (measured slower)
      LftArgs<double> c = a;
      c.cond = opt(HOP_OPT_FORCE_HANDOVER) ? 2 : 0;
      return launch(v2::lft_cond_cf_kernel<v2::SchedCondTrajF, 13, 4>, bytes, c);
    }
#endif
    // default: closed-form stage inverses, then the pipelined rerun
    {
      using PipeT = v2::PipeGeo<13, 4, v2::kPipeBS>;
      constexpr size_t bytes_pt = (size_t)PipeT::BYTES > (size_t)v2::Geo<13, 4>::WAVE_BYTES_T * kWavesPerBlock
                                      ? (size_t)PipeT::BYTES
                                      : (size_t)v2::Geo<13, 4>::WAVE_BYTES_T * kWavesPerBlock;
      static_assert(bytes_pt <= 160 * 1024, "one workgroup per CU");
      LftArgs<double> c = a;
      const bool force = opt(HOP_OPT_FORCE_HANDOVER);
      c.cond = (force ? 2 : 0) | why_bit;
      const hipError_t e = launch(v2::lft_cond_cf_kernel<v2::SchedCondTraj, 13, 4>, bytes, c);
      if (e != hipSuccess) return e;
      LftArgs<double> r = a;
      r.cond = 1 | (force ? 16 : 0) | (opt(HOP_OPT_NO_RERUN) ? 8 | why_bit : 0);
      return launch(v2::lft_rerun_pipe_kernel<v2::SchedLdlTraj, 13, 4, v2::kPipeBS>, bytes_pt, r);
    }
  }
  if (a.s <= 5) return dispatch_cond_small(a, stream);  // (lft_small.hip when not taken)
  if (a.s != 13 || a.m != 4) return hipErrorNotSupported;
  constexpr size_t bytes = v2::Geo<13, 4>::WAVE_BYTES * kWavesPerBlock;
  // + the symmetrisation scratch of SchedCondLSymL past the four waves' areas
  constexpr size_t bytes_symlate = bytes + (size_t)kWavesPerBlock * kProbPerWave * 13 * 13 * 8;
  static_assert(bytes_symlate <= 160 * 1024, "one workgroup per CU");
  if (opt(HOP_OPT_REFERENCE_ASSOC) || variant == 30)
    return launch(v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes, a);
#ifdef HOP_DEV
  switch (variant) {
    case 93:  // the default with round 4's one-wave LFT rerun launch (A/B of the pipeline)
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondLSymL, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes_symlate, true);
    case 96:  // the default without the periodic symmetrisation + rerun
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondLSymNS, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes, true);
    case 99:  // the round-3 query (the full X sweep, Sigma_eps + X_t eliminated) + rerun
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondLSymG, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes, true);
    case 42:  // stamps of the default (tools/stamps.py --cond), no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLSymLStamped, 13, 4>, bytes_symlate, a);
    case 59:  // stamps of the round-2 default (halved sums), no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLStamped, 13, 4>, bytes, a);
    case 43:  // image reads not overlapped with the sweeps, no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCond, 13, 4>, bytes, a);
    case 44:  // SYM2 conditioned kernel + rerun
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondL2, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes, true);
    case 45:  // SYM2 without the rerun launch
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondL2, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes, false);
    case 46:  // SYM2 stamps, no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondL2Stamped, 13, 4>, bytes, a);
    case 50:  // DMA: odd waves after the update, no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLStag1, 13, 4>, bytes, a);
    case 51:  // DMA: Q/QT after the E sweep, A/B after the X sweep, no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLStag2, 13, 4>, bytes, a);
    case 47:  // the unhalved sums alone (the default's kernel), no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLSym, 13, 4>, bytes, a);
    case 48:  // the update's Newton on the reciprocal alone, no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLNewt, 13, 4>, bytes, a);
    case 49:  // the one-block predict with LDS eps rows alone, no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLPeps, 13, 4>, bytes, a);
    case 52:  // the unhalved sums + the reciprocal Newton (47 + 48), no rerun
      return launch(v2::lft_cond_kernel<v2::SchedCondLSN, 13, 4>, bytes, a);
    case 41:  // the default's conditioned kernel without the rerun launch (A/B timing)
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondLSymL, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes_symlate, false);
    case 90:  // round 4's first placement: the symmetrisation before the DMA issue, + rerun
      return cond_rerun(v2::lft_cond_kernel<v2::SchedCondLSym, 13, 4>,
                        v2::lft_sweep_v2_kernel<v2::SchedLdlDma, 13, 4>, bytes, true);
    case 58:  // round-2 default (halved symmetric sums) without the rerun launch
      return launch(v2::lft_cond_kernel<v2::SchedCondL, 13, 4>, bytes, a);
    case 60: {  // fused hand-over: flagged problems recomputed at the end of the same
                // launch (lft_v2_body); the kernel then carries the LFT body's scratch and
                // measured 0.7-2 % slower than the default's second launch
      LftArgs<double> c = a;
      c.cond = opt(HOP_OPT_FORCE_HANDOVER) ? 2 : 0;
      return launch(v2::lft_cond_kernel<v2::SchedCondLSymF, 13, 4>, bytes, c);
    }
    case 2: return launch(v2::lft_sweep_v2_kernel<v2::Select, 13, 4>, bytes, a);
    case 8: return launch(v2::lft_sweep_v2_kernel<v2::Chain, 13, 4>, bytes, a);
    case 10: return launch(v2::lft_sweep_v2_kernel<v2::Sched, 13, 4>, bytes, a);
    case 12: return launch(v2::lft_sweep_v2_kernel<v2::SchedRow, 13, 4>, bytes, a);
    case 14: return launch(v2::lft_sweep_v2_kernel<v2::SchedLdl, 13, 4>, bytes, a);
    case 20: return launch(v2::lft_sweep_v2_kernel<v2::SchedStamped, 13, 4>, bytes, a);
    case 32: return launch(v2::lft_sweep_v2_kernel<v2::SchedLdlDmaStamped, 13, 4>, bytes, a);
    default: break;
  }
  if (opt(HOP_OPT_STAMPS))
    return launch(v2::lft_cond_kernel<v2::SchedCondLSymLStamped, 13, 4>, bytes_symlate, a);
#endif
  // more waves than SIMDs: the packed-image layout at two waves per SIMD (the rerun
  // launch keeps the LFT kernel's own layout)
#ifdef HOP_DEV
  const bool pack1 = variant == 92, pack2 = variant == 91;  // forced layouts (A/B)
#else
  constexpr bool pack1 = false, pack2 = false;
#endif
  if (!pack1 && (pack2 || (a.batch + kProbPerWave - 1) / kProbPerWave > 4ll * cu_count(stream))) {
    LftArgs<double> c = a;
    const bool force = opt(HOP_OPT_FORCE_HANDOVER);
    c.cond = (force ? 2 : 0) | why_bit;
    hipError_t e = launch(v2::lft_cond_kernel<v2::SchedCondLSymP, 13, 4>,
                          (size_t)v2::Geo<13, 4, 8, true>::WAVE_BYTES * kWavesPerBlock, c);
    if (e != hipSuccess) return e;
    LftArgs<double> r = a;  // as cond_pipe: triage, then the pipelined recompute
    r.cond = 1 | (force ? 16 : 0) | (opt(HOP_OPT_NO_RERUN) ? 8 | why_bit : 0);
    return launch(v2::lft_rerun_pipe_kernel<v2::SchedLdlDma, 13, 4, v2::kPipeBS>, bytes_pipe, r);
  }
  // default (variant 40): conditioned prefix + rerun of the problems it flagged; the
  // stage / terminal inverses of the unhalved symmetric sums (SYM2: 1-2 % faster than
  // the halved sums, profiles/history/r03_ab1_cond_schedules.txt, r03_ab_pe.txt); the periodic
  // symmetrisation after the step's DMA issue, in its own LDS scratch (SchedCondLSymL:
  // 0.4 % faster than before it, bitwise equal, profiles/history/r04_p18_ab_symlate.txt)
  return cond_pipe(v2::lft_cond_kernel<v2::SchedCondLSymL, 13, 4>, bytes_symlate);
}

}  // namespace hop

// fp32 blocks at s = 13, m = 4: the conditioned-prefix kernel on fp32 images
// (fp64 arithmetic), then the generic fp32 kernel in rerun mode for the problems
// it flagged.  HOP_OPT_REFERENCE_ASSOC keeps the generic path.
namespace hop {
hipError_t dispatch_lft_v2_f32(const LftArgs<float>& a, hipStream_t stream) {
  if (a.dbg_efg || a.dbg_pre || a.r_kstride != 0 || !a.r_is_inv || a.traj) return hipErrorNotSupported;
  if (a.s != 13 || a.m != 4) return hipErrorNotSupported;
  const int var = g_opt_variant;
  if (opt(HOP_OPT_REFERENCE_ASSOC) ||
      (var != 0 && var != 40 && var != 41 && (!kDevBuild || (var != 56 && var != 57 && var != 95))))
    return hipErrorNotSupported;
  using G = v2::Geo<13, 4, 4>;
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  LftArgs<float> c = a;
  c.cond = opt(HOP_OPT_FORCE_HANDOVER) ? 2 : 0;
#ifdef HOP_DEV
  if (var == 56 || var == 57)  // the predict on the f32 matrix cores (SchedCondMfma)
    hipLaunchKernelGGL((v2::lft_cond_kernel<v2::SchedCondMfma, 13, 4, float>),
                       dim3((unsigned)blocks), dim3(256), (size_t)(G::WAVE_BYTES * kWavesPerBlock),
                       stream, c);
  else
#endif
#ifdef HOP_DEV
  if (var == 95)  // plain converting reads (the round-2 fp32-block kernel, A/B)
    hipLaunchKernelGGL((v2::lft_cond_kernel<v2::SchedCond, 13, 4, float>), dim3((unsigned)blocks),
                       dim3(256), (size_t)(G::WAVE_BYTES * kWavesPerBlock), stream, c);
  else
#endif
  // QT / A / B reads under the two sweeps (SchedCondL: the fp64 default's placement)
  hipLaunchKernelGGL((v2::lft_cond_kernel<v2::SchedCondL, 13, 4, float>), dim3((unsigned)blocks),
                     dim3(256), (size_t)(G::WAVE_BYTES * kWavesPerBlock), stream, c);
  if (var == 41 || var == 57 || opt(HOP_OPT_NO_RERUN)) return hipGetLastError();
  LftArgs<float> r = a;
  r.cond = 1;
  return dispatch_lft<float>(r, stream);
}
}  // namespace hop

// Diagnostic (not part of include/hop.h): read (and optionally reset) the
// section stamps of the stamped variants (developer builds).
extern "C" int hop_debug_stamps(unsigned long long* host16, int reset) {
  if (hipMemcpyFromSymbol(host16, HIP_SYMBOL(hop::v2::g_hop_stamp),
                          16 * sizeof(unsigned long long)) != hipSuccess)
    return -3;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hop::v2::g_hop_stamp), z, sizeof(z)) != hipSuccess) return -3;
  }
  return 0;
}
