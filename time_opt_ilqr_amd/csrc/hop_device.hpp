// Device primitives of the MI355X (gfx950) horizon-selection engine.
//
// Data layout ("row groups"): a wave64 holds FOUR independent problems, one per
// 16-lane DPP row.  Inside a row, lane c holds column c of every small matrix
// (register i = row i), so an S x S matrix costs S registers per lane.  A
// product X*Y or X^T*Y is a sequence of one-instruction broadcast-FMAs
// (v_fmac_f64_dpp ... row_newbcast:L, see dpp_blocks.inc): the broadcast lane
// picks the contraction index, the register picks the output row.  No LDS
// traffic and no MFMA padding waste (s = 13 runs 13 of 16 lanes, 13 registers).
// LDS is used only for transposes / symmetrisation (one 16x17 tile per problem).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>

#include "dpp_blocks.inc"
#include "lu_pivot.hpp"
#include "wrap.hpp"

// Opening pad of every inline-asm statement that issues a VMEM instruction reading an
// SGPR operand (the LDS-DMA statements): three wait states, so that no descriptor /
// soffset SGPR is read within five wait states of a VALU write of it (v_readlane /
// v_readfirstlane just before the statement; hipcc pads only its own pairs).  Marked
// "vmnop": the build drops each one the compiled code around it makes unnecessary
// (tools/nop_elide.py) and checks the result (tools/check_dpp_hazards.py).
#define HOP_VMNOP "s_nop 2 ; vmnop\n\t"

namespace hop {

constexpr int kRowLanes = 16;     // lanes per problem
constexpr int kProbPerWave = 4;   // problems per wave64
constexpr int kWavesPerBlock = 4; // 256-thread workgroups
constexpr int kProbPerBlock = kProbPerWave * kWavesPerBlock;
constexpr int kLdsRow = 17;       // padded LDS row (elements)
constexpr int kLdsTile = 272;     // 16*17; == 16 (mod 32) -> conflict-free b64 transposed reads

// status bits (include/hop.h)
constexpr unsigned ST_JITTER = 1u, ST_LU = 2u, ST_NONFINITE = 4u, ST_FAIL = 8u;
// internal: the conditioned-prefix kernel hands the problem to the rerun launch
constexpr unsigned ST_RERUN = 16u;

template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
  }(std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class T, int S>
__device__ __forceinline__ void zero(T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) x[i] = T(0);
}
template <class T, int S>
__device__ __forceinline__ void copy(T (&d)[S], const T (&s)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) d[i] = s[i];
}

// out[i] (+/-)= sum_{j<K} X[i][j] * Y[j][c]   (X: lanes 0..K-1 hold its columns)
template <bool NEG, class T, int S, int K>
__device__ __forceinline__ void acc_xy(T (&out)[S], const T (&x)[S], const T (&y)[K]) {
  static_for<K>([&](auto J) {
    if constexpr (NEG) RowB<S>::template fma_neg<J>(out, x, y[J]);
    else RowB<S>::template fma<J>(out, x, y[J]);
  });
}

// out[i] (+/-)= sum_{j<K} X[j][i] * Y[j][c]   (X: lanes 0..S-1 hold its columns, K rows)
template <bool NEG, class T, int S, int K>
__device__ __forceinline__ void acc_xty(T (&out)[S], const T (&x)[K], const T (&y)[K]) {
  static_for<K>([&](auto J) {
    if constexpr (NEG) LaneB<S>::fma_neg(out, x[J], y[J]);
    else LaneB<S>::fma(out, x[J], y[J]);
  });
}

// ---------------------------------------------------------------------------
// LDS transposes (per-problem tile, row stride 17)
// ---------------------------------------------------------------------------
template <class T, int S>
__device__ __forceinline__ void lds_put(T* tile, int c, const T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) tile[i * kLdsRow + c] = x[i];
}
template <class T, int S>
__device__ __forceinline__ void lds_get(const T* tile, int c, T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) x[i] = tile[i * kLdsRow + c];
}
template <class T, int S>
__device__ __forceinline__ void lds_get_t(const T* tile, int c, T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) x[i] = tile[c * kLdsRow + i];
}
// x <- 0.5 (x + x^T)  (bitwise symmetric, same rounding as NumPy's 0.5*(A+A.T))
template <class T, int S>
__device__ __forceinline__ void symmetrize(T (&x)[S], T* tile, int c) {
  lds_put(tile, c, x);
  wave_sync();
  T t[S];
  lds_get_t(tile, c, t);
  wave_sync();
#pragma unroll
  for (int i = 0; i < S; ++i) x[i] = T(0.5) * (x[i] + t[i]);
}
template <class T, int S>
__device__ __forceinline__ void transpose(T (&dst)[S], const T (&src)[S], T* tile, int c) {
  lds_put(tile, c, src);
  wave_sync();
  lds_get_t(tile, c, dst);
  wave_sync();
}

// Sum over the 16 lanes of a row by a row_ror butterfly of 32-bit DPP moves
// (fp64 DPP allows only row_newbcast): no LDS round trips, 4 dependent adds.
// Lanes may differ in the last bit (each sums in its own order): use the value
// of one lane only.
template <int ROR>
__device__ __forceinline__ double ror_row(double v) {
  // a rotation within the row reads only enabled lanes, so no "old" value is ever
  // kept: mov_dpp (undefined old) spares the zero fill update_dpp(0, ...) costs
  const int2 w = __builtin_bit_cast(int2, v);
  const int lo = __builtin_amdgcn_mov_dpp(w.x, 0x120 + ROR, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(w.y, 0x120 + ROR, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_int2(lo, hi));
}
template <int ROR>
__device__ __forceinline__ float ror_row(float v) {
  const int w = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, w, 0x120 + ROR, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum_dpp(float v) {
  v += ror_row<8>(v);
  v += ror_row<4>(v);
  v += ror_row<2>(v);
  v += ror_row<1>(v);
  return v;
}
__device__ __forceinline__ double row_sum_dpp(double v) {
  v += ror_row<8>(v);
  v += ror_row<4>(v);
  v += ror_row<2>(v);
  v += ror_row<1>(v);
  return v;
}

// Sum of lanes [0, N) of x, on every lane of the row: N DPP broadcast FMAs against
// 1.0 (the reference's float(e @ (Q @ e)) style reductions).  fp64 DPP has only
// row_newbcast on gfx950, so the rotate-and-add butterfly (row_sum_dpp) costs two
// 32-bit DPP moves, their zero fills and an add per stage: 20 instructions against
// N + 1 here.
template <int N>
__device__ __forceinline__ double lane_sum(double x) {
  double acc = 0.0, one[N];
#pragma unroll
  for (int j = 0; j < N; ++j) one[j] = 1.0;
  LaneDot<N>::fma(acc, x, one);
  return acc;
}
// Sum over the 16 lanes of a row (every lane of the row gets the total).
template <class T>
__device__ __forceinline__ T row_sum(T v) {
  v += __shfl_xor(v, 8, 16);
  v += __shfl_xor(v, 4, 16);
  v += __shfl_xor(v, 2, 16);
  v += __shfl_xor(v, 1, 16);
  return v;
}

// ---------------------------------------------------------------------------
// SPD inverse with the reference's jitter semantics (utils.py:69-93):
//   out = (sym(in) + eps I)^{-1}, eps = 1e-9, x10 per failed factorisation,
//   up to max_tries, then one unguarded elimination (the LU-fallback slot).
// Gauss-Jordan "sweep" on column-per-lane data: pivot p broadcasts column p
// (lane p) and uses row p from the lane's own register p.  A pivot d <= 0 (or
// NaN) is exactly the condition under which LAPACK's potrf rejects (its
// pivots are the same Schur complements).  The caller passes a symmetric
// matrix (symmetrize() first).
// ---------------------------------------------------------------------------
// 1/d as v_rcp + one Newton step (the IEEE division sequence is ~10 dependent
// instructions); d <= 0 / NaN pivots are rejected by the caller's test anyway
__device__ __forceinline__ double recip_nr(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
}
__device__ __forceinline__ float recip_nr(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  return __builtin_fmaf(r, __builtin_fmaf(-d, r, 1.0f), r);
}

// One pivot of the symmetric sweep operator on (M + eps I) (Goodnight):
//   a_pp <- -1/d,  a_pc <- a_pc/d,  a_ip <- a_ip/d,  a_ic <- a_ic - a_ip a_pc/d,
// d = a_pp + eps.  Row p and column p are scaled by their own multiply instead of
// riding in the rank-1 update with a -e_p offset: the offset form computes
// a_ip/d as a_ip (1 - (d-1)/d), which cancels to ~1e-16 d relative accuracy and
// broke problems whose blocks reach 1e8 (cart-pole's zero angle weight gives
// E_k = (Q_k + 1e-9 I)^-1 entries of 5e8).
template <int p, class T, int S>
__device__ __forceinline__ void sweep_pivot(T (&r)[S], T eps, int c, bool& ok) {
  const T d = bcast<p>(r[p]) + eps;
  ok = ok && (d > T(0));
  const T rd = recip_nr(d);
  const bool piv = (c == p);
  const T sc = piv ? T(0) : -r[p] * rd;  // -a_pc/d off the pivot lane
  const T rowp = piv ? -rd : r[p] * rd;
  RowB<S>::template sweep<p>(r, sc);     // a_ic -= a_ip a_pc/d (lane p untouched)
  const T f = piv ? rd : T(1);
#pragma unroll
  for (int i = 0; i < S; ++i) r[i] *= f;  // column p: a_ip/d
  r[p] = rowp;
}

template <class T, int S>
__device__ __forceinline__ void sweep_neg_inverse(T (&r)[S], T eps, int c, bool& ok) {
  static_for<S>([&](auto P) {
    constexpr int p = P;
    sweep_pivot<p>(r, eps, c, ok);
  });
}

// In place: r <- (sym(r) + eps I)^{-1}.  The unsymmetrised input is parked in
// the problem's LDS tile, so a retry (rare) re-forms sym(r) from LDS instead of
// keeping a second register copy.  Rows that already succeeded redo the same
// sweep with the same eps (bitwise identical), so no per-row select is needed.
template <class T, int S>
__device__ __forceinline__ void sym_spd_inverse(T (&r)[S], T* tile, int c, int max_tries,
                                                unsigned& st) {
  lds_put(tile, c, r);
  wave_sync();
  {
    T t[S];
    lds_get_t(tile, c, t);
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = T(0.5) * (r[i] + t[i]);
  }
  T eps = T(1e-9);
  int tries = 0;
  bool done = false, nf = false, lu = false;
#pragma unroll 1
  while (true) {
    bool ok = true;
    sweep_neg_inverse(r, eps, c, ok);
    if (tries == 0 && __any(!ok)) {
      // chol_inv's _assert_finite (utils.py:77): a non-finite input never
      // factors; no ladder for its row, the result is NaN with ST_NONFINITE
      T z = T(0);
      if (c < S) {
#pragma unroll
        for (int i = 0; i < S; ++i) z = z + tile[i * kLdsRow + c] * T(0);
      }
      const unsigned long long m = __ballot(!(z == z));
      nf = !ok && ((m >> (16 * ((threadIdx.x & 63) >> 4))) & 0xffffull) != 0ull;
      if (nf) st |= ST_NONFINITE;
    }
    const bool last = tries >= max_tries;
    if (!done && !ok && !nf && last) {
      st |= ST_LU;
      lu = true;
    }
    done = ok || last || nf;
    if (!__any(!done)) break;
    if (!done) {
      eps *= T(10);
      ++tries;
      st |= ST_JITTER;
    }
    T t[S];
    lds_get_t(tile, c, t);
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = T(0.5) * (tile[i * kLdsRow + c] + t[i]);
  }
  if (__any(lu)) {  // the LU slot (utils.py:88-93): column c of solve(sym(A) + eps I, I)
    if (lu) {
      T x[S];
#pragma unroll
      for (int i = 0; i < S; ++i) x[i] = (i == c) ? T(1) : T(0);
      const bool okl = lu_lds_solve<T>(tile, kLdsRow, S, T(0), eps, x) == 0;
#pragma unroll
      for (int i = 0; i < S; ++i) r[i] = okl ? -x[i] : T(__builtin_nan(""));
    }
  }
  wave_sync();
#pragma unroll
  for (int i = 0; i < S; ++i) r[i] = nf ? T(__builtin_nan("")) : -r[i];
}

// Same, without the LU slot (utils.py:96-120 chol_solve): returns false when
// every jitter failed (the reference raises LinAlgError).  Input must already
// be symmetric; it is parked in the LDS tile for retries.
template <class T, int S>
__device__ __forceinline__ bool spd_inverse_nofallback(T (&r)[S], T* tile, int c, int max_tries,
                                                       unsigned& st) {
  lds_put(tile, c, r);
  wave_sync();
  T eps = T(1e-9);
  int tries = 0;
  bool done = false, good = false;
#pragma unroll 1
  while (true) {
    bool ok = true;
    sweep_neg_inverse(r, eps, c, ok);
    ++tries;
    good = ok;
    done = ok || (tries >= max_tries);
    if (!__any(!done)) break;
    if (!done) {
      eps *= T(10);
      st |= ST_JITTER;
    }
#pragma unroll
    for (int i = 0; i < S; ++i) r[i] = tile[i * kLdsRow + c];
  }
  wave_sync();
#pragma unroll
  for (int i = 0; i < S; ++i) r[i] = -r[i];
  return good;
}

// Two independent sweeps interleaved pivot by pivot (their dependent chains
// hide each other's latency): r1 with eps1, r2 with eps2.
template <class T, int S>
__device__ __forceinline__ void sweep_neg_inverse2(T (&r1)[S], T eps1, bool& ok1, T (&r2)[S],
                                                   T eps2, bool& ok2, int c) {
  static_for<S>([&](auto P) {
    constexpr int p = P;
    sweep_pivot<p>(r1, eps1, c, ok1);
    sweep_pivot<p>(r2, eps2, c, ok2);
  });
}

// backward_pass_truncated's solve (solver.py:211-219): is sym(Quu)+lam I PD
// without jitter (np.linalg.cholesky, ok0), and its chol_solve inverse with the
// jitter ladder (spd_inverse_nofallback semantics).  The two first attempts run
// interleaved; retries (rare) as spd_inverse_nofallback.
template <class T, int S>
__device__ __forceinline__ bool spd_inverse_nofallback_chk(T (&r)[S], T* tile, int c,
                                                           int max_tries, unsigned& st,
                                                           bool& ok0) {
  lds_put(tile, c, r);
  T chk[S];
#pragma unroll
  for (int i = 0; i < S; ++i) chk[i] = r[i];
  bool ok = true;
  ok0 = true;
  T eps = T(1e-9);
  sweep_neg_inverse2(chk, T(0), ok0, r, eps, ok, c);
  int tries = 1;
  bool good = ok, done = ok || (tries >= max_tries);
  if (__any(!done)) {
    wave_sync();
#pragma unroll 1
    while (true) {
      if (!done) {
        eps *= T(10);
        st |= ST_JITTER;
      }
#pragma unroll
      for (int i = 0; i < S; ++i) r[i] = tile[i * kLdsRow + c];
      ok = true;
      sweep_neg_inverse(r, eps, c, ok);
      ++tries;
      good = ok;
      done = ok || (tries >= max_tries);
      if (!__any(!done)) break;
    }
  }
  wave_sync();
#pragma unroll
  for (int i = 0; i < S; ++i) r[i] = -r[i];
  return good;
}

__device__ __forceinline__ bool finite_val(double x) { return __builtin_isfinite(x); }
__device__ __forceinline__ bool finite_val(float x) { return __builtin_isfinite(x); }

}  // namespace hop
