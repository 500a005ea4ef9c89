// Batched Riccati backward passes producing the feedback gains K_k, k_k and the
// value expansion V_k, one problem per 16-lane row (hop_device.hpp layout).
//   mode 0 = backward_pass_truncated        (solver.py:156-230)
//   mode 1 = value_expansions_and_gains_prefix (horizon_selection.py:97-212)
// Per step the Q-function assembly (Qx, Qu, Qxx, Quu, Qux), the regularised
// Quu solve (jitter / LM escalation semantics of utils.chol_solve and the
// reference loops) and the value update are fused; vectors live one entry per
// lane, matrices one column per lane.  Each problem runs its own horizon
// (horizon[b] = T* for mode 0, T_bar + S_right for mode 1).
#include <math.h>

#include "hop_device.hpp"
#include "hop_kernels.hpp"

namespace hop {

// Loads at clamped (always valid) addresses first, then the padding selects: a
// load under a lane condition becomes an exec-masked branch with its own wait.
template <class T, int S>
__device__ __forceinline__ void rload_col(const T* M, int rows, int cols, int c, T pad, T (&x)[S]) {
  // column c of a rows x cols row-major matrix, identity(pad)/zero padded
  const int cc = c < cols ? c : cols - 1;
#pragma unroll
  for (int i = 0; i < S; ++i) x[i] = M[(i < rows ? i : rows - 1) * cols + cc];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const bool in = (i < rows) && (c < cols);
    x[i] = in ? x[i] : ((i == c) ? pad : T(0));
  }
}
template <class T, int S>
__device__ __forceinline__ void rload_row(const T* M, int rows, int cols, int c, T pad, T (&x)[S]) {
  // row c of a rows x cols row-major matrix
  const int cr = c < rows ? c : rows - 1;
#pragma unroll
  for (int j = 0; j < S; ++j) x[j] = M[cr * cols + (j < cols ? j : cols - 1)];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const bool in = (c < rows) && (j < cols);
    x[j] = in ? x[j] : ((j == c) ? pad : T(0));
  }
}

// section stamps of the diagnostic instantiation (tools/stamps_riccati.py)
__device__ unsigned long long g_ric_stamp[16];

// The legacy chol_solve's last resort (ilqr_propagator.py:43): np.linalg.lstsq(A, B)
// of the symmetric A = Quu_reg is the minimum-norm solution pinv(A) B, and
// pinv(A) = V diag(1/lambda_k) V^T over the eigenpairs with |lambda_k| > rcond
// max|lambda| (gelsd's cutoff, rcond = eps * m: the singular values of a symmetric
// matrix are |lambda_k|).  Rare path, one lane per problem: cyclic Jacobi on A
// parked in the problem's tile (A at [0, m^2), V at [m^2, 2 m^2), m <= 11), then
// lane c forms column c of pinv(A).  need: this row takes the fallback.
template <class T, int MM>
__device__ __forceinline__ bool legacy_pinv(T (&Qi)[MM], const T (&A)[MM], T* tile, int c, int m,
                                            bool need) {
  const bool fits = 2 * m * m <= kLdsTile;
  wave_sync();
  if (need && fits && c < m) {
#pragma unroll
    for (int r = 0; r < MM; ++r)
      if (r < m) tile[r * m + c] = A[r];
  }
  wave_sync();
  T* a = tile;
  T* v = tile + m * m;
  if (need && fits && c == 0) {
    for (int i = 0; i < m * m; ++i) v[i] = T(0);
    for (int i = 0; i < m; ++i) v[i * m + i] = T(1);
    for (int sweep = 0; sweep < 64; ++sweep) {
      T off = T(0), tot = T(0);
      for (int p = 0; p < m; ++p)
        for (int q = 0; q < m; ++q) {
          const T x = a[p * m + q] * a[p * m + q];
          tot += x;
          if (p != q) off += x;
        }
      if (!(off > T(1e-60) * tot) || !(tot == tot)) break;
      for (int p = 0; p < m - 1; ++p)
        for (int q = p + 1; q < m; ++q) {
          const T apq = a[p * m + q];
          if (apq == T(0)) continue;
          const T theta = (a[q * m + q] - a[p * m + p]) / (T(2) * apq);
          T t = T(1) / (fabs(theta) + sqrt(theta * theta + T(1)));
          if (theta < T(0)) t = -t;
          const T cs = T(1) / sqrt(t * t + T(1)), sn = t * cs;
          for (int k = 0; k < m; ++k) {  // A <- A J (columns p, q)
            const T akp = a[k * m + p], akq = a[k * m + q];
            a[k * m + p] = cs * akp - sn * akq;
            a[k * m + q] = sn * akp + cs * akq;
          }
          for (int k = 0; k < m; ++k) {  // A <- J^T A (rows p, q)
            const T apk = a[p * m + k], aqk = a[q * m + k];
            a[p * m + k] = cs * apk - sn * aqk;
            a[q * m + k] = sn * apk + cs * aqk;
          }
          a[p * m + q] = T(0);
          a[q * m + p] = T(0);
          for (int k = 0; k < m; ++k) {  // V <- V J
            const T vkp = v[k * m + p], vkq = v[k * m + q];
            v[k * m + p] = cs * vkp - sn * vkq;
            v[k * m + q] = sn * vkp + cs * vkq;
          }
        }
    }
  }
  wave_sync();
  bool finite = true;
  if (need && fits) {
    T lmax = T(0);
    for (int k = 0; k < m; ++k) lmax = fmax(lmax, fabs(a[k * m + k]));
    const T cut = T(sizeof(T) == 8 ? 2.220446049250313e-16 : 1.1920929e-07) * T(m) * lmax;
    const int cc = c < m ? c : 0;
#pragma unroll
    for (int r = 0; r < MM; ++r) {
      T acc = T(0);
      if (r < m && c < m)
        for (int k = 0; k < m; ++k) {
          const T lk = a[k * m + k];
          if (fabs(lk) > cut) acc += v[r * m + k] * v[cc * m + k] / lk;
        }
      Qi[r] = acc;
      finite = finite && (acc == acc) && (acc - acc == T(0));
    }
  }
  wave_sync();
  return fits && finite;
}

// One pass of problem block blk; JCK: the J-curve form at horizon jl for the whole wave.
template <class T, int S, int MM, bool STAMP, bool JCK, int MODE>
__device__ __forceinline__ void riccati_body(const RiccatiArgs<T>& a, long long blk, int jl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* smem = reinterpret_cast<T*>(smem_raw);
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4, w = tid >> 6;
  constexpr bool JC = JCK;
  const long long prob = (blk * kWavesPerBlock + w) * kProbPerWave + g;
  const bool valid = prob < a.batch;
  const long long pb = valid ? prob : a.batch - 1;
  T* tile = smem + (w * kProbPerWave + g) * kLdsTile;
  // the problem's stage weight Q, loop-invariant, lives in a second LDS tile:
  // held in registers it was re-loaded from HBM every step under register pressure
  T* qt = smem + (kProbPerBlock + w * kProbPerWave + g) * kLdsTile;
#pragma unroll 1
  for (int i = c; i < kLdsTile; i += kRowLanes) {
    tile[i] = T(0);
    qt[i] = T(0);
  }
  wave_sync();

  const int n = a.n, m = a.m, NA = a.nalloc;
  constexpr int mode = MODE;  // a.mode, as a template argument (each mode compiles alone)
  const long long nn = (long long)n * n, nm = (long long)n * m, mmx = (long long)m * m;
  const T* Ap = a.A + pb * NA * nn;
  const T* Bp = a.Bm + pb * NA * nm;
  const T* Xp = a.X + pb * (NA + 1) * n;
  const T* Up = a.U + pb * NA * m;
  const T* xgp = a.xg + pb * a.xg_bstride;
  const T* urp = a.u_ref + pb * a.uref_bstride;
  const T* Qp = a.Q + pb * a.q_bstride;
  const T* Rp = a.R + pb * a.r_bstride;
  const T* Qfp = a.Qf + pb * a.qf_bstride;
  const int L = valid ? (JC ? jl : a.horizon[pb]) : 0;
  int Lw = L;
  Lw = max(Lw, __shfl_xor(Lw, 16));
  Lw = max(Lw, __shfl_xor(Lw, 32));
  Lw = __builtin_amdgcn_readfirstlane(Lw);
  const T lam0 = JC ? a.lm_value : a.lm[pb];
  unsigned long long sec[10] = {};
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

  // loop-invariant cost blocks
  {
    T qcol[S];
    rload_col(Qp, n, n, c, T(0), qcol);
    lds_put(qt, c, qcol);  // qt[i][c] = Q[i][c]
  }
  T rcol[MM], rrow[MM];
  rload_col(Rp, m, m, c, T(1), rcol);
  rload_row(Rp, m, m, c, T(1), rrow);
  const T xg_c = (c < n) ? xgp[c < n ? c : 0] : T(0);
  const T ur_c = (c < m) ? urp[c < m ? c : 0] : T(0);
  const bool wrap_c = (c < n) && ((a.wrap_mask >> c) & 1u);

  unsigned st = 0;
  bool alive = valid && L > 0 && L <= NA;
  if (valid && !(L > 0 && L <= NA)) st |= ST_FAIL;

  // terminal: Vxx = sym(Qf), Vx = Qf eT, V0 = 1/2 eT' Qf eT
  T Vxx[S];
  rload_col(Qfp, n, n, c, T(0), Vxx);
  T vx, v0;
  {
    T qfrow[S];
    rload_row(Qfp, n, n, c, T(0), qfrow);
    const int iT = (L > 0 && L <= NA) ? L : 0;
    T eT = (c < n) ? Xp[(long long)iT * n + (c < n ? c : 0)] - xg_c : T(0);
    if (wrap_c) eT = wrap_angle(eT);
    const bool fin = ((__ballot(!finite_val(eT)) >> (16 * g)) & 0xffffull) == 0ull;
    if (!fin && !a.legacy) {  // the legacy loops check nothing: NaN propagates
      st |= ST_NONFINITE | ST_FAIL;
      alive = false;
    }
    vx = T(0);
    LaneDot<S>::fma(vx, eT, qfrow);  // (Qf eT)[c]
    v0 = T(0.5) * row_sum_dpp((c < n) ? eT * vx : T(0));
    symmetrize(Vxx, tile, c);
    if (alive) {
      if (a.Vxx) {
        T* o = a.Vxx + (pb * (NA + 1) + L) * nn;
#pragma unroll
        for (int i = 0; i < S; ++i)
          if (i < n && c < n) o[i * n + c] = Vxx[i];
      }
      if (a.Vx && c < n) a.Vx[pb * (NA + 1) * n + (long long)L * n + c] = vx;
      if (a.V0 && c == 0) a.V0[pb * (NA + 1) + L] = v0;
    }
  }

  // step i's A, B, x, u are loaded one step ahead (software pipeline): the
  // global-load latency of step i-1 hides behind step i's arithmetic.
  // MERGE (fp64, S + MM <= 16): B's columns ride on lanes S..S+m-1 of the same
  // registers as A's ("ab" = [A | B] column per lane), so Vxx [A|B], A^T Vxx [A|B]
  // and B^T Vxx [A|B] are three products instead of five, and one load per row.
  constexpr bool MERGE = sizeof(T) == 8 && S + MM <= kRowLanes;
  T acol_n[S], bcol_n[S], x_n, u_n;
  const bool lane_a = c < S, lane_in = c < S ? c < n : (c - S) < m;
  const int col_ab = c < S ? (c < n ? c : n - 1) : (c - S < m ? c - S : m - 1);
  auto load_step = [&](int i) {
    if constexpr (MERGE) {
      const T* base = lane_a ? Ap + (long long)i * nn + col_ab : Bp + (long long)i * nm + col_ab;
      const int ld = lane_a ? n : m;
#pragma unroll
      for (int j = 0; j < S; ++j) acol_n[j] = base[(j < n ? j : n - 1) * ld];
#pragma unroll
      for (int j = 0; j < S; ++j) acol_n[j] = (j < n && lane_in) ? acol_n[j] : T(0);
    } else {
      rload_col(Ap + (long long)i * nn, n, n, c, T(0), acol_n);
      rload_col(Bp + (long long)i * nm, n, m, c, T(0), bcol_n);  // lanes c < m: column c of B_i
    }
    x_n = Xp[(long long)i * n + (c < n ? c : 0)];
    u_n = Up[(long long)i * m + (c < m ? c : 0)];
  };
  if (Lw > 0) load_step(Lw - 1);
#pragma unroll 1
  for (int i = Lw - 1; i >= 0; --i) {
    stamp(-1);
    const bool act = alive && (i < L);
    T e = (c < n) ? x_n - xg_c : T(0);
    if (wrap_c) e = wrap_angle(e);
    const T du = (c < m) ? u_n - ur_c : T(0);
    T acol[S], bcol[S];
    copy(acol, acol_n);
    if constexpr (!MERGE) copy(bcol, bcol_n);
    load_step(i > 0 ? i - 1 : 0);
    if (!__any(act)) continue;
    // the brute-force curve (solver.py:326-356) checks nothing itself: only its
    // chol_solve raises, so a non-finite e at t = 0 only feeds V_0 (inf/NaN in J)
    const bool e_ok = (JC && i == 0) || finite_val(e);
    const unsigned long long badm = __ballot(!(e_ok && finite_val(du)));
    const bool bad = !a.legacy && ((badm >> (16 * g)) & 0xffffull) != 0ull;

    stamp(0);
    // lx = Q e (+ cx), lu = R du, l0
    T lx = T(0), lu = T(0);
    {
      T qrow[S];
#pragma unroll
      for (int j = 0; j < S; ++j) qrow[j] = qt[c * kLdsRow + j];  // row c of Q
      LaneDot<S>::fma(lx, e, qrow);
    }
    LaneDot<MM>::fma(lu, du, rrow);
    T l0 = T(0.5) * row_sum_dpp((c < n) ? e * lx : T(0)) +
           T(0.5) * row_sum_dpp((c < m) ? du * lu : T(0)) + a.w_stage;
    T qst[S];
#pragma unroll
    for (int i = 0; i < S; ++i) qst[i] = qt[i * kLdsRow + c];  // column c of Q
    if (a.qx_extra) {  // wave-uniform branch; the load itself must not become a
                       // lane-divergent one (its join would wait on every
                       // outstanding load, the prefetch included)
      const T* xp = a.qx_extra + (pb * NA + i) * n;
      T v = xp[c < n ? c : 0];
      asm volatile("" : "+v"(v));
      lx += (c < n) ? v : T(0);
    }
    if (a.c_extra) l0 += a.c_extra[pb * NA + i];
    if (a.qxx_extra) {
      T ex[S];
      rload_col(a.qxx_extra + (pb * NA + i) * nn, n, n, c, T(0), ex);
#pragma unroll
      for (int r = 0; r < S; ++r) qst[r] += ex[r];
      symmetrize(qst, tile, c);
    }

    stamp(1);
    // Q-function assembly
    T qx = lx, qu = lu;
    T VA[S], Qxx[S], Quu[MM], Qux[MM];
    copy(Qxx, qst);
    if constexpr (MERGE) {
      T qab = T(0);
      LaneDot<S>::fma(qab, vx, acol);  // lanes < S: A^T Vx; lanes S..: B^T Vx
      qx += qab;                       // Qx = lx + A^T Vx
      qu += ror_row<kRowLanes - S>(qab);  // Qu = lu + B^T Vx, moved to lanes 0..m-1
      zero(VA);
      acc_xy<false>(VA, Vxx, acol);    // Vxx [A | B]
      acc_xty<false>(Qxx, acol, VA);   // Qst + A^T Vxx A   (lanes < S)
      T QB[MM];
      zero(QB);
      static_for<S>([&](auto J) { LaneBOff<MM, S>::fma(QB, acol[J], VA[J]); });  // B^T Vxx [A|B]
#pragma unroll
      for (int r = 0; r < MM; ++r) {
        Qux[r] = QB[r];                                        // lanes < n: B^T Vxx A
        Quu[r] = rcol[r] + ror_row<kRowLanes - S>(QB[r]);      // R + B^T Vxx B, lanes < m
      }
    } else {
      LaneDot<S>::fma(qx, vx, acol);  // Qx = lx + A^T Vx
      LaneDot<S>::fma(qu, vx, bcol);  // Qu = lu + B^T Vx   (lanes < m)
      zero(VA);
      acc_xy<false>(VA, Vxx, acol);   // Vxx A
      T VB[S];
      zero(VB);
      acc_xy<false>(VB, Vxx, bcol);   // Vxx B          (lanes < m)
      acc_xty<false>(Qxx, acol, VA);  // Qst + A^T Vxx A
      copy(Quu, rcol);
      acc_xty<false, T, MM, S>(Quu, bcol, VB);  // R + B^T Vxx B   (lanes < m)
      zero(Qux);
      acc_xty<false, T, MM, S>(Qux, bcol, VA);  // B^T Vxx A       (lanes < n)
    }

    // regularised solve: Quu_reg = sym(Quu) + lam I ; (Quu_reg + eps I)^-1
    stamp(2);
    T QuuT[MM];
    transpose(QuuT, Quu, tile, c);
    T Qi[MM];
    stamp(3);
    bool solved = false;
    if constexpr (mode == 0) {
#pragma unroll
      for (int r = 0; r < MM; ++r) Qi[r] = T(0.5) * (Quu[r] + QuuT[r]) + ((c == r) ? lam0 : T(0));
      // the reference first checks cholesky(Quu_reg) (no jitter), then solves with jitter
      bool ok = true;
      solved = spd_inverse_nofallback_chk(Qi, tile, c, 8, st, ok) && ok;
    } else if (a.legacy) {
      // legacy chol_solve (ilqr_propagator.py:33-43) on Quu_reg = _sym(Quu) + lm I:
      // 4 jitters, then lstsq (a non-finite Quu_reg: lstsq raises, the row fails)
      T Qs[MM];
#pragma unroll
      for (int r = 0; r < MM; ++r) Qs[r] = T(0.5) * (Quu[r] + QuuT[r]) + ((c == r) ? lam0 : T(0));
      copy(Qi, Qs);
      const bool okr = spd_inverse_nofallback(Qi, tile, c, 4, st);
      solved = okr;
      const bool need = act && !okr;
      if (__any(need)) {
        T z = T(0);
#pragma unroll
        for (int r = 0; r < MM; ++r) z = z + Qs[r] * T(0);
        const unsigned long long nm = __ballot(!(z == z) && c < m);
        const bool nonfin = ((nm >> (16 * g)) & 0xffffull) != 0ull;
        T P[MM];
        const bool okp = legacy_pinv<T, MM>(P, Qs, tile, c, m, need && !nonfin);
        if (need && !nonfin) {
#pragma unroll
          for (int r = 0; r < MM; ++r) Qi[r] = P[r];
          st |= ST_LU;
          solved = okp;
        }
        if (need && nonfin) st |= ST_NONFINITE;
      }
    } else {
      T lam = lam0 > T(1e-12) ? lam0 : T(1e-12);
      int tries = 0;
      bool done = false;
#pragma unroll 1
      while (true) {
#pragma unroll
        for (int r = 0; r < MM; ++r) Qi[r] = T(0.5) * (Quu[r] + QuuT[r]) + ((c == r) ? lam : T(0));
        const bool okr = spd_inverse_nofallback(Qi, tile, c, 8, st);
        ++tries;
        solved = okr;
        done = okr || tries >= a.reg_max_tries;
        if (!__any(!done && act)) break;
        if (!done) lam *= T(10);
      }
    }
    const bool fail_row = act && (bad || !solved);

    stamp(4);
    // gains
    T K[MM];
    zero(K);
    acc_xy<true, T, MM, MM>(K, Qi, Qux);  // K = -Quu_reg^-1 Qux   (column c)
    T kv = T(0);
    LaneDot<MM>::fma_neg(kv, qu, Qi);     // k = -Quu_reg^-1 Qu    (lanes < m)

    stamp(5);
    // value update
    T Vn[S];
    copy(Vn, Qxx);
    T vxn = qx;
    T v0n = v0;
    if constexpr (mode == 0) {
      LaneDot<MM>::fma(vxn, qu, K);        // + K^T Qu
      LaneDot<MM>::fma(vxn, kv, Qux);      // + Qux^T k
      T qk = T(0);
      LaneDot<MM>::fma(qk, kv, QuuT);      // (Quu k)[c]
      LaneDot<MM>::fma(vxn, qk, K);        // + K^T Quu k
      // K^T Qux + Qux^T K + K^T Quu K = K^T (Qux + Quu K) + Qux^T K (one product fewer)
      T QK[MM];
      copy(QK, Qux);
      acc_xy<false, T, MM, MM>(QK, Quu, K);  // Qux + Quu K
      acc_xty<false, T, S, MM>(Vn, K, QK);   // + K^T (Qux + Quu K)
      acc_xty<false, T, S, MM>(Vn, Qux, K);  // + Qux^T K
    } else {
      acc_xty<false, T, S, MM>(Vn, Qux, K);  // Qxx - Qux^T Quu^-1 Qux
      LaneDot<MM>::fma(vxn, kv, Qux);        // Qx - Qux^T Quu^-1 Qu
      v0n = l0 + v0 + T(0.5) * row_sum_dpp((c < m) ? qu * kv : T(0));
    }
    stamp(6);
    symmetrize(Vn, tile, c);
    // value_expansions (horizon_selection.py:209-210) raises on any non-finite V.
    // The brute-force curve raises only through the next step's chol_solve: a
    // non-finite Vxx / Vx fails there, a non-finite V_0 never does, and at t = 0
    // nothing follows -- only chol_solve(Quu_reg, Qux) itself can raise (Qux).
    bool vbad = !a.legacy && (!finite_val(vxn) || (!JC && !finite_val(v0n)));
#pragma unroll
    for (int r = 0; r < S; ++r) vbad = vbad || (!a.legacy && !finite_val(Vn[r]));
    if (JC && i == 0 && !a.legacy) {
      vbad = false;
#pragma unroll
      for (int r = 0; r < MM; ++r) vbad = vbad || !finite_val(Qux[r]);
    }
    const unsigned long long vbm = __ballot(vbad && c < n);
    const bool vfail = act && (((vbm >> (16 * g)) & 0xffffull) != 0ull);

    stamp(7);
    const bool commit = act && !fail_row && !vfail;
    if (act && (fail_row || vfail)) {
      st |= ST_FAIL;
      if (bad || vfail) st |= ST_NONFINITE;
      alive = false;
    }
    if (commit) {
#pragma unroll
      for (int r = 0; r < S; ++r) Vxx[r] = Vn[r];
      vx = vxn;
      v0 = v0n;
      if (!JC) {
        T* Ko = a.K + (pb * NA + i) * (long long)m * n;
#pragma unroll
        for (int r = 0; r < MM; ++r)
          if (r < m && c < n) Ko[r * n + c] = K[r];
        if (c < m) a.k[(pb * NA + i) * m + c] = kv;
      }
      if (a.Vxx) {
        T* o = a.Vxx + (pb * (NA + 1) + i) * nn;
#pragma unroll
        for (int r = 0; r < S; ++r)
          if (r < n && c < n) o[r * n + c] = Vn[r];
      }
      if (a.Vx && c < n) a.Vx[pb * (NA + 1) * n + (long long)i * n + c] = vxn;
      if (a.V0 && c == 0) a.V0[pb * (NA + 1) + i] = v0n;
    }
    stamp(8);
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      for (int j = 0; j < 10; ++j) atomicAdd(&g_ric_stamp[j], sec[j]);
      atomicAdd(&g_ric_stamp[15], 1ull);
    }
  }
  if (valid && c == 0) {
    if (JC) {  // V_0 of this horizon's sweep (the reference raises on failure: NaN)
      const long long o = prob * a.jc_tmax + (L - 1);
      a.jc_J[o] = alive ? v0 : T(NAN);
      a.jc_status[o] = (int)st;
    } else {
      a.status[prob] = (int)st;
    }
  }
}

template <class T, int S, int MM, int MODE, bool STAMP = false>
__global__ __launch_bounds__(256, 1) void riccati_kernel(RiccatiArgs<T> a) {
  riccati_body<T, S, MM, STAMP, false, MODE>(a, (long long)blockIdx.x, 0);
}

// The J-curve form: workgroups [b * jc_tmax, (b+1) * jc_tmax) run problem block b at
// every horizon, longest first, so the re-reads of its A, B, x, u meet in the caches.
// (Pairing horizons jc_tmax - h and h + 1 in one workgroup, as the exact-size kernel
// does, measured 1.5x slower here: the two inlined passes double the live registers.)
// A kernel of its own, so the single-pass modes compile without the J-curve branches
// (measured 4-10 % faster on the generic shapes).
template <class T, int S, int MM>
__global__ __launch_bounds__(256, 1) void riccati_jcurve_kernel(RiccatiArgs<T> a) {
  const unsigned tm = (unsigned)a.jc_tmax;
  riccati_body<T, S, MM, false, true, 1>(a, (long long)(blockIdx.x / tm),
                                      a.jc_tmax - (int)(blockIdx.x % tm));
}

template <class T, int S, int MM>
hipError_t launch_riccati(const RiccatiArgs<T>& a, hipStream_t stream) {
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  const size_t lds = (size_t)2 * kProbPerBlock * kLdsTile * sizeof(T);
  if (a.jc_J) {
    hipLaunchKernelGGL((riccati_jcurve_kernel<T, S, MM>),
                       dim3((unsigned)(blocks * a.jc_tmax)), dim3(256), lds, stream, a);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)blocks);
#ifdef HOP_DEV
  if (opt(HOP_OPT_STAMPS)) {  // diagnostic: section stamps (tools/stamps_riccati.py)
    if (a.mode == 0)
      hipLaunchKernelGGL((riccati_kernel<T, S, MM, 0, true>), grid, dim3(256), lds, stream, a);
    else
      hipLaunchKernelGGL((riccati_kernel<T, S, MM, 1, true>), grid, dim3(256), lds, stream, a);
    return hipGetLastError();
  }
#endif
  if (a.mode == 0)
    hipLaunchKernelGGL((riccati_kernel<T, S, MM, 0>), grid, dim3(256), lds, stream, a);
  else
    hipLaunchKernelGGL((riccati_kernel<T, S, MM, 1>), grid, dim3(256), lds, stream, a);
  return hipGetLastError();
}

template <class T>
hipError_t dispatch_riccati(const RiccatiArgs<T>& a, hipStream_t stream) {
  if constexpr (sizeof(T) == 8) {
    if (!opt(HOP_OPT_FORCE_GENERIC) && !a.legacy) {  // (HOP_OPT_STAMPS: the fast kernel's own stamps)
      const hipError_t e = dispatch_riccati_fast(a, stream);
      if (e != hipErrorNotSupported) return e;
    }
  }
  if (a.m <= 4) {
    if (a.n <= 4) return launch_riccati<T, 4, 4>(a, stream);
    if (a.n <= 8) return launch_riccati<T, 8, 4>(a, stream);
    if (a.n <= 12) return launch_riccati<T, 12, 4>(a, stream);
    return launch_riccati<T, 16, 4>(a, stream);
  }
  return launch_riccati<T, 16, 16>(a, stream);
}

template hipError_t dispatch_riccati<double>(const RiccatiArgs<double>&, hipStream_t);
template hipError_t dispatch_riccati<float>(const RiccatiArgs<float>&, hipStream_t);

}  // namespace hop

// Diagnostic (not part of include/hop.h): read (and optionally reset) the Riccati
// section stamps (HOP_OPT_STAMPS, developer builds).
extern "C" int hop_debug_ric_stamps(unsigned long long* host16, int reset) {
  if (hipMemcpyFromSymbol(host16, HIP_SYMBOL(hop::g_ric_stamp), 16 * sizeof(unsigned long long)) !=
      hipSuccess)
    return -3;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(hop::g_ric_stamp), z, sizeof(z)) != hipSuccess) return -3;
  }
  return 0;
}
