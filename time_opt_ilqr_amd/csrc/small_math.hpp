// Per-problem LFT sweep math for small s (one problem per lane), shared by the
// GPU kernel (lft_small.hip) and a host build used by the CPU test suite
// (tests/test_host_cpu.py compiles it with g++ and checks it against the
// oracle), so the arithmetic the kernel runs is exercised without a GPU.
//
// Symmetric matrices (E, W, Ebar, Gbar, G, QT^-1, Wt, X0) are stored packed
// (upper triangle, s(s+1)/2 values): at s = 5 the live set fits in registers,
// the symmetric sweep operator does half the FLOPs of a Gauss-Jordan inverse,
// and symmetric products are formed on the upper triangle only.
// Reference: horizon_selection.py:36-86 (LFT), utils.py:35-37 (_sym),
// utils.py:69-93 (chol_inv jitter ladder).
#pragma once

#ifndef HOP_HD
#define HOP_HD __host__ __device__
#endif

#include "lu_pivot.hpp"
#include "../../include/hop.h"

namespace hop {
namespace small {

constexpr unsigned kStJitter = 1u, kStLu = 2u, kStNonfinite = 4u;

// small_recip(d) = 1/d is supplied by the includer: the GPU kernel uses
// v_rcp + one Newton step (lft_small.hip), the host test build exact division.

template <class T, int S>
struct Gen {
  T a[S][S];
};

template <class T, int S>
struct Sym {
  static constexpr int NP = S * (S + 1) / 2;
  T v[NP];
  static HOP_HD constexpr int idx(int i, int j) {  // i <= j
    return i * S - i * (i - 1) / 2 + (j - i);
  }
  HOP_HD T& at(int i, int j) { return i <= j ? v[idx(i, j)] : v[idx(j, i)]; }
  HOP_HD T at(int i, int j) const { return i <= j ? v[idx(i, j)] : v[idx(j, i)]; }
};

// _sym(M) of a general matrix
template <class T, int S>
HOP_HD inline void sym_of(Sym<T, S>& out, const Gen<T, S>& m) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = i; j < S; ++j) out.at(i, j) = T(0.5) * (m.a[i][j] + m.a[j][i]);
}

// Symmetric sweep operator on (M + eps I): after all pivots x = -(M + eps I)^-1.
// Pivots are the Cholesky squares, so "all > 0" is the potrf test.
template <class T, int S>
HOP_HD inline bool sweep_neg_inverse(Sym<T, S>& x, T eps) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < S; ++i) x.at(i, i) += eps;
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const T d = x.at(p, p);
    ok = ok && (d > T(0));
    const T r = small_recip(d);
#pragma unroll
    for (int i = 0; i < S; ++i) {
      if (i == p) continue;
      const T aip = x.at(i, p) * r;
#pragma unroll
      for (int j = i; j < S; ++j) {
        if (j == p) continue;
        x.at(i, j) -= aip * x.at(p, j);
      }
    }
#pragma unroll
    for (int i = 0; i < S; ++i)
      if (i != p) x.at(i, p) *= r;
    x.at(p, p) = -r;
  }
  return ok;
}

// every packed entry finite (x * 0 is 0 for finite x, NaN otherwise)
template <class T, int S>
HOP_HD inline bool all_finite(const Sym<T, S>& m) {
  T z = T(0);
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) z = z + m.v[k] * T(0);
  return z == z;
}

// chol_inv (utils.py:69-93) on an already symmetric input: jitter 1e-9, x10 per
// failure; after max_tries the last attempt is kept (LU slot) and flagged.
template <class T, int S>
HOP_HD inline void spd_inverse(Sym<T, S>& m, int max_tries, unsigned& st) {
  const Sym<T, S> in = m;
  T eps = T(1e-9);
  bool ok = sweep_neg_inverse(m, eps);
  if (!ok && !all_finite(in)) {
    // chol_inv's _assert_finite (utils.py:77): a non-finite input never factors;
    // no ladder, the result is NaN with the non-finite bit (oracle spd_inverse)
    st |= kStNonfinite;
#pragma unroll
    for (int k = 0; k < Sym<T, S>::NP; ++k) m.v[k] = T(__builtin_nan(""));
    return;
  }
  if (!ok) {
    st |= kStJitter;
    for (int tries = 1;; ++tries) {
      eps *= T(10);
      m = in;
      ok = sweep_neg_inverse(m, eps);
      if (ok) break;
      if (tries >= max_tries) {
        // the LU slot: np.linalg.solve(A + eps I, I), partial pivoting (lu_pivot.hpp)
        st |= kStLu;
        T inv[S][S];  // the identity's columns, solved together (one factorisation)
#pragma unroll
        for (int i = 0; i < S; ++i)
#pragma unroll
          for (int c = 0; c < S; ++c) inv[i][c] = i == c ? T(1) : T(0);
        const bool okl = lu_sym_solve_regs<T, S, S>([&](int i, int j) { return in.at(i, j); }, eps, inv);
#pragma unroll
        for (int i = 0; i < S; ++i)
#pragma unroll
          for (int j = i; j < S; ++j) m.at(i, j) = okl ? -inv[i][j] : T(__builtin_nan(""));
        break;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) m.v[k] = -m.v[k];
}

// z^T (X + eps I)^-1 z by LDL^T elimination, same ladder (X symmetric)
template <class T, int S>
HOP_HD inline T quad_inverse(const Sym<T, S>& x0, const T (&z)[S], int max_tries, unsigned& st) {
  T eps = T(1e-9);
  for (int tries = 0;; ++tries) {
    Sym<T, S> x = x0;
    T b[S];
#pragma unroll
    for (int i = 0; i < S; ++i) b[i] = z[i];
    T acc = T(0);
    bool ok = true;
#pragma unroll
    for (int p = 0; p < S; ++p) {
      const T d = x.at(p, p) + eps;
      ok = ok && (d > T(0));
      const T r = small_recip(d);
      acc += b[p] * b[p] * r;
#pragma unroll
      for (int i = p + 1; i < S; ++i) {
        const T l = x.at(i, p) * r;
        b[i] -= l * b[p];
#pragma unroll
        for (int j = i; j < S; ++j) x.at(i, j) -= l * x.at(p, j);
      }
    }
    if (ok) return acc;
    if (tries == 0) {  // a non-finite input runs no ladder (chol_inv's _assert_finite)
      T zz = T(0);
#pragma unroll
      for (int i = 0; i < S; ++i) zz = zz + z[i] * T(0);
      if (!all_finite(x0) || !(zz == zz)) {
        st |= kStNonfinite;
        return T(__builtin_nan(""));
      }
      st |= kStJitter;
    }
    if (tries >= max_tries) {  // the LU slot: z^T solve(X + eps I, z), partial pivoting
      st |= kStLu;
      T y[S][1];
#pragma unroll
      for (int i = 0; i < S; ++i) y[i][0] = z[i];
      if (!lu_sym_solve_regs<T, S, 1>([&](int i, int j) { return x0.at(i, j); }, eps, y))
        return T(__builtin_nan(""));
      T q = T(0);
#pragma unroll
      for (int i = 0; i < S; ++i) q += z[i] * y[i][0];
      return q;
    }
    eps *= T(10);
  }
}

// ---- products (G: general, Y: symmetric) --------------------------------
// out = S_ * G^T   (general)
template <class T, int S>
HOP_HD inline void mul_sym_gt(Gen<T, S>& out, const Sym<T, S>& s, const Gen<T, S>& g) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < S; ++l) v += s.at(i, l) * g.a[j][l];
      out.a[i][j] = v;
    }
}
// out = S_ * G   (general)
template <class T, int S>
HOP_HD inline void mul_sym_g(Gen<T, S>& out, const Sym<T, S>& s, const Gen<T, S>& g) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < S; ++l) v += s.at(i, l) * g.a[l][j];
      out.a[i][j] = v;
    }
}
// out = G1 * G2   (general)
template <class T, int S>
HOP_HD inline void mul_gg(Gen<T, S>& out, const Gen<T, S>& x, const Gen<T, S>& y) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < S; ++l) v += x.a[i][l] * y.a[l][j];
      out.a[i][j] = v;
    }
}
// acc (upper triangle) += sgn * X * Y   (X*Y symmetric in exact arithmetic)
template <bool NEG, class T, int S>
HOP_HD inline void acc_sym_xy(Sym<T, S>& acc, const Gen<T, S>& x, const Gen<T, S>& y) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = i; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < S; ++l) v += x.a[i][l] * y.a[l][j];
      acc.at(i, j) = NEG ? acc.at(i, j) - v : acc.at(i, j) + v;
    }
}
// acc (upper triangle) += sgn * X^T * Y
template <bool NEG, class T, int S>
HOP_HD inline void acc_sym_xty(Sym<T, S>& acc, const Gen<T, S>& x, const Gen<T, S>& y) {
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = i; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < S; ++l) v += x.a[l][i] * y.a[l][j];
      acc.at(i, j) = NEG ? acc.at(i, j) - v : acc.at(i, j) + v;
    }
}

// ---- one step of the sweep ------------------------------------------------
template <class T, int S, int MM>
struct State {
  Sym<T, S> Eb, Gb;
  Gen<T, S> Fb;
  T best;
  int tbest;
  unsigned st;
};

// the stage blocks of step k (horizon_selection.py:57-64): E = chol_inv(Q_k),
// F = E A^T, G = _sym(A F + B R^-1 B^T); independent of every other step
template <class T, int S, int MM>
HOP_HD inline void stage_blocks(const Gen<T, S>& Q, const Gen<T, S>& A, const T (&Bk)[S][MM],
                                const T (&rinv)[MM][MM], int mt, unsigned& st, Sym<T, S>& E,
                                Gen<T, S>& F, Sym<T, S>& G) {
  sym_of(E, Q);
  spd_inverse(E, mt, st);                   // E = chol_inv(Q)
  mul_sym_gt(F, E, A);                      // F = E A^T
#pragma unroll
  for (int i = 0; i < Sym<T, S>::NP; ++i) G.v[i] = T(0);
  acc_sym_xy<false>(G, A, F);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    T y[MM];
#pragma unroll
    for (int q = 0; q < MM; ++q) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < MM; ++l) v += Bk[i][l] * rinv[l][q];
      y[q] = v;
    }
#pragma unroll
    for (int j = i; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int q = 0; q < MM; ++q) v += y[q] * Bk[j][q];
      G.at(i, j) += v;
    }
  }
}

// the prefix compose with step k's stage blocks (horizon_selection.py:66-75): the
// only loop-carried part of the sweep
// (inv: the chol_inv of W = E_k + Gbar, spd_inverse's semantics; the pipelined rerun
// passes one that runs the jitter ladder's attempts on separate lanes)
template <class T, int S, int MM, class Inv>
HOP_HD inline void compose_step(State<T, S, MM>& s, int k, const Sym<T, S>& E, const Gen<T, S>& F,
                                const Sym<T, S>& G, int mt, Inv&& inv) {
  if (k == 0) {
    s.Eb = E;
    s.Fb = F;
    s.Gb = G;
    return;
  }
  Sym<T, S> W;
#pragma unroll
  for (int i = 0; i < Sym<T, S>::NP; ++i) W.v[i] = E.v[i] + s.Gb.v[i];
  inv(W, mt, s.st);                         // W = (E_k + Gbar)^-1
  Gen<T, S> Z;
  mul_sym_gt(Z, W, s.Fb);                   // W Fbar^T
  acc_sym_xy<true>(s.Eb, s.Fb, Z);          // Ebar = _sym(Ebar - Fbar W Fbar^T)
  mul_sym_g(Z, W, F);                       // W F
  Gen<T, S> Fn;
  mul_gg(Fn, s.Fb, Z);                      // Fbar = Fbar W F
  s.Fb = Fn;
  s.Gb = G;
  acc_sym_xty<true>(s.Gb, F, Z);            // Gbar = _sym(G - F^T W F)
}
template <class T, int S, int MM>
HOP_HD inline void compose_step(State<T, S, MM>& s, int k, const Sym<T, S>& E, const Gen<T, S>& F,
                                const Sym<T, S>& G, int mt) {
  compose_step<T, S, MM>(s, k, E, F, G, mt,
                         [](Sym<T, S>& x, int t, unsigned& st) { spd_inverse(x, t, st); });
}

// stage + compose for step k (Q, A, B of step k given); returns nothing
template <class T, int S, int MM>
HOP_HD inline void stage_compose(State<T, S, MM>& s, int k, const Gen<T, S>& Q,
                                 const Gen<T, S>& A, const T (&Bk)[S][MM],
                                 const T (&rinv)[MM][MM], int mt) {
  Sym<T, S> E, G;
  Gen<T, S> F;
  stage_blocks<T, S, MM>(Q, A, Bk, rinv, mt, s.st, E, F, G);
  compose_step<T, S, MM>(s, k, E, F, G, mt);
}

// query horizon k+1 from QT_k; returns J
template <class T, int S, int MM>
HOP_HD inline T query(State<T, S, MM>& s, const Gen<T, S>& QT, const T (&z)[S], int mt) {
  Sym<T, S> X;
  sym_of(X, QT);
  spd_inverse(X, mt, s.st);                 // QT^-1
#pragma unroll
  for (int i = 0; i < Sym<T, S>::NP; ++i) X.v[i] += s.Gb.v[i];
  spd_inverse(X, mt, s.st);                 // Wt = (QT^-1 + Gbar)^-1
  Gen<T, S> V;
  mul_sym_gt(V, X, s.Fb);                   // Wt Fbar^T
  Sym<T, S> X0 = s.Eb;
  acc_sym_xy<true>(X0, s.Fb, V);            // X0 = _sym(Ebar - Fbar Wt Fbar^T)
  return T(0.5) * quad_inverse(X0, z, mt, s.st);
}

// ---- conditioned prefix (lft_sweep_v2.hip, SchedCond) ------
// The same J(t) with z0 folded into the prefix first: state (Sigma + eps I, m,
// gamma); per stage an LDL^T of S = Sigma_eps + E_k with the rank-1 streams of
// Sigma', m', gamma', the predict A Sigma' A^T + B R^-1 B^T, and per horizon a
// bordered elimination of Sigma_eps + X_t.  First attempts only: anything that
// would need chol_inv's ladder sets `bad` and the problem is recomputed by the
// LFT path (rerun launch).
template <class T, int S, int MM>
struct CondState {
  Sym<T, S> Sg;  // Sigma + eps I (upper triangle)
  T m[S];
  T gam;
  T best;
  int tbest;
  unsigned st;
  bool bad;
  int kf1;  // 1 + the first flagged horizon (0: none yet)
};

template <class T, int S, int MM>
HOP_HD inline void cond_init(CondState<T, S, MM>& c, const T (&z)[S]) {
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) c.Sg.v[k] = T(0);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    c.Sg.at(i, i) = T(1e-9);
    c.m[i] = z[i];
  }
  c.gam = T(0);
  c.best = T(0);
  c.tbest = 0;
  c.st = 0;
  c.bad = false;
  c.kf1 = 0;
}

// after horizon k + 1 is evaluated (and taken): the first horizon that raised a flag
// (a pivot, a Schur complement, a non-finite J); a flag set before the sweep
// (a forced hand-over) is horizon 0
template <class T, int S, int MM>
HOP_HD inline bool cond_flagged(const CondState<T, S, MM>& c) {
  return c.bad || (c.st & kStNonfinite) != 0u;
}
template <class T, int S, int MM>
HOP_HD inline void cond_mark(CondState<T, S, MM>& c, int k) {
  if (cond_flagged(c) && c.kf1 == 0) c.kf1 = k + 2;
}
// the status the conditioned kernel leaves: 0, or the hand-over word (include/hop.h)
template <class T, int S, int MM>
HOP_HD inline int cond_status_word(const CondState<T, S, MM>& c) {
  return cond_flagged(c) ? HOP_HANDOVER_WORD(c.kf1 > 0 ? c.kf1 - 1 : 0) : 0;
}

// (sym(M) + 1e-9 I)^-1 on the first attempt only (utils.py:69-93 without the ladder)
template <class T, int S>
HOP_HD inline bool spd_inverse_once(Sym<T, S>& m) {
  const bool ok = sweep_neg_inverse(m, T(1e-9));
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) m.v[k] = -m.v[k];
  return ok;
}

// condition on stage k (E = (Q_k + eps I)^-1), then predict through A_k, B_k
template <class T, int S, int MM>
HOP_HD inline void cond_step(CondState<T, S, MM>& c, const Sym<T, S>& E, const Gen<T, S>& A,
                             const T (&Bk)[S][MM], const T (&rinv)[MM][MM]) {
  Sym<T, S> M;
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) M.v[k] = c.Sg.v[k] + E.v[k];
  T Y[S][S + 1];  // L^-1 [Sigma_eps | m]
#pragma unroll
  for (int i = 0; i < S; ++i) {
#pragma unroll
    for (int j = 0; j < S; ++j) Y[i][j] = c.Sg.at(i, j);
    Y[i][S] = c.m[i];
  }
  T rd[S];
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const T d = M.at(p, p);
    c.bad = c.bad || !(d > T(0));
    const T r = small_recip(d);
    rd[p] = r;
#pragma unroll
    for (int i = p + 1; i < S; ++i) {
      const T l = M.at(p, i) * r;
#pragma unroll
      for (int j = i; j < S; ++j) M.at(i, j) -= l * M.at(p, j);
#pragma unroll
      for (int j = 0; j <= S; ++j) Y[i][j] -= l * Y[p][j];
    }
  }
  Sym<T, S> Sp = c.Sg;  // Sigma' = Sigma_eps - sum_p y_p y_p^T / d_p, m' and gamma' alike
  T mp[S];
#pragma unroll
  for (int i = 0; i < S; ++i) mp[i] = c.m[i];
#pragma unroll
  for (int p = 0; p < S; ++p) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const T yi = Y[p][i] * rd[p];
#pragma unroll
      for (int j = i; j < S; ++j) Sp.at(i, j) -= yi * Y[p][j];
      mp[i] -= yi * Y[p][S];
    }
    c.gam -= Y[p][S] * Y[p][S] * rd[p];
  }
  Gen<T, S> Tm;
  mul_sym_gt(Tm, Sp, A);  // Sigma' A^T
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) c.Sg.v[k] = T(0);
  acc_sym_xy<false>(c.Sg, A, Tm);  // A Sigma' A^T (upper)
#pragma unroll
  for (int i = 0; i < S; ++i) {
    T y[MM];
#pragma unroll
    for (int q = 0; q < MM; ++q) {
      T v = T(0);
#pragma unroll
      for (int l = 0; l < MM; ++l) v += Bk[i][l] * rinv[l][q];
      y[q] = v;
    }
#pragma unroll
    for (int j = i; j < S; ++j) {
      T v = T(0);
#pragma unroll
      for (int q = 0; q < MM; ++q) v += y[q] * Bk[j][q];
      c.Sg.at(i, j) += v;
    }
    c.Sg.at(i, i) += T(1e-9);
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    T v = T(0);
#pragma unroll
    for (int j = 0; j < S; ++j) v += A.a[i][j] * mp[j];
    c.m[i] = v;
  }
}

// J of horizon k+1: 1/2 (m^T (Sigma_eps + X_t)^-1 m - gamma), X_t = (QT_k + eps I)^-1.
// QT_k + eps I = [[P11, b], [b^T, cc]] is swept on its first S - 1 pivots only, which
// leaves P11^-1, u = P11^-1 b and sigma = cc - b^T P11^-1 b (the potrf test of QT_k +
// eps I is then: those pivots and sigma > 0).  With W = [[I, 0], [-u^T, 1]] and
// D = diag(P11^-1, 1/sigma), X_t = W^T D W, so
//   m^T (Sigma_eps + X_t)^-1 m = m~^T (W^-T Sigma_eps W^-1 + D)^-1 m~,  m~ = W^-T m,
// W^-1 = I + e_{S-1} [u; 0]^T.  The augmented terminal block's rho_reg = 1e-12 makes
// sigma ~ 1e-9: its 1/sigma then sits alone on the last diagonal entry, where no
// pivot cancels it.  Eliminating Sigma_eps + X_t itself (cond_query_direct) loses
// 1e-7 .. 1e-5 of q on real linearisations; this form holds ~1e-15 (tests/
// test_host_cpu.py against the 50-digit curves of tests/golden/real_lin_hp.npz).
template <class T, int S, int MM>
HOP_HD inline T cond_query(CondState<T, S, MM>& c, const Gen<T, S>& QT) {
  constexpr int NN = S - 1;
  Sym<T, S> x;
  sym_of(x, QT);
#pragma unroll
  for (int i = 0; i < S; ++i) x.at(i, i) += T(1e-9);
  // symmetric sweep of pivots 0 .. NN-1: x = [[-P11^-1, u], [u^T, sigma]]
#pragma unroll
  for (int p = 0; p < NN; ++p) {
    const T d = x.at(p, p);
    c.bad = c.bad || !(d > T(0));
    const T r = small_recip(d);
#pragma unroll
    for (int i = 0; i < S; ++i) {
      if (i == p) continue;
      const T aip = x.at(i, p) * r;
#pragma unroll
      for (int j = i; j < S; ++j) {
        if (j == p) continue;
        x.at(i, j) -= aip * x.at(p, j);
      }
    }
#pragma unroll
    for (int i = 0; i < S; ++i)
      if (i != p) x.at(i, p) *= r;
    x.at(p, p) = -r;
  }
  const T sig = x.at(NN, NN);
  c.bad = c.bad || !(sig > T(0));
  T u[NN];
#pragma unroll
  for (int i = 0; i < NN; ++i) u[i] = x.at(i, NN);
  // y = W^-T Sigma_eps W^-1 + D, b = W^-T m
  const Sym<T, S>& Sg = c.Sg;
  Sym<T, S> y;
  T b[S];
  const T snn = Sg.at(NN, NN);
#pragma unroll
  for (int i = 0; i < NN; ++i) {
    const T sin_ = Sg.at(i, NN) + u[i] * snn;  // row i of Sigma W^-1 at column NN, then W^-T
#pragma unroll
    for (int j = i; j < NN; ++j)
      y.at(i, j) = (Sg.at(i, j) + u[j] * Sg.at(i, NN)) + u[i] * (Sg.at(NN, j) + u[j] * snn) -
                   x.at(i, j);  // + P11^-1
    y.at(i, NN) = sin_;
    b[i] = c.m[i] + u[i] * c.m[NN];
  }
  y.at(NN, NN) = snn + small_recip(sig);
  b[NN] = c.m[NN];
  T acc = T(0);
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const T d = y.at(p, p);
    c.bad = c.bad || !(d > T(0));
    const T r = small_recip(d);
    acc += b[p] * b[p] * r;
#pragma unroll
    for (int i = p + 1; i < S; ++i) {
      const T l = y.at(p, i) * r;
      b[i] -= l * b[p];
#pragma unroll
      for (int j = i; j < S; ++j) y.at(i, j) -= l * y.at(p, j);
    }
  }
  return T(0.5) * (acc - c.gam);
}

// round 3's query: eliminate Sigma_eps + X_t with X_t formed by a full sweep
// (kept for the host comparison in tests/test_host_cpu.py)
template <class T, int S, int MM>
HOP_HD inline T cond_query_direct(CondState<T, S, MM>& c, const Gen<T, S>& QT) {
  Sym<T, S> x;
  sym_of(x, QT);
  c.bad = c.bad || !spd_inverse_once(x);
#pragma unroll
  for (int k = 0; k < Sym<T, S>::NP; ++k) x.v[k] += c.Sg.v[k];
  T b[S];
#pragma unroll
  for (int i = 0; i < S; ++i) b[i] = c.m[i];
  T acc = T(0);
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const T d = x.at(p, p);
    c.bad = c.bad || !(d > T(0));
    const T r = small_recip(d);
    acc += b[p] * b[p] * r;
#pragma unroll
    for (int i = p + 1; i < S; ++i) {
      const T l = x.at(p, i) * r;
      b[i] -= l * b[p];
#pragma unroll
      for (int j = i; j < S; ++j) x.at(i, j) -= l * x.at(p, j);
    }
  }
  return T(0.5) * (acc - c.gam);
}

template <class T>
HOP_HD inline bool finite_t(T x) {
  return x == x && x - x == T(0);
}

// argmin over [t_min, t_max] with np.argmin semantics (first minimiser, a NaN wins)
template <class T, class St>
HOP_HD inline void take(St& s, int t, T jk, int t_min, int t_max) {
  if (!finite_t(jk)) s.st |= kStNonfinite;
  if (t_max <= 0) return;
  if (t == t_min) {
    s.best = jk;
    s.tbest = t;
  } else if (t > t_min && t <= t_max) {
    const bool bnan = s.best != s.best, jnan = jk != jk;
    if (!bnan && (jnan || jk < s.best)) {
      s.best = jk;
      s.tbest = t;
    }
  }
}

}  // namespace small
}  // namespace hop
