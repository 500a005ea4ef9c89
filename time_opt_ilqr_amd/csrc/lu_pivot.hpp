// chol_inv's last resort, the LU slot (utils.py:88-93): np.linalg.solve(A + eps I, I)
// after every jitter failed, i.e. LAPACK gesv -- an LU factorisation with partial
// pivoting (the row of largest |a_ip| at or below the diagonal, the first one on a
// tie, as idamax) and triangular solves.  Without the row exchanges a block whose
// leading minors vanish (a zero pivot) cannot be solved although it is regular.
//
// Rare path: the kernels call it only for problems flagged ST_LU.  Each lane factors
// its own private copy (the arrays live in scratch for the larger sizes), so no
// LDS, no cross-lane traffic and no synchronisation are involved; the host test
// build (small_host.cpp) exercises the same code against NumPy.
#pragma once

#ifndef HOP_HD
#define HOP_HD __host__ __device__
#endif

namespace hop {

// In place: a (n x n, row-major in a[S][S]) <- L\U of P a, perm[i] = original row
// of row i.  Returns false on an exactly zero pivot (gesv: singular, LinAlgError).
template <class T, int S>
HOP_HD inline bool lu_factor(T (&a)[S][S], int n, int (&perm)[S]) {
  bool ok = true;
  for (int i = 0; i < n; ++i) perm[i] = i;
  for (int p = 0; p < n; ++p) {
    int piv = p;
    T big = a[p][p] < T(0) ? -a[p][p] : a[p][p];
    for (int i = p + 1; i < n; ++i) {
      const T v = a[i][p] < T(0) ? -a[i][p] : a[i][p];
      if (v > big) {
        big = v;
        piv = i;
      }
    }
    if (piv != p) {
      for (int j = 0; j < n; ++j) {
        const T t = a[p][j];
        a[p][j] = a[piv][j];
        a[piv][j] = t;
      }
      const int t = perm[p];
      perm[p] = perm[piv];
      perm[piv] = t;
    }
    const T d = a[p][p];
    if (!(d != T(0))) {
      ok = false;
      continue;
    }
    for (int i = p + 1; i < n; ++i) {
      const T l = a[i][p] / d;
      a[i][p] = l;
      for (int j = p + 1; j < n; ++j) a[i][j] -= l * a[p][j];
    }
  }
  return ok;
}

// x <- (P^T L U)^-1 b for the factors of lu_factor (b is overwritten)
template <class T, int S>
HOP_HD inline void lu_solve(const T (&a)[S][S], int n, const int (&perm)[S], T (&b)[S]) {
  T y[S];
  for (int i = 0; i < n; ++i) y[i] = b[perm[i]];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j) y[i] -= a[i][j] * y[j];
  for (int i = n - 1; i >= 0; --i) {
    T v = y[i];
    for (int j = i + 1; j < n; ++j) v -= a[i][j] * b[j];
    b[i] = v / a[i][i];
  }
  for (int i = n; i < S; ++i) b[i] = T(0);
}

// x = (sym(M) + eps I)^-1 rhs with M(i, j) = at(i, j), n x n; false when singular
template <class T, int S, class F>
HOP_HD inline bool lu_sym_solve(F at, int n, T eps, T (&x)[S]) {
  T a[S][S];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) a[i][j] = T(0.5) * (at(i, j) + at(j, i)) + (i == j ? eps : T(0));
  int perm[S];
  const bool ok = lu_factor<T, S>(a, n, perm);
  if (ok) lu_solve<T, S>(a, n, perm, x);
  return ok;
}

// The same factorisation and solves with every index a compile-time constant (S is
// the whole size), for the small-s kernels' per-lane LU slot: the row exchanges are
// selects, so the arrays stay in registers.  A loop-indexed private array lives in
// scratch: with the per-column lu_sym_solve (one factorisation per right-hand side)
// the small-s rerun kernel spent ~60 us per step in scratch round trips on blocks
// that reach the slot (the point-mass obstacle cost's indefinite Q_k, about half of
// the inverses).  The right-hand sides ride along the elimination in the order the
// forward substitution of lu_solve applies them, and the back substitution is
// lu_solve's, so the values equal lu_sym_solve's bit for bit
// (tests/test_host_cpu.py::test_lu_slot_registers_equal_per_column_solves).
// rhs (S x R, row i = right-hand-side row i) <- (sym(M) + eps I)^-1 rhs; false when an
// exactly zero pivot makes the block singular (gesv's LinAlgError)
template <class T, int S, int R, class F>
HOP_HD inline bool lu_sym_solve_regs(F at, T eps, T (&rhs)[S][R]) {
  T a[S][S];
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < S; ++j) a[i][j] = T(0.5) * (at(i, j) + at(j, i)) + (i == j ? eps : T(0));
  bool ok = true;
#pragma unroll
  for (int p = 0; p < S; ++p) {
    int piv = p;
    T big = a[p][p] < T(0) ? -a[p][p] : a[p][p];
#pragma unroll
    for (int i = p + 1; i < S; ++i) {
      const T v = a[i][p] < T(0) ? -a[i][p] : a[i][p];
      if (v > big) {
        big = v;
        piv = i;
      }
    }
#pragma unroll
    for (int i = p + 1; i < S; ++i) {
      const bool sw = piv == i;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const T t = a[p][j];
        a[p][j] = sw ? a[i][j] : t;
        a[i][j] = sw ? t : a[i][j];
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const T t = rhs[p][j];
        rhs[p][j] = sw ? rhs[i][j] : t;
        rhs[i][j] = sw ? t : rhs[i][j];
      }
    }
    const T d = a[p][p];
    ok = ok && (d != T(0));
#pragma unroll
    for (int i = p + 1; i < S; ++i) {
      const T l = a[i][p] / d;
      a[i][p] = l;
#pragma unroll
      for (int j = p + 1; j < S; ++j) a[i][j] -= l * a[p][j];
#pragma unroll
      for (int j = 0; j < R; ++j) rhs[i][j] -= l * rhs[p][j];
    }
  }
#pragma unroll
  for (int c = 0; c < R; ++c)
#pragma unroll
    for (int i = S - 1; i >= 0; --i) {
      T v = rhs[i][c];
#pragma unroll
      for (int j = i + 1; j < S; ++j) v -= a[i][j] * rhs[j][c];
      rhs[i][c] = v / a[i][i];
    }
  return ok;
}

#ifdef __HIPCC__
// The kernels' LU slot as an out-of-line call (a rare path: inlined, its private
// arrays raised the register pressure of the sweep loops around it).
// x (n values, private memory) <- (sym(M) + (diag + eps) I)^-1 x, M(i, j) = M[i ld + j]
// in LDS; returns 0, or -1 on an exactly zero pivot.
template <class T>
__device__ __noinline__ int lu_lds_solve(const T* M, int ld, int n, T diag, T eps, T* x) {
  T b[16];
  for (int i = 0; i < 16; ++i) b[i] = i < n ? x[i] : T(0);
  const bool ok = lu_sym_solve<T, 16>(
      [&](int i, int j) { return M[i * ld + j] + (i == j ? diag : T(0)); }, n, eps, b);
  for (int i = 0; i < n; ++i) x[i] = b[i];
  return ok ? 0 : -1;
}
#endif

}  // namespace hop
