// Host build of small_math.hpp for the CPU test suite (not part of libhop_amd.so):
//   g++ -O2 -std=c++17 -shared -fPIC -DHOP_HD= small_host.cpp -o libsmall_host.so
// Runs the exact per-problem arithmetic of lft_small.hip on the CPU.
#include <stdint.h>

namespace hop {
namespace small {
// exact division, except where the device's v_rcp + Newton step (lft_small.hip) gives
// NaN: d = 0 or +-inf (the residual fma(-d, rcp(d), 1) is 0 * inf there), so that a
// non-finite or zero pivot poisons the host result exactly as it does on the device
template <class T>
inline T small_recip(T d) {
  const T r = T(1) / d;
  return (d == T(0) || r == T(0) || r != r) ? T(__builtin_nan("")) : r;
}
}  // namespace small
}  // namespace hop

#include "small_math.hpp"
#include "wrap.hpp"

using namespace hop::small;

template <class T, int S, int MM>
static void run(const T* A, const T* B, const T* Q, const T* Rinv, const T* QT, const T* z0,
                int64_t batch, int n, int mt, int t_min, int t_max, T* J, int32_t* status,
                int32_t* t_star) {
  for (int64_t b = 0; b < batch; ++b) {
    State<T, S, MM> ps;
    ps.st = 0;
    ps.best = T(0);
    ps.tbest = 0;
    T z[S], rinv[MM][MM];
    for (int i = 0; i < S; ++i) z[i] = z0[b * S + i];
    for (int i = 0; i < MM; ++i)
      for (int j = 0; j < MM; ++j) rinv[i][j] = Rinv[b * MM * MM + i * MM + j];  // per problem
    for (int k = 0; k < n; ++k) {
      Gen<T, S> Qk, Ak, QTk;
      T Bk[S][MM];
      const int64_t o = (b * n + k) * S * S, ob = (b * n + k) * S * MM;
      for (int i = 0; i < S; ++i)
        for (int j = 0; j < S; ++j) {
          Qk.a[i][j] = Q[o + i * S + j];
          Ak.a[i][j] = A[o + i * S + j];
          QTk.a[i][j] = QT[o + i * S + j];
        }
      for (int i = 0; i < S; ++i)
        for (int j = 0; j < MM; ++j) Bk[i][j] = B[ob + i * MM + j];
      stage_compose<T, S, MM>(ps, k, Qk, Ak, Bk, rinv, mt);
      const T jk = query<T, S, MM>(ps, QTk, z, mt);
      J[b * n + k] = jk;
      take(ps, k + 1, jk, t_min, t_max);
    }
    status[b] = (int32_t)ps.st;
    t_star[b] = ps.tbest;
  }
}

// conditioned-prefix path (lft_small.hip COND kernels): status = the hand-over word
// (HOP_HANDOVER_WORD of the first flagged horizon) when the problem would be handed
// to the rerun launch
template <class T, int S, int MM, bool DIRECT = false>
static void run_cond(const T* A, const T* B, const T* Q, const T* Rinv, const T* QT, const T* z0,
                     int64_t batch, int n, int t_min, int t_max, T* J, int32_t* status,
                     int32_t* t_star) {
  for (int64_t b = 0; b < batch; ++b) {
    CondState<T, S, MM> cs;
    T z[S], rinv[MM][MM];
    for (int i = 0; i < S; ++i) z[i] = z0[b * S + i];
    for (int i = 0; i < MM; ++i)
      for (int j = 0; j < MM; ++j) rinv[i][j] = Rinv[b * MM * MM + i * MM + j];
    cond_init(cs, z);
    for (int k = 0; k < n; ++k) {
      Gen<T, S> Qk, Ak, QTk;
      T Bk[S][MM];
      const int64_t o = (b * n + k) * S * S, ob = (b * n + k) * S * MM;
      for (int i = 0; i < S; ++i)
        for (int j = 0; j < S; ++j) {
          Qk.a[i][j] = Q[o + i * S + j];
          Ak.a[i][j] = A[o + i * S + j];
          QTk.a[i][j] = QT[o + i * S + j];
        }
      for (int i = 0; i < S; ++i)
        for (int j = 0; j < MM; ++j) Bk[i][j] = B[ob + i * MM + j];
      Sym<T, S> E;
      sym_of(E, Qk);
      cs.bad = cs.bad || !spd_inverse_once(E);
      cond_step<T, S, MM>(cs, E, Ak, Bk, rinv);
      const T jk = DIRECT ? cond_query_direct<T, S, MM>(cs, QTk) : cond_query<T, S, MM>(cs, QTk);
      J[b * n + k] = jk;
      take(cs, k + 1, jk, t_min, t_max);
      cond_mark(cs, k);
    }
    status[b] = cond_status_word(cs);  // the kernels' hand-over word (include/hop.h)
    t_star[b] = cs.tbest;
  }
}

extern "C" int small_host_cond_sweep_f64(const double* A, const double* B, const double* Q,
                                         const double* Rinv, const double* QT, const double* z0,
                                         int64_t batch, int n, int s, int m, int t_min, int t_max,
                                         double* J, int32_t* status, int32_t* t_star) {
  if (s == 3 && m == 1) run_cond<double, 3, 1>(A, B, Q, Rinv, QT, z0, batch, n, t_min, t_max, J, status, t_star);
  else if (s == 5 && m == 1) run_cond<double, 5, 1>(A, B, Q, Rinv, QT, z0, batch, n, t_min, t_max, J, status, t_star);
  else return -1;
  return 0;
}

// the round-3 query (cond_query_direct), for the accuracy comparison
extern "C" int small_host_cond_sweep_direct_f64(const double* A, const double* B, const double* Q,
                                                const double* Rinv, const double* QT,
                                                const double* z0, int64_t batch, int n, int s,
                                                int m, int t_min, int t_max, double* J,
                                                int32_t* status, int32_t* t_star) {
  if (s == 3 && m == 1) run_cond<double, 3, 1, true>(A, B, Q, Rinv, QT, z0, batch, n, t_min, t_max, J, status, t_star);
  else if (s == 5 && m == 1) run_cond<double, 5, 1, true>(A, B, Q, Rinv, QT, z0, batch, n, t_min, t_max, J, status, t_star);
  else return -1;
  return 0;
}

extern "C" int small_host_cond_sweep_f32(const float* A, const float* B, const float* Q,
                                         const float* Rinv, const float* QT, const float* z0,
                                         int64_t batch, int n, int s, int m, int t_min, int t_max,
                                         float* J, int32_t* status, int32_t* t_star) {
  if (s == 5 && m == 1) run_cond<float, 5, 1>(A, B, Q, Rinv, QT, z0, batch, n, t_min, t_max, J, status, t_star);
  else return -1;
  return 0;
}

extern "C" int small_host_sweep_f64(const double* A, const double* B, const double* Q,
                                    const double* Rinv, const double* QT, const double* z0,
                                    int64_t batch, int n, int s, int m, int mt, int t_min,
                                    int t_max, double* J, int32_t* status, int32_t* t_star) {
  if (s == 3 && m == 1) run<double, 3, 1>(A, B, Q, Rinv, QT, z0, batch, n, mt, t_min, t_max, J, status, t_star);
  else if (s == 5 && m == 1) run<double, 5, 1>(A, B, Q, Rinv, QT, z0, batch, n, mt, t_min, t_max, J, status, t_star);
  else return -1;
  return 0;
}

extern "C" int small_host_sweep_f32(const float* A, const float* B, const float* Q,
                                    const float* Rinv, const float* QT, const float* z0,
                                    int64_t batch, int n, int s, int m, int mt, int t_min,
                                    int t_max, float* J, int32_t* status, int32_t* t_star) {
  if (s == 5 && m == 1) run<float, 5, 1>(A, B, Q, Rinv, QT, z0, batch, n, mt, t_min, t_max, J, status, t_star);
  else return -1;
  return 0;
}

// wrap.hpp on the host (tests/test_host_cpu.py checks it against Python's float %)
extern "C" void small_host_wrap_f64(const double* in, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = hop::wrap_angle(in[i]);
}
extern "C" void small_host_wrap_f32(const float* in, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = hop::wrap_angle(in[i]);
}

// The LU slot (lu_pivot.hpp) on the host: x = (sym(A) + eps I)^-1 b, n <= 16; 0 or -1
// when the pivoted factorisation meets an exactly zero pivot
extern "C" int small_host_lu_sym_solve_f64(const double* A, int n, double eps, const double* b,
                                           double* x) {
  double y[16];
  for (int i = 0; i < 16; ++i) y[i] = i < n ? b[i] : 0.0;
  const bool ok =
      hop::lu_sym_solve<double, 16>([&](int i, int j) { return A[i * n + j]; }, n, eps, y);
  for (int i = 0; i < n; ++i) x[i] = y[i];
  return ok ? 0 : -1;
}

// the small-s kernels' chol_inv (small_math.hpp spd_inverse, the ladder and the LU
// slot solved on registers) and quad_inverse at s = 5; st = the status bits
extern "C" void small_host_spd_inverse_s5_f64(const double* M, int max_tries, double* out,
                                              unsigned* st) {
  hop::small::Sym<double, 5> m;
  for (int i = 0; i < 5; ++i)
    for (int j = i; j < 5; ++j) m.at(i, j) = 0.5 * (M[i * 5 + j] + M[j * 5 + i]);
  *st = 0;
  hop::small::spd_inverse(m, max_tries, *st);
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) out[i * 5 + j] = m.at(i, j);
}
extern "C" double small_host_quad_inverse_s5_f64(const double* M, const double* z, int max_tries,
                                                 unsigned* st) {
  hop::small::Sym<double, 5> m;
  for (int i = 0; i < 5; ++i)
    for (int j = i; j < 5; ++j) m.at(i, j) = 0.5 * (M[i * 5 + j] + M[j * 5 + i]);
  double zz[5];
  for (int i = 0; i < 5; ++i) zz[i] = z[i];
  *st = 0;
  return hop::small::quad_inverse(m, zz, max_tries, *st);
}

// the hand-over word's field and the triage rule as include/hop.h defines them (the
// kernels use the same macros; tests/test_host_cpu.py decodes statuses with these)
extern "C" int small_host_handover_horizon(int32_t status) { return HOP_HANDOVER_HORIZON(status); }
extern "C" int small_host_handover_word(int32_t h) { return HOP_HANDOVER_WORD(h); }
extern "C" int small_host_triage_accepts(int32_t h, int32_t h_poison, int32_t h_qt, int32_t n) {
  return HOP_TRIAGE_ACCEPTS(h, h_poison, h_qt, n) ? 1 : 0;
}
