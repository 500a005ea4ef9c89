// Discrete-time dynamics x_{k+1} = F(x_k, u_k) of the reference's benchmark
// systems and one finite-difference column of their Jacobians, for the batched
// linearisation kernel (linearize.hip) and the host test build (dyn_host.cpp).
//   0 DoubleIntegrator   systems.py:28-33    n = 2,  m = 1
//   1 CartpoleSwingUp    systems.py:57-95    n = 4,  m = 1
//   2 Quadrotor          systems.py:119-210  n = 12, m = 4 (NaN guards 175-191)
//   3 PointmassNav       systems.py:237-249  n = 4,  m = 2
//   4 SegwayBalance      systems.py:303-333  n = 4,  m = 1
// Expressions follow the reference's order and are compiled without FMA
// contraction (HOP_DYN_BEGIN), so F is bit-identical to NumPy wherever no libm
// call is involved (DI, point mass, segway; angle_normalize is exact).  The
// quadrotor's small matrix products that NumPy hands to BLAS (Rz Ry Rx,
// Rb (e3 thrust) and Tmat omg, systems.py:156, 199-200) are formed in OpenBLAS's
// FMA order (dgemm: one ascending chain; dgemv on 3 rows: fma(a2, x2, fma(a0, x0,
// a1 x1)), both measured against NumPy here) -- with that, the host build
// reproduces the reference bit for bit.  The
// quadrotor's trigonometry is split out (QuadTrig) so that the Jacobian columns
// which do not move an Euler angle reuse the values of the base point: the
// values are the same numbers the reference recomputes, so nothing changes.
#pragma once
#include <math.h>

#include "wrap.hpp"

#ifndef HOP_HD
#define HOP_HD __host__ __device__
#endif

#if defined(__clang__)
#define HOP_DYN_BEGIN _Pragma("clang fp contract(off)")
#else
#define HOP_DYN_BEGIN  // host build: -ffp-contract=off
#endif

namespace hop {
namespace dyn {

enum System : int { kDI = 0, kCartpole = 1, kQuadrotor = 2, kPointmass = 3, kSegway = 4 };
constexpr int kNumSystems = 5;

HOP_HD constexpr int state_dim(int sys) {
  return sys == kDI ? 2 : sys == kQuadrotor ? 12 : (sys >= 1 && sys <= 4) ? 4 : 0;
}
HOP_HD constexpr int control_dim(int sys) {
  return sys == kQuadrotor ? 4 : sys == kPointmass ? 2 : (sys >= 0 && sys <= 4) ? 1 : 0;
}

HOP_HD inline bool finite_d(double v) { return v - v == 0.0; }  // false for NaN and +-inf

// sin and cos of one angle.  On the device one sincos: ocml's sin, cos and sincos
// run the same argument reduction and the same kernel polynomials and differ only
// in which results they select, so the values are bitwise those of separate
// sin/cos calls, for the reduction's cost once (the compiler does not merge two
// inlined reductions by itself).  HOP_SINCOS=0 keeps the separate calls (A/B).
#ifndef HOP_SINCOS
#define HOP_SINCOS 1
#endif
HOP_HD inline void sin_cos(double v, double& s, double& c) {
#if HOP_SINCOS && defined(__HIP_DEVICE_COMPILE__)
  sincos(v, &s, &c);
#else
  s = sin(v), c = cos(v);
#endif
}

// tan from the sin and cos already formed (device): one IEEE division instead of a
// second argument reduction and tan's own polynomial, within an ulp or two of libm's
// tan.  Off by default since round 6: the reference evaluates one F for
// every rollout, so a zero step of its line search reproduces the current X bit for
// bit and is rejected (J_new < J_old is strict, solver.py:233-286); with this tan in
// the line search's rollouts only, the first iteration's zero step moved X by an ulp
// against hop_rollout_f64's trajectory and could be accepted on rounding.  The FD
// linearisation (1/h amplifies ulps) and hop_rollout_f64 (the fixtures of
// tests/test_gpu_real_lin.py are its outputs) cannot take it, so every rollout keeps
// libm's tan (the sincos above is bitwise the separate calls and stays).  It saved 4.3 %
// of the line search (profiles/r05_tan_sc_ab.jsonl).  HOP_TAN_SC=1: the A/B.
#ifndef HOP_TAN_SC
#define HOP_TAN_SC 0
#endif
HOP_HD inline double tan_sc(double v, double s, double c) {
#if HOP_TAN_SC && defined(__HIP_DEVICE_COMPILE__)
  (void)v;
  return s / c;
#else
  (void)s, (void)c;
  return tan(v);
#endif
}

// Python's max(a, b) keeps a unless b > a (so a NaN b never wins)
HOP_HD inline double py_max(double a, double b) { return b > a ? b : a; }

// FD step of linearization.py:196/203/253/257: max(eps, rel * max(1.0, |v|))
HOP_HD inline double fd_step(double v, double eps, double rel) {
  HOP_DYN_BEGIN
  return py_max(eps, rel * py_max(1.0, fabs(v)));
}

HOP_HD inline void f_di(const double* x, const double* u, double dt, double* o) {
  HOP_DYN_BEGIN
  o[0] = x[0] + dt * x[1];
  o[1] = x[1] + dt * u[0];
}

HOP_HD inline void f_cartpole(const double* x, const double* u, double dt, double* o) {
  HOP_DYN_BEGIN
  const double g = 9.81, m_cart = 1.0, m_pole = 0.1, length = 0.5;
  const double total_mass = m_cart + m_pole;
  const double polemass_length = m_pole * length;
  const double th_u = x[2] - 3.141592653589793;  // math.pi
  double costh, sinth;
  sin_cos(th_u, sinth, costh);
  const double temp = (u[0] + polemass_length * x[3] * x[3] * sinth) / total_mass;
  const double denom = length * (4.0 / 3.0 - m_pole * costh * costh / total_mass);
  const double th_acc = (g * sinth - costh * temp) / denom;
  const double x_acc = temp - polemass_length * th_acc * costh / total_mass;
  o[0] = x[0] + dt * x[1];
  o[1] = x[1] + dt * x_acc;
  o[2] = wrap_angle(x[2] + dt * x[3]);
  o[3] = x[3] + dt * th_acc;
}

HOP_HD inline void f_pointmass(const double* x, const double* u, double dt, double* o) {
  HOP_DYN_BEGIN
  o[0] = x[0] + dt * x[2];
  o[1] = x[1] + dt * x[3];
  o[2] = x[2] + dt * u[0];
  o[3] = x[3] + dt * u[1];
}

HOP_HD inline void f_segway(const double* x, const double* u, double dt, double* o) {
  HOP_DYN_BEGIN
  const double g = 9.81, r = 0.15, M = 1.0, m = 2.0, l = 0.5;
  const double I = (1.0 / 3.0) * m * l * l;
  const double a1 = M + m, a2 = m * l, a3 = I + m * l * l;
  const double Den = a1 * a3 - a2 * a2;
  const double A_tau = a3 / (r * Den) - a2 / Den;
  const double A_th = -(a2 * m * g * l) / Den;
  const double B_tau = -a2 / (r * Den) + a1 / Den;
  const double B_th = (a1 * m * g * l) / Den;
  const double xdd = A_tau * u[0] + A_th * x[2];
  const double thdd = B_tau * u[0] + B_th * x[2];
  o[0] = x[0] + dt * x[1];
  o[1] = x[1] + dt * xdd;
  o[2] = wrap_angle(x[2] + dt * x[3]);
  o[3] = x[3] + dt * thdd;
}

// ---- quadrotor --------------------------------------------------------------
// sin/cos of the three Euler angles, tan(pitch) and the cos(pitch) that both
// the singularity guard and sec(pitch) = 1/cos(pitch) use (systems.py:145-163).
struct QuadTrig {
  double sphi, cphi, sth, cth, tth, spsi, cpsi;
};

HOP_HD inline void quad_trig_phi(double phi, QuadTrig& t) { sin_cos(phi, t.sphi, t.cphi); }
template <bool FAST = false>
HOP_HD inline void quad_trig_th(double th, QuadTrig& t) {
  sin_cos(th, t.sth, t.cth);
  if constexpr (FAST) t.tth = tan_sc(th, t.sth, t.cth);
  else t.tth = tan(th);
}
HOP_HD inline void quad_trig_psi(double psi, QuadTrig& t) { sin_cos(psi, t.spsi, t.cpsi); }
template <bool FAST = false>
HOP_HD inline QuadTrig quad_trig(const double* x) {
  QuadTrig t;
  quad_trig_phi(x[6], t);
  quad_trig_th<FAST>(x[7], t);
  quad_trig_psi(x[8], t);
  return t;
}

// F with the trigonometry of (x[6], x[7], x[8]) given.  Products against
// structural zeros of I, I^-1 and e3 thrust are dropped: a 0 * finite term adds
// +-0, which changes no sum (guards keep every operand finite).
HOP_HD inline void f_quadrotor_t(const double* x, const double* u, double dt, const QuadTrig& t,
                                 double* o) {
  HOP_DYN_BEGIN
  const double m = 1.0, g = 9.81, Ix = 0.02, Iy = 0.02, Iz = 0.04, kv = 0.05, kw = 0.01;
  bool fin = true;
  double nrm2 = 0.0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    fin = fin && finite_d(x[i]);
    nrm2 += x[i] * x[i];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) fin = fin && finite_d(u[j]);
  const double w0 = x[9], w1 = x[10], w2 = x[11];
  // guards (systems.py:175-191): non-finite input, ||x|| > 1e6, |cos(pitch)| <
  // 1e-3, any |omega| > 1e3 -> all-NaN next state
  if (!fin || sqrt(nrm2) > 1e6 || fabs(t.cth) < 1e-3 || fabs(w0) > 1e3 || fabs(w1) > 1e3 ||
      fabs(w2) > 1e3) {
    const double nan = __builtin_nan("");
#pragma unroll
    for (int i = 0; i < 12; ++i) o[i] = nan;
    return;
  }
  const double thrust = u[0];
  // third column of Rb = (Rz Ry) Rx, Rx[:, 2] = [0, -sphi, cphi]; each entry of
  // Rz Ry is one product (cpsi cth, -spsi, cpsi sth / spsi cth, cpsi, spsi sth /
  // -sth, 0, cth), Rb's are BLAS's chain fma(a2, b2, fma(a1, b1, a0 b0))
  const double rb02 = __builtin_fma(t.cpsi * t.sth, t.cphi, (-t.spsi) * (-t.sphi));
  const double rb12 = __builtin_fma(t.spsi * t.sth, t.cphi, t.cpsi * (-t.sphi));
  const double rb22 = t.cth * t.cphi;
  // acc = Rb (e3 thrust) / m - [0, 0, g] - kv vel  (e3 thrust = [0, 0, thrust])
  const double acc0 = rb02 * thrust / m - 0.0 - kv * x[3];
  const double acc1 = rb12 * thrust / m - 0.0 - kv * x[4];
  const double acc2 = rb22 * thrust / m - g - kv * x[5];
  // eulerdot = Tmat(phi, th) omg, sec(th) = 1 / cos(th).  NumPy's 3x3 gemv goes
  // to OpenBLAS's short-column tail, y = fma(a2, x2, fma(a0, x0, a1 x1))
  const double sec = 1.0 / t.cth;
  const double ed0 = __builtin_fma(t.cphi * t.tth, w2, w0 + t.sphi * t.tth * w1);
  const double ed1 = __builtin_fma(-t.sphi, w2, t.cphi * w1);
  const double ed2 = __builtin_fma(t.cphi * sec, w2, (t.sphi * sec) * w1);
  // omgdot = I^-1 (tau - omg x (I omg)) - kw omg  (diagonal I)
  const double iw0 = Ix * w0, iw1 = Iy * w1, iw2 = Iz * w2;
  const double v0 = u[1] - (w1 * iw2 - w2 * iw1);
  const double v1 = u[2] - (w2 * iw0 - w0 * iw2);
  const double v2 = u[3] - (w0 * iw1 - w1 * iw0);
  const double od0 = (1.0 / Ix) * v0 - kw * w0;
  const double od1 = (1.0 / Iy) * v1 - kw * w1;
  const double od2 = (1.0 / Iz) * v2 - kw * w2;
  o[0] = x[0] + dt * x[3];
  o[1] = x[1] + dt * x[4];
  o[2] = x[2] + dt * x[5];
  o[3] = x[3] + dt * acc0;
  o[4] = x[4] + dt * acc1;
  o[5] = x[5] + dt * acc2;
  o[6] = x[6] + dt * ed0;
  o[7] = x[7] + dt * ed1;
  o[8] = x[8] + dt * ed2;
  o[9] = x[9] + dt * od0;
  o[10] = x[10] + dt * od1;
  o[11] = x[11] + dt * od2;
}

template <bool FAST = false>
HOP_HD inline void f_quadrotor(const double* x, const double* u, double dt, double* o) {
  f_quadrotor_t(x, u, dt, quad_trig<FAST>(x), o);
}

// FAST: the line search's rollouts (tan from sin / cos)
template <int SYS, bool FAST = false>
HOP_HD inline void eval(const double* x, const double* u, double dt, double* o) {
  if constexpr (SYS == kDI) f_di(x, u, dt, o);
  else if constexpr (SYS == kCartpole) f_cartpole(x, u, dt, o);
  else if constexpr (SYS == kQuadrotor) f_quadrotor<FAST>(x, u, dt, o);
  else if constexpr (SYS == kPointmass) f_pointmass(x, u, dt, o);
  else f_segway(x, u, dt, o);
}

// ---- finite-difference columns (linearization.py:177-262) ------------------
// Trig slots of one step for the quadrotor: [0, 7) the base point, then the
// moved angle of the columns j = 6, 7, 8 at v + h (slots 7..13) and, for central
// differences, at v - h (14..20): phi (s, c), th (s, c, t), psi (s, c).
constexpr int kTrigBase = 7, kTrigSet = 7;
HOP_HD constexpr int trig_slots(int sys, bool central) {
  return sys == kQuadrotor ? (central ? kTrigBase + 2 * kTrigSet : kTrigBase + kTrigSet) : 0;
}
// number of trig jobs per step: the base point and one per moved angle and sign
HOP_HD constexpr int trig_jobs(int sys, bool central) {
  return sys == kQuadrotor ? (central ? 7 : 4) : 0;
}

// job 0: base trig of x; job 1 + 3 * sgn + a: angle a of x moved by +h (sgn 0)
// or -h (sgn 1), h = fd_step(x[6 + a]) as the column it serves computes it.
HOP_HD inline void quad_trig_job(const double* x, int job, double epsx, double relx,
                                 double* ts) {
  HOP_DYN_BEGIN
  if (job == 0) {
    const QuadTrig t = quad_trig(x);
    ts[0] = t.sphi, ts[1] = t.cphi, ts[2] = t.sth, ts[3] = t.cth, ts[4] = t.tth;
    ts[5] = t.spsi, ts[6] = t.cpsi;
    return;
  }
  const int sgn = (job - 1) / 3, ax = (job - 1) % 3;
  const double v = x[6 + ax];
  const double h = fd_step(v, epsx, relx);
  const double w = sgn == 0 ? v + h : v - h;
  double* o = ts + kTrigBase + sgn * kTrigSet;
  if (ax == 0) sin_cos(w, o[0], o[1]);
  else if (ax == 1) sin_cos(w, o[2], o[3]), o[4] = tan(w);
  else sin_cos(w, o[5], o[6]);
}

// the QuadTrig of column j's evaluation point: the base values, with the moved
// angle's values when j is an Euler angle (sgn 0: +h, 1: -h)
HOP_HD inline QuadTrig quad_trig_col(const double* ts, int j, int sgn) {
  QuadTrig t{ts[0], ts[1], ts[2], ts[3], ts[4], ts[5], ts[6]};
  const double* o = ts + kTrigBase + sgn * kTrigSet;
  if (j == 6) t.sphi = o[0], t.cphi = o[1];
  if (j == 7) t.sth = o[2], t.cth = o[3], t.tth = o[4];
  if (j == 8) t.spsi = o[5], t.cpsi = o[6];
  return t;
}

template <int SYS>
HOP_HD inline void eval_col(const double* x, const double* u, double dt, const double* ts, int j,
                            int sgn, double* o) {
  if constexpr (SYS == kQuadrotor) f_quadrotor_t(x, u, dt, quad_trig_col(ts, j, sgn), o);
  else eval<SYS>(x, u, dt, o);
}

// Column j of [A | B] at (x, u) (j < n: x_j, else u_{j-n}):
//   forward  linearization.py:241-258  (F(v + h e_j) - f0) / h, where v + h e_j
//            adds h * 0.0 to the other entries like x + hi * I_n[i]; the whole
//            column is NaN when f0 is not finite (245-250)
//   central  linearization.py:195-208  (F(v + h e_j) - F(v - h e_j)) / (2 h)
// h = fd_step(v_j).  Register arrays are only indexed by unrolled constants.
template <int SYS, bool CEN>
HOP_HD inline void fd_col(const double* x, const double* u, const double* f0, bool f0_finite,
                          const double* ts, double dt, int j, double epsx, double epsu,
                          double relx, double relu, double* col) {
  HOP_DYN_BEGIN
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  double xp[n], up[m], fp[n];
  const bool onx = j < n;
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < n; ++i) v = i == j ? x[i] : v;
#pragma unroll
  for (int i = 0; i < m; ++i) v = i + n == j ? u[i] : v;
  const double h = onx ? fd_step(v, epsx, relx) : fd_step(v, epsu, relu);
  if constexpr (!CEN) {
    if (!f0_finite) {
#pragma unroll
      for (int i = 0; i < n; ++i) col[i] = __builtin_nan("");
      return;
    }
#pragma unroll
    for (int i = 0; i < n; ++i) xp[i] = onx ? x[i] + (i == j ? h : 0.0) : x[i];
#pragma unroll
    for (int i = 0; i < m; ++i) up[i] = onx ? u[i] : u[i] + (i + n == j ? h : 0.0);
    eval_col<SYS>(xp, up, dt, ts, j, 0, fp);
#pragma unroll
    for (int i = 0; i < n; ++i) col[i] = (fp[i] - f0[i]) / h;
  } else {
    double fm[n];
#pragma unroll
    for (int i = 0; i < n; ++i) xp[i] = i == j ? x[i] + h : x[i];
#pragma unroll
    for (int i = 0; i < m; ++i) up[i] = i + n == j ? u[i] + h : u[i];
    eval_col<SYS>(xp, up, dt, ts, j, 0, fp);
#pragma unroll
    for (int i = 0; i < n; ++i) xp[i] = i == j ? x[i] - h : x[i];
#pragma unroll
    for (int i = 0; i < m; ++i) up[i] = i + n == j ? u[i] - h : u[i];
    eval_col<SYS>(xp, up, dt, ts, j, 1, fm);
#pragma unroll
    for (int i = 0; i < n; ++i) col[i] = (fp[i] - fm[i]) / (2.0 * h);
  }
}

}  // namespace dyn
}  // namespace hop
