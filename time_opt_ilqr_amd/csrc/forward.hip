// Forward pass of the time-optimal iLQR on the device:
//   rollout                    solver.py:42-62    hop_rollout_f64
//   cost_timeopt_true          solver.py:65-102   hop_cost_true_f64
//   forward_linesearch_fixedT  solver.py:233-286  hop_forward_linesearch_f64
//   extra_stage_cost of the point-mass maker (systems.py:271-293)
//                                                 hop_obstacle_cost_f64
// plus the accept / Levenberg-Marquardt / stop-rule bookkeeping of the outer
// loop (solver.py:737-752), hop_ilqr_accept_f64.
//
// The rollouts are sequential in k, so the parallelism is across problems and
// across the line-search step sizes: pass 1 gives one lane to every
// (problem, alpha) pair -- the reference tries the alphas in order and keeps the
// first whose true cost beats J_old; running them side by side and taking the
// smallest accepted index is the same choice -- plus one lane per problem for
// J_old.  Each lane keeps its candidate trajectory in a workspace row
// [problem][alpha][X' | U'] that it writes sequentially, so the writes fill L2
// lines while the lane walks the horizon.  Pass 2 (one workgroup per problem)
// picks the winner and copies its row (or X, U when nothing was accepted) into
// X', U' with coalesced loads and stores.
//
// The dynamics are dynamics.hpp's (bit-exact with NumPy for the libm-free
// systems); the cost follows the reference's evaluation order per step,
// c += (0.5 e.Qe + 0.5 du.Rdu) + w, then + c_extra.
#include <math.h>

#include "hop_device.hpp"
#include "hop_kernels.hpp"
#include "dynamics.hpp"

namespace hop {
namespace fwd {

using namespace hop::dyn;

constexpr int TPB = 64;

__device__ inline bool fin(double v) { return v - v == 0.0; }

// 0.5 v.(M v) for a row-major k x k matrix M (reference: 0.5 * float(v @ (M @ v)))
template <int K>
__device__ inline double half_quad(const double* __restrict__ M, const double* v) {
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    double r = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) r = fma(M[i * K + j], v[j], r);
    acc = fma(v[i], r, acc);
  }
  return 0.5 * acc;
}

// the same for a diagonal M (off-diagonal entries exactly 0): the dense chain's
// fma(0, v_j, r) terms add exact zeros, so this is bitwise the same number
template <int K>
__device__ inline double half_quad_diag(const double* __restrict__ M, const double* v) {
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < K; ++i) acc = fma(v[i], M[i * K + i] * v[i], acc);
  return 0.5 * acc;
}

// sum of the Gaussian obstacle penalties at position (px, py) (systems.py:271-293, c only)
__device__ inline double obstacle_c(const double* __restrict__ obs, int n_obs, double px,
                                    double py) {
  double c = 0.0;
  for (int o = 0; o < n_obs; ++o) {
    const double dx = px - obs[4 * o], dy = py - obs[4 * o + 1], r = obs[4 * o + 2];
    const double s = dx * dx + dy * dy;
    c += obs[4 * o + 3] * exp(-s / (2.0 * r * r));
  }
  return c;
}

// WM >= 0: the wrap mask is a compile-time constant (the system's default
// wrap_idx), so unwrapped components cost nothing; WM = -1: runtime mask (every
// component's wrap is evaluated and selected)
template <int n, int WM = -1>
__device__ inline void wrap_err(const double* a, const double* b, unsigned mask, double* e) {
  const unsigned mk = WM >= 0 ? (unsigned)WM : mask;
#pragma unroll
  for (int i = 0; i < n; ++i) {
    const double d = a[i] - b[i];
    e[i] = (mk >> i) & 1u ? wrap_angle(d) : d;
  }
}

// running-cost increment of step k (solver.py:87-95); false if e or du is not finite
// SH: every cost block is shared by the batch (all batch strides 0), so the block
// addresses are wave-uniform and the compiler reads them through the scalar cache
// (stage_inc_e: the same with the wrapped error e given)
template <int n, int m, bool SH = false>
__device__ inline bool stage_inc_e(const CostArgs& c, long long b_, const double* x,
                                   const double* e, const double* u, double& acc, bool diag) {
  const long long b = SH ? 0 : b_;
  double du[m];
  const double* ur = c.u_ref + b * c.ur_bs;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < n; ++i) ok = ok && fin(e[i]);
#pragma unroll
  for (int i = 0; i < m; ++i) {
    du[i] = u[i] - ur[i];
    ok = ok && fin(du[i]);
  }
  const double q = diag ? half_quad_diag<n>(c.Q + b * c.q_bs, e) : half_quad<n>(c.Q + b * c.q_bs, e);
  const double r =
      diag ? half_quad_diag<m>(c.R + b * c.r_bs, du) : half_quad<m>(c.R + b * c.r_bs, du);
  acc += (q + r) + c.w[b * c.w_bs];
  if (c.obs) acc += obstacle_c(c.obs, c.n_obs, x[0], x[1]);
  return ok;
}

template <int n, int m, bool SH = false, int WM = -1>
__device__ inline bool stage_inc(const CostArgs& c, long long b_, const double* x,
                                 const double* u, double& acc, bool diag = false) {
  const long long b = SH ? 0 : b_;
  double e[n], du[m];
  wrap_err<n, WM>(x, c.xg + b * c.xg_bs, c.wrap_mask, e);
  const double* ur = c.u_ref + b * c.ur_bs;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < n; ++i) ok = ok && fin(e[i]);
#pragma unroll
  for (int i = 0; i < m; ++i) {
    du[i] = u[i] - ur[i];
    ok = ok && fin(du[i]);
  }
  const double q = diag ? half_quad_diag<n>(c.Q + b * c.q_bs, e) : half_quad<n>(c.Q + b * c.q_bs, e);
  const double r =
      diag ? half_quad_diag<m>(c.R + b * c.r_bs, du) : half_quad<m>(c.R + b * c.r_bs, du);
  acc += (q + r) + c.w[b * c.w_bs];
  if (c.obs) acc += obstacle_c(c.obs, c.n_obs, x[0], x[1]);
  return ok;
}

template <int n, bool SH = false, int WM = -1>
__device__ inline double terminal_cost(const CostArgs& c, long long b_, const double* x,
                                       bool& ok, bool diag = false) {
  const long long b = SH ? 0 : b_;
  double e[n];
  wrap_err<n, WM>(x, c.xg + b * c.xg_bs, c.wrap_mask, e);
#pragma unroll
  for (int i = 0; i < n; ++i) ok = ok && fin(e[i]);
  return diag ? half_quad_diag<n>(c.Qf + b * c.qf_bs, e) : half_quad<n>(c.Qf + b * c.qf_bs, e);
}

// cost_timeopt_true over X [N+1][n], U [N][m] of problem b at horizon T
template <int n, int m>
__device__ double cost_true(const CostArgs& c, long long b, const double* X, const double* U,
                            int T) {
  if (T <= 0) return INFINITY;
  double acc = 0.0;
  bool ok = true;
  for (int k = 0; k < T; ++k) {
    double x[n], u[m];
#pragma unroll
    for (int i = 0; i < n; ++i) x[i] = X[k * n + i];
#pragma unroll
    for (int i = 0; i < m; ++i) u[i] = U[k * m + i];
    ok = stage_inc<n, m>(c, b, x, u, acc) && ok;
  }
  double xT[n];
#pragma unroll
  for (int i = 0; i < n; ++i) xT[i] = X[T * n + i];
  const double t = terminal_cost<n>(c, b, xT, ok);
  return ok ? acc + t : INFINITY;
}

// ---------------------------------------------------------------- rollout
template <int SYS>
__global__ __launch_bounds__(TPB) void rollout_kernel(RolloutArgs a) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  const long long b = (long long)blockIdx.x * TPB + threadIdx.x;
  if (b >= a.batch) return;
  const double* U = a.U + b * a.N * m;
  double* X = a.X + b * (long long)(a.N + 1) * n;
  double x[n];
#pragma unroll
  for (int i = 0; i < n; ++i) X[i] = x[i] = a.x0[b * a.x0_bs + i];
  int k = 0;
  for (; k < a.N; ++k) {
    double u[m], xn[n];
#pragma unroll
    for (int i = 0; i < m; ++i) u[i] = U[k * m + i];
    eval<SYS>(x, u, a.dt, xn);  // the trajectory the linearisation and select consume
    bool ok = true;
    double ss = 0.0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      ok = ok && fin(xn[i]);
      ss = fma(xn[i], xn[i], ss);
    }
    // reference: not finite or np.linalg.norm(xn) > max_state_norm -> X[k+1:] = NaN
    if (!ok || sqrt(ss) > a.max_state_norm) break;
#pragma unroll
    for (int i = 0; i < n; ++i) X[(k + 1) * n + i] = x[i] = xn[i];
  }
  for (int r = k + 1; r <= a.N; ++r)
#pragma unroll
    for (int i = 0; i < n; ++i) X[r * n + i] = NAN;
}

// ---------------------------------------------------------------- cost
template <int SYS>
__global__ __launch_bounds__(TPB) void cost_kernel(CostArgs c, const double* X, const double* U,
                                                   const int* T, long long batch, int N,
                                                   double* J) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  const long long b = (long long)blockIdx.x * TPB + threadIdx.x;
  if (b >= batch) return;
  const int t = T[b];
  J[b] = t > N ? NAN
               : cost_true<n, m>(c, b, X + b * (long long)(N + 1) * n, U + b * (long long)N * m,
                                 t);
}

// ---------------------------------------------------------------- line search
// pass 1: lane q = b * n_alpha + slot rolls out step size `slot`; lane
// batch * n_alpha + b computes problem b's J_old.
// Step k+1's rows of X, U, K, k are loaded at the top of step k (register double
// buffer), so their latency hides under step k's dynamics and cost.
// the two lanes of a (problem, alpha) pair exchange values through a DPP quad
// permutation [1, 0, 3, 2] (lanes 2j and 2j + 1 swap)
__device__ inline double pair_swap(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// PAIR (quadrotor, the default there): two lanes per (problem, alpha) rollout.  Lane h
// forms controls 2h, 2h + 1 (its two rows of K_k: half the K.dx chains, half the
// prefetched rows and their registers) and one of the two independent sin/cos pairs
// (h = 0: roll, h = 1: yaw); the partner's values arrive by pair_swap.  Everything
// else -- the error, the cost, the pitch's sin/cos/tan, the dynamics -- both lanes
// evaluate with the same operations in the same order, so the rollout, J and the
// rows written are bit-identical to the one-lane form.  Lane h writes half of each
// X', U' row.
template <int SYS, bool SH, int WM, bool PAIR = false>
__global__ __launch_bounds__(TPB) void linesearch_kernel(FwdArgs a) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  static_assert(!PAIR || (n == 12 && m == 4), "two-lane rollouts: the quadrotor");
  // shared cost blocks staged in LDS once per workgroup (every lane reads the same
  // address: a broadcast, no bank conflicts); per-problem blocks stay in HBM
  constexpr int NQ = n * n, NR = m * m;
  __shared__ double sc[2 * NQ + NR + n + m + 1];
  CostArgs cl = a.c;
  bool diag = false;
  if constexpr (SH) {
    const CostArgs& c = a.c;
    for (int i = threadIdx.x; i < 2 * NQ + NR + n + m + 1; i += TPB) {
      double v;
      if (i < NQ) v = c.Q[i];
      else if (i < 2 * NQ) v = c.Qf[i - NQ];
      else if (i < 2 * NQ + NR) v = c.R[i - 2 * NQ];
      else if (i < 2 * NQ + NR + n) v = c.xg[i - 2 * NQ - NR];
      else if (i < 2 * NQ + NR + n + m) v = c.u_ref[i - 2 * NQ - NR - n];
      else v = c.w[0];
      sc[i] = v;
    }
    __syncthreads();
    // every reference system has diagonal Q, R and terminal weight: then the cost
    // reads only the diagonals (wave-uniform branch, bitwise the same value)
    bool dg = true;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (i != j) dg = dg && sc[i * n + j] == 0.0 && sc[NQ + i * n + j] == 0.0;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < m; ++j)
        if (i != j) dg = dg && sc[2 * NQ + i * m + j] == 0.0;
    diag = dg;
    cl.Q = sc;
    cl.Qf = sc + NQ;
    cl.R = sc + 2 * NQ;
    cl.xg = sc + 2 * NQ + NR;
    cl.u_ref = sc + 2 * NQ + NR + n;
    cl.w = sc + 2 * NQ + NR + n + m;
  }
  // lanes [0, batch * n_alpha): (problem, step size) rollouts; the J_old lanes of
  // every problem come after them, so no wave mixes the two loops (a mixed wave
  // runs both, one after the other)
  constexpr int LP = PAIR ? 2 : 1;  // lanes per (problem, alpha) rollout
  const long long q = (long long)blockIdx.x * TPB + threadIdx.x;
  const long long nr = a.batch * a.n_alpha;
  if (q >= LP * nr + a.batch) return;
  const bool roll = q < LP * nr;
  const long long pr = roll ? q / LP : 0;
  const int h = PAIR ? (int)(q & 1) : 0;
  const long long b = roll ? pr / a.n_alpha : q - LP * nr;
  const int slot = roll ? (int)(pr - b * a.n_alpha) : a.n_alpha;
  const int N = a.N;
  const double* X = a.X + b * (long long)(N + 1) * n;
  const double* U = a.U + b * (long long)N * m;
  const int T = a.T_star[b];
  const bool active = (a.active == nullptr || a.active[b] != 0) && T >= 0 && T <= N;
  if (slot == a.n_alpha) {
    a.J_old[b] = T > N ? NAN : cost_true<n, m>(a.c, b, X, U, T);
    return;
  }
  double* J = a.Jc + b * a.n_alpha + slot;
  if (!active) {
    if (h == 0) *J = NAN;
    return;
  }
  const double alpha = a.alphas[slot];
  const double* K = a.K + b * (long long)N * m * n;
  const double* kf = a.kff + b * (long long)N * m;
  const long long row = (long long)(N + 1) * n + (long long)N * m;
  double* Xc = a.ws + (b * a.n_alpha + slot) * row;
  double* Uc = Xc + (long long)(N + 1) * n;
  if constexpr (PAIR) {
    constexpr int HN = n / 2, HM = m / 2;
    double x[n];
#pragma unroll
    for (int i = 0; i < n; ++i) x[i] = X[i];
#pragma unroll
    for (int i = 0; i < HN; ++i) Xc[HN * h + i] = h ? x[HN + i] : x[i];
    double acc = 0.0;
    bool ok = true;
    double nu[HM], nk[HM], nx[n], nK[HM * n];  // this lane's rows of the next step
    auto load = [&](int k) {
#pragma unroll
      for (int j = 0; j < HM; ++j) nu[j] = U[k * m + HM * h + j], nk[j] = kf[k * m + HM * h + j];
#pragma unroll
      for (int i = 0; i < n; ++i) nx[i] = X[k * n + i];
#pragma unroll
      for (int i = 0; i < HM * n; ++i) nK[i] = K[(long long)k * m * n + HM * h * n + i];
    };
    if (N > 0) load(0);
    for (int k = 0; k < N; ++k) {
      if constexpr (SH) asm volatile("" ::: "memory");
      double uh[HM];
      double e[n];  // the stage cost's error x - xg (k < T)
      if (k < T) {
        // the wrapped components split over the pair: lane 0 wraps dx = x - x_ref,
        // lane 1 the cost's e = x - xg (same operations, exchanged)
        static_assert(WM >= 0, "two-lane rollouts: the default wrap mask");
        const double* xgp = cl.xg + (SH ? 0 : b * cl.xg_bs);
        double dx[n];
#pragma unroll
        for (int i = 0; i < n; ++i) {
          if ((WM >> i) & 1) {
            const double wv = wrap_angle(x[i] - (h ? xgp[i] : nx[i]));
            const double o = pair_swap(wv);
            dx[i] = h ? o : wv;
            e[i] = h ? wv : o;
          } else {
            dx[i] = x[i] - nx[i];
            e[i] = x[i] - xgp[i];
          }
        }
#pragma unroll
        for (int j = 0; j < HM; ++j) {
          double r = 0.0;
#pragma unroll
          for (int i = 0; i < n; ++i) r = fma(nK[j * n + i], dx[i], r);
          uh[j] = nu[j] + (r + alpha * nk[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < HM; ++j) uh[j] = nu[j];
      }
      double u[m];
#pragma unroll
      for (int j = 0; j < HM; ++j) {
        const double o = pair_swap(uh[j]);
        u[j] = h ? o : uh[j];
        u[HM + j] = h ? uh[j] : o;
      }
      if (k + 1 < N) load(k + 1);
      if (k < T) ok = stage_inc_e<n, m, SH>(cl, b, x, e, u, acc, diag) && ok;
#pragma unroll
      for (int j = 0; j < HM; ++j) Uc[k * m + HM * h + j] = uh[j];
      // trigonometry: roll (h = 0) or yaw (h = 1) on this lane, the pitch on both
      QuadTrig t;
      const double ang = h ? x[8] : x[6];
      double sa, ca;
      sin_cos(ang, sa, ca);
      const double so = pair_swap(sa), co = pair_swap(ca);
      t.sphi = h ? so : sa, t.cphi = h ? co : ca;
      t.spsi = h ? sa : so, t.cpsi = h ? ca : co;
      quad_trig_th<true>(x[7], t);
      double xn[n];
      f_quadrotor_t(x, u, a.dt, t, xn);
      bool f = true;
#pragma unroll
      for (int i = 0; i < n; ++i) f = f && fin(xn[i]);
      if (!f) {  // rejected step size (both lanes see the same xn)
        if (h == 0) *J = NAN;
        return;
      }
#pragma unroll
      for (int i = 0; i < HN; ++i) Xc[(k + 1) * n + HN * h + i] = h ? xn[HN + i] : xn[i];
#pragma unroll
      for (int i = 0; i < n; ++i) x[i] = xn[i];
      if (k + 1 == T) acc += terminal_cost<n, SH, WM>(cl, b, x, ok, diag);
    }
    if (T == 0) ok = false;
    if (h == 0) *J = ok ? acc : INFINITY;
    return;
  }
  double x[n];
#pragma unroll
  for (int i = 0; i < n; ++i) Xc[i] = x[i] = X[i];
  double acc = 0.0;
  bool ok = true;  // finite e / du along the horizon
  double nu[m], nx[n], nk[m], nK[m * n];  // rows of the next step
  auto load = [&](int k) {
#pragma unroll
    for (int i = 0; i < m; ++i) nu[i] = U[k * m + i], nk[i] = kf[k * m + i];
#pragma unroll
    for (int i = 0; i < n; ++i) nx[i] = X[k * n + i];
#pragma unroll
    for (int i = 0; i < m * n; ++i) nK[i] = K[(long long)k * m * n + i];
  };
  if (N > 0) load(0);
  for (int k = 0; k < N; ++k) {
    // the shared cost blocks are re-read from LDS every step rather than hoisted
    // into (spilling) registers
    if constexpr (SH) asm volatile("" ::: "memory");
    double u[m], xn[n];
    if (k < T) {
      double dx[n];
      wrap_err<n, WM>(x, nx, a.c.wrap_mask, dx);
      // U'[k] = U[k] + (K_k dx + alpha k_k)   (solver.py:262-263)
#pragma unroll
      for (int i = 0; i < m; ++i) {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < n; ++j) r = fma(nK[i * n + j], dx[j], r);
        u[i] = nu[i] + (r + alpha * nk[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < m; ++i) u[i] = nu[i];
    }
    // step k's rows are dead: load step k+1's under this step's cost and dynamics
    if (k + 1 < N) load(k + 1);
    if (k < T) ok = stage_inc<n, m, SH, WM>(cl, b, x, u, acc, diag) && ok;
#pragma unroll
    for (int i = 0; i < m; ++i) Uc[k * m + i] = u[i];
    eval<SYS, true>(x, u, a.dt, xn);
    bool f = true;
#pragma unroll
    for (int i = 0; i < n; ++i) f = f && fin(xn[i]);
    if (!f) {  // rejected step size (solver.py:265-267, 272-274)
      *J = NAN;
      return;
    }
#pragma unroll
    for (int i = 0; i < n; ++i) Xc[(k + 1) * n + i] = x[i] = xn[i];
    if (k + 1 == T) {
      acc += terminal_cost<n, SH, WM>(cl, b, x, ok, diag);
    }
  }
  if (T == 0) ok = false;  // cost_timeopt_true: T* <= 0 -> inf
  *J = ok ? acc : INFINITY;
}

// pass 2: one workgroup per problem: the first alpha with J' < J_old, then the copy
template <int SYS>
__global__ __launch_bounds__(256) void linesearch_pick_kernel(FwdArgs a) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  const long long b = blockIdx.x;
  __shared__ int s_win;
  const int N = a.N;
  if (threadIdx.x == 0) {
    const double Jo = a.J_old[b];
    int win = -1;
    for (int s = 0; s < a.n_alpha; ++s) {
      const double Jn = a.Jc[b * a.n_alpha + s];
      if (Jn < Jo) {  // NaN (rejected / inactive) never wins
        win = s;
        break;
      }
    }
    const bool active = (a.active == nullptr || a.active[b] != 0);
    a.accepted[b] = active ? win : -2;
    a.J[b] = win >= 0 ? a.Jc[b * a.n_alpha + win] : Jo;
    s_win = win;
  }
  __syncthreads();
  const int win = s_win;
  const long long nx = (long long)(N + 1) * n, nu = (long long)N * m;
  const double* srcX = win >= 0 ? a.ws + (b * a.n_alpha + win) * (nx + nu) : a.X + b * nx;
  const double* srcU = win >= 0 ? srcX + nx : a.U + b * nu;
  double* dX = a.X_new + b * nx;
  double* dU = a.U_new + b * nu;
  for (long long e = threadIdx.x; e < nx; e += 256) dX[e] = srcX[e];
  for (long long e = threadIdx.x; e < nu; e += 256) dU[e] = srcU[e];
}

// ---------------------------------------------------------------- obstacles
// c, cx, cxx of the point-mass obstacle penalties at `count` states (rows of n)
__global__ __launch_bounds__(256) void obstacle_kernel(ObstacleArgs a) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= a.count) return;
  const int n = a.n;
  const double px = a.X[r * a.x_stride], py = a.X[r * a.x_stride + 1];
  double c = 0.0, g0 = 0.0, g1 = 0.0, h00 = 0.0, h01 = 0.0, h11 = 0.0;
  for (int o = 0; o < a.n_obs; ++o) {
    const double dx = px - a.obs[4 * o], dy = py - a.obs[4 * o + 1], rr = a.obs[4 * o + 2];
    // the reference's groupings: 2.0 * r * r, r * r, r ** 4 (pow)
    const double r2 = rr * rr, r4 = pow(rr, 4.0);
    const double ci = a.obs[4 * o + 3] * exp(-(dx * dx + dy * dy) / (2.0 * rr * rr));
    c += ci;
    g0 += -(ci / r2) * dx;
    g1 += -(ci / r2) * dy;
    h00 += ci * (dx * dx / r4 - 1.0 / r2);
    h01 += ci * (dx * dy / r4 - 0.0 / r2);
    h11 += ci * (dy * dy / r4 - 1.0 / r2);
  }
  if (a.c) a.c[r] = c;
  if (a.cx) {
    double* g = a.cx + r * n;
    for (int i = 0; i < n; ++i) g[i] = 0.0;
    g[0] = g0;
    g[1] = g1;
  }
  if (a.cxx) {
    double* h = a.cxx + r * n * n;
    for (int i = 0; i < n * n; ++i) h[i] = 0.0;
    h[0] = h00;
    h[1] = h01;
    h[n] = h01;
    h[n + 1] = h11;
  }
}

// ---------------------------------------------------------------- accept / LM / stop
// solver.py:737-752 per problem; warm = 1 for the warm-start update (solver.py:548-553:
// J0 is recorded whenever the Riccati pass succeeded and J0 is finite, lm unchanged)
__global__ __launch_bounds__(256) void accept_kernel(AcceptArgs a) {
  const long long b = (long long)blockIdx.x * 256 + threadIdx.x;
  if (b >= a.batch) return;
  if (a.done[b]) return;
  const int H = a.hist_cap;
  int nh = a.n_hist[b];
  const double J = a.J[b];
  const int acc = a.accepted[b];
  double* Jh = a.J_hist + b * H;
  int* Th = a.T_hist + b * H;
  if (a.warm) {
    if (acc != -2 && fin(J) && nh < H) {
      Jh[nh] = J;
      Th[nh] = a.T_star[b];
      a.n_hist[b] = ++nh;
    }
    return;
  }
  if (acc >= 0 && fin(J) && nh < H) {
    a.T_bar[b] = a.T_star[b];
    Jh[nh] = J;
    Th[nh] = a.T_star[b];
    a.n_hist[b] = ++nh;
    const double l = a.lm[b] / 10.0;
    a.lm[b] = l > 1e-12 ? l : 1e-12;
  } else {
    a.lm[b] = a.lm[b] * 10.0;
  }
  if (nh >= 2) {
    const double rel = fabs(Jh[nh - 1] - Jh[nh - 2]) / (fabs(Jh[nh - 2]) + 1e-12);
    if (rel < 1e-4 && nh >= 3 && Th[nh - 1] == Th[nh - 2] && Th[nh - 2] == Th[nh - 3])
      a.done[b] = 1;
  }
}

// the outer loop's per-iteration masks (hop_ilqr_select_mask): crash marking from the
// select block's status, then the line search's active mask from the Riccati status
__global__ __launch_bounds__(256) void select_mask_kernel(MaskArgs a) {
  const long long b = (long long)blockIdx.x * 256 + threadIdx.x;
  if (b >= a.batch) return;
  int done = a.done[b];
  if (!done && (a.sel_status[b] & (int)(ST_FAIL | ST_NONFINITE))) {
    a.crashed[b] = 1;
    a.done[b] = done = 1;
  }
  a.active[b] = !done && !(a.ric_status[b] & (int)ST_FAIL);
}

template <int SYS>
hipError_t launch_all(int which, const void* args, hipStream_t st) {
  switch (which) {
    case 0: {
      const RolloutArgs& a = *(const RolloutArgs*)args;
      hipLaunchKernelGGL((rollout_kernel<SYS>), dim3((unsigned)((a.batch + TPB - 1) / TPB)),
                         dim3(TPB), 0, st, a);
      break;
    }
    case 1: {
      const CostCall& a = *(const CostCall*)args;
      hipLaunchKernelGGL((cost_kernel<SYS>), dim3((unsigned)((a.batch + TPB - 1) / TPB)),
                         dim3(TPB), 0, st, a.c, a.X, a.U, a.T, a.batch, a.N, a.J);
      break;
    }
    default: {
      const FwdArgs& a = *(const FwdArgs*)args;
      long long lanes = a.batch * (a.n_alpha + 1);
      const CostArgs& c = a.c;
      const bool shared = !c.xg_bs && !c.ur_bs && !c.q_bs && !c.r_bs && !c.qf_bs && !c.w_bs;
      // the reference's wrap_idx of each system (systems.py:48, 110, 228, 263, 347)
      constexpr int WD = SYS == kCartpole || SYS == kSegway ? (1 << 2)
                         : SYS == kQuadrotor                ? (7 << 6)
                                                            : 0;
#ifdef HOP_DEV
      const bool one_lane = g_opt_variant == 93;  // the one-lane quadrotor rollout (A/B)
#else
      constexpr bool one_lane = false;
#endif
      if constexpr (SYS == kQuadrotor) {
        // two lanes per rollout while the launch still gives a SIMD at most one wave
        // (beyond that the SIMDs are full and the duplicated half of the work costs)
        const long long lanes2 = 2 * a.batch * a.n_alpha + a.batch;
        if (shared && c.wrap_mask == (unsigned)WD && !one_lane &&
            (lanes2 + 63) / 64 <= 4 * cu_count(st)) {
          lanes = lanes2;
          hipLaunchKernelGGL((linesearch_kernel<SYS, true, WD, true>),
                             dim3((unsigned)((lanes + TPB - 1) / TPB)), dim3(TPB), 0, st, a);
          hipError_t e = hipGetLastError();
          if (e != hipSuccess) return e;
          hipLaunchKernelGGL((linesearch_pick_kernel<SYS>), dim3((unsigned)a.batch), dim3(256), 0,
                             st, a);
          break;
        }
      }
      const dim3 grid((unsigned)((lanes + TPB - 1) / TPB));
      if (shared && c.wrap_mask == (unsigned)WD)
        hipLaunchKernelGGL((linesearch_kernel<SYS, true, WD>), grid, dim3(TPB), 0, st, a);
      else if (shared)
        hipLaunchKernelGGL((linesearch_kernel<SYS, true, -1>), grid, dim3(TPB), 0, st, a);
      else
        hipLaunchKernelGGL((linesearch_kernel<SYS, false, -1>), grid, dim3(TPB), 0, st, a);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((linesearch_pick_kernel<SYS>), dim3((unsigned)a.batch), dim3(256), 0,
                         st, a);
    }
  }
  return hipGetLastError();
}

}  // namespace fwd

hipError_t dispatch_forward(int sys, int which, const void* args, hipStream_t stream) {
  switch (sys) {
    case dyn::kDI: return fwd::launch_all<dyn::kDI>(which, args, stream);
    case dyn::kCartpole: return fwd::launch_all<dyn::kCartpole>(which, args, stream);
    case dyn::kQuadrotor: return fwd::launch_all<dyn::kQuadrotor>(which, args, stream);
    case dyn::kPointmass: return fwd::launch_all<dyn::kPointmass>(which, args, stream);
    default: return fwd::launch_all<dyn::kSegway>(which, args, stream);
  }
}

hipError_t dispatch_obstacle(const ObstacleArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(fwd::obstacle_kernel, dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0,
                     stream, a);
  return hipGetLastError();
}

hipError_t dispatch_select_mask(const MaskArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(fwd::select_mask_kernel, dim3((unsigned)((a.batch + 255) / 256)), dim3(256),
                     0, stream, a);
  return hipGetLastError();
}

hipError_t dispatch_accept(const AcceptArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(fwd::accept_kernel, dim3((unsigned)((a.batch + 255) / 256)), dim3(256), 0,
                     stream, a);
  return hipGetLastError();
}

}  // namespace hop
