// Host-visible kernel argument blocks and dispatchers (internal to libhop_amd.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/hop.h"

namespace hop {
// test / diagnostic controls (hop_set_options, include/hop.h); 0 = product defaults.
// Per host thread: a launch sees the options of the thread that issues it.
extern thread_local unsigned g_opt_flags;
extern thread_local int g_opt_variant;
inline bool opt(unsigned f) { return (g_opt_flags & f) != 0u; }
// queries that could not read the device's CU count (hop_cu_fallbacks)
extern std::atomic<int> g_cu_fallbacks;
// compute units of the device `stream` belongs to, cached per device id (atomics:
// launches from several host threads may fill the cache at once); the launches
// that pick a layout by waves per SIMD (4 SIMDs per CU) compare against 4 x this.
// A failed query counts in hop_cu_fallbacks() and assumes MI355X's 256 CUs; that
// changes only the layout choice (the results are bit-identical either way).
inline long long cu_count(hipStream_t stream) {
  static std::atomic<int> cached[64] = {};
  int dev = -1;
  if (hipStreamGetDevice(stream, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess)
    dev = -1;
  if (dev < 0 || dev >= 64) {
    g_cu_fallbacks.fetch_add(1, std::memory_order_relaxed);
    return 256;
  }
  int cus = cached[dev].load(std::memory_order_relaxed);
  if (cus > 0) return cus;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0) {
    g_cu_fallbacks.fetch_add(1, std::memory_order_relaxed);
    return 256;  // not cached: the next launch asks again
  }
  cached[dev].store(cus, std::memory_order_relaxed);
  return cus;
}
#ifdef HOP_DEV
inline constexpr bool kDevBuild = true;
#else
inline constexpr bool kDevBuild = false;
#endif
}  // namespace hop

namespace hop {

// Trajectory form of the LFT inputs (augmented.py:10-87 done on the device):
// the raw linearisation and cost terms the augmented blocks are built from.
template <class T>
struct TrajArgs {
  const T* A;      // [B][nalloc][n][n]
  const T* Bm;     // [B][nalloc][n][m]
  const T* ares;   // [B][nalloc][n]    a_k = F(x_k, u_k) - x_{k+1}
  const T* X;      // [B][nalloc+1][n]
  const T* U;      // [B][nalloc][m]
  const T* xg;     // [B or 1][n]
  const T* u_ref;  // [B or 1][m]
  const T* Q;      // [B or 1][n][n]   stage weight (raw; _sym'd in the builder)
  const T* P;      // [B or 1][n][n]   _sym(as_terminal_weight(alpha))
  const T* w;      // [B or 1]         time weight
  const T* qxx_extra;  // [B][nalloc][n][n] or null (extra_stage_cost)
  const T* qx_extra;   // [B][nalloc][n] or null
  const T* c_extra;    // [B][nalloc] or null
  long long xg_bs, ur_bs, q_bs, p_bs, w_bs;
  unsigned wrap_mask;
  T q_reg, rho_reg;
  int n, m;
};

template <class T>
struct AugArgs {
  TrajArgs<T> t;
  long long batch;
  int nalloc, nbuild;
  T* A_aug;   // [B][nbuild][s][s]
  T* B_aug;   // [B][nbuild][s][m]
  T* Q_aug;   // [B][nbuild][s][s]
  T* QT_aug;  // [B][nbuild][s][s]
  T* z0;      // [s] or null: z0 = e_s (augmented.py:57)
};

template <class T>
struct LftArgs {
  const T* A;    // [B][nalloc][s][s]   augmented A_k
  const T* B;    // [B][nalloc][s][m]   augmented B_k
  const T* Q;    // [B][nalloc][s][s]   augmented Q_k
  const T* R;    // R^-1 (r_is_inv) or R_k; batch/step strides in elements
  const T* QT;   // [B][nalloc][s][s]   terminal blocks, QT[k] <-> horizon k+1
  const T* z0;   // [B or 1][s]
  long long r_bstride, r_kstride, z_bstride;
  long long batch;
  int nalloc, n, s, m, max_tries, r_is_inv;
  int t_min, t_max;  // fused argmin window (t_max <= 0: off)
  T* J;              // [B][n]
  int* status;       // [B]
  int* t_star;       // [B] or null
  T* j_star;         // [B] or null
  T* dbg_efg;        // [B][n][3][s][s] or null  (E_k, F_k, G_k)
  T* dbg_pre;        // [B][n][3][s][s] or null  (Ebar_k, Fbar_k, Gbar_k)
  int traj;          // 1: A/B/Q/QT unused, blocks built in-kernel from `tr`
  int cond;          // SchedCond: bit 0 rerun launch (only ST_RERUN problems), bit 1 flag all;
                     // kCondRerunOnly: dispatch_lft_small launches only its LFT rerun
  int tile64;        // 1: A/B/Q/QT in the tile64 layout [B/64][nalloc][block elems][64]
  TrajArgs<T> tr;
};

template <class T>
struct RiccatiArgs {
  const T* A;      // [B][nalloc][n][n]
  const T* Bm;     // [B][nalloc][n][m]
  const T* X;      // [B][nalloc+1][n]
  const T* U;      // [B][nalloc][m]
  const T* xg;     // [B or 1][n]
  const T* u_ref;  // [B or 1][m]
  const T* Q;      // [B or 1][n][n]
  const T* R;      // [B or 1][m][m]
  const T* Qf;     // [B or 1][n][n]  (already as_terminal_weight'ed)
  const T* qxx_extra;  // [B][nalloc][n][n] or null
  const T* qx_extra;   // [B][nalloc][n] or null
  const T* c_extra;    // [B][nalloc] or null
  const int* horizon;  // [B]  L_b (terminal index)
  const T* lm;         // [B]
  long long xg_bstride, uref_bstride, q_bstride, r_bstride, qf_bstride;
  long long batch;
  int nalloc, n, m, mode, reg_max_tries, max_tries;
  unsigned wrap_mask;
  T w_stage;
  T* K;    // [B][nalloc][m][n]
  T* k;    // [B][nalloc][m]
  T* Vxx;  // [B][nalloc+1][n][n] or null
  T* Vx;   // [B][nalloc+1][n] or null
  T* V0;   // [B][nalloc+1] or null
  int* status;  // [B]
  // J-curve form (hop_bruteforce_jcurve_*, solver.py:293-358): when jc_J is set, the
  // generic J-curve kernel's workgroup x runs problem block x / jc_tmax at horizon
  // L = jc_tmax - x % jc_tmax, the exact-size kernel's workgroup x the pair of
  // horizons jc_tmax - h and h + 1 of block x / P (h = x % P, P = ceil(jc_tmax / 2));
  // one horizon per wave at a time, a block's horizons adjacent, longest first;
  // lm is the scalar lm_value, no K / k / V is stored and each (problem, horizon)
  // writes J[b][L-1] = V_0 and its status to jc_status[b][L-1]
  T* jc_J = nullptr;          // [B][jc_tmax]
  int* jc_status = nullptr;   // [B][jc_tmax]
  int jc_tmax = 0;
  T lm_value = T(0);
  // legacy twin (ilqr_propagator.py): chol_solve with 4 jitters, then the
  // least-squares solve of sym(Quu_reg) (np.linalg.lstsq, ilqr_propagator.py:33-43)
  // instead of the crash mark; no finiteness checks (the legacy loops have none);
  // Quu_reg = _sym(Quu) + lm I with lm as given (no 1e-12 floor, no lambda ladder).
  // Runs on the generic kernel only.
  int legacy = 0;
};

// batched finite-difference linearisation (linearize.hip, dynamics.hpp)
struct LinArgs {
  int sys;              // hop::dyn::System
  int central;          // 0 forward differences, 1 central
  double dt, epsx, epsu, relx, relu;
  const double* X;      // [B][nalloc+1][n]
  const double* U;      // [B][nalloc][m]
  long long batch;
  int nalloc, nuse;
  void* A;              // [B][nalloc][n][n]  (tile64: [B/64][nalloc][n n][64] of OT)
  void* B;              // [B][nalloc][n][m]  (tile64: [B/64][nalloc][n m][64])
  void* a_res;          // [B][nalloc][n] or null (tile64: [B/64][nalloc][n][64])
  double* Fx;           // [B][nalloc][n] or null (batch-major only)
  int tile64 = 0;       // 1: tile64 outputs of A, B, a_res + the Xt / Ut copies
  int out_f32 = 0;      // tile64 outputs as fp32 (computed in fp64)
  void* Xt = nullptr;   // [B/64][nalloc+1][n][64]  x_k, k <= nuse
  void* Ut = nullptr;   // [B/64][nalloc][m][64]    u_k, k < nuse
};

// batched dynamics step x' = F(x, u) (row strides in elements)
struct DynArgs {
  int sys;
  double dt;
  const double* X;
  const double* U;
  double* Xn;
  long long count, x_stride, u_stride, xn_stride;
};

// forward pass (forward.hip): rollout / true cost / line search / obstacles / accept
struct CostArgs {
  const double* xg; long long xg_bs;      // [B or 1][n]
  const double* u_ref; long long ur_bs;   // [B or 1][m]
  const double* Q; long long q_bs;        // [B or 1][n][n]
  const double* R; long long r_bs;        // [B or 1][m][m]
  const double* Qf; long long qf_bs;      // [B or 1][n][n]  (as_terminal_weight(alpha))
  const double* w; long long w_bs;        // [B or 1]
  const double* obs; int n_obs;           // [n_obs][4] = (cx, cy, radius, weight) or null
  unsigned wrap_mask;
};
struct RolloutArgs {
  double dt;
  const double* x0; long long x0_bs;      // [B or 1][n]
  const double* U;                        // [B][N][m]
  long long batch; int N;
  double max_state_norm;
  double* X;                              // [B][N+1][n]
};
struct CostCall {
  CostArgs c;
  const double* X; const double* U; const int* T;
  long long batch; int N;
  double* J;
};
struct FwdArgs {
  CostArgs c;
  double dt;
  const double* X; const double* U;       // [B][N+1][n], [B][N][m]
  const int* T_star; const int* active;   // [B]; active nullable
  const double* K; const double* kff;     // [B][N][m][n], [B][N][m]
  double alphas[8]; int n_alpha;
  long long batch; int N;
  double* Jc;                             // workspace [B][n_alpha]
  double* ws;                             // workspace [B][n_alpha][(N+1)n + Nm]
  double* J_old;                          // [B]
  double* X_new; double* U_new; double* J; int* accepted;
};
struct ObstacleArgs {
  const double* X; long long x_stride, count; int n;
  const double* obs; int n_obs;
  double* c; double* cx; double* cxx;     // [count], [count][n], [count][n][n] (nullable)
};
struct AcceptArgs {
  long long batch; int warm, hist_cap;
  const double* J; const int* accepted; const int* T_star;
  double* lm; int* T_bar; double* J_hist; int* T_hist; int* n_hist; int* done;
};
hipError_t dispatch_forward(int sys, int which, const void* args, hipStream_t stream);
hipError_t dispatch_obstacle(const ObstacleArgs& a, hipStream_t stream);
hipError_t dispatch_accept(const AcceptArgs& a, hipStream_t stream);
struct MaskArgs {
  long long batch;
  const int* sel_status; const int* ric_status; int* done; int* crashed; int* active;
};
hipError_t dispatch_select_mask(const MaskArgs& a, hipStream_t stream);
hipError_t dispatch_linearize(const LinArgs& a, hipStream_t stream);
hipError_t dispatch_dynamics(const DynArgs& a, hipStream_t stream);

template <class T>
hipError_t dispatch_lft(const LftArgs<T>& a, hipStream_t stream);
hipError_t dispatch_lft_v2(const LftArgs<double>& a, hipStream_t stream);
// the small-s row-group kernel's hand-overs go to lft_small.hip's LFT instantiation
// (its rerun launch alone): LftArgs.cond = 1 | kCondRerunOnly
constexpr int kCondRerunOnly = 64;
// fp64 s <= 5 augmented blocks on the conditioned kernel's row groups (lft_sweep_v2.hip)
// for batches up to kSmallRowGroupMax (above it lft_small.hip's one problem per lane
// fills the chip and wins: profiles/r06_small_rg_crossover.jsonl); HOP_OPT_SMALL_LANE
// and HOP_OPT_REFERENCE_ASSOC keep every batch on lft_small.hip
constexpr long long kSmallRowGroupMax = 16384;
inline bool cond_small_takes(int s, int m, long long batch) {
  if (batch > kSmallRowGroupMax || opt(HOP_OPT_REFERENCE_ASSOC | HOP_OPT_SMALL_LANE)) return false;
  return (m == 1 && s >= 2 && s <= 5) || (m == 2 && (s == 4 || s == 5));
}
hipError_t dispatch_cond_small(const LftArgs<double>& a, hipStream_t stream);
hipError_t dispatch_lft_v2_f32(const LftArgs<float>& a, hipStream_t stream);
template <class T>
hipError_t dispatch_lft_small(const LftArgs<T>& a, hipStream_t stream);
template <class T>
hipError_t dispatch_augment(const AugArgs<T>& a, hipStream_t stream);
template <class T>
hipError_t dispatch_riccati(const RiccatiArgs<T>& a, hipStream_t stream);
// exact-size fp64 Riccati kernel (n = 12, m = 4; riccati_fast.hip), NotSupported otherwise
hipError_t dispatch_riccati_fast(const RiccatiArgs<double>& a, hipStream_t stream);

}  // namespace hop
