// extern "C" boundary of libhop_amd.so (include/hop.h): argument validation,
// kernel dispatch, the horizon argmin kernel.
#include <algorithm>
#include <atomic>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hop.h"
#include "hop_device.hpp"
#include "hop_kernels.hpp"
#include "dynamics.hpp"

namespace hop {
// per host thread (re-entrant across host threads): a thread's
// hop_set_options changes only the launches that thread issues
thread_local unsigned g_opt_flags = 0u;
thread_local int g_opt_variant = 0;
std::atomic<int> g_cu_fallbacks{0};
}  // namespace hop

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int hip_status(hipError_t e) {
  if (e == hipSuccess) return HOP_OK;
  snprintf(g_err, sizeof(g_err), "HIP error %d: %s", (int)e, hipGetErrorString(e));
  return HOP_E_HIP;
}

// first minimiser of J[t_min-1 .. t_max-1]; NaN wins (np.argmin semantics)
template <class T>
__global__ __launch_bounds__(256) void select_kernel(const T* __restrict__ J, long long batch,
                                                     int ld, int t_min, int t_max,
                                                     int* __restrict__ t_star,
                                                     T* __restrict__ j_star) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const T* row = J + b * ld;
  T best = row[t_min - 1];
  int tb = t_min;
#pragma unroll 1
  for (int t = t_min + 1; t <= t_max; ++t) {
    if (best != best) break;
    const T v = row[t - 1];
    if (v != v || v < best) {
      best = v;
      tb = t;
    }
  }
  t_star[b] = tb;
  if (j_star) j_star[b] = best;
}

template <class T>
int lft_entry(const T* A, const T* B, const T* Q, const T* R, int64_t r_bs, int64_t r_ks,
              int32_t r_inv, const T* QT, const T* z0, int64_t z_bs, int64_t batch,
              int32_t n_alloc, int32_t n_use, int32_t s, int32_t m, int32_t max_tries,
              int32_t t_min, int32_t t_max, T* J, int32_t* status, int32_t* t_star, T* j_star,
              T* dbg_efg, T* dbg_pre, void* stream,
              const hop::TrajArgs<T>* traj = nullptr, bool tile64 = false) {
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (n_use <= 0 || batch == 0) return HOP_OK;  // reference: empty J
  if (s < 1 || s > HOP_MAX_DIM) return fail(HOP_E_SIZE, "s must be in [1, 16]");
  if (m < 1 || m > HOP_MAX_DIM) return fail(HOP_E_SIZE, "m must be in [1, 16]");
  if (n_use > n_alloc) return fail(HOP_E_ARG, "n_use > n_alloc (reference IndexError)");
  if ((!traj && (!A || !B || !Q || !QT || !z0)) || !R || !J || !status)
    return fail(HOP_E_ARG, "null input/output pointer");
  if (r_bs < 0 || r_ks < 0 || z_bs < 0) return fail(HOP_E_ARG, "negative stride");
  if (max_tries < 0 || max_tries > 64) return fail(HOP_E_ARG, "max_tries out of range");
  if (t_max > 0) {
    if (t_min < 1 || t_min > t_max || t_max > n_use)
      return fail(HOP_E_ARG, "need 1 <= t_min <= t_max <= n_use for the fused argmin");
    if (!t_star || !j_star) return fail(HOP_E_ARG, "t_star/j_star required when t_max > 0");
  }
  hop::LftArgs<T> a{};
  a.A = A; a.B = B; a.Q = Q; a.R = R; a.QT = QT; a.z0 = z0;
  a.r_bstride = r_bs; a.r_kstride = r_ks; a.z_bstride = z_bs;
  a.batch = batch; a.nalloc = n_alloc; a.n = n_use; a.s = s; a.m = m;
  a.max_tries = max_tries; a.r_is_inv = r_inv ? 1 : 0;
  a.t_min = t_min; a.t_max = t_max;
  a.J = J; a.status = status; a.t_star = t_star; a.j_star = j_star;
  a.dbg_efg = dbg_efg; a.dbg_pre = dbg_pre;
  if (tile64) {  // the one-problem-per-lane kernels only (their native layout)
    if (dbg_efg || dbg_pre) return fail(HOP_E_ARG, "tile64 layout: no debug outputs");
    if (r_ks != 0) return fail(HOP_E_ARG, "tile64 layout: no per-step R");
    a.tile64 = 1;
    if (traj) {  // raw linearisation in tile64 (hop_lft_sweep_traj_tile64_*)
      a.traj = 1;
      a.tr = *traj;
    }
    const hipError_t e = hop::dispatch_lft_small<T>(a, (hipStream_t)stream);
    if (e != hipErrorNotSupported) return hip_status(e);
    return fail(HOP_E_SIZE, "tile64 layout: no small-s kernel for this (s, m, dtype)");
  }
  if (traj) {  // in-kernel augmentation: the s = 13 and the small-s kernels
    a.traj = 1;
    a.tr = *traj;
    if constexpr (sizeof(T) == 8) {
      const hipError_t e = hop::dispatch_lft_v2(a, (hipStream_t)stream);
      if (e != hipErrorNotSupported) return hip_status(e);
    }
    const hipError_t e = hop::dispatch_lft_small<T>(a, (hipStream_t)stream);
    if (e != hipErrorNotSupported) return hip_status(e);
    return fail(HOP_E_SIZE, "no fused trajectory-form sweep for this shape");
  }
  if (!hop::opt(HOP_OPT_FORCE_GENERIC)) {
    if constexpr (sizeof(T) == 8) {
      const hipError_t e = hop::dispatch_lft_v2(a, (hipStream_t)stream);
      if (e != hipErrorNotSupported) return hip_status(e);
    } else {
      const hipError_t e = hop::dispatch_lft_v2_f32(a, (hipStream_t)stream);
      if (e != hipErrorNotSupported) return hip_status(e);
    }
    const hipError_t e = hop::dispatch_lft_small<T>(a, (hipStream_t)stream);  // s <= 5
    if (e != hipErrorNotSupported) return hip_status(e);
  }
  return hip_status(hop::dispatch_lft<T>(a, (hipStream_t)stream));
}

// tile64 <-> batch-major copy: dst element i of the tiled tensor
// [ntiles][n_alloc][E][64] is src[(64 t + p) n_alloc E + k E + e] (0 past the
// batch); inverse: the same map read the other way
template <class T>
__global__ __launch_bounds__(256) void tile64_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                     long long batch, int n_alloc, int elems,
                                                     int inverse, long long total) {
  const long long stride = (long long)gridDim.x * blockDim.x;
#pragma unroll 1
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int p = (int)(i & 63);
    long long r = i >> 6;
    const int e = (int)(r % elems);
    r /= elems;
    const int k = (int)(r % n_alloc);
    const long long t = r / n_alloc, b = 64 * t + p;
    const long long j = (b * n_alloc + k) * elems + e;
    if (!inverse) dst[i] = b < batch ? src[j] : T(0);
    else if (b < batch) dst[j] = src[i];
  }
}

template <class T>
int tile64_entry(const T* src, T* dst, int64_t batch, int32_t n_alloc, int32_t elems,
                 int32_t inverse, void* stream) {
  if (batch < 0 || n_alloc < 0 || elems < 1) return fail(HOP_E_ARG, "bad batch/n_alloc/elems");
  if (batch == 0 || n_alloc == 0) return HOP_OK;
  if (!src || !dst) return fail(HOP_E_ARG, "null pointer");
  const long long total = (batch + 63) / 64 * 64 * (long long)n_alloc * elems;
  const long long blocks = std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(tile64_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     src, dst, (long long)batch, n_alloc, elems, inverse ? 1 : 0, total);
  return hip_status(hipGetLastError());
}

template <class T>
int select_entry(const T* J, int64_t batch, int32_t ld, int32_t t_min, int32_t t_max,
                 int32_t* t_star, T* j_star, void* stream) {
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (batch == 0) return HOP_OK;
  if (!J || !t_star) return fail(HOP_E_ARG, "null pointer");
  if (t_min < 1 || t_min > t_max || t_max > ld)
    return fail(HOP_E_ARG, "need 1 <= t_min <= t_max <= ld");
  const long long blocks = (batch + 255) / 256;
  hipLaunchKernelGGL(select_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     J, (long long)batch, ld, t_min, t_max, t_star, j_star);
  return hip_status(hipGetLastError());
}

template <class T>
int riccati_entry(const T* A, const T* Bm, const T* X, const T* U, const T* xg, int64_t xg_bs,
                  const T* u_ref, int64_t ur_bs, const T* Q, int64_t q_bs, const T* R,
                  int64_t r_bs, const T* Qf, int64_t qf_bs, const T* qxx_extra,
                  const T* qx_extra, const T* c_extra, const int32_t* horizon, const T* lm,
                  T w_stage, uint32_t wrap_mask, int32_t mode, int32_t reg_max_tries,
                  int64_t batch, int32_t n_alloc, int32_t n, int32_t m, T* K, T* k, T* Vxx,
                  T* Vx, T* V0, int32_t* status, void* stream, int legacy = 0) {
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (batch == 0) return HOP_OK;
  if (n < 1 || n > HOP_MAX_DIM) return fail(HOP_E_SIZE, "n must be in [1, 16]");
  if (m < 1 || m > HOP_MAX_DIM) return fail(HOP_E_SIZE, "m must be in [1, 16]");
  if (n_alloc < 1) return fail(HOP_E_ARG, "n_alloc < 1");
  if (mode != 0 && mode != 1) return fail(HOP_E_ARG, "mode must be 0 or 1");
  if (reg_max_tries < 1) return fail(HOP_E_ARG, "reg_max_tries < 1");
  if (!A || !Bm || !X || !U || !xg || !u_ref || !Q || !R || !Qf || !horizon || !lm || !K || !k ||
      !status)
    return fail(HOP_E_ARG, "null pointer");
  hop::RiccatiArgs<T> a;
  a.A = A; a.Bm = Bm; a.X = X; a.U = U; a.xg = xg; a.u_ref = u_ref; a.Q = Q; a.R = R; a.Qf = Qf;
  a.qxx_extra = qxx_extra; a.qx_extra = qx_extra; a.c_extra = c_extra;
  a.horizon = horizon; a.lm = lm;
  a.xg_bstride = xg_bs; a.uref_bstride = ur_bs; a.q_bstride = q_bs; a.r_bstride = r_bs;
  a.qf_bstride = qf_bs;
  a.batch = batch; a.nalloc = n_alloc; a.n = n; a.m = m; a.mode = mode;
  a.reg_max_tries = reg_max_tries; a.max_tries = 8; a.wrap_mask = wrap_mask; a.w_stage = w_stage;
  a.K = K; a.k = k; a.Vxx = Vxx; a.Vx = Vx; a.V0 = V0; a.status = status;
  a.legacy = legacy;
  // mode 0 never reaches the lstsq fallback (the no-jitter Cholesky gate fails the
  // row first, ilqr_propagator.py:387-390), so only mode 1 carries the m limit
  if (legacy && mode == 1 && m > 11)
    return fail(HOP_E_SIZE, "legacy lstsq fallback: m must be <= 11");
  return hip_status(hop::dispatch_riccati<T>(a, (hipStream_t)stream));
}

// J-curve form: V_0 of the length-T sweep for every T in 1..t_max in one launch
template <class T>
int jcurve_entry(const T* A, const T* Bm, const T* X, const T* U, const T* xg, int64_t xg_bs,
                 const T* u_ref, int64_t ur_bs, const T* Q, int64_t q_bs, const T* R,
                 int64_t r_bs, const T* Qf, int64_t qf_bs, const T* qxx_extra,
                 const T* qx_extra, const T* c_extra, T lm_lambda, T w_stage, uint32_t wrap_mask,
                 int64_t batch, int32_t n_alloc, int32_t n, int32_t m, int32_t t_max, T* J,
                 int32_t* status, void* stream, int legacy = 0) {
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (n < 1 || n > HOP_MAX_DIM) return fail(HOP_E_SIZE, "n must be in [1, 16]");
  if (m < 1 || m > HOP_MAX_DIM) return fail(HOP_E_SIZE, "m must be in [1, 16]");
  if (t_max < 1) return fail(HOP_E_ARG, "t_max < 1");
  // the reference slices A_list[:T] for T <= T_max (an IndexError past N)
  if (t_max > n_alloc) return fail(HOP_E_ARG, "t_max > n_alloc (reference IndexError)");
  // one 256-lane workgroup per (16-problem block, horizon): the dispatch limit is in
  // work-items, so blocks * t_max * 256 must fit 32 bits (the generic kernel's grid;
  // the exact-size kernel's horizon pairs use half of it)
  if ((batch + 15) / 16 * (int64_t)t_max * 256 > 0xFFFFFFFFll)
    return fail(HOP_E_SIZE, "batch * t_max too large for one launch");
  if ((wrap_mask >> n) != 0u) return fail(HOP_E_ARG, "wrap_mask names a state >= n");
  if (batch == 0) return HOP_OK;
  if (!A || !Bm || !X || !U || !xg || !u_ref || !Q || !R || !Qf || !J || !status)
    return fail(HOP_E_ARG, "null pointer");
  hop::RiccatiArgs<T> a;
  a.A = A; a.Bm = Bm; a.X = X; a.U = U; a.xg = xg; a.u_ref = u_ref; a.Q = Q; a.R = R; a.Qf = Qf;
  a.qxx_extra = qxx_extra; a.qx_extra = qx_extra; a.c_extra = c_extra;
  a.horizon = nullptr; a.lm = nullptr;
  a.xg_bstride = xg_bs; a.uref_bstride = ur_bs; a.q_bstride = q_bs; a.r_bstride = r_bs;
  a.qf_bstride = qf_bs;
  a.batch = batch; a.nalloc = n_alloc; a.n = n; a.m = m; a.mode = 1;
  a.reg_max_tries = 1; a.max_tries = 8; a.wrap_mask = wrap_mask; a.w_stage = w_stage;
  a.K = nullptr; a.k = nullptr; a.Vxx = nullptr; a.Vx = nullptr; a.V0 = nullptr;
  a.status = nullptr;
  a.jc_J = J; a.jc_status = status; a.jc_tmax = t_max; a.lm_value = lm_lambda;
  a.legacy = legacy;
  if (legacy && m > 11) return fail(HOP_E_SIZE, "legacy lstsq fallback: m must be <= 11");
  return hip_status(hop::dispatch_riccati<T>(a, (hipStream_t)stream));
}

// ---- trajectory form (augmented.py:10-87 on the device) -------------------
template <class T>
int traj_check(const hop::TrajArgs<T>& t, int64_t batch, int32_t n_alloc, int32_t n_build) {
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (t.n < 1 || t.n + 1 > HOP_MAX_DIM) return fail(HOP_E_SIZE, "n must be in [1, 15]");
  if (t.m < 1 || t.m > HOP_MAX_DIM) return fail(HOP_E_SIZE, "m must be in [1, 16]");
  if (n_build > n_alloc) return fail(HOP_E_ARG, "n_use > n_alloc (reference IndexError)");
  // an empty batch (an empty shard) passes NULL data pointers: nothing is read
  if (batch > 0 && (!t.A || !t.Bm || !t.ares || !t.X || !t.U || !t.xg || !t.u_ref || !t.Q ||
                    !t.P || !t.w))
    return fail(HOP_E_ARG, "null input pointer");
  if (t.xg_bs < 0 || t.ur_bs < 0 || t.q_bs < 0 || t.p_bs < 0 || t.w_bs < 0)
    return fail(HOP_E_ARG, "negative stride");
  if ((t.wrap_mask >> t.n) != 0u) return fail(HOP_E_ARG, "wrap_mask names a state >= n");
  return HOP_OK;
}

template <class T>
hop::TrajArgs<T> traj_args(const T* A, const T* Bm, const T* a_res, const T* X, const T* U,
                           const T* xg, int64_t xg_bs, const T* u_ref, int64_t ur_bs,
                           const T* Q, int64_t q_bs, const T* P, int64_t p_bs, const T* w,
                           int64_t w_bs, const T* qxx_extra, const T* qx_extra,
                           const T* c_extra, uint32_t wrap_mask, T q_reg, T rho_reg, int32_t n,
                           int32_t m) {
  hop::TrajArgs<T> t{};
  t.A = A; t.Bm = Bm; t.ares = a_res; t.X = X; t.U = U; t.xg = xg; t.u_ref = u_ref;
  t.Q = Q; t.P = P; t.w = w; t.qxx_extra = qxx_extra; t.qx_extra = qx_extra;
  t.c_extra = c_extra; t.xg_bs = xg_bs; t.ur_bs = ur_bs; t.q_bs = q_bs; t.p_bs = p_bs;
  t.w_bs = w_bs; t.wrap_mask = wrap_mask; t.q_reg = q_reg; t.rho_reg = rho_reg;
  t.n = n; t.m = m;
  return t;
}

// the sweep builds the blocks itself (no workspace) for these shapes: the
// exact-size s = 13 kernel (fp64) and the small-s instantiations (lft_small.hip).
// fp64 small-s batches the row-group kernel takes go through hop_augment + that
// kernel instead: one problem per lane fills B / 64 SIMDs, and the blocks' round
// trip through HBM costs less than the idle chip below kSmallRowGroupMax (2.7x at
// B = 4,096 on the cart-pole, profiles/r06_small_rg_crossover.jsonl)
bool traj_fused(int32_t n, int32_t m, int32_t elem_bytes, bool has_extra, int64_t batch) {
  if (hop::opt(HOP_OPT_FORCE_GENERIC | HOP_OPT_TRAJ_UNFUSED) || has_extra) return false;
  if (elem_bytes == 8 && n == 12 && m == 4) return true;
  const int s = n + 1;
  if (elem_bytes == 8 && hop::cond_small_takes(s, m, batch)) return false;
  return (s == 2 && m == 1) || (s == 3 && m == 1) || (s == 4 && (m == 1 || m == 2)) ||
         (s == 5 && (m == 1 || m == 2));
}

constexpr int64_t kWsAlign = 256;
int64_t ws_round(int64_t b) { return (b + kWsAlign - 1) / kWsAlign * kWsAlign; }

// workspace of the unfused path: A_aug, B_aug, Q_aug, QT_aug ([batch][n_use]) and z0
int64_t traj_ws_bytes(int64_t batch, int32_t n_use, int32_t n, int32_t m, int32_t elem) {
  const int64_t s = n + 1, steps = batch * (int64_t)n_use;
  return 3 * ws_round(steps * s * s * elem) + ws_round(steps * s * m * elem) + ws_round(s * elem);
}

template <class T>
int augment_entry(const hop::TrajArgs<T>& t, int64_t batch, int32_t n_alloc, int32_t n_build,
                  T* A_aug, T* B_aug, T* Q_aug, T* QT_aug, T* z0, void* stream) {
  const int rc = traj_check(t, batch, n_alloc, n_build);
  if (rc != HOP_OK) return rc;
  if (batch == 0 || n_build <= 0) return HOP_OK;
  if (!A_aug || !B_aug || !Q_aug || !QT_aug) return fail(HOP_E_ARG, "null output pointer");
  hop::AugArgs<T> a{};
  a.t = t; a.batch = batch; a.nalloc = n_alloc; a.nbuild = n_build;
  a.A_aug = A_aug; a.B_aug = B_aug; a.Q_aug = Q_aug; a.QT_aug = QT_aug; a.z0 = z0;
  return hip_status(hop::dispatch_augment<T>(a, (hipStream_t)stream));
}

template <class T>
int lft_traj_entry(const hop::TrajArgs<T>& t, const T* R_inv, int64_t r_bs, int64_t batch,
                   int32_t n_alloc, int32_t n_use, int32_t max_tries, int32_t t_min,
                   int32_t t_max, T* J, int32_t* status, int32_t* t_star, T* j_star,
                   void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = traj_check(t, batch, n_alloc, n_use);
  if (rc != HOP_OK) return rc;
  if (n_use <= 0 || batch == 0) return HOP_OK;
  if (!R_inv) return fail(HOP_E_ARG, "null R_inv");
  const int32_t n = t.n, m = t.m, s = n + 1;
  const bool extra = t.qxx_extra || t.qx_extra || t.c_extra;
  if (traj_fused(n, m, (int32_t)sizeof(T), extra, batch)) {
    // the augmented blocks never touch HBM: the sweep builds them per step
    return lft_entry<T>(nullptr, nullptr, nullptr, R_inv, r_bs, 0, 1, nullptr, nullptr, 0,
                        batch, n_alloc, n_use, s, m, max_tries, t_min, t_max, J, status,
                        t_star, j_star, nullptr, nullptr, stream, &t);
  }
  const int64_t need = traj_ws_bytes(batch, n_use, n, m, (int32_t)sizeof(T));
  if (!workspace || workspace_bytes < need)
    return fail(HOP_E_ARG, "workspace too small (hop_lft_sweep_traj_workspace_bytes)");
  if (((uintptr_t)workspace) % kWsAlign != 0) return fail(HOP_E_ARG, "workspace not 256-B aligned");
  const int64_t steps = batch * (int64_t)n_use;
  unsigned char* p = (unsigned char*)workspace;
  T* Aa = (T*)p; p += ws_round(steps * s * s * sizeof(T));
  T* Qa = (T*)p; p += ws_round(steps * s * s * sizeof(T));
  T* Ta = (T*)p; p += ws_round(steps * s * s * sizeof(T));
  T* Ba = (T*)p; p += ws_round(steps * s * m * sizeof(T));
  T* z0 = (T*)p;
  rc = augment_entry<T>(t, batch, n_alloc, n_use, Aa, Ba, Qa, Ta, z0, stream);
  if (rc != HOP_OK) return rc;
  return lft_entry<T>(Aa, Ba, Qa, R_inv, r_bs, 0, 1, Ta, z0, 0, batch, n_use, n_use, s, m,
                      max_tries, t_min, t_max, J, status, t_star, j_star, nullptr, nullptr,
                      stream);
}

}  // namespace

extern "C" {

int hop_set_options(uint32_t flags, int32_t variant) {
  if (flags & ~(HOP_OPT_FORCE_GENERIC | HOP_OPT_FORCE_HANDOVER | HOP_OPT_REFERENCE_ASSOC |
                HOP_OPT_TRAJ_UNFUSED | HOP_OPT_STAMPS | HOP_OPT_NO_RERUN |
                HOP_OPT_SMALL_LANE | HOP_OPT_RERUN_LANE))
    return fail(HOP_E_ARG, "unknown option flag");
  if (!hop::kDevBuild && (variant != 0 || (flags & HOP_OPT_STAMPS)))
    return fail(HOP_E_ARG, "A/B schedules and stamps exist only in developer builds "
                           "(HOP_DEV_BUILD=1 python -m time_opt_ilqr_amd.build)");
  hop::g_opt_flags = flags;
  hop::g_opt_variant = variant;
  return HOP_OK;
}

int hop_get_options(uint32_t* flags, int32_t* variant) {
  if (flags) *flags = hop::g_opt_flags;
  if (variant) *variant = hop::g_opt_variant;
  return HOP_OK;
}

int hop_build_flags(void) { return hop::kDevBuild ? 1 : 0; }

int hop_cu_fallbacks(void) { return hop::g_cu_fallbacks.load(std::memory_order_relaxed); }

int hop_abi_version(void) { return HOP_ABI_VERSION; }
const char* hop_last_error(void) { return g_err; }

int hop_lft_sweep_f64(const double* A, const double* B, const double* Q, const double* R,
                      int64_t r_bs, int64_t r_ks, int32_t r_inv, const double* QT,
                      const double* z0, int64_t z_bs, int64_t batch, int32_t n_alloc,
                      int32_t n_use, int32_t s, int32_t m, int32_t max_tries, int32_t t_min,
                      int32_t t_max, double* J, int32_t* status, int32_t* t_star,
                      double* j_star, double* dbg_efg, double* dbg_prefix, void* stream) {
  return lft_entry<double>(A, B, Q, R, r_bs, r_ks, r_inv, QT, z0, z_bs, batch, n_alloc, n_use, s,
                           m, max_tries, t_min, t_max, J, status, t_star, j_star, dbg_efg,
                           dbg_prefix, stream);
}
int hop_lft_sweep_f32(const float* A, const float* B, const float* Q, const float* R,
                      int64_t r_bs, int64_t r_ks, int32_t r_inv, const float* QT,
                      const float* z0, int64_t z_bs, int64_t batch, int32_t n_alloc,
                      int32_t n_use, int32_t s, int32_t m, int32_t max_tries, int32_t t_min,
                      int32_t t_max, float* J, int32_t* status, int32_t* t_star, float* j_star,
                      float* dbg_efg, float* dbg_prefix, void* stream) {
  return lft_entry<float>(A, B, Q, R, r_bs, r_ks, r_inv, QT, z0, z_bs, batch, n_alloc, n_use, s,
                          m, max_tries, t_min, t_max, J, status, t_star, j_star, dbg_efg,
                          dbg_prefix, stream);
}

int hop_lft_sweep_tile64_f64(const double* A, const double* B, const double* Q, const double* R,
                             int64_t r_bs, int32_t r_inv, const double* QT, const double* z0,
                             int64_t z_bs, int64_t batch, int32_t n_alloc, int32_t n_use,
                             int32_t s, int32_t m, int32_t max_tries, int32_t t_min,
                             int32_t t_max, double* J, int32_t* status, int32_t* t_star,
                             double* j_star, void* stream) {
  return lft_entry<double>(A, B, Q, R, r_bs, 0, r_inv, QT, z0, z_bs, batch, n_alloc, n_use, s, m,
                           max_tries, t_min, t_max, J, status, t_star, j_star, nullptr, nullptr,
                           stream, nullptr, true);
}
int hop_lft_sweep_tile64_f32(const float* A, const float* B, const float* Q, const float* R,
                             int64_t r_bs, int32_t r_inv, const float* QT, const float* z0,
                             int64_t z_bs, int64_t batch, int32_t n_alloc, int32_t n_use,
                             int32_t s, int32_t m, int32_t max_tries, int32_t t_min,
                             int32_t t_max, float* J, int32_t* status, int32_t* t_star,
                             float* j_star, void* stream) {
  return lft_entry<float>(A, B, Q, R, r_bs, 0, r_inv, QT, z0, z_bs, batch, n_alloc, n_use, s, m,
                          max_tries, t_min, t_max, J, status, t_star, j_star, nullptr, nullptr,
                          stream, nullptr, true);
}
int64_t hop_tile64_elems(int64_t batch, int32_t n_alloc, int32_t elems) {
  if (batch < 0 || n_alloc < 0 || elems < 0) return -1;
  return (batch + 63) / 64 * 64 * (int64_t)n_alloc * elems;
}
int hop_tile64_f64(const double* src, double* dst, int64_t batch, int32_t n_alloc, int32_t elems,
                   int32_t inverse, void* stream) {
  return tile64_entry<double>(src, dst, batch, n_alloc, elems, inverse, stream);
}
int hop_tile64_f32(const float* src, float* dst, int64_t batch, int32_t n_alloc, int32_t elems,
                   int32_t inverse, void* stream) {
  return tile64_entry<float>(src, dst, batch, n_alloc, elems, inverse, stream);
}

int hop_select_horizon_f64(const double* J, int64_t batch, int32_t ld, int32_t t_min,
                           int32_t t_max, int32_t* t_star, double* j_star, void* stream) {
  return select_entry<double>(J, batch, ld, t_min, t_max, t_star, j_star, stream);
}
int hop_select_horizon_f32(const float* J, int64_t batch, int32_t ld, int32_t t_min,
                           int32_t t_max, int32_t* t_star, float* j_star, void* stream) {
  return select_entry<float>(J, batch, ld, t_min, t_max, t_star, j_star, stream);
}

int hop_riccati_f64(const double* A, const double* Bm, const double* X, const double* U,
                    const double* xg, int64_t xg_bs, const double* u_ref, int64_t ur_bs,
                    const double* Q, int64_t q_bs, const double* R, int64_t r_bs,
                    const double* Qf, int64_t qf_bs, const double* qxx_extra,
                    const double* qx_extra, const double* c_extra, const int32_t* horizon,
                    const double* lm, double w_stage, uint32_t wrap_mask, int32_t mode,
                    int32_t reg_max_tries, int64_t batch, int32_t n_alloc, int32_t n, int32_t m,
                    double* K, double* k, double* Vxx, double* Vx, double* V0, int32_t* status,
                    void* stream) {
  return riccati_entry<double>(A, Bm, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs,
                               qxx_extra, qx_extra, c_extra, horizon, lm, w_stage, wrap_mask,
                               mode, reg_max_tries, batch, n_alloc, n, m, K, k, Vxx, Vx, V0,
                               status, stream);
}
int hop_riccati_f32(const float* A, const float* Bm, const float* X, const float* U,
                    const float* xg, int64_t xg_bs, const float* u_ref, int64_t ur_bs,
                    const float* Q, int64_t q_bs, const float* R, int64_t r_bs, const float* Qf,
                    int64_t qf_bs, const float* qxx_extra, const float* qx_extra,
                    const float* c_extra, const int32_t* horizon, const float* lm,
                    float w_stage, uint32_t wrap_mask, int32_t mode, int32_t reg_max_tries,
                    int64_t batch, int32_t n_alloc, int32_t n, int32_t m, float* K, float* k,
                    float* Vxx, float* Vx, float* V0, int32_t* status, void* stream) {
  return riccati_entry<float>(A, Bm, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs,
                              qxx_extra, qx_extra, c_extra, horizon, lm, w_stage, wrap_mask,
                              mode, reg_max_tries, batch, n_alloc, n, m, K, k, Vxx, Vx, V0,
                              status, stream);
}

int hop_bruteforce_jcurve_f64(const double* A, const double* Bm, const double* X,
                              const double* U, const double* xg, int64_t xg_bs,
                              const double* u_ref, int64_t ur_bs, const double* Q, int64_t q_bs,
                              const double* R, int64_t r_bs, const double* Qf, int64_t qf_bs,
                              const double* qxx_extra, const double* qx_extra,
                              const double* c_extra, double lm_lambda, double w_stage,
                              uint32_t wrap_mask, int64_t batch, int32_t n_alloc, int32_t n,
                              int32_t m, int32_t t_max, double* J, int32_t* status,
                              void* stream) {
  return jcurve_entry<double>(A, Bm, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs,
                              qxx_extra, qx_extra, c_extra, lm_lambda, w_stage, wrap_mask, batch,
                              n_alloc, n, m, t_max, J, status, stream);
}
int hop_bruteforce_jcurve_f32(const float* A, const float* Bm, const float* X, const float* U,
                              const float* xg, int64_t xg_bs, const float* u_ref, int64_t ur_bs,
                              const float* Q, int64_t q_bs, const float* R, int64_t r_bs,
                              const float* Qf, int64_t qf_bs, const float* qxx_extra,
                              const float* qx_extra, const float* c_extra, float lm_lambda,
                              float w_stage, uint32_t wrap_mask, int64_t batch, int32_t n_alloc,
                              int32_t n, int32_t m, int32_t t_max, float* J, int32_t* status,
                              void* stream) {
  return jcurve_entry<float>(A, Bm, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs,
                             qxx_extra, qx_extra, c_extra, lm_lambda, w_stage, wrap_mask, batch,
                             n_alloc, n, m, t_max, J, status, stream);
}

int hop_riccati_legacy_f64(const double* A, const double* Bm, const double* X, const double* U,
                           const double* xg, int64_t xg_bs, const double* u_ref, int64_t ur_bs,
                           const double* Q, int64_t q_bs, const double* R, int64_t r_bs,
                           const double* Qf, int64_t qf_bs, const int32_t* horizon,
                           const double* lm, double w_stage, uint32_t wrap_mask, int32_t mode,
                           int64_t batch, int32_t n_alloc, int32_t n, int32_t m, double* K,
                           double* k, double* Vxx, double* Vx, double* V0, int32_t* status,
                           void* stream) {
  return riccati_entry<double>(A, Bm, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs,
                               nullptr, nullptr, nullptr, horizon, lm, w_stage, wrap_mask, mode,
                               1, batch, n_alloc, n, m, K, k, Vxx, Vx, V0, status, stream, 1);
}

int hop_bruteforce_jcurve_legacy_f64(const double* A, const double* Bm, const double* X,
                                     const double* U, const double* xg, int64_t xg_bs,
                                     const double* u_ref, int64_t ur_bs, const double* Q,
                                     int64_t q_bs, const double* R, int64_t r_bs,
                                     const double* Qf, int64_t qf_bs, double lm_lambda,
                                     double w_stage, uint32_t wrap_mask, int64_t batch,
                                     int32_t n_alloc, int32_t n, int32_t m, int32_t t_max,
                                     double* J, int32_t* status, void* stream) {
  return jcurve_entry<double>(A, Bm, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs,
                              nullptr, nullptr, nullptr, lm_lambda, w_stage, wrap_mask, batch,
                              n_alloc, n, m, t_max, J, status, stream, 1);
}

int hop_augment_f64(const double* A, const double* Bm, const double* a_res, const double* X,
                    const double* U, const double* xg, int64_t xg_bs, const double* u_ref,
                    int64_t ur_bs, const double* Q, int64_t q_bs, const double* P, int64_t p_bs,
                    const double* w, int64_t w_bs, const double* qxx_extra,
                    const double* qx_extra, const double* c_extra, uint32_t wrap_mask,
                    double q_reg, double rho_reg, int64_t batch, int32_t n_alloc,
                    int32_t n_build, int32_t n, int32_t m, double* A_aug, double* B_aug,
                    double* Q_aug, double* QT_aug, double* z0, void* stream) {
  return augment_entry<double>(
      traj_args<double>(A, Bm, a_res, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, P, p_bs, w, w_bs,
                        qxx_extra, qx_extra, c_extra, wrap_mask, q_reg, rho_reg, n, m),
      batch, n_alloc, n_build, A_aug, B_aug, Q_aug, QT_aug, z0, stream);
}
int hop_augment_f32(const float* A, const float* Bm, const float* a_res, const float* X,
                    const float* U, const float* xg, int64_t xg_bs, const float* u_ref,
                    int64_t ur_bs, const float* Q, int64_t q_bs, const float* P, int64_t p_bs,
                    const float* w, int64_t w_bs, const float* qxx_extra, const float* qx_extra,
                    const float* c_extra, uint32_t wrap_mask, float q_reg, float rho_reg,
                    int64_t batch, int32_t n_alloc, int32_t n_build, int32_t n, int32_t m,
                    float* A_aug, float* B_aug, float* Q_aug, float* QT_aug, float* z0,
                    void* stream) {
  return augment_entry<float>(
      traj_args<float>(A, Bm, a_res, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, P, p_bs, w, w_bs,
                       qxx_extra, qx_extra, c_extra, wrap_mask, q_reg, rho_reg, n, m),
      batch, n_alloc, n_build, A_aug, B_aug, Q_aug, QT_aug, z0, stream);
}

int64_t hop_lft_sweep_traj_workspace_bytes(int64_t batch, int32_t n_use, int32_t n, int32_t m,
                                           int32_t elem_bytes, int32_t has_extra) {
  if (batch <= 0 || n_use <= 0) return 0;
  if (traj_fused(n, m, elem_bytes, has_extra != 0, batch)) return 0;
  return traj_ws_bytes(batch, n_use, n, m, elem_bytes);
}

int hop_lft_sweep_traj_f64(const double* A, const double* Bm, const double* a_res,
                           const double* X, const double* U, const double* xg, int64_t xg_bs,
                           const double* u_ref, int64_t ur_bs, const double* Q, int64_t q_bs,
                           const double* P, int64_t p_bs, const double* w, int64_t w_bs,
                           const double* qxx_extra, const double* qx_extra,
                           const double* c_extra, uint32_t wrap_mask, double q_reg,
                           double rho_reg, const double* R_inv, int64_t r_bs, int64_t batch,
                           int32_t n_alloc, int32_t n_use, int32_t n, int32_t m,
                           int32_t max_tries, int32_t t_min, int32_t t_max, double* J,
                           int32_t* status, int32_t* t_star, double* j_star, void* workspace,
                           int64_t workspace_bytes, void* stream) {
  return lft_traj_entry<double>(
      traj_args<double>(A, Bm, a_res, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, P, p_bs, w, w_bs,
                        qxx_extra, qx_extra, c_extra, wrap_mask, q_reg, rho_reg, n, m),
      R_inv, r_bs, batch, n_alloc, n_use, max_tries, t_min, t_max, J, status, t_star, j_star,
      workspace, workspace_bytes, stream);
}
int hop_lft_sweep_traj_f32(const float* A, const float* Bm, const float* a_res, const float* X,
                           const float* U, const float* xg, int64_t xg_bs, const float* u_ref,
                           int64_t ur_bs, const float* Q, int64_t q_bs, const float* P,
                           int64_t p_bs, const float* w, int64_t w_bs, const float* qxx_extra,
                           const float* qx_extra, const float* c_extra, uint32_t wrap_mask,
                           float q_reg, float rho_reg, const float* R_inv, int64_t r_bs,
                           int64_t batch, int32_t n_alloc, int32_t n_use, int32_t n, int32_t m,
                           int32_t max_tries, int32_t t_min, int32_t t_max, float* J,
                           int32_t* status, int32_t* t_star, float* j_star, void* workspace,
                           int64_t workspace_bytes, void* stream) {
  return lft_traj_entry<float>(
      traj_args<float>(A, Bm, a_res, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, P, p_bs, w, w_bs,
                       qxx_extra, qx_extra, c_extra, wrap_mask, q_reg, rho_reg, n, m),
      R_inv, r_bs, batch, n_alloc, n_use, max_tries, t_min, t_max, J, status, t_star, j_star,
      workspace, workspace_bytes, stream);
}

extern "C++" {
template <class T>
int traj_tile64_entry(const hop::TrajArgs<T>& t, const T* R_inv, int64_t r_bs, int64_t batch,
                      int32_t n_alloc, int32_t n_use, int32_t max_tries, int32_t t_min,
                      int32_t t_max, T* J, int32_t* status, int32_t* t_star, T* j_star,
                      void* stream) {
  int rc = traj_check(t, batch, n_alloc, n_use);
  if (rc != HOP_OK) return rc;
  if (n_use <= 0 || batch == 0) return HOP_OK;
  if (!R_inv) return fail(HOP_E_ARG, "null R_inv");
  if (r_bs < 0) return fail(HOP_E_ARG, "negative stride");
  const int32_t s = t.n + 1;
  const bool shape = (s == 2 && t.m == 1) || (s == 3 && t.m == 1) ||
                     (s == 4 && (t.m == 1 || t.m == 2)) || (s == 5 && (t.m == 1 || t.m == 2));
  if (!shape) return fail(HOP_E_SIZE, "tile64 trajectory form: no small-s kernel for this shape");
  return lft_entry<T>(nullptr, nullptr, nullptr, R_inv, r_bs, 0, 1, nullptr, nullptr, 0, batch,
                      n_alloc, n_use, s, t.m, max_tries, t_min, t_max, J, status, t_star, j_star,
                      nullptr, nullptr, stream, &t, true);
}
}  // extern "C++"

int hop_lft_sweep_traj_tile64_f64(const double* A, const double* Bm, const double* a_res,
                                  const double* X, const double* U, const double* xg,
                                  int64_t xg_bs, const double* u_ref, int64_t ur_bs,
                                  const double* Q, int64_t q_bs, const double* P, int64_t p_bs,
                                  const double* w, int64_t w_bs, uint32_t wrap_mask, double q_reg,
                                  double rho_reg, const double* R_inv, int64_t r_bs,
                                  int64_t batch, int32_t n_alloc, int32_t n_use, int32_t n,
                                  int32_t m, int32_t max_tries, int32_t t_min, int32_t t_max,
                                  double* J, int32_t* status, int32_t* t_star, double* j_star,
                                  void* stream) {
  return traj_tile64_entry<double>(
      traj_args<double>(A, Bm, a_res, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, P, p_bs, w, w_bs,
                        nullptr, nullptr, nullptr, wrap_mask, q_reg, rho_reg, n, m),
      R_inv, r_bs, batch, n_alloc, n_use, max_tries, t_min, t_max, J, status, t_star, j_star,
      stream);
}
int hop_lft_sweep_traj_tile64_f32(const float* A, const float* Bm, const float* a_res,
                                  const float* X, const float* U, const float* xg, int64_t xg_bs,
                                  const float* u_ref, int64_t ur_bs, const float* Q, int64_t q_bs,
                                  const float* P, int64_t p_bs, const float* w, int64_t w_bs,
                                  uint32_t wrap_mask, float q_reg, float rho_reg,
                                  const float* R_inv, int64_t r_bs, int64_t batch,
                                  int32_t n_alloc, int32_t n_use, int32_t n, int32_t m,
                                  int32_t max_tries, int32_t t_min, int32_t t_max, float* J,
                                  int32_t* status, int32_t* t_star, float* j_star, void* stream) {
  return traj_tile64_entry<float>(
      traj_args<float>(A, Bm, a_res, X, U, xg, xg_bs, u_ref, ur_bs, Q, q_bs, P, p_bs, w, w_bs,
                       nullptr, nullptr, nullptr, wrap_mask, q_reg, rho_reg, n, m),
      R_inv, r_bs, batch, n_alloc, n_use, max_tries, t_min, t_max, J, status, t_star, j_star,
      stream);
}

int hop_system_dims(int32_t system, int32_t* n, int32_t* m) {
  if (system < 0 || system >= hop::dyn::kNumSystems) return fail(HOP_E_ARG, "unknown system id");
  if (n) *n = hop::dyn::state_dim(system);
  if (m) *m = hop::dyn::control_dim(system);
  return HOP_OK;
}

int hop_linearize_f64(int32_t system, double dt, const double* X, const double* U,
                      int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                      double epsx, double epsu, double relx, double relu, double* A,
                      double* Bm, double* a_res, double* Fx, void* stream) {
  if (system < 0 || system >= hop::dyn::kNumSystems) return fail(HOP_E_ARG, "unknown system id");
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (n_use > n_alloc) return fail(HOP_E_ARG, "n_use > n_alloc");
  if (central != 0 && central != 1) return fail(HOP_E_ARG, "central must be 0 or 1");
  if (batch == 0 || n_use <= 0) return HOP_OK;
  if (!X || !U || !A || !Bm) return fail(HOP_E_ARG, "null input/output pointer");
  if (batch * (int64_t)n_use > (int64_t)0xffffffffLL * 64)
    return fail(HOP_E_SIZE, "batch * n_use too large for one launch");
  hop::LinArgs a{};
  a.sys = system; a.central = central; a.dt = dt;
  a.epsx = epsx; a.epsu = epsu; a.relx = relx; a.relu = relu;
  a.X = X; a.U = U; a.batch = batch; a.nalloc = n_alloc; a.nuse = n_use;
  a.A = A; a.B = Bm; a.a_res = a_res; a.Fx = Fx;
  return hip_status(hop::dispatch_linearize(a, (hipStream_t)stream));
}

static int linearize_tile64(int32_t system, double dt, const double* X, const double* U,
                            int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                            double epsx, double epsu, double relx, double relu, void* A, void* Bm,
                            void* a_res, void* Xt, void* Ut, int f32, void* stream) {
  if (system < 0 || system >= hop::dyn::kNumSystems) return fail(HOP_E_ARG, "unknown system id");
  if (batch < 0) return fail(HOP_E_ARG, "batch < 0");
  if (n_use > n_alloc) return fail(HOP_E_ARG, "n_use > n_alloc");
  if (central != 0 && central != 1) return fail(HOP_E_ARG, "central must be 0 or 1");
  if (batch == 0 || n_use <= 0) return HOP_OK;
  if (!X || !U || !A || !Bm || !Xt || !Ut) return fail(HOP_E_ARG, "null input/output pointer");
  if ((batch + 63) / 64 * (int64_t)n_use > (int64_t)0xffffffffLL)
    return fail(HOP_E_SIZE, "batch * n_use too large for one launch");
  hop::LinArgs a{};
  a.sys = system; a.central = central; a.dt = dt;
  a.epsx = epsx; a.epsu = epsu; a.relx = relx; a.relu = relu;
  a.X = X; a.U = U; a.batch = batch; a.nalloc = n_alloc; a.nuse = n_use;
  a.A = A; a.B = Bm; a.a_res = a_res; a.Fx = nullptr;
  a.tile64 = 1; a.out_f32 = f32; a.Xt = Xt; a.Ut = Ut;
  return hip_status(hop::dispatch_linearize(a, (hipStream_t)stream));
}

int hop_linearize_tile64_f64(int32_t system, double dt, const double* X, const double* U,
                             int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                             double epsx, double epsu, double relx, double relu, double* A,
                             double* Bm, double* a_res, double* Xt, double* Ut, void* stream) {
  return linearize_tile64(system, dt, X, U, batch, n_alloc, n_use, central, epsx, epsu, relx,
                          relu, A, Bm, a_res, Xt, Ut, 0, stream);
}
int hop_linearize_tile64_f32(int32_t system, double dt, const double* X, const double* U,
                             int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                             double epsx, double epsu, double relx, double relu, float* A,
                             float* Bm, float* a_res, float* Xt, float* Ut, void* stream) {
  return linearize_tile64(system, dt, X, U, batch, n_alloc, n_use, central, epsx, epsu, relx,
                          relu, A, Bm, a_res, Xt, Ut, 1, stream);
}

int hop_dynamics_f64(int32_t system, double dt, const double* X, int64_t x_stride,
                     const double* U, int64_t u_stride, int64_t count, double* Xn,
                     int64_t xn_stride, void* stream) {
  if (system < 0 || system >= hop::dyn::kNumSystems) return fail(HOP_E_ARG, "unknown system id");
  if (count < 0) return fail(HOP_E_ARG, "count < 0");
  if (count == 0) return HOP_OK;
  if (!X || !U || !Xn) return fail(HOP_E_ARG, "null input/output pointer");
  const int n = hop::dyn::state_dim(system), m = hop::dyn::control_dim(system);
  if (x_stride < n || u_stride < m || xn_stride < n) return fail(HOP_E_ARG, "row stride too small");
  if (count > (int64_t)0xffffffffLL * 256) return fail(HOP_E_SIZE, "count too large for one launch");
  hop::DynArgs a{};
  a.sys = system; a.dt = dt; a.X = X; a.U = U; a.Xn = Xn;
  a.count = count; a.x_stride = x_stride; a.u_stride = u_stride; a.xn_stride = xn_stride;
  return hip_status(hop::dispatch_dynamics(a, (hipStream_t)stream));
}

static int cost_args(int32_t system, const double* xg, int64_t xg_bs, const double* u_ref,
                     int64_t ur_bs, const double* Q, int64_t q_bs, const double* R, int64_t r_bs,
                     const double* Qf, int64_t qf_bs, const double* w, int64_t w_bs,
                     const double* obstacles, int32_t n_obs, uint32_t wrap_mask,
                     hop::CostArgs* c) {
  if (system < 0 || system >= hop::dyn::kNumSystems) return fail(HOP_E_ARG, "unknown system id");
  if (!xg || !u_ref || !Q || !R || !Qf || !w) return fail(HOP_E_ARG, "null cost parameter");
  if (xg_bs < 0 || ur_bs < 0 || q_bs < 0 || r_bs < 0 || qf_bs < 0 || w_bs < 0)
    return fail(HOP_E_ARG, "negative batch stride");
  if (n_obs < 0 || n_obs > 64 || (n_obs > 0 && !obstacles))
    return fail(HOP_E_ARG, "obstacles: 0 <= n_obs <= 64 rows of (cx, cy, radius, weight)");
  const int n = hop::dyn::state_dim(system);
  if (n_obs > 0 && n < 2) return fail(HOP_E_ARG, "obstacles need a planar position (n >= 2)");
  if (wrap_mask >> n) return fail(HOP_E_ARG, "wrap index out of range");
  *c = hop::CostArgs{xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs, w, w_bs,
                     n_obs > 0 ? obstacles : nullptr, n_obs, wrap_mask};
  return HOP_OK;
}

int hop_rollout_f64(int32_t system, double dt, const double* x0, int64_t x0_batch_stride,
                    const double* U, int64_t batch, int32_t N, double max_state_norm, double* X,
                    void* stream) {
  if (system < 0 || system >= hop::dyn::kNumSystems) return fail(HOP_E_ARG, "unknown system id");
  if (batch < 0 || N < 0 || x0_batch_stride < 0) return fail(HOP_E_ARG, "negative size/stride");
  if (batch == 0) return HOP_OK;
  if (!x0 || !X || (N > 0 && !U)) return fail(HOP_E_ARG, "null pointer");
  hop::RolloutArgs a{dt, x0, x0_batch_stride, U, batch, N, max_state_norm, X};
  return hip_status(hop::dispatch_forward(system, 0, &a, (hipStream_t)stream));
}

int hop_cost_true_f64(int32_t system, const double* X, const double* U, const int32_t* T_star,
                      const double* xg, int64_t xg_bs, const double* u_ref, int64_t ur_bs,
                      const double* Q, int64_t q_bs, const double* R, int64_t r_bs,
                      const double* Qf, int64_t qf_bs, const double* w, int64_t w_bs,
                      const double* obstacles, int32_t n_obs, uint32_t wrap_mask, int64_t batch,
                      int32_t N, double* J, void* stream) {
  hop::CostCall a{};
  int rc = cost_args(system, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs, w, w_bs,
                     obstacles, n_obs, wrap_mask, &a.c);
  if (rc) return rc;
  if (batch < 0 || N < 0) return fail(HOP_E_ARG, "negative size");
  if (batch == 0) return HOP_OK;
  if (!X || !T_star || !J || (N > 0 && !U)) return fail(HOP_E_ARG, "null pointer");
  a.X = X; a.U = U; a.T = T_star; a.batch = batch; a.N = N; a.J = J;
  return hip_status(hop::dispatch_forward(system, 1, &a, (hipStream_t)stream));
}

size_t hop_forward_workspace_bytes(int32_t system, int64_t batch, int32_t N, int32_t n_alpha) {
  if (system < 0 || system >= hop::dyn::kNumSystems || batch < 0 || N < 0 || n_alpha < 0)
    return 0;
  const int64_t n = hop::dyn::state_dim(system), m = hop::dyn::control_dim(system);
  const int64_t row = (int64_t)(N + 1) * n + (int64_t)N * m;
  return (size_t)(batch * n_alpha * (1 + row) * (int64_t)sizeof(double));
}

int hop_forward_linesearch_f64(int32_t system, double dt, const double* X, const double* U,
                               const double* xg, int64_t xg_bs, const double* u_ref,
                               int64_t ur_bs, const double* Q, int64_t q_bs, const double* R,
                               int64_t r_bs, const double* Qf, int64_t qf_bs, const double* w,
                               int64_t w_bs, const double* obstacles, int32_t n_obs,
                               uint32_t wrap_mask, const int32_t* T_star, const int32_t* active,
                               const double* K, const double* k, const double* alphas,
                               int32_t n_alpha, int64_t batch, int32_t N, void* workspace,
                               size_t workspace_bytes, double* X_new, double* U_new, double* J,
                               double* J_old, int32_t* accepted, void* stream) {
  hop::FwdArgs a{};
  int rc = cost_args(system, xg, xg_bs, u_ref, ur_bs, Q, q_bs, R, r_bs, Qf, qf_bs, w, w_bs,
                     obstacles, n_obs, wrap_mask, &a.c);
  if (rc) return rc;
  if (batch < 0 || N < 0) return fail(HOP_E_ARG, "negative size");
  if (n_alpha < 1 || n_alpha > 8 || !alphas) return fail(HOP_E_ARG, "1 <= n_alpha <= 8 host alphas");
  if (batch == 0) return HOP_OK;
  if (!X || !T_star || !K || !k || !X_new || !U_new || !J || !J_old || !accepted ||
      (N > 0 && !U))
    return fail(HOP_E_ARG, "null pointer");
  const size_t need = hop_forward_workspace_bytes(system, batch, N, n_alpha);
  if (!workspace || workspace_bytes < need) return fail(HOP_E_ARG, "workspace too small");
  if (batch * (n_alpha + 1) > (int64_t)0xffffffffLL * 64 || batch > 0x7fffffffLL)
    return fail(HOP_E_SIZE, "batch too large for one launch");
  a.dt = dt; a.X = X; a.U = U; a.T_star = T_star; a.active = active; a.K = K; a.kff = k;
  for (int i = 0; i < n_alpha; ++i) a.alphas[i] = alphas[i];
  a.n_alpha = n_alpha; a.batch = batch; a.N = N;
  a.Jc = (double*)workspace;
  a.ws = a.Jc + batch * n_alpha;
  a.J_old = J_old; a.X_new = X_new; a.U_new = U_new; a.J = J; a.accepted = accepted;
  return hip_status(hop::dispatch_forward(system, 2, &a, (hipStream_t)stream));
}

int hop_obstacle_cost_f64(const double* X, int64_t x_stride, int64_t count, int32_t n,
                          const double* obstacles, int32_t n_obs, double* c, double* cx,
                          double* cxx, void* stream) {
  if (count < 0 || n < 2 || n > 16 || x_stride < n || n_obs < 0)
    return fail(HOP_E_ARG, "bad size/stride");
  if (count == 0) return HOP_OK;
  if (!X || (n_obs > 0 && !obstacles)) return fail(HOP_E_ARG, "null pointer");
  hop::ObstacleArgs a{X, x_stride, count, n, obstacles, n_obs, c, cx, cxx};
  return hip_status(hop::dispatch_obstacle(a, (hipStream_t)stream));
}

int hop_ilqr_accept_f64(int64_t batch, int32_t warm, const double* J, const int32_t* accepted,
                        const int32_t* T_star, double* lm, int32_t* T_bar, double* J_hist,
                        int32_t* T_hist, int32_t* n_hist, int32_t hist_cap, int32_t* done,
                        void* stream) {
  if (batch < 0 || hist_cap < 1) return fail(HOP_E_ARG, "bad size");
  if (batch == 0) return HOP_OK;
  if (!J || !accepted || !T_star || !lm || !T_bar || !J_hist || !T_hist || !n_hist || !done)
    return fail(HOP_E_ARG, "null pointer");
  hop::AcceptArgs a{batch, warm ? 1 : 0, hist_cap, J, accepted, T_star, lm, T_bar, J_hist,
                    T_hist, n_hist, done};
  return hip_status(hop::dispatch_accept(a, (hipStream_t)stream));
}

int hop_ilqr_select_mask(int64_t batch, const int32_t* sel_status, const int32_t* ric_status,
                         int32_t* done, int32_t* crashed, int32_t* active, void* stream) {
  if (batch < 0) return fail(HOP_E_ARG, "bad size");
  if (batch == 0) return HOP_OK;
  if (!sel_status || !ric_status || !done || !crashed || !active)
    return fail(HOP_E_ARG, "null pointer");
  hop::MaskArgs a{batch, sel_status, ric_status, done, crashed, active};
  return hip_status(hop::dispatch_select_mask(a, (hipStream_t)stream));
}

}  // extern "C"
