/*
 * hop.h -- C ABI of the MI355X (gfx950) horizon-selection engine (libhop_amd.so).
 *
 * Drop-in boundary for the hot path of dmmsjtu-umich/time-opt-ilqr: the batched
 * LFT propagator, the horizon argmin and the Riccati gain/value passes.  The
 * reference exposes these as Python functions (no FFI of its own); each entry
 * point below names the reference function it replaces.  The Python mirror in
 * time_opt_ilqr_amd/ (ctypes) and INTEGRATION.md show the binding.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer (hipMalloc / torch.cuda tensor storage),
 *    row-major, batch-major, contiguous unless a stride argument says otherwise.
 *    Strides are in ELEMENTS; a batch stride of 0 broadcasts one block to all
 *    problems.
 *  - Launches are asynchronous on `stream` (hipStream_t, NULL = default stream);
 *    the library never allocates, copies or synchronises on the hot path, so the
 *    calls are graph-capturable.
 *  - Return value: 0 = launched; <0 = rejected before launch (HOP_E_*), see
 *    hop_last_error() for the message.
 *  - Numerical outcomes are reported per problem in `status` (HOP_ST_* bits),
 *    matching the reference's exception / return conventions:
 *      HOP_ST_JITTER    chol_inv/chol_solve needed more than the first 1e-9 jitter
 *      HOP_ST_LU        chol_inv exhausted its jitter tries and used the fallback
 *      HOP_ST_NONFINITE a non-finite value (reference: FloatingPointError)
 *      HOP_ST_FAIL      not PD after every try (reference: LinAlgError, or
 *                       backward_pass_truncated's ok=False)
 */
#ifndef HOP_H
#define HOP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HOP_ABI_VERSION 1

#define HOP_OK 0
#define HOP_E_ARG (-1)
#define HOP_E_SIZE (-2)
#define HOP_E_HIP (-3)

#define HOP_ST_JITTER 1
#define HOP_ST_LU 2
#define HOP_ST_NONFINITE 4
#define HOP_ST_FAIL 8

#define HOP_MAX_DIM 16 /* augmented s = n+1 <= 16, m <= 16 */

int hop_abi_version(void);
const char* hop_last_error(void);

/*
 * Test / diagnostic controls.  Not part of any reference interface and never
 * needed by a caller: every entry point runs its default kernels with all flags
 * 0.  Per host thread: the dispatchers read the calling thread's setting at
 * launch time (no environment variables are consulted), so two threads may
 * launch with different options at once.
 *   HOP_OPT_FORCE_GENERIC   every sweep / Riccati pass on the generic kernels
 *                           (lft_sweep.hip, riccati.hip): the fast paths'
 *                           cross-check
 *   HOP_OPT_FORCE_HANDOVER  the conditioned-prefix kernels hand EVERY problem to
 *                           their rerun launch (tests the hand-over path)
 *   HOP_OPT_REFERENCE_ASSOC only the reference-association kernel (no
 *                           conditioned prefix): s = 13 fp64 / fp32 and every
 *                           small-s shape (s <= 5, both layouts, both forms)
 *   HOP_OPT_TRAJ_UNFUSED    trajectory form through hop_augment + the sweep
 *   HOP_OPT_STAMPS          section-stamped instantiations (developer builds)
 *   HOP_OPT_NO_RERUN        the conditioned-prefix kernels run without the
 *                           recompute of their rerun launch: a problem they hand
 *                           over keeps HOP_ST_HANDOVER in status and its J is not
 *                           valid (counts hand-overs; tests and tools only).  The
 *                           s = 13 fp64 paths still run the launch's non-finite
 *                           triage: a hand-over explained by non-finite inputs
 *                           gets the reference's outcome (ST_NONFINITE, NaN from
 *                           the first affected horizon) and is not counted
 *   HOP_OPT_SMALL_LANE      fp64 s <= 5 block sweeps of at most 16,384 problems on
 *                           the lane-per-problem kernel (lft_small.hip) instead of
 *                           the row-group kernel (lft_sweep_v2.hip SchedCondSmall):
 *                           the A/B and cross-check of the two
 *   HOP_OPT_RERUN_LANE      the fp64 s <= 5 rerun launch recomputes every hand-over
 *                           on its own lane (the one-lane LFT kernel) instead of the
 *                           pipelined rerun (lft_small.hip lft_small_rerun_kernel):
 *                           the A/B and bitwise cross-check of the two
 * `variant` selects an A/B schedule; only developer builds (HOP_DEV_BUILD=1 at
 * build time, hop_build_flags() & 1) compile them -- product builds return
 * HOP_E_ARG for variant != 0 or HOP_OPT_STAMPS.
 */
#define HOP_OPT_FORCE_GENERIC 1u
#define HOP_OPT_FORCE_HANDOVER 2u
#define HOP_OPT_REFERENCE_ASSOC 4u
#define HOP_OPT_TRAJ_UNFUSED 8u
#define HOP_OPT_STAMPS 16u
#define HOP_OPT_NO_RERUN 32u
#define HOP_OPT_SMALL_LANE 64u
#define HOP_OPT_RERUN_LANE 128u
#define HOP_ST_HANDOVER 16 /* status bit, set only under HOP_OPT_NO_RERUN */
/*
 * The hand-over word: the status a conditioned-prefix kernel leaves for a problem
 * it hands to its rerun launch, read by that launch (the s = 13 fp64 non-finite
 * triage) and returned to the caller only under HOP_OPT_NO_RERUN.  One definition
 * for every kernel that writes or reads it (lft_sweep_v2.hip, lft_small.hip,
 * small_math.hpp; tests/test_host_cpu.py decodes it from the host build):
 *   HOP_ST_HANDOVER | (h << HOP_HANDOVER_SHIFT)
 *   h = the first horizon (1-based) whose evaluation raised a flag of the
 *       conditioned form (a first-attempt pivot, a non-positive Schur complement,
 *       a non-finite J); 0 = flagged before horizon 1 (HOP_OPT_FORCE_HANDOVER);
 *       clamped to HOP_HANDOVER_H_MAX (a clamped h only makes the triage decline)
 *   developer builds under HOP_OPT_NO_RERUN also put the reason of the first flag
 *   in bits HOP_HANDOVER_REASON_SHIFT .. HOP_HANDOVER_SHIFT - 1
 */
#define HOP_HANDOVER_SHIFT 13
#define HOP_HANDOVER_H_MAX 262143 /* 2^18 - 1: h << 13 stays below the int32 sign bit */
#define HOP_HANDOVER_REASON_SHIFT 5
#define HOP_HANDOVER_WORD(h)                                                        \
  (HOP_ST_HANDOVER | ((int32_t)((h) < HOP_HANDOVER_H_MAX ? (h) : HOP_HANDOVER_H_MAX) \
                      << HOP_HANDOVER_SHIFT))
#define HOP_HANDOVER_HORIZON(st) ((int32_t)((uint32_t)(st) >> HOP_HANDOVER_SHIFT))
/*
 * The triage rule (rerun launch of the s = 13 fp64 kernels): with h_poison = 1 +
 * the first stage whose inputs are non-finite (1 for shared inputs), h_qt = the
 * first horizon whose terminal block is non-finite (N + 1 if none) and h the
 * hand-over word's horizon, the reference's outcome is the conditioned curve
 * before min(h_poison, h_qt), NaN from there on, ST_NONFINITE, when
 */
#define HOP_TRIAGE_ACCEPTS(h, h_poison, h_qt, n_use)                                  \
  (((h_poison) < (h_qt) ? (h_poison) : (h_qt)) <= (n_use) &&                          \
   (h) >= ((h_poison) < (h_qt) ? (h_poison) : (h_qt)) && (h_poison) <= (h_qt) + 1)
int hop_set_options(uint32_t flags, int32_t variant);
int hop_get_options(uint32_t* flags, int32_t* variant); /* the calling thread's; nullable */
int hop_build_flags(void); /* bit 0: developer build (A/B schedules and stamps compiled) */
int hop_cu_fallbacks(void); /* CU-count queries that failed and assumed 256 (layout only) */

/*
 * hop_lft_sweep_f64 / _f32
 * Replaces propagator_all_Jt_aug(A_aug, B_aug, Q_aug, R_list, z0, QT_aug_list,
 *                                T_use, R_inv_cached)
 *   /root/reference/horizon_selection.py:36-86 (legacy twin
 *   ilqr_propagator.py:209-232), for a batch of independent problems.
 *
 *   A_aug  [batch][n_alloc][s][s]   Q_aug [batch][n_alloc][s][s]
 *   B_aug  [batch][n_alloc][s][m]   QT_aug[batch][n_alloc][s][s] (QT[t-1] for horizon t)
 *   R      r_is_inverse=1: R_inv_cached;  r_is_inverse=0: raw R_k, inverted per
 *          step with chol_inv semantics.  Element (b,k) block at
 *          R + b*r_batch_stride + k*r_step_stride ([m][m]).
 *   z0     [batch or 1][s]  (z0_batch_stride = s or 0)
 *   n_use  = T_use (<= n_alloc); n_use <= 0 launches nothing (reference returns [])
 *   max_tries = chol_inv jitter tries (8 = utils.py; 4 = legacy ilqr_propagator.py)
 *   J      [batch][n_use]  out: J[b][t-1] = 1/2 z0^T P0^(t) z0
 *   status [batch]         out: HOP_ST_* bits
 *   t_min/t_max: if t_max > 0 the argmin of solver.py:522 is fused and written
 *          to t_star [batch] / j_star [batch] (both may be NULL otherwise).
 *   dbg_efg [batch][n_use][3][s][s] nullable: E_k, F_k, G_k (stage blocks)
 *   dbg_prefix [batch][n_use][3][s][s] nullable: Ebar_k, Fbar_k, Gbar_k
 *   s = 13, m = 4, fp64, no debug outputs: two stream-ordered launches, the
 *          conditioned-prefix kernel (z0 folded into the prefix first, same J to
 *          ~1e-12) and a rerun of the problems it could not take with the
 *          reference association (status and failure semantics unchanged): the
 *          rerun launch first resolves hand-overs explained by non-finite inputs
 *          (HOP_TRIAGE_ACCEPTS), then recomputes the rest, up to four problems per
 *          workgroup of sixteen as a pipeline over the workgroup's four waves
 *          (stage blocks and queries on four rows at once, the compose chain on two
 *          waves), more with the one-wave LFT kernel's code; either way bitwise the
 *          reference-association kernel's J, status, T* and J*.
 *   s <= 5 (both dtypes, m <= 2): the one-problem-per-lane kernels, the
 *          conditioned association and then the LFT kernel in rerun mode for the
 *          problems it hands over.
 */
int hop_lft_sweep_f64(const double* A_aug, const double* B_aug, const double* Q_aug,
                      const double* R, int64_t r_batch_stride, int64_t r_step_stride,
                      int32_t r_is_inverse, const double* QT_aug, const double* z0,
                      int64_t z0_batch_stride, int64_t batch, int32_t n_alloc, int32_t n_use,
                      int32_t s, int32_t m, int32_t max_tries, int32_t t_min, int32_t t_max,
                      double* J, int32_t* status, int32_t* t_star, double* j_star,
                      double* dbg_efg, double* dbg_prefix, void* stream);
int hop_lft_sweep_f32(const float* A_aug, const float* B_aug, const float* Q_aug,
                      const float* R, int64_t r_batch_stride, int64_t r_step_stride,
                      int32_t r_is_inverse, const float* QT_aug, const float* z0,
                      int64_t z0_batch_stride, int64_t batch, int32_t n_alloc, int32_t n_use,
                      int32_t s, int32_t m, int32_t max_tries, int32_t t_min, int32_t t_max,
                      float* J, int32_t* status, int32_t* t_star, float* j_star,
                      float* dbg_efg, float* dbg_prefix, void* stream);

/*
 * tile64 layout (the native layout of the s <= 5 one-problem-per-lane sweep)
 *   A block tensor of `elems` elements per (problem, step) -- s*s for A/Q/QT,
 *   s*m for B -- stored as [ceil(batch/64)][n_alloc][elems][64]: element e of
 *   step k of problem b at ((b/64)*n_alloc + k)*elems*64 + e*64 + b%64.  A wave
 *   of 64 problems then streams each block of a step as 64*elems contiguous
 *   elements; batch-major blocks are 64 scattered spans of elems elements, and at
 *   config 3 (s=5, fp32) that stream alone costs twice the tiled one.
 * hop_tile64_elems: element count of a tile64 tensor (padding slots included).
 * hop_tile64_f64/_f32: batch-major [batch][n_alloc][elems] -> tile64
 *   (inverse=0; padding slots written 0), or tile64 -> batch-major (inverse=1).
 *   A one-pass copy for callers holding batch-major blocks.
 * hop_lft_sweep_tile64_f64/_f32: hop_lft_sweep_* (same reference function,
 *   arguments and outputs) with A_aug, B_aug, Q_aug, QT_aug in tile64 layout;
 *   R (no per-step stride), z0 and every output as hop_lft_sweep_*.  Shapes with
 *   a small-s kernel only (s <= 5, m <= 2, both dtypes), else HOP_E_SIZE; padding
 *   slots are read but never reported.  Every small-s sweep (both layouts, both
 *   dtypes, blocks and trajectory form) runs the conditioned association and then
 *   the LFT kernel in rerun mode for the problems it hands over, as the s = 13
 *   fp64 path does; HOP_OPT_REFERENCE_ASSOC runs the LFT kernel alone.
 */
int64_t hop_tile64_elems(int64_t batch, int32_t n_alloc, int32_t elems);
int hop_tile64_f64(const double* src, double* dst, int64_t batch, int32_t n_alloc, int32_t elems,
                   int32_t inverse, void* stream);
int hop_tile64_f32(const float* src, float* dst, int64_t batch, int32_t n_alloc, int32_t elems,
                   int32_t inverse, void* stream);
int hop_lft_sweep_tile64_f64(const double* A_aug, const double* B_aug, const double* Q_aug,
                             const double* R, int64_t r_batch_stride, int32_t r_is_inverse,
                             const double* QT_aug, const double* z0, int64_t z0_batch_stride,
                             int64_t batch, int32_t n_alloc, int32_t n_use, int32_t s, int32_t m,
                             int32_t max_tries, int32_t t_min, int32_t t_max, double* J,
                             int32_t* status, int32_t* t_star, double* j_star, void* stream);
int hop_lft_sweep_tile64_f32(const float* A_aug, const float* B_aug, const float* Q_aug,
                             const float* R, int64_t r_batch_stride, int32_t r_is_inverse,
                             const float* QT_aug, const float* z0, int64_t z0_batch_stride,
                             int64_t batch, int32_t n_alloc, int32_t n_use, int32_t s, int32_t m,
                             int32_t max_tries, int32_t t_min, int32_t t_max, float* J,
                             int32_t* status, int32_t* t_star, float* j_star, void* stream);

/*
 * hop_lft_sweep_traj_tile64_f64 / _f32
 * hop_lft_sweep_traj_* (the select block of solver.py:514-522: the augmented
 * builders of augmented.py:10-87 + propagator_all_Jt_aug + argmin) with the raw
 * linearisation in the tile64 layout -- A [.][n_alloc][n*n][64], Bm
 * [.][n_alloc][n*m][64], a_res [.][n_alloc][n][64], U [.][n_alloc][m][64] and X
 * [.][n_alloc+1][n][64] (x_0 .. x_{n_use}) -- as hop_linearize_tile64_* writes it.
 * A wave of 64 problems then streams each step's raw blocks as contiguous spans
 * (the batch-major raw arrays are 64 scattered rows per piece).  Shared inputs
 * (xg, u_ref, Q, P, w, R_inv) and every output as hop_lft_sweep_traj_*; no
 * extra_stage_cost.  Small-s shapes only (s = n + 1 <= 5, m <= 2, both dtypes),
 * else HOP_E_SIZE.
 */
int hop_lft_sweep_traj_tile64_f64(const double* A, const double* Bm, const double* a_res,
                                  const double* X, const double* U, const double* xg,
                                  int64_t xg_batch_stride, const double* u_ref,
                                  int64_t u_ref_batch_stride, const double* Q,
                                  int64_t q_batch_stride, const double* P, int64_t p_batch_stride,
                                  const double* w, int64_t w_batch_stride, uint32_t wrap_mask,
                                  double q_reg, double rho_reg, const double* R_inv,
                                  int64_t r_batch_stride, int64_t batch, int32_t n_alloc,
                                  int32_t n_use, int32_t n, int32_t m, int32_t max_tries,
                                  int32_t t_min, int32_t t_max, double* J, int32_t* status,
                                  int32_t* t_star, double* j_star, void* stream);
int hop_lft_sweep_traj_tile64_f32(const float* A, const float* Bm, const float* a_res,
                                  const float* X, const float* U, const float* xg,
                                  int64_t xg_batch_stride, const float* u_ref,
                                  int64_t u_ref_batch_stride, const float* Q,
                                  int64_t q_batch_stride, const float* P, int64_t p_batch_stride,
                                  const float* w, int64_t w_batch_stride, uint32_t wrap_mask,
                                  float q_reg, float rho_reg, const float* R_inv,
                                  int64_t r_batch_stride, int64_t batch, int32_t n_alloc,
                                  int32_t n_use, int32_t n, int32_t m, int32_t max_tries,
                                  int32_t t_min, int32_t t_max, float* J, int32_t* status,
                                  int32_t* t_star, float* j_star, void* stream);

/*
 * hop_select_horizon_f64 / _f32
 * Replaces T = int(np.argmin(J[T_min-1:T_max]) + T_min)
 *   /root/reference/solver.py:522, 590, 613 (legacy ilqr_propagator.py:496, 547).
 *   J [batch][ld] ; first minimiser wins, a NaN wins like np.argmin.
 *   1 <= t_min <= t_max <= ld, else HOP_E_ARG (the reference would raise).
 */
int hop_select_horizon_f64(const double* J, int64_t batch, int32_t ld, int32_t t_min,
                           int32_t t_max, int32_t* t_star, double* j_star, void* stream);
int hop_select_horizon_f32(const float* J, int64_t batch, int32_t ld, int32_t t_min,
                           int32_t t_max, int32_t* t_star, float* j_star, void* stream);

/*
 * hop_augment_f64 / _f32
 * Replaces build_augmented_sequence_QR(F, A_list, B_list, X, U, xg, u_ref, Q, R, w,
 *            wrap_idx, q_reg, rho_reg, extra_stage_cost)
 *            /root/reference/augmented.py:10-60
 *      and build_terminal_aug_list(X, xg, alpha, wrap_idx, rho_reg)
 *            /root/reference/augmented.py:63-87
 * for a batch, on the device.  The dynamics stay with the caller: it passes
 * the affine residuals a_res[k] = F(x_k, u_k) - x_{k+1}
 * (compute_affine_residuals, linearization.py:269-270) and R_inv = chol_inv(R)
 * is the caller's (the sweep takes it as R_inv_cached).
 *
 *   A [batch][n_alloc][n][n]   Bm [batch][n_alloc][n][m]   a_res [batch][n_alloc][n]
 *   X [batch][n_alloc+1][n]    U  [batch][n_alloc][m]
 *   xg [.][n], u_ref [.][m], Q [.][n][n] (raw stage weight), w [.] (time weight),
 *   P [.][n][n] = _sym(as_terminal_weight(alpha)) (utils.py:49-62); batch
 *      strides in elements, 0 = shared.
 *   qxx_extra [batch][n_alloc][n][n], qx_extra [batch][n_alloc][n],
 *   c_extra [batch][n_alloc]: extra_stage_cost (c, cx, cxx) at (X_k, U_k), or NULL.
 *   wrap_mask bit i = wrap_idx contains i.  q_reg = 1e-9, rho_reg = 1e-12 in the
 *      reference.
 *   Outputs for steps k < n_build (s = n+1): A_aug, Q_aug, QT_aug [batch][n_build][s][s],
 *      B_aug [batch][n_build][s][m]; z0 [s] = e_s (nullable).
 */
int hop_augment_f64(const double* A, const double* Bm, const double* a_res, const double* X,
                    const double* U, const double* xg, int64_t xg_batch_stride,
                    const double* u_ref, int64_t u_ref_batch_stride, const double* Q,
                    int64_t q_batch_stride, const double* P, int64_t p_batch_stride,
                    const double* w, int64_t w_batch_stride, const double* qxx_extra,
                    const double* qx_extra, const double* c_extra, uint32_t wrap_mask,
                    double q_reg, double rho_reg, int64_t batch, int32_t n_alloc,
                    int32_t n_build, int32_t n, int32_t m, double* A_aug, double* B_aug,
                    double* Q_aug, double* QT_aug, double* z0, void* stream);
int hop_augment_f32(const float* A, const float* Bm, const float* a_res, const float* X,
                    const float* U, const float* xg, int64_t xg_batch_stride,
                    const float* u_ref, int64_t u_ref_batch_stride, const float* Q,
                    int64_t q_batch_stride, const float* P, int64_t p_batch_stride,
                    const float* w, int64_t w_batch_stride, const float* qxx_extra,
                    const float* qx_extra, const float* c_extra, uint32_t wrap_mask,
                    float q_reg, float rho_reg, int64_t batch, int32_t n_alloc,
                    int32_t n_build, int32_t n, int32_t m, float* A_aug, float* B_aug,
                    float* Q_aug, float* QT_aug, float* z0, void* stream);

/*
 * hop_lft_sweep_traj_f64 / _f32
 * Replaces the "select" block of ilqr_timeopt (solver.py:514-522):
 *   build_augmented_sequence_QR + build_terminal_aug_list
 *   + propagator_all_Jt_aug(..., T_use=n_use, R_inv_cached=R_inv) [+ argmin]
 * from the trajectory-form inputs of hop_augment_* (same meaning), for a batch.
 * For s = 13, m = 4, fp64 without extra_stage_cost the blocks are built inside
 * the sweep and never written to HBM (workspace unused, may be NULL).  Other
 * shapes run hop_augment into `workspace` and then the sweep; size it with
 * hop_lft_sweep_traj_workspace_bytes (256-B aligned; 0 = not needed).
 *   R_inv [batch or 1][m][m] (r_batch_stride = m*m or 0); J/status/t_min/t_max/
 *   t_star/j_star as hop_lft_sweep_*; max_tries as chol_inv (8).
 */
int64_t hop_lft_sweep_traj_workspace_bytes(int64_t batch, int32_t n_use, int32_t n, int32_t m,
                                           int32_t elem_bytes, int32_t has_extra);
int hop_lft_sweep_traj_f64(const double* A, const double* Bm, const double* a_res,
                           const double* X, const double* U, const double* xg,
                           int64_t xg_batch_stride, const double* u_ref,
                           int64_t u_ref_batch_stride, const double* Q, int64_t q_batch_stride,
                           const double* P, int64_t p_batch_stride, const double* w,
                           int64_t w_batch_stride, const double* qxx_extra,
                           const double* qx_extra, const double* c_extra, uint32_t wrap_mask,
                           double q_reg, double rho_reg, const double* R_inv,
                           int64_t r_batch_stride, int64_t batch, int32_t n_alloc,
                           int32_t n_use, int32_t n, int32_t m, int32_t max_tries,
                           int32_t t_min, int32_t t_max, double* J, int32_t* status,
                           int32_t* t_star, double* j_star, void* workspace,
                           int64_t workspace_bytes, void* stream);
int hop_lft_sweep_traj_f32(const float* A, const float* Bm, const float* a_res, const float* X,
                           const float* U, const float* xg, int64_t xg_batch_stride,
                           const float* u_ref, int64_t u_ref_batch_stride, const float* Q,
                           int64_t q_batch_stride, const float* P, int64_t p_batch_stride,
                           const float* w, int64_t w_batch_stride, const float* qxx_extra,
                           const float* qx_extra, const float* c_extra, uint32_t wrap_mask,
                           float q_reg, float rho_reg, const float* R_inv,
                           int64_t r_batch_stride, int64_t batch, int32_t n_alloc,
                           int32_t n_use, int32_t n, int32_t m, int32_t max_tries,
                           int32_t t_min, int32_t t_max, float* J, int32_t* status,
                           int32_t* t_star, float* j_star, void* workspace,
                           int64_t workspace_bytes, void* stream);

/*
 * hop_riccati_f64 / _f32
 * mode 0 replaces backward_pass_truncated(A_list, B_list, X, U, xg, u_ref, Q, R,
 *        alpha, T_star, lm_lambda, wrap_idx, extra_stage_cost)
 *        /root/reference/solver.py:156-230 (legacy ilqr_propagator.py:375-400)
 *        horizon[b] = T_star[b]; K/k written for steps 0..T*-1.
 * mode 1 replaces value_expansions_and_gains_prefix(A_list, B_list, X, U, xg,
 *        u_ref, Q, R, alpha, T_bar, S_right, lm_lambda, w_stage, wrap_idx,
 *        extra_stage_cost, reg_max_tries)  /root/reference/horizon_selection.py:97-212
 *        Arrays are indexed by i = t + S_right; horizon[b] = T_bar + S_right.
 *
 *   A [batch][n_alloc][n][n]  Bm [batch][n_alloc][n][m]
 *   X [batch][n_alloc+1][n]   U  [batch][n_alloc][m]
 *   xg [.][n], u_ref [.][m], Q [.][n][n], R [.][m][m], Qf [.][n][n]
 *      (batch strides in elements; Qf = as_terminal_weight(alpha), utils.py:49-62)
 *   qxx_extra [batch][n_alloc][n][n], qx_extra [batch][n_alloc][n],
 *   c_extra [batch][n_alloc]: extra_stage_cost (c, cx, cxx) evaluated by the
 *      caller at (X_k, U_k); all NULL when there is no extra cost.
 *   lm [batch] (lm_lambda), w_stage (mode 1), wrap_mask bit i = wrap_idx has i.
 *   Outputs: K [batch][n_alloc][m][n], k [batch][n_alloc][m];
 *      nullable Vxx [batch][n_alloc+1][n][n], Vx [batch][n_alloc+1][n],
 *      V0 [batch][n_alloc+1]; status [batch] (HOP_ST_FAIL = ok=False / raise).
 */
int hop_riccati_f64(const double* A, const double* Bm, const double* X, const double* U,
                    const double* xg, int64_t xg_batch_stride, const double* u_ref,
                    int64_t u_ref_batch_stride, const double* Q, int64_t q_batch_stride,
                    const double* R, int64_t r_batch_stride, const double* Qf,
                    int64_t qf_batch_stride, const double* qxx_extra, const double* qx_extra,
                    const double* c_extra, const int32_t* horizon, const double* lm,
                    double w_stage, uint32_t wrap_mask, int32_t mode, int32_t reg_max_tries,
                    int64_t batch, int32_t n_alloc, int32_t n, int32_t m, double* K, double* k,
                    double* Vxx, double* Vx, double* V0, int32_t* status, void* stream);
int hop_riccati_f32(const float* A, const float* Bm, const float* X, const float* U,
                    const float* xg, int64_t xg_batch_stride, const float* u_ref,
                    int64_t u_ref_batch_stride, const float* Q, int64_t q_batch_stride,
                    const float* R, int64_t r_batch_stride, const float* Qf,
                    int64_t qf_batch_stride, const float* qxx_extra, const float* qx_extra,
                    const float* c_extra, const int32_t* horizon, const float* lm,
                    float w_stage, uint32_t wrap_mask, int32_t mode, int32_t reg_max_tries,
                    int64_t batch, int32_t n_alloc, int32_t n, int32_t m, float* K, float* k,
                    float* Vxx, float* Vx, float* V0, int32_t* status, void* stream);

/*
 * hop_bruteforce_jcurve_f64 / _f32
 * replaces bruteforce_all_Jt_backward_expansion(A_list, B_list, X, U, xg, u_ref, Q,
 *          R, alpha, w, T_max, lm_lambda, wrap_idx, extra_stage_cost)
 *          /root/reference/solver.py:293-358 (the select step of
 *          ilqr_timeopt(method="bruteforce"), solver.py:525-532 / 607-614)
 *   J[b][T-1] = V_0 of the length-T value-expansion sweep (mode 1 arithmetic with
 *   the fixed lm_lambda and chol_solve's jitter ladder) for T = 1..t_max: all
 *   t_max sweeps of every problem in ONE launch (one workgroup per 16-problem block
 *   and horizon, a block's horizons adjacent, longest first).  Inputs as
 *   hop_riccati_*; t_max <= n_alloc.
 *   Outputs: J [batch][t_max]; status [batch][t_max] per horizon (HOP_ST_FAIL /
 *   HOP_ST_NONFINITE where the reference raises LinAlgError / FloatingPointError;
 *   J is NaN there).
 */
int hop_bruteforce_jcurve_f64(const double* A, const double* Bm, const double* X,
                              const double* U, const double* xg, int64_t xg_batch_stride,
                              const double* u_ref, int64_t u_ref_batch_stride, const double* Q,
                              int64_t q_batch_stride, const double* R, int64_t r_batch_stride,
                              const double* Qf, int64_t qf_batch_stride, const double* qxx_extra,
                              const double* qx_extra, const double* c_extra, double lm_lambda,
                              double w_stage, uint32_t wrap_mask, int64_t batch, int32_t n_alloc,
                              int32_t n, int32_t m, int32_t t_max, double* J, int32_t* status,
                              void* stream);
int hop_bruteforce_jcurve_f32(const float* A, const float* Bm, const float* X, const float* U,
                              const float* xg, int64_t xg_batch_stride, const float* u_ref,
                              int64_t u_ref_batch_stride, const float* Q, int64_t q_batch_stride,
                              const float* R, int64_t r_batch_stride, const float* Qf,
                              int64_t qf_batch_stride, const float* qxx_extra,
                              const float* qx_extra, const float* c_extra, float lm_lambda,
                              float w_stage, uint32_t wrap_mask, int64_t batch, int32_t n_alloc,
                              int32_t n, int32_t m, int32_t t_max, float* J, int32_t* status,
                              void* stream);

/*
 * hop_riccati_legacy_f64 / hop_bruteforce_jcurve_legacy_f64
 * The legacy twin's passes (ilqr_propagator.py): mode 0 replaces its
 *   backward_pass_truncated (ilqr_propagator.py:375-400), mode 1 its
 *   value_expansions_and_gains_prefix (ilqr_propagator.py:237-287), the J-curve
 *   entry its bruteforce_all_Jt_backward_expansion (ilqr_propagator.py:426-454).
 *   Mode 1 and the J curve solve with the legacy chol_solve
 *   (ilqr_propagator.py:33-43): 4 jitters, then np.linalg.lstsq of sym(Quu_reg)
 *   -- the minimum-norm pinv solve, marked HOP_ST_LU -- instead of a failure.
 *   Mode 0 is the legacy backward_pass_truncated: a Cholesky gate on Quu_reg
 *   without jitter fails the row (HOP_ST_FAIL, the reference's ok=False) before
 *   any solve, so its solves succeed at the first 1e-9 jitter and never reach
 *   lstsq.  Quu_reg = _sym(Quu) + lm I (no floor, no lambda ladder); no
 *   finiteness checks (NaN propagates; a non-finite Quu_reg that reaches lstsq
 *   fails the row, as numpy's lstsq raises).  The terminal weight is Qf = alpha I
 *   (the legacy passes take a scalar alpha).  Arguments as hop_riccati_f64 /
 *   hop_bruteforce_jcurve_f64 without the extra stage cost and reg_max_tries;
 *   mode 1 and the J curve need m <= 11 (HOP_E_SIZE otherwise).
 */
int hop_riccati_legacy_f64(const double* A, const double* Bm, const double* X, const double* U,
                           const double* xg, int64_t xg_batch_stride, const double* u_ref,
                           int64_t u_ref_batch_stride, const double* Q, int64_t q_batch_stride,
                           const double* R, int64_t r_batch_stride, const double* Qf,
                           int64_t qf_batch_stride, const int32_t* horizon, const double* lm,
                           double w_stage, uint32_t wrap_mask, int32_t mode, int64_t batch,
                           int32_t n_alloc, int32_t n, int32_t m, double* K, double* k,
                           double* Vxx, double* Vx, double* V0, int32_t* status, void* stream);
int hop_bruteforce_jcurve_legacy_f64(const double* A, const double* Bm, const double* X,
                                     const double* U, const double* xg, int64_t xg_batch_stride,
                                     const double* u_ref, int64_t u_ref_batch_stride,
                                     const double* Q, int64_t q_batch_stride, const double* R,
                                     int64_t r_batch_stride, const double* Qf,
                                     int64_t qf_batch_stride, double lm_lambda, double w_stage,
                                     uint32_t wrap_mask, int64_t batch, int32_t n_alloc,
                                     int32_t n, int32_t m, int32_t t_max, double* J,
                                     int32_t* status, void* stream);

/*
 * Batched dynamics and finite-difference linearisation.
 * System ids (the reference's systems.py makers, F discretised with the given dt):
 *   0 double integrator  make_double_integrator     systems.py:28-50    n=2,  m=1
 *   1 cart-pole          make_cartpole_swingup      systems.py:57-112   n=4,  m=1
 *   2 quadrotor          make_quadrotor             systems.py:119-230  n=12, m=4
 *   3 point mass         make_pointmass_navigation  systems.py:237-296  n=4,  m=2
 *   4 segway             make_segway_balance        systems.py:303-349  n=4,  m=1
 * hop_system_dims writes n and m of a system id (either pointer may be NULL).
 */
#define HOP_SYS_DOUBLE_INTEGRATOR 0
#define HOP_SYS_CARTPOLE 1
#define HOP_SYS_QUADROTOR 2
#define HOP_SYS_POINTMASS 3
#define HOP_SYS_SEGWAY 4
int hop_system_dims(int32_t system, int32_t* n, int32_t* m);

/*
 * hop_linearize_f64
 * Replaces linearize_forward_diff_traj(F, X, U, epsx, epsu, relx, relu)
 *            /root/reference/linearization.py:216-262   (central = 0)
 *      and linearize_central_diff_traj(F, X, U, epsx, epsu, relx, relu)
 *            /root/reference/linearization.py:177-211   (central = 1)
 *      plus compute_affine_residuals(F, X, U)  linearization.py:269-270
 * for a batch of trajectories, steps k < n_use (len(U) in the reference).
 *   X [batch][n_alloc+1][n]   U [batch][n_alloc][m]
 *   A [batch][n_alloc][n][n]  Bm [batch][n_alloc][n][m]  (the layout hop_augment_*,
 *      hop_lft_sweep_traj_* and hop_riccati_* read)
 *   a_res [batch][n_alloc][n] = F(x_k, u_k) - x_{k+1} (nullable)
 *   Fx    [batch][n_alloc][n] = F(x_k, u_k)          (nullable)
 *   h = max(eps, rel * max(1, |v|)) per entry (reference defaults 1e-5 / 1e-6);
 *   forward differences give an all-NaN (A_k, B_k) when F(x_k, u_k) is not finite.
 */
int hop_linearize_f64(int32_t system, double dt, const double* X, const double* U,
                      int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                      double epsx, double epsu, double relx, double relu, double* A,
                      double* Bm, double* a_res, double* Fx, void* stream);

/*
 * hop_linearize_tile64_f64 / _f32
 * hop_linearize_f64 (linearization.py:177-270, computed in fp64) writing the tile64
 * layout hop_lft_sweep_traj_tile64_* reads, as fp64 or fp32: A [ceil(B/64)][n_alloc]
 * [n*n][64], Bm [.][n_alloc][n*m][64], a_res [.][n_alloc][n][64] (nullable), and the
 * tile64 copies of the trajectory, Xt [.][n_alloc+1][n][64] (rows 0 .. n_use) and
 * Ut [.][n_alloc][m][64] (rows < n_use).  Padding slots of the last tile are 0;
 * steps >= n_use are not written.  X [batch][n_alloc+1][n], U [batch][n_alloc][m]
 * are fp64 batch-major as for hop_linearize_f64.  Size each output with
 * hop_tile64_elems(batch, n_alloc (+1 for Xt), elems).
 */
int hop_linearize_tile64_f64(int32_t system, double dt, const double* X, const double* U,
                             int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                             double epsx, double epsu, double relx, double relu, double* A,
                             double* Bm, double* a_res, double* Xt, double* Ut, void* stream);
int hop_linearize_tile64_f32(int32_t system, double dt, const double* X, const double* U,
                             int64_t batch, int32_t n_alloc, int32_t n_use, int32_t central,
                             double epsx, double epsu, double relx, double relu, float* A,
                             float* Bm, float* a_res, float* Xt, float* Ut, void* stream);

/*
 * hop_dynamics_f64
 * Replaces F(x, u) of the systems above (one discrete step) for `count`
 * independent pairs: Xn[q] = F(X[q], U[q]), rows `*_stride` elements apart.
 */
int hop_dynamics_f64(int32_t system, double dt, const double* X, int64_t x_stride,
                     const double* U, int64_t u_stride, int64_t count, double* Xn,
                     int64_t xn_stride, void* stream);

/*
 * Forward pass and outer-loop bookkeeping of ilqr_timeopt.
 * Cost parameters shared by the entry points below (device pointers, each with a
 * batch stride in elements: 0 = one block shared by the whole batch):
 *   xg [n], u_ref [m], Q [n][n], R [m][m], Qf [n][n] = as_terminal_weight(alpha)
 *   (utils.py:49-62), w [1] (the time weight), obstacles [n_obs][4] =
 *   (cx, cy, radius, weight) of the point-mass extra_stage_cost
 *   (systems.py:271-293; NULL / 0 for none), wrap_mask = bit i for wrap_idx i.
 */

/*
 * hop_rollout_f64
 * Replaces rollout(F, x0, U, max_state_norm)  /root/reference/solver.py:42-62
 *   x0 [batch or 1][n] (x0_batch_stride 0 or n), U [batch][N][m] -> X [batch][N+1][n];
 *   the first step whose state is not finite or has ||x|| > max_state_norm sets
 *   X[k+1:] = NaN.
 */
int hop_rollout_f64(int32_t system, double dt, const double* x0, int64_t x0_batch_stride,
                    const double* U, int64_t batch, int32_t N, double max_state_norm, double* X,
                    void* stream);

/*
 * hop_cost_true_f64
 * Replaces cost_timeopt_true(X, U, xg, u_ref, Q, R, alpha, w, T_star, wrap_idx,
 *          extra_stage_cost)  /root/reference/solver.py:65-102
 *   X [batch][N+1][n], U [batch][N][m], T_star [batch] -> J [batch]
 *   (+inf for T* <= 0 or non-finite data, NaN for T* > N where the reference
 *   would raise IndexError).
 */
int hop_cost_true_f64(int32_t system, const double* X, const double* U, const int32_t* T_star,
                      const double* xg, int64_t xg_bs, const double* u_ref, int64_t ur_bs,
                      const double* Q, int64_t q_bs, const double* R, int64_t r_bs,
                      const double* Qf, int64_t qf_bs, const double* w, int64_t w_bs,
                      const double* obstacles, int32_t n_obs, uint32_t wrap_mask, int64_t batch,
                      int32_t N, double* J, void* stream);

/*
 * hop_forward_linesearch_f64
 * Replaces forward_linesearch_fixedT(F, X, U, xg, u_ref, Q, R, alpha, w, T_star,
 *          k_list, K_list, alphas, wrap_idx, extra_stage_cost)
 *          /root/reference/solver.py:233-286
 *   K [batch][N][m][n], k [batch][N][m] (hop_riccati_f64 mode 0 output),
 *   alphas: HOST array of n_alpha <= 8 step sizes (reference (1, .5, .25, .1, .05)),
 *   active [batch] nullable (0 = skip: X' = X, U' = U, accepted = -2).
 *   Out: X_new [batch][N+1][n], U_new [batch][N][m], J [batch] (the accepted J'
 *   or J_old), J_old [batch], accepted [batch] = index of the accepted alpha or -1.
 *   workspace: hop_forward_workspace_bytes(system, batch, N, n_alpha) bytes.
 */
size_t hop_forward_workspace_bytes(int32_t system, int64_t batch, int32_t N, int32_t n_alpha);
int hop_forward_linesearch_f64(int32_t system, double dt, const double* X, const double* U,
                               const double* xg, int64_t xg_bs, const double* u_ref,
                               int64_t ur_bs, const double* Q, int64_t q_bs, const double* R,
                               int64_t r_bs, const double* Qf, int64_t qf_bs, const double* w,
                               int64_t w_bs, const double* obstacles, int32_t n_obs,
                               uint32_t wrap_mask, const int32_t* T_star, const int32_t* active,
                               const double* K, const double* k, const double* alphas,
                               int32_t n_alpha, int64_t batch, int32_t N, void* workspace,
                               size_t workspace_bytes, double* X_new, double* U_new, double* J,
                               double* J_old, int32_t* accepted, void* stream);

/*
 * hop_obstacle_cost_f64
 * Replaces the point-mass extra_stage_cost(x, u) -> (c, cx, cxx)
 *          /root/reference/systems.py:271-293
 * for `count` states X[r * x_stride + 0..n-1]: c [count], cx [count][n],
 * cxx [count][n][n] (each nullable).  Feeds qxx_extra / qx_extra / c_extra of
 * hop_augment_* / hop_lft_sweep_traj_* / hop_riccati_*.
 */
int hop_obstacle_cost_f64(const double* X, int64_t x_stride, int64_t count, int32_t n,
                          const double* obstacles, int32_t n_obs, double* c, double* cx,
                          double* cxx, void* stream);

/*
 * hop_ilqr_accept_f64
 * The accept / LM / stop-rule step of ilqr_timeopt  /root/reference/solver.py:737-752
 * (warm = 1: the warm-start record of solver.py:548-553) per problem:
 *   accepted (hop_forward_linesearch_f64) >= 0 and J finite -> T_bar = T_star,
 *   append (J, T_star) to J_hist/T_hist [batch][hist_cap], lm = max(lm/10, 1e-12);
 *   else lm *= 10.  done = 1 once |dJ|/(|J|+1e-12) < 1e-4 over the last two records
 *   and the last three T are equal.  Problems with done = 1 are left untouched.
 */
int hop_ilqr_accept_f64(int64_t batch, int32_t warm, const double* J, const int32_t* accepted,
                        const int32_t* T_star, double* lm, int32_t* T_bar, double* J_hist,
                        int32_t* T_hist, int32_t* n_hist, int32_t hist_cap, int32_t* done,
                        void* stream);

/*
 * hop_ilqr_select_mask
 * The per-iteration masks of the device outer loop (solver.py:514-525, 581-597):
 * a problem whose select block raised (sel_status has ST_FAIL or ST_NONFINITE:
 * the reference's FloatingPointError / LinAlgError out of propagator_all_Jt_aug)
 * and is not done yet is marked crashed and done; active = the problem is not
 * done and its truncated Riccati pass succeeded (ric_status has no ST_FAIL), the
 * line search's mask.  One launch instead of a chain of elementwise ops.
 */
int hop_ilqr_select_mask(int64_t batch, const int32_t* sel_status, const int32_t* ric_status,
                         int32_t* done, int32_t* crashed, int32_t* active, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HOP_H */
