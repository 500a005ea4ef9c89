// Batched dynamics and finite-difference linearisation along trajectories
//  on the device:
//   linearize_forward_diff_traj  linearization.py:216-262  -> A_k, B_k
//   linearize_central_diff_traj  linearization.py:177-211  -> A_k, B_k
//   compute_affine_residuals     linearization.py:269-270  -> a_k = F(x_k,u_k) - x_{k+1}
// for every step k < n_use of every problem, with the systems of dynamics.hpp.
// The outputs are laid out as the augment / sweep / Riccati entry points read
// them (A [batch][n_alloc][n][n], B [batch][n_alloc][n][m], a [batch][n_alloc][n]).
//
// One workgroup owns TILE = 64 consecutive (problem, step) pairs:
//   phase 1  x_k, u_k -> LDS (coalesced); for the quadrotor every thread takes one
//            trigonometry job (the base point, or one Euler angle moved by +-h),
//            so the sin/cos/tan a step needs are evaluated 4 (7 central) times
//            instead of once per column and never under lane divergence
//   phase 2  f0 = F(x_k, u_k) per step -> LDS; a_k and F(x_k, u_k) written
//            as contiguous runs
//   phase 3  one thread per (step, column): the perturbed evaluation(s) and
//            the column of A or B; a wave writes 4 steps x 16 columns (quadrotor)
//            so each store covers whole rows of A_k and B_k
// The per-step arithmetic is dynamics.hpp's, shared with the host test build.
#include "hop_device.hpp"
#include "hop_kernels.hpp"
#include "dynamics.hpp"

namespace hop {
namespace lin {

using namespace hop::dyn;

constexpr int TPB = 256;
constexpr int TILE = 64;
// A_k, B_k (and a_k, F(x_k, u_k)) are written once and read by the next stage
// from HBM (629 MB at B = 4096, N = 100, far past the MALL): non-temporal
// stores, 0.213 -> 0.158 ms (forward) and 0.239 -> 0.196 ms (central) for the
// quadrotor at B = 4096, N = 100 (tools/ab_libs.py, same process, bitwise equal)
#define HOP_LIN_STORE(v, p) __builtin_nontemporal_store((v), (p))

// LY 0: one workgroup per 64 consecutive (problem, step) pairs, fp64 batch-major
// outputs.  LY 2: one workgroup per (64-problem tile, step k), outputs of type OT in
// the tile64 layout [B/64][n_alloc][elems][64] (include/hop.h), plus the tile64
// copies of x_k (and x_{n_use} for k = n_use - 1) and u_k the trajectory-form
// select reads (hop_lft_sweep_traj_tile64_*): every store is 64 consecutive slots.
template <int SYS, bool CEN, class OT = double, int LY = 0>
__global__ __launch_bounds__(TPB) void linearize_kernel(LinArgs a) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS), NC = n + m;
  constexpr int TS = trig_slots(SYS, CEN) > 0 ? trig_slots(SYS, CEN) : 1;
  constexpr int NJOB = trig_jobs(SYS, CEN);
  __shared__ double sx[TILE * n], su[TILE * m], sf[TILE * n], st[TILE * TS];
  __shared__ long long srow[TILE];  // b * n_alloc + k, -1 past the end
  __shared__ long long sxrow[TILE];  // b * (n_alloc + 1) + k
  __shared__ int sfin[TILE];
  const int tid = threadIdx.x;
  const long long total = a.batch * (long long)a.nuse;
  const long long g0 = (long long)blockIdx.x * TILE;
  // LY 2: tile blk, step kt; slot ls of element e at ((blk * nal + kt) * E + e) * 64 + ls
  const long long blk = LY == 2 ? (long long)blockIdx.x / a.nuse : 0;
  const int kt = LY == 2 ? (int)((long long)blockIdx.x - blk * a.nuse) : 0;
  auto t64 = [&](long long nal, int E, int e, int ls) {
    return ((blk * nal + kt) * E + e) * 64 + ls;
  };
  if (tid < TILE) {
    long long r = -1, xr = 0;
    if constexpr (LY == 2) {
      const long long b = blk * TILE + tid;
      if (b < a.batch) {
        r = b * a.nalloc + kt;
        xr = r + b;
      }
    } else {
      const long long g = g0 + tid;
      if (g < total) {
        const long long b = g / a.nuse, k = g - b * a.nuse;
        r = b * a.nalloc + k;
        xr = r + b;
      }
    }
    srow[tid] = r;
    sxrow[tid] = xr;
  }
  __syncthreads();
  for (int e = tid; e < TILE * n; e += TPB) {
    const int ls = e / n, i = e - ls * n;
    sx[e] = srow[ls] >= 0 ? a.X[sxrow[ls] * n + i] : 0.0;
  }
  for (int e = tid; e < TILE * m; e += TPB) {
    const int ls = e / m, i = e - ls * m;
    su[e] = srow[ls] >= 0 ? a.U[srow[ls] * m + i] : 0.0;
  }
  __syncthreads();
  if constexpr (LY == 2) {  // the tile64 copies of x_k (x_{n_use} too) and u_k; padding slots 0
    OT* Xt = reinterpret_cast<OT*>(a.Xt);
    OT* Ut = reinterpret_cast<OT*>(a.Ut);
    for (int e = tid; e < TILE * n; e += TPB) {
      const int i = e / TILE, ls = e - i * TILE;
      HOP_LIN_STORE((OT)sx[ls * n + i], Xt + t64(a.nalloc + 1, n, i, ls));
      if (kt == a.nuse - 1)
        HOP_LIN_STORE(srow[ls] >= 0 ? (OT)a.X[(sxrow[ls] + 1) * n + i] : OT(0),
                      Xt + t64(a.nalloc + 1, n, i, ls) + 64 * n);
    }
    for (int e = tid; e < TILE * m; e += TPB) {
      const int i = e / TILE, ls = e - i * TILE;
      HOP_LIN_STORE((OT)su[ls * m + i], Ut + t64(a.nalloc, m, i, ls));
    }
  }
  if constexpr (NJOB > 0) {
    for (int q = tid; q < TILE * NJOB; q += TPB) {
      const int ls = q % TILE, job = q / TILE;
      quad_trig_job(sx + ls * n, job, a.epsx, a.relx, st + ls * TS);
    }
    __syncthreads();
  }
  // phase 2: f0, the residual and F(x_k, u_k)
  if (tid < TILE) {
    double f0[n];
    if constexpr (SYS == kQuadrotor) {
      const double* ts = st + tid * TS;
      f_quadrotor_t(sx + tid * n, su + tid * m, a.dt,
                    QuadTrig{ts[0], ts[1], ts[2], ts[3], ts[4], ts[5], ts[6]}, f0);
    } else {
      eval<SYS>(sx + tid * n, su + tid * m, a.dt, f0);
    }
    bool fin = true;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      sf[tid * n + i] = f0[i];
      fin = fin && finite_d(f0[i]);
    }
    sfin[tid] = fin;
  }
  __syncthreads();
  if constexpr (LY == 2) {
    OT* at = reinterpret_cast<OT*>(a.a_res);
    if (at) {
      for (int e = tid; e < TILE * n; e += TPB) {
        const int i = e / TILE, ls = e - i * TILE;
        const long long r = srow[ls];
        const double v = r >= 0 ? sf[ls * n + i] - a.X[(sxrow[ls] + 1) * n + i] : 0.0;
        HOP_LIN_STORE((OT)v, at + t64(a.nalloc, n, i, ls));
      }
    }
  } else if (a.a_res || a.Fx) {
    for (int e = tid; e < TILE * n; e += TPB) {
      const int ls = e / n, i = e - ls * n;
      const long long r = srow[ls];
      if (r < 0) continue;
      if (a.a_res)
        HOP_LIN_STORE(sf[e] - a.X[(sxrow[ls] + 1) * n + i],
                      reinterpret_cast<double*>(a.a_res) + r * n + i);
      if (a.Fx) HOP_LIN_STORE(sf[e], a.Fx + r * n + i);
    }
  }
  // phase 3: one (step, column) per thread (LY 2: a wave = one column of 64 slots)
  for (int it = tid; it < TILE * NC; it += TPB) {
    const int ls = LY == 2 ? it % TILE : it / NC, j = LY == 2 ? it / TILE : it - ls * NC;
    const long long r = srow[ls];
    if constexpr (LY == 2) {
      if (r < 0) {  // padding slot: zeros
        OT* At = reinterpret_cast<OT*>(a.A);
        OT* Bt = reinterpret_cast<OT*>(a.B);
#pragma unroll
        for (int i = 0; i < n; ++i) {
          if (j < n) HOP_LIN_STORE(OT(0), At + t64(a.nalloc, n * n, i * n + j, ls));
          else HOP_LIN_STORE(OT(0), Bt + t64(a.nalloc, n * m, i * m + (j - n), ls));
        }
        continue;
      }
    }
    if (r < 0) continue;
    double x[n], u[m], f0[n], col[n];
#pragma unroll
    for (int i = 0; i < n; ++i) x[i] = sx[ls * n + i], f0[i] = sf[ls * n + i];
#pragma unroll
    for (int i = 0; i < m; ++i) u[i] = su[ls * m + i];
    fd_col<SYS, CEN>(x, u, f0, sfin[ls] != 0, st + ls * TS, a.dt, j, a.epsx, a.epsu, a.relx,
                     a.relu, col);
    if constexpr (LY == 2) {
      OT* At = reinterpret_cast<OT*>(a.A);
      OT* Bt = reinterpret_cast<OT*>(a.B);
#pragma unroll
      for (int i = 0; i < n; ++i) {
        if (j < n) HOP_LIN_STORE((OT)col[i], At + t64(a.nalloc, n * n, i * n + j, ls));
        else HOP_LIN_STORE((OT)col[i], Bt + t64(a.nalloc, n * m, i * m + (j - n), ls));
      }
    } else if (j < n) {
      double* Ak = reinterpret_cast<double*>(a.A) + r * (n * n) + j;
#pragma unroll
      for (int i = 0; i < n; ++i) HOP_LIN_STORE(col[i], Ak + i * n);
    } else {
      double* Bk = reinterpret_cast<double*>(a.B) + r * (n * m) + (j - n);
#pragma unroll
      for (int i = 0; i < n; ++i) HOP_LIN_STORE(col[i], Bk + i * m);
    }
  }
}

// x_{k+1} = F(x_k, u_k) for `count` independent (x, u) pairs
template <int SYS>
__global__ __launch_bounds__(TPB) void dynamics_kernel(DynArgs a) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  const long long q = (long long)blockIdx.x * TPB + threadIdx.x;
  if (q >= a.count) return;
  double x[n], u[m], o[n];
#pragma unroll
  for (int i = 0; i < n; ++i) x[i] = a.X[q * a.x_stride + i];
#pragma unroll
  for (int i = 0; i < m; ++i) u[i] = a.U[q * a.u_stride + i];
  eval<SYS>(x, u, a.dt, o);
#pragma unroll
  for (int i = 0; i < n; ++i) a.Xn[q * a.xn_stride + i] = o[i];
}

template <int SYS, bool CEN>
hipError_t launch_lin(const LinArgs& a, hipStream_t stream) {
  if (a.tile64) {  // one workgroup per (64-problem tile, step)
    const long long blocks = (a.batch + TILE - 1) / TILE * (long long)a.nuse;
    if (a.out_f32)
      hipLaunchKernelGGL((linearize_kernel<SYS, CEN, float, 2>), dim3((unsigned)blocks),
                         dim3(TPB), 0, stream, a);
    else
      hipLaunchKernelGGL((linearize_kernel<SYS, CEN, double, 2>), dim3((unsigned)blocks),
                         dim3(TPB), 0, stream, a);
    return hipGetLastError();
  }
  const long long total = a.batch * (long long)a.nuse;
  const long long blocks = (total + TILE - 1) / TILE;
  hipLaunchKernelGGL((linearize_kernel<SYS, CEN>), dim3((unsigned)blocks), dim3(TPB), 0, stream,
                     a);
  return hipGetLastError();
}

template <int SYS>
hipError_t launch_lin_sys(const LinArgs& a, hipStream_t stream) {
  return a.central ? launch_lin<SYS, true>(a, stream) : launch_lin<SYS, false>(a, stream);
}

template <int SYS>
hipError_t launch_dyn(const DynArgs& a, hipStream_t stream) {
  const long long blocks = (a.count + TPB - 1) / TPB;
  hipLaunchKernelGGL((dynamics_kernel<SYS>), dim3((unsigned)blocks), dim3(TPB), 0, stream, a);
  return hipGetLastError();
}

}  // namespace lin

hipError_t dispatch_linearize(const LinArgs& a, hipStream_t stream) {
  switch (a.sys) {
    case dyn::kDI: return lin::launch_lin_sys<dyn::kDI>(a, stream);
    case dyn::kCartpole: return lin::launch_lin_sys<dyn::kCartpole>(a, stream);
    case dyn::kQuadrotor: return lin::launch_lin_sys<dyn::kQuadrotor>(a, stream);
    case dyn::kPointmass: return lin::launch_lin_sys<dyn::kPointmass>(a, stream);
    default: return lin::launch_lin_sys<dyn::kSegway>(a, stream);
  }
}

hipError_t dispatch_dynamics(const DynArgs& a, hipStream_t stream) {
  switch (a.sys) {
    case dyn::kDI: return lin::launch_dyn<dyn::kDI>(a, stream);
    case dyn::kCartpole: return lin::launch_dyn<dyn::kCartpole>(a, stream);
    case dyn::kQuadrotor: return lin::launch_dyn<dyn::kQuadrotor>(a, stream);
    case dyn::kPointmass: return lin::launch_dyn<dyn::kPointmass>(a, stream);
    default: return lin::launch_dyn<dyn::kSegway>(a, stream);
  }
}

}  // namespace hop
