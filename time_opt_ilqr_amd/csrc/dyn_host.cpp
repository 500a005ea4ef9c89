// Host build of dynamics.hpp for the CPU test suite (not part of libhop_amd.so):
//   g++ -O2 -std=c++17 -ffp-contract=off -fno-builtin-{sin,cos,tan} -shared -fPIC -DHOP_HD=
//       dyn_host.cpp -o libdyn_host.so
// Runs linearize.hip's per-step arithmetic (the trig jobs, f0, the columns) on
// the CPU, step by step, so the CPU tests pin it against the reference's fixtures.
#include <stdint.h>

#include "dynamics.hpp"

using namespace hop::dyn;

template <int SYS, bool CEN>
static void lin_run(double dt, const double* X, const double* U, int64_t batch, int nalloc,
                    int nuse, double epsx, double epsu, double relx, double relu, double* A,
                    double* B, double* a_res, double* Fx) {
  constexpr int n = state_dim(SYS), m = control_dim(SYS);
  constexpr int TS = trig_slots(SYS, CEN) > 0 ? trig_slots(SYS, CEN) : 1;
  for (int64_t b = 0; b < batch; ++b)
    for (int k = 0; k < nuse; ++k) {
      const int64_t r = b * nalloc + k, xr = r + b;
      const double* x = X + xr * n;
      const double* u = U + r * m;
      double ts[TS] = {}, f0[n], col[n];
      for (int job = 0; job < trig_jobs(SYS, CEN); ++job) quad_trig_job(x, job, epsx, relx, ts);
      if constexpr (SYS == kQuadrotor)
        f_quadrotor_t(x, u, dt, QuadTrig{ts[0], ts[1], ts[2], ts[3], ts[4], ts[5], ts[6]}, f0);
      else
        eval<SYS>(x, u, dt, f0);
      bool fin = true;
      for (int i = 0; i < n; ++i) fin = fin && finite_d(f0[i]);
      for (int i = 0; i < n; ++i) {
        if (a_res) a_res[r * n + i] = f0[i] - X[(xr + 1) * n + i];
        if (Fx) Fx[r * n + i] = f0[i];
      }
      for (int j = 0; j < n + m; ++j) {
        fd_col<SYS, CEN>(x, u, f0, fin, ts, dt, j, epsx, epsu, relx, relu, col);
        for (int i = 0; i < n; ++i) {
          if (j < n) A[r * n * n + i * n + j] = col[i];
          else B[r * n * m + i * m + (j - n)] = col[i];
        }
      }
    }
}

template <int SYS>
static void lin_sys(int central, double dt, const double* X, const double* U, int64_t batch,
                    int nalloc, int nuse, double epsx, double epsu, double relx, double relu,
                    double* A, double* B, double* a_res, double* Fx) {
  if (central)
    lin_run<SYS, true>(dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx);
  else
    lin_run<SYS, false>(dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx);
}

extern "C" {

int dyn_host_linearize(int sys, double dt, const double* X, const double* U, int64_t batch,
                       int nalloc, int nuse, int central, double epsx, double epsu, double relx,
                       double relu, double* A, double* B, double* a_res, double* Fx) {
  switch (sys) {
    case kDI: lin_sys<kDI>(central, dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx); break;
    case kCartpole: lin_sys<kCartpole>(central, dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx); break;
    case kQuadrotor: lin_sys<kQuadrotor>(central, dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx); break;
    case kPointmass: lin_sys<kPointmass>(central, dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx); break;
    case kSegway: lin_sys<kSegway>(central, dt, X, U, batch, nalloc, nuse, epsx, epsu, relx, relu, A, B, a_res, Fx); break;
    default: return -1;
  }
  return 0;
}

}  // extern "C"
