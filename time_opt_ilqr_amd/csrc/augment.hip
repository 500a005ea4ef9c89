// Batched augmented-block builders on the device:
//   build_augmented_sequence_QR  augmented.py:10-60  -> A_aug, B_aug, Q_aug
//   build_terminal_aug_list      augmented.py:63-87  -> QT_aug
// for every problem of a batch, from the raw linearisation (A_k, B_k, the affine
// residual a_k = F(x_k,u_k) - x_{k+1}) and the cost terms (Q, P = _sym(Qf), w).
// This is the path for shapes without an in-kernel builder (lft_sweep_v2.hip
// builds the blocks inside the sweep for s = 13, m = 4).
//
// HBM-bound: per step it reads n^2 + nm + 2n + m values (+ extras) and writes
// 3 s^2 + s m.  One workgroup owns 256/n consecutive steps of one problem: phase 1
// forms the per-step vectors (e_k, e_{k+1}, du_k, Q e, P e, a~) in LDS, phase 2
// writes the blocks as contiguous, coalesced runs.
#include "hop_device.hpp"
#include "hop_kernels.hpp"

namespace hop {
namespace aug {

constexpr int TPB = 256;
// steps per workgroup: phase 1 maps one thread per (step, state) pair, so a
// workgroup covers 256 / n steps (small n: long contiguous output runs)
__host__ __device__ inline int steps_per_block(int n) { return TPB / n; }

template <class T>
__global__ __launch_bounds__(TPB) void augment_kernel(AugArgs<T> a) {
  const TrajArgs<T>& t = a.t;
  const int n = t.n, m = t.m, s = n + 1;
  const int KS = steps_per_block(n);
  const int nchunk = (a.nbuild + KS - 1) / KS;
  const long long b = blockIdx.x / nchunk;
  const int k0 = (blockIdx.x % nchunk) * KS;
  const int ks = min(KS, a.nbuild - k0);
  const int NA = a.nalloc;
  // per-step vectors, [step][state] with row length n (KS * n <= 256)
  __shared__ T e0[TPB], e1[TPB], qe[TPB], pe[TPB], at[TPB];
  __shared__ T eqe[TPB], epe[TPB];
  __shared__ T sQ[16 * 16], sQs[16 * 16], sP[16 * 16];

  const T* xg = t.xg + b * t.xg_bs;
  const T* ur = t.u_ref + b * t.ur_bs;
  const T* Q = t.Q + b * t.q_bs;
  const T* P = t.P + b * t.p_bs;
  const T wt = t.w[b * t.w_bs];
  if (a.z0 && blockIdx.x == 0 && threadIdx.x < s) a.z0[threadIdx.x] = threadIdx.x == n ? T(1) : T(0);
  const int tid = threadIdx.x, kk = tid / n, i = tid - kk * n, k = k0 + kk;
  const bool row_ok = kk < ks;  // (threads past KS * n idle in phase 1)

  // phase 0: Q, _sym(Q) + q_reg I and P into LDS (one coalesced pass)
  for (int idx = tid; idx < n * n; idx += TPB) {
    const int r = idx / n, c = idx - r * n;
    const T q = Q[idx];
    sQ[idx] = q;
    sQs[idx] = T(0.5) * (q + Q[c * n + r]) + (r == c ? t.q_reg : T(0));
    sP[idx] = P[idx];
  }
  // phase 1a: errors (wrap_error, utils.py:131-137) and control deviations
  if (row_ok) {
    if (i < n) {
      T x0 = t.X[(b * (NA + 1) + k) * n + i] - xg[i];
      T x1 = t.X[(b * (NA + 1) + k + 1) * n + i] - xg[i];
      if ((t.wrap_mask >> i) & 1u) {
        x0 = wrap_angle(x0);
        x1 = wrap_angle(x1);
      }
      e0[kk * n + i] = x0;
      e1[kk * n + i] = x1;
    }
  }
  __syncthreads();
  // phase 1b: Q e_k (augmented.py:35-36), P e_{k+1} (:78), a~ = a_k - B_k du_k (:50)
  if (row_ok && i < n) {
    T v = T(0), p = T(0), bd = T(0);
    for (int j = 0; j < n; ++j) {
      v += sQ[i * n + j] * e0[kk * n + j];
      p += sP[i * n + j] * e1[kk * n + j];
    }
    const T* Bk = t.Bm + ((b * NA + k) * n + i) * m;
    const T* Uk = t.U + (b * NA + k) * m;
    for (int q = 0; q < m; ++q) bd += Bk[q] * (Uk[q] - ur[q]);  // B_k du_k
    qe[kk * n + i] = v;
    pe[kk * n + i] = p;
    at[kk * n + i] = t.ares[(b * NA + k) * n + i] - bd;
  }
  __syncthreads();
  // e^T Q e (:37) and e^T P e (:79; 2 * (1/2 e^T P e) is exact)
  if (row_ok && i == 0) {
    T v = T(0), p = T(0);
    for (int j = 0; j < n; ++j) {
      v += e0[kk * n + j] * qe[kk * n + j];
      p += e1[kk * n + j] * pe[kk * n + j];
    }
    T corner = v + T(2) * wt + t.rho_reg;
    if (t.c_extra) corner += T(2) * t.c_extra[b * NA + k];
    eqe[kk] = corner;
    epe[kk] = p + t.rho_reg;
  }
  __syncthreads();

  // phase 2: contiguous runs of the blocks of steps k0 .. k0+ks-1.  UNR
  // elements per thread per pass, loads at clamped indices first (independent,
  // in flight together), then the stores.
  constexpr int UNR = 4;
  const long long ss = (long long)s * s, base = (b * a.nbuild + k0);
  T* Qo = a.Q_aug + base * ss;
  T* To = a.QT_aug + base * ss;
  T* Ao = a.A_aug + base * ss;
  T* Bo = a.B_aug + base * s * m;
  const T* cx = t.qx_extra ? t.qx_extra + (b * NA + k0) * n : nullptr;
  const T* Ab = t.A + (b * NA + k0) * (long long)n * n;
  const int tot = ks * s * s;
  for (int p0 = tid; p0 < tot; p0 += UNR * TPB) {
    T ra[UNR];
    int q[UNR], ii[UNR], jj[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int idx = min(p0 + u * TPB, tot - 1);
      q[u] = idx / (s * s);
      const int r = idx - q[u] * s * s;
      ii[u] = r / s;
      jj[u] = r - ii[u] * s;
      const int ia = min(ii[u], n - 1), ja = min(jj[u], n - 1);
      ra[u] = Ab[(q[u] * n + ia) * n + ja];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int idx = p0 + u * TPB;
      if (idx >= tot) break;
      const int qq = q[u], i2 = ii[u], j2 = jj[u];
      T vq, vt, va;
      if (i2 < n && j2 < n) {
        // _sym(Q) + q_reg I (+ _sym(cxx)); the final _sym of the block is exact
        vq = sQs[i2 * n + j2];
        if (t.qxx_extra) {
          const T* X = t.qxx_extra + (b * NA + k0 + qq) * n * n;
          vq += T(0.5) * (X[i2 * n + j2] + X[j2 * n + i2]);
        }
        vt = sP[i2 * n + j2];
        va = ra[u];
      } else if (i2 < n) {  // last column: Q e (+ cx)
        vq = cx ? qe[qq * n + i2] + cx[qq * n + i2] : qe[qq * n + i2];
        vt = pe[qq * n + i2];
        va = at[qq * n + i2];
      } else if (j2 < n) {  // last row
        vq = cx ? qe[qq * n + j2] + cx[qq * n + j2] : qe[qq * n + j2];
        vt = pe[qq * n + j2];
        va = T(0);
      } else {
        vq = eqe[qq];
        vt = epe[qq];
        va = T(1);
      }
      Qo[idx] = vq;
      To[idx] = vt;
      Ao[idx] = va;
    }
  }
  const T* Bb = t.Bm + (b * NA + k0) * (long long)n * m;
  const int totb = ks * s * m;
  for (int idx = tid; idx < totb; idx += TPB) {
    const int qq = idx / (s * m), r = idx - qq * s * m, i2 = r / m, j2 = r - i2 * m;
    Bo[idx] = i2 < n ? Bb[(qq * n + i2) * m + j2] : T(0);
  }
}

}  // namespace aug

template <class T>
hipError_t dispatch_augment(const AugArgs<T>& a, hipStream_t stream) {
  const int ksb = aug::steps_per_block(a.t.n);
  const long long nchunk = (a.nbuild + ksb - 1) / ksb;
  const long long blocks = a.batch * nchunk;
  if (blocks <= 0) return hipSuccess;
  if (blocks > 0x7FFFFFFFll) return hipErrorInvalidValue;
  hipLaunchKernelGGL(aug::augment_kernel<T>, dim3((unsigned)blocks), dim3(aug::TPB), 0, stream,
                     a);
  return hipGetLastError();
}

template hipError_t dispatch_augment<double>(const AugArgs<double>&, hipStream_t);
template hipError_t dispatch_augment<float>(const AugArgs<float>&, hipStream_t);

}  // namespace hop
