// Batched LFT horizon sweep (the hot path): J(t) for every horizon t = 1..N of
// every problem, one forward pass that fuses, per step k,
//   stage   E_k = (Q_k+eps)^-1, F_k = E_k A_k^T, G_k = A_k E_k A_k^T + B_k R^-1 B_k^T
//   compose W = (E_k + Gbar)^-1, Ebar -= Fbar W Fbar^T, Fbar = Fbar W F_k,
//           Gbar = G_k - F_k^T W F_k
//   query   J_{k+1} = 1/2 z0^T (Ebar - Fbar (QT_k^-1 + Gbar)^-1 Fbar^T)^-1 z0
// Reference: horizon_selection.py:36-86 (propagator_all_Jt_aug); the argmin of
// solver.py:522 is fused as an option.  Fbar is carried transposed (H = Fbar^T)
// so that every product is an X*Y or X^T*Y broadcast chain (hop_device.hpp).
// Symmetrisation is applied to every inverse input (chol_inv's _sym,
// utils.py:74); sym is linear, so the reference's intermediate _sym calls on
// G, Ebar, Gbar are subsumed.
#include "hop_device.hpp"
#include "hop_kernels.hpp"

namespace hop {

template <class T, int S>
__device__ __forceinline__ void load_col(const T* M, int s, int c, T pad, T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const bool in = (i < s) && (c < s);
    const T v = M[in ? i * s + c : 0];
    x[i] = in ? v : ((i == c) ? pad : T(0));
  }
}
// row c of an s x s matrix = column c of its transpose
template <class T, int S>
__device__ __forceinline__ void load_row(const T* M, int s, int c, T (&x)[S]) {
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const bool in = (j < s) && (c < s);
    const T v = M[in ? c * s + j : 0];
    x[j] = in ? v : T(0);
  }
}
// row c of an s x m matrix (zero padded)
template <class T, int MM>
__device__ __forceinline__ void load_brow(const T* Bm, int s, int m, int c, T (&x)[MM]) {
#pragma unroll
  for (int j = 0; j < MM; ++j) {
    const bool in = (j < m) && (c < s);
    const T v = Bm[in ? c * m + j : 0];
    x[j] = in ? v : T(0);
  }
}
template <class T, int S>
__device__ __forceinline__ void store_col(T* M, int s, int c, const T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i < s && c < s) M[i * s + c] = x[i];
}
template <class T, int S>
__device__ __forceinline__ void store_col_t(T* M, int s, int c, const T (&x)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i)
    if (i < s && c < s) M[c * s + i] = x[i];
}

template <class T, int S, int MM>
__global__ __launch_bounds__(256, 1) void lft_sweep_kernel(LftArgs<T> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* smem = reinterpret_cast<T*>(smem_raw);
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4, w = tid >> 6;
  const long long prob = ((long long)blockIdx.x * kWavesPerBlock + w) * kProbPerWave + g;
  bool valid = prob < a.batch;
  const long long pb = valid ? prob : a.batch - 1;
  if (a.cond & 1) {  // rerun launch after the conditioned-prefix kernel (fp32 blocks)
    const bool need = valid && (a.status[prob] & (int)ST_RERUN);
    if (!__any(need)) return;  // wave-uniform; no workgroup barrier in this kernel
    valid = need;
  }
  T* tile = smem + (w * kProbPerWave + g) * kLdsTile;
#pragma unroll 1
  for (int i = c; i < kLdsTile; i += kRowLanes) tile[i] = T(0);
  wave_sync();

  const int s = a.s, m = a.m, N = a.n, mt = a.max_tries;
  const long long ss = (long long)s * s, sm = (long long)s * m;
  const T* Ap = a.A + pb * a.nalloc * ss;
  const T* Bp = a.B + pb * a.nalloc * sm;
  const T* Qp = a.Q + pb * a.nalloc * ss;
  const T* QTp = a.QT + pb * a.nalloc * ss;
  const T* Rp = a.R + pb * a.r_bstride;
  const T* zp = a.z0 + pb * a.z_bstride;

  const T zc = (c < s) ? zp[c < s ? c : 0] : T(0);

  unsigned st = 0;
  T rinv[MM];
  const bool r_fixed = (a.r_kstride == 0);
  if (r_fixed) {
    T rr[MM];
    load_col<T, MM>(Rp, m, c, T(1), rr);
    if (!a.r_is_inv) sym_spd_inverse(rr, tile, c, mt, st);
    copy(rinv, rr);
  }

  T Eb[S], H[S], Gb[S];
  T best = T(0);
  int tbest = 0;
  const bool fuse_argmin = a.t_max > 0;

#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    const T* Ak = Ap + k * ss;
    const T* Qk = Qp + k * ss;
    const T* QTk = QTp + k * ss;
    const T* Bk = Bp + k * sm;
    T E[S], at[S], brow[MM];
    load_col(Qk, s, c, T(1), E);
    load_row(Ak, s, c, at);
    load_brow<T, MM>(Bk, s, m, c, brow);
    if (!r_fixed) {
      T rr[MM];
      load_col<T, MM>(Rp + k * a.r_kstride, m, c, T(1), rr);
      if (!a.r_is_inv) sym_spd_inverse(rr, tile, c, mt, st);
      copy(rinv, rr);
    }

    // ---- stage: E, F = E A^T, G = A F + B R^-1 B^T
    sym_spd_inverse(E, tile, c, mt, st);
    T F[S];
    zero(F);
    acc_xy<false>(F, E, at);
    T G[S];
    zero(G);
    acc_xty<false>(G, at, F);
    T y[MM];
    zero(y);
    acc_xy<false, T, MM, MM>(y, rinv, brow);  // y = R^-1 B[c][:]^T
    acc_xty<false, T, S, MM>(G, brow, y);     // G += B R^-1 B^T

    if (a.dbg_efg != nullptr && valid) {
      T* o = a.dbg_efg + ((prob * N + k) * 3) * ss;
      store_col(o, s, c, E);
      store_col(o + ss, s, c, F);
      store_col(o + 2 * ss, s, c, G);
    }

    // ---- compose the prefix (Ebar, H = Fbar^T, Gbar)
    if (k == 0) {
      copy(Eb, E);
      transpose(H, F, tile, c);
      copy(Gb, G);
    } else {
      T W[S];
#pragma unroll
      for (int i = 0; i < S; ++i) W[i] = E[i] + Gb[i];
      sym_spd_inverse(W, tile, c, mt, st);   // W = (E_k + Gbar)^-1
      T Z[S];
      zero(Z);
      acc_xy<false>(Z, W, H);    // Z = W Fbar^T
      acc_xty<true>(Eb, H, Z);   // Ebar -= Fbar W Fbar^T
      zero(H);
      acc_xty<false>(H, F, Z);   // H' = (Fbar W F)^T = F^T W Fbar^T
      zero(Z);
      acc_xy<false>(Z, W, F);    // W F
      copy(Gb, G);
      acc_xty<true>(Gb, F, Z);   // Gbar = G - F^T W F
    }
    if (a.dbg_pre != nullptr && valid) {
      T* o = a.dbg_pre + ((prob * N + k) * 3) * ss;
      store_col(o, s, c, Eb);
      store_col_t(o + ss, s, c, H);
      store_col(o + 2 * ss, s, c, Gb);
    }

    // ---- query horizon t = k + 1
    T Xt[S];
    load_col(QTk, s, c, T(1), Xt);
    sym_spd_inverse(Xt, tile, c, mt, st);     // QT_k^-1
#pragma unroll
    for (int i = 0; i < S; ++i) Xt[i] += Gb[i];
    sym_spd_inverse(Xt, tile, c, mt, st);     // Wt = (QT^-1 + Gbar)^-1
    T V[S];
    zero(V);
    acc_xy<false>(V, Xt, H);     // Wt Fbar^T
    copy(Xt, Eb);
    acc_xty<true>(Xt, H, V);     // X0 = Ebar - Fbar Wt Fbar^T
    sym_spd_inverse(Xt, tile, c, mt, st);     // P0 = X0^-1
    T u = T(0);
    LaneDot<S>::fma(u, zc, Xt);  // (z0^T P0)[c]
    const T jk = T(0.5) * row_sum((c < s) ? u * zc : T(0));
    if (!finite_val(jk)) st |= ST_NONFINITE;
    if (valid && c == 0) a.J[prob * N + k] = jk;
    if (fuse_argmin) {
      const int t = k + 1;
      if (t == a.t_min) {
        best = jk;
        tbest = t;
      } else if (t > a.t_min && t <= a.t_max) {
        const bool bnan = best != best, jnan = jk != jk;
        if (!bnan && (jnan || jk < best)) {
          best = jk;
          tbest = t;
        }
      }
    }
  }
  if (valid && c == 0) {
    a.status[prob] = (int)st;
    if (fuse_argmin && a.t_star != nullptr) {
      a.t_star[prob] = tbest;
      a.j_star[prob] = best;
    }
  }
}

template <class T, int S, int MM>
hipError_t launch_lft(const LftArgs<T>& a, hipStream_t stream) {
  const long long blocks = (a.batch + kProbPerBlock - 1) / kProbPerBlock;
  const size_t lds = (size_t)kProbPerBlock * kLdsTile * sizeof(T);
  hipLaunchKernelGGL((lft_sweep_kernel<T, S, MM>), dim3((unsigned)blocks), dim3(256), lds, stream, a);
  return hipGetLastError();
}

template <class T>
hipError_t dispatch_lft(const LftArgs<T>& a, hipStream_t stream) {
  const int s = a.s, m = a.m;
  if (m <= 4) {
    if (s <= 4) return launch_lft<T, 4, 4>(a, stream);
    if (s <= 8) return launch_lft<T, 8, 4>(a, stream);
    if (s == 13) return launch_lft<T, 13, 4>(a, stream);
    return launch_lft<T, 16, 4>(a, stream);
  }
  return launch_lft<T, 16, 16>(a, stream);
}

template hipError_t dispatch_lft<double>(const LftArgs<double>&, hipStream_t);
template hipError_t dispatch_lft<float>(const LftArgs<float>&, hipStream_t);

}  // namespace hop
