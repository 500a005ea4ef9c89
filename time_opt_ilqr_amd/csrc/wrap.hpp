// wrap_error on one component (utils.py:127-137):
//   angle_normalize(a) = (a + pi) % (2 pi) - pi   with Python float-% semantics
// Shared by the kernels and the host test build (small_host.cpp).
//
// fmod without the library's iterative routine: n = trunc(x / y) from a
// reciprocal is exact or off by one; fma(-n, y, x) is then exact for the right
// n because fmod's result x - n y is representable, so a wrong n is detected by
// the range of r and r is recomputed with n -/+ 1 (never corrected by adding y,
// which could round).  Valid for |x / 2pi| < 2^52 (any realistic angle).
#pragma once

#ifndef HOP_HD
#define HOP_HD __host__ __device__
#endif

namespace hop {

HOP_HD inline double wrap_trunc(double v) { return __builtin_trunc(v); }
HOP_HD inline float wrap_trunc(float v) { return __builtin_truncf(v); }
HOP_HD inline double wrap_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
HOP_HD inline float wrap_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

template <class T>
HOP_HD inline T wrap_angle(T a) {
  const T pi = T(3.141592653589793);
  const T y = T(2.0 * 3.141592653589793);
  const T inv = T(1.0 / (2.0 * 3.141592653589793));
  const T x = a + pi;
  T n = wrap_trunc(x * inv);
  T r = wrap_fma(-n, y, x);
  // fmod range: sign of x, |r| < y; a wrong n is off by one (branch-free fix)
  const bool lo = x >= T(0) ? r < T(0) : r <= -y;
  const bool hi = x >= T(0) ? r >= y : r > T(0);
  n = lo ? n - T(1) : (hi ? n + T(1) : n);
  r = wrap_fma(-n, y, x);
  // Python: a non-zero remainder takes the divisor's sign; a zero one is +0
  const T rp = r < T(0) ? r + y : r;
  r = r != T(0) ? rp : T(0);
  return r - pi;
}

}  // namespace hop
