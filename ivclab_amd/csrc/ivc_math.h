// ivc_math.h — exact 8-point DCT-II / DCT-III arithmetic shared by the HIP kernels and the
// host-side unit test harness (tests/cpu_math_harness.cpp).
//
// The reference computes its 8x8 DCT with scipy.fft.dct/idct(norm='ortho') along axis -1
// then axis -2 (ivclab/signal/dct.py:24,26 and :42,44).  scipy dispatches to pocketfft,
// whose N = 8 DCT-II is: pre-butterfly, real FFT factored [2,4] (radb2 ido=4, radb4 ido=1),
// scale by fct, post-twiddle; DCT-III is the mirror.  The sequences below reproduce that
// op order exactly (SURVEY.md §8a "a2/a3 spec"), so every intermediate is rounded as in
// pocketfft.  Build with -ffp-contract=off: one fused multiply-add changes low bits and
// therefore flips round-half-even quantisation ties.
//
// Two forms are provided:
//   dct2_line / dct3_line  — the literal sequence, any float type, any norm.
//   dct2_row_int / dct2_col_unscaled — the DCT-II with every exact power-of-two scaling
//     (x2 pre-butterfly, fct = 1/4, the 1/2 post-twiddle) factored out.  For finite inputs
//     with no subnormal intermediates, fl(2^k * a) = 2^k * a and fl(2^k * a op 2^k * b) =
//     2^k * fl(a op b), so out = s * unscaled exactly, with s in {1/2, 1/4} per output
//     index.  The integer form also runs the exact add/sub prefix in int32.  Integer
//     inputs (u8/i8/u16/i16 pixels, integer residuals) never produce subnormals, so the
//     fused intra/inter kernels use this form and fold s into the reciprocal table.
#pragma once
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#if defined(__HIPCC__)
#define IVC_HD __host__ __device__ __forceinline__
#else
#define IVC_HD static inline
#endif

#include <stdint.h>

namespace ivc {

// pocketfft constants for N = 8 (radix-2 twiddle W0 is sin(8*ang), one ulp below sqrt(1/2))
template <typename T> struct PF;
template <> struct PF<double> {
  static constexpr double W0 = 0x1.6a09e667f3bccp-1;
  static constexpr double W1 = 0x1.6a09e667f3bcdp-1;
  static constexpr double TW0 = 0x1.f6297cff75cb0p-1, TW1 = 0x1.d906bcf328d46p-1,
                          TW2 = 0x1.a9b66290ea1a3p-1, TW3 = 0x1.6a09e667f3bccp-1,
                          TW4 = 0x1.1c73b39ae68c8p-1, TW5 = 0x1.87de2a6aea963p-2,
                          TW6 = 0x1.8f8b83c69a60ap-3;
  static constexpr double SQRT2 = 0x1.6a09e667f3bcdp+0;
  static constexpr double S2H = 0x1.6a09e667f3bcdp-1;  // SQRT2 * 0.5
};
template <> struct PF<float> {
  static constexpr float W0 = (float)0x1.6a09e667f3bccp-1;
  static constexpr float W1 = (float)0x1.6a09e667f3bcdp-1;
  static constexpr float TW0 = (float)0x1.f6297cff75cb0p-1, TW1 = (float)0x1.d906bcf328d46p-1,
                         TW2 = (float)0x1.a9b66290ea1a3p-1, TW3 = (float)0x1.6a09e667f3bccp-1,
                         TW4 = (float)0x1.1c73b39ae68c8p-1, TW5 = (float)0x1.87de2a6aea963p-2,
                         TW6 = (float)0x1.8f8b83c69a60ap-3;
  static constexpr float SQRT2 = (float)0x1.6a09e667f3bcdp+0;
  static constexpr float S2H = (float)0x1.6a09e667f3bcdp+0 * 0.5f;
};

// post-twiddle pair used by both forms: (a = e[k], b = e[kc]) with twiddles (tk, tkc)
template <typename T>
IVC_HD void pf_post(T& ek, T& ekc, T tk, T tkc) {
  T t1 = tk * ekc + tkc * ek;
  T t2 = tk * ek - tkc * ekc;
  ek = t1 + t2;
  ekc = t1 - t2;
}

// ---- literal DCT-II (pocketfft T_dcst23 type 2, N = 8), in place on c[0..7] ----------
template <typename T>
IVC_HD void dct2_line(T* c, T fct, bool ortho) {
  typedef PF<T> K;
  c[0] = c[0] * T(2);
  c[7] = c[7] * T(2);
  {
    T a = c[2], b = c[1]; c[2] = a - b; c[1] = b + a;
    a = c[4]; b = c[3]; c[4] = a - b; c[3] = b + a;
    a = c[6]; b = c[5]; c[6] = a - b; c[5] = b + a;
  }
  // radb2, ido = 4
  T d0 = c[0] + c[7], d4 = c[0] - c[7];
  T d3 = T(2) * c[3], d7 = T(-2) * c[4];
  T d1 = c[1] + c[5], tr2 = c[1] - c[5];
  T ti2 = c[2] + c[6], d2 = c[2] - c[6];
  T d6 = K::W0 * ti2 + K::W1 * tr2;
  T d5 = K::W0 * tr2 - K::W1 * ti2;
  // radb4, ido = 1, l1 = 2
  T e[8];
  {
    T r2 = d0 + d3, r1 = d0 - d3, r3 = T(2) * d1, r4 = T(2) * d2;
    e[0] = r2 + r3; e[4] = r2 - r3; e[6] = r1 + r4; e[2] = r1 - r4;
  }
  {
    T r2 = d4 + d7, r1 = d4 - d7, r3 = T(2) * d5, r4 = T(2) * d6;
    e[1] = r2 + r3; e[5] = r2 - r3; e[7] = r1 + r4; e[3] = r1 - r4;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = e[i] * fct;
  // post-twiddle k = 1,2,3 (kc = 7,6,5): c[k] = 0.5*(t1+t2), c[kc] = 0.5*(t1-t2)
  pf_post<T>(e[1], e[7], K::TW0, K::TW6);
  pf_post<T>(e[2], e[6], K::TW1, K::TW5);
  pf_post<T>(e[3], e[5], K::TW2, K::TW4);
  e[1] = T(0.5) * e[1]; e[7] = T(0.5) * e[7];
  e[2] = T(0.5) * e[2]; e[6] = T(0.5) * e[6];
  e[3] = T(0.5) * e[3]; e[5] = T(0.5) * e[5];
  e[4] = e[4] * K::TW3;
  if (ortho) e[0] = e[0] * K::S2H;
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = e[i];
}

// ---- literal DCT-III (pocketfft T_dcst23 type 3, N = 8), in place -------------------
template <typename T>
IVC_HD void dct3_line(T* c, T fct, bool ortho) {
  typedef PF<T> K;
  if (ortho) c[0] = c[0] * K::SQRT2;
  {
    T t1 = c[1] + c[7], t2 = c[1] - c[7];
    c[1] = K::TW0 * t2 + K::TW6 * t1; c[7] = K::TW0 * t1 - K::TW6 * t2;
    t1 = c[2] + c[6]; t2 = c[2] - c[6];
    c[2] = K::TW1 * t2 + K::TW5 * t1; c[6] = K::TW1 * t1 - K::TW5 * t2;
    t1 = c[3] + c[5]; t2 = c[3] - c[5];
    c[3] = K::TW2 * t2 + K::TW4 * t1; c[5] = K::TW2 * t1 - K::TW4 * t2;
  }
  c[4] = c[4] * (T(2) * K::TW3);
  // radf4, ido = 1, l1 = 2
  T d[8];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    T tr1 = c[k + 6] + c[k + 2];
    d[2 + 4 * k] = c[k + 6] - c[k + 2];
    T tr2 = c[k] + c[k + 4];
    d[1 + 4 * k] = c[k] - c[k + 4];
    d[4 * k] = tr2 + tr1;
    d[3 + 4 * k] = tr2 - tr1;
  }
  // radf2, ido = 4
  T e[8];
  e[0] = d[0] + d[4];
  e[7] = d[0] - d[4];
  e[4] = -d[7];
  e[3] = d[3];
  T tr2 = K::W0 * d[5] + K::W1 * d[6];
  T ti2 = K::W0 * d[6] - K::W1 * d[5];
  e[1] = d[1] + tr2;
  e[5] = d[1] - tr2;
  e[2] = ti2 + d[2];
  e[6] = ti2 - d[2];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = e[i] * fct;
  {
    T a = e[1], b = e[2]; e[1] = a - b; e[2] = b + a;
    a = e[3]; b = e[4]; e[3] = a - b; e[4] = b + a;
    a = e[5]; b = e[6]; e[5] = a - b; e[6] = b + a;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = e[i];
}

// ---- factored DCT-II (ortho): power-of-two scale per output index ---------------------
// scale of output index k: 1/2 for k in {0, 4}, 1/4 otherwise
IVC_HD double dct2_scale(int k) { return (k & 3) == 0 ? 0.5 : 0.25; }

// common post stage of the factored form: E[0..7] (unscaled radb4 outputs) -> out
IVC_HD void dct2_post_unscaled(double* E, double* out) {
  typedef PF<double> K;
  double e1 = E[1], e7 = E[7], e2 = E[2], e6 = E[6], e3 = E[3], e5 = E[5];
  pf_post<double>(e1, e7, K::TW0, K::TW6);
  pf_post<double>(e2, e6, K::TW1, K::TW5);
  pf_post<double>(e3, e5, K::TW2, K::TW4);
  out[0] = E[0] * K::S2H;
  out[4] = E[4] * K::TW3;
  out[1] = e1; out[7] = e7; out[2] = e2; out[6] = e6; out[3] = e3; out[5] = e5;
}

// Row pass on integer pixels x[0..7] (|x| < 2^16).  out[k] * dct2_scale(k) equals
// dct2_line<double>(x, 0.25, true)[k] bit for bit.
IVC_HD void dct2_row_int(const int* x, double* out) {
  typedef PF<double> K;
  // pre-butterfly (exact in int32)
  int c1 = x[1] + x[2], c2 = x[2] - x[1];
  int c3 = x[3] + x[4], c4 = x[4] - x[3];
  int c5 = x[5] + x[6], c6 = x[6] - x[5];
  // radb2 with the uniform factor 2 removed: D0=(x0+x7), D4=(x0-x7), D3=c3, D7=-c4
  int D0 = x[0] + x[7], D4 = x[0] - x[7];
  int d1 = c1 + c5, tr2 = c1 - c5, ti2 = c2 + c6, d2 = c2 - c6;
  double fti2 = (double)ti2, ftr2 = (double)tr2;
  double d6 = K::W0 * fti2 + K::W1 * ftr2;
  double d5 = K::W0 * ftr2 - K::W1 * fti2;
  double E[8];
  int r2 = D0 + c3, r1 = D0 - c3;
  E[0] = (double)(r2 + d1);
  E[4] = (double)(r2 - d1);
  E[6] = (double)(r1 + d2);
  E[2] = (double)(r1 - d2);
  double q2 = (double)(D4 - c4), q1 = (double)(D4 + c4);
  E[1] = q2 + d5;
  E[5] = q2 - d5;
  E[7] = q1 + d6;
  E[3] = q1 - d6;
  dct2_post_unscaled(E, out);
}

// Column pass on one column whose 8 entries share one power-of-two scale (the output of
// dct2_row_int).  out[i] * dct2_scale(i) * (input scale) equals the literal sequence.
IVC_HD void dct2_col_unscaled(const double* x, double* out) {
  typedef PF<double> K;
  double c1 = x[1] + x[2], c2 = x[2] - x[1];
  double c3 = x[3] + x[4], c4 = x[4] - x[3];
  double c5 = x[5] + x[6], c6 = x[6] - x[5];
  double D0 = x[0] + x[7], D4 = x[0] - x[7];
  double d1 = c1 + c5, tr2 = c1 - c5, ti2 = c2 + c6, d2 = c2 - c6;
  double d6 = K::W0 * ti2 + K::W1 * tr2;
  double d5 = K::W0 * tr2 - K::W1 * ti2;
  double E[8];
  double r2 = D0 + c3, r1 = D0 - c3;
  E[0] = r2 + d1;
  E[4] = r2 - d1;
  E[6] = r1 + d2;
  E[2] = r1 - d2;
  double q2 = D4 - c4, q1 = D4 + c4;
  E[1] = q2 + d5;
  E[5] = q2 - d5;
  E[7] = q1 + d6;
  E[3] = q1 - d6;
  dct2_post_unscaled(E, out);
}

// NumPy float -> int32 cast as x86 performs it (cvttsd2si): truncation toward zero,
// INT32_MIN for NaN and out-of-range values (patchquant.py:60,78 `.astype(np.int32)`).
template <typename T>
IVC_HD int32_t np_to_i32(T v) {
  return (v >= T(-2147483648.0) && v < T(2147483648.0)) ? (int32_t)v : (int32_t)(-2147483647 - 1);
}

// zig-zag position of each raster index (ivclab/utils/shape.py:10-19 ZigZag.zigzag_order)
#define IVC_ZZ_ORDER                                                                     \
  {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42, 3,  8,  12, 17, 25, 30, \
   41, 43, 9,  11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, \
   46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63}
// raster index at each zig-zag position (inverse permutation; = ivclab/signal/zigzag.py:15-24)
#define IVC_ZZ_SCAN                                                                      \
  {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, \
   41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, \
   30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63}

}  // namespace ivc
