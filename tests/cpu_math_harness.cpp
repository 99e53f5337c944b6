// Host build of the kernels' DCT arithmetic (ivclab_amd/csrc/ivc_math.h) for CPU unit tests:
// compiled by tests/test_cpu_math.py with g++ -O2 -ffp-contract=off and compared against the
// oracle (scipy/pocketfft via the reference-semantics restatement).  Test code only.
#include "../ivclab_amd/csrc/ivc_math.h"
#include <stdint.h>
using namespace ivc;

template <typename T>
static void block_2d(const T* in, T* out, int inverse, T fct, bool ortho) {
  T b[64];
  for (int i = 0; i < 64; ++i) b[i] = in[i];
  for (int r = 0; r < 8; ++r) {  // axis -1
    if (inverse) dct3_line<T>(b + 8 * r, fct, ortho); else dct2_line<T>(b + 8 * r, fct, ortho);
  }
  for (int k = 0; k < 8; ++k) {  // axis -2
    T col[8];
    for (int i = 0; i < 8; ++i) col[i] = b[8 * i + k];
    if (inverse) dct3_line<T>(col, fct, ortho); else dct2_line<T>(col, fct, ortho);
    for (int i = 0; i < 8; ++i) b[8 * i + k] = col[i];
  }
  for (int i = 0; i < 64; ++i) out[i] = b[i];
}

extern "C" {
void h_dct_f64(const double* in, double* out, long n, int inverse, double fct, int ortho) {
  for (long j = 0; j < n; ++j) block_2d<double>(in + 64 * j, out + 64 * j, inverse, fct, ortho != 0);
}
void h_dct_f32(const float* in, float* out, long n, int inverse, float fct, int ortho) {
  for (long j = 0; j < n; ++j) block_2d<float>(in + 64 * j, out + 64 * j, inverse, fct, ortho != 0);
}
// factored DCT-II on integer pixels: returns the fully scaled result
void h_dct2_int_factored(const int32_t* in, double* out, long n) {
  for (long j = 0; j < n; ++j) {
    double R[64];
    for (int r = 0; r < 8; ++r) dct2_row_int(in + 64 * j + 8 * r, R + 8 * r);
    for (int k = 0; k < 8; ++k) {
      double col[8], y[8];
      for (int i = 0; i < 8; ++i) col[i] = R[8 * i + k];
      dct2_col_unscaled(col, y);
      for (int i = 0; i < 8; ++i) out[64 * j + 8 * i + k] = y[i] * (dct2_scale(i) * dct2_scale(k));
    }
  }
}
}
