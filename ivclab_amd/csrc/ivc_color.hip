// ivc_color.hip — colour conversions of ivclab/signal/color.py on gfx950, bit-exact.
//
// rgb2ycbcr (color.py:15-38) is `image @ M.T + offset` in NumPy: a float64 matmul that NumPy
// hands to OpenBLAS dgemm.  The dgemm micro-kernels accumulate over k with fused
// multiply-adds from a zero accumulator, so each output is
//     fma(b, M[c][2], fma(g, M[c][1], r * M[c][0]))  then  + offset[c]
// (verified bit-for-bit against NumPy 2.2 / OpenBLAS 0.3.29 on u8 and float64 images; the
// golden fixtures pin it).  ycbcr2rgb (color.py:40-63) and rgb2gray (color.py:3-13) are plain
// elementwise NumPy expressions, restated in their evaluation order and dtype (float32 input
// stays float32 in ycbcr2rgb and rgb2gray, as NumPy 2 keeps Python-float scalars weak).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ivc_internal.h"

namespace ivc {

// BT.601 matrix and offsets exactly as written in color.py:27-33 (decimal literals -> f64)
__constant__ double c_ycc[9] = {0.299, 0.587, 0.114, -0.168736, -0.331264, 0.5,
                                0.5, -0.418688, -0.081312};

static unsigned color_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 256 * 16) g = 256 * 16;
  return (unsigned)(g < 1 ? 1 : g);
}

template <typename TI>
__global__ __launch_bounds__(256) void rgb2ycbcr_kernel(const TI* __restrict__ src, int64_t npix,
                                                        double* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += (int64_t)gridDim.x * 256) {
    const double r = (double)src[3 * i], g = (double)src[3 * i + 1], b = (double)src[3 * i + 2];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double acc = __builtin_fma(b, c_ycc[3 * c + 2], __builtin_fma(g, c_ycc[3 * c + 1], r * c_ycc[3 * c]));
      dst[3 * i + c] = acc + (c == 0 ? 0.0 : 128.0);
    }
  }
}

// T: arithmetic type (float for float32 input, double otherwise); Y keeps the input value
template <typename TI, typename T>
__global__ __launch_bounds__(256) void ycbcr2rgb_kernel(const TI* __restrict__ src, int64_t npix,
                                                        int64_t cstride, T* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += (int64_t)gridDim.x * 256) {
    const TI* p = src + cstride * i;
    const T Y = (T)p[0];
    const T Cb = (T)p[1] - (T)128.0, Cr = (T)p[2] - (T)128.0;
    T rgb[3];
    rgb[0] = Y + (T)1.402 * Cr;
    rgb[1] = (Y - (T)0.344136 * Cb) - (T)0.714136 * Cr;
    rgb[2] = Y + (T)1.772 * Cb;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const T v = rgb[c];
      // np.clip(v, 0, 255): NaN stays NaN
      dst[3 * i + c] = v != v ? v : (v < (T)0 ? (T)0 : (v > (T)255 ? (T)255 : v));
    }
  }
}

// np.mean(image, axis=-1, keepdims=True) for C < 8 channels: sequential sum in the
// accumulator type, then true division by C
template <typename TI, typename T>
__global__ __launch_bounds__(256) void rgb2gray_kernel(const TI* __restrict__ src, int64_t npix, int C,
                                                       T* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += (int64_t)gridDim.x * 256) {
    T acc = (T)src[(int64_t)C * i];
    for (int c = 1; c < C; ++c) acc = acc + (T)src[(int64_t)C * i + c];
    dst[i] = acc / (T)C;
  }
}

#define IVC_COLOR_DISPATCH(dtype, MACRO)      \
  switch (dtype) {                            \
    case IVC_U8: MACRO(uint8_t); break;       \
    case IVC_I8: MACRO(int8_t); break;        \
    case IVC_U16: MACRO(uint16_t); break;     \
    case IVC_I16: MACRO(int16_t); break;      \
    case IVC_U32: MACRO(uint32_t); break;     \
    case IVC_I32: MACRO(int32_t); break;      \
    case IVC_U64: MACRO(uint64_t); break;     \
    case IVC_I64: MACRO(int64_t); break;      \
    case IVC_F32: MACRO(float); break;        \
    case IVC_F64: MACRO(double); break;       \
    default: return hipErrorInvalidValue;     \
  }

hipError_t launch_rgb2ycbcr(const void* src, int dtype, int64_t npix, double* dst, hipStream_t s) {
  if (npix <= 0) return hipSuccess;
#define K(T) rgb2ycbcr_kernel<T><<<color_grid(npix), 256, 0, s>>>((const T*)src, npix, dst)
  IVC_COLOR_DISPATCH(dtype, K)
#undef K
  return hipGetLastError();
}

// float32 input -> float32 output; every other dtype -> float64
hipError_t launch_ycbcr2rgb(const void* src, int dtype, int64_t npix, int64_t cstride, void* dst,
                            hipStream_t s) {
  if (npix <= 0) return hipSuccess;
#define K(T)                                                                                   \
  if (dtype == IVC_F32)                                                                        \
    ycbcr2rgb_kernel<T, float><<<color_grid(npix), 256, 0, s>>>((const T*)src, npix, cstride,  \
                                                                (float*)dst);                  \
  else                                                                                         \
    ycbcr2rgb_kernel<T, double><<<color_grid(npix), 256, 0, s>>>((const T*)src, npix, cstride, \
                                                                 (double*)dst)
  IVC_COLOR_DISPATCH(dtype, K)
#undef K
  return hipGetLastError();
}

hipError_t launch_rgb2gray(const void* src, int dtype, int64_t npix, int C, void* dst, hipStream_t s) {
  if (npix <= 0) return hipSuccess;
  if (C < 1 || C >= 8) return hipErrorInvalidValue;
#define K(T)                                                                                     \
  if (dtype == IVC_F32)                                                                          \
    rgb2gray_kernel<T, float><<<color_grid(npix), 256, 0, s>>>((const T*)src, npix, C, (float*)dst); \
  else                                                                                           \
    rgb2gray_kernel<T, double><<<color_grid(npix), 256, 0, s>>>((const T*)src, npix, C, (double*)dst)
  IVC_COLOR_DISPATCH(dtype, K)
#undef K
  return hipGetLastError();
}

}  // namespace ivc
