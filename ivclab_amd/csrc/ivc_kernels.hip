// ivc_kernels.hip — gfx950 kernels for the 8x8 block transform / quantisation path.
//
// Reference methods replaced (paths under /root/reference):
//   DiscreteCosineTransform.transform / inverse_transform   ivclab/signal/dct.py:12-46
//   PatchQuant.quantize / dequantize                        ivclab/quantization/patchquant.py:44-78
//   ZigZag.flatten / unflatten, zigzag_scan                 ivclab/utils/shape.py:21-36, signal/zigzag.py:3-26
//   Patcher.patch (fused as addressing)                     ivclab/utils/shape.py:45-54
//   residual glue of VideoCodec.encode_decode               ivclab/video/videocodec.py:68-71
//
// Work decomposition (all transform kernels): a 256-thread workgroup owns 32 8x8 units;
// thread (u = tid/8, r = tid%8) owns row r of unit u.  Row pass in registers -> transpose
// through LDS -> column pass (thread now owns column r) -> results staged in LDS -> the
// workgroup writes its contiguous output span with 16-byte stores.  HBM traffic per unit
// is one read of the input and one write of the output.
#include "ivc_internal.h"
#include "ivc_math.h"

namespace ivc {

__constant__ int c_zz_order[64] = IVC_ZZ_ORDER;
__constant__ int c_zz_scan[64] = IVC_ZZ_SCAN;

static int g_num_cus = 0;
static int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0)
      g_num_cus = p.multiProcessorCount;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}

static unsigned grid_for(int64_t work_items, int per_block, int max_per_cu) {
  int64_t g = (work_items + per_block - 1) / per_block;
  int64_t cap = (int64_t)num_cus() * max_per_cu;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

int dtype_size(int dt) {
  switch (dt) {
    case IVC_U8: case IVC_I8: return 1;
    case IVC_U16: case IVC_I16: return 2;
    case IVC_U32: case IVC_I32: case IVC_F32: return 4;
    case IVC_U64: case IVC_I64: case IVC_F64: return 8;
    default: return 0;
  }
}
bool dtype_is_float(int dt) { return dt == IVC_F32 || dt == IVC_F64; }

template <typename T> __device__ __forceinline__ T rint_t(T v);
template <> __device__ __forceinline__ float rint_t<float>(float v) { return __builtin_rintf(v); }
template <> __device__ __forceinline__ double rint_t<double>(double v) { return __builtin_rint(v); }

// 8 consecutive elements at an address aligned to their total size (>= 8 bytes)
template <typename TI>
__device__ __forceinline__ void load8(const TI* __restrict__ p, TI* v) {
  constexpr int B = 8 * (int)sizeof(TI);
  if constexpr (B == 8) {
    *reinterpret_cast<uint2*>(v) = *reinterpret_cast<const uint2*>(p);
  } else {
#pragma unroll
    for (int j = 0; j < B / 16; ++j)
      reinterpret_cast<uint4*>(v)[j] = reinterpret_cast<const uint4*>(p)[j];
  }
}

#define IVC_CASE(code, TYPE, ...) \
  case code: {                    \
    typedef TYPE TI;              \
    __VA_ARGS__;                  \
  } break;
#define IVC_DISPATCH_ALL(dt, ...)                                                     \
  switch (dt) {                                                                       \
    IVC_CASE(IVC_U8, uint8_t, __VA_ARGS__) IVC_CASE(IVC_I8, int8_t, __VA_ARGS__)      \
    IVC_CASE(IVC_U16, uint16_t, __VA_ARGS__) IVC_CASE(IVC_I16, int16_t, __VA_ARGS__)  \
    IVC_CASE(IVC_U32, uint32_t, __VA_ARGS__) IVC_CASE(IVC_I32, int32_t, __VA_ARGS__)  \
    IVC_CASE(IVC_U64, uint64_t, __VA_ARGS__) IVC_CASE(IVC_I64, int64_t, __VA_ARGS__)  \
    IVC_CASE(IVC_F32, float, __VA_ARGS__) IVC_CASE(IVC_F64, double, __VA_ARGS__)      \
    default: return hipErrorInvalidValue;                                             \
  }

// ======================================================================================
// Standalone 2-D DCT-II / DCT-III of contiguous 8x8 units (dct.py:12-46).  With DEQ the
// unit is one plane of an int32 [blk][3][64] symbol block: (un-zig-zag ->) dequantise
// (patchquant.py:77-78: int32 * table in float64, truncating cast) -> DCT-III.
// ======================================================================================
template <typename TI, typename T, bool INV, bool DEQ>
__global__ __launch_bounds__(256) void dct8x8_kernel(const TI* __restrict__ src, int64_t nunit,
                                                     T* __restrict__ dst, T fct, int ortho,
                                                     int unzz, QTab tab) {
  __shared__ __attribute__((aligned(16))) T xs[32 * 72];
  const int tid = threadIdx.x, u = tid >> 3, r = tid & 7;
  for (int64_t g = blockIdx.x; g * 32 < nunit; g += gridDim.x) {
    const int64_t unit = g * 32 + u;
    T x[8];
    if (unit < nunit) {
      if constexpr (DEQ) {
        const int64_t blk = unit / 3;
        const int p = (int)(unit - blk * 3);
        const int32_t* q = reinterpret_cast<const int32_t*>(src) + blk * 192 + p * 64;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int j = r * 8 + k;
          const int32_t qv = q[unzz ? c_zz_order[j] : j];
          x[k] = (T)np_to_i32<double>((double)qv * tab.q[p * 64 + j]);
        }
      } else {
        alignas(16) TI v[8];
        load8<TI>(src + unit * 64 + r * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = (T)v[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = T(0);
    }
    if constexpr (INV) dct3_line<T>(x, fct, ortho != 0); else dct2_line<T>(x, fct, ortho != 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) xs[u * 72 + r * 9 + k] = x[k];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xs[u * 72 + i * 9 + r];
    __syncthreads();
    if constexpr (INV) dct3_line<T>(x, fct, ortho != 0); else dct2_line<T>(x, fct, ortho != 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) xs[u * 64 + i * 8 + r] = x[i];
    __syncthreads();
    const int64_t left = nunit - g * 32;
    const int nvalid = left < 32 ? (int)left : 32;
    constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-byte chunk
    T* out = dst + g * 32 * 64;
    for (int e = tid * EPC; e < nvalid * 64; e += 256 * EPC)
      *reinterpret_cast<uint4*>(out + e) = *reinterpret_cast<const uint4*>(xs + e);
    __syncthreads();
  }
}

hipError_t launch_dct8x8(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
                         int inverse, int norm, hipStream_t s) {
  if (nblk <= 0) return hipSuccess;
  // scipy: inorm 0 -> fct 1, 1 (ortho) -> 1/sqrt(2N) = 1/4, 2 -> 1/(2N) = 1/16; the inverse
  // transform uses 2 - inorm (scipy/fft/_pocketfft/helper.py _normalization)
  int inorm = inverse ? 2 - norm : norm;
  double fct = inorm == 0 ? 1.0 : (inorm == 1 ? 0.25 : 0.0625);
  int ortho = norm == IVC_NORM_ORTHO;
  unsigned grid = grid_for(nblk, 32, 8);
  QTab none{};
  if (dst_dtype == IVC_F32) {
    if (src_dtype != IVC_F32) return hipErrorInvalidValue;
    if (inverse)
      dct8x8_kernel<float, float, true, false><<<grid, 256, 0, s>>>(
          (const float*)src, nblk, (float*)dst, (float)fct, ortho, 0, none);
    else
      dct8x8_kernel<float, float, false, false><<<grid, 256, 0, s>>>(
          (const float*)src, nblk, (float*)dst, (float)fct, ortho, 0, none);
    return hipGetLastError();
  }
  if (dst_dtype != IVC_F64 || src_dtype == IVC_F32) return hipErrorInvalidValue;
  IVC_DISPATCH_ALL(src_dtype, {
    if (inverse)
      dct8x8_kernel<TI, double, true, false><<<grid, 256, 0, s>>>(
          (const TI*)src, nblk, (double*)dst, fct, ortho, 0, none);
    else
      dct8x8_kernel<TI, double, false, false><<<grid, 256, 0, s>>>(
          (const TI*)src, nblk, (double*)dst, fct, ortho, 0, none);
  });
  return hipGetLastError();
}

hipError_t launch_intra_decode(const int32_t* q, int64_t nblk, const QTab& t, int unzigzag,
                               double* out, hipStream_t s) {
  if (nblk <= 0) return hipSuccess;
  const int64_t nunit = nblk * 3;
  dct8x8_kernel<int32_t, double, true, true><<<grid_for(nunit, 32, 8), 256, 0, s>>>(
      q, nunit, out, 0.25, 1, unzigzag, t);
  return hipGetLastError();
}

// ======================================================================================
// Quantise / dequantise (patchquant.py:44-78).  Element-wise over the [blk][3][64] output,
// 4 outputs (one 16-byte store) per thread; C = 1 inputs broadcast over the 3 planes.
// ======================================================================================
template <typename TI, typename D>
__global__ __launch_bounds__(256) void quantize_kernel(const TI* __restrict__ src, int64_t nblk,
                                                       int C, QTab t, int32_t* __restrict__ dst) {
  const int64_t total = nblk * 48;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * 256) {
    const int64_t blk = g / 48;
    const int o = (int)(g - blk * 48) * 4, p = o >> 6, j = o & 63;
    const TI* sp = src + (blk * C + (C == 1 ? 0 : p)) * 64 + j;
    int v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = np_to_i32<D>(rint_t<D>((D)sp[e] / (D)t.q[p * 64 + j + e]));
    *reinterpret_cast<int4*>(dst + g * 4) = make_int4(v[0], v[1], v[2], v[3]);
  }
}

template <typename TI, typename D>
__global__ __launch_bounds__(256) void dequantize_kernel(const TI* __restrict__ src,
                                                         int64_t nblk, int C, QTab t,
                                                         int32_t* __restrict__ dst) {
  const int64_t total = nblk * 48;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * 256) {
    const int64_t blk = g / 48;
    const int o = (int)(g - blk * 48) * 4, p = o >> 6, j = o & 63;
    const TI* sp = src + (blk * C + (C == 1 ? 0 : p)) * 64 + j;
    int v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = np_to_i32<D>((D)sp[e] * (D)t.q[p * 64 + j + e]);
    *reinterpret_cast<int4*>(dst + g * 4) = make_int4(v[0], v[1], v[2], v[3]);
  }
}

template <bool DEQ>
static hipError_t launch_quant_common(const void* src, int src_dtype, int64_t nblk, int C,
                                      const QTab& t, int calc_dtype, int32_t* dst,
                                      hipStream_t s) {
  if (nblk <= 0) return hipSuccess;
  if (C != 1 && C != 3) return hipErrorInvalidValue;
  unsigned grid = grid_for(nblk * 48, 256, 16);
  if (calc_dtype == IVC_F32) {
    // float32 arithmetic only arises for float32 or <= 16-bit integer inputs
    if (dtype_size(src_dtype) > 2 && src_dtype != IVC_F32) return hipErrorInvalidValue;
    IVC_DISPATCH_ALL(src_dtype, {
      if constexpr (sizeof(TI) <= 2 || std::is_same<TI, float>::value) {
        if (DEQ)
          dequantize_kernel<TI, float><<<grid, 256, 0, s>>>((const TI*)src, nblk, C, t, dst);
        else
          quantize_kernel<TI, float><<<grid, 256, 0, s>>>((const TI*)src, nblk, C, t, dst);
      }
    });
  } else if (calc_dtype == IVC_F64) {
    IVC_DISPATCH_ALL(src_dtype, {
      if (DEQ)
        dequantize_kernel<TI, double><<<grid, 256, 0, s>>>((const TI*)src, nblk, C, t, dst);
      else
        quantize_kernel<TI, double><<<grid, 256, 0, s>>>((const TI*)src, nblk, C, t, dst);
    });
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_quantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                           int calc_dtype, int32_t* dst, hipStream_t s) {
  return launch_quant_common<false>(src, src_dtype, nblk, C, t, calc_dtype, dst, s);
}
hipError_t launch_dequantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                             int calc_dtype, int32_t* dst, hipStream_t s) {
  return launch_quant_common<true>(src, src_dtype, nblk, C, t, calc_dtype, dst, s);
}

// ======================================================================================
// Zig-zag permutation of 64-element rows (shape.py:21-36): flatten dst[j] = src[scan[j]]
// (the inverse of the reference's scatter by zigzag_order), unflatten dst[j] = src[order[j]].
// ======================================================================================
template <typename E>
__global__ __launch_bounds__(256) void zigzag_kernel(const E* __restrict__ src, int64_t nrow,
                                                     int64_t stride, int inverse,
                                                     E* __restrict__ dst) {
  const int64_t total = nrow * 64;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t row = i >> 6;
    const int j = (int)(i & 63);
    dst[i] = src[row * stride + (inverse ? c_zz_order[j] : c_zz_scan[j])];
  }
}

hipError_t launch_zigzag(const void* src, int64_t nrow, int64_t stride, int esize, int inverse,
                         void* dst, hipStream_t s) {
  if (nrow <= 0) return hipSuccess;
  unsigned grid = grid_for(nrow * 64, 256, 16);
  switch (esize) {
    case 1: zigzag_kernel<uint8_t><<<grid, 256, 0, s>>>((const uint8_t*)src, nrow, stride, inverse, (uint8_t*)dst); break;
    case 2: zigzag_kernel<uint16_t><<<grid, 256, 0, s>>>((const uint16_t*)src, nrow, stride, inverse, (uint16_t*)dst); break;
    case 4: zigzag_kernel<uint32_t><<<grid, 256, 0, s>>>((const uint32_t*)src, nrow, stride, inverse, (uint32_t*)dst); break;
    case 8: zigzag_kernel<uint64_t><<<grid, 256, 0, s>>>((const uint64_t*)src, nrow, stride, inverse, (uint64_t*)dst); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ======================================================================================
// Fused intra / inter transform coding:
//   SRC_IMAGE : patch(img[f]) -> DCT-II ortho -> quantise (-> zig-zag)
//   SRC_INTER : residual = frames[f+1] - MC(frames[f], mv[f]) (videocodec.py:68-71) -> same
// FAST (integer pixels, float64 DCT): ivc_math.h factored DCT, integer prefix in int32, the
// per-index power-of-two scales folded into t.rq; quotient = Yu * rq, with the exact
// IEEE division taken only when the product lies within 2^-30 of a rounding boundary
// (proof in DESIGN.md §Quantisation).  Output planes: C = 1 -> (lum, chrom, chrom) from one
// DCT (patchquant.py:59 broadcast), computed once for the identical chroma planes.
// ======================================================================================
enum { SRC_IMAGE = 0, SRC_INTER = 1 };

struct FusedArgs {
  const void* img;       // SRC_IMAGE: [F][H][W][C];  SRC_INTER: u8 frames [F+1][H][W]
  const int64_t* mv;     // SRC_INTER: [F][h][w]
  int32_t* out;          // [F][h][w][3][64]
  int64_t nframes;       // number of output frames F
  int H, W, h, w, tpr;   // tpr = tiles (of 32 blocks) per block row
  int sr;
  int dup12;             // table planes 1 and 2 identical (always true for PatchQuant tables)
};

template <typename TI, typename T, typename D, int C, bool FAST, bool ZZ, int SRC>
__global__ __launch_bounds__(256) void fused_encode_kernel(FusedArgs a, QTab t) {
  constexpr int XS_BYTES = 32 * 72 * (int)sizeof(T);
  constexpr int OS_BYTES = 32 * 192 * 4;
  // C == 1: the output staging aliases the transpose buffer (disjoint in time)
  constexpr int LDS_BYTES = C == 1 ? (XS_BYTES > OS_BYTES ? XS_BYTES : OS_BYTES)
                                   : XS_BYTES + OS_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  __shared__ D sq[192];
  __shared__ double srq[FAST ? 192 : 1];
  T* xs = reinterpret_cast<T*>(lds);
  int32_t* os = reinterpret_cast<int32_t*>(lds + (C == 1 ? 0 : XS_BYTES));

  const int tid = threadIdx.x, u = tid >> 3, r = tid & 7;
  for (int i = tid; i < 192; i += 256) {
    sq[i] = (D)t.q[i];
    if constexpr (FAST) srq[i] = t.rq[i];
  }
  __syncthreads();

  const int64_t tiles_per_frame = (int64_t)a.h * a.tpr;
  const int64_t ntiles = a.nframes * tiles_per_frame;
  const int n = 2 * a.sr + 1;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t f = tile / tiles_per_frame;
    const int rem = (int)(tile - f * tiles_per_frame);
    const int bi = rem / a.tpr;
    const int bj0 = (rem - bi * a.tpr) * 32;
    const int bj = bj0 + u;
    const bool ok = bj < a.w;

    // ---- gather this thread's row of every channel ----------------------------------
    TI v[8 * C];
    if (ok) {
      if constexpr (SRC == SRC_IMAGE) {
        const TI* p = reinterpret_cast<const TI*>(a.img) +
                      (((int64_t)f * a.H + 8 * bi + r) * a.W + 8 * bj) * C;
        if constexpr (C == 1) {
          alignas(16) TI tmp[8];
          load8<TI>(p, tmp);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = tmp[k];
        } else {
#pragma unroll
          for (int k = 0; k < 8 * C; ++k) v[k] = p[k];
        }
      } else {
        // residual of the motion-compensated prediction; prediction is zero where the
        // displaced block leaves the frame (motion.py:89-92)
        const uint8_t* fr = reinterpret_cast<const uint8_t*>(a.img);
        const int64_t HW = (int64_t)a.H * a.W;
        const uint8_t* cur = fr + (f + 1) * HW + (int64_t)(8 * bi + r) * a.W + 8 * bj;
        const int64_t m = a.mv[(f * a.h + bi) * a.w + bj];
        int64_t qd = m / n, rm = m - qd * n;
        if (rm < 0) { rm += n; qd -= 1; }
        const int dy = (int)qd - a.sr, dx = (int)rm - a.sr;
        const int ry = 8 * bi + dy, rx = 8 * bj + dx;
        const bool in = ry >= 0 && ry + 8 <= a.H && rx >= 0 && rx + 8 <= a.W;
        alignas(8) uint8_t cb[8];
        *reinterpret_cast<uint2*>(cb) = *reinterpret_cast<const uint2*>(cur);
        const uint8_t* ref = fr + f * HW + (int64_t)(ry + r) * a.W + rx;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (TI)((int)cb[k] - (in ? (int)ref[k] : 0));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8 * C; ++k) v[k] = TI(0);
    }

#pragma unroll
    for (int c = 0; c < C; ++c) {
      // ---- row pass (axis -1) ----------------------------------------------------------
      T x[8];
      if constexpr (FAST) {
        int xi[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) xi[k] = (int)v[k * C + c];
        dct2_row_int(xi, x);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = (T)v[k * C + c];
        dct2_line<T>(x, T(0.25), true);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) xs[u * 72 + r * 9 + k] = x[k];
      __syncthreads();
      T y[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = xs[u * 72 + i * 9 + r];
      __syncthreads();
      // ---- column pass (axis -2); thread now owns column k = r -------------------------
      if constexpr (FAST) {
        dct2_col_unscaled(y, x);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = y[i];
        dct2_line<T>(x, T(0.25), true);
      }
      // ---- quantise ----------------------------------------------------------------------
      const int np = C == 1 ? (a.dup12 ? 2 : 3) : 1;
      for (int pi = 0; pi < np; ++pi) {
        const int p = C == 1 ? pi : c;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int j = i * 8 + r;
          int q;
          if constexpr (FAST) {
            const double yq = x[i] * srq[p * 64 + j];
            const double rr = __builtin_rint(yq);
            if (__builtin_fabs(yq - rr) < 0.5 - 0x1p-30 && __builtin_fabs(yq) < 0x1p20) {
              q = (int)rr;
            } else {
              const double Y = x[i] * (dct2_scale(i) * dct2_scale(r));
              q = np_to_i32<double>(__builtin_rint(Y / (double)sq[p * 64 + j]));
            }
          } else {
            q = np_to_i32<D>(rint_t<D>((D)x[i] / sq[p * 64 + j]));
          }
          const int pos = ZZ ? c_zz_order[j] : j;
          os[u * 192 + p * 64 + pos] = q;
          if (C == 1 && p == 1 && a.dup12) os[u * 192 + 128 + pos] = q;
        }
      }
    }
    __syncthreads();
    // ---- contiguous store of the tile's nb x 3 x 64 int32 -------------------------------
    const int nb = a.w - bj0 < 32 ? a.w - bj0 : 32;
    int32_t* out = a.out + (((int64_t)f * a.h + bi) * a.w + bj0) * 192;
    for (int e = tid * 4; e < nb * 192; e += 1024)
      *reinterpret_cast<int4*>(out + e) = *reinterpret_cast<const int4*>(os + e);
    __syncthreads();
  }
}

void qtab_prepare_fused(QTab& t) {
  for (int p = 0; p < 3; ++p)
    for (int i = 0; i < 8; ++i)
      for (int k = 0; k < 8; ++k) {
        const int j = p * 64 + i * 8 + k;
        t.rq[j] = (dct2_scale(i) * dct2_scale(k)) * (1.0 / t.q[j]);
      }
}

template <typename TI, typename T, typename D, int C, bool FAST, int SRC>
static void launch_fused_zz(const FusedArgs& a, const QTab& t, int zigzag, unsigned grid,
                            hipStream_t s) {
  if (zigzag)
    fused_encode_kernel<TI, T, D, C, FAST, true, SRC><<<grid, 256, 0, s>>>(a, t);
  else
    fused_encode_kernel<TI, T, D, C, FAST, false, SRC><<<grid, 256, 0, s>>>(a, t);
}

static FusedArgs make_fused_args(const void* img, const int64_t* mv, int32_t* out,
                                 int64_t nframes, int64_t H, int64_t W, int sr,
                                 const QTab& t) {
  FusedArgs a;
  a.img = img; a.mv = mv; a.out = out; a.nframes = nframes;
  a.H = (int)H; a.W = (int)W; a.h = (int)(H / 8); a.w = (int)(W / 8);
  a.tpr = (a.w + 31) / 32;
  a.sr = sr;
  a.dup12 = 1;
  for (int i = 0; i < 64; ++i)
    if (t.q[64 + i] != t.q[128 + i]) a.dup12 = 0;
  return a;
}

hipError_t launch_intra_encode(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                               int C, const QTab& t_in, int calc_dtype, int zigzag, int32_t* out,
                               hipStream_t s) {
  if (nframes <= 0 || H <= 0 || W <= 0) return hipSuccess;
  if (C != 1 && C != 3) return hipErrorInvalidValue;
  QTab t = t_in;
  qtab_prepare_fused(t);
  FusedArgs a = make_fused_args(img, nullptr, out, nframes, H, W, 0, t);
  const int64_t ntiles = nframes * (int64_t)a.h * a.tpr;
  const unsigned grid = grid_for(ntiles, 1, 8);
  switch (dtype) {
    case IVC_U8:
      if (calc_dtype != IVC_F64) return hipErrorInvalidValue;
      if (C == 1) launch_fused_zz<uint8_t, double, double, 1, true, SRC_IMAGE>(a, t, zigzag, grid, s);
      else launch_fused_zz<uint8_t, double, double, 3, true, SRC_IMAGE>(a, t, zigzag, grid, s);
      break;
    case IVC_F64:
      if (calc_dtype != IVC_F64) return hipErrorInvalidValue;
      if (C == 1) launch_fused_zz<double, double, double, 1, false, SRC_IMAGE>(a, t, zigzag, grid, s);
      else launch_fused_zz<double, double, double, 3, false, SRC_IMAGE>(a, t, zigzag, grid, s);
      break;
    case IVC_F32:
      if (calc_dtype == IVC_F32) {
        if (C == 1) launch_fused_zz<float, float, float, 1, false, SRC_IMAGE>(a, t, zigzag, grid, s);
        else launch_fused_zz<float, float, float, 3, false, SRC_IMAGE>(a, t, zigzag, grid, s);
      } else if (calc_dtype == IVC_F64) {
        if (C == 1) launch_fused_zz<float, float, double, 1, false, SRC_IMAGE>(a, t, zigzag, grid, s);
        else launch_fused_zz<float, float, double, 3, false, SRC_IMAGE>(a, t, zigzag, grid, s);
      } else {
        return hipErrorInvalidValue;
      }
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_inter_residual(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W,
                                 int sr, const int64_t* mv, const QTab& t_in, int zigzag,
                                 int32_t* out, hipStream_t s) {
  if (nframes <= 0) return hipSuccess;
  QTab t = t_in;
  qtab_prepare_fused(t);
  FusedArgs a = make_fused_args(frames, mv, out, nframes, H, W, sr, t);
  const int64_t ntiles = nframes * (int64_t)a.h * a.tpr;
  launch_fused_zz<int16_t, double, double, 1, true, SRC_INTER>(a, t, zigzag,
                                                               grid_for(ntiles, 1, 8), s);
  return hipGetLastError();
}

// ======================================================================================
// Symbol histogram (feeds stats_marg / the Huffman table, entropy.py:6-29): per-workgroup
// LDS bins, the dominant zero symbol counted by wave ballots, one global add per bin.
// ======================================================================================
__global__ __launch_bounds__(256) void histogram_kernel(const int32_t* __restrict__ sym,
                                                        int64_t n, int32_t lo, int32_t nbins,
                                                        unsigned long long* __restrict__ hist,
                                                        int use_lds) {
  extern __shared__ unsigned int bins[];
  const int tid = threadIdx.x;
  if (use_lds) {
    for (int i = tid; i < nbins; i += 256) bins[i] = 0;
    __syncthreads();
  }
  const int64_t zb64 = (int64_t)0 - lo;
  const int zb = zb64 < 0 ? 0 : (zb64 >= nbins ? nbins - 1 : (int)zb64);
  unsigned zeros = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + tid; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b64 = (int64_t)sym[i] - lo;
    const int b = b64 < 0 ? 0 : (b64 >= nbins ? nbins - 1 : (int)b64);
    if (b == zb) {
      ++zeros;
    } else if (use_lds) {
      atomicAdd(&bins[b], 1u);
    } else {
      atomicAdd(&hist[b], 1ull);
    }
  }
  if (use_lds) {
    atomicAdd(&bins[zb], zeros);
    __syncthreads();
    for (int i = tid; i < nbins; i += 256)
      if (bins[i]) atomicAdd(&hist[i], (unsigned long long)bins[i]);
  } else if (zeros) {
    atomicAdd(&hist[zb], (unsigned long long)zeros);
  }
}

hipError_t launch_histogram(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins,
                            int64_t* hist, hipStream_t s) {
  if (n <= 0 || nbins <= 0) return hipSuccess;
  const int use_lds = nbins <= 16384;
  const size_t lds = use_lds ? (size_t)nbins * 4 : 0;
  histogram_kernel<<<grid_for(n, 256 * 16, 4), 256, lds, s>>>(
      sym, n, lo, nbins, reinterpret_cast<unsigned long long*>(hist), use_lds);
  return hipGetLastError();
}

}  // namespace ivc
