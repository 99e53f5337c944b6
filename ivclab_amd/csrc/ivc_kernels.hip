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
#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

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
// Standalone 2-D DCT-II / DCT-III of contiguous 8x8 units (dct.py:12-46).  (The decode chain
// dequantise -> DCT-III has its own kernel: ivc_decode.hip.)
// ======================================================================================
// IMG: the units are the blocks of Patcher.patch's view of an [H, W, C] image
// (shape.py:45-54: unit (by, bx, c) row r = image row 8 by + r, columns 8 bx .., channel c),
// read in place — the view is never gathered on the host; the output is the view's
// [H/8, W/8, C, 8, 8] layout
struct ImgLayout {
  int64_t W, C, per_row;    // image width, channels, units per block row (W / 8 * C)
};
template <typename TI, typename T, bool INV, bool IMG = false, typename TD = TinyDone>
__global__ __launch_bounds__(256) void dct8x8_kernel(const TI* __restrict__ src, int64_t nunit,
                                                     T* __restrict__ dst, T fct, int ortho,
                                                     ImgLayout im = ImgLayout{0, 1, 1},
                                                     TD done = TD{}) {
  __shared__ __attribute__((aligned(16))) T xs[32 * 72];
  src = tiny_src(src, done);
  const int tid = threadIdx.x, u = tid >> 3, r = tid & 7;
  for (int64_t g = blockIdx.x; g * 32 < nunit; g += gridDim.x) {
    const int64_t unit = g * 32 + u;
    T x[8];
    if (unit < nunit) {
      alignas(16) TI v[8];
      if constexpr (IMG) {
        const int64_t by = unit / im.per_row, rem = unit - by * im.per_row;
        const int64_t bx = rem / im.C, c = rem - bx * im.C;
        const TI* p = src + ((8 * by + r) * im.W + 8 * bx) * im.C + c;
        if (im.C == 1) {
          load8<TI>(p, v);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = p[k * im.C];
        }
      } else {
        load8<TI>(src + unit * 64 + r * 8, v);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (T)v[k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = T(0);
    }
    if constexpr (INV) dct3_line<T>(x, fct, ortho != 0); else dct2_line<T>(x, fct, ortho != 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) xs[u * 72 + r * 9 + k] = x[k];
    lds_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xs[u * 72 + i * 9 + r];
    lds_barrier();
    if constexpr (INV) dct3_line<T>(x, fct, ortho != 0); else dct2_line<T>(x, fct, ortho != 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) xs[u * 64 + i * 8 + r] = x[i];
    lds_barrier();
    const int64_t left = nunit - g * 32;
    const int nvalid = left < 32 ? (int)left : 32;
    constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-byte chunk
    T* out = dst + g * 32 * 64;
    for (int e = tid * EPC; e < nvalid * 64; e += 256 * EPC)
      *reinterpret_cast<uint4*>(out + e) = *reinterpret_cast<const uint4*>(xs + e);
    lds_barrier();
  }
  tiny_done(done);
}

// One block of a tiny host call (dct.transform(one (8, 8) block), the reference's per-block
// loops): one wave, the input from the kernel arguments, rows on lanes 0..7, the transpose
// through LDS with no workgroup barrier.  Same arithmetic as dct8x8_kernel.
template <typename TI, typename T, bool INV>
__global__ __launch_bounds__(64) void dct8x8_one_kernel(T* __restrict__ dst, T fct, int ortho,
                                                        TinyIn<512> done) {
  __shared__ __attribute__((aligned(16))) T xs[72];
  const int r = threadIdx.x;
  const TI* src = reinterpret_cast<const TI*>(done.in);
  T x[8];
  if (r < 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (T)src[r * 8 + k];
    if constexpr (INV) dct3_line<T>(x, fct, ortho != 0); else dct2_line<T>(x, fct, ortho != 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) xs[r * 9 + k] = x[k];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0);
  if (r < 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xs[i * 9 + r];
    if constexpr (INV) dct3_line<T>(x, fct, ortho != 0); else dct2_line<T>(x, fct, ortho != 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i * 8 + r] = x[i];
  }
  tiny_done(done);
}

// ---- tiny-call server --------------------------------------------------------------------
// One resident wave answers the per-block calls posted in a SrvBox (ivc_internal.h): it polls
// the request word with system-scope loads, stages the request's input in LDS, runs the same
// arithmetic as dct8x8_one_kernel / quantize_kernel / dequantize_kernel, writes the output and
// releases the completion word the host spins on (a request is read in one go with its
// checksum, SrvBox in ivc_internal.h).  It leaves its loop on a stop request, after
// idle_ticks without a request or after life_ticks in all (s_memrealtime, 100 MHz), and stores
// its generation into `exited` last, so the host relaunches it when needed and the grid always
// drains (tools/ubench/mailbox.hip: 4.3 us per 512 B round trip against ~6.4 us for a launch).
template <typename TI, typename T>
__device__ __forceinline__ void srv_dct(const unsigned char* sin, unsigned char* sout, T* xs,
                                        T fct, bool inverse, bool ortho) {
  const int r = threadIdx.x;
  const TI* src = reinterpret_cast<const TI*>(sin);
  T* dst = reinterpret_cast<T*>(sout);
  T x[8];
  if (r < 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (T)src[r * 8 + k];
    if (inverse) dct3_line<T>(x, fct, ortho); else dct2_line<T>(x, fct, ortho);
#pragma unroll
    for (int k = 0; k < 8; ++k) xs[r * 9 + k] = x[k];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0);
  if (r < 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xs[i * 9 + r];
    if (inverse) dct3_line<T>(x, fct, ortho); else dct2_line<T>(x, fct, ortho);
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i * 8 + r] = x[i];
  }
}
template <typename TI, typename D>
__device__ __forceinline__ void srv_quant(const unsigned char* sin, unsigned char* sout,
                                          const double* tq, int C, bool deq) {
  const TI* src = reinterpret_cast<const TI*>(sin);
  int32_t* dst = reinterpret_cast<int32_t*>(sout);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int e = threadIdx.x + 64 * k, p = e >> 6, j = e & 63;
    const TI v = src[(C == 1 ? 0 : p) * 64 + j];
    dst[e] = deq ? np_to_i32<D>((D)v * (D)tq[e]) : np_to_i32<D>(rint_t<D>((D)v / (D)tq[e]));
  }
}
__global__ __launch_bounds__(64) void tiny_server_kernel(SrvBox* b, uint32_t gen, uint64_t idle_ticks,
                                                         uint64_t life_ticks) {
  __shared__ __attribute__((aligned(16))) unsigned char sin[SRV_IO];
  __shared__ __attribute__((aligned(16))) unsigned char sout[SRV_IO];
  __shared__ __attribute__((aligned(16))) double xs[72];
  __shared__ double tq[192];
  const int lane = threadIdx.x;
  auto ld64 = [](const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
  uint32_t seen = __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(&b->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
  uint32_t tver = 0;                                  // table version in LDS (0: none)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = t0;
  const uint64_t* hw = reinterpret_cast<const uint64_t*>(&b->h);
  for (;;) {
    // one read of the whole request: lanes 0..7 the header's 8 words, every lane 3 input words
    const uint64_t hq = lane < 8 ? ld64(hw + lane) : 0ull;
    uint64_t w[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) w[k] = ld64(&b->in[lane + 64 * k]);
    const uint32_t r = __builtin_amdgcn_readfirstlane((uint32_t)hq);
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (r == SRV_STOP) break;
    if (r == seen) {
      if (now - last > idle_ticks || now - t0 > life_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    // the snapshot is used only if its checksum matches (else the host was still writing)
    uint64_t hs = lane < 6 ? srv_mix(hq, (uint32_t)lane) : 0ull;
#pragma unroll
    for (int k = 0; k < 3; ++k) hs += srv_mix(w[k], 6u + (uint32_t)(lane + 64 * k));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) hs += __shfl_xor(hs, o);
    const uint64_t want = __shfl(hq, 6);
    if (hs != want) continue;                         // (wave-uniform)
    seen = r;
    last = now;
    auto hword = [&](int i) { return (uint64_t)__shfl(hq, i); };
    const uint64_t q0 = hword(0), q1 = hword(1), q2 = hword(2), q3 = hword(3), q4 = hword(4), q5 = hword(5);
    const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)(q0 >> 32));
    const uint32_t sdt = __builtin_amdgcn_readfirstlane((uint32_t)q1);
    const uint32_t ddt = __builtin_amdgcn_readfirstlane((uint32_t)(q1 >> 32));
    const uint32_t inv = __builtin_amdgcn_readfirstlane((uint32_t)q2);
    const uint32_t orth = __builtin_amdgcn_readfirstlane((uint32_t)(q2 >> 32));
    const uint32_t C = __builtin_amdgcn_readfirstlane((uint32_t)q3);
    const uint32_t tv = __builtin_amdgcn_readfirstlane((uint32_t)(q3 >> 32));
    const uint32_t nout = __builtin_amdgcn_readfirstlane((uint32_t)(q4 >> 32));
    const double fct = __longlong_as_double((long long)q5);
#pragma unroll
    for (int k = 0; k < 3; ++k) reinterpret_cast<uint64_t*>(sin)[lane + 64 * k] = w[k];
    if (op != SRV_DCT && tv != tver) {
      for (int i = lane; i < 192; i += 64)
        tq[i] = __hip_atomic_load(&b->tab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      tver = tv;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0);
    if (op == SRV_DCT) {
      if (ddt == IVC_F32) {
        if (sdt == IVC_F32) srv_dct<float, float>(sin, sout, reinterpret_cast<float*>(xs), (float)fct, inv, orth);
      } else {
        switch (sdt) {
          IVC_CASE(IVC_U8, uint8_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_I8, int8_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_U16, uint16_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_I16, int16_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_U32, uint32_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_I32, int32_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_U64, uint64_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_I64, int64_t, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          IVC_CASE(IVC_F64, double, srv_dct<TI, double>(sin, sout, xs, fct, inv, orth))
          default: break;
        }
      }
    } else {
      const bool deq = op == SRV_DEQUANT;
      if (ddt == IVC_F32) {
        switch (sdt) {
          IVC_CASE(IVC_U8, uint8_t, srv_quant<TI, float>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_I8, int8_t, srv_quant<TI, float>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_U16, uint16_t, srv_quant<TI, float>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_I16, int16_t, srv_quant<TI, float>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_F32, float, srv_quant<TI, float>(sin, sout, tq, C, deq))
          default: break;
        }
      } else {
        switch (sdt) {
          IVC_CASE(IVC_U8, uint8_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_I8, int8_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_U16, uint16_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_I16, int16_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_U32, uint32_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_I32, int32_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_U64, uint64_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_I64, int64_t, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_F32, float, srv_quant<TI, double>(sin, sout, tq, C, deq))
          IVC_CASE(IVC_F64, double, srv_quant<TI, double>(sin, sout, tq, C, deq))
          default: break;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t i = (uint32_t)(lane + 64 * k);
      if (8 * i < nout)
        __hip_atomic_store(&b->out[i], reinterpret_cast<const uint64_t*>(sout)[i], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");     // the wave's output before the completion
    if (lane == 0) __hip_atomic_store(&b->done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) __hip_atomic_store(&b->exited, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_tiny_server(SrvBox* box, uint32_t gen, uint64_t idle_ticks, uint64_t life_ticks,
                              hipStream_t s) {
  tiny_server_kernel<<<1, 64, 0, s>>>(box, gen, idle_ticks, life_ticks);
  return hipGetLastError();
}

hipError_t launch_dct8x8(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
                         int inverse, int norm, hipStream_t s, const TinyDone* done) {
  const ImgLayout im0{0, 1, 1};
  if (nblk <= 0) return hipSuccess;
  // scipy: inorm 0 -> fct 1, 1 (ortho) -> 1/sqrt(2N) = 1/4, 2 -> 1/(2N) = 1/16; the inverse
  // transform uses 2 - inorm (scipy/fft/_pocketfft/helper.py _normalization)
  int inorm = inverse ? 2 - norm : norm;
  double fct = inorm == 0 ? 1.0 : (inorm == 1 ? 0.25 : 0.0625);
  int ortho = norm == IVC_NORM_ORTHO;
  if (nblk == 1 && done && done->inl && done->inl_bytes <= 512) {   // one block, tiny call
    return with_tiny<512>(done, [&](auto dn) -> hipError_t {
      if constexpr (IsTinyIn<decltype(dn)>::value) {
        if (dst_dtype == IVC_F32) {
          if (src_dtype != IVC_F32) return hipErrorInvalidValue;
          if (inverse)
            dct8x8_one_kernel<float, float, true><<<1, 64, 0, s>>>((float*)dst, (float)fct, ortho, dn);
          else
            dct8x8_one_kernel<float, float, false><<<1, 64, 0, s>>>((float*)dst, (float)fct, ortho, dn);
          return hipGetLastError();
        }
        if (dst_dtype != IVC_F64 || src_dtype == IVC_F32) return hipErrorInvalidValue;
        IVC_DISPATCH_ALL(src_dtype, {
          if (inverse)
            dct8x8_one_kernel<TI, double, true><<<1, 64, 0, s>>>((double*)dst, fct, ortho, dn);
          else
            dct8x8_one_kernel<TI, double, false><<<1, 64, 0, s>>>((double*)dst, fct, ortho, dn);
        });
        return hipGetLastError();
      } else {
        return hipErrorInvalidValue;              // (unreachable: the input fits)
      }
    });
  }
  unsigned grid = grid_for(nblk, 32, 8);
  if (dst_dtype == IVC_F32) {
    if (src_dtype != IVC_F32) return hipErrorInvalidValue;
    return with_tiny(done, [&](auto dn) -> hipError_t {
      using TD = decltype(dn);
      if (inverse)
        dct8x8_kernel<float, float, true, false, TD><<<grid, 256, 0, s>>>(
            (const float*)src, nblk, (float*)dst, (float)fct, ortho, im0, dn);
      else
        dct8x8_kernel<float, float, false, false, TD><<<grid, 256, 0, s>>>(
            (const float*)src, nblk, (float*)dst, (float)fct, ortho, im0, dn);
      return hipGetLastError();
    });
  }
  if (dst_dtype != IVC_F64 || src_dtype == IVC_F32) return hipErrorInvalidValue;
  return with_tiny(done, [&](auto dn) -> hipError_t {
    using TD = decltype(dn);
    IVC_DISPATCH_ALL(src_dtype, {
      if (inverse)
        dct8x8_kernel<TI, double, true, false, TD><<<grid, 256, 0, s>>>(
            (const TI*)src, nblk, (double*)dst, fct, ortho, im0, dn);
      else
        dct8x8_kernel<TI, double, false, false, TD><<<grid, 256, 0, s>>>(
            (const TI*)src, nblk, (double*)dst, fct, ortho, im0, dn);
    });
    return hipGetLastError();
  });
}

// DCT of the Patcher view of `rows` block rows of an [., W, C] image (dct.py:12-46 on
// shape.py:45-54's view): dst [rows, W/8, C, 8, 8]
hipError_t launch_dct8x8_image(const void* img, int src_dtype, int64_t rows, int64_t W, int64_t C,
                               void* dst, int dst_dtype, int inverse, int norm, hipStream_t s) {
  const int64_t nblk = rows * (W / 8) * C;
  if (nblk <= 0) return hipSuccess;
  const int inorm = inverse ? 2 - norm : norm;
  const double fct = inorm == 0 ? 1.0 : (inorm == 1 ? 0.25 : 0.0625);
  const int ortho = norm == IVC_NORM_ORTHO;
  const unsigned grid = grid_for(nblk, 32, 8);
  const ImgLayout im{W, C, W / 8 * C};
  if (dst_dtype == IVC_F32) {
    if (src_dtype != IVC_F32) return hipErrorInvalidValue;
    if (inverse)
      dct8x8_kernel<float, float, true, true><<<grid, 256, 0, s>>>((const float*)img, nblk,
                                                                    (float*)dst, (float)fct, ortho, im);
    else
      dct8x8_kernel<float, float, false, true><<<grid, 256, 0, s>>>((const float*)img, nblk,
                                                                     (float*)dst, (float)fct, ortho, im);
    return hipGetLastError();
  }
  if (dst_dtype != IVC_F64 || src_dtype == IVC_F32) return hipErrorInvalidValue;
  IVC_DISPATCH_ALL(src_dtype, {
    if (inverse)
      dct8x8_kernel<TI, double, true, true><<<grid, 256, 0, s>>>((const TI*)img, nblk,
                                                                 (double*)dst, fct, ortho, im);
    else
      dct8x8_kernel<TI, double, false, true><<<grid, 256, 0, s>>>((const TI*)img, nblk,
                                                                  (double*)dst, fct, ortho, im);
  });
  return hipGetLastError();
}

// ======================================================================================
// Quantise / dequantise (patchquant.py:44-78).  Element-wise over the [blk][3][64] output,
// 4 outputs (one 16-byte store) per thread; C = 1 inputs broadcast over the 3 planes.
// ======================================================================================
// The quantiser table: by value in the kernel arguments, or (a tiny call) a device copy the
// C-ABI keeps of the last table used, so the arguments stay small (each 512 B of arguments
// costs ~0.15 us of launch)
template <bool TP> struct TabArg {
  QTab t;
  __device__ const double* q() const { return t.q; }
};
template <> struct TabArg<true> {
  const double* p;
  __device__ const double* q() const { return p; }
};

template <typename TI, typename D, typename TD, bool TP = false>
__global__ __launch_bounds__(256) void quantize_kernel(const TI* __restrict__ src, int64_t nblk,
                                                       int C, TabArg<TP> tab,
                                                       int32_t* __restrict__ dst, TD done) {
  src = tiny_src(src, done);
  const double* tq = tab.q();
  const int64_t total = nblk * 48;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = g / 48;
    const int o = (int)(g - blk * 48) * 4, p = o >> 6, j = o & 63;
    const TI* sp = src + (blk * C + (C == 1 ? 0 : p)) * 64 + j;
    int v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = np_to_i32<D>(rint_t<D>((D)sp[e] / (D)tq[p * 64 + j + e]));
    *reinterpret_cast<int4*>(dst + g * 4) = make_int4(v[0], v[1], v[2], v[3]);
  }
  tiny_done(done);
}

template <typename TI, typename D, typename TD, bool TP = false>
__global__ __launch_bounds__(256) void dequantize_kernel(const TI* __restrict__ src,
                                                         int64_t nblk, int C, TabArg<TP> tab,
                                                         int32_t* __restrict__ dst, TD done) {
  src = tiny_src(src, done);
  const double* tq = tab.q();
  const int64_t total = nblk * 48;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = g / 48;
    const int o = (int)(g - blk * 48) * 4, p = o >> 6, j = o & 63;
    const TI* sp = src + (blk * C + (C == 1 ? 0 : p)) * 64 + j;
    int v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = np_to_i32<D>((D)sp[e] * (D)tq[p * 64 + j + e]);
    *reinterpret_cast<int4*>(dst + g * 4) = make_int4(v[0], v[1], v[2], v[3]);
  }
  tiny_done(done);
}

template <bool DEQ>
static hipError_t launch_quant_common(const void* src, int src_dtype, int64_t nblk, int C,
                                      const QTab& t, int calc_dtype, int32_t* dst,
                                      hipStream_t s, const TinyDone* done, const double* dtab) {
  if (nblk <= 0) return hipSuccess;
  if (C != 1 && C != 3) return hipErrorInvalidValue;
  unsigned grid = grid_for(nblk * 48, 256, 16);
  // one (3, 8, 8) stack (a tiny call): one wave, not four
  const unsigned nt = nblk * 48 <= 64 ? 64 : 256;
  if (calc_dtype != IVC_F32 && calc_dtype != IVC_F64) return hipErrorInvalidValue;
  // float32 arithmetic only arises for float32 or <= 16-bit integer inputs
  if (calc_dtype == IVC_F32 && dtype_size(src_dtype) > 2 && src_dtype != IVC_F32)
    return hipErrorInvalidValue;
  return with_tiny(done, [&](auto dn) -> hipError_t {
    using TD = decltype(dn);
    auto go = [&](auto tabc) {
      constexpr bool TP = decltype(tabc)::value;
      TabArg<TP> tab;
      if constexpr (TP) tab.p = dtab; else tab.t = t;
      IVC_DISPATCH_ALL(src_dtype, {
        if (calc_dtype == IVC_F32) {
          if constexpr (sizeof(TI) <= 2 || std::is_same<TI, float>::value) {
            if (DEQ)
              dequantize_kernel<TI, float, TD, TP><<<grid, nt, 0, s>>>((const TI*)src, nblk, C, tab, dst, dn);
            else
              quantize_kernel<TI, float, TD, TP><<<grid, nt, 0, s>>>((const TI*)src, nblk, C, tab, dst, dn);
          }
        } else {
          if (DEQ)
            dequantize_kernel<TI, double, TD, TP><<<grid, nt, 0, s>>>((const TI*)src, nblk, C, tab, dst, dn);
          else
            quantize_kernel<TI, double, TD, TP><<<grid, nt, 0, s>>>((const TI*)src, nblk, C, tab, dst, dn);
        }
      });
      return hipGetLastError();
    };
    // the device table only behind a tiny call's argument-borne input
    if constexpr (IsTinyIn<TD>::value) {
      if (dtab) return go(std::true_type{});
    }
    return go(std::false_type{});
  });
}

hipError_t launch_quantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                           int calc_dtype, int32_t* dst, hipStream_t s, const TinyDone* done,
                           const double* dtab) {
  return launch_quant_common<false>(src, src_dtype, nblk, C, t, calc_dtype, dst, s, done, dtab);
}
hipError_t launch_dequantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                             int calc_dtype, int32_t* dst, hipStream_t s, const TinyDone* done,
                             const double* dtab) {
  return launch_quant_common<true>(src, src_dtype, nblk, C, t, calc_dtype, dst, s, done, dtab);
}

// ======================================================================================
// Zig-zag permutation of 64-element rows (shape.py:21-36): flatten dst[j] = src[scan[j]]
// (the inverse of the reference's scatter by zigzag_order), unflatten dst[j] = src[order[j]].
// ======================================================================================
template <typename E, typename TD>
__global__ __launch_bounds__(256) void zigzag_kernel(const E* __restrict__ src, int64_t nrow,
                                                     int64_t stride, int inverse,
                                                     E* __restrict__ dst, TD done) {
  src = tiny_src(src, done);
  const int64_t total = nrow * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i >> 6;
    const int j = (int)(i & 63);
    dst[i] = src[row * stride + (inverse ? c_zz_order[j] : c_zz_scan[j])];
  }
  tiny_done(done);
}

hipError_t launch_zigzag(const void* src, int64_t nrow, int64_t stride, int esize, int inverse,
                         void* dst, hipStream_t s, const TinyDone* done) {
  if (nrow <= 0) return hipSuccess;
  unsigned grid = grid_for(nrow * 64, 256, 16);
  const unsigned nt = nrow <= 4 ? 64 : 256;    // a tiny call's few rows: one wave
  if (esize != 1 && esize != 2 && esize != 4 && esize != 8) return hipErrorInvalidValue;
  return with_tiny(done, [&](auto dn) -> hipError_t {
    using TD = decltype(dn);
    switch (esize) {
      case 1: zigzag_kernel<uint8_t, TD><<<grid, nt, 0, s>>>((const uint8_t*)src, nrow, stride, inverse, (uint8_t*)dst, dn); break;
      case 2: zigzag_kernel<uint16_t, TD><<<grid, nt, 0, s>>>((const uint16_t*)src, nrow, stride, inverse, (uint16_t*)dst, dn); break;
      case 4: zigzag_kernel<uint32_t, TD><<<grid, nt, 0, s>>>((const uint32_t*)src, nrow, stride, inverse, (uint32_t*)dst, dn); break;
      default: zigzag_kernel<uint64_t, TD><<<grid, nt, 0, s>>>((const uint64_t*)src, nrow, stride, inverse, (uint64_t*)dst, dn); break;
    }
    return hipGetLastError();
  });
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
//
// Wave-independent schedule: a wave owns tiles of 8 horizontally adjacent blocks (lane =
// 8*b + r: block b, row r, later column r) and a private LDS region (transpose image +
// output staging), so a tile needs no workgroup barrier.  The tile index is made provably
// wave-uniform (readfirstlane) so its decode and the buffer descriptors live in SGPRs.
// Every global access is an unconditional buffer op whose descriptor range drops the lanes
// of a ragged tile / the prefetch past the last tile: with no conditional memory ops the
// compiler can count vmcnt exactly, so the next tile's prefetched row is waited for
// without waiting for the previous tile's stores.  LDS layouts: transpose image [b][k][r]
// with block pitch 72 and k pitch 9 (conflict-free b64 writes and reads), output staging
// with block pitch 200 int32; each tile leaves as 6 x 1 KiB buffer_store_dwordx4.
// ======================================================================================
enum { SRC_IMAGE = 0, SRC_INTER = 1 };

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct FusedArgs {
  const void* img;       // SRC_IMAGE: [F][H][W][C];  SRC_INTER: u8 frames [F+1][H][W]
  const int64_t* mv;     // SRC_INTER: [F][h][w]
  int32_t* out;          // [F][h][w][3][64]
  uint32_t nframes;      // number of output frames F
  int H, W, h, w, tpr;   // tpr = tiles (of 8 blocks) per block row
  int sr;
  int split3;            // C = 3 coefficients: one wave per (group, plane) instead of per group
                         // (small launches: three times the waves, each a third of the work)
  int dup12;             // table planes 1 and 2 identical (always true for PatchQuant tables);
                         // C = 1 kernels take it as the template flag DUP
  // zero-run symbol modes (OUTM = OUT_COUNT / OUT_SYMBOLS): per-group symbol counts, their
  // exclusive offsets, the int32 stream and its capacity, the EOB symbol
  int32_t* zr_counts;
  const int64_t* zr_off;
  int32_t* zr_out;
  int64_t zr_cap;
  int32_t zr_eob;
  // OUT_SYMH (OUT_SYMBOLS + histogram): the clamped histogram of the emitted stream added onto
  // zr_hist[clamp(v - zr_hist_lo, 0, zr_hist_n - 1)] (int64 counts), so the Huffman-table
  // exchange needs no pass over the stream
  unsigned long long* zr_hist;
  int32_t zr_hist_lo, zr_hist_n;
  // OUT_COUNT hand-off to the symbol emitter (sym_emit_kernel): the group's quantised
  // coefficients by zig-zag position (lane) as int8 [gid][64][c8_stride], and as int16
  // [gid][64][2 c8_stride] for a group with a value outside int8 (zr_cflag[gid] = 1)
  int8_t* zr_c8;
  int16_t* zr_c16;
  uint8_t* zr_cflag;
  // a value outside int16 anywhere: *zr_cbad = 1, and the fused emission pass (which redoes the
  // transform) runs instead of the emitter: each kernel reads the word first (zr_gate: run
  // only when *zr_gate != 0)
  int* zr_cbad;
  const int* zr_gate;
  // store pacing (OUT_COEFS): slot s of wave w (of W) stores no earlier than
  // (*pace_t0 + (s * pace_d + w * pace_d / W) / 256) on the 100 MHz s_memrealtime clock;
  // pace_d = 0: unpaced
  uint64_t* pace_t0;     // pace block (pace_stamp_kernel): start time, late-slot counters
  uint32_t pace_d;       // 1/256 clock ticks per slot
  uint32_t pace_early;   // a wave's start-up slots, whose lateness is counted apart
#ifdef IVC_ABLATION
  int ablate;            // diagnostic builds only (tools/ablate): bit mask of skipped phases
#endif
};
#ifdef IVC_ABLATION
#define IVC_SKIP(a, bit) (((a).ablate & (bit)) != 0)
#else
#define IVC_SKIP(a, bit) false
#endif
// cache-policy bits of the streamed output stores / input loads (diagnostic builds may
// override them with -D to compare policies)
#ifndef IVC_STORE_AUX
#define IVC_STORE_AUX 2   // nt: streamed output (measured +0.8% on the cfg3 bench)
#endif
#ifndef IVC_LOAD_AUX
#define IVC_LOAD_AUX 0
#endif
#ifndef IVC_FUSED_WGCU
#define IVC_FUSED_WGCU 0   // > 0: at most this many workgroups per CU (diagnostic builds)
#endif
#ifndef IVC_FUSED_GRID
#define IVC_FUSED_GRID 0
#endif
#ifndef IVC_PACE_DEFAULT_GBPS
#define IVC_PACE_DEFAULT_GBPS 5800.0   // starting total HBM GB/s of the paced store sweep
#endif
#ifndef IVC_PREFETCH
#define IVC_PREFETCH 2   // load tiles in flight per wave (small tiles)
#endif
#ifndef IVC_WIDE_NG
#define IVC_WIDE_NG 2    // u8 luma: 8 rows x 128 bytes per wave load (whole cache lines)
#endif
#ifndef IVC_C3_PLANE_STORE
#define IVC_C3_PLANE_STORE 1   // C = 3 coefficients: each plane stored as soon as it is quantised
#endif
#ifndef IVC_C3_SPLIT
#define IVC_C3_SPLIT 1         // C = 3 coefficients, small launches: one wave per (group, plane)
#endif
#ifndef IVC_SLOT5
#define IVC_SLOT5 1            // emission slots: 4 mbcnt + a shift-add (tools/ab A/B: 0 = 6 mbcnt)
#endif
#ifndef IVC_SYM_COUNT_FRAC
#define IVC_SYM_COUNT_FRAC 8   // eighths of the resident grid for the count pass (8: all of it)
#endif
#ifndef IVC_SYM_EMIT_FRAC
#define IVC_SYM_EMIT_FRAC 8    // and for the pipelined emitter
#endif
#ifndef IVC_COUNT_PREFETCH
#define IVC_COUNT_PREFETCH 1   // the symbol count pass: one tile ahead (2: 7.05 vs 6.96 ms for
#endif                         // 256 x 4K pixels -> symbols, profiles/r05h_ab_symbols.log)
#ifndef IVC_COUNT_WAVES
#define IVC_COUNT_WAVES 7      // the symbol count pass: min waves per SIMD (1, the compiler's
#endif                         // choice: 7.47 vs 7.27 ms with the histogram, r05i_ab_symbols.log)
#ifndef IVC_C3_WAVES
#define IVC_C3_WAVES 1         // C = 3 coefficients: min waves per SIMD the registers must allow
#endif

constexpr int XS_PITCH = 72;   // T elements per block in the transpose image
// int32 per block in the output staging: 3 planes (192 + 8 pad), or 2 planes (128 + 8) when
// a C = 1 input's planes 1 and 2 are equal (DUP: plane 1 is stored twice)
template <int C, bool DUP>
constexpr int os_pitch() { return C == 1 && DUP ? 136 : 200; }
constexpr int OOB = 0x40000000;  // buffer offset beyond every descriptor range used here

// C = 3 plane-store mode (PST): one plane staged at a time, block pitch 72 int32 (= 8 mod 32,
// like 136 and 200: the quantiser's writes stay conflict-free), aliasing the transpose image
constexpr int PST_PITCH = 72;
template <typename T, int C, bool DUP, bool PST = false>
struct WaveLds {
  static constexpr int XS = 8 * XS_PITCH * (int)sizeof(T);
  static constexpr int OS = 8 * (PST ? PST_PITCH : os_pitch<C, DUP>()) * 4;
  // C = 1 and the plane-store mode alias them (the quantiser writes after the transpose reads)
  static constexpr int BYTES = (C == 1 || PST) ? (XS > OS ? XS : OS) : XS + OS;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// Store pacing.  A persistent grid whose waves store their groups as soon as they are
// computed scatters the concurrently written output over every wave's current group plus the
// waves' accumulated drift (tens of MiB), and HBM writes lose ~10-20% against an address-
// ordered sweep (tools/ubench/store_pattern4.hip, _6.hip).  Paced, wave w of W releases its
// slot-s store at t0 + s*D + w*D/W on the chip-wide constant clock, so the stores in flight at
// any instant are a few adjacent groups that sweep the buffer in address order, and no wave
// drifts.  A late wave stores at once; pacing never changes what is stored, only when.
// The rate the device sustains varies from board to board, and a schedule faster than it is
// worse than none (early waves idle while late ones store out of order), so every launch
// counts its late slots (more than a slot behind) and the host adapts the rate between
// launches (setup_pacing).
// Returns 1 if the slot was more than `slack` (1/256 ticks) late.
__device__ __forceinline__ uint32_t pace_until(uint64_t t256, uint32_t slack) {
  uint64_t now = __builtin_amdgcn_s_memrealtime();
  const uint32_t late = (now << 8) > t256 + slack ? 1u : 0u;
  while ((now << 8) < t256) {
    __builtin_amdgcn_s_sleep(1);
    now = __builtin_amdgcn_s_memrealtime();
  }
  return late;
}

// pace block: [0] schedule origin (ticks), [1..8] late-slot counters (sharded: one atomic
// word saturates near 90 updates/us), [9] the kernel's start (earliest workgroup entry),
// [10] the earliest late slot past the start-up window of any wave (diagnostics)
constexpr int PACE_SHARDS = 8, PACE_START = 1 + PACE_SHARDS, PACE_FIRST_LATE = PACE_START + 1,
              PACE_WORDS = PACE_FIRST_LATE + 1;
// a wave's first min(PACE_EARLY, slots / 8) slots are counted apart (late counter words: early
// slots in the low 32 bits, the rest in the high 32 bits): the start-up lateness while the grid
// is dispatched and the first tiles arrive is not the schedule outrunning the device
constexpr uint32_t PACE_EARLY = 64;
__global__ void pace_stamp_kernel(uint64_t* blk, uint32_t lead) {
  blk[0] = __builtin_amdgcn_s_memrealtime() + lead;
  for (int i = 1; i < PACE_START; ++i) blk[i] = 0;
  blk[PACE_START] = ~0ull;
  blk[PACE_FIRST_LATE] = ~0ull;
}


// A group = 8 horizontally adjacent blocks of one block row (one wave-step of compute and
// one 6 KiB store); a load tile = NG consecutive groups, whose 8 image rows the wave loads
// at once.  tpr counts load tiles per block row.
struct GroupLoc {
  uint32_t f;
  int bi, bj0, nb;
};

template <int NG>
__device__ __forceinline__ GroupLoc group_loc(const FusedArgs& a, uint32_t lt, int g) {
  const uint32_t tpf = (uint32_t)(a.h * a.tpr);
  GroupLoc L;
  L.f = lt / tpf;
  const uint32_t rem = lt - L.f * tpf;
  L.bi = (int)(rem / (uint32_t)a.tpr);
  L.bj0 = ((int)(rem - (uint32_t)L.bi * a.tpr) * NG + g) * 8;
  const int left = a.w - L.bj0;
  L.nb = left < 0 ? 0 : (left < 8 ? left : 8);
  return L;
}

// One lane's input row(s) as raw 32-bit words (u8 C = 1: 2 words); unpacked at use.
template <typename TI, int C, int SRC>
struct RowReg {
  static constexpr int NW = SRC == SRC_INTER ? 4 : (8 * C * (int)sizeof(TI)) / 4;
  uint32_t w[NW];
  __device__ __forceinline__ TI get(int idx) const {
    if constexpr (sizeof(TI) == 1) {
      return (TI)((w[idx >> 2] >> (8 * (idx & 3))) & 0xffu);
    } else if constexpr (sizeof(TI) == 2) {
      return (TI)((w[idx >> 1] >> (16 * (idx & 1))) & 0xffffu);
    } else if constexpr (sizeof(TI) == 4) {
      return __builtin_bit_cast(TI, w[idx]);
    } else {
      const uint64_t u = (uint64_t)w[2 * idx] | ((uint64_t)w[2 * idx + 1] << 32);
      return __builtin_bit_cast(TI, u);
    }
  }
};

template <int NW, int AUX>
__device__ __forceinline__ void buffer_words(__amdgpu_buffer_rsrc_t rs, int off, uint32_t* w) {
  if constexpr (NW % 4 == 0) {
#pragma unroll
    for (int j = 0; j < NW / 4; ++j) {
      const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * j, 0, AUX);
      w[4 * j] = x.x; w[4 * j + 1] = x.y; w[4 * j + 2] = x.z; w[4 * j + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < NW / 2; ++j) {
      const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, off + 8 * j, 0, AUX);
      w[2 * j] = x.x; w[2 * j + 1] = x.y;
    }
  }
}

// Raw input of load tile `lt`.
//  NG == 1: lane (b, r) holds row r of block b (8*C elements).
//  NG >= 2 (u8, C = 1): the wave reads 8 rows x 64*NG bytes with one 16-byte load per lane
//  per 128 bytes (lane L: row L/8, bytes 16*(L%8) of each 128-byte column), i.e. whole
//  cache lines per row; group_row() redistributes them to the (b, r) layout.
template <typename TI, int C, int NG>
struct TileRaw {
  static constexpr int NW = NG == 1 ? RowReg<TI, C, SRC_IMAGE>::NW : 2 * NG;
  uint32_t w[NW];
};

template <typename TI, int C, int NG>
__device__ __forceinline__ void load_tile(const FusedArgs& a, uint32_t lt, bool exists, int lane,
                                          TileRaw<TI, C, NG>& t) {
  const GroupLoc L = group_loc<NG>(a, exists ? lt : 0u, 0);
  const int64_t base = (((int64_t)L.f * a.H + 8 * L.bi) * a.W + 8 * L.bj0) * C;
  const uint32_t bytes = exists ? (uint32_t)(8 * a.W * C * (int)sizeof(TI)) : 0u;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const TI*>(a.img) + base, bytes);
  const int b = lane >> 3, r = lane & 7;
  if constexpr (NG == 1) {
    const int off = b < L.nb ? (r * a.W * C + 8 * b * C) * (int)sizeof(TI) : OOB;
    buffer_words<TileRaw<TI, C, NG>::NW, IVC_LOAD_AUX>(rs, off, t.w);
  } else {
    static_assert(sizeof(TI) == 1 && C == 1, "wide tiles are the u8 luma path");
#pragma unroll
    for (int j = 0; j < NG / 2; ++j) {
      const int col = 128 * j + 16 * r;                 // byte column inside the tile
      const int off = L.bj0 * 8 + col < a.W ? b * a.W + col : OOB;
      const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, IVC_LOAD_AUX);
      t.w[4 * j] = x.x; t.w[4 * j + 1] = x.y; t.w[4 * j + 2] = x.z; t.w[4 * j + 3] = x.w;
    }
  }
}

// Row r of block 8g + b for lane (b, r) from a wide tile: it sits in lane 8r + 4(g%2) + b/2,
// 16-byte column g/2, half b%2 — four ds_bpermute per group.
template <typename TI, int C, int NG>
__device__ __forceinline__ void group_row(const TileRaw<TI, C, NG>& t, int g, int lane,
                                          RowReg<TI, C, SRC_IMAGE>& v) {
  if constexpr (NG == 1) {
#pragma unroll
    for (int k = 0; k < TileRaw<TI, C, NG>::NW; ++k) v.w[k] = t.w[k];
  } else {
    const int b = lane >> 3, r = lane & 7;
    const int j = g >> 1;
    const int src = (8 * r + 4 * (g & 1) + (b >> 1)) * 4;
    const uint32_t p0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)t.w[4 * j]);
    const uint32_t p1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)t.w[4 * j + 1]);
    const uint32_t p2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)t.w[4 * j + 2]);
    const uint32_t p3 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)t.w[4 * j + 3]);
    v.w[0] = (b & 1) ? p2 : p0;
    v.w[1] = (b & 1) ? p3 : p1;
  }
}

// Residual rows of group `lt` (inter path, NG = 1): cur - block-copy prediction.
__device__ __forceinline__ void gather_inter(const FusedArgs& a, uint32_t lt, int b, int r,
                                             RowReg<int16_t, 1, SRC_INTER>& v) {
  const GroupLoc L = group_loc<1>(a, lt, 0);
  const uint8_t* fr = reinterpret_cast<const uint8_t*>(a.img);
  const int64_t HW = (int64_t)a.H * a.W;
  const __amdgpu_buffer_rsrc_t rmv =
      make_rsrc(a.mv + ((int64_t)L.f * a.h + L.bi) * a.w + L.bj0, (uint32_t)L.nb * 8u);
  const u32x2 mw = __builtin_amdgcn_raw_buffer_load_b64(rmv, b < L.nb ? b * 8 : OOB, 0, 0);
  const int64_t m = (int64_t)(((uint64_t)mw.y << 32) | mw.x);
  const __amdgpu_buffer_rsrc_t rcur = make_rsrc(
      fr + (int64_t)(L.f + 1) * HW + (int64_t)(8 * L.bi) * a.W + 8 * L.bj0, (uint32_t)(8 * a.W));
  const u32x2 cw = __builtin_amdgcn_raw_buffer_load_b64(rcur, b < L.nb ? r * a.W + 8 * b : OOB, 0, 0);
  const int n = 2 * a.sr + 1;
  int64_t qd = m / n, rm = m - qd * n;  // Python floor division (motion.py:83-84)
  if (rm < 0) { rm += n; qd -= 1; }
  const int dy = (int)qd - a.sr, dx = (int)rm - a.sr;
  const int ry = 8 * L.bi + dy, rx = 8 * (L.bj0 + b) + dx;
  // prediction is zero where the displaced block leaves the frame (motion.py:89-92)
  const bool in = b < L.nb && ry >= 0 && ry + 8 <= a.H && rx >= 0 && rx + 8 <= a.W;
  const __amdgpu_buffer_rsrc_t rref = make_rsrc(fr + (int64_t)L.f * HW, (uint32_t)HW);
  const int roff = (ry + r) * a.W + rx;
  const int o = in ? (roff & ~3) : OOB;
  const uint32_t q0 = __builtin_amdgcn_raw_buffer_load_b32(rref, o, 0, 0);
  const uint32_t q1 = __builtin_amdgcn_raw_buffer_load_b32(rref, o + 4, 0, 0);
  const uint32_t q2 = __builtin_amdgcn_raw_buffer_load_b32(rref, o + 8, 0, 0);
  const uint32_t sh = (uint32_t)(roff & 3);
  const uint32_t p0 = __builtin_amdgcn_alignbyte(q1, q0, sh);
  const uint32_t p1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    const uint32_t cs = k < 4 ? cw.x : cw.y, ps = k < 4 ? p0 : p1;
    const int d0 = (int)((cs >> (8 * (k & 3))) & 0xffu) - (int)((ps >> (8 * (k & 3))) & 0xffu);
    const int d1 = (int)((cs >> (8 * ((k + 1) & 3))) & 0xffu) - (int)((ps >> (8 * ((k + 1) & 3))) & 0xffu);
    v.w[k >> 1] = ((uint32_t)d0 & 0xffffu) | ((uint32_t)d1 << 16);
  }
}

// The staged group (LDS, block pitch OS_PITCH) leaves as 6 x 1 KiB buffer_store_dwordx4;
// lanes past a ragged group's edge, or a non-existent group, fall outside the descriptor.
template <int NG, int C, bool DUP, bool LUMA = false>
__device__ __forceinline__ void store_group(const FusedArgs& a, const int32_t* os, int lane,
                                            uint32_t lt, int g, bool exists) {
  constexpr int PITCH = os_pitch<C, DUP>();
  const GroupLoc L = group_loc<NG>(a, lt, g);
  if constexpr (LUMA) {     // plane 0 only: 2 x 1 KiB
    const __amdgpu_buffer_rsrc_t rl =
        make_rsrc(a.out + (((int64_t)L.f * a.h + L.bi) * a.w + L.bj0) * 64,
                  exists ? (uint32_t)L.nb * 256u : 0u);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int ch = lane + 64 * jj;
      const int4 val = *reinterpret_cast<const int4*>(os + (ch >> 4) * PITCH + (ch & 15) * 4);
      const u32x4 w4 = {(uint32_t)val.x, (uint32_t)val.y, (uint32_t)val.z, (uint32_t)val.w};
      __builtin_amdgcn_raw_buffer_store_b128(w4, rl, ch * 16, 0, IVC_STORE_AUX);
    }
    return;
  }
  const __amdgpu_buffer_rsrc_t ro =
      make_rsrc(a.out + (((int64_t)L.f * a.h + L.bi) * a.w + L.bj0) * 192,
                exists ? (uint32_t)L.nb * 768u : 0u);
#pragma unroll
  for (int jj = 0; jj < 6; ++jj) {
    const int ch = lane + 64 * jj;
    const int bb = ch / 48;
    int cc = ch - bb * 48;                               // 16-byte chunk inside the block
    if (C == 1 && DUP && cc >= 32) cc -= 16;             // plane 2 = staged plane 1
    const int4 val = *reinterpret_cast<const int4*>(os + bb * PITCH + cc * 4);
    const u32x4 w4 = {(uint32_t)val.x, (uint32_t)val.y, (uint32_t)val.z, (uint32_t)val.w};
    __builtin_amdgcn_raw_buffer_store_b128(w4, ro, ch * 16, 0, IVC_STORE_AUX);
  }
}

// Plane p of the staged group (PST: block pitch PST_PITCH) leaves as 2 x 1 KiB
// buffer_store_dwordx4: block bb's 256 bytes at byte (bb * 192 + p * 64) * 4 of the group.
template <int NG>
__device__ __forceinline__ void store_plane(const FusedArgs& a, const int32_t* os, int lane,
                                            uint32_t lt, int g, int p, bool exists) {
  const GroupLoc L = group_loc<NG>(a, lt, g);
  const __amdgpu_buffer_rsrc_t ro =
      make_rsrc(a.out + (((int64_t)L.f * a.h + L.bi) * a.w + L.bj0) * 192 + p * 64,
                exists && L.nb > 0 ? (uint32_t)(L.nb - 1) * 768u + 256u : 0u);
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int ch = lane + 64 * jj;
    const int bb = ch >> 4, cc = ch & 15;
    const int4 val = *reinterpret_cast<const int4*>(os + bb * PST_PITCH + cc * 4);
    const u32x4 w4 = {(uint32_t)val.x, (uint32_t)val.y, (uint32_t)val.z, (uint32_t)val.w};
    __builtin_amdgcn_raw_buffer_store_b128(w4, ro, bb * 768 + cc * 16, 0, IVC_STORE_AUX);
  }
}

// Output modes of the fused kernel: the quantised blocks themselves (OUT_COEFS: staged in LDS
// and stored), or the blocks' zero-run symbols (ivclab/entropy/zerorun.py:10-43) — their
// per-group counts (OUT_COUNT) or the symbol stream at scanned offsets (OUT_SYMBOLS).
// OUT_LUMA: the luma-table plane only ([F][h][w][64], 4 B/px out instead of the reference's
// 12 B/px 3-plane broadcast) — a reported variant, not the reference's output.
// OUT_SYMH: OUT_SYMBOLS plus the stream's histogram (FusedArgs::zr_hist).
// OUT_COEFH: OUT_COEFS plus the coefficients' histogram (FusedArgs::zr_hist), for the
// residual encoder of the sharded sequence step (the histogram pass over the output it
// replaces re-read 3.2 GB per 8-pair 8K chunk).
enum { OUT_COEFS = 0, OUT_COUNT = 1, OUT_SYMBOLS = 2, OUT_LUMA = 3, OUT_SYMH = 4, OUT_COEFH = 5 };

// Transform + quantise one group (lane (b, r)) from its raw rows into the LDS staging.
// PST (C = 3 coefficients): plane c is staged alone at os (aliasing xs) and handed to
// plane_done(c) right after its quantisation, before plane c + 1 reuses the region.
struct NoPlaneDone {
  __device__ __forceinline__ void operator()(int) const {}
};
template <typename TI, typename T, typename D, int C, bool FAST, bool ZZ, int SRC, bool CHECKMAG,
          bool DUP, bool LUMA = false, bool PST = false, typename PlaneDone = NoPlaneDone>
__device__ __forceinline__ void encode_group(const FusedArgs& a, const RowReg<TI, C, SRC>& v,
                                             T* xs, int32_t* os, const double* srq, const D* sq,
                                             int b, int r, uint32_t zp0, uint32_t zp1,
                                             PlaneDone plane_done = NoPlaneDone{}, int conly = -1) {
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (conly >= 0 && c != conly) continue;       // (split3: this wave's one plane)
    // ---- row pass (axis -1): lane owns row r of block b ------------------------------------
    T x[8];
    if constexpr (FAST) {
      int xi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) xi[k] = (int)v.get(k * C + c);
      if (IVC_SKIP(a, 1)) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = (double)xi[k];
      } else {
        dct2_row_int(xi, x);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (T)v.get(k * C + c);
      dct2_line<T>(x, T(0.25), true);
    }
    T y[8];
    if (IVC_SKIP(a, 8)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = x[i];
    } else {
      // transpose image [b][k][r], pitch 9: conflict-free b64 writes and reads
#pragma unroll
      for (int k = 0; k < 8; ++k) xs[b * XS_PITCH + k * 9 + r] = x[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = xs[b * XS_PITCH + r * 9 + i];
      __builtin_amdgcn_wave_barrier();
    }
    // ---- column pass (axis -2): lane now owns column r --------------------------------------
    if constexpr (FAST) {
      if (IVC_SKIP(a, 2)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = y[i];
      } else {
        dct2_col_unscaled(y, x);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = y[i];
      dct2_line<T>(x, T(0.25), true);
    }
    // ---- quantise ---------------------------------------------------------------------------
#pragma unroll
    for (int pi = 0; pi < (C == 1 ? 3 : 1); ++pi) {
      if (C == 1 && DUP && pi == 2) break;  // plane 2 == plane 1: stored from plane 1
      if (LUMA && pi > 0) break;
      const int p = C == 1 ? pi : c;
      int32_t* ob = PST ? os + b * PST_PITCH : os + b * os_pitch<C, DUP>() + p * 64;
      auto pos_of = [&](int i) {
        return ZZ ? (int)(((i < 4 ? zp0 : zp1) >> (8 * (i & 3))) & 63u) : i * 8 + r;
      };
      auto put = [&](int i, int32_t q) { ob[pos_of(i)] = q; };
      if (IVC_SKIP(a, 4)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) put(i, (int)x[i]);
      } else if constexpr (FAST) {
        // quotient via the scaled reciprocal, staged at once; values within 2^-30 of a
        // rounding boundary (or too large to bound the error) are redone below by exact
        // IEEE division (rare; one wave-uniform test)
        bool all_ok = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const double yq = x[i] * srq[p * 64 + i * 8 + r];
          const double rr = __builtin_rint(yq);
          bool ok = __builtin_fabs(yq - rr) < 0.5 - 0x1p-30;
          if (CHECKMAG) ok = ok && __builtin_fabs(yq) < 0x1p20;
          all_ok = all_ok && ok;
          put(i, (int)rr);
        }
        if (__ballot(!all_ok)) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const double yq = x[i] * srq[p * 64 + i * 8 + r];
            const double rr = __builtin_rint(yq);
            bool ok = __builtin_fabs(yq - rr) < 0.5 - 0x1p-30;
            if (CHECKMAG) ok = ok && __builtin_fabs(yq) < 0x1p20;
            if (!ok) {
              const double Y = x[i] * (dct2_scale(i) * dct2_scale(r));
              put(i, np_to_i32<double>(__builtin_rint(Y / (double)sq[p * 64 + i * 8 + r])));
            }
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          put(i, np_to_i32<D>(rint_t<D>((D)x[i] / sq[p * 64 + i * 8 + r])));
      }
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (PST) {
      plane_done(c);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// Zero-run coding of the group's 8 blocks x 3 planes from the zig-zag staging in LDS (the
// same staging OUT_COEFS stores).  Lane (b, r) takes zig-zag positions 8r .. 8r+7 of block
// b: a block's nonzero mask is the OR of its 8 lanes' bytes; its symbol count and each
// lane's first output slot follow from the mask, and the lane walks its 8 coefficients in
// stream order (same rules as ivc_entropy.hip's zr_mask).  Stream order is the reference's
// (h w c): block-major, planes inside a block.  OUT_SYMBOLS assembles the group's stream in
// the wave's LDS region, ZR_WIN symbols at a time, and stores it with whole-wave
// consecutive dword stores.
constexpr int ZR_WIN = XS_PITCH * 8 * 8 / 4;   // int32 symbols in a wave's transpose region
#ifndef IVC_EMIT_FIT
#define IVC_EMIT_FIT 1                           // 0: every group through the general emission
#endif
#ifndef IVC_EMIT_C8
#define IVC_EMIT_C8 1                            // emitter from the count pass's int8 hand-off
#endif
#ifndef IVC_EMIT_MASK
#define IVC_EMIT_MASK 1                          // fit path: run starts from scalar lane masks (0: DPP)
#endif

// Staging address of raster coefficient j inside a block-plane for the emission pass (the
// count pass and OUT_COEFS stage in zig-zag order).  Zig-zag staging makes the quantiser's
// writes 2-3-way bank conflicted (lane (b, r) writes zig-zag position zz(8i + r) of block b:
// 48 conflict cycles per group); this swizzle keeps both access patterns conflict-free:
//  * writes: for each raster row i the 8 addresses are distinct mod 8, so with the block pitch
//    (136 or 200, both = 8 mod 32) the 32 lanes of a ds_write_b32 lane group hit 32 banks;
//  * reads: lane k of the emission pass reads zig-zag position k, and each half (k < 32,
//    k >= 32) maps to 32 distinct banks.
// Found by a randomised search; the properties are checked at compile time below.
constexpr int c_sym_stage_h[64] = {
    7,  6,  0,  1,  3,  5,  4,  2,  10, 14, 13, 11, 8,  15, 9,  36, 19, 17, 16, 18, 12, 21,
    38, 39, 25, 26, 22, 27, 20, 32, 47, 37, 23, 24, 29, 35, 44, 33, 34, 46, 28, 30, 43, 45,
    41, 40, 55, 42, 31, 50, 53, 48, 51, 54, 49, 52, 60, 56, 63, 62, 57, 61, 59, 58};
constexpr int c_zz_order_h[64] = IVC_ZZ_ORDER;
constexpr bool sym_stage_ok() {
  bool used[64] = {};
  for (int j = 0; j < 64; ++j) {
    if (c_sym_stage_h[j] < 0 || c_sym_stage_h[j] >= 64 || used[c_sym_stage_h[j]]) return false;
    used[c_sym_stage_h[j]] = true;
  }
  for (int i = 0; i < 8; ++i) {                      // write rows: distinct mod 8
    int seen = 0;
    for (int r = 0; r < 8; ++r) seen |= 1 << (c_sym_stage_h[8 * i + r] & 7);
    if (seen != 0xff) return false;
  }
  for (int h = 0; h < 2; ++h) {                      // read halves: distinct mod 32
    unsigned long long seen = 0;
    for (int j = 0; j < 64; ++j)
      if ((c_zz_order_h[j] >> 5) == h) seen |= 1ull << (c_sym_stage_h[j] & 31);
    if (seen != 0xffffffffull) return false;
  }
  return true;
}
static_assert(sym_stage_ok(), "emission staging swizzle must be a conflict-free bijection");
// the staging address the emission pass reads for zig-zag position k (lane k)
__device__ __forceinline__ int sym_read_addr(int k) {
  int a = 0;
#pragma unroll
  for (int j = 0; j < 64; ++j)
    if (c_zz_order_h[j] == k) a = c_sym_stage_h[j];
  return a;
}

// OUT_SYMBOLS / OUT_SYMH, one block-plane at a time with lane i = zig-zag position i: the
// plane's nonzero mask is one ballot, its run starts and symbol count scalar bit operations,
// each lane's slot two mbcnt; a lane writes its value (or a run's 0 and its length) into the
// wave's LDS window (its last 64 words are the lanes' dummy slots), which is flushed to the
// stream with consecutive-address stores before a block-plane that might not fit.  Per
// group: two ds_write per block-plane instead of one per (plane, coefficient) slot and
// window pass: 11.6 vs 13.3 ms for 256 x 4K (same-process A/B, r02).
// OUT_SYMH also accumulates the stream's histogram (a.zr_hist) where the symbols leave: the
// flush that copies the window to the stream adds each symbol to the workgroup's LDS bins, so
// every symbol (values, run lengths, runs' 0s, EOBs, plane 2's repeat of plane 1) is counted
// once with a few VALU per 64 symbols.  The hot symbols (-8..7 and the EOB) have 32 copies of
// their bin, lane l adding to copy l % 32 — the copies of one value lie in 32 consecutive
// words, so a ds_add_u32 of 32 lanes hits 32 banks whatever the values; values in
// [-ZH_HALF, ZH_HALF) have one bin; the rest (rare) go to the global histogram behind one
// wave-uniform test per flush iteration.  (r03 measured two earlier forms: a branch per
// block-plane around the LDS atomic — ~13 scalar instructions each on the co-critical scalar
// unit, emission 4.9 -> 8.0 ms — and a branch-free per-block-plane add — ~8 VALU per
// block-plane, 7.66 ms.)
constexpr int ZH_HALF = 128, ZH_BINS = 2 * ZH_HALF;
constexpr int ZH_HOT_LO = -8, ZH_HOT_N = 17;            // -8..7, and the EOB as hot value 16
constexpr int ZH_HOT = ZH_BINS;                           // 32 copies per hot value
constexpr int ZH_TRASH = ZH_HOT + 32 * ZH_HOT_N;          // out-of-range values (uncounted)
constexpr int ZH_LDS = ZH_TRASH + 1;
struct ZrHistAcc {
  uint32_t* bins;      // workgroup LDS bins (OUT_SYMH)
};
__device__ __forceinline__ void zr_hist_global(const FusedArgs& a, int64_t v, uint32_t w) {
  int64_t k = v - a.zr_hist_lo;
  k = k < 0 ? 0 : (k >= a.zr_hist_n ? a.zr_hist_n - 1 : k);
  __hip_atomic_fetch_add(a.zr_hist + k, (unsigned long long)w, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}
// one symbol (or coefficient) v of weight w into the LDS bins (see above); lanes whose value
// is out of range add it to the global histogram behind one wave-uniform test
__device__ __forceinline__ void zh_add(const FusedArgs& a, uint32_t* bins, int32_t v, uint32_t w,
                                       int lane) {
  const uint32_t h0 = (uint32_t)(v - ZH_HOT_LO);             // -8..7 -> 0..15
  const uint32_t hv = v == a.zr_eob ? 16u : (h0 < 16u ? h0 : (uint32_t)ZH_HOT_N);
  const uint32_t k = (uint32_t)(v + ZH_HALF);
  const uint32_t kb = hv < (uint32_t)ZH_HOT_N ? ZH_HOT + 32 * hv + (lane & 31)
                                              : (k < (uint32_t)ZH_BINS ? k : (uint32_t)ZH_TRASH);
  atomicAdd(bins + kb, w);
  if (__builtin_expect(__ballot(kb == (uint32_t)ZH_TRASH) != 0, 0)) {
    if (kb == (uint32_t)ZH_TRASH) zr_hist_global(a, v, w);
  }
}
// the workgroup's bins into the global histogram (after a barrier)
__device__ __forceinline__ void zh_flush(const FusedArgs& a, const uint32_t* zh, int tid) {
  for (int i = tid; i < ZH_BINS; i += 256)
    if (zh[i]) zr_hist_global(a, i - ZH_HALF, zh[i]);
  for (int i0 = 0; i0 < ZH_HOT_N * 32; i0 += 256) {
    // the 32 copies of a hot value are 32 consecutive lanes of one wave
    const int i = i0 + tid;
    uint32_t c = i < ZH_HOT_N * 32 ? zh[ZH_HOT + i] : 0u;
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    if ((i & 31) == 0 && i < ZH_HOT_N * 32 && c) {
      const int hv = i >> 5;
      zr_hist_global(a, hv == 16 ? (int64_t)a.zr_eob : (int64_t)(hv + ZH_HOT_LO), c);
    }
  }
}

// a lane's histogram bin for symbol v (branch-free: both bin forms, one select)
__device__ __forceinline__ uint32_t zh_bin(const FusedArgs& a, int32_t v, int lane) {
  const uint32_t h0 = (uint32_t)(v - ZH_HOT_LO);             // -8..7 -> 0..15
  const uint32_t hv = v == a.zr_eob ? 16u : (h0 < 16u ? h0 : (uint32_t)ZH_HOT_N);
  const uint32_t k = (uint32_t)(v + ZH_HALF);
  const uint32_t hot = ZH_HOT + 32 * hv + (uint32_t)(lane & 31);
  const uint32_t cold = k < (uint32_t)ZH_BINS ? k : (uint32_t)ZH_TRASH;
  return hv < (uint32_t)ZH_HOT_N ? hot : cold;
}

// Emission of a whole group whose stream fits the wave's window (the count pass's count says
// so, a.zr_counts): every block-plane's symbols are placed with VALU only — the run starts
// come from the lane's own bits (zero, the previous lane nonzero by DPP, a nonzero later:
// m >> lane != 0), their ballot feeds the lane's slot (two mbcnt) — so the scalar unit keeps
// only the two popcounts and the running fill per block-plane, and no block has a window
// check (one basic block for the group).  Same slots and values as the general path below.
// a lane's emission slot: base + (bits of m below the lane) + 2 (bits of st below the lane)
__device__ __forceinline__ int emit_slot(uint64_t m, uint64_t st, int base) {
#if IVC_SLOT5
  // four mbcnt and one shift-add (st's count doubled) instead of six mbcnt
  uint32_t t = __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)base);
  t = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), t);
  uint32_t u = __builtin_amdgcn_mbcnt_lo((uint32_t)st, 0u);
  u = __builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), u);
  return (int)(t + 2 * u);
#else
  uint32_t t = __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)base);
  t = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), t);
  t = __builtin_amdgcn_mbcnt_lo((uint32_t)st, t);
  t = __builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), t);
  t = __builtin_amdgcn_mbcnt_lo((uint32_t)st, t);
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), t);
#endif
}
template <int C, bool DUP, bool HIST>
__device__ __forceinline__ void zr_group_emit_fit(const FusedArgs& a, int32_t* os, int64_t gbase,
                                                  int gcount, const int32_t (&xv)[8][(C == 1 && DUP) ? 2 : 3],
                                                  ZrHistAcc& H) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  constexpr int R1 = (C == 1 && DUP) ? 2 : 1;
  const int lane = threadIdx.x & 63;
  int32_t* zs = os;
  int fill = 0;
  const int32_t eob = a.zr_eob;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int32_t x = xv[b][p];
      const bool nz = x != 0;
      const uint64_t m = __ballot(nz);
      const uint64_t later = m >> lane;                         // this lane's bit and above
      const bool hl = later != 0;
#if IVC_EMIT_MASK
      // lane masks on the scalar unit: previous lane nonzero (lane 0: as if nonzero, a run may
      // start there) and a nonzero at or after the lane
      const uint64_t pm = (m << 1) | 1ull, hm = __ballot(hl);
      const uint64_t st = pm & hm & ~m;                          // run starts before the last nonzero
      const bool pnz = __builtin_amdgcn_inverse_ballot_w64(pm);
      const bool rs = __builtin_amdgcn_inverse_ballot_w64(st);
#else
      // the previous lane's nz (lane 0: as if nonzero, a run may start there)
      const bool pnz = __builtin_amdgcn_update_dpp(1, nz ? 1 : 0, 0x138, 0xf, 0xf, false) != 0;
      const bool rs = !nz && pnz && hl;                         // a run start before the last nonzero
      const uint64_t st = __ballot(rs);
#endif
      const int cnt = __builtin_popcountll(m) + 2 * __builtin_popcountll(st) + 1;
      // the lane's slot, fill included: mbcnt accumulates, so m's bits below the lane and st's
      // twice chain into one value (no shifts or adds)
      const int slot = emit_slot(m, st, fill);
      // a nonzero, a run's 0 + its length, or (the first zero after the last nonzero) the EOB
      const bool w1 = nz || pnz;
      const int32_t v1 = nz || hl ? x : eob;
      const int32_t v2 = rs ? (int32_t)__builtin_ctzll(later) : eob;
#pragma unroll
      for (int k = 0; k < (p == 1 ? R1 : 1); ++k) {
        int32_t* const d = w1 ? zs + slot + (k ? cnt : 0) : zs + ZR_WIN - 65 + lane;
        d[1] = v2;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // keep the two writes ordered
        d[0] = v1;
        fill += cnt;
      }
    }
  }
  (void)gcount;
  __builtin_amdgcn_wave_barrier();
  // the window -> the stream: a uniform loop; the store's buffer range drops slots past the
  // group's stream (and past the caller's capacity), the histogram adds weight 0 there
  const int64_t lim = a.zr_cap - gbase;
  const int nst = (int)(lim < (int64_t)fill ? (lim > 0 ? lim : 0) : (int64_t)fill);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      a.zr_out + (nst > 0 ? gbase : 0), 0, 4 * nst, 0x00020000);
  // whole 64-symbol rows without the weight test, then the partial row (the row offset stays
  // in the vector offset: the buffer range check that clips at the caller's capacity does not
  // include the scalar offset)
  const int nfull = fill >> 6;
  for (int r = 0; r < nfull; ++r) {
    const int32_t v = zs[64 * r + lane];
    __builtin_amdgcn_raw_buffer_store_b32(v, ro, 4 * (64 * r + lane), 0, 0);
    if constexpr (HIST) {
      const uint32_t kb = zh_bin(a, v, lane);
      atomicAdd(H.bins + kb, 1u);
      if (__builtin_expect(__ballot(kb == (uint32_t)ZH_TRASH) != 0, 0)) {
        if (kb == (uint32_t)ZH_TRASH) zr_hist_global(a, v, 1u);
      }
    }
  }
  if (fill & 63) {
    const int32_t v = zs[64 * nfull + lane];
    __builtin_amdgcn_raw_buffer_store_b32(v, ro, 4 * (64 * nfull + lane), 0, 0);
    if constexpr (HIST) {
      const bool in = lane < (fill & 63);
      const uint32_t kb = zh_bin(a, v, lane);
      atomicAdd(H.bins + kb, in ? 1u : 0u);
      if (__builtin_expect(__ballot(in && kb == (uint32_t)ZH_TRASH) != 0, 0)) {
        if (in && kb == (uint32_t)ZH_TRASH) zr_hist_global(a, v, 1u);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// A group's emission from its coefficients in registers (xv[b][p] = zig-zag position `lane`
// of block b, plane p) into the wave's window `os` (ZR_WIN words), then the stream.
template <int C, bool DUP, bool HIST>
__device__ __forceinline__ void zr_emit_regs(const FusedArgs& a, int32_t* os, int nb, int64_t gbase,
                                             int gcount,
                                             const int32_t (&xv)[8][(C == 1 && DUP) ? 2 : 3],
                                             ZrHistAcc& H) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  const int lane = threadIdx.x & 63;
  if (IVC_EMIT_FIT && nb == 8 && gcount <= ZR_WIN - 65) {
    zr_group_emit_fit<C, DUP, HIST>(a, os, gbase, gcount, xv, H);
    return;
  }
  int32_t* zs = os;
  int64_t base = gbase;
  int fill = 0;
  // (16-byte stores of aligned quads, as in zw_emit_kernel, measured slower here: 10.96 vs
  // 10.38 ms — a group's ~107 symbols are two dword stores per lane)
  auto flush = [&]() {
    __builtin_amdgcn_wave_barrier();
    const int64_t lim = a.zr_cap - base;
    for (int j = lane; j < fill; j += 64) {
      const int32_t v = zs[j];
      if (j < lim) a.zr_out[base + j] = v;
      if constexpr (HIST) zh_add(a, H.bins, v, 1u, lane);
    }
    __builtin_amdgcn_wave_barrier();
    base += fill;
    fill = 0;
  };
  constexpr int R1 = (C == 1 && DUP) ? 2 : 1;     // plane 2 repeats plane 1's symbols
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b >= nb) break;                         // wave-uniform
    int cnt[NP], pos[NP];
    bool w1[NP];
    int32_t v1[NP], v2[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int32_t x = xv[b][p];
      const uint64_t m = __ballot(x != 0);
      // scalar mask algebra kept short (the CU's one scalar unit issues about as many
      // instructions per group as each SIMD's VALU): last + 1 = 64 - clz, inside = bits [0, last]
      const int lz = m ? __builtin_clzll(m) : 64;
      const int last1 = 64 - lz;                                  // last + 1 (0: no nonzero)
      const uint64_t inside = m ? ~0ull >> lz : 0ull;
      const uint64_t zeros = ~m & inside;
      const uint64_t st = zeros & ~(zeros << 1);
      cnt[p] = __builtin_popcountll(m) + 2 * __builtin_popcountll(st) + 1;
      pos[p] = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) +
               2 * (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)st, 0u));
      // this lane's bits of m and st: the ballot's own predicate, and st as a lane mask
      // (one v_cndmask on the SGPR pair instead of a 64-bit shift-and-test)
      const bool nz = x != 0;
      const bool rs = __builtin_amdgcn_inverse_ballot_w64(st);
      // slot pos: a nonzero, a run's 0, or — on lane last + 1, whose pos is cnt - 1 — the EOB;
      // slot pos + 1: a run's length (it ends before the last nonzero), or the EOB after a
      // nonzero lane 63.  Inactive lanes write a private dummy word (no exec branches).
      w1[p] = nz || rs || lane == last1;
      v1[p] = nz || rs ? x : a.zr_eob;                      // x == 0 at a run start
      v2[p] = rs ? __builtin_ctzll(m >> lane) : a.zr_eob;
    }
    // one window check per block (its <= 3 x 97 symbols always fit an empty window)
    int tb = 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) tb += (p == 1 ? R1 : 1) * cnt[p];
    if (fill + tb > ZR_WIN - 65) flush();
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int k = 0; k < (p == 1 ? R1 : 1); ++k) {
        // one address per lane: slot pos + 1 is written first (a run's length, the EOB after
        // a nonzero lane 63 — both have w1 — or a don't-care that the next write fixes: after
        // a lane's single symbol comes the next emitting lane's first slot, or the next
        // block-plane's, which is written later or lies past `fill`), then slot pos;
        // lanes with nothing to write hit their dummy words
        int32_t* const d = w1[p] ? zs + fill + pos[p] : zs + ZR_WIN - 65 + lane;
        d[1] = v2[p];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // keep the two writes ordered
        d[0] = v1[p];
        fill += cnt[p];
      }
    }
  }
  flush();
}

template <int C, bool DUP, bool HIST>
__device__ __forceinline__ void zr_group_emit(const FusedArgs& a, int32_t* os, int nb,
                                              int64_t gbase, int gcount, ZrHistAcc& H) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;   // distinct planes in the staging
  constexpr int PITCH = os_pitch<C, DUP>();
  const int lane = threadIdx.x & 63;
  const int ra = sym_read_addr(lane);           // zig-zag position `lane` in the swizzled staging
  int32_t xv[8][NP];
#pragma unroll
  for (int b = 0; b < 8; ++b)
#pragma unroll
    for (int p = 0; p < NP; ++p) xv[b][p] = os[b * PITCH + p * 64 + ra];
  __builtin_amdgcn_wave_barrier();              // staging read: the region becomes the window
  zr_emit_regs<C, DUP, HIST>(a, os, nb, gbase, gcount, xv, H);
}

// The count pass's hand-off (a.zr_c8): lane k gathers zig-zag position k of the group's 8
// blocks x NP planes from the staging (lane-consecutive reads) and stores them as int8 — one
// 16-byte store per lane for NP = 2 — or, when any value of the group lies outside int8, as
// int16 in the group's slot of a.zr_c16 (flag 1).  The emitter then needs neither the pixels
// nor the transform.
constexpr int c8_stride(int NP) { return NP == 2 ? 16 : 32; }    // bytes per lane (>= 8 NP)
template <int C, bool DUP>
__device__ __forceinline__ void zr_export_coefs(const FusedArgs& a, const int32_t* os, int64_t gid) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  constexpr int PITCH = os_pitch<C, DUP>();
  constexpr int S8 = c8_stride(NP);
  const int lane = threadIdx.x & 63;
  int32_t v[8 * NP];
  int32_t vlo = INT32_MAX, vhi = INT32_MIN;                  // (min3/max3 chains: 2 VALU per 2 values)
#pragma unroll
  for (int b = 0; b < 8; ++b)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int32_t x = os[b * PITCH + p * 64 + lane];
      v[b * NP + p] = x;
      vlo = min(vlo, x);
      vhi = max(vhi, x);
    }
  const bool wide = vlo < -128 || vhi > 127, wider = vlo < -32768 || vhi > 32767;
  if (__ballot(wider) && lane == 0) atomicOr(a.zr_cbad, 1);
  uint32_t w8[S8 / 4];
#pragma unroll
  for (int k = 0; k < S8 / 4; ++k) {
    uint32_t d = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (4 * k + e < 8 * NP) d |= ((uint32_t)v[4 * k + e] & 0xffu) << (8 * e);
    w8[k] = d;
  }
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4* d8 = reinterpret_cast<u32x4*>(a.zr_c8 + (gid * 64 + lane) * S8);
#pragma unroll
  for (int k = 0; k < S8 / 16; ++k) d8[k] = u32x4{w8[4 * k], w8[4 * k + 1], w8[4 * k + 2], w8[4 * k + 3]};
  const bool any_wide = __ballot(wide) != 0;
  if (lane == 0) a.zr_cflag[gid] = any_wide ? 1 : 0;
  if (any_wide) {                                             // wave-uniform, rare
    uint32_t w16[S8 / 2];
#pragma unroll
    for (int k = 0; k < S8 / 2; ++k) {
      const int e0 = 2 * k, e1 = 2 * k + 1;
      const uint32_t lo = e0 < 8 * NP ? ((uint32_t)v[e0] & 0xffffu) : 0u;
      const uint32_t hi = e1 < 8 * NP ? ((uint32_t)v[e1] & 0xffffu) : 0u;
      w16[k] = lo | hi << 16;
    }
    u32x4* d16 = reinterpret_cast<u32x4*>(a.zr_c16 + (gid * 64 + lane) * S8);
#pragma unroll
    for (int k = 0; k < S8 / 8; ++k)
      d16[k] = u32x4{w16[4 * k], w16[4 * k + 1], w16[4 * k + 2], w16[4 * k + 3]};
  }
}

// OUT_COUNT: the group's symbol count from the zig-zag staging.  Lane (b, r) takes zig-zag
// positions 8r .. 8r+7 of block b; a block's nonzero mask is the OR of its 8 lanes' bytes.
template <int C, bool DUP, int OUTM>
__device__ __forceinline__ void zr_group(const FusedArgs& a, int32_t* os, int b, int r, int nb,
                                         int64_t gid, ZrHistAcc& H) {
  if constexpr (OUTM == OUT_SYMBOLS || OUTM == OUT_SYMH) {
    zr_group_emit<C, DUP, OUTM == OUT_SYMH>(a, os, nb, a.zr_off[gid], a.zr_counts[gid], H);
    return;
  }
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;   // distinct planes in the staging
  constexpr int PITCH = os_pitch<C, DUP>();
  const bool live = b < nb;
  const int lane = threadIdx.x & 63;
  uint64_t m[NP], st[NP];
  int cnt[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int4* src = reinterpret_cast<const int4*>(os + b * PITCH + p * 64 + 8 * r);
    const int4 v0 = src[0], v1 = src[1];
    const int32_t val[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) byte |= (uint32_t)(val[k] != 0) << k;
    // OR over the block's 8 lanes by DPP (quad_perm 1,0,3,2; 2,3,0,1; row_half_mirror):
    // VALU only, no LDS round trips
    uint32_t lo = live && r < 4 ? byte << (8 * r) : 0u;
    uint32_t hi = live && r >= 4 ? byte << (8 * (r - 4)) : 0u;
    lo |= (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0xB1, 0xf, 0xf, false);
    hi |= (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0xB1, 0xf, 0xf, false);
    lo |= (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0x4E, 0xf, 0xf, false);
    hi |= (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0x4E, 0xf, 0xf, false);
    lo |= (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0x141, 0xf, 0xf, false);
    hi |= (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0x141, 0xf, 0xf, false);
    const uint64_t lm = (uint64_t)hi << 32 | lo;
    const int last = lm ? 63 - __builtin_clzll(lm) : -1;
    const uint64_t inside = last < 0 ? 0ull : (last == 63 ? ~0ull : ((1ull << (last + 1)) - 1));
    const uint64_t zeros = ~lm & inside;
    m[p] = lm;
    st[p] = zeros & ~(zeros << 1);
    cnt[p] = live ? __builtin_popcountll(lm) + 2 * __builtin_popcountll(st[p]) + 1 : 0;
  }
  if (a.zr_c8) zr_export_coefs<C, DUP>(a, os, gid);
  __builtin_amdgcn_wave_barrier();                            // staging read: region free
  const int tb = cnt[0] + cnt[1] + cnt[NP - 1];               // the block's symbols
  int v = 0;                                                  // lane 8b holds block b's total
#pragma unroll
  for (int bb = 0; bb < 8; ++bb) v += __builtin_amdgcn_readlane(tb, 8 * bb);
  if (lane == 0) a.zr_counts[gid] = v;
}

// OUT_COEFH: the staged group's coefficients into the histogram bins (plane 1 twice when it
// is also stored as plane 2); blocks past the frame's edge are not counted
template <int C, bool DUP>
__device__ __forceinline__ void coef_hist(const FusedArgs& a, const int32_t* os, int nb,
                                          uint32_t* bins) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  constexpr int PITCH = os_pitch<C, DUP>();
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b >= nb) break;                         // wave-uniform
#pragma unroll
    for (int p = 0; p < NP; ++p)
      zh_add(a, bins, os[b * PITCH + p * 64 + lane], (C == 1 && DUP && p == 1) ? 2u : 1u, lane);
  }
}

template <typename TI, typename T, typename D, int C, bool FAST, bool ZZ, int SRC, bool CHECKMAG,
          int NG, bool DUP, int OUTM = OUT_COEFS>
__global__ __launch_bounds__(256, ((OUTM == OUT_SYMH || OUTM == OUT_SYMBOLS) && C == 1 && DUP) ? 6
                                  : (C == 3 && OUTM == OUT_COEFS ? IVC_C3_WAVES
                                     : (OUTM == OUT_COUNT && C == 1 ? IVC_COUNT_WAVES : 1)))
void fused_encode_kernel(FusedArgs a, QTab t) {
  static_assert(OUTM == OUT_COEFS || OUTM == OUT_LUMA || OUTM == OUT_COEFH || (ZZ && SRC == SRC_IMAGE),
                "symbols need zig-zag order");
  static_assert(OUTM != OUT_LUMA || C == 1, "the luma-only output is for C = 1 images");
  constexpr bool COEF = OUTM == OUT_COEFS || OUTM == OUT_LUMA || OUTM == OUT_COEFH;
  constexpr bool SYM = OUTM == OUT_SYMBOLS || OUTM == OUT_SYMH;   // emission pass
  // C = 3 coefficients: each plane stored as soon as it is quantised, so one plane is staged and
  // the staging aliases the transpose image (21.5 KB of LDS per workgroup instead of 47 KB)
  constexpr bool PST = IVC_C3_PLANE_STORE && C == 3 && OUTM == OUT_COEFS;
  typedef WaveLds<T, C, DUP, PST> L;
  __shared__ __attribute__((aligned(16))) unsigned char lds[4 * L::BYTES];
  __shared__ double srq[FAST ? 192 : 1];
  // (the table itself, for the division path and the FAST path's exact fallback; read from the
  // kernel argument instead, the 3-channel encoder measured 10 % slower: 0.4606 against
  // 0.4198 ms, profiles/r05f_ab_cfg2.log, profiles/r05e_ab_cfg2.log)
  __shared__ D sq[192];
  __shared__ uint32_t zh[OUTM == OUT_SYMH || OUTM == OUT_COEFH ? ZH_LDS : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  const int b = lane >> 3, r = lane & 7;
  if (a.zr_gate && *a.zr_gate == 0) return;           // (the emitter's fallback, not needed)
  for (int i = tid; i < 192; i += 256) {
    sq[i] = (D)t.q[i];
    // s_i * s_k * RN(1/q): the DCT's power-of-two output scales folded into the reciprocal
    // (1.0 / q is IEEE-correctly rounded here as on the host)
    if constexpr (FAST) srq[i] = (dct2_scale((i >> 3) & 7) * dct2_scale(i & 7)) * (1.0 / t.q[i]);
  }
  // zig-zag positions of this lane's column (raster i*8 + r), packed 4 per register
  // (the emission pass stages through the bank-conflict-free swizzle instead)
  uint32_t zp0 = 0, zp1 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (SYM) {
      zp0 |= (uint32_t)c_sym_stage_h[i * 8 + r] << (8 * i);
      zp1 |= (uint32_t)c_sym_stage_h[(i + 4) * 8 + r] << (8 * i);
    } else {
      zp0 |= (uint32_t)(ZZ ? c_zz_order[i * 8 + r] : i * 8 + r) << (8 * i);
      zp1 |= (uint32_t)(ZZ ? c_zz_order[(i + 4) * 8 + r] : (i + 4) * 8 + r) << (8 * i);
    }
  }
  ZrHistAcc hacc{nullptr};
  if constexpr (OUTM == OUT_SYMH || OUTM == OUT_COEFH) {
    for (int i = tid; i < ZH_LDS; i += 256) zh[i] = 0;
    hacc.bins = zh;
  }
  lds_barrier();  // tables only; the loop below never synchronises across waves (but the
                    // symbol histogram's bins are flushed after a barrier at the end)

  unsigned char* mine = lds + wave * L::BYTES;
  T* xs = reinterpret_cast<T*>(mine);
  int32_t* os = reinterpret_cast<int32_t*>(mine + ((C == 1 || PST) ? 0 : L::XS));
  const uint32_t nlt = a.nframes * (uint32_t)(a.h * a.tpr);
  const uint32_t nwaves = gridDim.x * 4u;
  uint32_t lt = blockIdx.x * 4u + wave;

  // pacing clock of this wave's slots (slot = groups stored so far), in 1/256 ticks
  uint64_t pace_next = 0;
  if (COEF && a.pace_d) {
    pace_next = (*a.pace_t0 << 8) + (uint64_t)a.pace_d * (blockIdx.x * 4u + wave) / nwaves;
    if (tid == 0)
      __hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(a.pace_t0) + PACE_START,
                             (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // late slots of the wave's first PACE_EARLY slots (start-up: the grid is still being
  // dispatched and the first tiles loaded while the schedule runs) and of the rest
  uint32_t nlate_early = 0, nlate = 0, pslot = 0, first_late = 0xffffffffu;
  // the pacing wait of the next slot (PST: before a group's first plane store)
  auto pace_slot = [&]() {
    const uint32_t l = pace_until(pace_next, a.pace_d);
    if (pslot < a.pace_early) {
      nlate_early += l;
    } else {
      nlate += l;
      if (l && first_late == 0xffffffffu) first_late = pslot;
    }
    ++pslot;
    pace_next += a.pace_d;
  };
  auto store_prev = [&](uint32_t plt, int pg, bool have_prev) {
    if constexpr (COEF && !PST) {
      if (a.pace_d && have_prev) pace_slot();
      store_group<NG, C, DUP, OUTM == OUT_LUMA>(a, os, lane, plt, pg, have_prev && !IVC_SKIP(a, 16));
    }
  };
  uint32_t plt = 0;
  int pg = 0;
  bool have_prev = false;

  // (3-channel images: one tile ahead — the two-tile rounds measured slower there, 0.4266 vs
  // 0.4198 ms for 64 x 1080p RGB and 14.9 vs 8.7 us for one frame, profiles/r05e_ab_cfg2.log)
  constexpr int PF = (SRC == SRC_IMAGE && TileRaw<TI, C, NG>::NW <= 8)
                        ? (C == 3 ? 1 : (OUTM == OUT_COUNT ? IVC_COUNT_PREFETCH : IVC_PREFETCH)) : 1;
  if (PST && a.split3) {
    // one wave per (group, plane): virtual unit vt = 3 lt + c; the group's rows are loaded
    // whole (the wave uses one channel of them) and its plane stored as soon as it is quantised
    if constexpr (PST) {
      const uint32_t nvt = 3u * nlt;
      for (uint32_t vt = lt; vt < nvt; vt += nwaves) {
        const uint32_t t3 = vt / 3u;
        const int c = (int)(vt - 3u * t3);
        TileRaw<TI, C, NG> raw;
        load_tile<TI, C, NG>(a, t3, true, lane, raw);
        RowReg<TI, C, SRC> v;
        group_row<TI, C, NG>(raw, 0, lane, v);
        encode_group<TI, T, D, C, FAST, ZZ, SRC, CHECKMAG, DUP, false, PST>(
            a, v, xs, os, srq, sq, b, r, zp0, zp1,
            [&](int cc) { store_plane<NG>(a, os, lane, t3, 0, cc, !IVC_SKIP(a, 16)); }, c);
      }
    }
  } else if constexpr (PF > 1) {
    // Software pipeline per wave in rounds of PF load tiles (nwaves apart).  At the start of
    // a round the wave issues the loads of the whole next round at once, so the chip's read
    // stream arrives in bursts between long runs of stores instead of an even 1:12 mix with
    // them (HBM read/write turnarounds: tools/ubench/store_pattern8.hip); the next round's
    // tiles land in a second register ring that becomes the current one at the round's end
    // (its wait covers loads a whole round old).  Every group first issues the stores of the
    // previous group (staged in LDS).  Ragged and past-the-end tiles go through zero-range
    // descriptors instead of branches.
    TileRaw<TI, C, NG> ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const uint32_t t0 = lt + p * nwaves;
      load_tile<TI, C, NG>(a, t0, t0 < nlt && !IVC_SKIP(a, 32), lane, ring[p]);
    }
    for (; lt < nlt; lt += PF * nwaves) {
      TileRaw<TI, C, NG> nxt[PF];
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const uint32_t nt = lt + (PF + p) * nwaves;
        load_tile<TI, C, NG>(a, nt, nt < nlt && !IVC_SKIP(a, 32), lane, nxt[p]);
      }
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const uint32_t tp = lt + p * nwaves;
        const bool ex = tp < nlt;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          store_prev(plt, pg, have_prev);
          RowReg<TI, C, SRC> v;
          group_row<TI, C, NG>(ring[p], g, lane, v);
          encode_group<TI, T, D, C, FAST, ZZ, SRC, CHECKMAG, DUP, OUTM == OUT_LUMA, PST>(
              a, v, xs, os, srq, sq, b, r, zp0, zp1, [&](int c) {
                if constexpr (PST) {
                  if (c == 0 && a.pace_d && ex) pace_slot();
                  store_plane<NG>(a, os, lane, tp, g, c, ex && !IVC_SKIP(a, 16));
                }
              });
          if constexpr (OUTM == OUT_COEFH) {
            if (ex) coef_hist<C, DUP>(a, os, group_loc<NG>(a, tp, g).nb, hacc.bins);
          }
          if constexpr (!COEF) {
            if (ex) zr_group<C, DUP, OUTM>(a, os, b, r, group_loc<NG>(a, tp, g).nb, (int64_t)tp * NG + g, hacc);
          }
          plt = tp;
          pg = g;
          have_prev = ex;
        }
      }
#pragma unroll
      for (int p = 0; p < PF; ++p) ring[p] = nxt[p];
    }
  } else {
    // Software pipeline per wave, one tile ahead.  Group (lt, g) first issues the stores of
    // the previous group (staged in LDS); group 0 then issues the prefetch of load tile
    // lt + nwaves; then the group is transformed.  The prologue issues the same number of
    // (range-dropped) stores, so every path into a wait for tile lt's rows has the same ops
    // behind that load and the compiler's vmcnt wait never includes the stores.
    TileRaw<TI, C, NG> raw;
    if constexpr (SRC == SRC_IMAGE) {
      load_tile<TI, C, NG>(a, lt, lt < nlt, lane, raw);
      if constexpr (COEF) {
#pragma unroll
        for (int g = 1; g < NG; ++g) store_group<NG, C, DUP, OUTM == OUT_LUMA>(a, os, lane, 0u, 0, false);
      }
    }
    for (; lt < nlt; lt += nwaves) {
      TileRaw<TI, C, NG> nraw;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        store_prev(plt, pg, have_prev);
        RowReg<TI, C, SRC> v;
        if constexpr (SRC == SRC_IMAGE) {
          if (g == 0) {
            const uint32_t nt = lt + nwaves;
            load_tile<TI, C, NG>(a, nt, nt < nlt && !IVC_SKIP(a, 32), lane, nraw);
          }
          group_row<TI, C, NG>(raw, g, lane, v);
        } else {
          gather_inter(a, lt, b, r, v);
        }
        encode_group<TI, T, D, C, FAST, ZZ, SRC, CHECKMAG, DUP, OUTM == OUT_LUMA, PST>(
            a, v, xs, os, srq, sq, b, r, zp0, zp1, [&](int c) {
              if constexpr (PST) {
                if (c == 0 && a.pace_d) pace_slot();
                store_plane<NG>(a, os, lane, lt, g, c, !IVC_SKIP(a, 16));
              }
            });
        if constexpr (OUTM == OUT_COEFH) coef_hist<C, DUP>(a, os, group_loc<NG>(a, lt, g).nb, hacc.bins);
        if constexpr (!COEF)
          zr_group<C, DUP, OUTM>(a, os, b, r, group_loc<NG>(a, lt, g).nb, (int64_t)lt * NG + g, hacc);
        plt = lt;
        pg = g;
        have_prev = true;
      }
      if constexpr (SRC == SRC_IMAGE) raw = nraw;
    }
  }
  if constexpr (COEF) {
    if constexpr (!PST) {
      if (a.pace_d && have_prev) pace_slot();
      store_group<NG, C, DUP, OUTM == OUT_LUMA>(a, os, lane, plt, pg, have_prev && !IVC_SKIP(a, 16));
    }
    if ((nlate | nlate_early) && lane == 0) {
      unsigned long long* blk = reinterpret_cast<unsigned long long*>(a.pace_t0);
      __hip_atomic_fetch_add(blk + 1 + blockIdx.x % PACE_SHARDS,
                             (unsigned long long)nlate_early | ((unsigned long long)nlate << 32),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nlate)
        __hip_atomic_fetch_min(blk + PACE_FIRST_LATE, (unsigned long long)first_late,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (OUTM == OUT_SYMH || OUTM == OUT_COEFH) {
    lds_barrier();
    zh_flush(a, zh, tid);
  }
}


// Library scratch is stream-ordered (hipMallocAsync on the caller's stream).  The device's
// default memory pool is told once to keep freed blocks, so repeated calls reuse memory
// instead of mapping and unmapping gigabytes per call.
static std::once_flag g_pool_once[64];
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev >= 0 && dev < 64)
    std::call_once(g_pool_once[dev], [dev] {
      hipMemPool_t pool;
      if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
        uint64_t keep = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      }
    });
  return hipMallocAsync(p, bytes ? bytes : 16, s);
}

static std::mutex g_occ_mu;
static std::unordered_map<const void*, int> g_occ;

// Persistent grids: as many 256-thread groups as the device holds at once (occupancy of
// this kernel, cached per kernel), never more than the work needs.
unsigned resident_grid_ptr(const void* kernel, int64_t work_groups_needed) {
  int per_cu = 0;
  {
    std::lock_guard<std::mutex> g(g_occ_mu);
    auto it = g_occ.find(kernel);
    if (it != g_occ.end()) {
      per_cu = it->second;
    } else {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      g_occ[kernel] = per_cu;
    }
  }
  int64_t g = (int64_t)num_cus() * per_cu;
  if (work_groups_needed < g) g = work_groups_needed;
  return (unsigned)(g < 1 ? 1 : g);
}

template <typename K>
static unsigned resident_grid(K kernel, int64_t work_groups_needed) {
  return resident_grid_ptr(reinterpret_cast<const void*>(kernel), work_groups_needed);
}

// Store pacing of the coefficient-writing fused kernels (see pace_until).  The rate is the
// total HBM rate (input + output bytes) the paced sweep is timed for, per device and encoder.
// Every paced launch is measured: setup_pacing reserves a slot of a ring (PACE_RING) for it
// and finish_pacing closes exactly that slot (the pace block copied to pinned memory, the
// duration from two events), so launches from several host threads never share a slot.
// Completed measurements are folded in launch order when a later launch is set up, or when
// the statistics are read.  Each fold starts from the rate THAT launch ran at (S.rate): a
// burst of launches enqueued without synchronisation all ran at one rate, and folding k of
// their failures must not compound into 0.98^k.
//  * late slots above PACE_LATE_HI of the launch's slots, and the launch moved less than its
//    schedule: the schedule outran the device.  The rate drops to the lower of 98% of the
//    launch's rate and 1.1x what it actually moved (over the pace the sweep runs ~10% under
//    it), never below what the last good launch moved (that floor decays 2% per failure so a
//    device that really slowed down is followed), and the launch's rate becomes the "too
//    fast" mark;
//  * late but the launch moved at least its schedule's rate: the lateness did not come from
//    the rate (e.g. a schedule origin already behind when the kernel started); recorded, no
//    step back;
//  * otherwise the rate creeps up from the launch's rate (+1.5% per launch while under 96%
//    of the mark, +0.3% nearer it), never past 98% of the mark (the edge is sharp and
//    bimodal: launches at 99% of a failed rate still fail half the time), which itself rises
//    0.1% per good launch so a transient cannot cap the rate for good;
//  * the first measured launch of the process only records (fresh output pages: slow).
// ivc_store_pace_settle drops the rate to the last rate that held its schedule (and below the
// mark by a margin) — callers that enqueue many launches at once use it after a warm-up so the
// whole burst runs at a validated rate.  Fixed-rate sweeps (IVC_PACE_FIXED, two boxes): good
// launches hold the schedule to within ~35 us; the edge sat at 5.9 and 6.1-6.2 TB/s.
// IVC_PACE_GBPS / ivc_set_store_pace set the starting rate (0 disables pacing).
static std::mutex g_pace_mu;
static double g_pace_start = -1.0;
// late-slot fractions are bimodal: < 1% below the device's rate, 20-50% once over it
constexpr double PACE_LATE_HI = 0.05, PACE_MAX_GBPS = 7600.0;
constexpr int PACE_RING = 32, PACE_TRACE = 256;
// Lead of the schedule origin over the stamp kernel's clock read (ticks of 10 ns).  The
// kernel's first workgroups enter ~5 us after the stamp, and a wave needs ~20 us (its first
// tile loads, first groups) before its first store: with the origin at +3 us the first ~10 %
// of every wave's slots ran late (20-48 % of them) and the late waves' out-of-order stores
// cost 4 % of the launch; with +30 us no start-up slot is late (same-box A/B over leads of
// 3, 15, 30, 50, 80, 120 and 200 us, tools/gpu_r03_lead.sh: 4.968 -> 4.717 ms; past 50 us the
// idle wait costs more than it saves).  IVC_PACE_LEAD overrides it (experiments).
static uint32_t pace_lead() {
  static const uint32_t v = [] {
    const char* e = getenv("IVC_PACE_LEAD");
    const long x = e ? atol(e) : 3000;
    return (uint32_t)(x < 0 ? 0 : (x > 1000000 ? 1000000 : x));
  }();
  return v;
}

enum PaceSlotState { PS_FREE = 0, PS_ARMED, PS_CLOSED, PS_VOID };
struct PaceSlot {
  uint64_t* host = nullptr;       // pinned copy of the pace block
  hipEvent_t t0 = nullptr, t1 = nullptr;  // around the kernel (timing)
  hipEvent_t done = nullptr;      // after the pace block's copy
  double slots = 0, slots_per_wave = 0, bytes = 0, rate = 0;
  int state = PS_FREE;
  int64_t gen = 0;                // the controller generation it was launched under
};
struct PaceStats {
  int64_t measured = 0, over = 0, late_fast = 0;
  double sum_late = 0, max_late = 0, sum_gbps = 0;
};
// one folded measurement: rate the launch ran at, the late fraction of its slots past the
// start-up window, event-timed GB/s, the kernel's first workgroup entry relative to the
// schedule origin (us; > 0: origin behind), the earliest late slot past the start-up window as
// a fraction of the slots per wave (-1: none late), the rate after the fold, the late
// fraction of the start-up slots
struct PaceTraceRec {
  double rate, late, gbps, lag_us, first_late, next_rate, late_early;
};
struct PaceState {
  uint64_t* blk = nullptr;        // device pace block
  PaceSlot ring[PACE_RING];
  int head = 0, count = 0;        // oldest reserved measurement, number reserved
  double rate = 0, too_fast = 1e30, last_late = -1;
  double good_rate = 0, good_gbps = 0;  // the last launch that held its schedule
  bool seen_first = false;        // the process's first measured launch (not adapted on)
  PaceStats st;
  PaceTraceRec trace[PACE_TRACE];
  int64_t ntrace = 0;             // records since the last reset (ring of PACE_TRACE)
  int64_t gen = 0;                // bumped by ivc_set_store_pace: older launches are not folded
};
// per device and per encoder (0: image source, 1: inter residual source, 2: luma-only image)
static PaceState g_pace[64][3];

static double pace_start_rate() {
  if (g_pace_start < 0) {
    const char* e = getenv("IVC_PACE_GBPS");
    g_pace_start = e ? atof(e) : IVC_PACE_DEFAULT_GBPS;
    if (!(g_pace_start >= 0)) g_pace_start = 0;
  }
  return g_pace_start;
}

// IVC_PACE_FIXED (set): keep the rate where ivc_set_store_pace / IVC_PACE_GBPS put it and
// only record the launches' measurements (rate sweeps, tools/ab/ab_intra.py --pace).
static bool pace_fixed() {
  static const bool f = getenv("IVC_PACE_FIXED") != nullptr;
  return f;
}

static double pace_early_slots(double slots_per_wave) {
  return std::min<double>(PACE_EARLY, std::floor(slots_per_wave / 8));
}

// One completed measurement into the controller (caller holds g_pace_mu).
static void pace_fold(PaceState& P, const PaceSlot& S) {
  uint64_t late = 0, late_early = 0;
  for (int i = 0; i < PACE_SHARDS; ++i) {
    late_early += S.host[1 + i] & 0xffffffffull;
    late += S.host[1 + i] >> 32;
  }
  float ms = 0;
  const bool timed = hipEventElapsedTime(&ms, S.t0, S.t1) == hipSuccess && ms > 0;
  const double early_slots = S.slots / S.slots_per_wave * pace_early_slots(S.slots_per_wave);
  const double rest_slots = S.slots - early_slots;
  const double f = rest_slots > 0 ? (double)late / rest_slots : 0.0;
  const double f_early = early_slots > 0 ? (double)late_early / early_slots : 0.0;
  const double gbps = timed ? S.bytes / (ms * 1e-3) / 1e9 : 0.0;
  const uint64_t t0 = S.host[0], start = S.host[PACE_START], fl = S.host[PACE_FIRST_LATE];
  const double lag_us = start != ~0ull ? ((double)(int64_t)(start - t0)) * 1e-2 : 0.0;
  const double first_late = fl != ~0ull && S.slots_per_wave > 0 ? (double)fl / S.slots_per_wave : -1.0;
  P.last_late = f;
  P.st.measured += 1;
  P.st.sum_late += f;
  P.st.max_late = std::max(P.st.max_late, f);
  P.st.sum_gbps += gbps;
  const bool first = !P.seen_first;            // fresh output pages: slow
  P.seen_first = true;
  const bool over = f > PACE_LATE_HI;
  if (over) P.st.over += 1;
  if (!pace_fixed() && !first) {
    if (over && gbps > 0 && gbps >= 0.99 * S.rate) {
      P.st.late_fast += 1;                     // late, yet at least as fast as the schedule
    } else if (over) {
      P.too_fast = std::min(P.too_fast, S.rate);
      double r = 0.98 * S.rate;
      if (gbps > 0) r = std::min(r, 1.1 * gbps);
      r = std::max(r, P.good_gbps);
      P.good_gbps *= 0.98;
      P.rate = std::max(std::min(P.rate, r), 100.0);
    } else {
      P.good_rate = S.rate;
      P.good_gbps = gbps;
      P.too_fast *= 1.001;
      const double cap = std::min(PACE_MAX_GBPS, 0.98 * P.too_fast);
      const double step = S.rate < 0.96 * P.too_fast ? 1.015 : 1.003;
      P.rate = std::max(P.rate, std::min(S.rate * step, cap));
    }
  }
  PaceTraceRec& T = P.trace[P.ntrace % PACE_TRACE];
  T = {S.rate, f, gbps, lag_us, first_late, P.rate, f_early};
  P.ntrace += 1;
}

// Folds every completed measurement, oldest first (caller holds g_pace_mu).  Stops at a slot
// whose launch is still being enqueued or whose copy has not landed.
static void pace_harvest(PaceState& P) {
  while (P.count > 0) {
    PaceSlot& S = P.ring[P.head];
    if (S.state == PS_ARMED) break;
    if (S.state == PS_CLOSED) {
      if (hipEventQuery(S.done) != hipSuccess) break;   // its copy may still land in S.host
      // dropped when pacing was switched off or the rate set anew since its launch
      if (P.rate > 0 && S.gen == P.gen) pace_fold(P, S);
    }
    S.state = PS_FREE;
    P.head = (P.head + 1) % PACE_RING;
    P.count -= 1;
  }
  (void)hipGetLastError();
}

static PaceState* pace_state_current(int kind) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  return &g_pace[dev][kind];
}

double store_pace_gbps() {
  std::lock_guard<std::mutex> g(g_pace_mu);
  PaceState* P = pace_state_current(0);
  if (P && P->blk) {
    pace_harvest(*P);
    return P->rate;
  }
  return pace_start_rate();
}

double store_pace_late_fraction() {
  std::lock_guard<std::mutex> g(g_pace_mu);
  PaceState* P = pace_state_current(0);
  if (!P) return -1;
  if (P->blk) pace_harvest(*P);
  return P->last_late;
}

int store_pace_stats(int kind, double* out, int n) {
  std::lock_guard<std::mutex> g(g_pace_mu);
  PaceState* P = pace_state_current(kind);
  if (!P) return 0;
  if (P->blk) pace_harvest(*P);
  const PaceStats& s = P->st;
  const double m = s.measured > 0 ? (double)s.measured : 1.0;
  const double v[10] = {(double)s.measured, (double)s.over, s.sum_late / m, s.max_late,
                        P->blk ? P->rate : pace_start_rate(), P->last_late, s.sum_gbps / m,
                        (double)P->count, (double)s.late_fast,
                        P->too_fast < 1e29 ? P->too_fast : 0.0};
  for (int i = 0; i < n && i < 10; ++i) out[i] = v[i];
  return n < 10 ? n : 10;
}

int store_pace_trace(int kind, double* out, int max_records) {
  std::lock_guard<std::mutex> g(g_pace_mu);
  PaceState* P = pace_state_current(kind);
  if (!P) return 0;
  if (P->blk) pace_harvest(*P);
  const int64_t have = std::min<int64_t>(P->ntrace, PACE_TRACE);
  const int64_t n = std::min<int64_t>(have, max_records);
  for (int64_t i = 0; i < n; ++i) {         // the n most recent, oldest first
    const PaceTraceRec& T = P->trace[(P->ntrace - n + i) % PACE_TRACE];
    double* o = out + 7 * i;
    o[0] = T.rate; o[1] = T.late; o[2] = T.gbps; o[3] = T.lag_us; o[4] = T.first_late;
    o[5] = T.next_rate; o[6] = T.late_early;
  }
  return (int)n;
}

void store_pace_reset_stats() {
  std::lock_guard<std::mutex> g(g_pace_mu);
  for (auto& d : g_pace)
    for (auto& p : d) {
      if (p.blk) pace_harvest(p);
      p.st = PaceStats();
      p.ntrace = 0;
    }
}

void store_pace_settle(double margin) {
  std::lock_guard<std::mutex> g(g_pace_mu);
  for (int kind = 0; kind < 3; ++kind) {
    PaceState* P = pace_state_current(kind);
    if (!P || !P->blk || P->rate <= 0) continue;
    pace_harvest(*P);
    if (P->good_rate > 0) P->rate = std::min(P->rate, P->good_rate);
    if (P->too_fast < 1e29) P->rate = std::min(P->rate, (1.0 - margin) * P->too_fast);
    P->rate = std::max(P->rate, 100.0);
  }
}

void set_store_pace_gbps(double gbps) {
  std::lock_guard<std::mutex> g(g_pace_mu);
  g_pace_start = gbps > 0 ? gbps : 0.0;
  for (auto& d : g_pace)
    for (auto& p : d) {
      p.rate = g_pace_start;
      p.too_fast = 1e30;
      p.good_rate = p.good_gbps = 0;
      p.gen += 1;                 // launches of the previous rate are never folded into this one
    }
}

static bool pace_alloc(PaceState& P) {
  if (hipMalloc((void**)&P.blk, 8 * PACE_WORDS) != hipSuccess) {
    P.blk = nullptr;
    return false;
  }
  for (auto& S : P.ring) {
    if (hipHostMalloc((void**)&S.host, 8 * PACE_WORDS, hipHostMallocDefault) != hipSuccess ||
        hipEventCreate(&S.t0) != hipSuccess || hipEventCreate(&S.t1) != hipSuccess ||
        hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess) {
      S.host = nullptr;            // this slot (and the rest) stay unusable
      return false;                // blk stays set: the ring is partially usable (process-long)
    }
  }
  return true;
}

// Turns pacing on for a launch of `nwaves` persistent waves that store `slots` groups each
// (of `group_bytes` input + output bytes): a one-lane kernel on the same stream stamps the
// start time (the clock pace_lead() ticks ahead, covering the launch gap) and clears the counters.
// Returns the reserved measurement slot (-1: the launch is paced but not measured), which the
// caller hands to finish_pacing after the kernel.  Concurrent launches on other streams may
// overwrite the device's pace block between a stamp and its kernel; that only shifts a
// schedule by a launch gap or blurs one launch's late count.
static int setup_pacing(FusedArgs& a, int kind, int64_t nwaves, int64_t slots,
                        double group_bytes, hipStream_t s) {
  if (slots < 8) return -1;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
  std::lock_guard<std::mutex> g(g_pace_mu);
  PaceState& P = g_pace[dev][kind];
  if (!P.blk) {
    if (pace_start_rate() <= 0) return -1;
    if (!pace_alloc(P)) {
      (void)hipGetLastError();
      if (!P.blk) return -1;
    }
    P.rate = pace_start_rate();
  }
  pace_harvest(P);
  if (P.rate <= 0) return -1;
  // ticks (10 ns) per slot: the whole grid's slot bytes at the target rate
  const double d256 = (double)nwaves * group_bytes / (P.rate * 1e9) * 1e8 * 256.0;
  if (!(d256 >= 1.0) || d256 > 4.0e9) return -1;
  int slot = -1;
  if (P.count < PACE_RING) {
    const int k = (P.head + P.count) % PACE_RING;
    PaceSlot& S = P.ring[k];
    if (S.host && S.done && hipEventRecord(S.t0, s) == hipSuccess) {
      S.slots = (double)nwaves * (double)slots;
      S.slots_per_wave = (double)slots;
      S.bytes = (double)nwaves * (double)slots * group_bytes;
      S.rate = P.rate;
      S.gen = P.gen;
      S.state = PS_ARMED;
      P.count += 1;
      slot = k;
    }
    (void)hipGetLastError();
  }
  pace_stamp_kernel<<<1, 1, 0, s>>>(P.blk, pace_lead());
  a.pace_t0 = P.blk;
  a.pace_d = (uint32_t)d256;
  a.pace_early = (uint32_t)pace_early_slots((double)slots);
  return slot;
}

// After a paced launch: close its measurement (end event, pace block copy, done event).
static void finish_pacing(int kind, int slot, hipStream_t s) {
  int dev = 0;
  if (slot < 0 || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
  std::lock_guard<std::mutex> g(g_pace_mu);
  PaceState& P = g_pace[dev][kind];
  PaceSlot& S = P.ring[slot];
  if (S.state != PS_ARMED) return;
  const bool ok =
      hipEventRecord(S.t1, s) == hipSuccess &&
      hipMemcpyAsync(S.host, P.blk, 8 * PACE_WORDS, hipMemcpyDeviceToHost, s) == hipSuccess &&
      hipEventRecord(S.done, s) == hipSuccess;
  S.state = ok ? PS_CLOSED : PS_VOID;
  (void)hipGetLastError();
}

// NG: groups of 8 blocks per wave load (wide, whole-cache-line row loads for u8 luma)
template <typename TI, typename T, typename D, int C, bool FAST, bool ZZ, int SRC, bool CM,
          int NGW = IVC_WIDE_NG, int OUTM = OUT_COEFS>
static void launch_fused_one(const FusedArgs& a_in, const QTab& t, hipStream_t s) {
  constexpr int NG = (sizeof(TI) == 1 && C == 1 && SRC == SRC_IMAGE) ? NGW : 1;
  FusedArgs a = a_in;
  a.tpr = (a.w + 8 * NG - 1) / (8 * NG);
  const int64_t nlt = (int64_t)a.nframes * a.h * a.tpr;
  // IVC_FUSED_GRID: 0 = exactly resident (persistent waves), k > 0 = k tiles per wave
  auto grid = [&](auto k) -> unsigned {
    if constexpr (IVC_FUSED_GRID == 0) {
      unsigned g = resident_grid(k, (nlt + 3) / 4);
      if (IVC_FUSED_WGCU > 0 && g > (unsigned)(num_cus() * IVC_FUSED_WGCU))
        g = (unsigned)(num_cus() * IVC_FUSED_WGCU);
      return g;
    } else {
      const int64_t g = (nlt + 4 * IVC_FUSED_GRID - 1) / (4 * IVC_FUSED_GRID);
      return (unsigned)(g < 1 ? 1 : g);
    }
  };
  // input + output bytes of one group (8 blocks)
  const double out_bytes = OUTM == OUT_LUMA ? 256.0 : 768.0;
  const double gbytes = 8.0 * (SRC == SRC_INTER ? 64.0 * 2 + 8.0 + out_bytes
                                                : 64.0 * C * sizeof(TI) + out_bytes);
  // pacing state per encoder: image source, inter residual, luma-only image
  const int kind = OUTM == OUT_LUMA ? 2 : SRC;
  // unpaced: the luma-only variant (its PMC, profiles/r04g_pmc_luma.json, shows it issue-bound,
  // not store-order-bound, and faster without the schedule) and the 3-channel image encoder
  // (cfg2, 64 x 1080p RGB: 0.429 ms unpaced against 0.445-0.493 ms paced at any start rate,
  // profiles/r05d_ab_cfg2.log — it is issue/latency-bound, 3 transforms per 8-block group)
  constexpr bool unpaced = OUTM == OUT_LUMA || (C == 3 && SRC == SRC_IMAGE);
  auto go = [&](auto k) {
    // 3-channel coefficients, few groups (fewer than 2 per resident wave: one frame of cfg2):
    // one wave per (group, plane)
    if (C == 3 && OUTM == OUT_COEFS && SRC == SRC_IMAGE && IVC_C3_PLANE_STORE && IVC_C3_SPLIT &&
        nlt < 8 * (int64_t)resident_grid(k, (int64_t)1 << 40)) {
      a.split3 = 1;
      const unsigned g3 = resident_grid(k, (3 * nlt + 3) / 4);
      k<<<g3, 256, 0, s>>>(a, t);
      return;
    }
    const unsigned g = grid(k);
    const int64_t nw = 4 * (int64_t)g;
    const int slot = unpaced ? -1 : setup_pacing(a, kind, nw, (nlt + nw - 1) / nw * NG, gbytes, s);
    k<<<g, 256, 0, s>>>(a, t);
    finish_pacing(kind, slot, s);
  };
  if (C == 1 && (a.dup12 || OUTM == OUT_LUMA))
    go(fused_encode_kernel<TI, T, D, C, FAST, ZZ, SRC, CM, NG, C == 1, OUTM>);
  else
    go(fused_encode_kernel<TI, T, D, C, FAST, ZZ, SRC, CM, NG, false, OUTM>);
}

// The FAST quotient check needs |quotient| < 2^20.  Integer pixels
// and residuals of u8 frames bound every DCT-II ortho coefficient by 64*255/4 < 4096, so a
// table with min |q| > 1/256 proves the bound and the per-value magnitude test is dropped.
static bool needs_magnitude_check(const QTab& t) {
  for (int i = 0; i < 192; ++i)
    if (!(__builtin_fabs(t.q[i]) > 1.0 / 256.0) || __builtin_isinf(t.q[i])) return true;
  return false;
}

template <typename TI, typename T, typename D, int C, bool FAST, int SRC>
static void launch_fused_zz(const FusedArgs& a, const QTab& t, int zigzag, int64_t ntiles,
                            hipStream_t s) {
  const bool cm = FAST && needs_magnitude_check(t);
  if (zigzag) {
    if (cm) launch_fused_one<TI, T, D, C, FAST, true, SRC, true>(a, t, s);
    else launch_fused_one<TI, T, D, C, FAST, true, SRC, false>(a, t, s);
  } else {
    if (cm) launch_fused_one<TI, T, D, C, FAST, false, SRC, true>(a, t, s);
    else launch_fused_one<TI, T, D, C, FAST, false, SRC, false>(a, t, s);
  }
}

static FusedArgs make_fused_args(const void* img, const int64_t* mv, int32_t* out,
                                 int64_t nframes, int64_t H, int64_t W, int sr,
                                 const QTab& t) {
  FusedArgs a;
  a.img = img; a.mv = mv; a.out = out; a.nframes = (uint32_t)nframes;
  a.H = (int)H; a.W = (int)W; a.h = (int)(H / 8); a.w = (int)(W / 8);
  a.tpr = (a.w + 7) / 8;
  a.sr = sr;
  a.zr_counts = nullptr;
  a.zr_off = nullptr;
  a.zr_out = nullptr;
  a.zr_cap = 0;
  a.zr_eob = 0;
  a.zr_hist = nullptr;
  a.zr_hist_lo = 0;
  a.zr_hist_n = 0;
  a.zr_c8 = nullptr;
  a.zr_c16 = nullptr;
  a.zr_cflag = nullptr;
  a.zr_cbad = nullptr;
  a.zr_gate = nullptr;
  a.pace_t0 = nullptr;
  a.pace_d = 0;
  a.pace_early = 0;
  a.split3 = 0;
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
  const QTab& t = t_in;
  FusedArgs a = make_fused_args(img, nullptr, out, nframes, H, W, 0, t);
  const int64_t ntiles = nframes * (int64_t)a.h * a.tpr;
  if (ntiles >= (1LL << 31)) return hipErrorInvalidValue;  // 32-bit tile indices
  switch (dtype) {
    case IVC_U8:
      if (calc_dtype != IVC_F64) return hipErrorInvalidValue;
      if (C == 1) launch_fused_zz<uint8_t, double, double, 1, true, SRC_IMAGE>(a, t, zigzag, ntiles, s);
      else launch_fused_zz<uint8_t, double, double, 3, true, SRC_IMAGE>(a, t, zigzag, ntiles, s);
      break;
    case IVC_F64:
      if (calc_dtype != IVC_F64) return hipErrorInvalidValue;
      if (C == 1) launch_fused_zz<double, double, double, 1, false, SRC_IMAGE>(a, t, zigzag, ntiles, s);
      else launch_fused_zz<double, double, double, 3, false, SRC_IMAGE>(a, t, zigzag, ntiles, s);
      break;
    case IVC_F32:
      if (calc_dtype == IVC_F32) {
        if (C == 1) launch_fused_zz<float, float, float, 1, false, SRC_IMAGE>(a, t, zigzag, ntiles, s);
        else launch_fused_zz<float, float, float, 3, false, SRC_IMAGE>(a, t, zigzag, ntiles, s);
      } else if (calc_dtype == IVC_F64) {
        if (C == 1) launch_fused_zz<float, float, double, 1, false, SRC_IMAGE>(a, t, zigzag, ntiles, s);
        else launch_fused_zz<float, float, double, 3, false, SRC_IMAGE>(a, t, zigzag, ntiles, s);
      } else {
        return hipErrorInvalidValue;
      }
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// The luma-table plane only of a u8 C = 1 batch: out [F][h][w][64] int32 (plane 0 of what
// launch_intra_encode writes).  A reported variant (5 B/px of HBM traffic instead of 13): the
// reference's PatchQuant.quantize broadcasts C = 1 to 3 planes (patchquant.py:59).
hipError_t launch_intra_encode_luma(const uint8_t* img, int64_t nframes, int64_t H, int64_t W,
                                    const QTab& t, int zigzag, int32_t* out, hipStream_t s) {
  if (nframes <= 0 || H <= 0 || W <= 0) return hipSuccess;
  FusedArgs a = make_fused_args(img, nullptr, out, nframes, H, W, 0, t);
  if (nframes * (int64_t)a.h * a.tpr >= (1LL << 31)) return hipErrorInvalidValue;
  const bool cm = needs_magnitude_check(t);
#define LUMA_GO(ZZV, CMV) \
  launch_fused_one<uint8_t, double, double, 1, true, ZZV, SRC_IMAGE, CMV, IVC_WIDE_NG, OUT_LUMA>(a, t, s)
  if (zigzag) { if (cm) LUMA_GO(true, true); else LUMA_GO(true, false); }
  else { if (cm) LUMA_GO(false, true); else LUMA_GO(false, false); }
#undef LUMA_GO
  return hipGetLastError();
}

// ---- pixels -> zero-run symbols (IntraCodec.image2symbols' hot part, intracodec.py:66-81):
// count pass, int64 scan of the per-group counts, emission pass.
// The symbol emitter of the two-pass pixels -> symbols path (IVC_EMIT_C8): group gid's
// coefficients come from the count pass's hand-off (int8, or int16 for a group flagged wide),
// not from the pixels, so the pass is the emission alone — no pixel loads, no transform.
// One wave per group (grid-stride); the window and the histogram bins as in the fused pass.
// Exits at once when the count pass met a value outside int16 (*zr_cbad): the fused emission
// pass runs instead.
template <int C, bool DUP, bool HIST, int NG>
__global__ __launch_bounds__(256) void sym_emit_kernel(FusedArgs a, int64_t ngroups,
                                                       const int32_t* __restrict__ gcounts,
                                                       const int64_t* __restrict__ goffs,
                                                       const uint8_t* __restrict__ gflags) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  constexpr int S8 = c8_stride(NP);
  __shared__ __attribute__((aligned(16))) int32_t win[4 * ZR_WIN];
  __shared__ uint32_t zh[HIST ? ZH_LDS : 1];
  if (*a.zr_cbad) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  ZrHistAcc hacc{nullptr};
  if constexpr (HIST) {
    for (int i = tid; i < ZH_LDS; i += 256) zh[i] = 0;
    hacc.bins = zh;
    lds_barrier();
  }
  int32_t* os = win + wave * ZR_WIN;
  const int64_t nw = (int64_t)gridDim.x * 4;
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  // a group's block column within its block row, kept incrementally (the count pass numbers
  // the groups row by row: gid % (tpr NG) groups of 8 blocks from the row's start)
  const int gpr = a.tpr * NG;
  const int64_t gid0 = (int64_t)blockIdx.x * 4 + wave;
  int gx = (int)(gid0 % gpr);
  const int gstep = (int)(nw % gpr);
  // the next group's count, offset, flag word and int8 coefficients are loaded while this
  // group is emitted
  struct Pre {
    int count;
    int64_t off;
    uint32_t flagw;
    i32x4 w[S8 / 16];
  };
  auto fetch = [&](int64_t gg, Pre& P) {
    // (read-only, non-aliased kernel arguments: scalar loads, waited for at their first use
    // in the next iteration, not right after the issue as uniform vector loads were)
    P.count = gcounts[gg];
    P.off = goffs[gg];
    P.flagw = *reinterpret_cast<const uint32_t*>(gflags + (gg & ~(int64_t)3));
    const i32x4* src = reinterpret_cast<const i32x4*>(a.zr_c8 + (gg * 64 + lane) * S8);
#pragma unroll
    for (int k = 0; k < S8 / 16; ++k) P.w[k] = __builtin_nontemporal_load(src + k);
  };
  Pre cur;
  if (gid0 < ngroups) fetch(gid0, cur);
  for (int64_t gid = gid0; gid < ngroups; gid += nw) {
    Pre nxt;
    if (gid + nw < ngroups) fetch(gid + nw, nxt);
    const int gcount = cur.count;
    const int nbl = a.w - 8 * gx;
    const int nb = nbl < 0 ? 0 : (nbl < 8 ? nbl : 8);
    gx += gstep;
    if (gx >= gpr) gx -= gpr;
    if (gcount != 0) {                                           // (0: a group past the row's end)
      int32_t xv[8][NP];
      if (((cur.flagw >> (8 * (gid & 3))) & 0xffu) == 0) {
#pragma unroll
        for (int e = 0; e < 8 * NP; ++e) {
          const uint32_t word = (uint32_t)cur.w[e / 16][(e / 4) & 3];
          xv[e / NP][e % NP] = (int32_t)(int8_t)(uint8_t)(word >> (8 * (e & 3)));
        }
      } else {                                                   // rare: the group's int16 slot
        const i32x4* src = reinterpret_cast<const i32x4*>(a.zr_c16 + (gid * 64 + lane) * S8);
        i32x4 w[S8 / 8];
#pragma unroll
        for (int k = 0; k < S8 / 8; ++k) w[k] = src[k];
#pragma unroll
        for (int e = 0; e < 8 * NP; ++e) {
          const uint32_t word = (uint32_t)w[e / 8][(e / 2) & 3];
          xv[e / NP][e % NP] = (int32_t)(int16_t)(uint16_t)(word >> (16 * (e & 1)));
        }
      }
      zr_emit_regs<C, DUP, HIST>(a, os, nb, cur.off, gcount, xv, hacc);
    }
    cur = nxt;
  }
  if constexpr (HIST) {
    lds_barrier();
    zh_flush(a, zh, tid);
  }
}

template <typename TI, int C, bool DUP, bool CM, int OUTM>
static void launch_fused_zr(const FusedArgs& a_in, const QTab& t, hipStream_t s) {
  constexpr int NG = (sizeof(TI) == 1 && C == 1) ? IVC_WIDE_NG : 1;
  FusedArgs a = a_in;
  a.tpr = (a.w + 8 * NG - 1) / (8 * NG);
  const int64_t nlt = (int64_t)a.nframes * a.h * a.tpr;
  auto k = fused_encode_kernel<TI, double, double, C, true, true, SRC_IMAGE, CM, NG, DUP, OUTM>;
  unsigned grid = resident_grid(k, (nlt + 3) / 4);
  if (OUTM == OUT_COUNT && IVC_SYM_COUNT_FRAC < 8) grid = grid * IVC_SYM_COUNT_FRAC / 8 + 1;
  k<<<grid, 256, 0, s>>>(a, t);
}

// The count pass and the emitter pipelined over K chunks of whole frames (like the zero-run
// encode, ivc_entropy.hip): chunk j's count pass on the caller's stream, its scan (continuing
// chunk j - 1's total) and then its emission on the second stream.  A
// chunk's groups are contiguous (frame-major group numbering), so every per-group array is
// addressed from the chunk's first group; chunks start on whole block rows, so the emitter's
// column bookkeeping is unchanged.
#ifndef IVC_SYM_CHUNKS
#define IVC_SYM_CHUNKS 16
#endif
// groups per chunk at least: smaller chunks measured slower than no pipelining (64 x 4K frames:
// 2.18 ms unpipelined, 2.08 with 4 chunks of 259 K groups, 2.45 with 8, 3.34 with 16 —
// profiles/r04aq_ab_small_batch.log; 256 frames: 20 chunks of 207 K groups fine, 24 of 173 K not)
#ifndef IVC_SYM_MIN_CHUNK
#define IVC_SYM_MIN_CHUNK 196608
#endif
static int sym_chunks(int64_t nframes, int64_t ngroups, int64_t gpf) {
  int K = IVC_SYM_CHUNKS;
  if (K > PIPE_EVENTS - 2) K = PIPE_EVENTS - 2;
  if (ngroups / IVC_SYM_MIN_CHUNK < K) K = (int)(ngroups / IVC_SYM_MIN_CHUNK);
  if (K < 1) K = 1;
  if (const int f = tuning(IVC_TUNE_SYM_CHUNKS)) K = std::min(f, PIPE_EVENTS - 2);  // any size
  if (K > nframes) K = (int)nframes;
  if (gpf % 4 != 0) K = 1;                           // the emitter reads the flags 4 at a time
  return K;
}

// hist[i] += part[i] when the count passes found no value outside int16 (*gate == 0): the
// pipelined emitters' histogram joins the caller's only once every chunk's count pass has
// run, so an emitter that started before a later chunk set cbad never reaches hist (the fused
// OUT_SYMH pass, gated the other way, then counts every frame)
__global__ __launch_bounds__(256) void hist_gated_add_kernel(unsigned long long* __restrict__ hist,
                                                             const unsigned long long* __restrict__ part,
                                                             int32_t n, const int* __restrict__ gate) {
  if (*gate) return;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    if (part[i]) hist[i] += part[i];
}

template <int C, bool DUP, int NG, typename CountFn>
static hipError_t intra_symbols_pipelined(const FusedArgs& a, int64_t gpf, int K, int64_t* agg,
                                          CountFn count, hipStream_t s) {
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  constexpr int S8 = c8_stride(NP);
  PipeCtx* pp = nullptr;
  hipError_t e = pipe_ctx(&pp);
  if (e != hipSuccess) return e;
  PipeCtx& P = *pp;
  std::lock_guard<std::mutex> lock(P.mu);
  int64_t* off = const_cast<int64_t*>(a.zr_off);
  if ((e = hipMemsetAsync(off, 0, 8, s)) != hipSuccess) return e;
  // the emitters' histogram goes to a scratch copy, added to hist after the join (above)
  unsigned long long* hpart = nullptr;
  if (a.zr_hist) {
    if ((e = scratch_alloc((void**)&hpart, (size_t)a.zr_hist_n * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(hpart, 0, (size_t)a.zr_hist_n * 8, s)) != hipSuccess) {
      (void)hipFreeAsync(hpart, s);
      return e;
    }
  }
  struct FreeOnExit {
    void* p;
    hipStream_t s;
    ~FreeOnExit() { if (p) (void)hipFreeAsync(p, s); }
  } hfree{hpart, s};
  if ((e = hipEventRecord(P.ev[PIPE_EVENTS - 2], s)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(P.aux, P.ev[PIPE_EVENTS - 2], 0)) != hipSuccess) return e;
  PipeJoin join{P, s, true};
  const int64_t fpc = ((int64_t)a.nframes + K - 1) / K;
  const size_t fbytes = (size_t)a.H * a.W * C;          // u8 frames
  auto k = a.zr_hist ? sym_emit_kernel<C, DUP, true, NG> : sym_emit_kernel<C, DUP, false, NG>;
  for (int j = 0; j < K; ++j) {
    const int64_t f0 = (int64_t)j * fpc, f1 = std::min<int64_t>(f0 + fpc, a.nframes);
    if (f1 <= f0) break;
    const int64_t g0 = f0 * gpf, len = (f1 - f0) * gpf;
    FusedArgs ac = a;
    if (hpart) ac.zr_hist = hpart;
    ac.img = static_cast<const uint8_t*>(a.img) + f0 * fbytes;
    ac.nframes = (uint32_t)(f1 - f0);
    ac.zr_counts = a.zr_counts + g0;
    ac.zr_off = off + g0;
    ac.zr_c8 = a.zr_c8 + g0 * 64 * S8;
    ac.zr_c16 = a.zr_c16 + g0 * 64 * S8;
    ac.zr_cflag = a.zr_cflag + g0;
    count(ac);
    // the scan on the second stream, ahead of its emitter: the caller's stream runs the count
    // passes back to back
    if ((e = hipEventRecord(P.ev[j], s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(P.aux, P.ev[j], 0)) != hipSuccess) return e;
    if ((e = launch_exclusive_scan_i32_carry(ac.zr_counts, len, agg, off + g0, P.aux)) != hipSuccess)
      return e;
    unsigned eg = resident_grid(k, (len + 3) / 4);
    if (IVC_SYM_EMIT_FRAC < 8) eg = eg * IVC_SYM_EMIT_FRAC / 8 + 1;
    k<<<eg, 256, 0, P.aux>>>(ac, len, ac.zr_counts, ac.zr_off, ac.zr_cflag);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  join.armed = false;
  if ((e = hipEventRecord(P.ev[PIPE_EVENTS - 1], P.aux)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(s, P.ev[PIPE_EVENTS - 1], 0)) != hipSuccess) return e;
  if (hpart) {
    hist_gated_add_kernel<<<(a.zr_hist_n + 255) / 256 < 1024 ? (a.zr_hist_n + 255) / 256 : 1024, 256, 0, s>>>(
        a.zr_hist, hpart, a.zr_hist_n, a.zr_cbad);
    e = hipGetLastError();
  }
  return e;
}

template <typename TI, int C, bool DUP, bool CM>
static hipError_t intra_symbols_t(const FusedArgs& a0, const QTab& t, int64_t* nsym,
                                  hipStream_t s) {
  constexpr int NG = (sizeof(TI) == 1 && C == 1) ? IVC_WIDE_NG : 1;
  const int64_t tpr = (a0.w + 8 * NG - 1) / (8 * NG);
  const int64_t ngroups = (int64_t)a0.nframes * a0.h * tpr * NG;
  FusedArgs a = a0;
  int32_t* counts = nullptr;
  int64_t* agg = nullptr;
  int64_t* off = nullptr;
  constexpr int NP = (C == 1 && DUP) ? 2 : 3;
  // the coefficient hand-off (IVC_EMIT_C8): only when the stream is emitted
  bool c8 = IVC_EMIT_C8 && a.zr_cap > 0;
  int8_t* c8buf = nullptr;
  int16_t* c16buf = nullptr;
  uint8_t* cflag = nullptr;
  int* cbad = nullptr;
  hipError_t e = scratch_alloc((void**)&counts, (size_t)ngroups * 4, s);
  if (e == hipSuccess) e = scratch_alloc((void**)&agg, (size_t)scan_scratch_elems(ngroups) * 8, s);
  if (e == hipSuccess) e = scratch_alloc((void**)&off, (size_t)(ngroups + 1) * 8, s);
  if (c8 && e == hipSuccess) {
    const size_t per = (size_t)64 * c8_stride(NP);
    hipError_t e8 = scratch_alloc((void**)&c8buf, (size_t)ngroups * per, s);
    if (e8 == hipSuccess) e8 = scratch_alloc((void**)&c16buf, (size_t)ngroups * 2 * per, s);
    if (e8 == hipSuccess) e8 = scratch_alloc((void**)&cflag, (size_t)ngroups + 16, s);
    if (e8 == hipSuccess) e8 = scratch_alloc((void**)&cbad, 16, s);
    if (e8 == hipSuccess) e8 = hipMemsetAsync(cbad, 0, 16, s);
    if (e8 != hipSuccess) {
      // no room for the hand-off: the path without it (count pass, scan, fused emission)
      for (void** pp : {(void**)&c8buf, (void**)&c16buf, (void**)&cflag, (void**)&cbad}) {
        if (*pp) (void)hipFreeAsync(*pp, s);
        *pp = nullptr;
      }
      (void)hipGetLastError();
      c8 = false;
    }
  }
  if (e == hipSuccess) {
    a.zr_counts = counts;
    a.zr_off = off;
    a.zr_c8 = c8buf;
    a.zr_c16 = c16buf;
    a.zr_cflag = cflag;
    a.zr_cbad = cbad;
  }
  const int64_t gpf = (int64_t)a0.h * tpr * NG;                // groups per frame
  const int K = (e == hipSuccess && c8) ? sym_chunks(a.nframes, ngroups, gpf) : 1;
  if (K > 1) {
    FusedArgs ap = a;
    ap.tpr = (int)tpr;                    // the emitter's group_loc tiles of NG groups
    e = intra_symbols_pipelined<C, DUP, NG>(
        ap, gpf, K, agg, [&](const FusedArgs& ac) { launch_fused_zr<TI, C, DUP, CM, OUT_COUNT>(ac, t, s); }, s);
    if (e == hipSuccess) e = hipMemcpyAsync(nsym, off + ngroups, 8, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) {
      // the fused emission pass over every frame, only when the emitters stood down (*cbad)
      a.zr_gate = cbad;
      if (a.zr_hist) launch_fused_zr<TI, C, DUP, CM, OUT_SYMH>(a, t, s);
      else launch_fused_zr<TI, C, DUP, CM, OUT_SYMBOLS>(a, t, s);
      e = hipGetLastError();
    }
  } else if (e == hipSuccess) {
    launch_fused_zr<TI, C, DUP, CM, OUT_COUNT>(a, t, s);
    e = launch_exclusive_scan_i32(counts, ngroups, agg, off, s);
  }
  if (K <= 1 && e == hipSuccess) e = hipMemcpyAsync(nsym, off + ngroups, 8, hipMemcpyDeviceToDevice, s);
  if (K <= 1 && e == hipSuccess && a.zr_cap > 0) {
    if (c8) {
      // the emitter; the fused emission pass only when the emitter stood down (*cbad)
      auto k = a.zr_hist ? sym_emit_kernel<C, DUP, true, NG> : sym_emit_kernel<C, DUP, false, NG>;
      FusedArgs ae = a;
      ae.tpr = (int)tpr;                  // group_loc's tiles of NG groups, as the count pass
      k<<<resident_grid(k, (ngroups + 3) / 4), 256, 0, s>>>(ae, ngroups, ae.zr_counts, ae.zr_off,
                                                            ae.zr_cflag);
      a.zr_gate = cbad;
    }
    if (a.zr_hist) launch_fused_zr<TI, C, DUP, CM, OUT_SYMH>(a, t, s);
    else launch_fused_zr<TI, C, DUP, CM, OUT_SYMBOLS>(a, t, s);
    e = hipGetLastError();
  }
  if (counts) (void)hipFreeAsync(counts, s);
  if (agg) (void)hipFreeAsync(agg, s);
  if (off) (void)hipFreeAsync(off, s);
  for (void* pp : {(void*)c8buf, (void*)c16buf, (void*)cflag, (void*)cbad})
    if (pp) (void)hipFreeAsync(pp, s);
  return e;
}

hipError_t launch_intra_symbols(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                                int C, const QTab& t, int32_t eob, int32_t* out, int64_t capacity,
                                int64_t* nsym, hipStream_t s, int64_t* hist, int32_t hist_lo,
                                int32_t hist_n) {
  if (dtype != IVC_U8 || (C != 1 && C != 3)) return hipErrorInvalidValue;
  FusedArgs a = make_fused_args(img, nullptr, nullptr, nframes, H, W, 0, t);
  a.zr_out = out;
  a.zr_cap = capacity;
  a.zr_eob = eob;
  a.zr_hist = hist_n > 0 ? reinterpret_cast<unsigned long long*>(hist) : nullptr;
  a.zr_hist_lo = hist_lo;
  a.zr_hist_n = hist_n;
  if (nframes <= 0 || H <= 0 || W <= 0) return hipMemsetAsync(nsym, 0, 8, s);
  if (nframes * (int64_t)a.h * a.tpr >= (1LL << 31)) return hipErrorInvalidValue;
  const bool cm = needs_magnitude_check(t);
  if (C == 1) {
    if (a.dup12) return cm ? intra_symbols_t<uint8_t, 1, true, true>(a, t, nsym, s)
                           : intra_symbols_t<uint8_t, 1, true, false>(a, t, nsym, s);
    return cm ? intra_symbols_t<uint8_t, 1, false, true>(a, t, nsym, s)
              : intra_symbols_t<uint8_t, 1, false, false>(a, t, nsym, s);
  }
  return cm ? intra_symbols_t<uint8_t, 3, false, true>(a, t, nsym, s)
            : intra_symbols_t<uint8_t, 3, false, false>(a, t, nsym, s);
}

hipError_t launch_inter_residual(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W,
                                 int sr, const int64_t* mv, const QTab& t_in, int zigzag,
                                 int32_t* out, hipStream_t s, int64_t* hist, int32_t hist_lo,
                                 int32_t hist_n) {
  if (nframes <= 0) return hipSuccess;
  const QTab& t = t_in;
  FusedArgs a = make_fused_args(frames, mv, out, nframes, H, W, sr, t);
  const int64_t ntiles = nframes * (int64_t)a.h * a.tpr;
  if (ntiles >= (1LL << 31)) return hipErrorInvalidValue;  // 32-bit tile indices
  if (hist && hist_n > 0) {
    // the coefficients' histogram accumulated by the encoder itself (OUT_COEFH)
    a.zr_hist = reinterpret_cast<unsigned long long*>(hist);
    a.zr_hist_lo = hist_lo;
    a.zr_hist_n = hist_n;
    const bool cm = needs_magnitude_check(t);
#define RES_H(ZZV, CMV) \
  launch_fused_one<int16_t, double, double, 1, true, ZZV, SRC_INTER, CMV, IVC_WIDE_NG, OUT_COEFH>(a, t, s)
    if (zigzag) { if (cm) RES_H(true, true); else RES_H(true, false); }
    else { if (cm) RES_H(false, true); else RES_H(false, false); }
#undef RES_H
    return hipGetLastError();
  }
  launch_fused_zz<int16_t, double, double, 1, true, SRC_INTER>(a, t, zigzag, ntiles, s);
  return hipGetLastError();
}

// ======================================================================================
// Symbol histogram (feeds stats_marg / the Huffman table, entropy.py:6-29).  Zero-run and
// coefficient streams are concentrated near zero (the cfg3 stream: values -3..4 are 89% of
// the symbols, 1 alone 29%), so a wave's LDS atomics on one bin serialise ~20-way.  Each
// thread therefore counts the HOT values -3..4 in registers (one compare-add per counter,
// flushed once through a wave reduction and the same clamp as every other value) and only
// the rest go to per-workgroup LDS bins; one global add per bin per workgroup at the end.
// ======================================================================================
constexpr int HIST_HOT_LO = -3, HIST_HOT_N = 8, HIST_UNROLL = 4;
#ifndef IVC_HIST_PACKED
#define IVC_HIST_PACKED 1
#endif

template <typename S>
__device__ __forceinline__ int hist_bin(S v, int64_t lo, int32_t nbins) {
  // clamp into the end bins; v - lo is formed unsigned once v > lo (no overflow)
  if ((int64_t)v <= lo) return 0;
  if ((uint64_t)(int64_t)v - (uint64_t)lo >= (uint64_t)nbins) return nbins - 1;
  return (int)((uint64_t)(int64_t)v - (uint64_t)lo);
}

template <typename S>
__global__ __launch_bounds__(256) void histogram_kernel(const S* __restrict__ sym, int64_t n,
                                                        int64_t lo, int32_t nbins,
                                                        unsigned long long* __restrict__ hist,
                                                        int use_lds) {
  extern __shared__ unsigned int bins[];
  const int tid = threadIdx.x;
  if (use_lds) {
    for (int i = tid; i < nbins; i += 256) bins[i] = 0;
    lds_barrier();
  }
  uint32_t hot[HIST_HOT_N];
#pragma unroll
  for (int k = 0; k < HIST_HOT_N; ++k) hot[k] = 0;
#if IVC_HIST_PACKED
  // the hot counts of the current iteration as 8 byte lanes of one 64-bit register (one
  // shift and one add per symbol instead of 8 compare-adds), unpacked into `hot` after every
  // iteration (<= 16 symbols per thread, far below a byte's 255)
  uint64_t pk = 0;
  auto unpack = [&]() {
#pragma unroll
    for (int k = 0; k < HIST_HOT_N; ++k) hot[k] += (uint32_t)(pk >> (8 * k)) & 0xffu;
    pk = 0;
  };
#endif
  auto count = [&](S v) {
    // unsigned difference: v - HIST_HOT_LO wraps instead of overflowing for v near INT64_MAX
    const uint64_t u = (uint64_t)(int64_t)v - (uint64_t)(int64_t)HIST_HOT_LO;
#if IVC_HIST_PACKED
    const bool h = u < (uint64_t)HIST_HOT_N;
    pk += h ? 1ull << (8u * ((uint32_t)u & 7u)) : 0ull;
    if (!h) {
#else
    if (u < (uint64_t)HIST_HOT_N) {
#pragma unroll
      for (int k = 0; k < HIST_HOT_N; ++k) hot[k] += u == (uint64_t)k ? 1u : 0u;
    } else {
#endif
      const int b = hist_bin(v, lo, nbins);
      if (use_lds) atomicAdd(&bins[b], 1u);
      else atomicAdd(&hist[b], 1ull);
    }
  };
#if !IVC_HIST_PACKED
  auto unpack = [&]() {};
#endif
  // a stream that does not start on 16 B: the first `head` symbols apart
  constexpr int PER = 16 / (int)sizeof(S);
  int64_t head = (int64_t)(((16u - ((uintptr_t)sym & 15u)) & 15u) / sizeof(S));
  if (head > n) head = n;
  if (blockIdx.x == 0 && tid < head) count(sym[tid]);
  unpack();
  sym += head;
  n -= head;
  // 16 B per lane, HIST_UNROLL loads in flight per iteration (the stream is read once)
  typedef S vec_t __attribute__((ext_vector_type(PER)));
  const vec_t* sv = reinterpret_cast<const vec_t*>(sym);
  const int64_t nv = n / PER, stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + tid;
  for (; i + (HIST_UNROLL - 1) * stride < nv; i += HIST_UNROLL * stride) {
    vec_t x[HIST_UNROLL];
#pragma unroll
    for (int u = 0; u < HIST_UNROLL; ++u) x[u] = __builtin_nontemporal_load(sv + i + u * stride);
#pragma unroll
    for (int u = 0; u < HIST_UNROLL; ++u)
#pragma unroll
      for (int k = 0; k < PER; ++k) count(x[u][k]);
    unpack();
  }
  for (; i < nv; i += stride) {
    const vec_t a = __builtin_nontemporal_load(sv + i);
#pragma unroll
    for (int k = 0; k < PER; ++k) count(a[k]);
    unpack();
  }
  if (blockIdx.x == 0 && tid < (int)(n - nv * PER)) count(sym[nv * PER + tid]);
  unpack();
  // hot counters: wave sums, added by lane 0 to the (clamped) bin of each hot value
#pragma unroll
  for (int k = 0; k < HIST_HOT_N; ++k) {
    uint32_t c = hot[k];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
    hot[k] = c;
  }
  if ((tid & 63) == 0) {
#pragma unroll
    for (int k = 0; k < HIST_HOT_N; ++k) {
      if (!hot[k]) continue;
      const int b = hist_bin((S)(HIST_HOT_LO + k), lo, nbins);
      if (use_lds) atomicAdd(&bins[b], hot[k]);
      else atomicAdd(&hist[b], (unsigned long long)hot[k]);
    }
  }
  if (use_lds) {
    lds_barrier();
    for (int i2 = tid; i2 < nbins; i2 += 256)
      if (bins[i2]) atomicAdd(&hist[i2], (unsigned long long)bins[i2]);
  }
}

// workgroups per CU of the histogram launches: 4 fills the chip (the stream alone is
// HBM-bound); fewer leave LDS and wave slots to kernels on other streams.  Process-wide
// (every device, every thread, every histogram launch incl. intra_encode's fused one);
// atomic so a set on one thread never races a launch reading it on another
static std::atomic<int> g_hist_wg_per_cu{4};
int histogram_wg_per_cu() { return g_hist_wg_per_cu.load(std::memory_order_relaxed); }
void set_histogram_wg_per_cu(int k) { g_hist_wg_per_cu.store(k > 0 ? k : 4, std::memory_order_relaxed); }

template <typename S>
static hipError_t launch_hist(const S* sym, int64_t n, int64_t lo, int32_t nbins, int64_t* hist,
                              hipStream_t s) {
  if (n <= 0 || nbins <= 0) return hipSuccess;
  const int use_lds = nbins <= 16384;
  const size_t lds = use_lds ? (size_t)nbins * 4 : 0;
  histogram_kernel<S><<<grid_for(n, 256 * 16, histogram_wg_per_cu()), 256, lds, s>>>(
      sym, n, lo, nbins, reinterpret_cast<unsigned long long*>(hist), use_lds);
  return hipGetLastError();
}

hipError_t launch_histogram(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins,
                            int64_t* hist, hipStream_t s) {
  return launch_hist<int32_t>(sym, n, lo, nbins, hist, s);
}

hipError_t launch_histogram_i64(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins,
                                int64_t* hist, hipStream_t s) {
  return launch_hist<int64_t>(sym, n, lo, nbins, hist, s);
}

}  // namespace ivc
