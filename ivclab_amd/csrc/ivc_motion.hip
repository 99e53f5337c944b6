// ivc_motion.hip — full-search block matching and block-copy motion compensation (gfx950).
//
// Reference: /root/reference/ivclab/video/motion.py
//   compute_motion_vector          :8-58  candidates from ref (arg 1), blocks from cur (arg 2),
//                                         dy outer / dx inner in [-sr, sr], out-of-frame
//                                         candidates skipped (:41-43), SSD in the input dtype
//                                         (:46), first strict minimum (:48), index (:55)
//   reconstruct_with_motion_vector :60-97 block copy, zeros out of frame (:89-92)
//
// The scan order is a reduction here: each candidate's SSD is independent, and the first
// strict minimum of a raster scan equals the lexicographic minimum of (ssd, raster index)
// over the eligible candidates (valid, and for floats ssd < +inf, since the reference's
// running minimum starts at float('inf')).  So candidates can be evaluated in any order
// and combined with that key.
#include <type_traits>

#include "ivc_internal.h"

namespace ivc {

static int g_cus = 0;
static unsigned me_grid(int64_t items, int per_block, int max_per_cu) {
  if (g_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    g_cus = (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0)
                ? p.multiProcessorCount : 256;
  }
  int64_t g = (items + per_block - 1) / per_block, cap = (int64_t)g_cus * max_per_cu;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

// ---------------------------------------------------------------- SSD semantics -------
// MODE 0: NumPy semantics of T.  Integers: the subtraction and the square wrap to T's
// width, the 64 squares are summed exactly in int64 (signed T) / uint64 (unsigned T), as
// np.sum does.  Floats: pairwise order of np.sum over 64 contiguous elements.
// MODE 1: u8 storage, exact integer SSD (the float64 result on integer-valued frames).
template <typename T, int MODE, bool FLT = std::is_floating_point<T>::value>
struct Ssd;

template <typename T>
struct Ssd<T, 0, true> {
  typedef T acc;
  __device__ static acc run(const T* cb, const T* __restrict__ R, int64_t W) {
    T c[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      T d = cb[v] - R[v];
      c[v] = d * d;
    }
#pragma unroll
    for (int u = 1; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        T d = cb[u * 8 + v] - R[u * W + v];
        c[v] = c[v] + d * d;
      }
    return ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
  }
  __device__ static bool eligible(acc s) { return s < (acc)INFINITY; }
};

template <typename T>
struct Ssd<T, 0, false> {
  typedef typename std::make_unsigned<T>::type UT;
  typedef typename std::conditional<(sizeof(T) <= 4), uint32_t, uint64_t>::type WT;
  typedef typename std::conditional<std::is_signed<T>::value, int64_t, uint64_t>::type acc;
  __device__ static acc run(const T* cb, const T* __restrict__ R, int64_t W) {
    uint64_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const UT d = (UT)((WT)(UT)cb[u * 8 + v] - (WT)(UT)R[u * W + v]);
        const UT q = (UT)((WT)d * (WT)d);
        s += (uint64_t)(acc)(T)q;  // sign-extend signed squares, then wrap-add
      }
    return (acc)s;
  }
  __device__ static bool eligible(acc) { return true; }
};

template <>
struct Ssd<uint8_t, 1, false> {
  typedef int32_t acc;
  __device__ static acc run(const uint8_t* cb, const uint8_t* __restrict__ R, int64_t W) {
    int s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const int d = (int)cb[u * 8 + v] - (int)R[u * W + v];
        s += d * d;
      }
    return s;
  }
  __device__ static bool eligible(acc) { return true; }
};

// ---------------------------------------------------------------- generic search ------
// One 256-thread workgroup per 8x8 block; thread t evaluates candidates t, t+256, ... in
// raster order reading the reference window through the L1/L2 (neighbouring workgroups
// share windows); (ssd, index) minimum reduced through LDS.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void me_generic_kernel(const T* __restrict__ ref,
                                                         const T* __restrict__ cur,
                                                         int64_t nframes, int H, int W, int sr,
                                                         int64_t* __restrict__ mv) {
  typedef Ssd<T, MODE> S;
  typedef typename S::acc acc;
  __shared__ T cb[64];
  __shared__ acc sval[256];
  __shared__ int sidx[256];
  const int tid = threadIdx.x;
  const int h = H / 8, w = W / 8, n = 2 * sr + 1, nc = n * n;
  const int64_t nblk = nframes * h * w;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t f = blk / ((int64_t)h * w);
    const int rem = (int)(blk - f * h * w), by = rem / w, bx = rem - by * w;
    const int y = 8 * by, x = 8 * bx;
    const int64_t fo = f * (int64_t)H * W;
    if (tid < 64) cb[tid] = cur[fo + (int64_t)(y + (tid >> 3)) * W + x + (tid & 7)];
    __syncthreads();
    acc best = acc(0);
    int bidx = 0x7fffffff;
    for (int c = tid; c < nc; c += 256) {
      const int dy = c / n - sr, dx = c - (c / n) * n - sr;
      const int ry = y + dy, rx = x + dx;
      if (ry < 0 || ry + 8 > H || rx < 0 || rx + 8 > W) continue;
      const acc s = S::run(cb, ref + fo + (int64_t)ry * W + rx, W);
      if (!S::eligible(s)) continue;
      if (bidx == 0x7fffffff || s < best) { best = s; bidx = c; }
    }
    sval[tid] = best;
    sidx[tid] = bidx;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (tid < off) {
        const int ib = sidx[tid + off];
        if (ib != 0x7fffffff) {
          const int ia = sidx[tid];
          const acc vb = sval[tid + off], va = sval[tid];
          if (ia == 0x7fffffff || vb < va || (!(va < vb) && ib < ia)) {
            sval[tid] = vb;
            sidx[tid] = ib;
          }
        }
      }
      __syncthreads();
    }
    if (tid == 0) mv[blk] = sidx[0] == 0x7fffffff ? (int64_t)sr * n + sr : (int64_t)sidx[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- fast exact u8 search
// Integer-valued u8 frames (IVC_ME_EXACT_U8 — the reference run on frame.astype(float64),
// videocodec.py:38), search range SR in {4, 8, 16}.
//   SSD(b, d) = sum(c^2) + S2(d) - 2 X(b, d),  S2(d) = sum of r^2 over the window,
//   X(b, d)   = sum c*r  (v_dot4_u32_u8: 4 byte MACs per instruction).
// sum(c^2) is constant per block, so K = S2 - 2X orders the candidates exactly like the SSD
// (every term is an exact integer < 2^24): same minimum, same ties, same raster tie-break.
// A workgroup owns BX = 256 / (2SR+1) consecutive blocks of one block row; thread
// (b, dyi) evaluates the 2SR+1 dx candidates of one dy for block b.  The reference window
// of the workgroup sits in LDS as dwords; the 4 byte-shifts of each ref row are built
// with v_alignbyte and reused by the thread's 2SR+1 candidates.  S2 comes from LDS box
// sums (horizontal then vertical 8-sums of r^2).
template <int SR>
__global__ __launch_bounds__(256) void me_fast_u8_kernel(const uint8_t* __restrict__ ref,
                                                         const uint8_t* __restrict__ cur,
                                                         int64_t nframes, int H, int W,
                                                         int64_t* __restrict__ mv) {
  constexpr int N = 2 * SR + 1;             // candidates per axis
  constexpr int BX = 256 / N;               // blocks per workgroup
  constexpr int NGX = (N + 3) / 4;          // dx groups of 4
  constexpr int NW = NGX + 2;               // ref dwords a thread reads per row
  constexpr int RH = 8 + 2 * SR;            // ref region rows
  constexpr int RWD = 2 * BX + NW;          // ref region width in dwords (>= 8BX+2SR bytes)
  constexpr int NPOS = 8 * (BX - 1) + N;    // window x-positions per row
  static_assert(SR % 4 == 0, "region start must be dword aligned");
  __shared__ uint32_t sref[RH * RWD];
  __shared__ uint32_t scur[BX * 16];
  __shared__ int sh2[RH * NPOS];
  __shared__ int ss2[N * NPOS];
  __shared__ int sk[256];
  __shared__ int si[256];
  const int tid = threadIdx.x;
  const int h = H / 8, w = W / 8;
  const int tpr = (w + BX - 1) / BX;
  const int64_t ntiles = nframes * h * tpr;
  const int64_t HW = (int64_t)H * W;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t f = tile / ((int64_t)h * tpr);
    const int rem = (int)(tile - f * h * tpr);
    const int by = rem / tpr, bx0 = (rem - by * tpr) * BX;
    const int y0 = 8 * by - SR, x0 = 8 * bx0 - SR;
    const uint8_t* R = ref + f * HW;
    const uint8_t* Cf = cur + f * HW;
    // ---- stage the reference window (zeros outside the frame) and the current blocks ---
    for (int i = tid; i < RH * RWD; i += 256) {
      const int row = i / RWD, dw = i - row * RWD;
      const int gy = y0 + row, gx = x0 + 4 * dw;
      uint32_t v = 0;
      if (gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W)
        v = *reinterpret_cast<const uint32_t*>(R + (int64_t)gy * W + gx);
      sref[i] = v;
    }
    for (int i = tid; i < BX * 16; i += 256) {
      const int blk = i >> 4, row = (i >> 1) & 7, half = i & 1;
      const int bx = bx0 + blk;
      uint32_t v = 0;
      if (bx < w) v = *reinterpret_cast<const uint32_t*>(Cf + (int64_t)(8 * by + row) * W + 8 * bx + 4 * half);
      scur[i] = v;
    }
    __syncthreads();
    // ---- window sums of squares: horizontal 8-sums, then vertical ------------------------
    for (int i = tid; i < RH * NPOS; i += 256) {
      const int row = i / NPOS, c = i - row * NPOS;
      const uint32_t* rw = sref + row * RWD;
      const int d0 = c >> 2, sh = c & 3;
      const uint32_t lo = __builtin_amdgcn_alignbyte(rw[d0 + 1], rw[d0], sh);
      const uint32_t hi = __builtin_amdgcn_alignbyte(rw[d0 + 2], rw[d0 + 1], sh);
      sh2[i] = (int)__builtin_amdgcn_udot4(hi, hi, __builtin_amdgcn_udot4(lo, lo, 0u, false), false);
    }
    __syncthreads();
    for (int i = tid; i < N * NPOS; i += 256) {
      const int dyi = i / NPOS, c = i - dyi * NPOS;
      int sum = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += sh2[(dyi + u) * NPOS + c];
      ss2[i] = sum;
    }
    __syncthreads();
    // ---- cross terms: thread (b, dyi) over all dx ----------------------------------------
    int bestk = 0x7fffffff, besti = 0x7fffffff;
    const int b = tid / N, dyi = tid - b * N;
    const int bx = bx0 + b;
    if (b < BX && bx < w) {
      const int dy = dyi - SR;
      const bool vy = 8 * by + dy >= 0 && 8 * by + dy + 8 <= H;
      if (vy) {
        uint32_t cw[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) cw[k] = scur[b * 16 + k];
        uint32_t acc[NGX * 4];
#pragma unroll
        for (int k = 0; k < NGX * 4; ++k) acc[k] = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint32_t* rw = sref + (dyi + u) * RWD + 2 * b;
          uint32_t wv[NW];
#pragma unroll
          for (int j = 0; j < NW; ++j) wv[j] = rw[j];
#pragma unroll
          for (int g = 0; g < NGX; ++g) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const uint32_t lo = s == 0 ? wv[g] : __builtin_amdgcn_alignbyte(wv[g + 1], wv[g], s);
              const uint32_t hi = s == 0 ? wv[g + 1] : __builtin_amdgcn_alignbyte(wv[g + 2], wv[g + 1], s);
              acc[4 * g + s] = __builtin_amdgcn_udot4(lo, cw[2 * u], acc[4 * g + s], false);
              acc[4 * g + s] = __builtin_amdgcn_udot4(hi, cw[2 * u + 1], acc[4 * g + s], false);
            }
          }
        }
        const int* s2 = ss2 + dyi * NPOS + 8 * b;
#pragma unroll
        for (int dxi = 0; dxi < N; ++dxi) {
          const int dx = dxi - SR;
          const bool vx = 8 * bx + dx >= 0 && 8 * bx + dx + 8 <= W;
          const int k = s2[dxi] - 2 * (int)acc[dxi];
          const bool better = vx && k < bestk;
          bestk = better ? k : bestk;
          besti = better ? dyi * N + dxi : besti;
        }
      }
    }
    sk[tid] = bestk;
    si[tid] = besti;
    __syncthreads();
    if (tid < BX && bx0 + tid < w) {
      int bk = 0x7fffffff, bi = 0x7fffffff;
      for (int d = 0; d < N; ++d) {   // dy order: first strict minimum = lowest raster index
        const int i = si[tid * N + d];
        if (i != 0x7fffffff && (bi == 0x7fffffff || sk[tid * N + d] < bk)) { bk = sk[tid * N + d]; bi = i; }
      }
      mv[(f * h + by) * w + bx0 + tid] = bi == 0x7fffffff ? (int64_t)SR * N + SR : (int64_t)bi;
    }
    __syncthreads();
  }
}

hipError_t launch_motion_estimate(const void* ref, const void* cur, int dtype, int64_t nframes,
                                  int64_t H, int64_t W, int sr, int mode, int64_t* mv,
                                  hipStream_t s) {
  const int64_t nblk = nframes * (H / 8) * (W / 8);
  if (nblk <= 0) return hipSuccess;
  const unsigned grid = me_grid(nblk, 1, 8);
  const int h = (int)H, w = (int)W;
#define ME_LAUNCH(T, M) \
  me_generic_kernel<T, M><<<grid, 256, 0, s>>>((const T*)ref, (const T*)cur, nframes, h, w, sr, mv)
  if (mode == IVC_ME_EXACT_U8) {
    if (dtype != IVC_U8) return hipErrorInvalidValue;
    const int64_t rows = nframes * (H / 8);
    switch (sr) {
      case 4: me_fast_u8_kernel<4><<<me_grid(rows * ((W / 8 + 27) / 28), 1, 8), 256, 0, s>>>(
                  (const uint8_t*)ref, (const uint8_t*)cur, nframes, h, w, mv); break;
      case 8: me_fast_u8_kernel<8><<<me_grid(rows * ((W / 8 + 14) / 15), 1, 8), 256, 0, s>>>(
                  (const uint8_t*)ref, (const uint8_t*)cur, nframes, h, w, mv); break;
      case 16: me_fast_u8_kernel<16><<<me_grid(rows * ((W / 8 + 6) / 7), 1, 8), 256, 0, s>>>(
                  (const uint8_t*)ref, (const uint8_t*)cur, nframes, h, w, mv); break;
      default: ME_LAUNCH(uint8_t, 1); break;
    }
    return hipGetLastError();
  }
  if (mode != IVC_ME_NUMPY) return hipErrorInvalidValue;
  switch (dtype) {
    case IVC_U8: ME_LAUNCH(uint8_t, 0); break;
    case IVC_I8: ME_LAUNCH(int8_t, 0); break;
    case IVC_U16: ME_LAUNCH(uint16_t, 0); break;
    case IVC_I16: ME_LAUNCH(int16_t, 0); break;
    case IVC_U32: ME_LAUNCH(uint32_t, 0); break;
    case IVC_I32: ME_LAUNCH(int32_t, 0); break;
    case IVC_U64: ME_LAUNCH(uint64_t, 0); break;
    case IVC_I64: ME_LAUNCH(int64_t, 0); break;
    case IVC_F32: ME_LAUNCH(float, 0); break;
    case IVC_F64: ME_LAUNCH(double, 0); break;
    default: return hipErrorInvalidValue;
  }
#undef ME_LAUNCH
  return hipGetLastError();
}

// ---------------------------------------------------------------- compensation --------
template <typename E>
__global__ __launch_bounds__(256) void mc_kernel(const E* __restrict__ ref, int64_t nframes,
                                                 int H, int W, int C,
                                                 const int64_t* __restrict__ mv, int sr,
                                                 E* __restrict__ out) {
  const int64_t total = nframes * H * W * C;
  const int n = 2 * sr + 1, h = H / 8, w = W / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    int64_t t = i / C;
    const int c = (int)(i - t * C);
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const int64_t f = t / H;
    const int64_t m = mv[(f * h + (y >> 3)) * w + (x >> 3)];
    int64_t q = m / n, rm = m - q * n;  // Python floor division (motion.py:83-84)
    if (rm < 0) { rm += n; q -= 1; }
    const int64_t dy = q - sr, dx = rm - sr;
    const int64_t ry = (y & ~7) + dy, rx = (x & ~7) + dx;
    const bool in = ry >= 0 && ry + 8 <= H && rx >= 0 && rx + 8 <= W;
    out[i] = in ? ref[((f * H + y + dy) * W + x + dx) * C + c] : E(0);
  }
}

hipError_t launch_motion_compensate(const void* ref, int esize, int64_t nframes, int64_t H,
                                    int64_t W, int64_t C, const int64_t* mv, int sr, void* out,
                                    hipStream_t s) {
  const int64_t total = nframes * H * W * C;
  if (total <= 0) return hipSuccess;
  const unsigned grid = me_grid(total, 256, 16);
  const int h = (int)H, w = (int)W, c = (int)C;
  switch (esize) {
    case 1: mc_kernel<uint8_t><<<grid, 256, 0, s>>>((const uint8_t*)ref, nframes, h, w, c, mv, sr, (uint8_t*)out); break;
    case 2: mc_kernel<uint16_t><<<grid, 256, 0, s>>>((const uint16_t*)ref, nframes, h, w, c, mv, sr, (uint16_t*)out); break;
    case 4: mc_kernel<uint32_t><<<grid, 256, 0, s>>>((const uint32_t*)ref, nframes, h, w, c, mv, sr, (uint32_t*)out); break;
    case 8: mc_kernel<uint64_t><<<grid, 256, 0, s>>>((const uint64_t*)ref, nframes, h, w, c, mv, sr, (uint64_t*)out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ivc
