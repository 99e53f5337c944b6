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

#include <cstdlib>

#include "ivc_internal.h"

namespace ivc {

// S2 scratch: stream-ordered (scratch_alloc / hipFreeAsync on the launch stream), so
// concurrent streams never share it.
static int32_t* me_s2_alloc(int64_t elems, hipStream_t s) {
  void* p = nullptr;
  if (scratch_alloc(&p, (size_t)elems * 4, s) != hipSuccess) return nullptr;
  return (int32_t*)p;
}

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
    lds_barrier();
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
    lds_barrier();
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
      lds_barrier();
    }
    if (tid == 0) mv[blk] = sidx[0] == 0x7fffffff ? (int64_t)sr * n + sr : (int64_t)sidx[0];
    lds_barrier();
  }
}

// ---------------------------------------------------------------- float search -------
// NumPy semantics for float32 / float64 frames (the ME VideoCodec runs on its non-integer
// float64 luma, videocodec.py:38,52): every candidate's SSD in the reference's rounding order
// (np.sum's pairwise order over the 64 contiguous squares: column sums down the rows, then
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))), no fused multiply-add.
//
// A 512-thread workgroup takes a round of NB horizontally adjacent blocks of one block row:
// the round's reference window (8 + 2sr rows x 8 NB + 2sr columns, zero outside the frame)
// and its blocks (column-major) are staged in LDS; thread (b, e) owns block b's candidate
// column dx = e - sr and walks its dy in runs of FLT_DY: per block column v it loads the
// FLT_DY + 7 window values of column e + v once (each serves up to 8 candidates) and the
// block's column v, and folds each candidate's column sum into its pairwise tree (three
// partial sums live per candidate).  Lanes of neighbouring blocks read the same window
// words (broadcast), and consecutive lanes consecutive words (conflict-free).  The block's
// (SSD, raster index) minimum over its 2sr+1 threads: an LDS atomic minimum of the SSD bits
// (non-negative doubles order like their bits), a barrier, then the minimum index among the
// threads holding that SSD — the reference's first strict minimum.
template <typename T> struct FltBits;
template <> struct FltBits<double> {
  typedef unsigned long long U;
  __device__ static U bits(double v) { return (U)__double_as_longlong(v); }
};
template <> struct FltBits<float> {
  typedef unsigned int U;
  __device__ static U bits(float v) { return (U)__float_as_uint(v); }
};


// An empty asm that takes the FLT_DY partial sums in and out (so they are computed before
// it) and clobbers memory (so no LDS load moves above it).
template <typename T>
__device__ __forceinline__ void flt_pin(T (&a)[FLT_DY]) {
  static_assert(FLT_DY == 11 || FLT_DY == 6, "flt_pin lists FLT_DY operands");
  if constexpr (FLT_DY == 11)
    __asm__ volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                     "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]) :: "memory");
  else
    __asm__ volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5])
                     :: "memory");
}

// list (optional): rounds to search, list[0] = their count, list[1..] = round indices (the
// rounds the pruned float64 search deferred, below); null = every round of the batch
template <typename T, int SR>
__global__ __launch_bounds__(FLT_WG, sizeof(T) == 8 ? 2 : 4) void me_flt_kernel(const T* __restrict__ ref,
                                                           const T* __restrict__ cur,
                                                           int64_t nframes, int H, int W,
                                                           int64_t* __restrict__ mv,
                                                           const uint32_t* __restrict__ list) {
  typedef typename FltBits<T>::U U;
  typedef FltGeom<T, SR> G;
  extern __shared__ __attribute__((aligned(16))) unsigned char flt_smem[];
  constexpr int sr = SR, n = G::N, nbr = G::NBR, WR = G::WR, WC = G::WC, WRP = G::WRP;
  const int h = H / 8, w = W / 8;
  T* win = reinterpret_cast<T*>(flt_smem);                // [WRP][WC]
  T* cb = win + WRP * WC;                                 // [nbr][v][u], pitch CBP
  U* kmin = reinterpret_cast<U*>(cb + nbr * G::CBP);      // [nbr]
  unsigned* imin = reinterpret_cast<unsigned*>(kmin + nbr);
  const int segs = (w + nbr - 1) / nbr;
  const int64_t rounds = list ? (int64_t)list[0] : nframes * h * segs;
  const int tid = threadIdx.x;
  const int sb = tid / n, se = tid - sb * n;              // block of the round, candidate column
  for (int64_t ri = blockIdx.x; ri < rounds; ri += gridDim.x) {
    const int64_t r = list ? (int64_t)list[1 + ri] : ri;
    const int64_t f = r / ((int64_t)h * segs);
    const int rem = (int)(r - f * h * segs), by = rem / segs, bx0 = (rem - by * segs) * nbr;
    const int nb = w - bx0 < nbr ? w - bx0 : nbr;
    const T* rf = ref + f * (int64_t)H * W;
    const T* cf = cur + f * (int64_t)H * W;
    const int y0 = 8 * by - sr, x0 = 8 * bx0 - sr, wc = nb * 8 + 2 * sr;
    for (int i = tid; i < WRP * wc; i += FLT_WG) {
      const int yy = i / wc, xx = i - yy * wc, gy = y0 + yy, gx = x0 + xx;
      win[yy * WC + xx] = (yy < WR && gy >= 0 && gy < H && gx >= 0 && gx < W)
                              ? rf[(int64_t)gy * W + gx] : T(0);
    }
    for (int i = tid; i < nb * 64; i += FLT_WG) {
      const int b = i >> 6, u = (i >> 3) & 7, v = i & 7;
      cb[b * G::CBP + v * 8 + u] = cf[(int64_t)(8 * by + u) * W + 8 * (bx0 + b) + v];
    }
    for (int i = tid; i < nb; i += FLT_WG) {
      kmin[i] = ~(U)0;
      imin[i] = ~0u;
    }
    lds_barrier();
    T best = T(0);
    int bidx = -1;
    const int rx = 8 * (bx0 + sb) + se - sr;
    if (sb < nb && rx >= 0 && rx + 8 <= W) {
      const T* cblk = cb + sb * G::CBP;
#pragma unroll 1
      for (int dy0 = 0; dy0 < n; dy0 += FLT_DY) {
        T ta[FLT_DY], tb[FLT_DY], tc[FLT_DY];
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          T cv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) cv[u] = cblk[v * 8 + u];
          const T* col = win + dy0 * WC + sb * 8 + se + v;
          T rv[FLT_DY + 7];
#pragma unroll
          for (int k = 0; k < FLT_DY + 7; ++k) rv[k] = col[k * WC];
#pragma unroll
          for (int k = 0; k < FLT_DY; ++k) {
            T d = cv[0] - rv[k];
            T sk = d * d;
#pragma unroll
            for (int u = 1; u < 8; ++u) {
              d = cv[u] - rv[k + u];
              sk = sk + d * d;
            }
            // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
            if (v == 0) ta[k] = sk;
            if (v == 1) ta[k] = ta[k] + sk;
            if (v == 2 || v == 4) tb[k] = sk;
            if (v == 3) ta[k] = ta[k] + (tb[k] + sk);
            if (v == 5) tb[k] = tb[k] + sk;
            if (v == 6) tc[k] = sk;
            if (v == 7) tb[k] = tb[k] + (tc[k] + sk);
          }
          // keep the schedule column by column: the partial sums are finished here, before
          // the next column's window loads (otherwise the compiler hoists every column's
          // loads to the top and spills)
          flt_pin<T>(ta);                      // live from column 0
          if (v >= 2) flt_pin<T>(tb);          // from column 2
          if (v == 6) flt_pin<T>(tc);          // columns 6-7 only
        }
#pragma unroll
        for (int k = 0; k < FLT_DY; ++k) {
          const int d = dy0 + k, ry = 8 * by + d - sr;
          const T tot = ta[k] + tb[k];
          // eligible: in frame and below the reference's initial float('inf'); first strict
          // minimum in raster order (dy ascending within the thread)
          if (d < n && ry >= 0 && ry + 8 <= H && tot < (T)INFINITY && (bidx < 0 || tot < best)) {
            best = tot;
            bidx = d * n + se;
          }
        }
      }
    }
    if (bidx >= 0) atomicMin(&kmin[sb], FltBits<T>::bits(best));
    lds_barrier();
    if (bidx >= 0 && FltBits<T>::bits(best) == kmin[sb]) atomicMin(&imin[sb], (unsigned)bidx);
    lds_barrier();
    if (tid < nb)
      mv[(f * h + by) * w + bx0 + tid] = imin[tid] == ~0u ? (int64_t)sr * n + sr : (int64_t)imin[tid];
    lds_barrier();
  }
}

template <typename T, int SR>
static void launch_me_flt_sr(const T* ref, const T* cur, int64_t nframes, int64_t H, int64_t W,
                             int64_t* mv, hipStream_t s) {
  typedef FltGeom<T, SR> G;
  const int w = (int)(W / 8), h = (int)(H / 8);
  const int64_t rounds = nframes * h * ((w + G::NBR - 1) / G::NBR);
  const size_t lds = G::LDS;
  if constexpr (sizeof(T) == 8) {
    // the pruned search, then me_flt_kernel on the rounds it deferred (launches of < 2^31
    // rounds: 32-bit round indices in the list)
    const int mode = tuning(IVC_TUNE_F64_ME);      // ivc_set_tuning: 1 unpruned, 2 defer all
    if (rounds > 0 && mode != 1) {
      const int64_t rpf = (int64_t)h * ((w + G::NBR - 1) / G::NBR);          // rounds per frame
      const int64_t fmax = (((int64_t)1 << 31) - 1) / rpf;
      const int64_t chunk = nframes < fmax ? nframes : fmax;
      uint32_t* defer = nullptr;
      if (scratch_alloc((void**)&defer, (size_t)(chunk * rpf + 1) * 4, s) == hipSuccess) {
        const int64_t HW = H * W;
        for (int64_t f0 = 0; f0 < nframes; f0 += chunk) {
          const int64_t nf = nframes - f0 < chunk ? nframes - f0 : chunk;
          (void)hipMemsetAsync(defer, 0, 4, s);
          const int64_t nr = nf * rpf;
          launch_me_f64p(SR, (const double*)ref + f0 * HW, (const double*)cur + f0 * HW, nf, (int)H,
                         (int)W, mv + f0 * h * w, defer, mode == 2, s);
          me_flt_kernel<T, SR><<<me_grid(nr, 1, IVC_FLT_WGCU), FLT_WG, lds, s>>>(
              ref + f0 * HW, cur + f0 * HW, nf, (int)H, (int)W, mv + f0 * h * w, defer);
        }
        (void)hipFreeAsync(defer, s);
        return;
      }
      (void)hipGetLastError();                   // no scratch: the unpruned search
    }
  }
  // f64: 144 VGPRs, one 512-thread workgroup per CU; f32: two (88 VGPRs, LDS permitting)
  const unsigned grid = me_grid(rounds, 1, sizeof(T) == 4 && lds * 2 <= 160 * 1024 ? 2 : IVC_FLT_WGCU);
  me_flt_kernel<T, SR><<<grid, FLT_WG, lds, s>>>(ref, cur, nframes, (int)H, (int)W, mv, nullptr);
}

// The float search for the search ranges it is compiled for (window geometry is static, so
// every LDS offset is an immediate); false sends the caller to the generic kernel.
template <typename T>
static bool launch_me_flt(const T* ref, const T* cur, int64_t nframes, int64_t H, int64_t W,
                          int sr, int64_t* mv, hipStream_t s) {
  if (H < 8 || W < 8) return false;
  switch (sr) {
    case 4: launch_me_flt_sr<T, 4>(ref, cur, nframes, H, W, mv, s); return true;
    case 8: launch_me_flt_sr<T, 8>(ref, cur, nframes, H, W, mv, s); return true;
    case 16: launch_me_flt_sr<T, 16>(ref, cur, nframes, H, W, mv, s); return true;
    default: return false;
  }
}

// ---------------------------------------------------------------- fast exact u8 search
// Integer-valued u8 frames (IVC_ME_EXACT_U8 — the reference run on frame.astype(float64),
// videocodec.py:38), search range SR in {4, 8, 16}.
//   SSD(b, d) = sum(c^2) + S2(d) - 2 X(b, d),  S2(d) = sum of r^2 over the window,
//   X(b, d)   = sum c*r  (v_dot4_u32_u8: 4 byte MACs per instruction).
// sum(c^2) is constant per block, so K = S2 - 2X orders the candidates exactly like the SSD
// (every term is an exact integer < 2^24): same minimum, same ties, same raster tie-break.
//
// S2 comes from a box-filter pre-pass over each reference frame (me_s2_kernel).  The search
// is wave-independent: a wave owns BPW adjacent blocks; lane (block, g, dr) evaluates the
// DYT x 4 candidates dy in [dr*DYT, dr*DYT + DYT) x dx in [4g, 4g + 4) of its block.  The
// blocks' reference windows are staged in a wave-private LDS region (no barrier), the next
// group's windows are prefetched into registers while the current one is searched, the
// 4 byte-shifts of a ref row come from v_alignbyte and serve all of the lane's dy, and the
// lexicographic (K, raster index) minimum is reduced across the block's lanes with
// shuffles.

// S2[f][y][x] = sum of squares of the 8x8 window with top-left (y, x), for y <= H-8, x <= W-8.
// Thread = 4 consecutive x of one frame and a run of S2Y output rows: the horizontal
// 8-sums of r^2 come from dot4 on byte-shifted dwords, the vertical 8-sum slides down the
// run with the last 8 horizontal sums kept in registers.
constexpr int S2Y = 64;

__device__ __forceinline__ void s2_hrow(__amdgpu_buffer_rsrc_t rs, int off, uint32_t* hs) {
  const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
  const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4, 0, 0);
  const uint32_t w2 = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 8, 0, 0);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint32_t lo = s == 0 ? w0 : __builtin_amdgcn_alignbyte(w1, w0, s);
    const uint32_t hi = s == 0 ? w1 : __builtin_amdgcn_alignbyte(w2, w1, s);
    hs[s] = __builtin_amdgcn_udot4(hi, hi, __builtin_amdgcn_udot4(lo, lo, 0u, false), false);
  }
}

__global__ __launch_bounds__(256) void me_s2_kernel(const uint8_t* __restrict__ ref,
                                                    int64_t nframes, int H, int W,
                                                    int32_t* __restrict__ s2) {
  const int nx = (W - 8) / 4 + 1;                  // x groups covering x = 0 .. W-8
  const int ny = (H - 8) / S2Y + 1;                // row runs covering y = 0 .. H-8
  const int64_t total = nframes * (int64_t)nx * ny;
  const int64_t HW = (int64_t)H * W;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int xg = (int)(i % nx);
    const int64_t t = i / nx;
    const int yr = (int)(t % ny);
    const int64_t f = t / ny;
    const int x = 4 * xg, y0 = yr * S2Y;
    const int y1 = min(y0 + S2Y, H - 7);          // exclusive
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(ref + f * HW), 0, (int)HW, 0x00020000);
    int32_t* out = s2 + f * HW + x;
    const int nvalid = min(4, W - 7 - x);         // outputs of this group inside the row
    uint32_t h[8][4];
    uint32_t acc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s2_hrow(rs, (y0 + k) * W + x, h[k]);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[s] += h[k][s];
    }
    for (int y = y0; y < y1; y += 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int yy = y + k;
        if (yy < y1) {
          if (nvalid == 4) {
            // 16-byte aligned: x and W are multiples of 4 and 8
            *reinterpret_cast<int4*>(out + (int64_t)yy * W) =
                make_int4((int)acc[0], (int)acc[1], (int)acc[2], (int)acc[3]);
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
              if (s < nvalid) out[(int64_t)yy * W + s] = (int32_t)acc[s];
          }
          if (yy + 1 < y1) {                       // slide: drop row yy, add row yy + 8
            uint32_t hn[4];
            s2_hrow(rs, (yy + 8) * W + x, hn);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              acc[s] += hn[s] - h[k][s];
              h[k][s] = hn[s];
            }
          }
        }
      }
    }
  }
}

static unsigned me_fast_grid(const void* kernel, int64_t wgs) {
  const int64_t g = 2 * (int64_t)resident_grid_ptr(kernel, wgs);
  return (unsigned)(g < wgs ? g : wgs);
}

#ifndef IVC_ME_XCD
#define IVC_ME_XCD 1
#endif
#ifndef IVC_ME_CHUNK_BYTES
#define IVC_ME_CHUNK_BYTES (256LL << 20)   // S2 scratch per chunk of frame pairs
#endif

template <int SR> struct MeCfg;
// PITCH: LDS row pitch of a staged window (dwords), chosen so a row read of a 32-lane half
// hits distinct banks (searched offline; SR = 4 is 2-way at best with 4 blocks per wave)
template <> struct MeCfg<8> { static constexpr int BPW = 2, NDR = 6, DYT = 3, PITCH = 9; };   // 30 of 32 lanes
template <> struct MeCfg<4> { static constexpr int BPW = 4, NDR = 5, DYT = 2, PITCH = 5; };   // 15 of 16 lanes

typedef unsigned int me_u32x4 __attribute__((ext_vector_type(4)));

template <int DYT> __device__ __forceinline__ void row_fence(uint32_t (&acc)[DYT][4]);
template <> __device__ __forceinline__ void row_fence<3>(uint32_t (&a)[3][4]) {
  asm volatile("" : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[0][2]), "+v"(a[0][3]), "+v"(a[1][0]),
               "+v"(a[1][1]), "+v"(a[1][2]), "+v"(a[1][3]), "+v"(a[2][0]), "+v"(a[2][1]),
               "+v"(a[2][2]), "+v"(a[2][3]) :: "memory");
}
template <> __device__ __forceinline__ void row_fence<2>(uint32_t (&a)[2][4]) {
  asm volatile("" : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[0][2]), "+v"(a[0][3]), "+v"(a[1][0]),
               "+v"(a[1][1]), "+v"(a[1][2]), "+v"(a[1][3]) :: "memory");
}

template <int SR>
__global__ __launch_bounds__(256) void me_fast_u8_kernel(const uint8_t* __restrict__ ref,
                                                         const uint8_t* __restrict__ cur,
                                                         const int32_t* __restrict__ s2,
                                                         int64_t nframes, int H, int W,
                                                         int64_t* __restrict__ mv) {
  typedef MeCfg<SR> Cfg;
  constexpr int N = 2 * SR + 1;             // candidates per axis
  constexpr int NGX = (N + 3) / 4;          // dx groups of 4
  constexpr int BPW = Cfg::BPW, NDR = Cfg::NDR, DYT = Cfg::DYT;
  constexpr int SEG = 64 / BPW;             // lanes per block (aligned segment)
  constexpr int LPB = NGX * NDR;            // active lanes per block
  constexpr int NW = NGX + 2;               // window width in dwords (>= 8 + 2SR bytes + 3)
  constexpr int WR = 8 + 2 * SR;            // window rows
  constexpr int WIN = WR * NW;              // window dwords fetched per block
  constexpr int P = Cfg::PITCH;             // LDS row pitch (>= NW)
  // rows a lane reads: dy0 + 0 .. dy0 + DYT + 6 for dy0 up to (NDR - 1) DYT; rows past the
  // window (only for candidates dy >= N, masked at selection) read unwritten LDS instead of
  // being tested and zeroed per row
  constexpr int ROWS = WR > NDR * DYT + 7 ? WR : NDR * DYT + 7;
  constexpr int WINL = ROWS * P;            // LDS dwords per block window
  constexpr int PW = (BPW * WIN + 63) / 64; // window dwords staged per lane
  constexpr int CUR = BPW * 16;             // cur dwords per group (<= 64)
  constexpr int STAGE = BPW * WINL + CUR;
  static_assert(P >= NW, "pitch");
  static_assert(LPB <= SEG && CUR <= 64, "lanes");
  static_assert(NDR * DYT >= N, "dy coverage");
  static_assert(SR % 4 == 0, "window start must be dword aligned");
  __shared__ uint32_t lds[4 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  uint32_t* st = lds + wave * STAGE;
  const int h = H / 8, w = W / 8;
  const int gpr = (w + BPW - 1) / BPW;                   // block groups per block row
  const uint32_t gpf = (uint32_t)(h * gpr);
  const uint32_t ngroups = (uint32_t)nframes * gpf;
  const uint32_t nwaves = gridDim.x * 4u;
  const int64_t HW = (int64_t)H * W;
  // lane role: block lb on lanes [lb*SEG, lb*SEG + LPB), lane lr -> (dx group g, dy range dr)
  const int lb = lane / SEG, lr = lane - lb * SEG;
  const int g = lr % NGX, dr = lr / NGX;
  const bool active = lr < LPB;

  // window dwords (block-major) then the BPW current blocks (8 rows x 2 dwords each)
  auto fetch = [&](uint32_t grp, bool exists, uint32_t* wreg, uint32_t& creg) {
    const uint32_t gg = exists ? grp : 0u;
    const uint32_t f = gg / gpf;
    const uint32_t rem = gg - f * gpf;
    const int by = (int)(rem / (uint32_t)gpr);
    const int bx0 = (int)(rem - (uint32_t)by * gpr) * BPW;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(ref + (int64_t)f * HW), 0, exists ? (int)HW : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(cur + (int64_t)f * HW), 0, exists ? (int)HW : 0, 0x00020000);
    // wave-uniform: every window of the group lies inside the frame (no per-dword checks)
    const bool inner = 8 * by >= SR && 8 * by + 8 + SR <= H && 8 * bx0 >= SR &&
                       8 * (bx0 + BPW) + SR <= W;
    const int oy = 8 * by - SR, ox = 8 * bx0 - SR;
    if (inner) {
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const int e = lane + 64 * j;
        const int blk = e / WIN, o = e - blk * WIN;
        const int row = o / NW, dw = o - row * NW;
        const bool ok = (64 * j + 63 < BPW * WIN) || e < BPW * WIN;
        wreg[j] = __builtin_amdgcn_raw_buffer_load_b32(
            rr, ok ? (oy + row) * W + ox + 8 * blk + 4 * dw : 0x40000000, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const int e = lane + 64 * j;
        const int blk = e / WIN, o = e - blk * WIN;
        const int row = o / NW, dw = o - row * NW;
        const int gy = oy + row, gx = ox + 8 * blk + 4 * dw;
        const bool ok = e < BPW * WIN && bx0 + blk < w && gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W;
        wreg[j] = __builtin_amdgcn_raw_buffer_load_b32(rr, ok ? gy * W + gx : 0x40000000, 0, 0);
      }
    }
    const int blk = lane >> 4, c = lane & 15;
    const bool okc = lane < CUR && bx0 + blk < w;
    creg = __builtin_amdgcn_raw_buffer_load_b32(
        rc, okc ? (8 * by + (c >> 1)) * W + 8 * (bx0 + blk) + 4 * (c & 1) : 0x40000000, 0, 0);
  };

  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share
  // one), so logical workgroup (b % 8) * (G / 8) + b / 8 gives each XCD a contiguous run of
  // groups: adjacent blocks, whose windows and S2 rows overlap, then share one L2
  uint32_t wg = blockIdx.x;
  if (IVC_ME_XCD && (gridDim.x & 7u) == 0u) wg = (wg & 7u) * (gridDim.x >> 3) + (wg >> 3);
  uint32_t grp = wg * 4u + wave;
  uint32_t wraw[PW], craw;
  fetch(grp, grp < ngroups, wraw, craw);
  for (; grp < ngroups; grp += nwaves) {
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int e = lane + 64 * j;
      const int blk = e / WIN, o = e - blk * WIN, row = o / NW;
      if (e < BPW * WIN) st[blk * WINL + row * P + (o - row * NW)] = wraw[j];
    }
    if (lane < CUR) st[BPW * WINL + lane] = craw;
    __builtin_amdgcn_wave_barrier();
    const uint32_t ng = grp + nwaves;
    fetch(ng, ng < ngroups, wraw, craw);                   // prefetch the next group

    const uint32_t f = grp / gpf;
    const uint32_t rem = grp - f * gpf;
    const int by = (int)(rem / (uint32_t)gpr);
    const int bx = (int)(rem - (uint32_t)by * gpr) * BPW + lb;
    int bestk = 0x7fffffff, besti = 0x7fffffff;
    if (active && bx < w) {
      const uint32_t* win = st + lb * WINL;
      const uint32_t* cb = st + BPW * WINL + lb * 16;
      uint32_t cw[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) cw[k] = cb[k];
      uint32_t acc[DYT][4];
#pragma unroll
      for (int d = 0; d < DYT; ++d)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[d][s] = 0;
      const int dy0 = dr * DYT;
      // row words are read one row ahead of their use (the fence below would otherwise
      // expose the LDS latency once per row)
      auto row_words = [&](int row, uint32_t& a0, uint32_t& a1, uint32_t& a2) {
        const uint32_t* p = win + row * P + g;
        a0 = p[0]; a1 = p[1]; a2 = p[2];
      };
      uint32_t w0, w1, w2;
      row_words(dy0, w0, w1, w2);
#pragma unroll
      for (int rr = 0; rr < DYT + 7; ++rr) {
        uint32_t n0 = 0u, n1 = 0u, n2 = 0u;
        if (rr + 1 < DYT + 7) row_words(dy0 + rr + 1, n0, n1, n2);
        uint32_t lo[4], hi[4];
        lo[0] = w0; hi[0] = w1;
#pragma unroll
        for (int s = 1; s < 4; ++s) {
          lo[s] = __builtin_amdgcn_alignbyte(w1, w0, s);
          hi[s] = __builtin_amdgcn_alignbyte(w2, w1, s);
        }
#pragma unroll
        for (int d = 0; d < DYT; ++d) {
          const int u = rr - d;                          // block row matched by this ref row
          if (u >= 0 && u < 8) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              acc[d][s] = __builtin_amdgcn_udot4(lo[s], cw[2 * u], acc[d][s], false);
              acc[d][s] = __builtin_amdgcn_udot4(hi[s], cw[2 * u + 1], acc[d][s], false);
            }
          }
        }
        // keep the schedule row by row: the compiler otherwise hoists every row's LDS reads
        // and byte shifts ahead of the dot products (~100 more live registers, 3 waves per
        // SIMD instead of 6); the empty asm pins the row's accumulators and orders memory
        row_fence<DYT>(acc);
        w0 = n0; w1 = n1; w2 = n2;
      }
      // the lane's candidates in raster order (dy outer, dx inner): first strict minimum.
      // K = S2 - 2X lies in [-64*255^2, 64*255^2] (SSD = K + sum c^2 >= 0), so
      // 32 (K + 2^22) + (raster rank within the lane, < 32) is a positive int32 key whose
      // minimum is the lane's first strict minimum: one v_min per candidate
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(s2 + (int64_t)f * HW), 0, (int)(HW * 4), 0x00020000);
      const int ry0 = 8 * by + dy0 - SR, rx0 = 8 * bx + 4 * g - SR;
      bool vx[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) vx[s] = 4 * g + s < N && rx0 + s >= 0 && rx0 + s + 8 <= W;
      uint32_t best = 0xffffffffu;
#pragma unroll
      for (int d = 0; d < DYT; ++d) {
        const int ry = ry0 + d;
        const bool vy = dy0 + d < N && ry >= 0 && ry + 8 <= H;
        // rx0 is a multiple of 4, so rx0 < 0 means all four candidates are off-frame
        const me_u32x4 sq = __builtin_amdgcn_raw_buffer_load_b128(
            rs, vy && rx0 >= 0 ? (ry * W + rx0) * 4 : 0x40000000, 0, 0);
        const uint32_t sv[4] = {sq.x, sq.y, sq.z, sq.w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const uint32_t key = (sv[s] << 5) + ((1u << 27) + 4u * d + s) - (acc[d][s] << 6);
          best = vy && vx[s] ? min(best, key) : best;
        }
      }
      if (best != 0xffffffffu) {
        bestk = (int)(best >> 5);                          // K + 2^22 (same bias on every lane)
        const int r = (int)(best & 31u);
        besti = (dy0 + (r >> 2)) * N + 4 * g + (r & 3);
      }
    }
    // lexicographic (K, index) minimum over the block's aligned lane segment; lanes with no
    // candidate carry (INT_MAX, INT_MAX)
#pragma unroll
    for (int off = 1; off < SEG; off <<= 1) {
      const int ok_ = __shfl_xor(bestk, off), oi = __shfl_xor(besti, off);
      const bool take = ok_ < bestk || (ok_ == bestk && oi < besti);
      bestk = take ? ok_ : bestk;
      besti = take ? oi : besti;
    }
    if (lr == 0 && bx < w)
      mv[((int64_t)f * h + by) * w + bx] = besti == 0x7fffffff ? (int64_t)SR * N + SR : (int64_t)besti;
    __builtin_amdgcn_wave_barrier();
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
    // +-16: the matrix-core search (no S2 plane; the whole batch, chunked by the launcher)
    if (sr == 16 && launch_me_mfma16((const uint8_t*)ref, (const uint8_t*)cur, nframes, h, w, mv, s))
      return hipGetLastError();
    // +-4 / +-8: the dot4 search; it addresses a frame's S2 plane (4 B per pixel) with 32-bit
    // buffer offsets
    if ((sr == 4 || sr == 8) && H * W * 4 < ((int64_t)1 << 31)) {
      // Frame pairs go in chunks of about IVC_ME_CHUNK_BYTES of S2 (one int32 per reference
      // pixel, stream-ordered scratch; at least one frame): a chunk the size of the 256 MB
      // Infinity Cache is still cache-resident when the search reads it right after the
      // pre-pass wrote it
      const int64_t hw = H * W;
      int64_t chunk = (int64_t)IVC_ME_CHUNK_BYTES / (4 * hw);
      if (chunk < 1) chunk = 1;
      if (chunk > nframes) chunk = nframes;
      int32_t* s2 = me_s2_alloc(chunk * hw, s);
      if (!s2) return hipErrorOutOfMemory;
      for (int64_t f0 = 0; f0 < nframes; f0 += chunk) {
        const int64_t nf = nframes - f0 < chunk ? nframes - f0 : chunk;
        const uint8_t* rf = (const uint8_t*)ref + f0 * hw;
        const uint8_t* cf = (const uint8_t*)cur + f0 * hw;
        int64_t* mf = mv + f0 * (H / 8) * (W / 8);
        const unsigned s2grid = me_grid(nf * ((W - 8) / 4 + 1) * ((H - 8) / S2Y + 1), 256, 8);
        me_s2_kernel<<<s2grid, 256, 0, s>>>(rf, nf, h, w, s2);
        // persistent (group stride = all waves), launched at 2x what fits at once: the waves
        // of the second residency round fill the SIMDs as the first ones drain (measured
        // faster than an exactly resident grid, the kernel being VALU-throughput bound)
        const int64_t groups_bpw1 = nf * (H / 8) * (W / 8);
#define ME_FAST(R, BPW)                                                                       \
  me_fast_u8_kernel<R><<<me_fast_grid(reinterpret_cast<const void*>(me_fast_u8_kernel<R>),      \
                                      ((groups_bpw1 + BPW - 1) / BPW + 3) / 4),                 \
                         256, 0, s>>>(rf, cf, s2, nf, h, w, mf)
        if (sr == 4) ME_FAST(4, 4);
        else ME_FAST(8, 2);
#undef ME_FAST
      }
      (void)hipFreeAsync(s2, s);
      return hipGetLastError();
    }
    switch (sr) {
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
    case IVC_F32:
      if (!launch_me_flt<float>((const float*)ref, (const float*)cur, nframes, H, W, sr, mv, s))
        ME_LAUNCH(float, 0);
      break;
    case IVC_F64:
      if (!launch_me_flt<double>((const double*)ref, (const double*)cur, nframes, H, W, sr, mv, s))
        ME_LAUNCH(double, 0);
      break;
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
