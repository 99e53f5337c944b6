// ivc_decode.hip — the decode half of IntraCodec on gfx950 (IntraCodec.symbols2image,
// ivclab/image/intracodec.py:84-146, after the zero-run decode):
//   ZigZag.unflatten            ivclab/utils/shape.py:30-36
//   PatchQuant.dequantize       ivclab/quantization/patchquant.py:62-78  (C = 1 broadcasts
//                               over the 3 table planes, int32 x table in float64, truncated)
//   DCT.inverse_transform       ivclab/signal/dct.py:30-46               (pocketfft DCT-III,
//                               ortho, rows then columns: ivc_math.h dct3_line)
//   rearrange 'hp wp c h w -> (hp h) (wp w) c'  (intracodec.py:124, the unpatch)
//   ycbcr2rgb                   ivclab/signal/color.py:40-63             (optional)
//
// One wave owns a group of 8 consecutive blocks (lane = 8 b + r: block b, row r, later column
// r), a private LDS region and no workgroup barrier in its loop.  A group's input (8 x C x 256
// B of int32) arrives as 16-byte buffer loads issued one group ahead, is staged in LDS, and
// each lane gathers its row in raster order (the zig-zag permutation is the gather's address
// pattern).  Per table plane: dequantise, DCT-III of the row, transpose through LDS, DCT-III of
// the column.  Output layouts:
//   DEC_BLOCKS  [nblk][3][8][8] float64 (= inverse_transform(dequantize(unflatten(q)))): each
//               plane is staged (8 x 512 B) and leaves as 16-byte stores;
//   DEC_IMAGE   [F][H][W][3] float64 (the unpatched image): a lane keeps its column of all 3
//               planes (24 doubles: pixel-interleaved output needs every plane), optionally
//               converts them to RGB in registers, and the group leaves two image rows at a
//               time (2 x nb x 192 contiguous bytes) through a 3 KB staging area.
// HBM per block: C x 256 B in, 1536 B out.  Stores are non-temporal (streamed output).
#include <algorithm>

#include "ivc_internal.h"
#include "ivc_math.h"

namespace ivc {

__constant__ int c_dec_zz_order[64] = IVC_ZZ_ORDER;

enum { DEC_BLOCKS = 0, DEC_IMAGE = 1 };

struct DecArgs {
  const int32_t* q;      // [nblk][C][64] int32, zig-zag or raster order inside each 64
  double* out;           // DEC_BLOCKS: [nblk][3][64]; DEC_IMAGE: [rows * 8][W][3]
  int64_t nblk;          // blocks (= F * h * w for DEC_IMAGE)
  int64_t ngroups;       // groups of <= 8 blocks (DEC_IMAGE: groups never cross a block row)
  int w, gpr;            // DEC_IMAGE: blocks per block row, groups per block row
  int64_t W3;            // DEC_IMAGE: doubles per image row (W * 3)
};

typedef unsigned int dec_u32x4 __attribute__((ext_vector_type(4)));

constexpr int DQ_PITCH = 68;     // int32 per staged block-plane (16-byte rows, shifted banks)
constexpr int DX_WAVE = 8 * 72;  // doubles per wave: transpose image [b][k pitch 9] / staging
#ifndef IVC_DEC_STORE_AUX
#define IVC_DEC_STORE_AUX 2      // nt: streamed output
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dec_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

struct DecGroup {
  int64_t blk0;   // first block (input order)
  int64_t row;    // DEC_IMAGE: block row over all frames (f * h + by)
  int bx0, nb;    // DEC_IMAGE: first block column; blocks in the group (1..8)
};

template <int OUTL>
__device__ __forceinline__ DecGroup dec_group(const DecArgs& a, int64_t g) {
  DecGroup G;
  if constexpr (OUTL == DEC_IMAGE) {
    G.row = g / a.gpr;
    const int gx = (int)(g - G.row * a.gpr);
    G.bx0 = gx * 8;
    G.nb = min(8, a.w - G.bx0);
    G.blk0 = G.row * a.w + G.bx0;
  } else {
    G.row = 0;
    G.bx0 = 0;
    G.blk0 = g * 8;
    G.nb = (int)min<int64_t>(8, a.nblk - G.blk0);
  }
  return G;
}

// the group's input as NCH 16-byte chunks per lane (chunk c = j * 64 + lane); a group that
// does not exist or a ragged group's missing blocks fall outside the descriptor (zeros)
template <int C, int OUTL>
__device__ __forceinline__ void dec_load(const DecArgs& a, int64_t g, int lane, dec_u32x4* v) {
  constexpr int NCH = 2 * C;
  uint32_t bytes = 0;
  const int32_t* base = a.q;
  if (g < a.ngroups) {
    const DecGroup G = dec_group<OUTL>(a, g);
    base = a.q + G.blk0 * (C * 64);
    bytes = (uint32_t)G.nb * (C * 256u);
  }
  const __amdgpu_buffer_rsrc_t rs = dec_rsrc(base, bytes);
#pragma unroll
  for (int j = 0; j < NCH; ++j)
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (j * 64 + lane) * 16, 0, 0);
}

template <int C, bool ZZ, int OUTL, bool RGB>
__global__ __launch_bounds__(256) void intra_decode_kernel(DecArgs a, QTab t) {
  static_assert(OUTL == DEC_IMAGE || !RGB, "RGB output needs the image layout");
  constexpr int QS = 8 * C * DQ_PITCH;
  constexpr int NCH = 2 * C;
  __shared__ __attribute__((aligned(16))) int32_t qs_all[4 * QS];
  __shared__ __attribute__((aligned(16))) double xs_all[4 * DX_WAVE];
  __shared__ double tq[192];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = lane >> 3, r = lane & 7;
  for (int i = tid; i < 192; i += 256) tq[i] = t.q[i];
  // raster positions gathered by this lane (row r of its block), as stored in the input
  uint32_t pos[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < 8; ++k)
    pos[k >> 2] |= (uint32_t)(ZZ ? c_dec_zz_order[r * 8 + k] : r * 8 + k) << (8 * (k & 3));
  __syncthreads();   // the table only: the loop never synchronises across waves

  int32_t* qs = qs_all + wave * QS;
  double* xs = xs_all + wave * DX_WAVE;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t g = (int64_t)blockIdx.x * 4 + wave;
  dec_u32x4 raw[NCH];
  dec_load<C, OUTL>(a, g, lane, raw);
  for (; g < a.ngroups; g += nw) {
    dec_u32x4 nxt[NCH];
    dec_load<C, OUTL>(a, g + nw, lane, nxt);
    const DecGroup G = dec_group<OUTL>(a, g);
    // stage the group's input: chunk c = block-plane c / 16, quad c % 16
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = j * 64 + lane;
      *reinterpret_cast<dec_u32x4*>(qs + (c >> 4) * DQ_PITCH + (c & 15) * 4) = raw[j];
    }
    __builtin_amdgcn_wave_barrier();
    double o[RGB || OUTL == DEC_IMAGE ? 3 : 1][8];
    int32_t qv[8];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if (C == 3 || p == 0) {
        const int32_t* qb = qs + (b * C + (C == 3 ? p : 0)) * DQ_PITCH;
#pragma unroll
        for (int k = 0; k < 8; ++k) qv[k] = qb[(pos[k >> 2] >> (8 * (k & 3))) & 0xff];
      }
      double x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)   // patchquant.py:77-78: int32 * table (float64), truncated
        x[k] = (double)np_to_i32<double>((double)qv[k] * tq[p * 64 + r * 8 + k]);
      dct3_line<double>(x, 0.25, true);                 // axis -1 (row r)
#pragma unroll
      for (int k = 0; k < 8; ++k) xs[b * 72 + r * 9 + k] = x[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = xs[b * 72 + i * 9 + r];
      __builtin_amdgcn_wave_barrier();
      dct3_line<double>(x, 0.25, true);                 // axis -2 (column r)
      if constexpr (OUTL == DEC_BLOCKS) {
        // plane p of the group's blocks: [b][i][r], 8 x 512 B, block b's plane at
        // out + ((blk0 + b) * 3 + p) * 64
#pragma unroll
        for (int i = 0; i < 8; ++i) xs[b * 64 + i * 8 + r] = x[i];
        __builtin_amdgcn_wave_barrier();
        const __amdgpu_buffer_rsrc_t ro = dec_rsrc(a.out + (G.blk0 * 3 + p) * 64, (uint32_t)G.nb * 1536u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = j * 64 + lane;                  // block c / 32, chunk c % 32
          const dec_u32x4 v = *reinterpret_cast<const dec_u32x4*>(xs + (c >> 5) * 64 + (c & 31) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(v, ro, (c >> 5) * 1536 + (c & 31) * 16, 0,
                                                 IVC_DEC_STORE_AUX);
        }
        __builtin_amdgcn_wave_barrier();
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[p][i] = x[i];
      }
    }
    if constexpr (OUTL == DEC_IMAGE) {
      if constexpr (RGB) {
        // color.py:40-63, elementwise in float64; np.clip(v, 0, 255) keeps NaN
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const double Y = o[0][i], Cb = o[1][i] - 128.0, Cr = o[2][i] - 128.0;
          double v[3];
          v[0] = Y + 1.402 * Cr;
          v[1] = (Y - 0.344136 * Cb) - 0.714136 * Cr;
          v[2] = Y + 1.772 * Cb;
#pragma unroll
          for (int c = 0; c < 3; ++c)
            o[c][i] = v[c] != v[c] ? v[c] : (v[c] < 0.0 ? 0.0 : (v[c] > 255.0 ? 255.0 : v[c]));
        }
      }
      // two image rows at a time: stage [ri][px = 8 b + r][p], then 16-byte stores of the
      // rows' nb * 192 contiguous bytes each
      const int nb12 = G.nb * 12;
      double* rowp = a.out + (G.row * 8) * a.W3 + (int64_t)G.bx0 * 24;
#pragma unroll
      for (int i0 = 0; i0 < 8; i0 += 2) {
#pragma unroll
        for (int ri = 0; ri < 2; ++ri)
#pragma unroll
          for (int p = 0; p < 3; ++p) xs[(ri * 64 + lane) * 3 + p] = o[p][i0 + ri];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int ri = 0; ri < 2; ++ri) {
          const __amdgpu_buffer_rsrc_t ro = dec_rsrc(rowp + (i0 + ri) * a.W3, (uint32_t)nb12 * 16u);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int c = j * 64 + lane;                // chunk of this row (96 at most)
            const dec_u32x4 v = *reinterpret_cast<const dec_u32x4*>(xs + ri * 192 + c * 2);
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, c < 96 ? c * 16 : 0x40000000, 0,
                                                   IVC_DEC_STORE_AUX);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j) raw[j] = nxt[j];
  }
}

template <int C, bool ZZ, int OUTL, bool RGB>
static hipError_t launch_dec(const DecArgs& a, const QTab& t, hipStream_t s) {
  auto k = intra_decode_kernel<C, ZZ, OUTL, RGB>;
  const unsigned grid = resident_grid_ptr(reinterpret_cast<const void*>(k), (a.ngroups + 3) / 4);
  k<<<grid, 256, 0, s>>>(a, t);
  return hipGetLastError();
}

// [nblk][3][64] int32 -> [nblk][3][8][8] float64 (ivc_intra_decode)
hipError_t launch_intra_decode(const int32_t* q, int64_t nblk, const QTab& t, int unzigzag,
                               double* out, hipStream_t s) {
  if (nblk <= 0) return hipSuccess;
  DecArgs a{};
  a.q = q;
  a.out = out;
  a.nblk = nblk;
  a.ngroups = (nblk + 7) / 8;
  return unzigzag ? launch_dec<3, true, DEC_BLOCKS, false>(a, t, s)
                  : launch_dec<3, false, DEC_BLOCKS, false>(a, t, s);
}

// [F][h][w][C][64] int32 -> [F][H][W][3] float64 image (+ ycbcr2rgb)
hipError_t launch_intra_decode_image(const int32_t* q, int64_t nframes, int64_t H, int64_t W,
                                     int C, const QTab& t, int unzigzag, int to_rgb, double* out,
                                     hipStream_t s) {
  if (nframes <= 0 || H <= 0 || W <= 0) return hipSuccess;
  if ((C != 1 && C != 3) || H % 8 || W % 8) return hipErrorInvalidValue;
  DecArgs a{};
  a.q = q;
  a.out = out;
  a.w = (int)(W / 8);
  a.gpr = (a.w + 7) / 8;
  a.nblk = nframes * (H / 8) * a.w;
  a.ngroups = nframes * (H / 8) * a.gpr;
  a.W3 = W * 3;
#define DEC_IMG(CC, ZZ)                                                        \
  return to_rgb ? launch_dec<CC, ZZ, DEC_IMAGE, true>(a, t, s)                 \
                : launch_dec<CC, ZZ, DEC_IMAGE, false>(a, t, s)
  if (C == 1) {
    if (unzigzag) { DEC_IMG(1, true); } else { DEC_IMG(1, false); }
  } else {
    if (unzigzag) { DEC_IMG(3, true); } else { DEC_IMG(3, false); }
  }
#undef DEC_IMG
}

}  // namespace ivc
