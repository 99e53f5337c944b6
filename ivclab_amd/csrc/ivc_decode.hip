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
#include <type_traits>

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
  const int* skip;       // optional: the kernel does nothing when *skip != 0
};

typedef unsigned int dec_u32x4 __attribute__((ext_vector_type(4)));

constexpr int DQ_PITCH = 68;     // int32 per staged block-plane (16-byte rows, shifted banks)
constexpr int DX_WAVE = 8 * 72;  // doubles per wave: transpose image [b][k pitch 9] / staging
#ifndef IVC_DEC_STORE_AUX
#define IVC_DEC_STORE_AUX 2      // nt: streamed output
#endif
#ifndef IVC_DEC_PAD_ZERO
#define IVC_DEC_PAD_ZERO 1       // sym_image_kernel: no per-symbol bound test (see the parse)
#endif
#ifndef IVC_DEC_FOLD16
#define IVC_DEC_FOLD16 1         // sym_image_kernel, DQ_INT: the 1/16 scaling folded into the table
#endif
// ablation builds only (tools/ab), bits: 1 = the image stores skipped (behind a runtime test the
// compiler cannot fold), 2 = sym_image_kernel's parse skipped (the staging stays zero)
#ifndef IVC_DEC_ABLATE
#define IVC_DEC_ABLATE 0
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

// Dequantise + IDCT (+ RGB) of one group staged in LDS (qs: block-plane b * C + p at
// qs + (b * C + p) * DQ_PITCH, zig-zag or raster order inside) and its output: DEC_BLOCKS
// [nblk][3][8][8] or DEC_IMAGE rows.  Shared by intra_decode_kernel (coefficients from HBM) and
// sym_image_kernel (coefficients expanded from the zero-run stream).
// DQ_FAST: |q * table| < 2^31 is known (int16 coefficients, finite |table| < 2^16, checked on
// the host), so NumPy's float64 -> int32 cast of the dequantised value is a truncation
// (v_trunc_f64) with no range handling.  DQ_INT: every table entry is moreover a positive
// integer, so q * table is an exact integer (no truncation) and never -0.0.
enum { DQ_GENERAL = 0, DQ_FAST = 1, DQ_INT = 2 };
template <int C, int OUTL, bool RGB, typename Q = int32_t, int QP = DQ_PITCH, int DQM = DQ_GENERAL>
__device__ __forceinline__ void dec_group_math(const DecArgs& a, const DecGroup& G,
                                               const Q* qs, double* xs, const double* tq,
                                               const uint32_t* pos, int b, int r, int lane) {
  double o[RGB || OUTL == DEC_IMAGE ? 3 : 1][8];
  int32_t qv[8];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    if (C == 3 || p == 0) {
      const Q* qb = qs + (b * C + (C == 3 ? p : 0)) * QP;
#pragma unroll
      for (int k = 0; k < 8; ++k) qv[k] = qb[(pos[k >> 2] >> (8 * (k & 3))) & 0xff];
    }
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // patchquant.py:77-78: int32 * table (float64), truncated
      if constexpr (DQM == DQ_INT)
        x[k] = (double)qv[k] * tq[p * 64 + r * 8 + k];
      else if constexpr (DQM == DQ_FAST)   // + 0.0: a truncated -0.x is -0.0, the int32 round trip gives +0.0
        x[k] = __builtin_trunc((double)qv[k] * tq[p * 64 + r * 8 + k]) + 0.0;
      else
        x[k] = (double)np_to_i32<double>((double)qv[k] * tq[p * 64 + r * 8 + k]);
    }
    // both passes' ortho factor 1/4 applied once at the end as 1/16: every step is a sum,
    // difference or product with a constant, exact under power-of-two scaling (the values
    // are far from the subnormal and overflow ranges), so the result is bit-identical
    dct3_line<double>(x, 1.0, true);                  // axis -1 (row r)
#pragma unroll
    for (int k = 0; k < 8; ++k) xs[b * 72 + r * 9 + k] = x[k];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xs[b * 72 + i * 9 + r];
    __builtin_amdgcn_wave_barrier();
    dct3_line<double>(x, 1.0, true);                  // axis -2 (column r)
    if constexpr (!(DQM == DQ_INT && IVC_DEC_FOLD16)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = x[i] * 0.0625;
    }
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
        // np.clip(v, 0, 255): the dequantised values are finite int32s, so v is finite (no
        // NaN case); min keeps -0.0 (np.clip keeps it too), negatives become +0.0
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double m = __builtin_fmin(v[c], 255.0);
          o[c][i] = m < 0.0 ? 0.0 : m;
        }
      }
    }
    const int nb12 = G.nb * 12;
    double* rowp = a.out + (G.row * 8) * a.W3 + (int64_t)G.bx0 * 24;
    // two image rows at a time: stage [ri][px = 8 b + r][p], then 16-byte stores of the
    // rows' nb * 192 contiguous bytes each
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
          if (!(IVC_DEC_ABLATE & 1) || a.W3 < 0)
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, c < 96 ? c * 16 : 0x40000000, 0,
                                                   IVC_DEC_STORE_AUX);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// raster positions gathered by lane (b, r): row r of its block, as stored in the staging
template <bool ZZ>
__device__ __forceinline__ void dec_gather_pos(int r, uint32_t* pos) {
  pos[0] = pos[1] = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    pos[k >> 2] |= (uint32_t)(ZZ ? c_dec_zz_order[r * 8 + k] : r * 8 + k) << (8 * (k & 3));
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
  if (a.skip && *a.skip) return;
  for (int i = tid; i < 192; i += 256) tq[i] = t.q[i];
  uint32_t pos[2];
  dec_gather_pos<ZZ>(r, pos);
  lds_barrier();   // the table only: the loop never synchronises across waves

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
    dec_group_math<C, OUTL, RGB>(a, G, qs, xs, tq, pos, b, r, lane);
#pragma unroll
    for (int j = 0; j < NCH; ++j) raw[j] = nxt[j];
  }
}

// ---- zero-run symbols -> image, fused (IntraCodec.symbols2image, intracodec.py:84-146 with
// zerorun.py:44-88 in front): for a well-formed stream (the fast decoder's conditions,
// ivc_entropy.hip), the coefficients never reach HBM.  A wave takes a group of 8 blocks of a
// block row — C x nb consecutive block-planes of the stream, starting at gstart[g] (found
// from the EOB bit mask by sym_locate_kernel) — and expands its symbols 64 at a time straight
// into the zeroed LDS staging of dec_group_math: lane j takes symbol j of the chunk; its slot
// type follows from the previous symbol (a run-length slot iff it is 0), its coefficient count
// (1 for a nonzero value, the run length for a 0, none for run-length and EOB slots) and its
// EOB flag are prefix-summed across the wave in one packed DPP scan, and each EOB lane records
// in LDS the offset at which the next block-plane starts, so a nonzero value lands at (its
// block-plane, offset - that block-plane's start).  Any violation (a block-plane past 64 coefficients, a
// group whose EOB count or bounds do not match) sets `fail`, and the general path (zero-run
// decode into coefficients + intra_decode_kernel, gated on the device) overwrites the image.
// HBM per pixel: the stream's ~6.8 B (cfg3: 4 B/symbol) + 24 B of RGB float64.
__device__ __forceinline__ int dec_wave_incl_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return v;
}
struct SymImageArgs {
  const int32_t* sym;
  int64_t n;
  int32_t eob;
  const int64_t* gstart;   // [ngroups + 1]: first symbol of each group (-1: not found)
  int* fail;
};

// A group's symbols (854 on average for the cfg3 stream, at most 24 x 97) are staged into the
// wave's LDS with all their 16-byte loads in flight at once — up to SYM_SEG symbols per round,
// in the region the IDCT's transpose uses afterwards — and parsed from there (a first version
// loaded 64 symbols per iteration, one HBM latency per chunk: 25 ms for the cfg3 stream).
constexpr int SYM_SEG = 1280;                          // symbols staged per round (5 KB)
// coefficients staged as int16 (a value outside int16 sends the stream to the general path):
// half the LDS of int32 rows, 4 workgroups per CU instead of 3
constexpr int SYM_QP = 72;                             // int16 per staged block-plane (144 B)
constexpr int SYM_XW = SYM_SEG + 8;                    // int32 words: [3] = prev, [4 ..] symbols
constexpr int SYM_XD = (SYM_XW / 2 > DX_WAVE ? SYM_XW / 2 : DX_WAVE);   // doubles per wave

template <int C, bool RGB, int DQM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void sym_image_kernel(DecArgs a, SymImageArgs z, QTab t,
                                                                                              const int64_t* grange) {
  constexpr int QS = 8 * C * SYM_QP;                   // int16 per wave
  __shared__ __attribute__((aligned(16))) int16_t qs_all[4 * QS];
  __shared__ int bps_all[4 * 32];                       // block-plane start offsets per wave
  __shared__ __attribute__((aligned(16))) double xs_all[4 * SYM_XD];
  __shared__ double tq[192];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = lane >> 3, r = lane & 7;
  // DQ_INT: q * table is an exact integer, so q * (table / 16) = (q * table) / 16 exactly and
  // the IDCT's 1/16 rides in the table (IVC_DEC_FOLD16: 24 float64 multiplies per lane and group)
  for (int i = tid; i < 192; i += 256) tq[i] = (DQM == DQ_INT && IVC_DEC_FOLD16) ? t.q[i] * 0.0625 : t.q[i];
  uint32_t pos[2];
  dec_gather_pos<true>(r, pos);
  lds_barrier();   // the table only

  int16_t* qs = qs_all + wave * QS;
  int* bps = bps_all + wave * 32;
  double* xs = xs_all + wave * SYM_XD;
  int32_t* st = reinterpret_cast<int32_t*>(xs) + 4;    // st[-1]: the symbol before the round
  const int64_t nw = (int64_t)gridDim.x * 4;
  bool bad = false;
  // groups [g_lo, g_hi): all, or one chunk of a pipelined call (grange, written on the device)
  const int64_t g_lo = grange ? grange[0] : 0, g_hi = grange ? grange[1] : a.ngroups;
  // the group bounds are loaded one group ahead (scalar loads in flight during the group)
  int64_t g = g_lo + (int64_t)blockIdx.x * 4 + wave;
  int64_t Sn = g < g_hi ? z.gstart[g] : 0, En = g < g_hi ? z.gstart[g + 1] : 0;
  for (; g < g_hi; g += nw) {
    const DecGroup G = dec_group<DEC_IMAGE>(a, g);
    const int64_t S = Sn, E = En;
    if (g + nw < g_hi) {
      Sn = z.gstart[g + nw];
      En = z.gstart[g + nw + 1];
    }
    const int nbp = C * G.nb;                          // block-planes (EOBs) of the group
    if (S < 0 || E <= S || E > z.n || E - S > (int64_t)nbp * 130) {
      bad = true;                                      // wave-uniform
      continue;
    }
    const int len = (int)(E - S);
    const __amdgpu_buffer_rsrc_t rs = dec_rsrc(z.sym + S, (uint32_t)len * 4u);
    // zero the coefficient staging (C x 8 rows of SYM_QP int16)
#pragma unroll
    for (int j = 0; j < (QS / 8 + 63) / 64; ++j) {
      const int c = j * 64 + lane;
      if (c < QS / 8) *reinterpret_cast<dec_u32x4*>(qs + 8 * c) = dec_u32x4{0, 0, 0, 0};
    }
    if (lane == 0) bps[0] = 0;
    int pcarry = 0;         // coefficients of the group before the chunk
    int bpcarry = 0;        // EOBs before the chunk
    int prevc = 1;          // the symbol before the round (a group starts at a value slot)
    if (IVC_DEC_ABLATE & 2) bpcarry = nbp;
    for (int s0 = 0; s0 < ((IVC_DEC_ABLATE & 2) ? 0 : len); s0 += SYM_SEG) {
      // one round: every load in flight, then the LDS writes
      dec_u32x4 v[SYM_SEG / 256];
#pragma unroll
      for (int j = 0; j < SYM_SEG / 256; ++j)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (s0 + j * 256 + lane * 4) * 4, 0, 0);
      const int nxt = (int)__builtin_amdgcn_raw_buffer_load_b32(rs, (s0 + SYM_SEG) * 4, 0, 0);
      __builtin_amdgcn_wave_barrier();                 // the previous round's reads are done
#pragma unroll
      for (int j = 0; j < SYM_SEG / 256; ++j)
        *reinterpret_cast<dec_u32x4*>(st + j * 256 + lane * 4) = v[j];
      if (lane == 0) {
        st[-1] = prevc;
        st[SYM_SEG] = nxt;
      }
      __builtin_amdgcn_wave_barrier();
      const int rlen = len - s0 < SYM_SEG ? len - s0 : SYM_SEG;
      // 4 symbols per lane (lane l: symbols 4l .. 4l + 3 of a 256-symbol chunk): one wave scan
      // and one LDS round trip per 256 symbols.  A run length is clamped to 127 (anything past
      // 64 already makes its block-plane fail the offset checks), so a chunk's coefficient
      // count fits 16 bits and the EOB count sits above it.
      for (int c0 = 0; c0 < rlen; c0 += 256) {
        const int i0 = c0 + 4 * lane;
        const dec_u32x4 q = *reinterpret_cast<const dec_u32x4*>(st + i0);
        // (the neighbours from the neighbouring lanes by DPP wave shifts instead — these strided
        // reads are 4-way bank conflicts — measured 0.2 % slower, profiles/r05an_*)
        const int pvs = st[i0 - 1], nxs = st[i0 + 4];
        const int v[4] = {(int)q.x, (int)q.y, (int)q.z, (int)q.w};
        int pk[4];
        bool eobf[4], isval[4];
        int lt = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int prv = e ? v[e - 1] : pvs, nx = e < 3 ? v[e + 1] : nxs;
          // Past the group's last symbol (its last EOB) the staging holds zeros (the buffer
          // range ends there): the first is a value slot holding 0, which adds one coefficient
          // past the last block-plane (no write, no EOB, no failure), every later one a
          // run-length slot — so the tail needs no validity test
          const bool valid = IVC_DEC_PAD_ZERO || i0 + e < rlen;
          const bool slot = valid && prv != 0;         // not a run-length slot
          const bool ise = v[e] == z.eob;
          eobf[e] = slot && ise;
          isval[e] = slot && !ise;
          const int run = nx < 1 ? 1 : (nx > 127 ? 127 : nx);
          // (EOB flag << 16) | coefficient count, as one select chain: EOB, else a value's
          // count (the run length for a 0), else (a run-length slot) nothing
          const int f = ise ? (1 << 16) : (v[e] == 0 ? run : 1);
          pk[e] = slot ? f : 0;
          lt += pk[e];
        }
        const int incl = dec_wave_incl_sum(lt);
        int pre = incl - lt;
        int pex[4], bp[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pex[e] = pcarry + (pre & 0xffff);          // this slot's coefficient offset
          bp[e] = bpcarry + (pre >> 16);              // its block-plane
          pre += pk[e];
          if (eobf[e] && bp[e] < nbp) bps[bp[e] + 1] = pex[e];
        }
        __builtin_amdgcn_wave_barrier();
        // every block-plane start read first (one LDS wait), then the checks and the writes
        int bs[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) bs[e] = bps[bp[e] < nbp ? bp[e] : 0];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool bpok = bp[e] < nbp;
          const int off = pex[e] - bs[e];             // offset inside the block-plane
          // (non-short-circuit & and |: lane masks combined by the scalar unit, no branches)
          const bool nzv = isval[e] & (v[e] != 0);
          const bool wr = nzv & (off < 64) & bpok & (v[e] == (int)(int16_t)v[e]);
          bad |= (nzv & !wr) | (eobf[e] & ((off > 64) | !bpok));
          if (wr) qs[__umul24(bp[e], SYM_QP) + off] = (int16_t)v[e];
        }
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        pcarry += tot & 0xffff;
        bpcarry += tot >> 16;
      }
      prevc = st[SYM_SEG - 1];
    }
    if (bpcarry != nbp) bad = true;
    __builtin_amdgcn_wave_barrier();
    dec_group_math<C, DEC_IMAGE, RGB, int16_t, SYM_QP, DQM>(a, G, qs, xs, tq, pos, b, r, lane);
  }
  if (__ballot(bad) && lane == 0) atomicOr(z.fail, 1);
}

// group starts from the EOB bit mask of zf_count (bit i of tile t: symbol t * 4096 + i is an
// EOB slot) and tile_first (EOBs before each tile): the symbol after EOB number C * blk0(g) - 1
// starts group g; one wave per 4096-symbol tile, lane = 64 symbols.  A lane holds EOBs
// [e, e + cnt) of the stream; the group starts among their successors are found by arithmetic
// (one division per lane: the first block-plane >= e + 1 that starts a group, then steps of
// 8 C block-planes, or to the next block row) and each one's EOB located in the lane's mask.
// The stream start is group 0's, the position after the last expected EOB is gstart[ngroups].
__global__ __launch_bounds__(256) void sym_locate_kernel(const uint32_t* __restrict__ mask,
                                                         const int64_t* __restrict__ tile_first,
                                                         int64_t t_begin, int64_t ntiles, int C,
                                                         int w, int gpr, int64_t nbp_total,
                                                         int64_t* gstart) {
  const int lane = threadIdx.x & 63;
  const int64_t nwv = (int64_t)gridDim.x * 4;
  if (t_begin == 0 && blockIdx.x == 0 && threadIdx.x == 0) gstart[0] = 0;
  const int64_t D = (int64_t)C * w;                    // block-planes per block row
  const int64_t GS = 8 * (int64_t)C;                   // block-planes per full group
  for (int64_t t = t_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < ntiles; t += nwv) {
    const uint64_t mk = (uint64_t)mask[t * 128 + 2 * lane] | ((uint64_t)mask[t * 128 + 2 * lane + 1] << 32);
    const int cnt = __builtin_popcountll(mk);
    const int incl = dec_wave_incl_sum(cnt);
    if (cnt == 0) continue;
    const int64_t e = tile_first[t] + (incl - cnt);   // EOB index of this lane's first EOB
    // block-plane numbers after this lane's EOBs: (e, e + cnt]
    const int64_t lo = e + 1, hi = e + cnt < nbp_total ? e + cnt : nbp_total;
    int64_t row = lo / D;
    int64_t rem = lo - row * D;
    rem = (rem + GS - 1) / GS * GS;                    // the first group start at or after lo
    if (rem >= D) {
      ++row;
      rem = 0;
    }
    for (int64_t bpn = row * D + rem; bpn <= hi;) {
      // EOB number bpn - 1 is the lane's (bpn - 1 - e)-th: position of that set bit
      int k = (int)(bpn - 1 - e);
      uint64_t m = mk;
      for (; k > 0; --k) m &= m - 1;
      const int bit = __builtin_ctzll(m);
      gstart[row * gpr + rem / GS] = t * 4096 + lane * 64 + bit + 1;
      rem += GS;
      if (rem >= D) {
        ++row;
        rem = 0;
      }
      bpn = row * D + rem;
    }
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
                                     hipStream_t s, const int* skip) {
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
  a.skip = skip;
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

// symbols -> image, fused: gstart from the EOB mask, then the group kernel (see above).
// The pipelined call (launch_symbols2image) runs both per chunk of tiles: locate_range on
// tiles [t0, t1), image_range on the groups of a device-written range.
static DecArgs s2i_args(int64_t nframes, int64_t H, int64_t W, double* out) {
  DecArgs a{};
  a.out = out;
  a.w = (int)(W / 8);
  a.gpr = (a.w + 7) / 8;
  a.nblk = nframes * (H / 8) * a.w;
  a.ngroups = nframes * (H / 8) * a.gpr;
  a.W3 = W * 3;
  return a;
}

hipError_t launch_sym_locate_range(const uint32_t* eobmask, const int64_t* tile_first, int64_t t0,
                                   int64_t t1, int64_t nframes, int64_t H, int64_t W, int C,
                                   int64_t* gstart, hipStream_t s) {
  const DecArgs a = s2i_args(nframes, H, W, nullptr);
  const int64_t nb = (t1 - t0 + 3) / 4;
  if (nb <= 0) return hipSuccess;
  sym_locate_kernel<<<(unsigned)(nb < 256 * 16 ? nb : 256 * 16), 256, 0, s>>>(
      eobmask, tile_first, t0, t1, C, a.w, a.gpr, (int64_t)C * a.nblk, gstart);
  return hipGetLastError();
}

// the groups chunk c owns: those whose first block-plane follows an EOB of the chunk's tiles,
// i.e. first block-plane in [E_c + 1, E_{c+1} + 1) with E = EOBs before the chunk (tile_first
// at its first tile); chunk 0 also owns group 0, the last chunk every group to the end
__global__ void s2i_group_range_kernel(const int64_t* tile_first, int64_t tc0, int64_t tc1,
                                       int first, int last, int C, int w, int gpr,
                                       int64_t ngroups, int64_t* range) {
  const int64_t D = (int64_t)C * w, GS = 8 * (int64_t)C;
  auto first_group_from = [&](int64_t b) -> int64_t {   // first group whose first block-plane >= b
    if (b <= 0) return 0;
    int64_t row = b / D, rem = b - row * D;
    rem = (rem + GS - 1) / GS * GS;
    if (rem >= D) {
      ++row;
      rem = 0;
    }
    const int64_t g = row * gpr + rem / GS;
    return g < ngroups ? g : ngroups;
  };
  range[0] = first ? 0 : first_group_from(tile_first[tc0] + 1);
  range[1] = last ? ngroups : first_group_from(tile_first[tc1] + 1);
}

hipError_t launch_sym_group_range(const int64_t* tile_first, int64_t tc0, int64_t tc1, int first,
                                  int last, int64_t nframes, int64_t H, int64_t W, int C,
                                  int64_t* range, hipStream_t s) {
  const DecArgs a = s2i_args(nframes, H, W, nullptr);
  s2i_group_range_kernel<<<1, 1, 0, s>>>(tile_first, tc0, tc1, first, last, C, a.w, a.gpr,
                                         a.ngroups, range);
  return hipGetLastError();
}

hipError_t launch_sym_image_range(const int32_t* sym, int64_t n, int32_t eob, int64_t nframes,
                                  int64_t H, int64_t W, int C, const QTab& t, int to_rgb,
                                  double* out, const int64_t* gstart, int* fail,
                                  const int64_t* grange, hipStream_t s) {
  const DecArgs a = s2i_args(nframes, H, W, out);
  SymImageArgs z{sym, n, eob, gstart, fail};
  auto go = [&](auto k) {
    // (a chunk's launch keeps the whole resident grid: 3/4 or 7/8 of it, leaving room for the
    // next chunk's EOB pass, measured 9-10 % slower)
    const unsigned grid = resident_grid_ptr(reinterpret_cast<const void*>(k), (a.ngroups + 3) / 4);
    k<<<grid, 256, 0, s>>>(a, z, t, grange);
  };
  // int16 coefficients times a finite table below 2^16 in magnitude stay inside int32 (and
  // with a table of positive integers the product is exact)
  bool fast = true, integral = true;
  for (int i = 0; i < 192; ++i) {
    const double v = t.q[i];
    if (!(__builtin_fabs(v) < 65536.0)) fast = false;
    if (!(v > 0.0 && v < 65536.0 && v == __builtin_trunc(v))) integral = false;
  }
  const int dqm = !fast ? DQ_GENERAL : (integral ? DQ_INT : DQ_FAST);
  auto pick = [&](auto rgb_c) {
    constexpr bool R = decltype(rgb_c)::value;
    if (C == 3) {
      if (dqm == DQ_INT) go(sym_image_kernel<3, R, DQ_INT>);
      else if (dqm == DQ_FAST) go(sym_image_kernel<3, R, DQ_FAST>);
      else go(sym_image_kernel<3, R, DQ_GENERAL>);
    } else {
      if (dqm == DQ_INT) go(sym_image_kernel<1, R, DQ_INT>);
      else if (dqm == DQ_FAST) go(sym_image_kernel<1, R, DQ_FAST>);
      else go(sym_image_kernel<1, R, DQ_GENERAL>);
    }
  };
  if (to_rgb) pick(std::true_type{});
  else pick(std::false_type{});
  return hipGetLastError();
}

hipError_t launch_sym_image(const int32_t* sym, int64_t n, int32_t eob, const uint32_t* eobmask,
                            const int64_t* tile_first, int64_t ntiles, int64_t nframes, int64_t H,
                            int64_t W, int C, const QTab& t, int to_rgb, double* out,
                            int64_t* gstart, int* fail, hipStream_t s) {
  const DecArgs a = s2i_args(nframes, H, W, out);
  hipError_t e = hipMemsetAsync(gstart, 0xff, (size_t)(a.ngroups + 1) * 8, s);
  if (e == hipSuccess)
    e = launch_sym_locate_range(eobmask, tile_first, 0, ntiles, nframes, H, W, C, gstart, s);
  if (e == hipSuccess)
    e = launch_sym_image_range(sym, n, eob, nframes, H, W, C, t, to_rgb, out, gstart, fail,
                               nullptr, s);
  return e;
}

}  // namespace ivc
