// ivc_me_mfma.hip — the +-16 exact-u8 full search (MotionCompensator.compute_motion_vector,
// ivclab/video/motion.py:8-58, on integer-valued frames) on the matrix cores.
//
// For a tile of 16 horizontally adjacent 8x8 blocks j of one block row and one vertical
// displacement dy, the cross-correlations of every block with every window position u of
// the tile's reference rows are ONE matrix product:
//   Y[u][j] = sum_{r, c} ref[y0 + dy + r][x0 + u + c] * cur_j[r][c]        (u in [0, 160))
//           = A_dy[u][(r, c)] . B[(r, c)][j],  K = 64 = the block's pixels
// with A_dy a Hankel matrix of the reference rows (row u = the 8x8 window at u) and B the
// tile's blocks, one v_mfma_i32_16x16x64_i8 per 16 window positions.  Block j needs only
// u = 8j + dx, dx in [0, 32] (33 of the 160 rows; the rest of the product is discarded).
// The bytes enter the i8 MFMA as a - 128 (XOR 0x80):
//   sum a b = Y' + 128 S1(window) + 128 S1(block) - 64 * 128^2,   Y' = sum (a-128)(b-128)
//   SSD = sum b^2 - 2 sum a b + S2(window) = K' + const_j,   K' = S2 - 256 S1 - 2 Y'
// so for a fixed block the candidates order by K' exactly as by the reference's SSD (every
// term an exact integer): same minimum, same ties.  With a' = a - 128 (the staged bytes),
// a (256 - a) = 2^14 - a'^2, so W = 256 S1 - S2 = 2^20 - S2'(window) (in [0, 2^20]); per tile
// the workgroup computes S2' of its 33 x 160 windows from the staged rows (sdot4 row sums, a
// prefix down the rows) into E[dy][u] = 128 W + 127 - rank (E_OUT-based for a window outside
// the frame).  The MFMA runs as
// D[j][u] = B^T A + C (block rows, window columns), so a lane holds 4 blocks at ONE window
// position and needs one E per MFMA; C = 0 where the window is one of block j's candidates
// (u - 8j in [0, 32]) and -2^22 where it is not.  A candidate's key is (D << 8) + E =
// 128 (-K') + 127 - rank: one v_lshl_add per MFMA output and a running v_max per block, with
// no per-M-tile masking.  rank = (dy - the wave's first dy) * 10 + u / 16 (< 90: 7 bits) = the
// candidate's raster position among the lane's candidates of the block, so the lane's maximum
// key is its first strict minimum of K'; lanes and waves are merged on (K', raster index) -
// the reference's first strict minimum in raster order (motion.py:48).  Key ranges (int32,
// no wrap): valid [-266.34 M, 403 M]; masked [-1340 M, -671 M]; window outside the frame
// [-937 M, -268.44 M]; both [-2011 M, ...]: VALID_MIN (-267.4 M) separates the valid keys.
//
// Work: a workgroup (4 waves) per tile; wave w takes a contiguous range of dy (9, 8, 8, 8),
// M-tile (16 window positions) outer and dy inner, so each MFMA reads one new reference row
// (8 bytes per lane) from LDS and reuses the other.  The tile's 40 reference rows are staged
// as four byte-shifted copies (copy_s[row][w] = bytes 4w + s .. 4w + s + 3, XOR 0x80), so
// a lane's 8 bytes at window position u are two aligned dwords of copy (u & 3).
#include "ivc_internal.h"

#include <type_traits>

#ifndef IVC_ME_EPRE
#define IVC_ME_EPRE 4  // window-energy rows read this many rows ahead (0: as the compiler places them;
                       // r06 A/Bs: profiles/r06w_ab_me_energy.log, r06x_ab_me_energy_base.log)
#endif
#ifndef IVC_ME_EBASE
#define IVC_ME_EBASE 1 // (with EPRE) the rows' LDS addresses from one base per 8 rows
#endif
#ifndef IVC_ME_EFAST
#define IVC_ME_EFAST 1 // interior tiles form the energies without the frame checks
#endif
#ifndef IVC_ME_ABL
#define IVC_ME_ABL 0   // tools/ab timing builds only (results wrong; profiles/r06f_ab_me_ablation.log):
                       // 1 no energies, 2 keys of one quad only, 4 no staging writes, 8 no search
#endif

namespace ivc {
namespace mf {
// E's base for a window outside the frame (E in [-671 M, -537 M]), and the least valid key
// (the ranges: file header)
constexpr int E_OUT = -(1 << 29), VALID_MIN = -(1 << 28) + (1 << 20);
constexpr int MASK_C = -(1 << 22);               // C of a (block, window) pair that is no candidate
}  // namespace mf

typedef int mf_v4i __attribute__((ext_vector_type(4)));
typedef unsigned int mf_u32x2 __attribute__((ext_vector_type(2)));

// ---- two block rows per tile --------------------------------------------------
// A tile is 8 adjacent blocks of block row by (top) and the 8 below them (bottom): 16 MFMA
// rows.  The bottom blocks' windows at dy' are the top blocks' windows at dy = dy' + 8 (the
// same reference rows), so one MFMA over the reference rows at offset R (R in [0, 40], rows
// yb + R .. of yb = 8 by - 16) serves the top blocks' candidates dy = R and the bottom blocks'
// dy' = R - 8.  Against one block row of 16: the window positions per tile drop from 160 to
// 96 (6 M-tiles), MFMAs per 16 blocks from 330 to 246, key formations from 660 to 528 register
// operations (a register is a quad of blocks: top 0-3, top 4-7, bottom 0-3, bottom 4-7, and a
// quad is live in 4 of the 6 M-tiles and for 33 of the 41 offsets R), and the LDS from 51.7 KB
// to 39.4 KB: 4 workgroups per CU instead of 3.  Ties and keys as in the header: rank =
// (R - the wave's first R) * 6 + mt orders a lane's candidates of a block in raster order.
namespace mf2 {
constexpr int SR = 16, N = 2 * SR + 1, TBX = 8;   // blocks per tile row
constexpr int NR = 41;                             // offsets R
constexpr int ROWS = 48;                           // staged reference rows
constexpr int U = 96, NMT = U / 16;                // window positions, M-tiles
constexpr int NPAIR = 13;                          // staged 8-byte pairs per row (104 bytes)
constexpr int PITCH = 30;                          // dwords per copy row (26 + 1 used); 2 PITCH = 28 mod 32
constexpr int ITEMS = ROWS * NPAIR;
constexpr int IPT = (ITEMS + 255) / 256;
constexpr int COPY = 1448;                         // >= ROWS * PITCH, = 8 mod 32
static_assert(COPY >= ROWS * PITCH && COPY % 32 == 8 && (2 * PITCH) % 8 == 4, "bank layout");
constexpr int E_OFF = 4 * COPY;                    // E[R][u]
constexpr int RED_OFF = E_OFF + NR * U;
constexpr int LDS_DW = RED_OFF + 4 * 16 * 2;
static_assert(LDS_DW * 4 <= 40960, "4 workgroups per CU");
// wave w: offsets [r0, r0 + nr): 11, 10, 10, 10
__host__ __device__ constexpr int wave_r0(int w) { return w == 0 ? 0 : 10 * w + 1; }
__host__ __device__ constexpr int wave_nr(int w) { return w == 0 ? 11 : 10; }
}  // namespace mf2

template <int WV>    // 0: wave 0, 1: waves 1 and 2, 3: wave 3 (liveness of the halves by R)
__device__ __forceinline__ void me2_search(const uint32_t* lds, int* red, int wave, int g, int l16,
                                           mf_v4i bop) {
  using namespace mf2;
  using mf::MASK_C;
  using mf::VALID_MIN;
  const int r0 = wave_r0(wave);
  constexpr int NRW = WV == 0 ? 11 : 10;
  const uint32_t* cb = lds + (l16 & 3) * COPY;
  const int* ev = reinterpret_cast<const int*>(lds + E_OFF) + l16 + r0 * U;
  // block operand rows: register i (D row 4g + i) holds quad i = (i >> 1 ? bottom : top),
  // blocks 4 (i & 1) .. + 3, lane group g = block 4 (i & 1) + g of it
  const mf_v4i bks = mf_v4i{bop.z, bop.w, bop.x, bop.y};
  int acc[4] = {INT_MIN, INT_MIN, INT_MIN, INT_MIN};
  // quads 0 / 2 (blocks 0-3) serve M-tiles 0-3, quads 1 / 3 (blocks 4-7) M-tiles 2-5: three
  // segments of two M-tiles with the live quads fixed at compile time, each M-tile one basic
  // block (a fully unrolled search lets the scheduler hoist every LDS read: spills)
  auto mtile = [&](int mt, auto q01c, auto q23c) {
    constexpr bool q01 = decltype(q01c)::value, q23 = decltype(q23c)::value;
    const int wd = 4 * mt + (l16 >> 2);
    const int v0 = 16 * mt + l16 - 8 * g, v1 = v0 - 32;          // u - 8 j for j = g, 4 + g
    const int c0 = (unsigned)v0 <= 32u ? 0 : MASK_C, c1 = (unsigned)v1 <= 32u ? 0 : MASK_C;
    const mf_v4i cm = mf_v4i{c0, c1, c0, c1};
    auto row = [&](int kk) {
      const int rr = r0 + 2 * g + kk;
      return mf_u32x2{cb[rr * PITCH + wd], cb[rr * PITCH + wd + 1]};
    };
    mf_v4i T;
    {
      const mf_u32x2 a0 = row(0), a1 = row(1);
      T = mf_v4i{(int)a0.x, (int)a0.y, (int)a1.x, (int)a1.y};
    }
#pragma unroll
    for (int dl = 0; dl < NRW; ++dl) {
      if (dl > 0) {
        const mf_u32x2 rn = row(dl + 1);
        if (dl & 1) {
          T.x = (int)rn.x;
          T.y = (int)rn.y;
        } else {
          T.z = (int)rn.x;
          T.w = (int)rn.y;
        }
      }
      const uint32_t e = (uint32_t)ev[dl * U + 16 * mt];
      const mf_v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8((dl & 1) ? bks : bop, T, cm, 0, 0, 0);
      // R = r0 + dl: top live for R <= 32, bottom for R >= 8 (compile time except waves 1-2,
      // where both always are)
      const bool top = WV == 0 ? true : (WV == 3 ? dl <= 1 : true);
      const bool bot = WV == 0 ? dl >= 8 : true;
      if (top && q01) acc[0] = max(acc[0], (int)(((uint32_t)d.x << 8) + e));
      if (IVC_ME_ABL & 2) {
        acc[1] ^= d.y;
        acc[2] ^= d.z;
        acc[3] ^= d.w;
        continue;
      }
      if (top && q23) acc[1] = max(acc[1], (int)(((uint32_t)d.y << 8) + e));
      if (bot && q01) acc[2] = max(acc[2], (int)(((uint32_t)d.z << 8) + e));
      if (bot && q23) acc[3] = max(acc[3], (int)(((uint32_t)d.w << 8) + e));
    }
  };
  // (the two M-tiles of a segment as two interleaved MFMA chains were measured slower: the
  // extra registers spill at 128 VGPRs)
#pragma unroll 1
  for (int mt = 0; mt < 2; ++mt) mtile(mt, std::true_type{}, std::false_type{});
#pragma unroll 1
  for (int mt = 2; mt < 4; ++mt) mtile(mt, std::true_type{}, std::true_type{});
#pragma unroll 1
  for (int mt = 4; mt < NMT; ++mt) mtile(mt, std::false_type{}, std::true_type{});
  // per block: best -K' over the 16 lanes, then the least raster index among its holders
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int key = acc[i];
    const bool valid = key >= VALID_MIN;
    const int nk = valid ? key >> 7 : INT_MIN;
    const int rank = 127 - (key & 127);
    const int R = r0 + rank / NMT;
    const int u = 16 * (rank % NMT) + l16;
    const int j = 4 * (i & 1) + g;
    const int dy = (i >> 1) ? R - 8 : R;
    const int ri = dy * N + u - 8 * j;
    int best = nk;
    best = max(best, __builtin_amdgcn_update_dpp(INT_MIN, best, 0xB1, 0xf, 0xf, false));
    best = max(best, __builtin_amdgcn_update_dpp(INT_MIN, best, 0x4E, 0xf, 0xf, false));
    best = max(best, __builtin_amdgcn_update_dpp(INT_MIN, best, 0x141, 0xf, 0xf, false));
    best = max(best, __builtin_amdgcn_update_dpp(INT_MIN, best, 0x140, 0xf, 0xf, false));
    int bri = valid && nk == best ? ri : INT_MAX;
    bri = min(bri, __builtin_amdgcn_update_dpp(INT_MAX, bri, 0xB1, 0xf, 0xf, false));
    bri = min(bri, __builtin_amdgcn_update_dpp(INT_MAX, bri, 0x4E, 0xf, 0xf, false));
    bri = min(bri, __builtin_amdgcn_update_dpp(INT_MAX, bri, 0x141, 0xf, 0xf, false));
    bri = min(bri, __builtin_amdgcn_update_dpp(INT_MAX, bri, 0x140, 0xf, 0xf, false));
    // (r05: letting a row's unique holder write its entry and reducing by DPP only on ties
    // measured no faster, 4.679 against 4.663 ms, profiles/r05f_ab_me.log)
    if (l16 == 0) {
      const int blk = 8 * (i >> 1) + j;                  // tile block: row-major, 0..15
      red[2 * (wave * 16 + blk)] = best;
      red[2 * (wave * 16 + blk) + 1] = bri;
    }
  }
}

__global__ __launch_bounds__(256, 4) void me_mfma16x2_kernel(const uint8_t* __restrict__ ref,
                                                             const uint8_t* __restrict__ cur,
                                                             int64_t nframes, int H, int W,
                                                             int64_t* __restrict__ mv) {
  using namespace mf2;
  using mf::E_OUT;
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_DW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = (int)__builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  const int g = lane >> 4, l16 = lane & 15;
  const int h = H / 8, w = W / 8;
  const int tpr = (w + TBX - 1) / TBX, trows = (h + 1) / 2;
  const uint32_t tpf = (uint32_t)(trows * tpr);
  const uint32_t ntiles = (uint32_t)nframes * tpf;
  const int64_t HW = (int64_t)H * W;
  struct Loads {
    uint32_t raw[IPT][3];
    mf_v4i bop;
  };
  auto tile_xy = [&](uint32_t t, uint32_t& f, int& by, int& bx0) {
    f = t / tpf;
    const uint32_t rem = t - f * tpf;
    by = 2 * (int)(rem / (uint32_t)tpr);
    bx0 = (int)(rem - (uint32_t)(by / 2) * tpr) * TBX;
  };
  // lane l16 = 4g' + i (MFMA row) loads quad i's block g': top/bottom i >> 1, column 4 (i & 1) + g'
  const int qi = l16 & 3, qg = l16 >> 2;
  auto load = [&](uint32_t t, Loads& L) {
    const bool exists = t < ntiles;
    uint32_t f;
    int by, bx0;
    tile_xy(exists ? t : 0u, f, by, bx0);
    const int xb = 8 * bx0 - SR, yb = 8 * by - SR;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(ref + (int64_t)f * HW), 0, exists ? (int)HW : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(cur + (int64_t)f * HW), 0, exists ? (int)HW : 0, 0x00020000);
    int tt = tid;
    asm volatile("" : "+v"(tt));           // (the item offsets: formed per tile, not kept live)
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tt + 256 * k;
      const int row = i / NPAIR, p = i - row * NPAIR;
      const int y = yb + row;
      const bool ok = i < ITEMS && y >= 0 && y < H;
      const int off = ok ? y * W + xb + 8 * p : 0x40000000;
      const mf_u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(rr, off, 0, 0);
      L.raw[k][0] = a.x;
      L.raw[k][1] = a.y;
      L.raw[k][2] = __builtin_amdgcn_raw_buffer_load_b32(rr, off + 8, 0, 0);
    }
    {
      const int bx = bx0 + 4 * (qi & 1) + qg, byy = by + (qi >> 1);
      const int off = bx < w && byy < h ? (8 * byy + 2 * g) * W + 8 * bx : 0x40000000;
      const mf_u32x2 r0 = __builtin_amdgcn_raw_buffer_load_b64(rc, off, 0, 0);
      const mf_u32x2 r1 = __builtin_amdgcn_raw_buffer_load_b64(rc, off + W, 0, 0);
      L.bop = mf_v4i{(int)r0.x, (int)r0.y, (int)r1.x, (int)r1.y};
    }
  };

  uint32_t tile = blockIdx.x;
  if ((gridDim.x & 7u) == 0u) tile = (tile & 7u) * (gridDim.x >> 3) + (tile >> 3);   // XCD runs
  Loads L;
  load(tile, L);
  int* red = reinterpret_cast<int*>(lds + RED_OFF);
  // the merge of the waves' per-block results of a searched tile (threads 0..15, one block
  // each): run for tile t at the start of tile t + 1, after its first barrier — red[] is next
  // written by tile t + 1's search, two barriers later — so no barrier of its own and the
  // other 240 threads stage meanwhile
  auto merge = [&](uint32_t pf, int pby, int pbx0) {
    if (tid < 16) {
      const int blk = tid, bx = pbx0 + (blk & 7), byy = pby + (blk >> 3);
      int k = red[2 * blk], ri = red[2 * blk + 1];
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) {
        const int ok_ = red[2 * (ww * 16 + blk)], oi = red[2 * (ww * 16 + blk) + 1];
        if (ok_ > k || (ok_ == k && oi < ri)) {
          k = ok_;
          ri = oi;
        }
      }
      if (bx < w && byy < h)
        mv[((int64_t)pf * h + byy) * w + bx] = ri == INT_MAX ? (int64_t)SR * N + SR : (int64_t)ri;
    }
  };
  uint32_t pf = 0;
  int pby = 0, pbx0 = 0;
  bool have_prev = false;
  for (; tile < ntiles; tile += gridDim.x) {
    uint32_t f;
    int by, bx0;
    tile_xy(tile, f, by, bx0);
    // the previous tile's LDS reads are done and its search's red[] writes have landed (this
    // barrier is the loop header: without lds_barrier's wait the merge below read stale
    // entries, ivc_internal.h)
    lds_barrier();
    if (have_prev) merge(pf, pby, pbx0);
    int ts = tid;
    asm volatile("" : "+v"(ts));
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = ts + 256 * k;
      if (i < ITEMS && !(IVC_ME_ABL & 4)) {
        const int row = i / NPAIR, p = i - row * NPAIR;
        uint32_t* d = lds + row * PITCH + 2 * p;
        const uint32_t w0 = L.raw[k][0] ^ 0x80808080u, w1 = L.raw[k][1] ^ 0x80808080u,
                       w2 = L.raw[k][2] ^ 0x80808080u;
        d[0] = w0;
        d[1] = w1;
#pragma unroll
        for (int s = 1; s < 4; ++s) {
          d[s * COPY] = __builtin_amdgcn_alignbyte(w1, w0, s);
          d[s * COPY + 1] = __builtin_amdgcn_alignbyte(w2, w1, s);
        }
      }
    }
    lds_barrier();
    {
      // window energies E[R][u] = B + 128 (-S2') (the header's form), two threads per
      // column u: threads 0..95 the offsets R < 20 from rows 0..26, threads 128..223 the
      // offsets R >= 20 from rows 20..47 (each a prefix over its rows)
      const int half = tid >> 7;
      int u = tid & 127;
      // (opaque: the per-offset constants derived from u are formed in the tile loop instead of
      // being hoisted out of it, where they stay live — or spill — through the search)
      asm volatile("" : "+v"(u));
      if (u < U && !(IVC_ME_ABL & 1)) {
        const uint32_t* cw = lds + (u & 3) * COPY + (u >> 2);
        const int xb = 8 * bx0 - SR, yb = 8 * by - SR;
        const bool xok = xb + u >= 0 && xb + u + 8 <= W;
        const int rlo = half ? 20 : 0, rhi = half ? NR : 20;     // offsets of this thread
        auto energy = [&](auto hf, auto edge) {
          constexpr int RL = decltype(hf)::value ? 20 : 0, RH = decltype(hf)::value ? NR : 20;
          constexpr bool EDGE = decltype(edge)::value;
          constexpr int NROW = RH + 7 - RL;
          int P[NROW + 1];
          int pr = 0;
#if IVC_ME_EPRE > 0
          // the rows read IVC_ME_EPRE ahead (each read otherwise waits its whole LDS latency)
          uint32_t b0[IVC_ME_EPRE], b1[IVC_ME_EPRE];
#if IVC_ME_EBASE
          // one opaque base per 8 rows, so each row's two dwords are one ds_read2 with constant
          // offsets (the compiler otherwise forms every row's address with its own add)
          int rb[(NROW + 7) / 8];
#pragma unroll
          for (int k = 0; k < (NROW + 7) / 8; ++k) {
            rb[k] = (u & 3) * COPY + (u >> 2) + (RL + 8 * k) * PITCH;
            asm volatile("" : "+v"(rb[k]));
          }
          auto rd = [&](int r, int dw) { return lds[rb[(r - RL) >> 3] + ((r - RL) & 7) * PITCH + dw]; };
#else
          auto rd = [&](int r, int dw) { return cw[r * PITCH + dw]; };
#endif
#pragma unroll
          for (int k = 0; k < IVC_ME_EPRE; ++k) {
            b0[k] = rd(RL + k, 0);
            b1[k] = rd(RL + k, 1);
          }
#endif
#pragma unroll
          for (int r = RL; r < RH + 7; ++r) {
#if IVC_ME_EPRE > 0
            const int w0 = (int)b0[(r - RL) % IVC_ME_EPRE], w1 = (int)b1[(r - RL) % IVC_ME_EPRE];
            if (r + IVC_ME_EPRE < RH + 7) {
              b0[(r - RL) % IVC_ME_EPRE] = rd(r + IVC_ME_EPRE, 0);
              b1[(r - RL) % IVC_ME_EPRE] = rd(r + IVC_ME_EPRE, 1);
            }
            asm volatile("" ::: "memory");
#else
            const int w0 = (int)cw[r * PITCH], w1 = (int)cw[r * PITCH + 1];
#endif
            pr = __builtin_amdgcn_sdot4(w1, w1, __builtin_amdgcn_sdot4(w0, w0, pr, false), false);
            P[r - RL] = pr;
            if (r >= RL + 7) {
              const int R = r - 7;
              const int t = (r - 8 >= RL ? P[r - 8 - RL] : 0) - pr;
              const int wv = R < 11 ? 0 : (R - 1) / 10;
              const int rank = (R - wave_r0(wv)) * NMT + (u >> 4);
              if (EDGE) {
                const bool ok = xok && (unsigned)(yb + R) <= (unsigned)(H - 8);
                lds[E_OFF + R * U + u] = (uint32_t)((ok ? (1 << 27) + 127 - rank : E_OUT) + 128 * t);
              } else {
                lds[E_OFF + R * U + u] = (uint32_t)((1 << 27) + 127 - rank + 128 * t);
              }
            }
          }
        };
        (void)rlo;
        (void)rhi;
#if IVC_ME_EFAST
        // a tile whose windows all lie inside the frame (workgroup-uniform) skips the checks
        const bool inner = xb >= 0 && xb + U + 8 <= W && yb >= 0 && yb + NR + 7 <= H;
        if (inner) {
          if (half) energy(std::true_type{}, std::false_type{});
          else energy(std::false_type{}, std::false_type{});
        } else
#endif
        {
          if (half) energy(std::true_type{}, std::true_type{});
          else energy(std::false_type{}, std::true_type{});
        }
      }
    }
    const mf_v4i bop = mf_v4i{L.bop.x ^ (int)0x80808080u, L.bop.y ^ (int)0x80808080u,
                              L.bop.z ^ (int)0x80808080u, L.bop.w ^ (int)0x80808080u};
    lds_barrier();
    load(tile + gridDim.x, L);                          // the next tile's inputs, in flight
    if (IVC_ME_ABL & 8) {
      if (tid < 16) red[2 * tid] = bop.x;
    } else if (wave == 0) me2_search<0>(lds, red, wave, g, l16, bop);
    else if (wave == 3) me2_search<3>(lds, red, wave, g, l16, bop);
    else me2_search<1>(lds, red, wave, g, l16, bop);
    pf = f;
    pby = by;
    pbx0 = bx0;
    have_prev = true;
  }
  // the last tile's merge (every wave reaches this barrier: the loop bound is workgroup-uniform)
  lds_barrier();
  if (have_prev) merge(pf, pby, pbx0);
}

// A batch of frame pairs on the matrix cores, in launches of under 2^31 tiles (32-bit tile
// counters).  Returns false when the kernel does not apply (the caller keeps its own path): a
// frame of 2 GiB or more (32-bit buffer offsets).
bool launch_me_mfma16(const uint8_t* ref, const uint8_t* cur, int64_t nf, int H, int W, int64_t* mv,
                      hipStream_t s) {
  if ((int64_t)H * W >= ((int64_t)1 << 31)) return false;
  const int h = H / 8, w = W / 8;
  const int64_t tpf = (int64_t)((h + 1) / 2) * ((w + mf2::TBX - 1) / mf2::TBX);   // tiles per frame
  if (nf <= 0 || tpf <= 0) return true;
  const int64_t fmax = (((int64_t)1 << 31) - 1) / tpf;                            // frames per launch
  const int64_t HW = (int64_t)H * W;
  for (int64_t f0 = 0; f0 < nf; f0 += fmax) {
    const int64_t n = nf - f0 < fmax ? nf - f0 : fmax;
    const int64_t tiles = n * tpf;
    int64_t grid = 2 * (int64_t)resident_grid_ptr(reinterpret_cast<const void*>(me_mfma16x2_kernel), tiles);
    if (grid > tiles) grid = tiles;
    me_mfma16x2_kernel<<<(unsigned)grid, 256, 0, s>>>(ref + f0 * HW, cur + f0 * HW, n, H, W,
                                                      mv + f0 * (int64_t)h * w);
  }
  return true;
}

}  // namespace ivc
