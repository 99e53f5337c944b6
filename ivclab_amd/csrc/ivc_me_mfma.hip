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

namespace ivc {
namespace mf {
constexpr int SR = 16, N = 2 * SR + 1, TB = 16;   // candidates per axis, blocks per tile
constexpr int ROWS = 2 * SR + 8;                 // reference rows of a tile (40)
constexpr int U = 160;                           // window positions per dy (10 M-tiles of 16)
constexpr int NMT = U / 16;
// LDS banks of 4-byte reads are (dword address) mod 32 per 32-lane half.  COPY = 8 (mod 32) and
// PITCH = 46 put the search's reads (lane (g, l16): copy l16 & 3, word 4 mt + l16 / 4, row
// 2g + ..., g in {0, 1} per half) on 32 distinct banks ({8c + q} and {8c + q + 28}), and the
// window-energy pass's (lane u: copy u & 3, word u / 4 + ...) on 32 as well
constexpr int PITCH = 46;                        // dwords per copy row (44 in use)
constexpr int NPAIR = 22;                        // staged dword pairs per row (44 dwords)
constexpr int ITEMS = ROWS * NPAIR;              // staging items (row, pair) per tile
constexpr int IPT = (ITEMS + 255) / 256;
constexpr int COPY = ROWS * PITCH + 24;          // dwords per copy (= 8 mod 32)
static_assert(COPY % 32 == 8 && (2 * PITCH) % 8 == 4, "bank layout");
constexpr int E_OFF = 4 * COPY;                  // E[dy][u] (int32)
constexpr int RED_OFF = E_OFF + N * U;         // per wave and block: (K' << 11 | raster)
constexpr int LDS_DW = RED_OFF + 4 * TB * 2;
// E's base for a window outside the frame (E in [-671 M, -537 M]), and the least valid key
// (the ranges: file header)
constexpr int E_OUT = -(1 << 29), VALID_MIN = -(1 << 28) + (1 << 20);
constexpr int MASK_C = -(1 << 22);               // C of a (block, window) pair that is no candidate
// wave w searches dy in [8w, 8w + 8) (wave 3 also dy = 32): whole rank groups, so a dy's group
// within the wave is dl / 4 (compile time)
__host__ __device__ constexpr int wave_dy0(int w) { return 8 * w; }
__host__ __device__ constexpr int wave_ndy(int w) { return w == 3 ? 9 : 8; }
}  // namespace mf

#ifndef IVC_ME_2ROW
#define IVC_ME_2ROW 1        // two block rows per tile (me_mfma16x2_kernel); 0: one block row
#endif

typedef int mf_v4i __attribute__((ext_vector_type(4)));
typedef unsigned int mf_u32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256, 3) void me_mfma16_kernel(const uint8_t* __restrict__ ref,
                                                        const uint8_t* __restrict__ cur,
                                                        int64_t nframes, int H, int W,
                                                        int64_t* __restrict__ mv) {
  using namespace mf;
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_DW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = (int)__builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  const int g = lane >> 4, l16 = lane & 15;      // k-group (block rows 2g, 2g+1) / M or N index
  const int h = H / 8, w = W / 8;
  const int tpr = (w + TB - 1) / TB;
  const uint32_t tpf = (uint32_t)(h * tpr);
  const uint32_t ntiles = (uint32_t)nframes * tpf;
  const int64_t HW = (int64_t)H * W;
  const int dyw0 = wave_dy0(wave);

  struct Loads {
    uint32_t raw[IPT][3];
    mf_v4i bop;
  };
  auto tile_xy = [&](uint32_t t, uint32_t& f, int& by, int& bx0) {
    f = t / tpf;
    const uint32_t rem = t - f * tpf;
    by = (int)(rem / (uint32_t)tpr);
    bx0 = (int)(rem - (uint32_t)by * tpr) * TB;
  };
  // a tile's global inputs: reference row pairs and this lane's block operand (block l16's
  // rows 2g, 2g+1)
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
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
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
      // MFMA row l16 = block pi(l16) = 4 (l16 & 3) + (l16 >> 2): result register i of lane group
      // g (D row 4g + i) then holds block 4i + g, so a register holds one whole quad of blocks
      const int bx = bx0 + 4 * (l16 & 3) + (l16 >> 2);
      const int off = bx < w ? (8 * by + 2 * g) * W + 8 * bx : 0x40000000;
      const mf_u32x2 r0 = __builtin_amdgcn_raw_buffer_load_b64(rc, off, 0, 0);
      const mf_u32x2 r1 = __builtin_amdgcn_raw_buffer_load_b64(rc, off + W, 0, 0);
      L.bop = mf_v4i{(int)r0.x, (int)r0.y, (int)r1.x, (int)r1.y};
    }
  };

  uint32_t tile = blockIdx.x;
  if ((gridDim.x & 7u) == 0u) tile = (tile & 7u) * (gridDim.x >> 3) + (tile >> 3);   // XCD runs
  Loads L;
  load(tile, L);
  for (; tile < ntiles; tile += gridDim.x) {
    uint32_t f;
    int by, bx0;
    tile_xy(tile, f, by, bx0);
    __syncthreads();                                   // the previous tile's LDS reads are done
    // ---- staging: 4 byte-shifted copies (XOR 0x80), then E[dy][u] from them ----------------
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
      if (i < ITEMS) {
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
    __syncthreads();
    if (tid < U) {
      // thread = window column u: with a' = a - 128 (the staged bytes), a (256 - a) = 2^14 - a'^2,
      // so W = 256 S1 - S2 = 2^20 - S2' over the window; horizontal 8-sums of a'^2 by sdot4 on
      // the copy holding bytes u .., the vertical 8-sum sliding down the 40 rows.
      // E = 128 W + 127 - rank, rank = (dy within its wave) * 10 + u / 16
      const int u = tid;
      const uint32_t* cw = lds + (u & 3) * COPY + (u >> 2);
      const int xb = 8 * bx0 - SR, yb = 8 * by - SR;
      const bool xok = xb + u >= 0 && xb + u + 8 <= W;
      // E = B + 128 (-S2') with B = 2^27 + 127 - rank for a window inside the frame and
      // E_OUT (no rank) outside: the column test folds into this lane's B, the row test is
      // wave-uniform (and skipped for tiles whose 40 rows all lie inside the frame)
      int bd[9];
#pragma unroll
      for (int d = 0; d < 9; ++d) bd[d] = xok ? (1 << 27) + 127 - (u >> 4) - 10 * d : E_OUT;
      // P[r] = prefix sum over rows <= r of the rows' 8-sums (two accumulating sdot4 per row);
      // a window's -S2' = P[r - 8] - P[r]
      auto energy = [&](auto all_rows) {
        int P[ROWS];
        int pr = 0;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          const int w0 = (int)cw[r * PITCH], w1 = (int)cw[r * PITCH + 1];
          pr = __builtin_amdgcn_sdot4(w1, w1, __builtin_amdgcn_sdot4(w0, w0, pr, false), false);
          P[r] = pr;
          if (r >= 7) {
            const int dy = r - 7;
            const int t = (r >= 8 ? P[r - 8] : 0) - pr;
            const int b0 = bd[dy < 32 ? (dy & 7) : 8];
            const int bsel = decltype(all_rows)::value || (unsigned)(yb + dy) <= (unsigned)(H - 8) ? b0 : E_OUT;
            lds[E_OFF + dy * U + u] = (uint32_t)(bsel + 128 * t);
          }
        }
      };
      if (yb >= 0 && yb + ROWS <= H)
        energy(std::true_type{});
      else
        energy(std::false_type{});
    }
    const mf_v4i bop = mf_v4i{L.bop.x ^ (int)0x80808080u, L.bop.y ^ (int)0x80808080u,
                              L.bop.z ^ (int)0x80808080u, L.bop.w ^ (int)0x80808080u};
    __syncthreads();
    load(tile + gridDim.x, L);                          // the next tile's inputs, in flight

    // ---- search: M-tile outer, dy inner (one new reference row per MFMA) -----------------
    // M-tile mt (window positions u in [16 mt, 16 mt + 16)) serves blocks [2 mt - 4, 2 mt + 1]:
    // the quads k - 1 and k for mt in {2k, 2k + 1}.  Iteration k rotates the block operand by
    // DPP quad_perm so that result register 0 holds quad (k + 3) & 3 (= k - 1) and register 1
    // quad k: only those two registers are turned into keys (registers 2 and 3 hold quads none
    // of whose windows are in this M-tile); the C mask kills the quads -1 and 4 (k = 0, 4) and
    // the non-candidate windows of the live quads.  After iteration k quad k - 1 has seen all
    // its windows and is reduced; quad k's running key moves to register 0's accumulator.
    const uint32_t* cb = lds + (l16 & 3) * COPY;      // this lane's copy (u & 3 = l16 & 3)
    const int* ev = reinterpret_cast<const int*>(lds + E_OFF) + l16 + dyw0 * U;
    const int cj = l16 - 8 * g;                       // u - 8 (4q + g) = 16 mt + cj - 32 q
    int* red = reinterpret_cast<int*>(lds + RED_OFF);
    auto dpp_max16 = [](int x) {
      x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0xB1, 0xf, 0xf, false));    // quad_perm 1,0,3,2
      x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x4E, 0xf, 0xf, false));    // quad_perm 2,3,0,1
      x = max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x141, 0xf, 0xf, false));   // row_half_mirror
      return max(x, __builtin_amdgcn_update_dpp(INT_MIN, x, 0x140, 0xf, 0xf, false)); // row_mirror
    };
    auto dpp_min16 = [](int x) {
      x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0xB1, 0xf, 0xf, false));
      x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x4E, 0xf, 0xf, false));
      x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x141, 0xf, 0xf, false));
      return min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x140, 0xf, 0xf, false));
    };
    // per block: the best -K' over the 16 lanes of a k-group, then the least raster index among
    // the lanes holding it (DPP all-reduces within 16-lane rows); the waves merge below
    auto finish = [&](int q, int key) {
      const bool valid = key >= VALID_MIN;
      const int nk = valid ? key >> 7 : INT_MIN;          // -K' (+ a per-block constant)
      const int rank = 127 - (key & 127);
      const int dy = dyw0 + rank / 10;
      const int u = 16 * (rank % 10) + l16;
      const int blk = 4 * q + g;
      const int ri = dy * N + u - 8 * blk;                // raster index dy * 33 + dx
      const int best = dpp_max16(nk);
      const int bri = dpp_min16(valid && nk == best ? ri : INT_MAX);
      if (l16 == 0) {
        red[2 * (wave * TB + blk)] = best;
        red[2 * (wave * TB + blk) + 1] = bri;
      }
    };
    // quad_perm rotations of the block operand: lane i of a quad takes lane (i + r) & 3's
    auto rot = [](const mf_v4i& x, auto ctrl) {
      constexpr int c = decltype(ctrl)::value;
      return mf_v4i{__builtin_amdgcn_mov_dpp(x.x, c, 0xf, 0xf, false),
                    __builtin_amdgcn_mov_dpp(x.y, c, 0xf, 0xf, false),
                    __builtin_amdgcn_mov_dpp(x.z, c, 0xf, 0xf, false),
                    __builtin_amdgcn_mov_dpp(x.w, c, 0xf, 0xf, false)};
    };
    mf_v4i bk = rot(bop, std::integral_constant<int, 0x93>{});   // r = 3: quads 3, 0, 1, 2
    mf_v4i bks = mf_v4i{bk.z, bk.w, bk.x, bk.y};      // block rows 2g + 1 | 2g
    int acc0 = INT_MIN, acc1 = INT_MIN;                 // running best key of quads k - 1, k
#pragma unroll 1
    for (int k = 0; k < NMT / 2; ++k) {
      const int q0 = (k + 3) & 3, q1 = k & 3;
#pragma unroll
      for (int hm = 0; hm < 2; ++hm) {
        const int mt = 2 * k + hm;
        const int wd = 4 * mt + (l16 >> 2);             // word of window position u = 16 mt + l16
        const int v0 = 16 * mt + cj - 32 * q0, v1 = 16 * mt + cj - 32 * q1;
        const mf_v4i cm = mf_v4i{(unsigned)v0 <= 32u ? 0 : MASK_C, (unsigned)v1 <= 32u ? 0 : MASK_C, 0, 0};
        const int* em = ev + 16 * mt;                   // E[dyw0 ..][u]
        const mf_v4i e0 = mf_v4i{em[0], em[U], em[2 * U], em[3 * U]};
        const mf_v4i e1 = mf_v4i{em[4 * U], em[5 * U], em[6 * U], em[7 * U]};
        // the window operand of step dl is rows (dl, dl + 1) (+ dyw0 + 2g), bytes u .. u+7.  One
        // 4-dword tuple T = [P | Q] serves every step without register copies: step dl + 1
        // overwrites the half holding row dl with row dl + 2, so the tuple alternates between
        // [row dl | row dl + 1] (even dl, block operand bk: block rows 2g | 2g + 1) and
        // [row dl + 1 | row dl] (odd dl, bks: the block operand with its halves swapped)
        auto row = [&](int kk) {
          const int rr = dyw0 + 2 * g + kk;
          return mf_u32x2{cb[rr * PITCH + wd], cb[rr * PITCH + wd + 1]};
        };
        mf_v4i T;
        {
          const mf_u32x2 r0 = row(0), r1 = row(1);
          T = mf_v4i{(int)r0.x, (int)r0.y, (int)r1.x, (int)r1.y};
        }
        auto step = [&](int dl, uint32_t e) {
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
          const mf_v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8((dl & 1) ? bks : bk, T, cm, 0, 0, 0);
          acc0 = max(acc0, (int)(((uint32_t)d.x << 8) + e));
          acc1 = max(acc1, (int)(((uint32_t)d.y << 8) + e));
        };
        step(0, (uint32_t)e0.x);
        step(1, (uint32_t)e0.y);
        step(2, (uint32_t)e0.z);
        step(3, (uint32_t)e0.w);
        step(4, (uint32_t)e1.x);
        step(5, (uint32_t)e1.y);
        step(6, (uint32_t)e1.z);
        step(7, (uint32_t)e1.w);
        if (wave == 3) step(8, (uint32_t)em[8 * U]);         // dy = 32: wave 3's ninth
      }
      if (k > 0) finish(q0, acc0);                      // quad k - 1 is complete
      acc0 = acc1;
      acc1 = INT_MIN;
      bk = rot(bk, std::integral_constant<int, 0x39>{});  // r + 1: quad_perm 1,2,3,0
      bks = mf_v4i{bk.z, bk.w, bk.x, bk.y};
    }
    __syncthreads();
    if (tid < TB) {
      const int j = tid, bx = bx0 + j;
      int k = red[2 * j], ri = red[2 * j + 1];
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) {
        const int ok_ = red[2 * (ww * TB + j)], oi = red[2 * (ww * TB + j) + 1];
        if (ok_ > k || (ok_ == k && oi < ri)) {
          k = ok_;
          ri = oi;
        }
      }
      if (bx < w) mv[((int64_t)f * h + by) * w + bx] = ri == INT_MAX ? (int64_t)SR * N + SR : (int64_t)ri;
    }
  }
}

// ---- two block rows per tile (IVC_ME_2ROW) --------------------------------------------------
// A tile is 8 adjacent blocks of block row by (top) and the 8 below them (bottom): 16 MFMA
// rows.  The bottom blocks' windows at dy' are the top blocks' windows at dy = dy' + 8 (the
// same reference rows), so one MFMA over the reference rows at offset R (R in [0, 40], rows
// yb + R .. of yb = 8 by - 16) serves the top blocks' candidates dy = R and the bottom blocks'
// dy' = R - 8.  Against one block row of 16: the window positions per tile drop from 160 to
// 96 (6 M-tiles), MFMAs per 16 blocks from 330 to 246, key formations from 660 to 528 register
// operations (a register is a quad of blocks: top 0-3, top 4-7, bottom 0-3, bottom 4-7, and a
// quad is live in 4 of the 6 M-tiles and for 33 of the 41 offsets R), and the LDS from 51.7 KB
// to 39.4 KB: 4 workgroups per CU instead of 3.  Ties and keys as in me_mfma16_kernel: rank =
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
      if (top && q23) acc[1] = max(acc[1], (int)(((uint32_t)d.y << 8) + e));
      if (bot && q01) acc[2] = max(acc[2], (int)(((uint32_t)d.z << 8) + e));
      if (bot && q23) acc[3] = max(acc[3], (int)(((uint32_t)d.w << 8) + e));
    }
  };
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
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
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
  for (; tile < ntiles; tile += gridDim.x) {
    uint32_t f;
    int by, bx0;
    tile_xy(tile, f, by, bx0);
    __syncthreads();                                   // the previous tile's LDS reads are done
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
      if (i < ITEMS) {
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
    __syncthreads();
    {
      // window energies E[R][u] = B + 128 (-S2') (me_mfma16_kernel's form), two threads per
      // column u: threads 0..95 the offsets R < 20 from rows 0..26, threads 128..223 the
      // offsets R >= 20 from rows 20..47 (each a prefix over its rows)
      const int half = tid >> 7, u = tid & 127;
      if (u < U) {
        const uint32_t* cw = lds + (u & 3) * COPY + (u >> 2);
        const int xb = 8 * bx0 - SR, yb = 8 * by - SR;
        const bool xok = xb + u >= 0 && xb + u + 8 <= W;
        const int rlo = half ? 20 : 0, rhi = half ? NR : 20;     // offsets of this thread
        auto energy = [&](auto hf) {
          constexpr int RL = decltype(hf)::value ? 20 : 0, RH = decltype(hf)::value ? NR : 20;
          int P[RH + 7 - RL + 1];
          int pr = 0;
#pragma unroll
          for (int r = RL; r < RH + 7; ++r) {
            const int w0 = (int)cw[r * PITCH], w1 = (int)cw[r * PITCH + 1];
            pr = __builtin_amdgcn_sdot4(w1, w1, __builtin_amdgcn_sdot4(w0, w0, pr, false), false);
            P[r - RL] = pr;
            if (r >= RL + 7) {
              const int R = r - 7;
              const int t = (r - 8 >= RL ? P[r - 8 - RL] : 0) - pr;
              const int wv = R < 11 ? 0 : (R - 1) / 10;
              const int rank = (R - wave_r0(wv)) * NMT + (u >> 4);
              const bool ok = xok && (unsigned)(yb + R) <= (unsigned)(H - 8);
              lds[E_OFF + R * U + u] = (uint32_t)((ok ? (1 << 27) + 127 - rank : E_OUT) + 128 * t);
            }
          }
        };
        (void)rlo;
        (void)rhi;
        if (half) energy(std::true_type{});
        else energy(std::false_type{});
      }
    }
    const mf_v4i bop = mf_v4i{L.bop.x ^ (int)0x80808080u, L.bop.y ^ (int)0x80808080u,
                              L.bop.z ^ (int)0x80808080u, L.bop.w ^ (int)0x80808080u};
    __syncthreads();
    load(tile + gridDim.x, L);                          // the next tile's inputs, in flight
    if (wave == 0) me2_search<0>(lds, red, wave, g, l16, bop);
    else if (wave == 3) me2_search<3>(lds, red, wave, g, l16, bop);
    else me2_search<1>(lds, red, wave, g, l16, bop);
    __syncthreads();
    if (tid < 16) {
      const int blk = tid, bx = bx0 + (blk & 7), byy = by + (blk >> 3);
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
        mv[((int64_t)f * h + byy) * w + bx] = ri == INT_MAX ? (int64_t)SR * N + SR : (int64_t)ri;
    }
  }
}

// One chunk of frame pairs on the matrix cores.  Returns false when the kernel does not apply
// (the caller keeps its own path): a frame of 2 GiB or more, or 2^31 tiles.
bool launch_me_mfma16(const uint8_t* ref, const uint8_t* cur, int64_t nf, int H, int W, int64_t* mv,
                      hipStream_t s) {
  if ((int64_t)H * W >= ((int64_t)1 << 31)) return false;
  const int h = H / 8, w = W / 8;
  if (IVC_ME_2ROW) {
    const int64_t tiles2 = nf * ((h + 1) / 2) * ((w + mf2::TBX - 1) / mf2::TBX);
    if (tiles2 <= 0) return true;
    if (tiles2 >= ((int64_t)1 << 31)) return false;
    int64_t grid = 2 * (int64_t)resident_grid_ptr(reinterpret_cast<const void*>(me_mfma16x2_kernel), tiles2);
    if (grid > tiles2) grid = tiles2;
    me_mfma16x2_kernel<<<(unsigned)grid, 256, 0, s>>>(ref, cur, nf, H, W, mv);
    return true;
  }
  const int64_t tiles = nf * h * ((w + mf::TB - 1) / mf::TB);
  if (tiles <= 0) return true;
  if (tiles >= ((int64_t)1 << 31)) return false;     // 32-bit tile counters
  int64_t grid = 2 * (int64_t)resident_grid_ptr(reinterpret_cast<const void*>(me_mfma16_kernel), tiles);
  if (grid > tiles) grid = tiles;
  me_mfma16_kernel<<<(unsigned)grid, 256, 0, s>>>(ref, cur, nf, H, W, mv);
  return true;
}

}  // namespace ivc
