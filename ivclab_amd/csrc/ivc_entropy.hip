// ivc_entropy.hip — zero-run coding of zig-zag blocks on gfx950 (ZeroRunCoder,
// ivclab/entropy/zerorun.py:10-88): the consumer of the fused encoder's zig-zag output and
// the producer of the Huffman alphabet.
//
// Encode (one wave per block, lane i = coefficient i): the block's nonzero mask is one
// wave ballot; the last nonzero index, the zero-run starts and the symbol count are scalar
// bit operations on that mask, and each lane finds its output slot with mbcnt (popcount of
// the mask bits below it).  Three passes: per-block symbol counts -> exclusive int64 scan
// -> emission at the block offsets.
//
// Decode: a symbol is a run-length slot iff it follows an odd number of consecutive zero
// symbols (the parse alternates value / run-length slots inside a run of zeros, and any
// nonzero symbol is followed by a value slot).  One max-scan types every slot; one scan of
// (EOB count, segmented intra-block length) places every value; the first block overflow
// in stream order and the end-of-stream cases reproduce the reference's errors.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <algorithm>
#include <mutex>
#include <type_traits>

#include "ivc_internal.h"

namespace ivc {

// A second stream (and events) per device for the pipelined calls (symbols2image, zero-run
// encode, inter encode; PipeCtx in ivc_internal.h): work on it is ordered against the caller's
// stream by events; the mutex serialises the enqueue of concurrent host threads.
#ifndef IVC_PIPE_PRIORITY
#define IVC_PIPE_PRIORITY 1
#endif
static PipeCtx g_pipe[64];
static std::once_flag g_pipe_once[64];
hipError_t pipe_ctx(PipeCtx** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  PipeCtx& P = g_pipe[dev];
  std::call_once(g_pipe_once[dev], [&P] {
    bool good;
    if (IVC_PIPE_PRIORITY) {
      // the highest priority: a queue of its own rather than one shared with the caller's
      // stream when the process has more streams than hardware queues (GPU_MAX_HW_QUEUES)
      int lo = 0, hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
      good = hipStreamCreateWithPriority(&P.aux, hipStreamNonBlocking, hi) == hipSuccess;
    } else {
      good = hipStreamCreateWithFlags(&P.aux, hipStreamNonBlocking) == hipSuccess;
    }
    for (auto& ev : P.ev)
      good = good && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
    P.ok = good;
  });
  if (!P.ok) return hipErrorNotInitialized;
  *out = &P;
  return hipSuccess;
}

// ---------------------------------------------------------------- generic tile scan ---
// Exclusive scan of gen(i), i in [0, n), with an associative Op over T; sink(i, excl, v)
// receives every element's exclusive prefix.  Three kernels: tile aggregates, an exclusive
// scan of the aggregates (one workgroup when they fit one tile, else the same scan applied to
// them, recursively), and the tile-local scan.  Each thread owns SCAN_I consecutive elements;
// the tile kernels loop over tiles (grid capped at SCAN_GRID workgroups).  `skip` (device
// int, may be null): when nonzero at launch every kernel returns at once (a decode whose fast
// path succeeded skips the general one without a host round trip).
constexpr int SCAN_T = 256, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;
constexpr int64_t SCAN_GRID = 256 * 8;

// (EOB value slots before, segment-contains-EOB flag, length since the last EOB): the
// decoder's scan state (declared here so the shuffle overloads precede the templates)
struct ZrState {
  int64_t blocks;
  int64_t reset;
  int64_t len;
};

__device__ __forceinline__ int64_t shfl_up_t(int64_t v, int d) {
  return (int64_t)__shfl_up((long long)v, (unsigned)d);
}
__device__ __forceinline__ ZrState shfl_up_t(const ZrState& v, int d) {
  return ZrState{shfl_up_t(v.blocks, d), shfl_up_t(v.reset, d), shfl_up_t(v.len, d)};
}

template <typename T, typename Op>
__device__ T wave_incl_scan(T v, Op op) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = shfl_up_t(v, d);
    if (lane >= d) v = op(o, v);
  }
  return v;
}

// exclusive scan of one value per thread over the 256-thread workgroup; returns the
// exclusive prefix, total = workgroup aggregate
template <typename T, typename Op>
__device__ T wg_excl_scan(T v, Op op, T* lds4, T& total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T incl = wave_incl_scan(v, op);
  if (lane == 63) lds4[wave] = incl;
  lds_barrier();
  T before = Op::identity();
  for (int w = 0; w < wave; ++w) before = op(before, lds4[w]);
  total = op(op(op(lds4[0], lds4[1]), lds4[2]), lds4[3]);
  lds_barrier();
  const T excl_in_wave = shfl_up_t(incl, 1);
  return op(before, lane == 0 ? Op::identity() : excl_in_wave);
}

template <typename T, typename Op, typename Gen>
__global__ __launch_bounds__(SCAN_T) void scan_tile_aggregate(int64_t n, Gen gen, Op op, T* agg,
                                                              const int* skip) {
  if (skip && *skip) return;
  __shared__ T lds4[4];
  const int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t i0 = t * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    T v = Op::identity();
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k)
      if (i0 + k < n) v = op(v, gen(i0 + k));
    T total;
    (void)wg_excl_scan(v, op, lds4, total);
    if (threadIdx.x == 0) agg[t] = total;
  }
}

// exclusive scan of at most SCAN_TILE tile aggregates in place (one workgroup); agg[ntiles] =
// total
template <typename T, typename Op>
__global__ __launch_bounds__(SCAN_T) void scan_aggregates(T* agg, int64_t ntiles, Op op,
                                                          const int* skip) {
  if (skip && *skip) return;
  __shared__ T lds4[4];
  T carry = Op::identity();
  for (int64_t base = 0; base < ntiles; base += SCAN_T) {
    const int64_t i = base + threadIdx.x;
    const T v = i < ntiles ? agg[i] : Op::identity();
    T total;
    const T ex = wg_excl_scan(v, op, lds4, total);
    if (i < ntiles) agg[i] = op(carry, ex);
    carry = op(carry, total);
  }
  if (threadIdx.x == 0) agg[ntiles] = carry;
}

template <typename T, typename Op, typename Gen, typename Sink>
__global__ __launch_bounds__(SCAN_T) void scan_tile_apply(int64_t n, Gen gen, Op op,
                                                          const T* agg, Sink sink,
                                                          const int* skip) {
  if (skip && *skip) return;
  __shared__ T lds4[4];
  const int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t i0 = t * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    T vals[SCAN_I];
    T v = Op::identity();
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
      vals[k] = i0 + k < n ? gen(i0 + k) : Op::identity();
      v = op(v, vals[k]);
    }
    T total;
    T run = op(agg[t], wg_excl_scan(v, op, lds4, total));
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
      if (i0 + k < n) sink(i0 + k, run, vals[k]);
      run = op(run, vals[k]);
    }
  }
}

// the recursive level: the aggregates themselves, scanned in place (each element is read and
// rewritten by the same thread), a[n] = total
template <typename T>
struct AggGen {
  const T* a;
  __device__ T operator()(int64_t i) const { return a[i]; }
};
template <typename T, typename Op>
struct AggSink {
  T* a;
  int64_t n;
  __device__ void operator()(int64_t i, const T& excl, const T& v) const {
    a[i] = excl;
    if (i == n - 1) a[n] = Op{}(excl, v);
  }
};

// elements of T the scan of n values needs as scratch: every level's aggregates + total
static int64_t scan_levels_elems(int64_t n) {
  const int64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  return nt + 1 + (nt > SCAN_TILE ? scan_levels_elems(nt) : 0);
}

// agg: device scratch of >= scan_levels_elems(n) elements
template <typename T, typename Op, typename Gen, typename Sink>
static hipError_t device_scan(int64_t n, Gen gen, Op op, Sink sink, T* agg, hipStream_t s,
                              const int* skip = nullptr) {
  if (n <= 0) return hipSuccess;
  const int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  const unsigned grid = (unsigned)(ntiles < SCAN_GRID ? ntiles : SCAN_GRID);
  scan_tile_aggregate<T, Op, Gen><<<grid, SCAN_T, 0, s>>>(n, gen, op, agg, skip);
  if (ntiles <= SCAN_TILE) {
    scan_aggregates<T, Op><<<1, SCAN_T, 0, s>>>(agg, ntiles, op, skip);
  } else {
    const hipError_t e = device_scan<T>(ntiles, AggGen<T>{agg}, op, AggSink<T, Op>{agg, ntiles},
                                        agg + ntiles + 1, s, skip);
    if (e != hipSuccess) return e;
  }
  scan_tile_apply<T, Op, Gen, Sink><<<grid, SCAN_T, 0, s>>>(n, gen, op, agg, sink, skip);
  return hipGetLastError();
}

int64_t scan_scratch_elems(int64_t n) { return scan_levels_elems(n); }

struct SumI64 {
  __device__ int64_t operator()(int64_t a, int64_t b) const { return a + b; }
  __device__ static int64_t identity() { return 0; }
};
struct MaxI64 {
  __device__ int64_t operator()(int64_t a, int64_t b) const { return a > b ? a : b; }
  __device__ static int64_t identity() { return INT64_MIN; }
};

// ---------------------------------------------------------------- encode --------------
// Per-block symbol stream of zerorun.py:18-38 from the 64-bit nonzero mask m of the first
// B coefficients: last = highest set bit; inside = bits [0, last]; run starts = zeros
// inside whose predecessor is nonzero (or i = 0); count = |m| + 2 |starts| + 1 (EOB).
struct ZrMask {
  uint64_t m, starts;
  int last;
};

__device__ __forceinline__ ZrMask zr_mask(int32_t x, bool valid) {
  ZrMask z;
  z.m = __ballot(valid && x != 0);
  z.last = z.m ? 63 - __builtin_clzll(z.m) : -1;
  const uint64_t inside = z.last < 0 ? 0ull : (z.last == 63 ? ~0ull : ((1ull << (z.last + 1)) - 1));
  const uint64_t zeros = ~z.m & inside;
  z.starts = zeros & ~(zeros << 1);
  return z;
}

__device__ __forceinline__ uint32_t popc_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// blocks handled per wave-iteration (independent loads in flight)
#ifndef IVC_ZR_UNROLL
#define IVC_ZR_UNROLL 4
#endif
constexpr int ZR_UNROLL = IVC_ZR_UNROLL;

__global__ __launch_bounds__(256) void zr_count_kernel(const int32_t* __restrict__ src,
                                                       int64_t nblk, int stride, int B,
                                                       int32_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const bool valid = lane < B;
  for (int64_t b0 = wave * ZR_UNROLL; b0 < nblk; b0 += nw * ZR_UNROLL) {
    int32_t x[ZR_UNROLL];
#pragma unroll
    for (int u = 0; u < ZR_UNROLL; ++u)
      x[u] = (valid && b0 + u < nblk) ? __builtin_nontemporal_load(src + (b0 + u) * stride + lane) : 0;
#pragma unroll
    for (int u = 0; u < ZR_UNROLL; ++u) {
      const ZrMask z = zr_mask(x[u], valid);
      if (lane == 0 && b0 + u < nblk)
        counts[b0 + u] = __builtin_popcountll(z.m) + 2 * __builtin_popcountll(z.starts) + 1;
    }
  }
}

struct CountGen {
  const int32_t* c;
  __device__ int64_t operator()(int64_t i) const { return c[i]; }
};
struct OffsetSink {
  int64_t* off;
  int64_t n;
  __device__ void operator()(int64_t i, int64_t excl, int64_t v) const {
    off[i] = excl;
    if (i == n - 1) off[n] = excl + v;
  }
};

// OffsetSink continuing a previous scan: every prefix plus *carry (the previous chunk's total,
// which the previous scan wrote at off[0]; thread 0 rewrites that same value)
struct OffsetCarrySink {
  int64_t* off;
  int64_t n;
  const int64_t* carry;
  __device__ void operator()(int64_t i, int64_t excl, int64_t v) const {
    const int64_t c = *carry;
    off[i] = excl + c;
    if (i == n - 1) off[n] = excl + v + c;
  }
};

__global__ __launch_bounds__(256) void zr_emit_kernel(const int32_t* __restrict__ src, int64_t nblk,
                                                      int stride, int B, int32_t eob,
                                                      const int64_t* __restrict__ off,
                                                      int32_t* __restrict__ out, int64_t capacity) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const bool valid = lane < B;
  for (int64_t b0 = wave * ZR_UNROLL; b0 < nblk; b0 += nw * ZR_UNROLL) {
    int32_t x[ZR_UNROLL];
#pragma unroll
    for (int u = 0; u < ZR_UNROLL; ++u)
      x[u] = (valid && b0 + u < nblk) ? __builtin_nontemporal_load(src + (b0 + u) * stride + lane) : 0;
#pragma unroll
    for (int u = 0; u < ZR_UNROLL; ++u) {
      const int64_t blk = b0 + u;
      if (blk >= nblk) break;
      const ZrMask z = zr_mask(x[u], valid);
      const int64_t base = off[blk];
      const int64_t cnt = __builtin_popcountll(z.m) + 2 * __builtin_popcountll(z.starts) + 1;
      // the stream is written only while it fits the caller's capacity
      const int64_t lim = capacity - base;
      const bool nz = __builtin_amdgcn_inverse_ballot_w64(z.m),      // lane bits of the masks
                 st = __builtin_amdgcn_inverse_ballot_w64(z.starts);
      const int64_t p = (int64_t)popc_below(z.m) + 2 * (int64_t)popc_below(z.starts);
      if (nz && p < lim) out[base + p] = x[u];
      if (st) {
        // run length = distance to the next nonzero coefficient (one exists: the run ends
        // before `last`)
        const int run = __builtin_ctzll(z.m >> lane);
        if (p < lim) out[base + p] = 0;
        if (p + 1 < lim) out[base + p + 1] = run;
      }
      if (lane == 0 && cnt - 1 < lim) out[base + cnt - 1] = eob;
    }
  }
}

static unsigned zr_grid(int64_t nblk) {
  const int64_t waves = (nblk + ZR_UNROLL - 1) / ZR_UNROLL;
  int64_t grid = (waves + 3) / 4;
  if (grid > 256 * 16) grid = 256 * 16;
  return (unsigned)(grid < 1 ? 1 : grid);
}

// ---- wide path: dense 64-coefficient rows (block_size = row stride = 64, 16-B aligned) --
// A wave takes ZW_BLK consecutive blocks per iteration with 16-byte loads: lane l holds
// coefficients 4(l%16) .. 4(l%16)+3 of block l/16 of each 4-block load.  A block's 64-bit
// nonzero mask is the OR over its 16 lanes of their nibbles (4 xor-shuffles), so every lane
// knows its block's mask, run starts and symbol count (same rules as zr_mask).  Emission
// assembles the ZW_BLK blocks' contiguous symbol range in the wave's LDS and stores it with
// consecutive-address whole-wave dword stores.
constexpr int ZW_LOADS = 4, ZW_BLK = 4 * ZW_LOADS;
constexpr int ZW_MAXSYM = 97;                 // symbols of a 64-coefficient block, at most
constexpr int ZW_STAGE = ZW_BLK * ZW_MAXSYM;  // int32 per wave

typedef int32_t zv4 __attribute__((ext_vector_type(4)));

struct ZwMask {
  uint64_t m, st;
  int cnt;
};

// OR over the 16 lanes of a DPP row (quad_perm 1,0,3,2; 2,3,0,1; row_half_mirror;
// row_mirror): VALU only, no LDS round trips
__device__ __forceinline__ uint32_t or_row16(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false);
  return v;
}

__device__ __forceinline__ ZwMask zw_mask(zv4 x, int lane) {
  const uint32_t nib = (uint32_t)(x.x != 0) | (uint32_t)(x.y != 0) << 1 |
                       (uint32_t)(x.z != 0) << 2 | (uint32_t)(x.w != 0) << 3;
  const int i = lane & 15;
  const uint32_t lo = or_row16(i < 8 ? nib << (4 * i) : 0u);
  const uint32_t hi = or_row16(i >= 8 ? nib << (4 * (i - 8)) : 0u);
  ZwMask z;
  z.m = (uint64_t)hi << 32 | lo;
  const int last = z.m ? 63 - __builtin_clzll(z.m) : -1;
  const uint64_t inside = last < 0 ? 0ull : (last == 63 ? ~0ull : ((1ull << (last + 1)) - 1));
  const uint64_t zeros = ~z.m & inside;
  z.st = zeros & ~(zeros << 1);
  z.cnt = __builtin_popcountll(z.m) + 2 * __builtin_popcountll(z.st) + 1;
  return z;
}

// Unconditional 16-byte load (past-the-end blocks read the last block and are dropped by
// the caller): no exec-masked loads, so the compiler's vmcnt waits stay exact.
__device__ __forceinline__ zv4 zw_load(const int32_t* src, int64_t nblk, int64_t b0, int u,
                                        int lane) {
  int64_t blk = b0 + 4 * u + (lane >> 4);
  blk = blk < nblk ? blk : nblk - 1;
  return __builtin_nontemporal_load(reinterpret_cast<const zv4*>(src + blk * 64) + (lane & 15));
}

// ---- dense rows through an int8 hand-off (r04) -------------------------------------------
// The two passes below read the 256-byte rows twice (count, emit).  With the hand-off the
// count pass (zw_count_kernel<true>) also stores each group's coefficients as int8 in its own
// register layout — lane (i, q)'s 16 bytes = coefficients 4i .. 4i + 3 of blocks q, 4 + q,
// 8 + q, 12 + q — or, for a group with a value outside int8, as int16 in a slot of a small side
// area.  The emission pass (zc_emit_kernel) reads 1 KB per group instead of 4 KB, turns it into
// lane k = coefficient k with one ds_bpermute per block, and places every block's symbols with
// ballot/mbcnt into the wave's LDS window, then stores the group's contiguous range.  A value
// outside int16 (or the int16 slots running out) sets `bad`: the emitter stands down and
// zw_emit_kernel runs from the int32 rows instead (gated on the device).
#ifndef IVC_ZC
#define IVC_ZC 1
#endif
#ifndef IVC_SLOT5
#define IVC_SLOT5 1   // emission slots: 4 mbcnt + a shift-add (0: 6 mbcnt)
#endif
#ifndef IVC_ZC_NT
#define IVC_ZC_NT 1
#endif
constexpr int ZC_BLK = 16;
constexpr int ZC_WIN = 1664;   // words per wave: the group's <= 16 x 97 symbols, padded

struct ZcScratch {
  uint8_t* c8;       // [ng][64 lanes][16 B], byte 4u + e = coefficient 4i + e of block 4u + q
  uint8_t* c16;      // [cap16][64 lanes][32 B], int16 j the same value as byte j
  int32_t* flag;     // [ng]: 0, or the group's int16 slot + 1
  int32_t* ctl;      // [0] int16 slots taken, [1] bad
  int64_t cap16;
};

// The wide path scans per-ZW_BLK-block group counts (nblk / 16 int32 written and scanned,
// not nblk); the emit pass derives each block's offset from its group's offset and the
// counts of the group's earlier blocks, and writes offsets[blk] itself.
#ifndef IVC_ZW_COUNT_GROUPS
#define IVC_ZW_COUNT_GROUPS 2   // 16-block groups per wave-iteration of the count pass (r05,
                                // pipelined call: 2 against 4, 10.33 -> 10.16 ms; 1: 10.33 ms,
                                // profiles/r05y_ab_zerorun_count_groups.log)
#endif
// groups [g_begin, g_end) (g_end < 0: all)
template <bool EXPORT>
__global__ __launch_bounds__(256) void zw_count_kernel(const int32_t* __restrict__ src, int64_t nblk,
                                                       int32_t* __restrict__ gcounts, ZcScratch z,
                                                       int64_t g_begin = 0, int64_t g_end = -1) {
  constexpr int NGR = IVC_ZW_COUNT_GROUPS;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t ng_all = (nblk + ZW_BLK - 1) / ZW_BLK;
  const int64_t ng = g_end < 0 || g_end > ng_all ? ng_all : g_end;
  for (int64_t b0 = (g_begin + wave * NGR) * ZW_BLK; b0 < ng * ZW_BLK; b0 += nw * ZW_BLK * NGR) {
    zv4 x[NGR * ZW_LOADS];
#pragma unroll
    for (int u = 0; u < NGR * ZW_LOADS; ++u) x[u] = zw_load(src, nblk, b0, u, lane);
#pragma unroll
    for (int g = 0; g < NGR; ++g) {
      int tot = 0;
#pragma unroll
      for (int l = 0; l < ZW_LOADS; ++l) {
        const int u = g * ZW_LOADS + l;
        const ZwMask zm = zw_mask(x[u], lane);
        const int c = b0 + 4 * u + (lane >> 4) < nblk ? zm.cnt : 0;
        // lanes 0, 16, 32, 48 hold the load's four blocks
        tot += __builtin_amdgcn_readlane(c, 0) + __builtin_amdgcn_readlane(c, 16) +
               __builtin_amdgcn_readlane(c, 32) + __builtin_amdgcn_readlane(c, 48);
      }
      const int64_t gi = b0 / ZW_BLK + g;
      if (lane == 0 && gi < ng) gcounts[gi] = tot;
      if constexpr (EXPORT) {
        if (gi < ng) {                                        // wave-uniform
          // (blocks past nblk in the last group hold the last block's values: never emitted)
          int32_t vlo = INT32_MAX, vhi = INT32_MIN;
          uint32_t w8[ZW_LOADS];
#pragma unroll
          for (int l = 0; l < ZW_LOADS; ++l) {
            const zv4 v = x[g * ZW_LOADS + l];
            w8[l] = ((uint32_t)v.x & 0xffu) | ((uint32_t)v.y & 0xffu) << 8 |
                    ((uint32_t)v.z & 0xffu) << 16 | ((uint32_t)v.w & 0xffu) << 24;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              vlo = min(vlo, v[e]);
              vhi = max(vhi, v[e]);
            }
          }
          const bool wide = vlo < -128 || vhi > 127, wider = vlo < -32768 || vhi > 32767;
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#if IVC_ZC_NT
          __builtin_nontemporal_store(u32x4{w8[0], w8[1], w8[2], w8[3]},
                                      reinterpret_cast<u32x4*>(z.c8 + (gi * 64 + lane) * 16));
#else
          *reinterpret_cast<u32x4*>(z.c8 + (gi * 64 + lane) * 16) = u32x4{w8[0], w8[1], w8[2], w8[3]};
#endif
          int flag = 0;
          if (__ballot(wide)) {                               // wave-uniform, rare
            if (__ballot(wider)) {
              if (lane == 0) atomicOr(z.ctl + 1, 1);
            } else {
              int slot = 0;
              if (lane == 0) slot = atomicAdd(z.ctl, 1);
              slot = __shfl(slot, 0);
              if (slot < z.cap16) {
                uint32_t w16[2 * ZW_LOADS];
#pragma unroll
                for (int l = 0; l < ZW_LOADS; ++l) {
                  const zv4 v = x[g * ZW_LOADS + l];
                  w16[2 * l] = ((uint32_t)v.x & 0xffffu) | ((uint32_t)v.y & 0xffffu) << 16;
                  w16[2 * l + 1] = ((uint32_t)v.z & 0xffffu) | ((uint32_t)v.w & 0xffffu) << 16;
                }
                u32x4* d16 = reinterpret_cast<u32x4*>(z.c16 + ((int64_t)slot * 64 + lane) * 32);
                d16[0] = u32x4{w16[0], w16[1], w16[2], w16[3]};
                d16[1] = u32x4{w16[4], w16[5], w16[6], w16[7]};
                flag = slot + 1;
              } else if (lane == 0) {
                atomicOr(z.ctl + 1, 1);
              }
            }
          }
          if (lane == 0) z.flag[gi] = flag;
        }
      }
    }
  }
}

#ifndef IVC_ZW_EMIT_GROUPS
#define IVC_ZW_EMIT_GROUPS 4   // 16-block groups loaded per wave-iteration of the emit pass (1: +11%, 8: +11%)
#endif
#ifndef IVC_ZW_STORE4
#define IVC_ZW_STORE4 1
#endif
// per wave: the symbols of a group staged at word (address of out[wbase] / 4 mod 4, so LDS
// and stream share 16-byte alignment), then each lane's dummy words (2, overlapping)
constexpr int ZW_STAGE_D = ZW_STAGE + 4 + 68;   // dummy words: 64 lanes + 1, padded to 16 B
__global__ __launch_bounds__(256) void zw_emit_kernel(const int32_t* __restrict__ src, int64_t nblk,
                                                      int32_t eob, const int64_t* __restrict__ goff,
                                                      int64_t* __restrict__ off,
                                                      int32_t* __restrict__ out, int64_t capacity,
                                                      const int32_t* run_if) {
  __shared__ __attribute__((aligned(16))) int32_t stage[4 * ZW_STAGE_D];
  if (run_if && *run_if == 0) return;           // (the int8 hand-off path emitted instead)
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  int32_t* const zbase = stage + (threadIdx.x >> 6) * ZW_STAGE_D;
  int32_t* const dummy = zbase + ZW_STAGE + 4 + (threadIdx.x & 63);
  const int i = lane & 15, q = lane >> 4;
  const uint64_t low = i == 0 ? 0ull : (~0ull >> (64 - 4 * i));   // positions below 4i
  constexpr int EG = IVC_ZW_EMIT_GROUPS;
  for (int64_t b00 = wave * ZW_BLK * EG; b00 < nblk; b00 += nw * ZW_BLK * EG) {
    zv4 xx[EG * ZW_LOADS];
#pragma unroll
    for (int u = 0; u < EG * ZW_LOADS; ++u) xx[u] = zw_load(src, nblk, b00, u, lane);
#pragma unroll
   for (int gg = 0; gg < EG; ++gg) {
    const int64_t b0 = b00 + gg * ZW_BLK;
    if (b0 >= nblk) break;                                        // wave-uniform
    const zv4* x = xx + gg * ZW_LOADS;
    const int64_t g = b0 / ZW_BLK;
    const int64_t wbase = goff[g], wend = goff[g + 1];
    // (the caller's stream need not start 16-byte aligned: the shift follows the address)
    const int sh = IVC_ZW_STORE4 ? (int)(((uintptr_t)(out + wbase) >> 2) & 3u) : 0;
    int32_t* const zs = zbase + sh;
    int run = 0;                                                  // symbols of earlier blocks
#pragma unroll
    for (int u = 0; u < ZW_LOADS; ++u) {
      const ZwMask z = zw_mask(x[u], lane);
      const int64_t blk = b0 + 4 * u + q;
      const bool live = blk < nblk;
      const int c = live ? z.cnt : 0;
      const int c0 = __builtin_amdgcn_readlane(c, 0), c1 = __builtin_amdgcn_readlane(c, 16),
                c2 = __builtin_amdgcn_readlane(c, 32), c3 = __builtin_amdgcn_readlane(c, 48);
      const int bpre = run + (q > 0 ? c0 : 0) + (q > 1 ? c1 : 0) + (q > 2 ? c2 : 0);
      run += c0 + c1 + c2 + c3;
      if (live) {
        if (i == 0) off[blk] = wbase + bpre;   // the block offsets: 4 x 8 B per load
        int p = bpre + __builtin_popcountll(z.m & low) + 2 * __builtin_popcountll(z.st & low);
        const int32_t v[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
        // two ds_write per coefficient at one address, no exec branches: first every slot
        // p + 1 (a run's length, or a don't-care), then every slot p (a value or a run's 0):
        // the slot after a single symbol is the first slot of the next symbol, written in the
        // second round (or the block's EOB, written after); lanes with nothing to write hit
        // their dummy words
        const uint32_t mb = (uint32_t)(z.m >> (4 * i)) & 15u, sb = (uint32_t)(z.st >> (4 * i)) & 15u;
        int32_t* d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool nz = (mb >> j) & 1u, rs = (sb >> j) & 1u;
          d[j] = nz || rs ? zs + p : dummy;
          p += (int)nz + 2 * (int)rs;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j][1] = __builtin_ctzll(z.m >> (4 * i + j));   // run length
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the rounds stay ordered
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j][0] = v[j];                // v[j] == 0 at a run start
        if (i == 0) zs[bpre + z.cnt - 1] = eob;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // the ZW_BLK blocks' symbols are the contiguous range [wbase, wend); written while they
    // fit the caller's capacity
    const int n = (int)(wend - wbase);
#if IVC_ZW_STORE4
    // 16-byte stores of the aligned quads (LDS words 4t .. 4t + 3 = stream words wbase - sh +
    // 4t ..); the partial quads at the ends and past capacity go word by word
    const int64_t A = wbase - sh;
    const int nq = (sh + n + 3) >> 2;
    for (int t = lane; t < nq; t += 64) {
      const int w0 = 4 * t;
      const int64_t ga = A + w0;
      if (w0 >= sh && w0 + 4 <= sh + n && ga + 4 <= capacity) {
        *reinterpret_cast<zv4*>(out + ga) = *reinterpret_cast<const zv4*>(zbase + w0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (w0 + e >= sh && w0 + e < sh + n && ga + e < capacity) out[ga + e] = zbase[w0 + e];
      }
    }
#else
    const int64_t lim = capacity - wbase;
    for (int k = lane; k < n; k += 64)
      if (k < lim) out[wbase + k] = zs[k];
#endif
    __builtin_amdgcn_wave_barrier();
   }
  }
}

// one wave per group; the block offsets off[blk] are written here (the scan wrote the group
// offsets and the stream length)
__global__ __launch_bounds__(256) void zc_emit_kernel(int64_t nblk, int32_t eob,
                                                      const int64_t* __restrict__ goff,
                                                      const uint8_t* __restrict__ c8,
                                                      const uint8_t* __restrict__ c16,
                                                      const int32_t* __restrict__ gflag,
                                                      const int32_t* __restrict__ bad,
                                                      int64_t* __restrict__ off,
                                                      int32_t* __restrict__ out, int64_t capacity,
                                                      int64_t g_begin = 0, int64_t g_end = -1) {
  __shared__ __attribute__((aligned(16))) int32_t win[4 * ZC_WIN];
  if (*bad) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t ng_all = (nblk + ZC_BLK - 1) / ZC_BLK;
  const int64_t ng = g_end < 0 || g_end > ng_all ? ng_all : g_end;
  int32_t* const os = win + wave * ZC_WIN;
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  struct Pre {
    int64_t base;
    int flag;
    i32x4 w;
  };
  auto fetch = [&](int64_t g, Pre& P) {
    P.base = goff[g];
    P.flag = gflag[g];
#if IVC_ZC_NT
    P.w = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(c8 + (g * 64 + lane) * 16));
#else
    P.w = *reinterpret_cast<const i32x4*>(c8 + (g * 64 + lane) * 16);
#endif
  };
  const int64_t g0 = g_begin + (int64_t)blockIdx.x * 4 + wave;
  Pre cur;
  if (g0 < ng) fetch(g0, cur);
  for (int64_t g = g0; g < ng; g += nw) {
    Pre nxt;
    if (g + nw < ng) fetch(g + nw, nxt);
    const int nb = (int)(nblk - g * ZC_BLK < ZC_BLK ? nblk - g * ZC_BLK : ZC_BLK);
    // lane k = coefficient k: block 4u + q's value comes from lane (k >> 2) + 16 q, dword u,
    // byte k & 3 (one ds_bpermute per block)
    int32_t xv[ZC_BLK];
    const int sel = (lane >> 2) * 4;
    if (cur.flag == 0) {
#pragma unroll
      for (int b = 0; b < ZC_BLK; ++b) {
        const int v = __builtin_amdgcn_ds_bpermute(sel + 64 * (b & 3), cur.w[b >> 2]);
        xv[b] = __builtin_amdgcn_sbfe(v, 8 * (lane & 3), 8);
      }
    } else {                                                  // rare: the group's int16 slot
      const i32x4* src = reinterpret_cast<const i32x4*>(c16 + ((int64_t)(cur.flag - 1) * 64 + lane) * 32);
      const i32x4 a0 = src[0], a1 = src[1];
      const int d[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int b = 0; b < ZC_BLK; ++b) {
        const int u = b >> 2;
        const int lo = __builtin_amdgcn_ds_bpermute(sel + 64 * (b & 3), d[2 * u]);
        const int hi = __builtin_amdgcn_ds_bpermute(sel + 64 * (b & 3), d[2 * u + 1]);
        xv[b] = __builtin_amdgcn_sbfe((lane & 2) ? hi : lo, 16 * (lane & 1), 16);
      }
    }
    int fill = 0, offv = 0;
#pragma unroll
    for (int b = 0; b < ZC_BLK; ++b) {
      if (b < nb) {                                           // wave-uniform
      // same slots and values as zr_group_emit_fit (ivc_kernels.hip): a nonzero, a run's 0 and
      // its length, or the EOB on the first zero after the last nonzero
      const int32_t x = xv[b];
      const bool nz = x != 0;
      const uint64_t m = __ballot(nz);
      const uint64_t later = m >> lane;
      const bool hl = later != 0;
      const uint64_t pm = (m << 1) | 1ull, hm = __ballot(hl);
      const uint64_t st = pm & hm & ~m;
      const bool pnz = __builtin_amdgcn_inverse_ballot_w64(pm);
      const bool rs = __builtin_amdgcn_inverse_ballot_w64(st);
      const int cnt = __builtin_popcountll(m) + 2 * __builtin_popcountll(st) + 1;
      // the lane's slot, fill included (mbcnt accumulates: m's bits below the lane, st's twice)
#if IVC_SLOT5
      uint32_t slot = __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)fill);
      slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), slot);
      uint32_t s2 = __builtin_amdgcn_mbcnt_lo((uint32_t)st, 0u);
      s2 = __builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), s2);
      slot += 2 * s2;
#else
      uint32_t slot = __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)fill);
      slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), slot);
      slot = __builtin_amdgcn_mbcnt_lo((uint32_t)st, slot);
      slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), slot);
      slot = __builtin_amdgcn_mbcnt_lo((uint32_t)st, slot);
      slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(st >> 32), slot);
#endif
      const bool w1 = nz || pnz;
      const int32_t v1 = nz || hl ? x : eob;
      // only the lanes with something to write touch LDS (exec-masked, so the idle lanes' words
      // no longer share banks with the block's slots): a value, a run's 0 or the EOB at the
      // slot; a run's length after it, or the EOB after a nonzero lane 63
      if (w1) os[slot] = v1;
      if (rs || (nz && lane == 63)) os[slot + 1] = rs ? (int32_t)__builtin_ctzll(later) : eob;
      offv = lane == b ? fill : offv;
      fill += cnt;
      }
    }
    if (lane < nb) off[g * ZC_BLK + lane] = cur.base + offv;
    __builtin_amdgcn_wave_barrier();
    // the group's symbols are the contiguous range [base, base + fill); stored while they fit
    // the caller's capacity (the buffer range drops the rest)
    const int64_t lim = capacity - cur.base;
    const int nst = (int)(lim < (int64_t)fill ? (lim > 0 ? lim : 0) : (int64_t)fill);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        out + (nst > 0 ? cur.base : 0), 0, 4 * nst, 0x00020000);
    for (int j0 = 0; j0 < fill; j0 += 64)
      __builtin_amdgcn_raw_buffer_store_b32(os[j0 + lane], ro, 4 * (j0 + lane), 0, 0);
    __builtin_amdgcn_wave_barrier();
    cur = nxt;
  }
}

static bool zw_ok(const int32_t* src, int stride, int B) {
  return stride == 64 && B == 64 && ((uintptr_t)src & 15u) == 0;
}

static unsigned zw_grid(int64_t nblk, int per_cu) {
  const int64_t waves = (nblk + ZW_BLK - 1) / ZW_BLK;
  int64_t grid = (waves + 3) / 4;
  if (grid > 256 * per_cu) grid = 256 * per_cu;
  return (unsigned)(grid < 1 ? 1 : grid);
}

// GroupOffsetSink continuing a previous chunk's scan (carry = its total, at goff[0] here)
struct GroupOffsetCarrySink {
  int64_t* goff;
  int64_t ng;
  const int64_t* carry;
  int64_t* total;             // the stream length, written by the last chunk only
  __device__ void operator()(int64_t i, int64_t excl, int64_t v) const {
    const int64_t c = *carry;
    goff[i] = excl + c;
    if (i == ng - 1) {
      goff[ng] = excl + v + c;
      if (total) *total = excl + v + c;
    }
  }
};

// group offsets goff[0..ng] and the stream length at off[nblk]
struct GroupOffsetSink {
  int64_t* goff;
  int64_t ng;
  int64_t* total;
  __device__ void operator()(int64_t i, int64_t excl, int64_t v) const {
    goff[i] = excl;
    if (i == ng - 1) {
      goff[ng] = excl + v;
      *total = excl + v;
    }
  }
};

// Scratch of launch_zerorun_offsets / launch_zerorun_emit: per-block int32 counts (generic
// path) or per-group int32 counts + int64 group offsets (wide path), and the scan's
// aggregates.
// + the int8 hand-off (zc_*): c8, per-group flags, 2 control words, int16 slots for 1 in 8
// groups (more wide groups send the call to zw_emit_kernel)
static int64_t zc_cap16(int64_t ng) { return ng / 8 + 64; }
static int64_t zr_base_bytes(int64_t nblk) {
  const int64_t ng = (nblk + ZW_BLK - 1) / ZW_BLK;
  const int64_t wide = ((4 * ng + 7) & ~int64_t(7)) + 8 * (ng + 1);
  const int64_t cnt = 4 * nblk > wide ? 4 * nblk : wide;
  return ((((cnt + 7) & ~int64_t(7)) + 8 * scan_scratch_elems(nblk)) + 255) & ~int64_t(255);
}
static int64_t zc_bytes(int64_t nblk) {
  const int64_t ng = (nblk + ZC_BLK - 1) / ZC_BLK;
  return 1024 * ng + ((4 * ng + 255) & ~int64_t(255)) + 256 + 2048 * zc_cap16(ng);
}
int64_t zerorun_scratch_bytes(int64_t nblk) {
  return zr_base_bytes(nblk) + (IVC_ZC ? zc_bytes(nblk) : 0);
}

namespace {
struct ZrScratch {
  int32_t* counts;   // per block (generic) or per group (wide)
  int64_t* goff;     // wide path: ng + 1 group offsets
  int64_t* agg;
  ZcScratch zc;
};
ZrScratch zr_scratch(void* scratch, int64_t nblk) {
  const int64_t ng = (nblk + ZW_BLK - 1) / ZW_BLK;
  const int64_t wide = ((4 * ng + 7) & ~int64_t(7)) + 8 * (ng + 1);
  const int64_t cnt = 4 * nblk > wide ? 4 * nblk : wide;
  char* b = (char*)scratch;
  ZrScratch z;
  z.counts = (int32_t*)b;
  z.goff = (int64_t*)(b + ((4 * ng + 7) & ~int64_t(7)));
  z.agg = (int64_t*)(b + ((cnt + 7) & ~int64_t(7)));
  char* c = b + zr_base_bytes(nblk);
  z.zc.c8 = (uint8_t*)c;
  c += 1024 * ng;
  z.zc.flag = (int32_t*)c;
  c += (4 * ng + 255) & ~int64_t(255);
  z.zc.ctl = (int32_t*)c;
  c += 256;
  z.zc.c16 = (uint8_t*)c;
  z.zc.cap16 = zc_cap16(ng);
  return z;
}
}  // namespace

// off[nblk] = stream length (always); the generic path also writes off[0..nblk) here, the
// wide path in launch_zerorun_emit.
hipError_t launch_zerorun_offsets(const int32_t* src, int64_t nblk, int stride, int B,
                                  void* scratch, int64_t* off, hipStream_t s) {
  if (nblk <= 0) return hipMemsetAsync(off, 0, sizeof(int64_t), s);
  const ZrScratch z = zr_scratch(scratch, nblk);
  if (zw_ok(src, stride, B)) {
    const int64_t ng = (nblk + ZW_BLK - 1) / ZW_BLK;
    if (IVC_ZC) {
      hipError_t e = hipMemsetAsync(z.zc.ctl, 0, 8, s);
      if (e != hipSuccess) return e;
      zw_count_kernel<true><<<zw_grid((nblk + IVC_ZW_COUNT_GROUPS - 1) / IVC_ZW_COUNT_GROUPS, 8), 256, 0, s>>>(
          src, nblk, z.counts, z.zc);
    } else {
      zw_count_kernel<false><<<zw_grid((nblk + IVC_ZW_COUNT_GROUPS - 1) / IVC_ZW_COUNT_GROUPS, 8), 256, 0, s>>>(
          src, nblk, z.counts, z.zc);
    }
    return device_scan<int64_t>(ng, CountGen{z.counts}, SumI64{}, GroupOffsetSink{z.goff, ng, off + nblk},
                                z.agg, s);
  }
  zr_count_kernel<<<zr_grid(nblk), 256, 0, s>>>(src, nblk, stride, B, z.counts);
  return device_scan<int64_t>(nblk, CountGen{z.counts}, SumI64{}, OffsetSink{off, nblk}, z.agg, s);
}

// off[0..n] = exclusive int64 prefix of counts[0..n), off[n] = total (agg: scratch of
// scan_scratch_elems(n) int64)
hipError_t launch_exclusive_scan_i32(const int32_t* counts, int64_t n, int64_t* agg, int64_t* off,
                                     hipStream_t s) {
  if (n <= 0) return hipMemsetAsync(off, 0, sizeof(int64_t), s);
  return device_scan<int64_t>(n, CountGen{counts}, SumI64{}, OffsetSink{off, n}, agg, s);
}

// off[0..n] = off[0] + exclusive int64 prefix of counts[0..n): a chunk of a longer scan whose
// earlier chunks left their total at off[0] (the pipelined pixels -> symbols call)
hipError_t launch_exclusive_scan_i32_carry(const int32_t* counts, int64_t n, int64_t* agg,
                                           int64_t* off, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return device_scan<int64_t>(n, CountGen{counts}, SumI64{},
                              GroupOffsetCarrySink{off, n, off, nullptr}, agg, s);
}

// symbols of every block at its offset; symbols at or past `capacity` are not written.
// `scratch` is launch_zerorun_offsets' (same src/nblk).
hipError_t launch_zerorun_emit(const int32_t* src, int64_t nblk, int stride, int B, int32_t eob,
                               void* scratch, int64_t* off, int32_t* out, int64_t capacity,
                               hipStream_t s) {
  if (nblk <= 0) return hipSuccess;
  if (zw_ok(src, stride, B)) {
    const ZrScratch z = zr_scratch(scratch, nblk);
    if (IVC_ZC)
      zc_emit_kernel<<<zw_grid(nblk, 6), 256, 0, s>>>(nblk, eob, z.goff, z.zc.c8, z.zc.c16, z.zc.flag,
                                                      z.zc.ctl + 1, off, out, capacity);
    zw_emit_kernel<<<zw_grid((nblk + IVC_ZW_EMIT_GROUPS - 1) / IVC_ZW_EMIT_GROUPS, 6), 256, 0, s>>>(
        src, nblk, eob, z.goff, off, out, capacity, IVC_ZC ? z.zc.ctl + 1 : nullptr);
  } else {
    zr_emit_kernel<<<zr_grid(nblk), 256, 0, s>>>(src, nblk, stride, B, eob, off, out, capacity);
  }
  return hipGetLastError();
}

// Zero-run encode in one call (ivc_zerorun_encode_dev): dense rows through the int8 hand-off are
// pipelined over K chunks of groups — on the caller's stream chunk j's count pass, on the second
// stream its scan (continuing chunk j - 1's total) and then its emission, so the memory-bound
// count pass of chunk j + 1 overlaps the issue-bound emission of chunk j.  Other rows: the two
// passes in order.
#ifndef IVC_ZR_CHUNKS
#define IVC_ZR_CHUNKS 32
#endif
#ifndef IVC_ZR_COUNT_WGCU
#define IVC_ZR_COUNT_WGCU 8     // the pipelined call's workgroups per CU: count pass
#endif
#ifndef IVC_ZR_EMIT_WGCU
#define IVC_ZR_EMIT_WGCU 5      // and emission (6: 10.41 / 10.15 ms against 10.18 / 9.86 ms for 5 on
#endif                          // two boxes; several other pairs fall to 13-15 ms: the two
                                // streams' grids then serialise — profiles/r05x/z/aa_ab_zerorun_*)
#ifndef IVC_ZR_MIN_CHUNK
#define IVC_ZR_MIN_CHUNK 98304
#endif
hipError_t launch_zerorun_encode(const int32_t* src, int64_t nblk, int stride, int B, int32_t eob,
                                 void* scratch, int64_t* off, int32_t* out, int64_t capacity,
                                 hipStream_t s) {
  const int64_t ng = (nblk + ZW_BLK - 1) / ZW_BLK;
  int K = IVC_ZR_CHUNKS;
  if (K > PIPE_EVENTS - 2) K = PIPE_EVENTS - 2;
  // groups per chunk at least (64 x 4K frames: 3.02 ms unpipelined, 2.85 with 16 chunks of 97 K
  // groups, 3.15 with 32 of 48 K — profiles/r04aq_ab_small_batch.log)
  if (ng / IVC_ZR_MIN_CHUNK < K) K = (int)(ng / IVC_ZR_MIN_CHUNK);
  if (K < 1) K = 1;
  if (const int f = tuning(IVC_TUNE_ZR_CHUNKS)) K = std::min(f, PIPE_EVENTS - 2);  // any size
  if (!IVC_ZC || !zw_ok(src, stride, B)) K = 1;
  if (K <= 1) {
    hipError_t e = launch_zerorun_offsets(src, nblk, stride, B, scratch, off, s);
    if (e == hipSuccess) e = launch_zerorun_emit(src, nblk, stride, B, eob, scratch, off, out, capacity, s);
    return e;
  }
  PipeCtx* pp = nullptr;
  hipError_t e = pipe_ctx(&pp);
  if (e != hipSuccess) return e;
  PipeCtx& P = *pp;
  std::lock_guard<std::mutex> lock(P.mu);
  const ZrScratch z = zr_scratch(scratch, nblk);
  if ((e = hipMemsetAsync(z.zc.ctl, 0, 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(z.goff, 0, 8, s)) != hipSuccess) return e;
  if ((e = hipEventRecord(P.ev[PIPE_EVENTS - 2], s)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(P.aux, P.ev[PIPE_EVENTS - 2], 0)) != hipSuccess) return e;
  PipeJoin join{P, s, true};
  // chunks of whole NGR-group batches so no count wave straddles two chunks
  const int64_t unit = IVC_ZW_COUNT_GROUPS;
  const int64_t per = ((ng + K - 1) / K + unit - 1) / unit * unit;
  for (int j = 0; j < K; ++j) {
    const int64_t g0 = std::min<int64_t>((int64_t)j * per, ng), g1 = std::min<int64_t>(g0 + per, ng);
    if (g1 <= g0) break;
    const int64_t len = g1 - g0;
    zw_count_kernel<true><<<zw_grid((len * ZW_BLK + IVC_ZW_COUNT_GROUPS - 1) / IVC_ZW_COUNT_GROUPS, IVC_ZR_COUNT_WGCU), 256, 0, s>>>(
        src, nblk, z.counts, z.zc, g0, g1);
    // the chunk's scan on the second stream ahead of its emission, so the caller's stream runs
    // the count passes back to back (small scan kernels there waited behind the high-priority
    // emission: 11.00 -> 10.65 ms, profiles/r04al_ab_zerorun_scan_aux.log)
    if ((e = hipEventRecord(P.ev[j], s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(P.aux, P.ev[j], 0)) != hipSuccess) return e;
    e = device_scan<int64_t>(len, CountGen{z.counts + g0}, SumI64{},
                             GroupOffsetCarrySink{z.goff + g0, len, z.goff + g0,
                                                  g1 == ng ? off + nblk : nullptr},
                             z.agg, P.aux);
    if (e != hipSuccess) return e;
    zc_emit_kernel<<<zw_grid(len * ZW_BLK, IVC_ZR_EMIT_WGCU), 256, 0, P.aux>>>(nblk, eob, z.goff, z.zc.c8, z.zc.c16,
                                                              z.zc.flag, z.zc.ctl + 1, off, out,
                                                              capacity, g0, g1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  join.armed = false;
  if ((e = hipEventRecord(P.ev[PIPE_EVENTS - 1], P.aux)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(s, P.ev[PIPE_EVENTS - 1], 0)) != hipSuccess) return e;
  // a value outside int16 anywhere (or the int16 slots ran out): every group from the int32 rows
  zw_emit_kernel<<<zw_grid((nblk + IVC_ZW_EMIT_GROUPS - 1) / IVC_ZW_EMIT_GROUPS, 6), 256, 0, s>>>(
      src, nblk, eob, z.goff, off, out, capacity, z.zc.ctl + 1);
  return hipGetLastError();
}

// ---------------------------------------------------------------- decode --------------
// Slot typing: lastnz(i) = index of the last nonzero symbol before i (max-scan); slot i is
// a run-length slot iff i - 1 - lastnz(i) is odd.
struct NzPosGen {
  const int32_t* s;
  __device__ int64_t operator()(int64_t i) const { return s[i] != 0 ? i : -1; }
};
struct RlTypeSink {
  uint8_t* is_rl;
  __device__ void operator()(int64_t i, int64_t excl, int64_t) const {
    const int64_t last = excl < -1 ? -1 : excl;     // identity (no nonzero before) -> -1
    is_rl[i] = (uint8_t)(((i - 1 - last) & 1) != 0);
  }
};

// segmented scan: the EOB value slot resets the length and contributes 0 to it
struct ZrOp {
  __device__ ZrState operator()(const ZrState& a, const ZrState& b) const {
    ZrState r;
    r.blocks = a.blocks + b.blocks;
    r.reset = a.reset | b.reset;
    r.len = b.reset ? b.len : a.len + b.len;
    return r;
  }
  __device__ static ZrState identity() { return ZrState{0, 0, 0}; }
};

__device__ __forceinline__ int64_t zr_run_of(const int32_t* s, int64_t i, int64_t n) {
  if (i + 1 >= n) return 0;
  const int64_t r = s[i + 1];
  return r < 0 ? 0 : r;      // [0] * negative = []
}

struct ZrGen {
  const int32_t* s;
  const uint8_t* is_rl;
  int64_t n;
  int32_t eob;
  __device__ ZrState operator()(int64_t i) const {
    if (is_rl[i]) return ZrState{0, 0, 0};
    const int32_t v = s[i];
    if (v == eob) return ZrState{1, 1, 0};
    return ZrState{0, 0, v == 0 ? zr_run_of(s, i, n) : 1};
  }
};

struct ZrSink {
  const int32_t* s;
  const uint8_t* is_rl;
  int64_t n, expected;
  int B;
  int32_t eob;
  int32_t* out;
  unsigned long long* first_overflow;   // (slot << 32) | length, minimum over overflows
  __device__ void operator()(int64_t i, const ZrState& ex, const ZrState& v) const {
    if (is_rl[i] || ex.blocks >= expected) return;
    const int32_t sym = s[i];
    if (sym == eob) return;
    const int64_t pos = ex.len;                       // length of the block before slot i
    const int64_t after = pos + v.len;                // len(block) after this slot
    if (sym != 0 && pos < B) out[ex.blocks * B + pos] = sym;
    if (sym == 0 && i + 1 >= n) return;               // ends after a zero: handled at the end
    if (after > B) {
      const uint64_t L = after > 0xffffffffll ? 0xffffffffull : (uint64_t)after;
      atomicMin(first_overflow, ((unsigned long long)i << 32) | L);
    }
  }
};

// err[0] = code (0 ok, 1 block size exceeded, 2 unexpected end, 3 ended right after a zero
// symbol, 4 too few blocks), err[1], err[2] = message arguments
__device__ void zr_decode_verdict_body(const int32_t* s, const uint8_t* is_rl, int64_t n,
                                       int64_t expected, int32_t eob, const ZrState* total,
                                       const unsigned long long* first_overflow, int64_t* err) {
  const unsigned long long ov = *first_overflow;
  int64_t code = 0, a0 = 0, a1 = 0;
  const int64_t got = n > 0 ? total->blocks : 0;
  if (ov != ~0ull) {
    code = 1;
    a0 = (int64_t)(ov & 0xffffffffull);
  } else if (got < expected) {
    const bool last_value = n > 0 && !is_rl[n - 1];
    if (n > 0 && last_value && s[n - 1] == 0) {
      code = 3;
      a0 = n;
    } else if (n == 0 || (last_value && s[n - 1] == eob)) {
      code = 4;
      a0 = expected;
      a1 = got;
    } else {
      code = 2;
    }
  }
  err[0] = code;
  err[1] = a0;
  err[2] = a1;
}

struct ZrTotalSink {
  ZrState* total;
  int64_t n;
  __device__ void operator()(int64_t i, const ZrState& ex, const ZrState& v) const {
    if (i == n - 1) *total = ZrOp{}(ex, v);
  }
};

template <typename A, typename B2>
struct BothSinks {
  A a;
  B2 b;
  __device__ void operator()(int64_t i, const ZrState& ex, const ZrState& v) const {
    a(i, ex, v);
    b(i, ex, v);
  }
};

// ---- fast decode of well-formed streams ----------------------------------------------
// In a stream with no two adjacent zero symbols and no run length <= 0 — every stream the
// encoder emits — slot i is a run-length slot iff symbol i - 1 is 0 (a zero can then only be
// a value slot: a zero run-length slot would follow a zero value slot), so typing is local
// and the EOB value slots (the block ends) are symbols equal to eob after a nonzero.  Two
// passes: (1) per tile of ZF_TILE symbols, count the EOB slots and test the two conditions
// (16-byte loads, one read of the stream); an int64 scan of the tile counts gives each tile's
// first block; (2) per tile, the blocks whose EOB lies in it (the first one starts in the
// previous tile: a halo of ZF_HALO symbols, longer than any block) are expanded one per wave
// iteration — lane j takes symbol j of the block, its coefficient count (1 for a nonzero
// value, the run length for a zero, 0 for a run-length slot) is prefix-summed across the
// wave, and the nonzero values land in a zeroed 64-entry row written with one coalesced
// store.  Any violation (a block longer than B coefficients or than the halo, fewer blocks
// than expected, adjacent zeros, a non-positive run, eob = 0) sets `fail`, and the general
// decoder above runs instead (its kernels read the verdict on the device: no host round
// trip), so errors and their messages are the general decoder's.
constexpr int ZF_TILE = 4096, ZF_HALO = 128;

// (eobmask, optional: bit i of word t * 128 + i / 32 = symbol t * ZF_TILE + i is an EOB slot —
// the symbols -> image path locates its groups from it)
// The next tile's loads are issued before this tile is counted (a wave has 8 KB of reads in
// flight instead of 4: one load latency per tile measured 3.3 ms for the cfg3 stream, 4.3 TB/s).
// symbol offset inside the tile of lane `lane` of wave w at step k (a wave-contiguous quarter
// per wave, the predecessor of a lane-0 quad from lane 63's previous step, measured the same)
__device__ __forceinline__ int zf_off(int w, int k, int lane) { return (k * 256 + w * 64 + lane) * 4; }
struct ZfTile {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  i32x4 q[ZF_TILE / 1024];
  int p0[ZF_TILE / 1024];
};
__device__ __forceinline__ void zf_load_tile(const int32_t* __restrict__ s, int64_t n, int64_t t,
                                             int w, int lane, ZfTile& T) {
#pragma unroll
  for (int k = 0; k < ZF_TILE / 1024; ++k) {
    const int64_t i = t * ZF_TILE + zf_off(w, k, lane);
    if (i + 3 < n) {
      T.q[k] = __builtin_nontemporal_load(reinterpret_cast<const ZfTile::i32x4*>(s + i));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) T.q[k][e] = i + e < n ? s[i + e] : 1;
    }
    // the symbol before the wave's first: one scalar load per wave (a wave-uniform address),
    // issued with the quads — not a per-lane load (one dword load per lane doubled the vector
    // memory instructions), nor a lane-0 vector load after the quad (a second latency)
    {
      const int64_t iw = t * ZF_TILE + zf_off(w, k, 0);
      T.p0[k] = iw > 0 && iw <= n ? s[iw - 1] : 1;   // the stream's first slot is a value slot
    }
  }
}
// tiles [t_begin, t_end) (t_end < 0: to the stream's end)
__global__ __launch_bounds__(256) void zf_count_kernel(const int32_t* __restrict__ s, int64_t n,
                                                       int32_t eob, int32_t* __restrict__ tile_eobs,
                                                       int* fail, uint32_t* __restrict__ eobmask,
                                                       int64_t t_begin = 0, int64_t t_end = -1) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t ntiles = t_end < 0 ? (n + ZF_TILE - 1) / ZF_TILE : t_end;
  ZfTile cur;
  if (t_begin + (int64_t)blockIdx.x < ntiles) zf_load_tile(s, n, t_begin + blockIdx.x, w, lane, cur);
  for (int64_t t = t_begin + blockIdx.x; t < ntiles; t += gridDim.x) {
    ZfTile nxt;
    if (t + gridDim.x < ntiles) zf_load_tile(s, n, t + gridDim.x, w, lane, nxt);
    int cnt = 0;
    bool bad = false;
    // a tile wholly inside the stream needs no per-symbol bounds test (all but the last)
    auto count_tile = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
      for (int k = 0; k < ZF_TILE / 1024; ++k) {
        const int off = zf_off(w, k, lane);
        const int64_t i = t * ZF_TILE + off;
        const int v[4] = {cur.q[k].x, cur.q[k].y, cur.q[k].z, cur.q[k].w};
        // the symbol before: the previous lane's last (DPP), lane 0's from the scalar load
        int pv = __builtin_amdgcn_update_dpp(cur.p0[k], v[3], 0x138, 0xf, 0xf, false);   // wave_shr:1
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (FULL || i + e < n) {
            const bool eb = v[e] == eob && pv != 0;
            bits |= eb ? 1u << e : 0u;
            bad |= pv == 0 && v[e] <= 0;
          }
          pv = v[e];
        }
        cnt += __builtin_popcount(bits);
        if (eobmask) {
          // 8 lanes' nibbles make one word: OR by DPP (quad_perm 1,0,3,2 / 2,3,0,1, row_half_mirror)
          bits <<= 4 * (lane & 7);
          bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xf, 0xf, false);
          bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x4E, 0xf, 0xf, false);
          bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x141, 0xf, 0xf, false);
          if ((lane & 7) == 0) eobmask[t * (ZF_TILE / 32) + off / 32] = bits;
        }
      }
    };
    if ((t + 1) * ZF_TILE <= n) count_tile(std::true_type{});
    else count_tile(std::false_type{});
    // the wave's count by DPP (no LDS: an LDS wait would also wait for the prefetched scalar load)
    cnt += __builtin_amdgcn_update_dpp(0, cnt, 0x111, 0xf, 0xf, false);   // row_shr:1
    cnt += __builtin_amdgcn_update_dpp(0, cnt, 0x112, 0xf, 0xf, false);   // row_shr:2
    cnt += __builtin_amdgcn_update_dpp(0, cnt, 0x114, 0xf, 0xf, false);   // row_shr:4
    cnt += __builtin_amdgcn_update_dpp(0, cnt, 0x118, 0xf, 0xf, false);   // row_shr:8
    cnt += __builtin_amdgcn_update_dpp(0, cnt, 0x142, 0xa, 0xf, false);   // row_bcast:15
    cnt += __builtin_amdgcn_update_dpp(0, cnt, 0x143, 0xc, 0xf, false);   // row_bcast:31
    const int wc = __builtin_amdgcn_readlane(cnt, 63);
    if (__ballot(bad) && lane == 0) atomicOr(fail, 1);
    if (lane == 0 && wc) atomicAdd(tile_eobs + t, wc);      // tile_eobs zeroed by the caller
    cur = nxt;
  }
}

// inclusive prefix sum over the wave by DPP (no LDS round trips): Hillis-Steele inside each
// row of 16 lanes (row_shr 1, 2, 4, 8), then row_bcast:15 carries row 0 into row 1 and row 2
// into row 3, row_bcast:31 carries rows 0-1 into rows 2-3 (CDNA keeps the GFX9 broadcasts)
__device__ __forceinline__ int zf_wave_incl_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return v;
}

__global__ __launch_bounds__(256) void zf_expand_kernel(const int32_t* __restrict__ s, int64_t n,
                                                        int32_t eob, int B,
                                                        const int64_t* __restrict__ tile_first,
                                                        int64_t expected, int32_t* __restrict__ out,
                                                        int* fail) {
  __shared__ __attribute__((aligned(16))) int32_t sh[ZF_HALO + ZF_TILE + 4];
  __shared__ int32_t epos[ZF_TILE];         // EOB slots of the tile, relative to the halo start
  __shared__ int32_t rows[4][64];
  __shared__ int cnt_w[4], last_halo;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t ntiles = (n + ZF_TILE - 1) / ZF_TILE;
  constexpr int PER = ZF_TILE / 256;        // tile symbols per thread (EOB compaction)
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t T0 = t * ZF_TILE, T1 = T0 + ZF_TILE < n ? T0 + ZF_TILE : n;
    const int64_t h0 = T0 - ZF_HALO > 0 ? T0 - ZF_HALO : 0;
    const int len = (int)(T1 - h0);          // symbols staged (halo + tile)
    const int hl = (int)(T0 - h0);           // halo length
    {
      // 16-byte loads, all in flight before the first LDS write (h0 is a multiple of 4 and
      // the stream 16-byte aligned; the quad past the stream's end goes element by element)
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      constexpr int NQ = (ZF_HALO + ZF_TILE) / 4 / 256 + 1;
      i32x4 q[NQ];
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int j = 4 * (tid + 256 * k);
        if (j + 3 < len) {
          q[k] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(s + h0 + j));
        } else {
          q[k] = i32x4{0, 0, 0, 0};
          for (int e = 0; e < 4; ++e)
            if (j + e < len) q[k][e] = s[h0 + j + e];
        }
      }
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int j = 4 * (tid + 256 * k);
        if (j < len) *reinterpret_cast<i32x4*>(sh + j) = q[k];
      }
    }
    if (tid == 0) last_halo = T0 == 0 ? -1 : -2;
    lds_barrier();
    auto is_eob = [&](int j) {               // j relative to h0, symbol h0 + j
      return sh[j] == eob && (h0 + j == 0 || sh[j - 1] != 0);
    };
    // the last EOB of the halo: where the tile's first block starts
    if (tid < hl && is_eob(tid)) atomicMax(&last_halo, tid);
    // EOB slots of the tile, compacted in stream order (thread = PER consecutive symbols)
    const int j0 = hl + tid * PER;
    int c = 0;
#pragma unroll
    for (int e = 0; e < PER; ++e) c += (j0 + e < len && is_eob(j0 + e)) ? 1 : 0;
    const int incl = zf_wave_incl_sum(c);
    if (lane == 63) cnt_w[wave] = incl;
    lds_barrier();
    int before = 0;
    for (int w = 0; w < wave; ++w) before += cnt_w[w];
    const int m = cnt_w[0] + cnt_w[1] + cnt_w[2] + cnt_w[3];
    int o = before + incl - c;
#pragma unroll
    for (int e = 0; e < PER; ++e)
      if (j0 + e < len && is_eob(j0 + e)) epos[o++] = j0 + e;
    lds_barrier();
    if (m > 0 && last_halo == -2 && tid == 0) atomicOr(fail, 1);   // a block longer than the halo
    const int64_t first = tile_first[t];
    for (int k = wave; k < m; k += 4) {
      const int64_t blk = first + k;
      if (blk >= expected) break;
      const int st = (k == 0 ? last_halo : epos[k - 1]) + 1, en = epos[k];
      const int bl = en - st;                // symbols before the EOB
      int32_t* row = rows[wave];
      row[lane] = 0;
      if (bl > 128 || st < 0) {              // only in a malformed stream
        if (lane == 0) atomicOr(fail, 1);
        continue;
      }
      int carry = 0;
      bool over = false;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int j = half * 64 + lane;
        const bool valid = j < bl;
        const int cur = valid ? sh[st + j] : 1;
        const int pv = j == 0 ? 1 : sh[st + j - 1];
        const bool rl = valid && pv == 0;
        // a run length counts min(run, B + 1): one past B already makes the block overflow,
        // and the clamp keeps the int32 scan from wrapping on a malformed huge run (a run
        // <= 0 is flagged by zf_count; clamping it to 0 keeps `pos` inside the row)
        const int rn = cur == 0 ? min(max(sh[st + j + 1], 0), B + 1) : 1;
        const int cc = !valid || rl ? 0 : rn;
        const int inc = zf_wave_incl_sum(cc);
        const int pos = carry + inc - cc;
        if (valid && !rl && cur != 0 && pos < B) row[pos] = cur;
        carry += __builtin_amdgcn_readlane(inc, 63);
        if (bl <= 64) break;
      }
      over = carry > B;
      __builtin_amdgcn_wave_barrier();
      if (over) {
        if (lane == 0) atomicOr(fail, 1);
      } else if (lane < B) {
        out[blk * B + lane] = row[lane];
      }
      __builtin_amdgcn_wave_barrier();
    }
    lds_barrier();
  }
}

// ok = the fast decode stands (no violation, enough blocks): err = 0; else the general
// decoder runs (its kernels see ok == 0)
__global__ void zf_finish(const int* fail, const int64_t* total_eobs, int64_t expected, int* ok,
                          int64_t* err) {
  const bool good = *fail == 0 && *total_eobs >= expected;
  *ok = good ? 1 : 0;
  if (good) {
    err[0] = 0;
    err[1] = 0;
    err[2] = 0;
  }
}

__global__ void zr_zero_fill(int32_t* out, int64_t count, const int* skip) {
  if (skip && *skip) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256)
    out[i] = 0;
}

__global__ void zr_decode_verdict_gated(const int32_t* s, const uint8_t* is_rl, int64_t n,
                                        int64_t expected, int32_t eob, const ZrState* total,
                                        const unsigned long long* first_overflow, int64_t* err,
                                        const int* skip) {
  if (skip && *skip) return;
  zr_decode_verdict_body(s, is_rl, n, expected, eob, total, first_overflow, err);
}

namespace {
constexpr int S2I_MAX_CHUNKS = 256;   // (events reused modulo PIPE_EVENTS - 2: a wait binds at enqueue)
struct ZrDecScratch {
  uint8_t* is_rl;
  int64_t* agg;
  ZrState* zagg;
  ZrState* total;
  unsigned long long* ovf;
  int32_t* tile_eobs;
  int64_t* tile_first;      // ntf + 1
  int64_t* fagg;
  int* flags;               // [0] fail, [1] ok
  uint32_t* eobmask;        // symbols -> image: ntf * ZF_TILE / 32 words
  int64_t* gstart;          // symbols -> image: ngroups + 1
  int64_t* grange;          // symbols -> image, pipelined: [S2I_MAX_CHUNKS][2] group ranges
};
int64_t align16(int64_t b) { return (b + 15) / 16 * 16; }
ZrDecScratch zr_dec_scratch(void* scratch, int64_t n, int64_t* bytes, int64_t ngroups = -1) {
  const int64_t nt = scan_scratch_elems(n);
  const int64_t ntf = (n + ZF_TILE - 1) / ZF_TILE;
  uint8_t* b = (uint8_t*)scratch;
  ZrDecScratch z;
  int64_t o = 0;
  z.is_rl = b + o; o += align16(n);
  z.agg = (int64_t*)(b + o); o += align16(nt * 8);
  z.zagg = (ZrState*)(b + o); o += align16(nt * (int64_t)sizeof(ZrState));
  z.total = (ZrState*)(b + o); o += align16(sizeof(ZrState));
  z.ovf = (unsigned long long*)(b + o); o += 16;
  z.tile_eobs = (int32_t*)(b + o); o += align16(ntf * 4);
  z.tile_first = (int64_t*)(b + o); o += align16((ntf + 1) * 8);
  z.fagg = (int64_t*)(b + o); o += align16(scan_scratch_elems(ntf) * 8);
  z.flags = (int*)(b + o); o += 16;
  z.eobmask = nullptr;
  z.gstart = nullptr;
  z.grange = nullptr;
  if (ngroups >= 0) {
    z.eobmask = (uint32_t*)(b + o); o += align16(ntf * (ZF_TILE / 32) * 4);
    z.gstart = (int64_t*)(b + o); o += align16((ngroups + 1) * 8);
    z.grange = (int64_t*)(b + o); o += align16(S2I_MAX_CHUNKS * 2 * 8);
  }
  if (bytes) *bytes = o;
  return z;
}
}  // namespace

int64_t zr_decode_scratch_bytes(int64_t n) {
  int64_t bytes = 0;
  (void)zr_dec_scratch(nullptr, n, &bytes);
  return bytes;
}

static hipError_t zr_decode_general(const ZrDecScratch& z, const int32_t* sym, int64_t n,
                                    int64_t expected, int B, int32_t eob, int32_t* out,
                                    int64_t* err, const int* skip, hipStream_t s);

hipError_t launch_zerorun_decode(const int32_t* sym, int64_t n, int64_t expected, int B,
                                 int32_t eob, int32_t* out, void* scratch, int64_t* err,
                                 hipStream_t s) {
  const ZrDecScratch z = zr_dec_scratch(scratch, n, nullptr);
  hipError_t e;
  const int* skip = nullptr;
  if (n > 0 && expected > 0 && B >= 1 && B <= 64 && eob != 0 && ((uintptr_t)sym & 15) == 0) {
    const int64_t ntf = (n + ZF_TILE - 1) / ZF_TILE;
    const unsigned grid = (unsigned)(ntf < 256 * 8 ? ntf : 256 * 8);
    if ((e = hipMemsetAsync(z.flags, 0, 16, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(z.tile_eobs, 0, (size_t)ntf * 4, s)) != hipSuccess) return e;
    zf_count_kernel<<<grid, 256, 0, s>>>(sym, n, eob, z.tile_eobs, z.flags, nullptr);
    e = device_scan<int64_t>(ntf, CountGen{z.tile_eobs}, SumI64{}, OffsetSink{z.tile_first, ntf},
                             z.fagg, s);
    if (e != hipSuccess) return e;
    zf_expand_kernel<<<grid, 256, 0, s>>>(sym, n, eob, B, z.tile_first, expected, out, z.flags);
    zf_finish<<<1, 1, 0, s>>>(z.flags, z.tile_first + ntf, expected, z.flags + 1, err);
    skip = z.flags + 1;
  }
  return zr_decode_general(z, sym, n, expected, B, eob, out, err, skip, s);
}

// the general decoder (every stream; skipped on the device when the fast one stood)
static hipError_t zr_decode_general(const ZrDecScratch& z, const int32_t* sym, int64_t n,
                                    int64_t expected, int B, int32_t eob, int32_t* out,
                                    int64_t* err, const int* skip, hipStream_t s) {
  hipError_t e;
  if ((e = hipMemsetAsync(z.ovf, 0xff, sizeof(unsigned long long), s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(z.total, 0, sizeof(ZrState), s)) != hipSuccess) return e;
  const int64_t nz = expected * B;
  if (nz > 0) {
    const int64_t g = (nz + 255) / 256;
    zr_zero_fill<<<(unsigned)(g < 256 * 16 ? g : 256 * 16), 256, 0, s>>>(out, nz, skip);
  }
  if (n > 0) {
    e = device_scan<int64_t>(n, NzPosGen{sym}, MaxI64{}, RlTypeSink{z.is_rl}, z.agg, s, skip);
    if (e != hipSuccess) return e;
    ZrSink place{sym, z.is_rl, n, expected, B, eob, out, z.ovf};
    e = device_scan<ZrState>(n, ZrGen{sym, z.is_rl, n, eob}, ZrOp{},
                             BothSinks<ZrSink, ZrTotalSink>{place, ZrTotalSink{z.total, n}}, z.zagg,
                             s, skip);
    if (e != hipSuccess) return e;
  }
  zr_decode_verdict_gated<<<1, 1, 0, s>>>(sym, z.is_rl, n, expected, eob, z.total, z.ovf, err, skip);
  return hipGetLastError();
}

// IntraCodec.symbols2image on the device (intracodec.py:84-146): a well-formed stream goes
// through the fused symbols -> image kernel (ivc_decode.hip: the coefficients stay in LDS);
// otherwise — decided on the device — the general zero-run decoder fills `coef` and the
// coefficient -> image kernel runs, so errors are the general decoder's.
int64_t sym_image_scratch_bytes(int64_t n, int64_t ngroups) {
  int64_t bytes = 0;
  (void)zr_dec_scratch(nullptr, n, &bytes, ngroups);
  return bytes;
}

// ivc_set_tuning(IVC_TUNE_S2I_NO_FALLBACK, 1) (see launch_symbols2image)
static bool s2i_no_fallback() { return tuning(IVC_TUNE_S2I_NO_FALLBACK) == 1; }

constexpr int64_t IVC_S2I_REJECTED = -100;
__global__ void s2i_rejected_verdict(const int* ok, int64_t* err) {
  if (*ok) return;
  err[0] = IVC_S2I_REJECTED;
  err[1] = 0;
  err[2] = 0;
}

// Pipelined symbols -> image: the stream is cut into K chunks of tiles; on the caller's stream
// chunk j's EOB count, its tile scan (continuing chunk j - 1's totals) and its group starts
// run in order, and on a second stream the decode of the groups chunk j - 1 owns starts as soon
// as chunk j's starts are known (its last group ends in chunk j) — so the stream pass of chunk
// j + 1 overlaps the decode of chunk j - 1 (the decode leaves VGPRs and wave slots for it).
#ifndef IVC_S2I_CHUNKS
#define IVC_S2I_CHUNKS 64        // with the 13 K-tile minimum: cfg3 (865 K tiles) in 64 chunks,
#endif                           // 64 frames in 16 (r05: 15.30 -> 15.13 and 3.918 -> 3.890 ms
                                 // against 32 / 16 K, profiles/r05ar_ab_decode_chunking.log)
#ifndef IVC_S2I_COUNT_WGCU
#define IVC_S2I_COUNT_WGCU 2     // the pipelined call's EOB pass: workgroups per CU (2: 14.89,
                                 // 4: 14.93, 6: 17.47 (the streams serialise), 8: 15.08 ms,
                                 // profiles/r05ab_ab_decode_count_grid.log)
#endif
#ifndef IVC_S2I_MIN_CHUNK
#define IVC_S2I_MIN_CHUNK 13312
#endif
static int s2i_chunks(int64_t ntf) {
  // ivc_set_tuning(IVC_TUNE_S2I_CHUNKS, K) pipelines any stream of >= K tiles
  if (const int f = tuning(IVC_TUNE_S2I_CHUNKS)) {
    int K = f;
    if (K > S2I_MAX_CHUNKS) K = S2I_MAX_CHUNKS;
    if (ntf < K) K = (int)ntf;
    return K < 1 ? 1 : K;
  }
  int K = IVC_S2I_CHUNKS;
  if (K > S2I_MAX_CHUNKS) K = S2I_MAX_CHUNKS;
  // stream tiles per chunk at least (64 x 4K frames, 216 K tiles: 4.25 ms in one pass, 4.10
  // with 8 or 16 chunks, 4.18 with 32 — profiles/r04ar_ab64_decode_chunks.log)
  if (ntf / IVC_S2I_MIN_CHUNK < K) K = (int)(ntf / IVC_S2I_MIN_CHUNK);
  return K < 1 ? 1 : K;
}

static hipError_t s2i_pipelined(const int32_t* sym, int64_t n, int32_t eob, int64_t ntf, int K,
                                int64_t nframes, int64_t H, int64_t W, int C, const QTab& t,
                                int to_rgb, double* out, const ZrDecScratch& z, hipStream_t s) {
  PipeCtx* pp = nullptr;
  hipError_t e = pipe_ctx(&pp);
  if (e != hipSuccess) return e;
  PipeCtx& P = *pp;
  std::lock_guard<std::mutex> lock(P.mu);
  const int64_t ngroups = nframes * (H / 8) * ((W / 8 + 7) / 8);
  if ((e = hipMemsetAsync(z.gstart, 0xff, (size_t)(ngroups + 1) * 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(z.tile_first, 0, 8, s)) != hipSuccess) return e;
  if ((e = hipEventRecord(P.ev[PIPE_EVENTS - 2], s)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(P.aux, P.ev[PIPE_EVENTS - 2], 0)) != hipSuccess) return e;
  PipeJoin join{P, s, true};
  const int64_t per = (ntf + K - 1) / K;
  auto tile0 = [&](int j) { return std::min<int64_t>((int64_t)j * per, ntf); };
  for (int j = 0; j < K; ++j) {
    const int64_t a = tile0(j), b = tile0(j + 1);
    if (b > a) {
      const int64_t len = b - a;
      const unsigned grid = (unsigned)(len < 256 * IVC_S2I_COUNT_WGCU ? len : 256 * IVC_S2I_COUNT_WGCU);
      zf_count_kernel<<<grid, 256, 0, s>>>(sym, n, eob, z.tile_eobs, z.flags, z.eobmask, a, b);
      e = device_scan<int64_t>(len, CountGen{z.tile_eobs + a}, SumI64{},
                               OffsetCarrySink{z.tile_first + a, len, z.tile_first + a}, z.fagg, s);
      if (e == hipSuccess)
        e = launch_sym_locate_range(z.eobmask, z.tile_first, a, b, nframes, H, W, C, z.gstart, s);
      if (e != hipSuccess) return e;
    }
    // chunk j's group range (its E bounds are final now)
    if ((e = launch_sym_group_range(z.tile_first, a, b, j == 0, j == K - 1, nframes, H, W, C,
                                    z.grange + 2 * j, s)) != hipSuccess)
      return e;
    hipEvent_t evj = P.ev[j % (PIPE_EVENTS - 2)];
    if ((e = hipEventRecord(evj, s)) != hipSuccess) return e;
    if (j >= 1) {                                  // chunk j - 1's groups end by chunk j's starts
      if ((e = hipStreamWaitEvent(P.aux, evj, 0)) != hipSuccess) return e;
      if ((e = launch_sym_image_range(sym, n, eob, nframes, H, W, C, t, to_rgb, out, z.gstart,
                                      z.flags, z.grange + 2 * (j - 1), P.aux)) != hipSuccess)
        return e;
    }
  }
  if ((e = launch_sym_image_range(sym, n, eob, nframes, H, W, C, t, to_rgb, out, z.gstart, z.flags,
                                  z.grange + 2 * (K - 1), P.aux)) != hipSuccess)
    return e;
  join.armed = false;
  if ((e = hipEventRecord(P.ev[PIPE_EVENTS - 1], P.aux)) != hipSuccess) return e;
  return hipStreamWaitEvent(s, P.ev[PIPE_EVENTS - 1], 0);
}

hipError_t launch_symbols2image(const int32_t* sym, int64_t n, int64_t nframes, int64_t H,
                                int64_t W, int C, const QTab& t, int32_t eob, int to_rgb,
                                double* out, int32_t* coef, void* scratch, int64_t* err,
                                hipStream_t s) {
  const int64_t w = W / 8, gpr = (w + 7) / 8;
  const int64_t ngroups = nframes * (H / 8) * gpr;
  const int64_t expected = nframes * (H / 8) * w * C;     // block-planes
  const ZrDecScratch z = zr_dec_scratch(scratch, n, nullptr, ngroups);
  hipError_t e;
  const int* skip = nullptr;
  if (n > 0 && expected > 0 && eob != 0 && ((uintptr_t)sym & 15) == 0) {
    const int64_t ntf = (n + ZF_TILE - 1) / ZF_TILE;
    if ((e = hipMemsetAsync(z.flags, 0, 16, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(z.tile_eobs, 0, (size_t)ntf * 4, s)) != hipSuccess) return e;
    const int K = s2i_chunks(ntf);
    if (K <= 1) {
      const unsigned grid = (unsigned)(ntf < 256 * 8 ? ntf : 256 * 8);
      zf_count_kernel<<<grid, 256, 0, s>>>(sym, n, eob, z.tile_eobs, z.flags, z.eobmask);
      e = device_scan<int64_t>(ntf, CountGen{z.tile_eobs}, SumI64{}, OffsetSink{z.tile_first, ntf},
                               z.fagg, s);
      if (e != hipSuccess) return e;
      e = launch_sym_image(sym, n, eob, z.eobmask, z.tile_first, ntf, nframes, H, W, C, t, to_rgb,
                           out, z.gstart, z.flags, s);
      if (e != hipSuccess) return e;
    } else if ((e = s2i_pipelined(sym, n, eob, ntf, K, nframes, H, W, C, t, to_rgb, out, z, s)) !=
               hipSuccess) {
      return e;
    }
    zf_finish<<<1, 1, 0, s>>>(z.flags, z.tile_first + ntf, expected, z.flags + 1, err);
    skip = z.flags + 1;
  }
  // (ivc_set_tuning(IVC_TUNE_S2I_NO_FALLBACK, 1): the fused kernel's image stands alone, so a test can
  // tell that it — not the general path — produced the image; when the fused path rejects the
  // stream, err[0] = IVC_S2I_REJECTED instead of the general decoder's verdict)
  if (skip && s2i_no_fallback()) {
    s2i_rejected_verdict<<<1, 1, 0, s>>>(skip, err);
    return hipGetLastError();
  }
  e = zr_decode_general(z, sym, n, expected, 64, eob, coef, err, skip, s);
  if (e != hipSuccess) return e;
  return launch_intra_decode_image(coef, nframes, H, W, C, t, 1, to_rgb, out, s, skip);
}

// ---------------------------------------------------------------- symbol range --------
// min / max of an int32 stream: the Huffman alphabet bounds of IntraCodec
// (ivclab/image/intracodec.py:161-163 takes min - 20, max + 20 + 1).
__global__ void minmax_init(int32_t* mm) {
  mm[0] = INT32_MAX;
  mm[1] = INT32_MIN;
}

// 16 B per lane, 4 loads in flight (after an unaligned head; the tail by workgroup 0)
__global__ __launch_bounds__(256) void minmax_kernel(const int32_t* __restrict__ sym, int64_t n,
                                                     int32_t* mm) {
  int32_t lo = INT32_MAX, hi = INT32_MIN;
  auto see = [&](int32_t v) {
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  };
  const int tid = threadIdx.x;
  int64_t head = (int64_t)(((16u - ((uintptr_t)sym & 15u)) & 15u) / 4u);
  if (head > n) head = n;
  if (blockIdx.x == 0 && tid < head) see(sym[tid]);
  sym += head;
  n -= head;
  typedef int32_t v4 __attribute__((ext_vector_type(4)));
  const v4* sv = reinterpret_cast<const v4*>(sym);
  const int64_t nv = n / 4, stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + tid;
  for (; i + 3 * stride < nv; i += 4 * stride) {
    v4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(sv + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      see(x[u].x); see(x[u].y); see(x[u].z); see(x[u].w);
    }
  }
  for (; i < nv; i += stride) {
    const v4 x = __builtin_nontemporal_load(sv + i);
    see(x.x); see(x.y); see(x.z); see(x.w);
  }
  if (blockIdx.x == 0 && tid < (int)(n - nv * 4)) see(sym[nv * 4 + tid]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const int32_t ol = __shfl_xor(lo, d), oh = __shfl_xor(hi, d);
    lo = ol < lo ? ol : lo;
    hi = oh > hi ? oh : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

hipError_t launch_minmax_i32(const int32_t* sym, int64_t n, int32_t* mm, hipStream_t s) {
  minmax_init<<<1, 1, 0, s>>>(mm);
  if (n > 0) {
    int64_t g = (n + 256 * 64 - 1) / (256 * 64);
    if (g > 256 * 4) g = 256 * 4;
    minmax_kernel<<<(unsigned)g, 256, 0, s>>>(sym, n, mm);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- edge histogram ----
// stats_marg's np.histogram(image.astype(float64).flatten(), bins=edges) (entropy.py:22-25)
// for any sorted float64 edges: value x counts in bin i when edges[i] <= x < edges[i+1], the
// last bin closed (x == edges[-1] counts in it), everything else (outside, NaN) dropped —
// the comparisons np.histogram's searchsorted path makes, exactly.  Per value: a binary
// search for the first edge > x.  Edges and per-workgroup counts in LDS when they fit
// (EDGE_LDS_MAX edges), else the edges are read through the caches and the counts go to
// global atomics.
constexpr int EDGE_LDS_MAX = 4096;

template <bool LDS>
__global__ __launch_bounds__(256) void edge_histogram_kernel(const double* __restrict__ x,
                                                             int64_t n,
                                                             const double* __restrict__ edges_g,
                                                             int nedges,
                                                             unsigned long long* __restrict__ counts) {
  __shared__ double e_s[LDS ? EDGE_LDS_MAX : 1];
  __shared__ unsigned int c_s[LDS ? EDGE_LDS_MAX : 1];
  const int nb = nedges - 1;
  const double* edges = edges_g;
  if (LDS) {
    for (int i = threadIdx.x; i < nedges; i += 256) e_s[i] = edges_g[i];
    for (int i = threadIdx.x; i < nb; i += 256) c_s[i] = 0;
    lds_barrier();
    edges = e_s;
  }
  const double lo = edges[0], hi = edges[nb];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = __builtin_nontemporal_load(x + i);
    if (!(v >= lo && v <= hi)) continue;                  // outside or NaN: dropped
    int b;
    if (v == hi) {
      b = nb - 1;                                         // the closed last bin
    } else {
      int l = 0, r = nedges;                              // first edge > v lies in (0, nedges)
      while (r - l > 1) {
        const int m = (l + r) >> 1;
        if (edges[m] <= v) l = m; else r = m;
      }
      b = l;
    }
    if (LDS) atomicAdd(&c_s[b], 1u);
    else atomicAdd(&counts[b], 1ull);
  }
  if (LDS) {
    lds_barrier();
    for (int j = threadIdx.x; j < nb; j += 256)
      if (c_s[j]) atomicAdd(&counts[j], (unsigned long long)c_s[j]);
  }
}

hipError_t launch_edge_histogram(const double* x, int64_t n, const double* edges, int32_t nedges,
                                 int64_t* counts, hipStream_t s) {
  if (n <= 0 || nedges < 2) return hipSuccess;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  int64_t g = (n + 256 * 16 - 1) / (256 * 16);
  if (g > (int64_t)cus * 4) g = (int64_t)cus * 4;
  if (g < 1) g = 1;
  auto* c = reinterpret_cast<unsigned long long*>(counts);
  if (nedges <= EDGE_LDS_MAX) edge_histogram_kernel<true><<<(unsigned)g, 256, 0, s>>>(x, n, edges, nedges, c);
  else edge_histogram_kernel<false><<<(unsigned)g, 256, 0, s>>>(x, n, edges, nedges, c);
  return hipGetLastError();
}

}  // namespace ivc
