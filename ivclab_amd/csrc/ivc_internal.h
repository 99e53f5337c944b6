// ivc_internal.h — launchers shared between the kernels (ivc_kernels.hip, ivc_motion.hip)
// and the C-ABI layer (ivc_capi.hip).  Not part of the public interface (include/ivc.h).
#pragma once
#include <mutex>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "../../include/ivc.h"

namespace ivc {

// The workgroup barrier of every kernel: the wave's own LDS operations drained, then the
// barrier.  hipcc (ROCm 7.2) leaves out the lgkmcnt(0) wait at some barriers (loop headers
// reached with LDS writes still in flight from the back edge), and on gfx950 another wave then
// occasionally reads the LDS word as it was before the write: me_mfma16x2_kernel's cross-wave
// merge picked up a stale per-wave result in 12 of 300 cfg5 steps, 0 of 450 with the wait
// (tools/race_probe.py, profiles/r05ai_race_probe.log).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// the per-device second stream of the pipelined calls (ivc_entropy.hip)
constexpr int PIPE_EVENTS = 66;
struct PipeCtx {
  hipStream_t aux = nullptr;
  hipEvent_t ev[PIPE_EVENTS] = {};
  std::mutex mu;
  bool ok = false;
};
hipError_t pipe_ctx(PipeCtx** out);
// Joins the second stream back into the caller's stream when a pipelined enqueue leaves early
// (an error after work was queued on it): the caller's later frees then wait for that work.
struct PipeJoin {
  PipeCtx& P;
  hipStream_t s;
  bool armed = false;
  ~PipeJoin() {
    if (!armed) return;
    (void)hipEventRecord(P.ev[PIPE_EVENTS - 1], P.aux);
    (void)hipStreamWaitEvent(s, P.ev[PIPE_EVENTS - 1], 0);
  }
};


// quantisation table as kernel argument (by value: no per-call upload on the stream)
//   q[p*64 + i*8 + k]  : table value in the calc dtype (exactly representable)
struct QTab {
  double q[192];
};

// ivc_set_tuning overrides (ivc_capi.hip): 0 = the library's own choice
int tuning(int key);

// error raised by a launcher; turned into a status + message by the C-ABI layer
struct Error {
  int code;
  const char* msg;
};

int dtype_size(int dtype);
bool dtype_is_float(int dtype);

// Completion signal of a tiny host call (ivc_capi.hip): the last workgroup of the kernel to
// finish — counted on `count` (device memory, left at 0) — stores `seq` into the page-locked
// word `flag` with a system-scope release after every workgroup's writes are visible.  A null
// `flag` (every other caller) adds nothing.  `inl` (host side only): the call's input, which
// the launcher passes inside the kernel arguments (TinyIn<N>, N = the launcher's capacity)
// when it fits: the kernel reads it from its argument segment instead of over the bus from
// host memory (~1 us less per call, tools/ubench/tiny_call.hip, profiles/r05i_tiny_call.log;
// each 512 B of arguments costs ~0.15 us of launch, so the capacity is sized per kernel).
constexpr int kTinyInline = 1536;    // the largest capacity: a (3, 8, 8) float64 stack
struct TinyDone {
  uint32_t* flag;
  uint32_t* count;
  uint32_t seq;
  const void* inl = nullptr;
  size_t inl_bytes = 0;
  void* stage = nullptr;             // the page-locked input block the kernel reads otherwise
};
template <int N>
struct TinyIn {
  uint32_t* flag;
  uint32_t* count;
  uint32_t seq;
  alignas(16) unsigned char in[N];
};
template <typename TD> struct IsTinyIn : std::false_type {};
template <int N> struct IsTinyIn<TinyIn<N>> : std::true_type {};
// launch f(TinyIn<N>) when the call's input travels in the arguments, else f(TinyDone);
// f returns the launch status.  An input offered inline but larger than this launcher's N is
// copied into the page-locked block first, so the kernel never reads a stale block whatever N
// the launcher chose (tests/test_gpu_parity.py::test_tiny_inline_capacity_mismatch).
template <int N = kTinyInline, typename F>
inline hipError_t with_tiny(const TinyDone* d, F&& f) {
  if (d && d->inl && d->inl_bytes <= (size_t)N) {
    TinyIn<N> t;
    t.flag = d->flag;
    t.count = d->count;
    t.seq = d->seq;
    __builtin_memcpy(t.in, d->inl, d->inl_bytes);
    return f(t);
  }
  if (d && d->inl && d->inl_bytes && d->stage) __builtin_memcpy(d->stage, d->inl, d->inl_bytes);
  return f(d ? *d : TinyDone{nullptr, nullptr, 0});
}
// the kernel's input: the argument segment's copy for a TinyIn launch
template <typename T, typename TD>
__device__ __forceinline__ const T* tiny_src(const T* src, const TD& d) {
  if constexpr (IsTinyIn<TD>::value) return reinterpret_cast<const T*>(d.in);
  else return src;
}
template <typename TD>
__device__ __forceinline__ void tiny_done(const TD& d) {
  if (d.flag == nullptr) return;                      // uniform
  __threadfence_system();                             // this thread's writes, system scope
  lds_barrier();
  if (threadIdx.x == 0) {
    if (gridDim.x == 1) {                             // the common tiny call: no counter
      __hip_atomic_store(d.flag, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    const uint32_t n = __hip_atomic_fetch_add(d.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (n == gridDim.x - 1) {
      __hip_atomic_store(d.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(d.flag, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// all launchers enqueue on `s` and return hipSuccess / the launch error
hipError_t launch_dct8x8(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
                         int inverse, int norm, hipStream_t s, const TinyDone* done = nullptr);
hipError_t launch_dct8x8_image(const void* img, int src_dtype, int64_t rows, int64_t W, int64_t C,
                               void* dst, int dst_dtype, int inverse, int norm, hipStream_t s);
// dtab (tiny calls only): a device copy of t the kernel reads instead of the argument copy
hipError_t launch_quantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                           int calc_dtype, int32_t* dst, hipStream_t s, const TinyDone* done = nullptr,
                           const double* dtab = nullptr);
hipError_t launch_dequantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                             int calc_dtype, int32_t* dst, hipStream_t s,
                             const TinyDone* done = nullptr, const double* dtab = nullptr);
hipError_t launch_zigzag(const void* src, int64_t nrow, int64_t stride, int esize, int inverse,
                         void* dst, hipStream_t s, const TinyDone* done = nullptr);
// returns hipErrorInvalidValue for an unsupported dtype / C combination
hipError_t launch_intra_encode(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                               int C, const QTab& t, int calc_dtype, int zigzag, int32_t* out,
                               hipStream_t s);
hipError_t launch_intra_encode_luma(const uint8_t* img, int64_t nframes, int64_t H, int64_t W,
                                    const QTab& t, int zigzag, int32_t* out, hipStream_t s);
// decode chain (ivc_decode.hip): [nblk][3][64] -> [nblk][3][8][8] f64, and
// [F][h][w][C][64] -> [F][H][W][3] f64 image (optionally ycbcr2rgb)
hipError_t launch_intra_decode(const int32_t* q, int64_t nblk, const QTab& t, int unzigzag,
                               double* out, hipStream_t s);
hipError_t launch_intra_decode_image(const int32_t* q, int64_t nframes, int64_t H, int64_t W,
                                     int C, const QTab& t, int unzigzag, int to_rgb, double* out,
                                     hipStream_t s, const int* skip = nullptr);
// fused zero-run symbols -> image (ivc_decode.hip) and its driver with the general fallback
// (ivc_entropy.hip)
hipError_t launch_sym_image(const int32_t* sym, int64_t n, int32_t eob, const uint32_t* eobmask,
                            const int64_t* tile_first, int64_t ntiles, int64_t nframes, int64_t H,
                            int64_t W, int C, const QTab& t, int to_rgb, double* out,
                            int64_t* gstart, int* fail, hipStream_t s);
hipError_t launch_sym_locate_range(const uint32_t* eobmask, const int64_t* tile_first, int64_t t0,
                                   int64_t t1, int64_t nframes, int64_t H, int64_t W, int C,
                                   int64_t* gstart, hipStream_t s);
hipError_t launch_sym_group_range(const int64_t* tile_first, int64_t tc0, int64_t tc1, int first,
                                  int last, int64_t nframes, int64_t H, int64_t W, int C,
                                  int64_t* range, hipStream_t s);
hipError_t launch_sym_image_range(const int32_t* sym, int64_t n, int32_t eob, int64_t nframes,
                                  int64_t H, int64_t W, int C, const QTab& t, int to_rgb,
                                  double* out, const int64_t* gstart, int* fail,
                                  const int64_t* grange, hipStream_t s);
int64_t sym_image_scratch_bytes(int64_t n, int64_t ngroups);
hipError_t launch_symbols2image(const int32_t* sym, int64_t n, int64_t nframes, int64_t H,
                                int64_t W, int C, const QTab& t, int32_t eob, int to_rgb,
                                double* out, int32_t* coef, void* scratch, int64_t* err,
                                hipStream_t s);
// store pacing of the fused coefficient kernels (ivc_kernels.hip): target total HBM GB/s, 0 = off
double store_pace_gbps();
double store_pace_late_fraction();
void set_store_pace_gbps(double gbps);
int store_pace_stats(int kind, double* out, int n);
void store_pace_reset_stats();
int store_pace_trace(int kind, double* out, int max_records);
void store_pace_settle(double margin);
// workgroups per CU of the histogram launches (ivc_kernels.hip)
int histogram_wg_per_cu();
void set_histogram_wg_per_cu(int k);
unsigned resident_grid_ptr(const void* kernel, int64_t work_groups_needed);
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s);
// zero-run coding (ivc_entropy.hip)
int64_t scan_scratch_elems(int64_t n);
hipError_t launch_exclusive_scan_i32(const int32_t* counts, int64_t n, int64_t* agg, int64_t* off,
                                     hipStream_t s);
hipError_t launch_exclusive_scan_i32_carry(const int32_t* counts, int64_t n, int64_t* agg,
                                           int64_t* off, hipStream_t s);
hipError_t launch_intra_symbols(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                                int C, const QTab& t, int32_t eob, int32_t* out, int64_t capacity,
                                int64_t* nsym, hipStream_t s, int64_t* hist = nullptr,
                                int32_t hist_lo = 0, int32_t hist_n = 0);
int64_t zerorun_scratch_bytes(int64_t nblk);
hipError_t launch_zerorun_offsets(const int32_t* src, int64_t nblk, int stride, int B,
                                  void* scratch, int64_t* off, hipStream_t s);
hipError_t launch_zerorun_emit(const int32_t* src, int64_t nblk, int stride, int B, int32_t eob,
                               void* scratch, int64_t* off, int32_t* out, int64_t capacity,
                               hipStream_t s);
// offsets + emission in one call (pipelined over chunks of groups for dense rows)
hipError_t launch_zerorun_encode(const int32_t* src, int64_t nblk, int stride, int B, int32_t eob,
                                 void* scratch, int64_t* off, int32_t* out, int64_t capacity,
                                 hipStream_t s);
int64_t zr_decode_scratch_bytes(int64_t n);
hipError_t launch_rgb2ycbcr(const void* src, int dtype, int64_t npix, double* dst, hipStream_t s);
hipError_t launch_ycbcr2rgb(const void* src, int dtype, int64_t npix, int64_t cstride, void* dst,
                            hipStream_t s);
hipError_t launch_rgb2gray(const void* src, int dtype, int64_t npix, int C, void* dst, hipStream_t s);
int huffman_lengths(const double* w, int32_t n, uint8_t* len);
int huffman_encode(const int32_t* sym, int64_t n, int32_t lo, const uint8_t* len, int32_t nalpha,
                   uint32_t* words, int64_t cap, int64_t* nbits);
int huffman_decode(const uint32_t* words, int64_t nwords, int64_t count, int32_t lo,
                   const uint8_t* len, int32_t nalpha, int32_t* out);
hipError_t launch_minmax_i32(const int32_t* sym, int64_t n, int32_t* mm, hipStream_t s);
hipError_t launch_zerorun_decode(const int32_t* sym, int64_t n, int64_t expected, int B,
                                 int32_t eob, int32_t* out, void* scratch, int64_t* err,
                                 hipStream_t s);
hipError_t launch_histogram_i64(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins,
                                int64_t* hist, hipStream_t s);
hipError_t launch_edge_histogram(const double* x, int64_t n, const double* edges, int32_t nedges,
                                 int64_t* counts, hipStream_t s);
hipError_t launch_histogram(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins,
                            int64_t* hist, hipStream_t s);

hipError_t launch_motion_estimate(const void* ref, const void* cur, int dtype, int64_t nframes,
                                  int64_t H, int64_t W, int sr, int mode, int64_t* mv,
                                  hipStream_t s);
// the matrix-core +-16 search of a batch (ivc_me_mfma.hip); false: not applicable (a frame of
// 2 GiB or more)
bool launch_me_mfma16(const uint8_t* ref, const uint8_t* cur, int64_t nf, int H, int W, int64_t* mv,
                      hipStream_t s);
hipError_t launch_motion_compensate(const void* ref, int esize, int64_t nframes, int64_t H,
                                    int64_t W, int64_t C, const int64_t* mv, int sr, void* out,
                                    hipStream_t s);
hipError_t launch_inter_residual(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W,
                                 int sr, const int64_t* mv, const QTab& t, int zigzag,
                                 int32_t* out, hipStream_t s, int64_t* hist = nullptr,
                                 int32_t hist_lo = 0, int32_t hist_n = 0);



// ---- float motion search geometry (ivc_motion.hip me_flt_kernel, ivc_me_f64.hip) ----
#ifndef IVC_FLT_DY
#define IVC_FLT_DY 11
#endif
#ifndef IVC_FLT_WGCU
#define IVC_FLT_WGCU 1     // f64 workgroups per CU (2 needs <= 128 VGPRs: FLT_DY 6)
#endif
constexpr int FLT_WG = 512, FLT_DY = IVC_FLT_DY;

// Round geometry: NBR blocks per round (2sr+1 threads each), capped so that the window, the
// blocks and the minimum arrays fit FLT_LDS bytes (the default per-workgroup LDS limit).
constexpr int FLT_LDS = 64 * 1024;
template <typename T, int SR> struct FltGeom {
  // WR window rows plus the rows a partial last dy run reads past them (zeros, never used)
  static constexpr int N = 2 * SR + 1, WR = 8 + 2 * SR;
  static constexpr int RUNS = (N + FLT_DY - 1) / FLT_DY, WRP = RUNS * FLT_DY + 7;
  // a block's 64 pixels at a pitch 16 B past 64 elements: the blocks a half-wave's 16-byte
  // reads broadcast from then start on different banks
  static constexpr int CBP = 64 + 16 / (int)sizeof(T);
  static constexpr int PER_NB = (WRP * 8 + CBP) * (int)sizeof(T) + (int)sizeof(T) + 4;
  static constexpr int NB_LDS = (FLT_LDS - WRP * 2 * SR * (int)sizeof(T)) / PER_NB;
  static constexpr int NBR = FLT_WG / N < NB_LDS ? FLT_WG / N : NB_LDS;
  static constexpr int WC = NBR * 8 + 2 * SR;
  static constexpr size_t LDS = ((size_t)WRP * WC + (size_t)NBR * CBP) * sizeof(T) +
                                (size_t)NBR * (sizeof(T) + 4);
  static_assert(NBR >= 1 && LDS <= (size_t)FLT_LDS, "round does not fit the LDS budget");
};

// The pruned float64 search (ivc_me_f64.hip) of nf frame pairs for sr in {4, 8, 16}: writes
// mv for the rounds it settles and appends the others to defer (defer[0] = their count, zeroed
// by the caller) for me_flt_kernel; defer_all appends every round.  False: sr not compiled.
bool launch_me_f64p(int sr, const double* ref, const double* cur, int64_t nf, int H, int W,
                    int64_t* mv, uint32_t* defer, int defer_all, hipStream_t s);


// ---- tiny-call server (ivc_kernels.hip tiny_server_kernel, ivc_capi.hip server_call) ----
// A resident one-wave kernel serving the reference's per-block calls (one (8, 8) DCT, one
// (C, 8, 8) quantise / dequantise) through a mailbox in coherent page-locked host memory,
// instead of one kernel launch per call.  Host -> device fields first, device -> host after;
// each group on its own 128-byte lines.
enum { SRV_DCT = 1, SRV_QUANT = 2, SRV_DEQUANT = 3 };
constexpr uint32_t SRV_STOP = 0xffffffffu;
constexpr int SRV_IO = 1536;                     // bytes of input and of output at most
// A request is read in one go: the header line and the whole input area, every poll (no
// dependent second read).  The host writes the header and the input, then a 64-bit checksum
// of them and of the sequence (srv_sum), then the sequence; the server acts on a poll only if
// the sequence is new and the checksum matches what it read, and polls again otherwise (a
// snapshot taken while the host was still writing).
struct SrvHdr {
  uint32_t req;                                  // request sequence (host writes last)
  uint32_t op, src_dtype, dst_dtype, inverse, ortho, C, tab_ver, nin, nout;
  double fct;
  uint64_t sum;                                  // srv_sum of words 0..5 and the input
  uint64_t pad;
};
static_assert(sizeof(SrvHdr) == 64, "one 64-byte header");
struct alignas(128) SrvBox {
  SrvHdr h;
  uint32_t pad0[16];
  alignas(128) uint64_t in[SRV_IO / 8];
  double tab[192];                               // the quantiser table of version tab_ver
  alignas(128) uint32_t done;                    // last request served (device writes last)
  uint32_t exited;                               // generation of the server that left its loop
  uint32_t pad3[30];
  alignas(128) uint64_t out[SRV_IO / 8];
};
__host__ __device__ inline uint64_t srv_mix(uint64_t w, uint32_t k) {
  return (w ^ ((uint64_t)(k + 1) * 0x9E3779B97F4A7C15ull)) * 0xD6E8FEB86659FD93ull;
}
hipError_t launch_tiny_server(SrvBox* box, uint32_t gen, uint64_t idle_ticks, uint64_t life_ticks,
                              hipStream_t s);

}  // namespace ivc
