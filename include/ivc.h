/*
 * ivc.h — C-ABI of the MI355X-native ivclab block-codec core (libivc.so).
 *
 * The reference (n2oblife/ivclab) is pure Python/NumPy and has no FFI of its own; the
 * drop-in boundary is its Python class API.  Every entry point below replaces the body of
 * one reference method (cited per function); the Python host mirror in ivclab_amd/ keeps
 * the reference signatures and calls these through ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only.  No torch / numpy types in any signature.
 *  - Return value: IVC_OK (0) on success, a negative IVC_E* code on failure; the message
 *    for the calling thread is available from ivc_last_error().
 *  - Functions WITHOUT the _dev suffix take HOST buffers (C-contiguous), stage them through
 *    per-device scratch memory owned by the library, and return when the result is back in
 *    the caller's host buffer (synchronous, like the NumPy reference).
 *  - Functions WITH the _dev suffix take DEVICE pointers (caller-owned, e.g. torch tensors)
 *    and a hipStream_t passed as void*; they only enqueue work (asynchronous).
 *  - Element-type codes (ivc_dtype) name the NumPy dtype the reference would see; the
 *    arithmetic follows NumPy's promotion rules for that dtype.
 */
#ifndef IVC_H
#define IVC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types (NumPy dtype of the array handed to the reference method) */
enum ivc_dtype {
  IVC_U8 = 1, IVC_I8 = 2, IVC_U16 = 3, IVC_I16 = 4, IVC_U32 = 5, IVC_I32 = 6,
  IVC_U64 = 7, IVC_I64 = 8, IVC_F32 = 9, IVC_F64 = 10
};

/* scipy.fft norm argument of DiscreteCosineTransform(norm=...) (ivclab/signal/dct.py:9-10) */
enum ivc_norm { IVC_NORM_BACKWARD = 0, IVC_NORM_ORTHO = 1, IVC_NORM_FORWARD = 2 };

/* motion-estimation SSD semantics */
enum ivc_me_mode {
  IVC_ME_NUMPY = 0,    /* NumPy semantics of the element type: modular integer sub/square,
                          pairwise float sums (ivclab/video/motion.py:46)                  */
  IVC_ME_EXACT_U8 = 1  /* u8 storage of integer-valued frames, SSD exact = the reference run
                          on frame.astype(float64) (what VideoCodec passes, videocodec.py:38) */
};

enum ivc_status {
  IVC_OK = 0, IVC_E_ARG = -1, IVC_E_DTYPE = -2, IVC_E_SHAPE = -3, IVC_E_DEVICE = -4,
  IVC_E_NOMEM = -5
};

/* ---------------------------------------------------------------- runtime ---------- */
const char* ivc_last_error(void);
int ivc_version(void);
/* 1: the exact-u8 +-16 motion search runs on the matrix cores (me_mfma16x2_kernel); it is the
   only +-16 exact-u8 search the library ships (kept for callers that probed it) */
int ivc_me_mfma_enabled(void);
/* Pipeline tuning overrides (process-wide, thread-safe; replace environment test hooks, so a
 * stray variable in the caller's environment never changes a call).  value 0 restores the
 * library's own choice.  Chunk counts force the number of pipelined chunks (any chunk size,
 * clamped to what the call allows); IVC_TUNE_S2I_NO_FALLBACK = 1 makes symbols -> image report
 * err[0] = -100 instead of running the general decoder when the fused parse rejects.      */
enum ivc_tuning_key {
  IVC_TUNE_ZR_CHUNKS = 0,        /* ZeroRunCoder.encode (ivc_zerorun_encode*)              */
  IVC_TUNE_SYM_CHUNKS = 1,       /* pixels -> symbols (ivc_intra_symbols*)                 */
  IVC_TUNE_S2I_CHUNKS = 2,       /* symbols -> image (ivc_symbols2image*)                  */
  IVC_TUNE_INTER_CHUNKS = 3,     /* fused inter encode (ivc_inter_encode*)                 */
  IVC_TUNE_S2I_NO_FALLBACK = 4,
  /* float64 motion search (ivc_motion_estimate* in IVC_ME_NUMPY mode on float64 frames):
     1 = without the float32 bound phase (every candidate in float64), 2 = the bound phase
     defers every round to the float64 search (exercises the deferral path); 0 = pruned */
  IVC_TUNE_F64_ME = 5,
  /* 1 = the per-block calls (one (8, 8) DCT, one (C, 8, 8) quantise / dequantise through the
     host-buffer entry points) launch a kernel each instead of using the resident tiny-call
     server; 0 = the server */
  IVC_TUNE_TINY_SERVER = 6,
  IVC_TUNE_COUNT = 7
};
int ivc_set_tuning(int key, int value);
/* the current override of `key` (0: none), or IVC_E_ARG for an unknown key */
int ivc_tuning(int key);
int ivc_device_count(void);
int ivc_set_device(int device);
/* 1 if the loaded code object matches the current device (gfx950), 0 otherwise */
int ivc_device_ok(void);
/* Host-buffer calls whose output is in page-locked memory (ivc_host_alloc) move their data in
 * chunks of chunk_bytes (the larger of input and output per chunk) that go
 * upload -> kernel -> download on 3 streams, overlapping one chunk's copies with another's;
 * 0 (the default: a half-duplex host link gains nothing from it) runs every call in one
 * piece.  Process-wide.                                                                   */
int ivc_set_host_pipeline(int64_t chunk_bytes);
/* the current chunk size of ivc_set_host_pipeline (0: off) */
int64_t ivc_host_pipeline(void);
/* release the library's cached scratch buffers on the current device, and the pinned host
 * blocks ivc_host_free has cached (process-wide)                                          */
int ivc_release_scratch(void);
/* Page-locked host memory for the host-buffer entry points' arrays: a transfer from or to a
 * block of ivc_host_alloc is one DMA (no staging copy); freed blocks are cached by size and
 * reused, up to 1 GiB (the oldest go first; env IVC_HOST_CACHE_MB overrides;
 * ivc_release_scratch drains it).  NULL when the runtime cannot pin more memory.          */
void* ivc_host_alloc(int64_t bytes);
int ivc_host_free(void* p);
/* Store pacing of the fused coefficient encoders (ivc_intra_encode*, ivc_inter_encode*):
 * persistent waves release their output stores on the chip-wide clock so that the stores
 * in flight sweep the output in address order.  The rate is the total HBM
 * rate (input + output GB/s) the sweep is timed for; it adapts per device from each launch's
 * count of late slots.  ivc_set_store_pace sets the starting rate (0 turns pacing off;
 * default: the IVC_PACE_GBPS environment variable, else the library's built-in rate);
 * ivc_store_pace returns the current device's rate, ivc_store_pace_late the late fraction
 * of the last measured launch (-1 if none).  Timing only: outputs are identical with and
 * without pacing.  No reference counterpart.                                             */
int ivc_set_store_pace(double total_gbps);
double ivc_store_pace(void);
double ivc_store_pace_late(void);
/* Measurement statistics of the current device's paced launches since the last reset
 * (encoder 0 = image source, 1 = inter residual, 2 = luma-only image), folding every completed launch first:
 * out[0] launches measured, [1] launches over the late threshold, [2] mean and [3] maximum
 * late fraction, [4] current rate (GB/s), [5] last late fraction, [6] mean achieved GB/s of
 * the measured launches (bytes / event time), [7] measurements still in flight, [8] launches
 * over the late threshold that still moved at least their schedule's rate, [9] the lowest
 * rate that fell off its schedule (0: none yet).  Writes min(n, 10) values and returns that
 * count (a negative status on a bad argument).                                             */
int ivc_store_pace_stats(int encoder, double* out, int n);
int ivc_store_pace_reset_stats(void);
/* Per-launch trace since the last reset: the most recent min(max_records, available, 256)
 * measured launches, oldest first, 7 doubles each: rate the launch ran at (GB/s), late-slot
 * fraction past each wave's start-up slots (its first min(64, slots / 8); what the rate adapts
 * on), achieved GB/s (bytes / event time), the kernel's first workgroup entry minus the
 * schedule origin (us), the earliest late slot past the start-up as a fraction of a wave's
 * slots (-1: none), the rate after folding it, the late fraction of the start-up slots.
 * Returns the number of records written.  (ivc_store_pace_stats' late fractions are those
 * past the start-up.)                                                                      */
int ivc_store_pace_trace(int encoder, double* out, int max_records);
/* Drop the current device's rates to the last rate that held its schedule and to at most
 * (1 - margin) x the lowest rate that fell off it: for callers about to enqueue many launches
 * without synchronisation (they all run at one rate).                                      */
int ivc_store_pace_settle(double margin);

/* ---------------------------------------------------------------- DCT -------------- */
/* 2-D DCT-II (inverse=0) / DCT-III (inverse=1) of nblk contiguous 8x8 blocks, applied along
 * the last axis then the second-to-last, exactly as scipy.fft.dct/idct (pocketfft) computes
 * it.  dst_dtype must be IVC_F32 or IVC_F64 (scipy: float32 stays float32, every integer
 * type and float64 compute in float64).
 * Replaces: DiscreteCosineTransform.transform          ivclab/signal/dct.py:12-28
 *           DiscreteCosineTransform.inverse_transform  ivclab/signal/dct.py:30-46        */
int ivc_dct8x8(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
               int inverse, int norm);
int ivc_dct8x8_dev(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
                   int inverse, int norm, void* stream);
/* The same transform of the blocks of Patcher.patch's view of a C-contiguous [H, W, C] image
 * (H, W multiples of 8), read in place: dst = [H/8, W/8, C, 8, 8], i.e.
 * transform(patch(img)) without gathering the strided view first.
 * Replaces: DiscreteCosineTransform.transform on Patcher.patch
 *           ivclab/signal/dct.py:12-28 + ivclab/utils/shape.py:45-54                      */
int ivc_dct8x8_image(const void* img, int src_dtype, int64_t H, int64_t W, int64_t C, void* dst,
                     int dst_dtype, int inverse, int norm);
int ivc_dct8x8_image_dev(const void* img, int src_dtype, int64_t H, int64_t W, int64_t C,
                         void* dst, int dst_dtype, int inverse, int norm, void* stream);

/* ---------------------------------------------------------------- quantization ----- */
/* src: nblk x C x 64 (C = 1 or 3; C = 1 broadcasts over the 3 table planes), table: the
 * 3 x 64 scaled quantization table as returned by get_quantization_table() (values exactly
 * representable in calc_dtype), calc_dtype: NumPy result type of src / table (IVC_F32 or
 * IVC_F64).  dst: nblk x 3 x 64 int32 = astype(int32)(round_half_even(src / table)).
 * Replaces: PatchQuant.quantize    ivclab/quantization/patchquant.py:44-60              */
int ivc_quantize(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                 int calc_dtype, int32_t* dst);
int ivc_quantize_dev(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                     int calc_dtype, int32_t* dst, void* stream);

/* dst = astype(int32)(src * table) computed in calc_dtype (truncation toward zero).
 * Replaces: PatchQuant.dequantize  ivclab/quantization/patchquant.py:62-78              */
int ivc_dequantize(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                   int calc_dtype, int32_t* dst);
int ivc_dequantize_dev(const void* src, int src_dtype, int64_t nblk, int C,
                       const double* table, int calc_dtype, int32_t* dst, void* stream);

/* ---------------------------------------------------------------- zig-zag ---------- */
/* nrow rows of 64 elements of elem_size bytes (1, 2, 4 or 8).  inverse=0: ZigZag.flatten
 * (dst[order[k]] = src[k]); inverse=1: ZigZag.unflatten (dst[k] = src[order[k]]).
 * src_row_stride (elements, >= 64) lets unflatten read rows wider than 64.
 * Replaces: ZigZag.flatten / unflatten  ivclab/utils/shape.py:21-36,
 *           zigzag_scan                 ivclab/signal/zigzag.py:3-26                    */
int ivc_zigzag(const void* src, int64_t nrow, int64_t src_row_stride, int elem_size,
               int inverse, void* dst);
int ivc_zigzag_dev(const void* src, int64_t nrow, int64_t src_row_stride, int elem_size,
                   int inverse, void* dst, void* stream);

/* ---------------------------------------------------------------- fused intra ------ */
/* patch -> DCT-II(ortho) -> quantize (-> zig-zag) over nframes images [H][W][C]
 * (H, W multiples of 8, C = 1 or 3).  out: [nframes][H/8][W/8][3][64] int32 (raster or
 * zig-zag order inside each 64).  Equals PatchQuant.quantize(DCT.transform(Patcher.patch(img)))
 * (+ ZigZag.flatten) bit for bit.  table/calc_dtype as ivc_quantize (calc = result type of
 * the DCT dtype and the table dtype).  hist (optional, may be NULL): int64[nbins] histogram
 * of the emitted coefficients, bin = value - hist_lo, values outside [hist_lo,
 * hist_lo+nbins) counted in the first/last bin; accumulated (not cleared) by the call.
 * Replaces the hot part of IntraCodec.image2symbols  ivclab/image/intracodec.py:66-75     */
int ivc_intra_encode(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W, int C,
                     const double* table, int calc_dtype, int zigzag, int32_t* out);
int ivc_intra_encode_dev(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                         int C, const double* table, int calc_dtype, int zigzag, int32_t* out,
                         int64_t* hist, int32_t hist_lo, int32_t nbins, void* stream);

/* The luma-table plane only of u8 grayscale frames [nframes][H][W]: out [nframes][H/8][W/8][64]
 * int32 = plane 0 of ivc_intra_encode_dev's output (C = 1, float64 arithmetic).  Not a
 * reference output (PatchQuant.quantize broadcasts C = 1 to the 3 table planes,
 * patchquant.py:59): a reported variant that moves 5 instead of 13 bytes per pixel.        */
int ivc_intra_encode_luma_dev(const uint8_t* img, int64_t nframes, int64_t H, int64_t W,
                              const double* table, int zigzag, int32_t* out, void* stream);

/* (un-zig-zag ->) dequantize -> DCT-III(ortho) of nblk blocks of 3 x 64 int32 symbols.
 * out: nblk x 3 x 8 x 8 float64 = DCT.inverse_transform(PatchQuant.dequantize(ZigZag.unflatten(q)))
 * Replaces the hot part of IntraCodec.symbols2image  ivclab/image/intracodec.py:115-121   */
int ivc_intra_decode(const int32_t* q, int64_t nblk, const double* table, int calc_dtype,
                     int unzigzag, double* out);
int ivc_intra_decode_dev(const int32_t* q, int64_t nblk, const double* table, int calc_dtype,
                         int unzigzag, double* out, void* stream);

/* The decode chain with the unpatch fused: q [nframes][H/8][W/8][C][64] int32 (C = 1 or 3;
 * zig-zag order when unzigzag) -> out [nframes][H][W][3] float64 =
 * rearrange(DCT.inverse_transform(PatchQuant.dequantize(ZigZag.unflatten(q))),
 *           'hp wp c h w -> (hp h) (wp w) c')
 * (C = 1 broadcasts over the 3 table planes, patchquant.py:77); to_rgb = 1 applies ycbcr2rgb
 * (color.py:40-63) to the result.
 * Replaces IntraCodec.symbols2image after the zero-run decode  intracodec.py:115-141       */
int ivc_intra_decode_image(const int32_t* q, int64_t nframes, int64_t H, int64_t W, int C,
                           const double* table, int unzigzag, int to_rgb, double* out);
int ivc_intra_decode_image_dev(const int32_t* q, int64_t nframes, int64_t H, int64_t W, int C,
                               const double* table, int unzigzag, int to_rgb, double* out,
                               void* stream);
/* IntraCodec.symbols2image (intracodec.py:84-146) for 8x8 blocks of 64 coefficients: the
 * zero-run decode of nsym symbols into nframes x H/8 x W/8 x C blocks (errors reported in
 * err[3] exactly as ivc_zerorun_decode; out is then undefined), then ivc_intra_decode_image
 * with unzigzag = 1, all on the device.  The caller crops and squeezes as the reference does. */
int ivc_symbols2image(const int32_t* sym, int64_t nsym, int64_t nframes, int64_t H, int64_t W,
                      int C, const double* table, int32_t eob, int to_rgb, double* out,
                      int64_t* err);
int ivc_symbols2image_dev(const int32_t* sym, int64_t nsym, int64_t nframes, int64_t H, int64_t W,
                          int C, const double* table, int32_t eob, int to_rgb, double* out,
                          int64_t* err, void* stream);

/* ---------------------------------------------------------------- motion ----------- */
/* Full-search block matching, 8x8 blocks, displacement +-sr, SSD, first strict minimum in
 * raster order of (dy, dx).  ref/cur: nframes x H x W (frame f of cur is matched against
 * frame f of ref; H, W multiples of 8).  mv: nframes x H/8 x W/8 int64 indices
 * (dy+sr)*(2sr+1)+(dx+sr).  mode: ivc_me_mode (IVC_ME_EXACT_U8 requires dtype IVC_U8).
 * Replaces: MotionCompensator.compute_motion_vector  ivclab/video/motion.py:8-58        */
int ivc_motion_estimate(const void* ref, const void* cur, int dtype, int64_t nframes,
                        int64_t H, int64_t W, int sr, int mode, int64_t* mv);
int ivc_motion_estimate_dev(const void* ref, const void* cur, int dtype, int64_t nframes,
                            int64_t H, int64_t W, int sr, int mode, int64_t* mv, void* stream);

/* Block-copy motion compensation: out[y:y+8, x:x+8, :] = ref[y+dy:.., x+dx:.., :] for each
 * block, zeros where the displaced block leaves the frame.  ref/out: nframes x H x W x C,
 * elem_size bytes per element; mv as produced above.
 * Replaces: MotionCompensator.reconstruct_with_motion_vector  ivclab/video/motion.py:60-97 */
int ivc_motion_compensate(const void* ref, int elem_size, int64_t nframes, int64_t H,
                          int64_t W, int64_t C, const int64_t* mv, int sr, void* out);
int ivc_motion_compensate_dev(const void* ref, int elem_size, int64_t nframes, int64_t H,
                              int64_t W, int64_t C, const int64_t* mv, int sr, void* out,
                              void* stream);

/* ---------------------------------------------------------------- fused inter ------ */
/* Open-loop P-frame residual coding of a u8 luma sequence: for every
 * frame f >= 1 of frames[nframes][H][W]: mv = ME(frames[f-1], frames[f]) (exact-u8 SSD),
 * prediction = MC(frames[f-1], mv), residual = float64(frames[f]) - prediction,
 * out = quantize(DCT(patch(residual))) as in ivc_intra_encode with C = 1.
 * mv: (nframes-1) x H/8 x W/8 int64, out: (nframes-1) x H/8 x W/8 x 3 x 64 int32.
 * Replaces VideoCodec.encode_decode's hot path  ivclab/video/videocodec.py:52-73         */
int ivc_inter_encode_dev(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W, int sr,
                         const double* table, int calc_dtype, int zigzag, int64_t* mv,
                         int32_t* out, void* stream);
/* ivc_inter_encode_dev that also accumulates the clamped histogram of the quantised output
 * (all 3 planes, as written) onto hist[clamp(v - hist_lo, 0, hist_n - 1)] (device int64) in
 * the encoder itself: the coefficient half of the global Huffman table's input
 * (ivclab/entropy/entropy.py:6-29 stats_marg over VideoCodec's residual symbols,
 * ivclab/video/videocodec.py:33,62) without a pass over the output.                   */
int ivc_inter_encode_hist_dev(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W,
                              int sr, const double* table, int calc_dtype, int zigzag,
                              int64_t* mv, int32_t* out, int64_t* hist, int32_t hist_lo,
                              int32_t hist_n, void* stream);

/* ---------------------------------------------------------------- histogram -------- */
/* hist[v - lo] += 1 for each symbol (values clamped into [lo, lo+nbins-1]); accumulates.
 * Feeds the global Huffman table (ivclab/entropy/entropy.py:6-29 stats_marg).            */
int ivc_histogram_i32(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins, int64_t* hist);
int ivc_histogram_i32_dev(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins,
                          int64_t* hist, void* stream);
/* The same over int64 symbols: the motion-vector indices of ivc_motion_estimate /
 * ivc_inter_encode_dev ((2 sr + 1)^2 bins for VideoCodec's motion Huffman table,
 * ivclab/video/videocodec.py:33,62).                                                       */
int ivc_histogram_i64(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins, int64_t* hist);
int ivc_histogram_i64_dev(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins,
                          int64_t* hist, void* stream);
/* stats_marg (ivclab/entropy/entropy.py:6-29) for any data and any bin edges:
 * np.histogram(x, bins=edges) counts of float64 values x (the caller casts, as the reference
 * does with image.astype(np.float64)) over nedges sorted float64 edges: x counts in bin i
 * when edges[i] <= x < edges[i+1], x == edges[nedges-1] in the last bin, values outside and
 * NaN dropped.  counts (nedges - 1 int64) are accumulated onto.  Edges that decrease are
 * refused with NumPy's message (host entry point; the _dev form expects sorted edges).     */
int ivc_histogram_f64_edges(const double* x, int64_t n, const double* edges, int32_t nedges,
                            int64_t* counts);
int ivc_histogram_f64_edges_dev(const double* x, int64_t n, const double* edges, int32_t nedges,
                                int64_t* counts, void* stream);
/* Workgroups per CU of the histogram launches (default 4, which fills the chip; 0 restores
 * the default).  A histogram on a side stream next to a VALU-bound kernel (the frame-sharded
 * bench step overlaps chunk k's histogram with chunk k+1's motion search) runs better with
 * 1-2, leaving LDS and wave slots to the other stream.  Timing only: counts are identical.
 * The setting is process-wide: it applies to every device, thread and histogram launch
 * (including intra_encode's fused histogram) until set again.  No reference counterpart.  */
int ivc_set_histogram_occupancy(int wg_per_cu);
int ivc_histogram_occupancy(void);

/* ---------------------------------------------------------------- colour ----------- */
/* rgb2ycbcr (ivclab/signal/color.py:15-38): npix pixels of 3 channels (any dtype) ->
 * float64 YCbCr, NumPy's `image @ M.T + offset` bit for bit (OpenBLAS dgemm k-order FMA).  */
int ivc_rgb2ycbcr(const void* src, int src_dtype, int64_t npix, double* dst);
int ivc_rgb2ycbcr_dev(const void* src, int src_dtype, int64_t npix, double* dst, void* stream);
/* ycbcr2rgb (color.py:40-63): channels 0..2 of npix pixels of `channels` (>= 3) values ->
 * clipped RGB, float32 for float32 input, float64 otherwise.                               */
int ivc_ycbcr2rgb(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst);
int ivc_ycbcr2rgb_dev(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst,
                      void* stream);
/* rgb2gray (color.py:3-13): mean over the `channels` (1..7) values of each pixel, float32
 * for float32 input, float64 otherwise.                                                    */
int ivc_rgb2gray(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst);
int ivc_rgb2gray_dev(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst,
                     void* stream);

/* ---------------------------------------------------------------- zero-run coding -- */
/* ZeroRunCoder.encode (ivclab/entropy/zerorun.py:10-43): src holds nblk rows of row_stride
 * int32 coefficients in (h w c) order; the first block_size (0..64, <= row_stride) of each
 * row are coded: nonzero values as themselves, each zero run before the row's last nonzero
 * as (0, run length), then eob.  The int32 stream goes to out (at most capacity symbols are
 * written); *nsym = its full length.  Returns IVC_E_SHAPE (with *nsym set) when the stream
 * is longer than capacity (bound: nblk * (block_size + (block_size + 1) / 2 + 1)).       */
int ivc_zerorun_encode(const int32_t* src, int64_t nblk, int32_t row_stride, int32_t block_size,
                       int32_t eob, int32_t* out, int64_t capacity, int64_t* nsym);
/* Device variant: offsets (device, nblk + 1 int64) receives each block's first symbol and
 * offsets[nblk] = the stream length; symbols past capacity are not written.  Asynchronous. */
int ivc_zerorun_encode_dev(const int32_t* src, int64_t nblk, int32_t row_stride,
                           int32_t block_size, int32_t eob, int64_t* offsets, int32_t* out,
                           int64_t capacity, void* stream);
/* ZeroRunCoder.decode (zerorun.py:46-88) of nsym (< 2^32) symbols into nblk blocks of
 * block_size int32 (out, zero-filled first).  The stream's own errors are results, not
 * failures: err[0] = 0 decoded; 1 "Block size exceeded: err[1]" (first in stream order);
 * 2 "Unexpected end of encoded symbols"; 3 the stream ends right after a zero symbol (the
 * reference's IndexError reading the run length at index err[1]); 4 "Expected err[1]
 * blocks, got err[2]".  Symbols after the nblk-th block are ignored, as in the reference. */
int ivc_zerorun_decode(const int32_t* sym, int64_t nsym, int64_t nblk, int32_t block_size,
                       int32_t eob, int32_t* out, int64_t* err);
/* IntraCodec.image2symbols' hot part fused (ivclab/image/intracodec.py:66-81 with
 * is_source_rgb=False): u8 frames [nframes][H][W][C] (C = 1 or 3, H and W multiples of 8)
 * -> patch -> DCT -> quantise -> zig-zag -> zero-run symbols, one int32 stream over
 * frames, then blocks in (h w c) order — the concatenation of ZeroRunCoder.encode of each
 * frame.  The coefficients never reach memory.  At most capacity symbols are written;
 * *nsym = the stream length (device int64 for _dev).  Host call: IVC_E_SHAPE with *nsym
 * set when capacity is too small.                                                        */
int ivc_intra_symbols(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W, int C,
                      const double* table, int32_t eob, int32_t* out, int64_t capacity,
                      int64_t* nsym);
int ivc_intra_symbols_dev(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                          int C, const double* table, int32_t eob, int32_t* out,
                          int64_t capacity, int64_t* nsym, void* stream);
/* ivc_intra_symbols_dev that also accumulates the clamped histogram of the whole stream (also
 * the symbols past capacity) onto hist[clamp(v - hist_lo, 0, hist_n - 1)] (device
 * int64[hist_n]; nothing is added when capacity = 0, which runs no emission pass): the counts IntraCodec.train_huffman_from_image's stats_marg takes
 * (intracodec.py:160-166, entropy.py:6-29) with no further pass over the stream.          */
int ivc_intra_symbols_hist_dev(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                               int C, const double* table, int32_t eob, int32_t* out,
                               int64_t capacity, int64_t* nsym, int64_t* hist, int32_t hist_lo,
                               int32_t hist_n, void* stream);
/* mm[0] = min, mm[1] = max of n int32 symbols (INT32_MAX, INT32_MIN when n = 0): the
 * Huffman alphabet bounds of IntraCodec.train_huffman_from_image (intracodec.py:161-163). */
int ivc_minmax_i32(const int32_t* sym, int64_t n, int32_t* mm);
int ivc_minmax_i32_dev(const int32_t* sym, int64_t n, int32_t* mm, void* stream);
/* Device variant: every pointer is device memory (err: 3 int64).  Asynchronous.           */
int ivc_zerorun_decode_dev(const int32_t* sym, int64_t nsym, int64_t nblk, int32_t block_size,
                           int32_t eob, int32_t* out, int64_t* err, void* stream);

/* ---------------------------------------------------------------- Huffman (host) --- */
/* HuffmanCoder (ivclab/entropy/huffman.py:5-61) on the host, where the north star keeps the
 * serial bit-packing.  lengths: Huffman code lengths of n weights (all > 0; ties merge in
 * index order).  Canonical codes; bits MSB-first in 32-bit words.  Tie-breaking differs
 * from the reference's `constriction` trees (absent here): bitstreams are not pinned.      */
int ivc_huffman_lengths(const double* probs, int32_t n, uint8_t* lengths);
/* symbols in [lower_bound, lower_bound + nalpha); IVC_E_ARG for a symbol outside, or
 * IVC_E_SHAPE (with *nbits set) when cap_words is too small.                              */
int ivc_huffman_encode(const int32_t* sym, int64_t n, int32_t lower_bound,
                       const uint8_t* lengths, int32_t nalpha, uint32_t* words,
                       int64_t cap_words, int64_t* nbits);
int ivc_huffman_decode(const uint32_t* words, int64_t nwords, int64_t count, int32_t lower_bound,
                       const uint8_t* lengths, int32_t nalpha, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* IVC_H */
