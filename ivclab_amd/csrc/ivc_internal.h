// ivc_internal.h — launchers shared between the kernels (ivc_kernels.hip, ivc_motion.hip)
// and the C-ABI layer (ivc_capi.hip).  Not part of the public interface (include/ivc.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ivc.h"

namespace ivc {

// quantisation table as kernel argument (by value: no per-call upload on the stream)
//   q[p*64 + i*8 + k]  : table value in the calc dtype (exactly representable)
struct QTab {
  double q[192];
};

// error raised by a launcher; turned into a status + message by the C-ABI layer
struct Error {
  int code;
  const char* msg;
};

int dtype_size(int dtype);
bool dtype_is_float(int dtype);

// all launchers enqueue on `s` and return hipSuccess / the launch error
hipError_t launch_dct8x8(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
                         int inverse, int norm, hipStream_t s);
hipError_t launch_quantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                           int calc_dtype, int32_t* dst, hipStream_t s);
hipError_t launch_dequantize(const void* src, int src_dtype, int64_t nblk, int C, const QTab& t,
                             int calc_dtype, int32_t* dst, hipStream_t s);
hipError_t launch_zigzag(const void* src, int64_t nrow, int64_t stride, int esize, int inverse,
                         void* dst, hipStream_t s);
// returns hipErrorInvalidValue for an unsupported dtype / C combination
hipError_t launch_intra_encode(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                               int C, const QTab& t, int calc_dtype, int zigzag, int32_t* out,
                               hipStream_t s);
hipError_t launch_intra_decode(const int32_t* q, int64_t nblk, const QTab& t, int unzigzag,
                               double* out, hipStream_t s);
unsigned resident_grid_ptr(const void* kernel, int64_t work_groups_needed);
hipError_t launch_histogram_i64(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins,
                                int64_t* hist, hipStream_t s);
hipError_t launch_histogram(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins,
                            int64_t* hist, hipStream_t s);

hipError_t launch_motion_estimate(const void* ref, const void* cur, int dtype, int64_t nframes,
                                  int64_t H, int64_t W, int sr, int mode, int64_t* mv,
                                  hipStream_t s);
hipError_t launch_motion_compensate(const void* ref, int esize, int64_t nframes, int64_t H,
                                    int64_t W, int64_t C, const int64_t* mv, int sr, void* out,
                                    hipStream_t s);
hipError_t launch_inter_residual(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W,
                                 int sr, const int64_t* mv, const QTab& t, int zigzag,
                                 int32_t* out, hipStream_t s);


}  // namespace ivc
