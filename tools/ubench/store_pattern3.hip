// Write-pattern microbenchmark, part 3: does spreading a wave's stores over time (other
// work between them) change the HBM write rate?  Persistent waves, 6 KiB per wave-step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// SPREAD: ALU work (dependent v_fma_f64 chain of WORK ops) between consecutive stores;
// WORK ops are split evenly between the 6 stores when SPREAD, else done after all six
template <int WORK, bool SPREAD>
__global__ __launch_bounds__(256) void mixed(uint8_t* out, int64_t nchunks, double* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  u32x4 v = {1u, 2u, 3u, 4u};
  double x = lane * 1e-3;
  for (int64_t c = blockIdx.x * 4 + wave; c < nchunks; c += nw) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + c * 6144, 0, 6144, 0x00020000);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, 2);
      if (SPREAD) {
#pragma unroll
        for (int k = 0; k < WORK / 6; ++k) x = __builtin_fma(x, 1.0000001, 1e-9);
      }
    }
    if (!SPREAD) {
#pragma unroll
      for (int k = 0; k < WORK; ++k) x = __builtin_fma(x, 1.0000001, 1e-9);
    }
    v.x = (unsigned)x;
  }
  if (x == 12345.0) *sink = x;
}

__global__ __launch_bounds__(256) void one_per_wave(uint8_t* out, int64_t n, double*) {
  const int lane = threadIdx.x & 63;
  const int64_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const u32x4 v = {1u, 2u, 3u, 4u};
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + c * 1024, 0, c < n ? 1024 : 0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, lane * 16, 0, 0);
}

int main() {
  const int64_t bytes = 25480396800LL;
  uint8_t* out;
  double* sink;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
#define RUN(name, K, n, grid)                                                    \
  {                                                                              \
    K<<<grid, 256>>>(out, n, sink);                                              \
    (void)hipEventRecord(a);                                                     \
    for (int i = 0; i < 3; ++i) K<<<grid, 256>>>(out, n, sink);                 \
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);                       \
    float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 3;                     \
    printf("%-36s grid %8d  %7.3f ms  %7.1f GB/s\n", name, (int)(grid), ms, bytes / ms / 1e6); \
  }
  const int64_t n6 = bytes / 6144;
  for (int rep = 0; rep < 2; ++rep) {
    RUN("one 1K store per wave", one_per_wave, bytes / 1024, bytes / 4096);
    RUN("6 stores, no work", (mixed<0, false>), n6, 1536);
    RUN("6 stores, 60 fma after", (mixed<60, false>), n6, 1536);
    RUN("6 stores, 60 fma spread", (mixed<60, true>), n6, 1536);
    RUN("6 stores, 180 fma after", (mixed<180, false>), n6, 1536);
    RUN("6 stores, 180 fma spread", (mixed<180, true>), n6, 1536);
    RUN("6 stores, 360 fma after", (mixed<360, false>), n6, 1536);
    RUN("6 stores, 360 fma spread", (mixed<360, true>), n6, 1536);
  }
  return 0;
}
