// Write-pattern microbenchmark, part 5: persistent waves (6 KiB of stores + ALU work per
// step, tile = k * nwaves + w) with a start-up stagger proportional to the wave index, so
// that waves storing at the same time own adjacent tiles.  Optional periodic re-sync
// against a global progress counter.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void sleep_cycles(uint32_t c) {
  // s_sleep N waits ~64*N cycles
  while (c >= 64 * 64) { __builtin_amdgcn_s_sleep(64); c -= 64 * 64; }
  while (c >= 64) { __builtin_amdgcn_s_sleep(1); c -= 64; }
}

template <int WORK>
__global__ __launch_bounds__(256) void staggered(uint8_t* out, int64_t nchunks, double* sink,
                                                 uint32_t stagger_cycles, int resync,
                                                 unsigned* progress) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w = blockIdx.x * 4 + wave;
  u32x4 v = {1u, 2u, 3u, 4u};
  double x = lane * 1e-3;
  if (stagger_cycles) sleep_cycles((uint32_t)((uint64_t)stagger_cycles * w / nw));
  int64_t k = 0;
  for (int64_t c = w; c < nchunks; c += nw, ++k) {
#pragma unroll
    for (int i = 0; i < WORK; ++i) x = __builtin_fma(x, 1.0000001, 1e-9);
    if (resync && (k & 15) == 15) {
      // wait until at least (c - nw/2) stores of the sweep are done: bounded spin
      for (int spin = 0; spin < 200; ++spin) {
        const unsigned p = __hip_atomic_load(progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int64_t)p * 64 + nw / 2 >= c) break;
        __builtin_amdgcn_s_sleep(8);
      }
    }
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + c * 6144, 0, 6144, 0x00020000);
#pragma unroll
    for (int j = 0; j < 6; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, 2);
    if (resync && lane == 0 && (c & 63) == 0) __hip_atomic_fetch_add(progress, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v.x = (unsigned)x;
  }
  if (x == 12345.0) *sink = x;
}

int main() {
  const int64_t bytes = 25480396800LL;
  uint8_t* out;
  double* sink;
  unsigned* prog;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess || hipMalloc(&prog, 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int64_t n6 = bytes / 6144;
  const int grid = 1536;
  auto run = [&](const char* name, auto K, uint32_t st, int rs) {
    float tot = 0;
    for (int i = 0; i < 4; ++i) {
      (void)hipMemset(prog, 0, 4);
      (void)hipEventRecord(a);
      K<<<grid, 256>>>(out, n6, sink, st, rs, prog);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (i) tot += ms;
    }
    tot /= 3;
    printf("%-28s stagger %7u resync %d  %7.3f ms  %7.1f GB/s\n", name, st, rs, tot, bytes / tot / 1e6);
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (uint32_t st : {0u, 4000u, 16000u, 32000u, 64000u}) {
      run("work 60", staggered<60>, st, 0);
      run("work 180", staggered<180>, st, 0);
    }
    run("work 60", staggered<60>, 16000u, 1);
    run("work 180", staggered<180>, 32000u, 1);
  }
  return 0;
}
