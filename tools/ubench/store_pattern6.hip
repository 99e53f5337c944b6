// Write-pattern microbenchmark, part 6: clock-paced persistent stores.  Wave w of W stores
// its step-k chunk (k * W + w, 6 KiB) no earlier than t0 + (k + w / W) * D on the chip-wide
// 100 MHz s_memrealtime clock, so the chunks being written at any instant sweep the buffer
// in address order (the pattern of a one-store-per-wave fill) instead of spreading over the
// W * 6 KiB window and the waves' drift.  D (10 ns ticks per step) is scanned.
//   hipcc --offload-arch=gfx950 -O3 -o ub/sp6 tools/ubench/store_pattern6.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void stamp(uint64_t* t) { *t = __builtin_amdgcn_s_memrealtime(); }

template <int WORK>
__global__ __launch_bounds__(256) void paced(uint8_t* out, int64_t nchunks, double* sink,
                                             const uint64_t* t0p, uint32_t D, uint32_t lead,
                                             uint32_t* late) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w = blockIdx.x * 4 + wave;
  const uint64_t t0 = *t0p + lead;
  // 32.32 fixed point: release(k) = t0 + k * D + w * D / W
  const uint64_t off = (uint64_t)D * (uint64_t)w / (uint64_t)nw;
  u32x4 v = {1u, 2u, 3u, 4u};
  double x = lane * 1e-3;
  uint32_t nlate = 0;
  int64_t k = 0;
  for (int64_t c = w; c < nchunks; c += nw, ++k) {
#pragma unroll
    for (int i = 0; i < WORK; ++i) x = __builtin_fma(x, 1.0000001, 1e-9);
    v.x = (unsigned)x;
    if (D) {
      const uint64_t rel = t0 + (uint64_t)k * D + off;
      uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now > rel + D) ++nlate;
      while (now < rel) {
        __builtin_amdgcn_s_sleep(1);
        now = __builtin_amdgcn_s_memrealtime();
      }
    }
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + c * 6144, 0, 6144, 0x00020000);
#pragma unroll
    for (int j = 0; j < 6; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, 2);
  }
  if (x == 12345.0) *sink = x;
  if (lane == 0 && nlate) atomicAdd(late, nlate);
}

int main() {
  const int64_t bytes = 25480396800LL;
  uint8_t* out;
  double* sink;
  uint64_t* t0;
  uint32_t* late;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess ||
      hipMalloc(&t0, 8) != hipSuccess || hipMalloc(&late, 4) != hipSuccess)
    return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int64_t n6 = bytes / 6144;
  auto run = [&](const char* name, auto K, int grid, uint32_t D, uint32_t lead) {
    float tot = 0;
    uint32_t nl = 0;
    for (int i = 0; i < 4; ++i) {
      (void)hipMemset(late, 0, 4);
      (void)hipEventRecord(a);
      stamp<<<1, 1>>>(t0);
      K<<<grid, 256>>>(out, n6, sink, t0, D, lead, late);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (i) tot += ms;
      (void)hipMemcpy(&nl, late, 4, hipMemcpyDeviceToHost);
    }
    tot /= 3;
    const int64_t steps = (n6 + grid * 4 - 1) / (grid * 4);
    printf("%-12s grid %5d D %5u lead %4u  %7.3f ms  %7.1f GB/s  (%lld steps, ideal %.3f ms, late %u)\n",
           name, grid, D, lead, tot, bytes / tot / 1e6, (long long)steps, steps * D * 1e-5, nl);
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (int grid : {1024, 1536}) {
      run("unpaced w60", paced<60>, grid, 0, 0);
      for (uint32_t D : {400u, 450u, 500u, 550u, 600u})
        run("paced w60", paced<60>, grid, D * grid / 1536, 300);
      run("unpaced w180", paced<180>, grid, 0, 0);
      for (uint32_t D : {450u, 500u, 550u, 600u})
        run("paced w180", paced<180>, grid, D * grid / 1536, 300);
    }
  }
  return 0;
}
