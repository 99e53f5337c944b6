// Write-pattern microbenchmark, part 4: one 1 KiB store per wave (the fast pattern) with the
// workgroup -> address map scrambled inside windows of 2^LOGW workgroups (4 KiB each):
// is the write rate a matter of address order in time?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int LOGW>
__global__ __launch_bounds__(256) void scrambled(uint8_t* out, int64_t nwg) {
  const int lane = threadIdx.x & 63;
  const int64_t wg = blockIdx.x;
  int64_t m = wg;
  if (LOGW > 0) {
    const int64_t win = wg >> LOGW, lo = wg & ((1LL << LOGW) - 1);
    m = (win << LOGW) | ((lo * 0x9E3779B1LL) & ((1LL << LOGW) - 1));   // odd multiplier: bijection
  }
  const int64_t c = m * 4 + (threadIdx.x >> 6);
  const u32x4 v = {1u, 2u, 3u, 4u};
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + c * 1024, 0, m < nwg ? 1024 : 0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, lane * 16, 0, 0);
}

int main() {
  const int64_t bytes = 25769803776LL;   // 24 GiB: a whole number of every window
  uint8_t* out;
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int64_t nwg = bytes / 4096;
#define RUN(name, K)                                                             \
  {                                                                              \
    K<<<nwg, 256>>>(out, nwg);                                                   \
    (void)hipEventRecord(a);                                                     \
    for (int i = 0; i < 3; ++i) K<<<nwg, 256>>>(out, nwg);                      \
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);                       \
    float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 3;                     \
    printf("%-34s %7.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);          \
  }
  for (int rep = 0; rep < 2; ++rep) {
    RUN("in order", scrambled<0>);
    RUN("scrambled in 64 KiB", scrambled<4>);
    RUN("scrambled in 1 MiB", scrambled<8>);
    RUN("scrambled in 16 MiB", scrambled<12>);
    RUN("scrambled in 64 MiB", scrambled<14>);
    RUN("scrambled in 256 MiB", scrambled<16>);
    RUN("scrambled in 1 GiB", scrambled<18>);
  }
  return 0;
}
