// Write-pattern microbenchmark, part 2: contiguous-per-wave vs interleaved-across-the-
// workgroup store orders, persistent and not.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define STORE(rs, off) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0)

// WG region of 4*CH KiB: contiguous per wave (wave w: pieces [w*CH, (w+1)*CH))
template <int CH, bool PERSIST>
__global__ __launch_bounds__(256) void wave_contig(uint8_t* out, int64_t nregions) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32x4 v = {1u, 2u, 3u, 4u};
  for (int64_t r = blockIdx.x; r < nregions; r += PERSIST ? gridDim.x : nregions) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + r * 4 * CH * 1024, 0, 4 * CH * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < CH; ++j) STORE(rs, (wave * CH + j) * 1024 + lane * 16);
  }
}

// WG region of 4*CH KiB: interleaved (step j: wave w writes piece 4j + w)
template <int CH, bool PERSIST>
__global__ __launch_bounds__(256) void wg_inter(uint8_t* out, int64_t nregions) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32x4 v = {1u, 2u, 3u, 4u};
  for (int64_t r = blockIdx.x; r < nregions; r += PERSIST ? gridDim.x : nregions) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + r * 4 * CH * 1024, 0, 4 * CH * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < CH; ++j) STORE(rs, (4 * j + wave) * 1024 + lane * 16);
  }
}

// persistent, wave-contiguous, but the region index comes from an atomic ticket per WG step
template <int CH>
__global__ __launch_bounds__(256) void ticket(uint8_t* out, int64_t nregions, unsigned long long* ctr) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32x4 v = {1u, 2u, 3u, 4u};
  __shared__ int64_t slot;
  for (;;) {
    if (threadIdx.x == 0) slot = (int64_t)atomicAdd(ctr, 1ull);
    __syncthreads();
    const int64_t r = slot;
    __syncthreads();
    if (r >= nregions) break;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + r * 4 * CH * 1024, 0, 4 * CH * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < CH; ++j) STORE(rs, (4 * j + wave) * 1024 + lane * 16);
  }
}

int main() {
  const int64_t bytes = 25480396800LL;
  uint8_t* out;
  unsigned long long* ctr;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&ctr, 8) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  auto report = [&](const char* name, int grid, float ms) {
    printf("%-40s grid %8d  %7.3f ms  %7.1f GB/s\n", name, grid, ms, bytes / ms / 1e6);
  };
#define RUN(name, K, CH, grid)                                                   \
  {                                                                              \
    const int64_t nr = bytes / (4 * CH * 1024);                                  \
    K<<<grid, 256>>>(out, nr);                                                   \
    (void)hipEventRecord(a);                                                     \
    for (int i = 0; i < 3; ++i) K<<<grid, 256>>>(out, nr);                      \
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);                       \
    float ms; (void)hipEventElapsedTime(&ms, a, b); report(name, grid, ms / 3);   \
  }
#define RUNT(name, CH, grid)                                                     \
  {                                                                              \
    const int64_t nr = bytes / (4 * CH * 1024);                                  \
    float tot = 0;                                                               \
    for (int i = 0; i < 4; ++i) {                                                \
      (void)hipMemset(ctr, 0, 8);                                                \
      (void)hipEventRecord(a);                                                   \
      ticket<CH><<<grid, 256>>>(out, nr, ctr);                                   \
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);                     \
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (i) tot += ms;          \
    }                                                                            \
    report(name, grid, tot / 3);                                                 \
  }
  const int64_t r1 = bytes / 4096, r6 = bytes / (4 * 6 * 1024), r12 = bytes / (4 * 12 * 1024);
  RUN("np wave-contig 1K", (wave_contig<1, false>), 1, (int)r1);
  RUN("np wave-contig 6K", (wave_contig<6, false>), 6, (int)r6);
  RUN("np wg-interleave 6K", (wg_inter<6, false>), 6, (int)r6);
  RUN("np wave-contig 12K", (wave_contig<12, false>), 12, (int)r12);
  RUN("np wg-interleave 12K", (wg_inter<12, false>), 12, (int)r12);
  for (int occ : {4, 6, 8}) {
    const int g = 256 * occ;
    printf("-- persistent, %d WG per CU\n", occ);
    RUN("p wave-contig 6K", (wave_contig<6, true>), 6, g);
    RUN("p wg-interleave 6K", (wg_inter<6, true>), 6, g);
    RUN("p wave-contig 12K", (wave_contig<12, true>), 12, g);
    RUN("p wg-interleave 12K", (wg_inter<12, true>), 12, g);
    RUNT("p ticket wg-interleave 6K", 6, g);
    RUNT("p ticket wg-interleave 12K", 12, g);
  }
  return 0;
}
