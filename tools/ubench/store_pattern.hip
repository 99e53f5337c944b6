// Write-pattern microbenchmark: how the HBM write rate depends on the contiguous chunk each
// wave writes per step and on grid shape (persistent strided vs one chunk per wave).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/store_pattern tools/ubench/store_pattern.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// persistent: wave w writes chunks w, w + nwaves, ... of CH KiB (CH stores of 1 KiB each)
template <int CH, int AUX>
__global__ __launch_bounds__(256) void persist(uint8_t* out, int64_t nchunks) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const u32x4 v = {1u, 2u, 3u, 4u};
  for (int64_t c = blockIdx.x * 4 + wave; c < nchunks; c += nw) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + c * CH * 1024, 0, CH * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < CH; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, AUX);
  }
}

// wave-interleaved: step k, wave w writes 1 KiB piece (k * nwaves + w) ... but CH pieces per
// step, each nwaves KiB apart (so the grid sweeps memory compactly)
template <int CH, int AUX>
__global__ __launch_bounds__(256) void sweep(uint8_t* out, int64_t npieces) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const u32x4 v = {1u, 2u, 3u, 4u};
  for (int64_t p = blockIdx.x * 4 + wave; p < npieces; p += nw * CH) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int64_t q = p + j * nw;
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + q * 1024, 0, q < npieces ? 1024 : 0, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, lane * 16, 0, AUX);
    }
  }
}

int main() {
  const int64_t bytes = 25480396800LL;  // the cfg3 output
  uint8_t* out;
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  int cus = 256;
  auto run = [&](const char* name, auto kern, int64_t n, int grid) {
    kern<<<grid, 256>>>(out, n);
    hipEventRecord(a);
    for (int i = 0; i < 3; ++i) kern<<<grid, 256>>>(out, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ms /= 3;
    printf("%-34s grid %7d  %7.3f ms  %7.1f GB/s\n", name, grid, ms, bytes / ms / 1e6);
  };
  for (int occ : {4, 6, 8}) {
    printf("-- %d workgroups per CU\n", occ);
    const int g = cus * occ;
    run("persist 1K", persist<1, 0>, bytes / 1024, g);
    run("persist 6K", persist<6, 0>, bytes / 6144, g);
    run("persist 12K", persist<12, 0>, bytes / 12288, g);
    run("persist 12K nt", persist<12, 2>, bytes / 12288, g);
    run("persist 48K", persist<48, 0>, bytes / 49152, g);
    run("sweep 6 pieces", sweep<6, 0>, bytes / 1024, g);
    run("sweep 12 pieces", sweep<12, 0>, bytes / 1024, g);
    run("sweep 12 pieces nt", sweep<12, 2>, bytes / 1024, g);
  }
  printf("-- one chunk per wave (non-persistent)\n");
  run("1 chunk of 1K per wave", persist<1, 0>, bytes / 1024, (int)(bytes / 1024 / 4));
  run("1 chunk of 12K per wave", persist<12, 0>, bytes / 12288, (int)(bytes / 12288 / 4));
  hipFree(out);
  return 0;
}
