// Write-pattern microbenchmark, part 12: the symbols -> image decode's HBM pattern without its
// arithmetic.  Each 8-block group (512 px of 3 planes) writes the RGB float64 image it decodes
// as 8 row segments of 1536 B (rows W * 24 B apart, two 16-byte stores per lane per row, as
// sym_image_kernel / intra_decode_kernel do) and reads R bytes of input per group (the decode
// reads the zero-run stream twice, ~13.4 B/px: ~6.9 KB per group; 0 = writes only).  Modes:
//   image  : the decode's layout (row segments), persistent waves, group g = k * W + w
//   blocks : the same bytes as one contiguous 12 KiB run per group (the blocks layout)
//   fresh  : image layout, one group per wave, no persistence (grid = groups / 4 workgroups)
//   paced  : image layout, persistent, stores released on a clock schedule (target rates swept)
// It measures the rate the decode's store/read mix reaches on this part when nothing else
// limits it: the floor DESIGN.md 5e compares the decode against.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/store_pattern12 tools/ubench/store_pattern12.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int H = 2160, W = 3840, GW = W / 64, GH = H / 8;   // groups per row / per column
constexpr int64_t ROWB = (int64_t)W * 24;                     // bytes per RGB float64 image row

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)n, 0x00020000);
}

template <int MODE>   // 0 image, 1 blocks
__device__ __forceinline__ void group(char* out, const char* in, int64_t g, int rd, int lane) {
  u32x4 acc = {(uint32_t)g, (uint32_t)lane, 1u, 2u};
  if (rd > 0) {
    const __amdgpu_buffer_rsrc_t ri = rsrc(in + g * rd, (uint32_t)rd);
    for (int c = lane; 16 * c < rd; c += 64) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ri, 16 * c, 0, 0);
      acc += v;
    }
  }
  if (MODE == 0) {
    const int64_t f = g / (GW * GH), rem = g % (GW * GH), gy = rem / GW, gx = rem % GW;
    char* base = out + f * (int64_t)H * ROWB + gy * 8 * ROWB + gx * 1536;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const __amdgpu_buffer_rsrc_t ro = rsrc(base + i * ROWB, 1536u);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = j * 64 + lane;
        __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)i, ro, c < 96 ? c * 16 : 0x40000000, 0, 2);
      }
    }
  } else {
    const __amdgpu_buffer_rsrc_t ro = rsrc(out + g * 12288, 12288u);
#pragma unroll
    for (int j = 0; j < 12; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(acc + (uint32_t)j, ro, (j * 64 + lane) * 16, 0, 2);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void persistent_k(char* out, const char* in, int64_t groups, int rd) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < groups; g += nw)
    group<MODE>(out, in, g, rd, lane);
}

__global__ void stamp_k(uint64_t* t) { *t = __builtin_amdgcn_s_memrealtime(); }

// paced: wave w of W stores its step-k group (k W + w) no earlier than t0 + k D + w D / W on the
// 100 MHz clock (D in 1/256 ticks), so the groups being written sweep the image in order
// (the headline encoder's store schedule); late groups are counted
__global__ __launch_bounds__(256) void paced_k(char* out, const char* in, int64_t groups, int rd,
                                               const uint64_t* t0p, uint32_t D, uint32_t* late) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint64_t rel = (*t0p + 3000) * 256 + (uint64_t)D * (uint64_t)w / (uint64_t)nw;
  uint32_t nlate = 0;
  for (int64_t g = w; g < groups; g += nw, rel += D) {
    uint64_t now = __builtin_amdgcn_s_memrealtime() * 256;
    if (now > rel + D) ++nlate;
    while (now < rel) {
      __builtin_amdgcn_s_sleep(1);
      now = __builtin_amdgcn_s_memrealtime() * 256;
    }
    group<0>(out, in, g, rd, lane);
  }
  if (lane == 0 && nlate) atomicAdd(late, nlate);
}

__global__ __launch_bounds__(256) void fresh_k(char* out, const char* in, int64_t groups, int rd) {
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g < groups) group<0>(out, in, g, rd, threadIdx.x & 63);
}

int main() {
  const int F = 48;
  const int64_t groups = (int64_t)F * GW * GH;
  const int64_t outB = (int64_t)F * H * ROWB;
  const int rdmax = 7168;
  char *out = nullptr, *in = nullptr;
  if (hipMalloc(&out, outB) != hipSuccess || hipMalloc(&in, groups * rdmax) != hipSuccess) {
    printf("hipMalloc failed\n");
    return 1;
  }
  (void)hipMemset(in, 1, groups * rdmax);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("%d frames of 4K RGB float64 (%.2f GB out), %lld groups, %d CUs\n", F, outB / 1e9,
         (long long)groups, cus);
  struct Cfg { const char* name; int mode; int rd; int wgs_per_cu; };
  const Cfg cfgs[] = {{"image  ", 0, 0, 4}, {"image  ", 0, 6912, 4}, {"image  ", 0, 6912, 8},
                      {"image  ", 0, 3072, 4}, {"blocks ", 1, 0, 4}, {"blocks ", 1, 6912, 4},
                      {"fresh  ", 2, 0, 0}, {"fresh  ", 2, 6912, 0}};
  for (const Cfg& c : cfgs) {
    std::vector<float> t;
    for (int rep = 0; rep < 7; ++rep) {
      (void)hipEventRecord(e0, 0);
      if (c.mode == 2) {
        fresh_k<<<(unsigned)((groups + 3) / 4), 256>>>(out, in, groups, c.rd);
      } else if (c.mode == 0) {
        persistent_k<0><<<cus * c.wgs_per_cu, 256>>>(out, in, groups, c.rd);
      } else {
        persistent_k<1><<<cus * c.wgs_per_cu, 256>>>(out, in, groups, c.rd);
      }
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double ms = t[t.size() / 2];
    const double wb = (double)groups * 12288, rb = (double)groups * c.rd;
    printf("%s reads %4d B/group  wg/CU %d: %.3f ms  writes %.0f GB/s  total %.0f GB/s\n", c.name, c.rd,
           c.wgs_per_cu, ms, wb / (ms * 1e-3) / 1e9, (wb + rb) / (ms * 1e-3) / 1e9);
  }
  // paced sweeps at target total rates (reads + writes), 4 workgroups per CU
  uint64_t* t0 = nullptr;
  uint32_t* late = nullptr;
  (void)hipMalloc(&t0, 8);
  (void)hipMalloc(&late, 4);
  const int rds[] = {0, 6912};
  for (int rd : rds) {
    const double per_group = 12288.0 + rd;
    const unsigned grid = cus * 4;
    const double W = grid * 4.0;
    for (double tbs = 4.8; tbs < 6.65; tbs += 0.3) {
      // D: 1/256 ticks (10 ns) per step of W groups at tbs TB/s
      const double step_s = W * per_group / (tbs * 1e12);
      const uint32_t D = (uint32_t)(step_s / 10e-9 * 256.0);
      std::vector<float> t;
      uint32_t lt = 0;
      for (int rep = 0; rep < 6; ++rep) {
        (void)hipMemset(late, 0, 4);
        stamp_k<<<1, 1>>>(t0);
        (void)hipEventRecord(e0, 0);
        paced_k<<<grid, 256>>>(out, in, groups, rd, t0, D, late);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0) t.push_back(ms);
        (void)hipMemcpy(&lt, late, 4, hipMemcpyDeviceToHost);
      }
      std::sort(t.begin(), t.end());
      const double ms = t[t.size() / 2];
      printf("paced   reads %4d B/group  target %.2f TB/s: %.3f ms  total %.0f GB/s  late %u of %lld\n", rd,
             tbs, ms, (double)groups * per_group / (ms * 1e-3) / 1e9, lt, (long long)groups);
    }
  }
  (void)hipFree(t0);
  (void)hipFree(late);
  (void)hipFree(out);
  (void)hipFree(in);
  return 0;
}
