// Write-pattern microbenchmark, part 12: a prefetcher role.  One workgroup in R (the rest are
// "compute" workgroups: paced 6 KiB group stores + each group's 512 B tile read, as part 7)
// only reads input: when the clock enters epoch e (P slots of the paced schedule), the
// prefetchers read the input the compute waves will load in epoch e + 1 — 8 loads of 1 KiB in
// flight per wave, results discarded — so the compute waves' loads hit the Infinity Cache
// (part 10: cached input costs the write sweep nothing) and the HBM reads come in one burst
// per epoch.  The compute waves' own loads never wait behind prefetches (other waves).
//   hipcc --offload-arch=gfx950 -O3 -o ub/sp12 tools/ubench/store_pattern12.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__global__ void stamp(uint64_t* t) { *t = __builtin_amdgcn_s_memrealtime() + 300; }

__device__ __forceinline__ int64_t tile_off(int64_t G, int lane) {
  const int64_t f = G / (60 * 270), rem = G - f * 60 * 270;
  const int64_t bi = rem / 60, gc = rem - bi * 60;
  return (f * 2160 + 8 * bi + (lane >> 3)) * 3840 + gc * 64 + 8 * (lane & 7);
}

template <int R, int P>
__global__ __launch_bounds__(256) void roles(uint8_t* out, int64_t ngroups, const uint8_t* in,
                                             int64_t in_bytes, const uint64_t* t0p, uint32_t D,
                                             uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t base = *t0p << 8;
  const bool pref = R > 0 && (blockIdx.x % R) == R - 1;
  const int64_t ncomp_wg = R > 0 ? gridDim.x - gridDim.x / R : gridDim.x;
  const int64_t nw = ncomp_wg * 4;                          // compute waves
  if (pref) {
    // prefetcher p of NP: epoch e+1's groups [(e+1) P nw, (e+2) P nw), 2 groups (one 8-row x
    // 128 B tile, 16 B per lane) per load, tiles p, p + NP, ...
    const int64_t np = (int64_t)(gridDim.x / R) * 4;
    const int64_t p = (blockIdx.x / R) * 4 + wave;
    uint32_t acc = 0;
    const int64_t nepochs = (ngroups + P * nw - 1) / (P * nw);
    for (int64_t e = 0; e + 1 < nepochs; ++e) {
      const uint64_t start = base + (uint64_t)e * P * D;
      uint64_t now = __builtin_amdgcn_s_memrealtime() << 8;
      while (now < start) {
        __builtin_amdgcn_s_sleep(2);
        now = __builtin_amdgcn_s_memrealtime() << 8;
      }
      const int64_t g0 = (e + 1) * P * nw, g1 = g0 + P * nw < ngroups ? g0 + P * nw : ngroups;
      for (int64_t t = g0 / 2 + p; 2 * t < g1; t += 8 * np) {
        u32x4 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int64_t G = 2 * (t + k * np);
          const int64_t o = tile_off(G, lane & ~7) + 16 * (lane & 7);   // row lane/8, 128 B
          const bool ok = G < g1 && o + 16 <= in_bytes;
          __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<uint8_t*>(in) + (ok ? (o & ~(int64_t)0xffff) : 0), 0, ok ? 0x20000 : 0, 0x00020000);
          x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o & 0xffff), 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= x[k].x ^ x[k].w;
      }
    }
    if (acc == 0x12345678u) *sink = acc;
    return;
  }
  const int64_t cb = R > 0 ? blockIdx.x - blockIdx.x / R : blockIdx.x;   // compute WG index
  const int64_t w = cb * 4 + wave;
  uint64_t rel = base + (uint64_t)D * (uint64_t)w / (uint64_t)nw;
  auto load = [&](int64_t G) -> u32x2 {
    const int64_t o = tile_off(G, lane);
    const bool ok = G < ngroups && o + 8 <= in_bytes;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(in) + (ok ? (o & ~(int64_t)0xffff) : 0), 0, ok ? 0x20000 : 0, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(o & 0xffff), 0, 0);
  };
  u32x2 nx = load(w);
  for (int64_t G = w; G < ngroups; G += nw) {
    const u32x2 cur = nx;
    nx = load(G + nw);
    u32x4 v = {cur.x, cur.y, 3u, 4u};
    if (D) {
      uint64_t now = __builtin_amdgcn_s_memrealtime();
      while ((now << 8) < rel) {
        __builtin_amdgcn_s_sleep(1);
        now = __builtin_amdgcn_s_memrealtime();
      }
      rel += D;
    }
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + G * 6144, 0, 6144, 0x00020000);
#pragma unroll
    for (int j = 0; j < 6; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, 2);
  }
}

int main() {
  const int64_t ngroups = 256LL * 270 * 60;            // cfg3: 256 4K frames
  const int64_t out_bytes = ngroups * 6144, in_bytes = 256LL * 2160 * 3840;
  uint8_t *out, *in;
  uint64_t* t0;
  uint32_t* sink;
  if (hipMalloc(&out, out_bytes) != hipSuccess || hipMalloc(&in, in_bytes) != hipSuccess ||
      hipMalloc(&t0, 8) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess)
    return 1;
  (void)hipMemset(in, 1, in_bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int grid = 1792;   // 7 workgroups per CU, as the intra kernel
  auto run = [&](const char* name, auto K, int R, double gbps) {
    const double ncw = (R > 0 ? grid - grid / R : grid) * 4.0;
    const uint32_t D = (uint32_t)(ncw * 6656.0 / (gbps * 1e9) * 1e8 * 256);
    float tot = 0;
    for (int i = 0; i < 4; ++i) {
      (void)hipEventRecord(a);
      stamp<<<1, 1>>>(t0);
      K<<<grid, 256>>>(out, ngroups, in, in_bytes, t0, D, sink);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (i) tot += ms;
    }
    tot /= 3;
    const double tb = out_bytes + in_bytes;
    printf("%-12s pace %5.0f  %7.3f ms  %7.1f GB/s total (ideal %.3f ms)\n", name, gbps, tot,
           tb / tot / 1e6, tb / gbps / 1e6);
  };
  for (int rep = 0; rep < 2; ++rep)
    for (double g : {6400.0, 6800.0, 7200.0}) {
      run("no pf", roles<0, 8>, 0, g);
      run("R7 P4", roles<7, 4>, 7, g);
      run("R7 P8", roles<7, 8>, 7, g);
      run("R7 P16", roles<7, 16>, 7, g);
      run("R14 P8", roles<14, 8>, 14, g);
    }
  return 0;
}
