// Write-pattern microbenchmark, part 9: as part 8 (paced 6 KiB group stores, the intra
// kernel's 512 B-per-group tile reads issued K groups at a time), but the read bursts can be
// aligned on the chip-wide clock: every wave issues the loads of its next K groups as soon as
// the clock passes the epoch boundary t0 + e*K*D (checked while it waits for its store
// slots), so that all reads of an epoch reach HBM within a short window instead of being
// spread over a whole slot.
//   hipcc --offload-arch=gfx950 -O3 -o ub/sp9 tools/ubench/store_pattern9.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__global__ void stamp(uint64_t* t) { *t = __builtin_amdgcn_s_memrealtime() + 300; }

__device__ __forceinline__ uint64_t clk256() { return __builtin_amdgcn_s_memrealtime() << 8; }

// ALIGN: 0 = burst at the wave's own first slot of the epoch (part 8), 1 = burst when the
// clock passes the epoch boundary
template <int K, int ALIGN>
__global__ __launch_bounds__(256) void paced_rw(uint8_t* out, int64_t ngroups, const uint8_t* in,
                                                int64_t in_bytes, const uint64_t* t0p,
                                                uint32_t D) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w = blockIdx.x * 4 + wave;
  const uint64_t base = *t0p << 8;
  uint64_t rel = base + (uint64_t)D * (uint64_t)w / (uint64_t)nw;
  auto load = [&](int64_t G) -> u32x2 {
    const int64_t f = G / (60 * 270), rem = G - f * 60 * 270;
    const int64_t bi = rem / 60, gc = rem - bi * 60;
    const int64_t o = (f * 2160 + 8 * bi + (lane >> 3)) * 3840 + gc * 64 + 8 * (lane & 7);
    const bool ok = G < ngroups && o + 8 <= in_bytes;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(in) + (ok ? (o & ~(int64_t)0xffff) : 0), 0, ok ? 0x20000 : 0, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(o & 0xffff), 0, 0);
  };
  u32x2 cur[K], nxt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) cur[k] = load(w + k * nw);
  int64_t e = 0;
  for (int64_t G0 = w; G0 < ngroups; G0 += K * nw, ++e) {
    const uint64_t tb = base + (uint64_t)e * K * D;
    bool issued = false;
    auto burst = [&]() {
#pragma unroll
      for (int k = 0; k < K; ++k) nxt[k] = load(G0 + (K + k) * nw);
      issued = true;
    };
    if (!ALIGN) burst();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t G = G0 + k * nw;
      u32x4 v = {cur[k].x, cur[k].y, 3u, 4u};
      uint64_t now = clk256();
      while (now < rel) {
        if (ALIGN && !issued && now >= tb) burst();
        __builtin_amdgcn_s_sleep(1);
        now = clk256();
      }
      rel += D;
      if (ALIGN && !issued && now >= tb) burst();
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + G * 6144, 0, G < ngroups ? 6144 : 0, 0x00020000);
#pragma unroll
      for (int j = 0; j < 6; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, 2);
    }
    if (ALIGN && !issued) burst();
#pragma unroll
    for (int k = 0; k < K; ++k) cur[k] = nxt[k];
  }
}

int main() {
  const int64_t ngroups = 256LL * 270 * 60;            // cfg3: 256 4K frames
  const int64_t out_bytes = ngroups * 6144, in_bytes = 256LL * 2160 * 3840;
  uint8_t *out, *in;
  uint64_t* t0;
  if (hipMalloc(&out, out_bytes) != hipSuccess || hipMalloc(&in, in_bytes) != hipSuccess ||
      hipMalloc(&t0, 8) != hipSuccess)
    return 1;
  (void)hipMemset(in, 1, in_bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int grid = 1792;   // 7 workgroups per CU, as the intra kernel
  auto run = [&](const char* name, auto Kf, double gbps) {
    const double bytes_per_group = 6144.0 + 512.0;
    const uint32_t D = (uint32_t)(grid * 4.0 * bytes_per_group / (gbps * 1e9) * 1e8 * 256);
    float tot = 0;
    for (int i = 0; i < 4; ++i) {
      (void)hipEventRecord(a);
      stamp<<<1, 1>>>(t0);
      Kf<<<grid, 256>>>(out, ngroups, in, in_bytes, t0, D);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (i) tot += ms;
    }
    tot /= 3;
    const double tb = out_bytes + in_bytes;
    printf("%-12s pace %5.0f  %7.3f ms  %7.1f GB/s total (ideal %.3f ms)\n", name, gbps, tot,
           tb / tot / 1e6, tb / gbps / 1e6);
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (double g : {6000.0, 6200.0, 6400.0, 6600.0, 7000.0}) {
      run("K4 own", paced_rw<4, 0>, g);
      run("K4 aligned", paced_rw<4, 1>, g);
      run("K8 own", paced_rw<8, 0>, g);
      run("K8 aligned", paced_rw<8, 1>, g);
      run("K2 own", paced_rw<2, 0>, g);
    }
  }
  return 0;
}
