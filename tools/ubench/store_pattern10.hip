// Write-pattern microbenchmark, part 10: as part 8 (K = 4 read bursts) with the input read
// modulo a window of `wrap` bytes — a window small enough to stay in the 256 MiB Infinity
// Cache shows what the read stream costs the writes when it does not reach HBM.
// Part 8 text: as part 7, but each wave reads the
// input of its next K groups at once, at the first slot of every K-slot epoch, so the read
// stream arrives in chip-wide bursts instead of an even 1:12 mix with the writes.
// (part 7 text follows) paced 6 KiB group stores (as store_pattern6) with the
// intra kernel's input reads mixed in — per group 512 B read either in the kernel's tile
// shape (8 image rows x 64 B of a 4K luma frame, rows 3840 B apart) or as one contiguous
// 512 B run — to see what the read stream costs the write stream and whether its shape
// matters.  The read data is folded into the stored value, two groups of prefetch.
//   hipcc --offload-arch=gfx950 -O3 -o ub/sp10 tools/ubench/store_pattern10.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__global__ void stamp(uint64_t* t) { *t = __builtin_amdgcn_s_memrealtime() + 300; }

enum { RD_NONE = 0, RD_TILE = 1, RD_SEQ = 2 };

template <int MODE, int K>
__global__ __launch_bounds__(256) void paced_rw(uint8_t* out, int64_t ngroups, const uint8_t* in,
                                                int64_t in_bytes, const uint64_t* t0p,
                                                uint32_t D, int64_t wrap) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w = blockIdx.x * 4 + wave;
  uint64_t rel = D ? (*t0p << 8) + (uint64_t)D * (uint64_t)w / (uint64_t)nw : 0;
  auto load = [&](int64_t G) -> u32x2 {
    if (MODE == RD_NONE) return u32x2{0, 0};
    int64_t o;
    if (MODE == RD_TILE) {
      const int64_t f = G / (60 * 270), rem = G - f * 60 * 270;
      const int64_t bi = rem / 60, gc = rem - bi * 60;
      o = (f * 2160 + 8 * bi + (lane >> 3)) * 3840 + gc * 64 + 8 * (lane & 7);
    } else {
      o = G * 512 + lane * 8;
    }
    o %= wrap;
    const bool ok = G < ngroups && o + 8 <= in_bytes;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(in) + (ok ? (o & ~(int64_t)0xffff) : 0), 0, ok ? 0x20000 : 0, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(o & 0xffff), 0, 0);
  };
  u32x2 cur[K], nxt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) cur[k] = load(w + k * nw);
  for (int64_t G0 = w; G0 < ngroups; G0 += K * nw) {
#pragma unroll
    for (int k = 0; k < K; ++k) nxt[k] = load(G0 + (K + k) * nw);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t G = G0 + k * nw;
      u32x4 v = {cur[k].x, cur[k].y, 3u, 4u};
      if (D) {
        uint64_t now = __builtin_amdgcn_s_memrealtime();
        while ((now << 8) < rel) {
          __builtin_amdgcn_s_sleep(1);
          now = __builtin_amdgcn_s_memrealtime();
        }
        rel += D;
      }
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + G * 6144, 0, G < ngroups ? 6144 : 0, 0x00020000);
#pragma unroll
      for (int j = 0; j < 6; ++j) __builtin_amdgcn_raw_buffer_store_b128(v, rs, j * 1024 + lane * 16, 0, 2);
    }
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
  int64_t wrap = in_bytes;
  auto run = [&](const char* name, auto K, double gbps, bool reads) {
    const double bytes_per_group = 6144.0 + (reads ? 512.0 : 0.0);
    const uint32_t D = gbps > 0 ? (uint32_t)(grid * 4.0 * bytes_per_group / (gbps * 1e9) * 1e8 * 256) : 0;
    float tot = 0;
    for (int i = 0; i < 4; ++i) {
      (void)hipEventRecord(a);
      stamp<<<1, 1>>>(t0);
      K<<<grid, 256>>>(out, ngroups, in, in_bytes, t0, D, wrap);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b); if (i) tot += ms;
    }
    tot /= 3;
    const double tb = out_bytes + (reads ? in_bytes : 0);
    printf("wrap %5lld MiB %-10s pace %5.0f  %7.3f ms  %7.1f GB/s total  %7.1f GB/s writes\n", (long long)(wrap >> 20), name, gbps, tot,
           tb / tot / 1e6, out_bytes / tot / 1e6);
  };
  for (int64_t wr : {(int64_t)64 << 20, (int64_t)160 << 20, in_bytes}) {
    wrap = wr;
    for (double g : {0.0, 6000.0, 6400.0, 6800.0, 7200.0}) {
      run("tile K4", paced_rw<RD_TILE, 4>, g, true);
      run("tile K1", paced_rw<RD_TILE, 1>, g, true);
    }
  }
  return 0;
}
