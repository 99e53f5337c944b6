// Write-pattern microbenchmark, part 11: part 10 showed that input reads served by the
// 256 MiB Infinity Cache cost the paced write sweep nothing (7.2 TB/s total), while the same
// reads from HBM cap it near 6.0–6.4.  Here every wave, at the first slot of each P-slot epoch,
// prefetches the input of its groups P..2P-1 slots ahead (the same addresses, 8 B per lane,
// results folded into a dummy sum one epoch later), so the HBM reads arrive in bursts and the
// per-slot loads hit the Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -o ub/sp11 tools/ubench/store_pattern11.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__global__ void stamp(uint64_t* t) { *t = __builtin_amdgcn_s_memrealtime() + 300; }

template <int P>
__global__ __launch_bounds__(256) void paced_pf(uint8_t* out, int64_t ngroups, const uint8_t* in,
                                                int64_t in_bytes, const uint64_t* t0p, uint32_t D,
                                                uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w = blockIdx.x * 4 + wave;
  uint64_t rel = D ? (*t0p << 8) + (uint64_t)D * (uint64_t)w / (uint64_t)nw : 0;
  auto load = [&](int64_t G) -> u32x2 {
    const int64_t f = G / (60 * 270), rem = G - f * 60 * 270;
    const int64_t bi = rem / 60, gc = rem - bi * 60;
    const int64_t o = (f * 2160 + 8 * bi + (lane >> 3)) * 3840 + gc * 64 + 8 * (lane & 7);
    const bool ok = G < ngroups && o + 8 <= in_bytes;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(in) + (ok ? (o & ~(int64_t)0xffff) : 0), 0, ok ? 0x20000 : 0, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(o & 0xffff), 0, 0);
  };
  u32x2 pf[P > 0 ? P : 1];
  uint32_t dummy = 0;
  if (P > 0) {
#pragma unroll
    for (int k = 0; k < P; ++k) pf[k] = load(w + k * nw);     // epoch 0's own input
  }
  u32x2 nx = load(w);
  int64_t s = 0;
  for (int64_t G = w; G < ngroups; G += nw, ++s) {
    if (P > 0 && (s % (P > 0 ? P : 1)) == 0) {
#pragma unroll
      for (int k = 0; k < P; ++k) dummy += pf[k].x ^ pf[k].y;  // last epoch's prefetches
#pragma unroll
      for (int k = 0; k < P; ++k) pf[k] = load(G + (P + k) * nw);
    }
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
  if (dummy == 0x12345678u) *sink = dummy;
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
  auto run = [&](const char* name, auto K, double gbps) {
    const uint32_t D = gbps > 0 ? (uint32_t)(grid * 4.0 * 6656.0 / (gbps * 1e9) * 1e8 * 256) : 0;
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
    printf("%-8s pace %5.0f  %7.3f ms  %7.1f GB/s total (ideal %.3f ms)\n", name, gbps, tot,
           tb / tot / 1e6, gbps > 0 ? tb / gbps / 1e6 : 0.0);
  };
  for (int rep = 0; rep < 2; ++rep)
    for (double g : {0.0, 6400.0, 6800.0, 7200.0}) {
      run("no pf", paced_pf<0>, g);
      run("pf 8", paced_pf<8>, g);
      run("pf 16", paced_pf<16>, g);
      run("pf 32", paced_pf<32>, g);
    }
  return 0;
}
