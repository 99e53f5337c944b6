// Round-trip latency of a persistent one-wave "tiny call" server: the host writes a request
// (512 B of float64 + a sequence word) into coherent page-locked memory, a resident wave that
// polls the sequence word with system-scope loads reads the request, doubles the 64 values,
// writes them back into page-locked memory and releases a completion word the host spins on.
// Against the launch-per-call path of tools/ubench/tiny_call.hip (~6.4-7 us).
// Variants: W polling waves (see server_k).  The server ends on a stop request, after 20 ms without a request, or after 2 s in any case
// (s_memrealtime, 100 MHz), so the grid always drains.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/mailbox.hip -o tools/ubench/mailbox && tools/ubench/mailbox
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

struct alignas(256) Box {
  uint32_t req;            // host -> device: request sequence (0xffffffff: stop)
  uint32_t pad0[63];
  double in[64];
  uint32_t done;           // device -> host: completed sequence
  uint32_t pad1[63];
  double out[64];
  uint32_t exited;         // device -> host: the server has left its loop
};

// W waves poll the request word independently, started a fraction of a poll apart, so a request
// is seen about a W-th of a read round trip sooner; the first wave to see it claims it through an
// LDS compare-and-swap and serves it.
__global__ void server_k(Box* b, uint64_t idle_ticks, uint64_t max_ticks, int stagger) {
  __shared__ uint32_t served;
  __shared__ uint32_t left;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (threadIdx.x == 0) served = 0, left = 0;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = t0;
  uint32_t seen = 0;
  for (int i = 0; i < wave * stagger; ++i) __builtin_amdgcn_s_sleep(8);
  for (;;) {
    uint32_t r = 0;
    if (lane == 0) r = __hip_atomic_load(&b->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    r = __builtin_amdgcn_readfirstlane(r);
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (r == 0xffffffffu || now - last > idle_ticks || now - t0 > max_ticks) break;
    if (r == seen) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    seen = r;
    last = now;
    uint32_t won = 0;
    if (lane == 0) {
      uint32_t cur = __hip_atomic_load(&served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      won = cur != r && __hip_atomic_compare_exchange_strong(&served, &cur, r, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (!__builtin_amdgcn_readfirstlane(won)) continue;
    const double v = __hip_atomic_load(&b->in[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&b->out[lane], v * 2.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");       // the wave's stores before the flag
    if (lane == 0) __hip_atomic_store(&b->done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  uint32_t last_out = 0;
  if (lane == 0) last_out = __hip_atomic_fetch_add(&left, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == (uint32_t)nw - 1;
  if (lane == 0 && last_out) __hip_atomic_store(&b->exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static int run(Box* b, hipStream_t s, int waves, int stagger) {
  memset((void*)b, 0, sizeof(Box));
  server_k<<<1, 64 * waves, 0, s>>>(b, 2000000ull /*20 ms*/, 200000000ull /*2 s*/, stagger);
  double in[64], out[64];
  for (int i = 0; i < 64; ++i) in[i] = i * 0.25;
  std::vector<double> t;
  int bad = 0, lost = 0;
  for (int it = 1; it <= 3000; ++it) {
    const auto a = std::chrono::steady_clock::now();
    memcpy((void*)b->in, in, sizeof(in));
    __atomic_store_n(&b->req, (uint32_t)it, __ATOMIC_RELEASE);
    const auto lim = a + std::chrono::milliseconds(10);
    while (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) != (uint32_t)it) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() > lim) { ++lost; break; }
    }
    memcpy(out, (const void*)b->out, sizeof(out));
    const auto z = std::chrono::steady_clock::now();
    for (int i = 0; i < 64; ++i) bad += out[i] != in[i] * 2.0;
    if (it > 100) t.push_back(std::chrono::duration<double, std::micro>(z - a).count());
    in[it & 63] += 1.0;
    if (lost) break;
  }
  __atomic_store_n(&b->req, 0xffffffffu, __ATOMIC_RELEASE);
  hipStreamSynchronize(s);
  const double med = median(t);
  std::sort(t.begin(), t.end());
  printf("mailbox round trip, %d wave(s), stagger %3d: median %.2f us, p10 %.2f, p90 %.2f over %zu calls; "
         "wrong %d lost %d exited %u\n", waves, stagger, med, t.empty() ? 0 : t[t.size() / 10],
         t.empty() ? 0 : t[t.size() * 9 / 10], t.size(), bad, lost, b->exited);
  return bad || lost;
}

int main() {
  Box* b = nullptr;
  if (hipHostMalloc((void**)&b, sizeof(Box), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    printf("hipHostMalloc failed\n");
    return 1;
  }
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int fail = 0;
  const int cfg[][2] = {{1, 0}, {2, 0}, {2, 40}, {4, 0}, {4, 20}, {8, 10}, {16, 5}, {1, 0}};
  for (const auto& c : cfg) fail |= run(b, s, c[0], c[1]);
  hipHostFree(b);
  return fail;
}
