// Round-trip latency of the one-wave mailbox (tools/ubench/mailbox.hip) with the REQUEST block
// in fine-grained device memory written by the host through the BAR (posted writes; the wave
// polls local memory instead of reading across PCIe), the response still in coherent
// page-locked host memory.  Prints "no host access" and exits if the device memory cannot be
// mapped for the host.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/mailbox_vram.hip -o tools/ubench/mailbox_vram
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

struct alignas(256) Req {
  uint32_t req;
  uint32_t pad0[63];
  double in[64];
};
struct alignas(256) Resp {
  uint32_t done;
  uint32_t pad1[63];
  double out[64];
  uint32_t exited;
};

__global__ void server_k(const Req* q, Resp* r, uint64_t idle_ticks, uint64_t max_ticks) {
  const int lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = t0;
  uint32_t seen = 0;
  for (;;) {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_load(&q->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    v = __builtin_amdgcn_readfirstlane(v);
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (v == 0xffffffffu || now - last > idle_ticks || now - t0 > max_ticks) break;
    if (v == seen) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    seen = v;
    last = now;
    const double x = __hip_atomic_load(&q->in[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->out[lane], x * 2.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (lane == 0) __hip_atomic_store(&r->done, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (lane == 0) __hip_atomic_store(&r->exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  Req* q = nullptr;
  Resp* r = nullptr;
  if (hipExtMallocWithFlags((void**)&q, sizeof(Req), hipDeviceMallocFinegrained) != hipSuccess) {
    printf("no fine-grained device memory\n");
    return 0;
  }
  hipPointerAttribute_t at;
  Req* qh = q;                       // the device address itself, when the BAR maps it
  if (hipPointerGetAttributes(&at, q) == hipSuccess && at.hostPointer != nullptr) qh = (Req*)at.hostPointer;
  printf("host pointer %p (device %p)\n", (void*)qh, (void*)q);
  fflush(stdout);
  (void)hipMemset(q, 0, sizeof(Req));
  (void)hipDeviceSynchronize();
  printf("host read of the request word: %u\n", __atomic_load_n(&qh->req, __ATOMIC_ACQUIRE));
  fflush(stdout);
  if (hipHostMalloc((void**)&r, sizeof(Resp), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
  memset((void*)r, 0, sizeof(Resp));
  (void)hipMemset(q, 0, sizeof(Req));
  (void)hipDeviceSynchronize();
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  server_k<<<1, 64, 0, s>>>(q, r, 2000000ull, 200000000ull);
  double in[64], out[64];
  for (int i = 0; i < 64; ++i) in[i] = i * 0.25;
  std::vector<double> t;
  int bad = 0, lost = 0;
  for (int it = 1; it <= 3000; ++it) {
    const auto a = std::chrono::steady_clock::now();
    memcpy((void*)qh->in, in, sizeof(in));
    __atomic_thread_fence(__ATOMIC_SEQ_CST);          // the input's posted writes before the word
    __atomic_store_n(&qh->req, (uint32_t)it, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();                          // out of the write-combining buffer now
    const auto lim = a + std::chrono::milliseconds(10);
    while (__atomic_load_n(&r->done, __ATOMIC_ACQUIRE) != (uint32_t)it) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() > lim) { ++lost; break; }
    }
    memcpy(out, (const void*)r->out, sizeof(out));
    const auto z = std::chrono::steady_clock::now();
    for (int i = 0; i < 64; ++i) bad += out[i] != in[i] * 2.0;
    if (it > 100) t.push_back(std::chrono::duration<double, std::micro>(z - a).count());
    in[it & 63] += 1.0;
    if (lost) break;
  }
  __atomic_store_n(&qh->req, 0xffffffffu, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
  (void)hipStreamSynchronize(s);
  std::sort(t.begin(), t.end());
  printf("vram-request mailbox round trip: median %.2f us, p10 %.2f, p90 %.2f over %zu calls; wrong %d lost %d exited %u\n",
         t.empty() ? 0 : t[t.size() / 2], t.empty() ? 0 : t[t.size() / 10],
         t.empty() ? 0 : t[t.size() * 9 / 10], t.size(), bad, lost, r->exited);
  return bad || lost;
}
