// ivc_capi.hip — the extern "C" boundary of libivc.so (declared in include/ivc.h).
//
// Validates arguments the way the reference's NumPy code would fail (shape / dtype), maps
// launch errors to status codes with a per-thread message, and implements the host-buffer
// entry points by staging through per-device scratch memory on a library-owned stream.
#include <stdio.h>
#include <string.h>

#include <condition_variable>
#include <functional>
#include <list>
#include <map>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <cstdlib>
#include <vector>

#include "ivc_internal.h"

namespace ivc {
// ivc_set_tuning overrides, read once per call by the launchers
std::atomic<int> g_tuning[IVC_TUNE_COUNT] = {};
int tuning(int key) { return g_tuning[key].load(std::memory_order_relaxed); }
}  // namespace ivc

using namespace ivc;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int fail_hip(hipError_t e, const char* what) {
  return fail(IVC_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

bool valid_dtype(int dt) { return dt >= IVC_U8 && dt <= IVC_F64; }
bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// ---------------------------------------------------------------- host copies ----------
// Host buffers handed to the library are pageable NumPy memory: hipMemcpy from or to them
// runs at ~10 GB/s.  Large transfers instead go through a per-device ring of pinned chunks:
// the CPU copies chunk k between the caller's buffer and a pinned slot (split over a small
// thread pool) while the DMA engine moves chunk k - 1 (H2D) or k + 1 (D2H) at pinned speed.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool;      // never destroyed: its detached workers block on it
    return *p;
  }
  // memcpy of n bytes split over the pool's workers and the calling thread
  void copy(void* dst, const void* src, size_t n) {
    const size_t min_part = 1u << 20;
    int parts = (int)std::min<size_t>(workers_.size() + 1, std::max<size_t>(1, n / min_part));
    if (parts <= 1) {
      memcpy(dst, src, n);
      return;
    }
    const size_t step = (n / parts + 63) & ~(size_t)63;
    std::unique_lock<std::mutex> lk(mu_);
    int pending = 0;
    for (int i = 1; i < parts; ++i) {
      const size_t off = step * i;
      if (off >= n) break;
      const size_t len = std::min(step, n - off);
      ++pending;
      tasks_.push_back([=] { memcpy((char*)dst + off, (const char*)src + off, len); });
    }
    outstanding_ += pending;
    lk.unlock();
    cv_.notify_all();
    memcpy(dst, src, std::min(step, n));
    lk.lock();
    done_cv_.wait(lk, [&] { return outstanding_ == 0; });
  }

 private:
  CopyPool() {
    unsigned hw = std::thread::hardware_concurrency();
    const int nw = (int)std::max(1u, std::min(7u, hw > 2 ? hw / 2 - 1 : 1u));
    for (int i = 0; i < nw; ++i) workers_.emplace_back([this] { run(); });
    for (auto& t : workers_) t.detach();     // process-long (no join at exit)
  }
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !tasks_.empty(); });
        f = std::move(tasks_.back());
        tasks_.pop_back();
      }
      f();
      std::lock_guard<std::mutex> lk(mu_);
      if (--outstanding_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::function<void()>> tasks_;
  std::vector<std::thread> workers_;
  int outstanding_ = 0;
};

// ---------------------------------------------------------------- pinned host blocks ---
// ivc_host_alloc: page-locked host memory the drop-in classes allocate their NumPy results in
// (ivclab_amd._native.empty).  A transfer between such a block and the device is one DMA at
// full PCIe speed with no CPU copy and no first-touch page faults; freed blocks are cached by
// size (up to host_cache_max(): 1 GiB, or IVC_HOST_CACHE_MB; past it the oldest cached blocks
// are released) so repeated calls of the same shapes reuse them; ivc_release_scratch returns
// the cached blocks to the system.
std::mutex g_host_mu;
std::map<uintptr_t, size_t> g_host_live;          // block start -> bytes
std::list<std::pair<size_t, void*>> g_host_cache; // freed blocks, oldest first
size_t g_host_cached = 0;
constexpr size_t kHostGrain = 2u << 20;

size_t host_cache_max() {
  static const size_t v = [] {
    const char* e = getenv("IVC_HOST_CACHE_MB");
    if (e && *e) {
      char* end = nullptr;
      const long long mb = strtoll(e, &end, 10);
      if (end && *end == 0 && mb >= 0) return (size_t)mb << 20;
    }
    return (size_t)1 << 30;
  }();
  return v;
}

void host_cache_drain() {
  std::lock_guard<std::mutex> g(g_host_mu);
  for (auto& kv : g_host_cache) (void)hipHostFree(kv.second);
  g_host_cache.clear();
  g_host_cached = 0;
}

bool host_pinned(const void* p, size_t bytes) {
  std::lock_guard<std::mutex> g(g_host_mu);
  const uintptr_t a = (uintptr_t)p;
  auto it = g_host_live.upper_bound(a);
  if (it == g_host_live.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}

// ---------------------------------------------------------------- device context -------
constexpr int kMaxDev = 64;
constexpr int kSlots = 6;
constexpr int kPinSlots = 4;
constexpr size_t kPinChunk = 8u << 20;      // bytes per pinned slot
constexpr size_t kPinMin = 1u << 20;        // smaller transfers go straight from pageable memory
constexpr int kAux = 3;                     // pipelined host-buffer calls: streams
constexpr size_t kPipeMin = 4u << 20;       // smaller outputs go in one piece
// bytes per pipelined chunk (the larger of in / out); 0 = no pipelining (ivc_set_host_pipeline).
// Off by default: on the MI355X boxes measured the host link is effectively half duplex
// (56.6 GB/s one way, 27.5 GB/s each way at once), so overlapping one chunk's upload with
// another's download gains nothing and the chunking costs 5-12 % (profiles/r04g_class_api.json)
std::atomic<size_t> g_pipe_chunk{0};
struct DevCtx {
  std::mutex mu;
  hipStream_t stream = nullptr;
  hipStream_t aux[kAux] = {};
  hipEvent_t aux_ev = nullptr;              // the main stream's upload, for the aux streams
  int aux_state = 0;                        // 0 untried, 1 ready, -1 unavailable
  void* tiny = nullptr;                     // page-locked, device-mapped block for tiny calls
  int tiny_state = 0;                       // 0 untried, 1 ready, -1 unavailable
  uint32_t tiny_seq = 0;                    // last completion value written behind a tiny call
  uint32_t* tiny_count = nullptr;           // finished workgroups of the running tiny call
  double* tiny_tab = nullptr;               // device copy of the last quantiser table of a tiny call
  QTab tiny_tab_host;                       // its values
  bool tiny_tab_valid = false;
  // the resident tiny-call server (tiny_server_kernel): its mailbox (coherent page-locked
  // host memory), its own stream, the generation of the last launch and the request sequence
  SrvBox* srv = nullptr;
  hipStream_t srv_stream = nullptr;
  int srv_state = 0;                        // 0 untried, 1 ready, -1 unavailable
  bool srv_launched = false;
  uint32_t srv_gen = 0, srv_seq = 0, srv_tab_ver = 0;
  QTab srv_tab;
  bool srv_tab_valid = false;
  void* slot[kSlots] = {};
  size_t cap[kSlots] = {};
  void* pin[kPinSlots] = {};
  hipEvent_t pin_ev[kPinSlots] = {};
  int pin_state = 0;                        // 0 untried, 1 ready, -1 unavailable
  int pin_next = 0;
};
DevCtx g_ctx[kMaxDev];

bool aux_ready(DevCtx* c) {
  if (c->aux_state == 0) {
    c->aux_state = 1;
    for (int i = 0; i < kAux && c->aux_state == 1; ++i)
      if (hipStreamCreateWithFlags(&c->aux[i], hipStreamNonBlocking) != hipSuccess) c->aux_state = -1;
    if (c->aux_state == 1 && hipEventCreateWithFlags(&c->aux_ev, hipEventDisableTiming) != hipSuccess)
      c->aux_state = -1;
    (void)hipGetLastError();
  }
  return c->aux_state == 1;
}

constexpr size_t kTinyMax = 64u << 10;      // bytes of input and of output for a tiny call

// after the input and output blocks: the completion word a tiny call's stream writes
constexpr size_t kTinyFlag = 2 * kTinyMax;
bool tiny_ready(DevCtx* c) {
  if (c->tiny_state == 0) {
    // coherent (fine-grained) whatever HIP_HOST_COHERENT says: the host reads the completion
    // word and the output the kernel released at system scope straight from this block
    c->tiny_state = hipHostMalloc(&c->tiny, 2 * kTinyMax + 256,
                                  hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess ? 1 : -1;
    if (c->tiny_state == 1) *reinterpret_cast<volatile uint32_t*>((char*)c->tiny + kTinyFlag) = 0;
    // the finished-workgroup counter of tiny_done (device memory, left at 0 by every call)
    if (c->tiny_state == 1 && (hipMalloc((void**)&c->tiny_count, 4) != hipSuccess ||
                               hipMemset(c->tiny_count, 0, 4) != hipSuccess))
      c->tiny_state = -1;
    (void)hipGetLastError();
  }
  return c->tiny_state == 1;
}

// The device copy of a tiny quantise / dequantise call's table (the per-block loops pass the
// same table every call): compared by value, copied (synchronously: rare) when it changes;
// nullptr when no copy can be made (the table then travels in the arguments).
const double* tiny_table(DevCtx* c, const QTab& t) {
  if (!c->tiny_tab && hipMalloc((void**)&c->tiny_tab, sizeof(QTab)) != hipSuccess) {
    c->tiny_tab = nullptr;
    (void)hipGetLastError();
    return nullptr;
  }
  if (!c->tiny_tab_valid || memcmp(c->tiny_tab_host.q, t.q, sizeof(QTab)) != 0) {
    c->tiny_tab_valid = false;
    // stream-ordered behind any earlier tiny call that still reads the old copy
    if (hipMemcpyAsync(c->tiny_tab, t.q, sizeof(QTab), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    c->tiny_tab_host = t;
    c->tiny_tab_valid = true;
  }
  return c->tiny_tab;
}

bool pinned_ready(DevCtx* c) {
  if (c->pin_state == 0) {
    c->pin_state = 1;
    for (int i = 0; i < kPinSlots && c->pin_state == 1; ++i)
      if (hipHostMalloc(&c->pin[i], kPinChunk, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming) != hipSuccess)
        c->pin_state = -1;                  // keep what was allocated; use the pageable path
    (void)hipGetLastError();
  }
  return c->pin_state == 1;
}

// at process exit, every resident tiny-call server is asked to leave (it would leave by itself
// after its idle time in any case)
void stop_servers() {
  for (int d = 0; d < kMaxDev; ++d) {
    DevCtx& c = g_ctx[d];
    if (c.srv_state == 1 && c.srv_launched && c.srv) __atomic_store_n(&c.srv->h.req, SRV_STOP, __ATOMIC_RELEASE);
  }
}
void register_server_exit() {
  static std::once_flag once;
  std::call_once(once, [] { std::atexit(stop_servers); });
}

int current_device(int* dev) {
  hipError_t e = hipGetDevice(dev);
  if (e != hipSuccess) return fail_hip(e, "hipGetDevice");
  if (*dev < 0 || *dev >= kMaxDev) return fail(IVC_E_DEVICE, "device index out of range");
  return IVC_OK;
}

// Host-buffer call: lock the device context, stage inputs, run, copy outputs back.
struct Staging {
  DevCtx* ctx = nullptr;
  int next = 0;
  int status = IVC_OK;
  std::unique_lock<std::mutex> lock;

  int open() {
    int dev = 0;
    int rc = current_device(&dev);
    if (rc) return rc;
    ctx = &g_ctx[dev];
    lock = std::unique_lock<std::mutex>(ctx->mu);
    if (!ctx->stream) {
      hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
      if (e != hipSuccess) return fail_hip(e, "hipStreamCreate");
    }
    return IVC_OK;
  }
  void* alloc(size_t bytes) {
    if (status) return nullptr;
    if (next >= kSlots) { status = fail(IVC_E_ARG, "internal: too many staging buffers"); return nullptr; }
    const int i = next++;
    if (bytes == 0) bytes = 16;
    if (ctx->cap[i] < bytes) {
      if (ctx->slot[i]) (void)hipFree(ctx->slot[i]);
      ctx->slot[i] = nullptr;
      ctx->cap[i] = 0;
      hipError_t e = hipMalloc(&ctx->slot[i], bytes);
      if (e != hipSuccess) {
        status = fail(IVC_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        return nullptr;
      }
      ctx->cap[i] = bytes;
    }
    return ctx->slot[i];
  }
  // next pinned slot, once the DMA that last used it has finished
  int take_pin() {
    const int k = ctx->pin_next;
    ctx->pin_next = (k + 1) % kPinSlots;
    hipError_t e = hipEventSynchronize(ctx->pin_ev[k]);
    if (e != hipSuccess) status = fail_hip(e, "hipEventSynchronize");
    return k;
  }
  void* in(const void* host, size_t bytes) {
    void* d = alloc(bytes);
    if (!d || !bytes) return d;
    if (bytes < kPinMin || host_pinned(host, bytes) || !pinned_ready(ctx)) {
      hipError_t e = hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, ctx->stream);
      if (e != hipSuccess) status = fail_hip(e, "hipMemcpyAsync H2D");
      return d;
    }
    // CPU copy of chunk k into a pinned slot overlaps the DMA of chunk k - 1
    for (size_t off = 0; off < bytes && !status; off += kPinChunk) {
      const size_t n = std::min(kPinChunk, bytes - off);
      const int k = take_pin();
      if (status) break;
      CopyPool::get().copy(ctx->pin[k], (const char*)host + off, n);
      hipError_t e = hipMemcpyAsync((char*)d + off, ctx->pin[k], n, hipMemcpyHostToDevice, ctx->stream);
      if (e == hipSuccess) e = hipEventRecord(ctx->pin_ev[k], ctx->stream);
      if (e != hipSuccess) status = fail_hip(e, "hipMemcpyAsync H2D");
    }
    return d;
  }
  int launched(hipError_t e, const char* what) {
    if (status) return status;
    if (e == hipErrorInvalidValue) return status = fail(IVC_E_DTYPE, std::string(what) + ": unsupported dtype/argument combination");
    if (e != hipSuccess) return status = fail_hip(e, what);
    return IVC_OK;
  }
  int out(void* host, const void* dev, size_t bytes) {
    if (status) return status;
    if (!bytes) return IVC_OK;
    if (bytes < kPinMin || host_pinned(host, bytes) || !pinned_ready(ctx)) {
      hipError_t e = hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream);
      if (e != hipSuccess) return status = fail_hip(e, "hipMemcpyAsync D2H");
      return IVC_OK;
    }
    // up to kPinSlots DMAs in flight; the CPU drains chunk k into the caller's buffer while
    // the DMA engine fills the next slots (synchronous: the data is in `host` on return)
    const size_t nchunk = (bytes + kPinChunk - 1) / kPinChunk;
    std::vector<int> slot_of(nchunk);
    auto issue = [&](size_t c) {
      const size_t off = c * kPinChunk, n = std::min(kPinChunk, bytes - off);
      const int k = take_pin();
      if (status) return;
      slot_of[c] = k;
      hipError_t e = hipMemcpyAsync(ctx->pin[k], (const char*)dev + off, n, hipMemcpyDeviceToHost,
                                    ctx->stream);
      if (e == hipSuccess) e = hipEventRecord(ctx->pin_ev[k], ctx->stream);
      if (e != hipSuccess) status = fail_hip(e, "hipMemcpyAsync D2H");
    };
    size_t issued = 0;
    for (; issued < nchunk && issued < (size_t)kPinSlots - 1 && !status; ++issued) issue(issued);
    for (size_t c = 0; c < nchunk && !status; ++c) {
      const int k = slot_of[c];
      hipError_t e = hipEventSynchronize(ctx->pin_ev[k]);
      if (e != hipSuccess) return status = fail_hip(e, "hipEventSynchronize");
      const size_t off = c * kPinChunk, n = std::min(kPinChunk, bytes - off);
      if (issued < nchunk) issue(issued++);   // reuses a slot already drained
      CopyPool::get().copy((char*)host + off, ctx->pin[k], n);
    }
    return status;
  }
  // A unit-separable op (DCT blocks, quantiser blocks, zig-zag rows, block rows of an image)
  // from `src` to the page-locked `dst` (the drop-in's own result arrays, ivc_host_alloc):
  // chunks of units go upload -> kernel -> download round-robin on kAux streams, so one
  // chunk's upload, another's kernel and a third's download overlap (the PCIe link is full
  // duplex).  A page-locked `src` is uploaded chunk by chunk; a pageable one whole, through the
  // staging ring on the main stream, which the aux streams then wait for.  Returns false, with
  // nothing enqueued, when it does not apply (a small or pageable output): the caller then
  // runs the op in one piece.  launch(d_in, d_out, units, stream) -> hipError_t.
  template <typename L>
  bool pipelined(const void* src, size_t ib, void* dst, size_t ob, int64_t n, const char* what,
                 L&& launch) {
    if (status || n <= 0) return false;
    const size_t IB = ib * (size_t)n, OB = ob * (size_t)n;
    const size_t chunk = g_pipe_chunk.load(std::memory_order_relaxed);
    if (chunk == 0 || OB < kPipeMin || !host_pinned(dst, OB) || !aux_ready(ctx)) return false;
    const bool in_pinned = host_pinned(src, IB);
    char* d_in = (char*)(in_pinned ? alloc(IB) : in(src, IB));
    char* d_out = (char*)alloc(OB);
    if (status) return true;
    if (!in_pinned) {
      hipError_t e = hipEventRecord(ctx->aux_ev, ctx->stream);
      for (int i = 0; i < kAux && e == hipSuccess; ++i) e = hipStreamWaitEvent(ctx->aux[i], ctx->aux_ev, 0);
      if (e != hipSuccess) { status = fail_hip(e, "hipStreamWaitEvent"); return true; }
    }
    const size_t big = ib > ob ? ib : ob;
    const int64_t per = (int64_t)(chunk / big > 0 ? chunk / big : 1);
    aux_used = true;
    for (int64_t u0 = 0, k = 0; u0 < n && !status; u0 += per, ++k) {
      hipStream_t s = ctx->aux[k % kAux];
      const int64_t nu = per < n - u0 ? per : n - u0;
      hipError_t e = hipSuccess;
      if (in_pinned)
        e = hipMemcpyAsync(d_in + u0 * ib, (const char*)src + u0 * ib, nu * ib, hipMemcpyHostToDevice, s);
      if (e != hipSuccess) { status = fail_hip(e, "hipMemcpyAsync H2D"); break; }
      e = launch(d_in + u0 * ib, d_out + u0 * ob, nu, s);
      if (launched(e, what)) break;
      e = hipMemcpyAsync((char*)dst + u0 * ob, d_out + u0 * ob, nu * ob, hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) status = fail_hip(e, "hipMemcpyAsync D2H");
    }
    return true;
  }
  bool aux_used = false;
  // A tiny call (one 8x8 block, a (3, 8, 8) stack: the reference's per-block loops,
  // exercises/ch3/E3-1_claude.py:47-60): the input travels inside the kernel arguments (up
  // to kTinyInline bytes; larger ones are copied into a page-locked block the device
  // addresses directly), the kernel writes its output into page-locked memory over the bus
  // (no DMA transfers to set up), then one wait and a copy out: one launch per call.
  // Returns false, nothing done, when the sizes do not qualify.
  //   Completion: the op's kernel itself — its last workgroup to finish (tiny_done,
  // ivc_internal.h) — writes a sequence number into a page-locked word with a system-scope
  // release, and the host spins on it.  Per call (tools/ubench/tiny_call.hip,
  // profiles/r05_tiny_call.log): a blocking hipStreamSynchronize costs ~5 us more, a second
  // one-wave kernel writing the word ~2 us more (the inter-kernel gap), hipStreamWriteValue32
  // ~2.5 us more.  The spin gives up after 50 ms and synchronises, which also reports a failed
  // kernel.
  template <typename L>
  bool tiny(const void* src, size_t IB, void* dst, size_t OB, const char* what, L&& launch) {
    if (status || IB > kTinyMax || OB > kTinyMax || !tiny_ready(ctx)) return false;
    char* ti = (char*)ctx->tiny;
    char* to = ti + kTinyMax;
    uint32_t* flag = reinterpret_cast<uint32_t*>(ti + kTinyFlag);
    const uint32_t seq = ++ctx->tiny_seq;
    TinyDone td{flag, ctx->tiny_count, seq};
    if (IB <= (size_t)kTinyInline) {           // the input rides in the kernel arguments
      td.inl = src;
      td.inl_bytes = IB;
      td.stage = ti;                          // ... or, past the launcher's capacity, in `ti`
    } else if (IB) {
      memcpy(ti, src, IB);
    }
    if (launched(launch(ti, to, ctx->stream, &td), what)) return true;
    bool done = false;
    const auto t0 = std::chrono::steady_clock::now();
    // busy-spin for the first ~200 us (a tiny call finishes in ~7 us on an idle GPU), then
    // yield the core between polls while the GPU is busy with other work
    bool relaxed = false;
    for (uint32_t i = 1;; ++i) {
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) {
        done = true;
        break;
      }
      if (relaxed) std::this_thread::yield();
      else __builtin_ia32_pause();
      if ((i & 255u) == 0) {
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > std::chrono::milliseconds(50)) break;
        relaxed = dt > std::chrono::microseconds(200);
      }
    }
    if (!done) {
      hipError_t e = hipStreamSynchronize(ctx->stream);
      if (e != hipSuccess) { status = fail_hip(e, "hipStreamSynchronize"); return true; }
    }
    if (OB) memcpy(dst, to, OB);
    return true;
  }
  // A per-block call through the resident tiny-call server (ivc_kernels.hip tiny_server_kernel):
  // the request is written into the mailbox, the server's wave answers it, the output is copied
  // out — no kernel launch per call (tools/ubench/mailbox.hip: 4.0-4.2 us per round trip against
  // ~6.4 us for a launch and its completion).  The server leaves after kSrvIdle ticks without a
  // request (so a device-wide synchronisation waits at most that long after the last call) or
  // kSrvLife in all, and is relaunched on the next call.  Returns false (the caller then takes
  // the launch path) when the server is off (ivc_set_tuning(IVC_TUNE_TINY_SERVER, 1)),
  // unavailable, retired, or the call too large.
  static constexpr uint64_t kSrvIdle = 50000, kSrvLife = 100000000;     // 0.5 ms, 1 s (100 MHz)
  bool server(uint32_t op, int sdt, int ddt, int inverse, int ortho, double fct, int C, const QTab* t,
              const void* src, size_t IB, void* dst, size_t OB) {
    if (status || tuning(IVC_TUNE_TINY_SERVER) == 1 || IB > (size_t)SRV_IO || OB > (size_t)SRV_IO)
      return false;
    DevCtx* c = ctx;
    if (c->srv_state == 0) {
      c->srv_state = -1;
      if (hipHostMalloc((void**)&c->srv, sizeof(SrvBox), hipHostMallocCoherent | hipHostMallocMapped) ==
              hipSuccess &&
          hipStreamCreateWithFlags(&c->srv_stream, hipStreamNonBlocking) == hipSuccess) {
        memset((void*)c->srv, 0, sizeof(SrvBox));
        c->srv_state = 1;
        register_server_exit();
      }
      (void)hipGetLastError();
    }
    if (c->srv_state != 1) return false;
    SrvBox* b = c->srv;
    auto relaunch = [&]() -> bool {
      if (++c->srv_gen == 0) c->srv_gen = 1;
      if (launch_tiny_server(b, c->srv_gen, kSrvIdle, kSrvLife, c->srv_stream) != hipSuccess) {
        (void)hipGetLastError();
        c->srv_state = -1;
        c->srv_launched = false;
        return false;
      }
      c->srv_launched = true;
      return true;
    };
    auto gone = [&]() { return __atomic_load_n(&b->exited, __ATOMIC_ACQUIRE) == c->srv_gen; };
    if ((!c->srv_launched || gone()) && !relaunch()) return false;
    if (t && (!c->srv_tab_valid || memcmp(c->srv_tab.q, t->q, sizeof(QTab)) != 0)) {
      memcpy(b->tab, t->q, sizeof(QTab));
      if (++c->srv_tab_ver == 0) c->srv_tab_ver = 1;
      c->srv_tab = *t;
      c->srv_tab_valid = true;
    }
    uint32_t seq = ++c->srv_seq;
    if (seq == 0 || seq == SRV_STOP) seq = c->srv_seq = 1;
    // header and input, then the checksum the server verifies its one-read snapshot against
    // (over the header words with the new sequence and the whole input area), then the sequence
    SrvHdr hd;
    memset(&hd, 0, sizeof(hd));
    hd.req = seq;
    hd.op = op;
    hd.src_dtype = (uint32_t)sdt;
    hd.dst_dtype = (uint32_t)ddt;
    hd.inverse = (uint32_t)inverse;
    hd.ortho = (uint32_t)ortho;
    hd.C = (uint32_t)C;
    hd.tab_ver = c->srv_tab_ver;
    hd.nin = (uint32_t)IB;
    hd.nout = (uint32_t)OB;
    hd.fct = fct;
    memcpy((void*)b->in, src, IB);
    uint64_t hq[8];
    memcpy(hq, &hd, sizeof(hq));
    uint64_t sum = 0;
    for (uint32_t k = 0; k < 6; ++k) sum += srv_mix(hq[k], k);
    const volatile uint64_t* inw = b->in;
    for (uint32_t k = 0; k < (uint32_t)SRV_IO / 8; ++k) sum += srv_mix(inw[k], 6u + k);
    volatile uint32_t* hv = reinterpret_cast<volatile uint32_t*>(&b->h);
    const uint32_t* hs = reinterpret_cast<const uint32_t*>(&hd);
    for (int k = 1; k < 12; ++k) hv[k] = hs[k];                     // words after req
    __atomic_store_n(&b->h.sum, sum, __ATOMIC_RELEASE);
    __atomic_store_n(&b->h.req, seq, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
      if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq) break;
      __builtin_ia32_pause();
      if ((i & 255u) == 0) {
        // the server may have left between our check and the request: a new one serves it.
        // No answer within 200 ms (a relaunch queued behind a GPU full of other work, or no
        // relaunch possible): the server is retired for this process and this call, like every
        // later one, takes the launch path — slower, never an error.  A late server still
        // answers the posted request into the mailbox, which nothing reads any more, and leaves
        // after its idle time.
        if ((gone() && !relaunch()) ||
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
          c->srv_state = -1;
          return false;
        }
      }
    }
    memcpy(dst, (const void*)b->out, OB);
    return true;
  }
  int sync() {
    hipError_t e = hipSuccess;
    if (aux_used)
      for (int i = 0; i < kAux; ++i) {
        hipError_t ei = hipStreamSynchronize(ctx->aux[i]);
        if (e == hipSuccess) e = ei;
      }
    if (status) return status;
    hipError_t em = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = em;
    if (e != hipSuccess) return status = fail_hip(e, "hipStreamSynchronize");
    return IVC_OK;
  }
};

int dev_launch(hipError_t e, const char* what) {
  if (e == hipErrorInvalidValue)
    return fail(IVC_E_DTYPE, std::string(what) + ": unsupported dtype/argument combination");
  if (e != hipSuccess) return fail_hip(e, what);
  return IVC_OK;
}

int load_table(const double* table, QTab* t) {
  if (!table) return fail(IVC_E_ARG, "quantization table is NULL");
  memset(t, 0, sizeof(*t));
  for (int i = 0; i < 192; ++i) {
    t->q[i] = table[i];
    if (!(table[i] == table[i])) return fail(IVC_E_ARG, "quantization table holds NaN");
  }
  return IVC_OK;
}

#define CHECK(cond, code, msg) \
  do {                         \
    if (!(cond)) return fail(code, msg); \
  } while (0)
#define TRY(x)          \
  do {                  \
    int rc_ = (x);      \
    if (rc_) return rc_; \
  } while (0)

// ---------------------------------------------------------------- argument checks ------
int check_dct(int src_dtype, int64_t nblk, int dst_dtype, int norm) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "dct8x8: invalid source dtype");
  CHECK(dst_dtype == IVC_F32 || dst_dtype == IVC_F64, IVC_E_DTYPE, "dct8x8: output must be float32 or float64");
  CHECK((dst_dtype == IVC_F32) == (src_dtype == IVC_F32), IVC_E_DTYPE,
        "dct8x8: scipy computes float32 input in float32 and every other dtype in float64");
  CHECK(nblk >= 0, IVC_E_SHAPE, "dct8x8: negative block count");
  CHECK(norm >= 0 && norm <= 2, IVC_E_ARG, "dct8x8: norm must be backward/ortho/forward");
  return IVC_OK;
}
int check_quant(int src_dtype, int64_t nblk, int C, int calc) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "quantize: invalid source dtype");
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, "quantize: channel axis must broadcast against 3 table planes");
  CHECK(calc == IVC_F32 || calc == IVC_F64, IVC_E_DTYPE, "quantize: calc dtype must be float32/float64");
  CHECK(nblk >= 0, IVC_E_SHAPE, "quantize: negative block count");
  return IVC_OK;
}
int check_frames(int64_t nframes, int64_t H, int64_t W, const char* what) {
  CHECK(nframes >= 0 && H >= 0 && W >= 0, IVC_E_SHAPE, std::string(what) + ": negative size");
  CHECK(H % 8 == 0 && W % 8 == 0, IVC_E_SHAPE, std::string(what) + ": H and W must be multiples of 8");
  CHECK(H < (1LL << 30) && W < (1LL << 30), IVC_E_SHAPE, std::string(what) + ": frame too large");
  return IVC_OK;
}
int check_sr(int sr) {
  CHECK(sr >= 0 && sr <= 4096, IVC_E_ARG, "search_range must be in [0, 4096]");
  return IVC_OK;
}

}  // namespace

// ======================================================================================
extern "C" {

const char* ivc_last_error(void) { return g_err.c_str(); }
int ivc_version(void) { return 10000; }
int ivc_me_mfma_enabled(void) { return 1; }

int ivc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ivc_set_device(int device) {
  hipError_t e = hipSetDevice(device);
  return e == hipSuccess ? IVC_OK : fail_hip(e, "hipSetDevice");
}

int ivc_device_ok(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

void* ivc_host_alloc(int64_t bytes) {
  if (bytes <= 0) return nullptr;
  const size_t n = ((size_t)bytes + kHostGrain - 1) / kHostGrain * kHostGrain;
  std::lock_guard<std::mutex> g(g_host_mu);
  void* p = nullptr;
  // the most recently freed block of this size
  auto it = g_host_cache.end();
  for (auto j = g_host_cache.begin(); j != g_host_cache.end(); ++j)
    if (j->first == n) it = j;
  if (it != g_host_cache.end()) {
    p = it->second;
    g_host_cache.erase(it);
    g_host_cached -= n;
  } else if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  g_host_live[(uintptr_t)p] = n;
  return p;
}

int ivc_host_free(void* p) {
  if (!p) return IVC_OK;
  std::lock_guard<std::mutex> g(g_host_mu);
  auto it = g_host_live.find((uintptr_t)p);
  if (it == g_host_live.end()) return fail(IVC_E_ARG, "ivc_host_free: not a block of ivc_host_alloc");
  const size_t n = it->second;
  g_host_live.erase(it);
  if (n > host_cache_max()) {
    (void)hipHostFree(p);
    return IVC_OK;
  }
  // keep the newest: the oldest cached blocks go back to the system to make room
  while (g_host_cached + n > host_cache_max() && !g_host_cache.empty()) {
    (void)hipHostFree(g_host_cache.front().second);
    g_host_cached -= g_host_cache.front().first;
    g_host_cache.pop_front();
  }
  g_host_cache.emplace_back(n, p);
  g_host_cached += n;
  return IVC_OK;
}

int ivc_set_host_pipeline(int64_t chunk_bytes) {
  if (chunk_bytes < 0) return fail(IVC_E_ARG, "ivc_set_host_pipeline: chunk must be >= 0");
  g_pipe_chunk.store((size_t)chunk_bytes, std::memory_order_relaxed);
  return IVC_OK;
}

int64_t ivc_host_pipeline(void) { return (int64_t)g_pipe_chunk.load(std::memory_order_relaxed); }

int ivc_set_tuning(int key, int value) {
  if (key < 0 || key >= IVC_TUNE_COUNT) return fail(IVC_E_ARG, "ivc_set_tuning: unknown key");
  if (value < 0) return fail(IVC_E_ARG, "ivc_set_tuning: value must be >= 0");
  ivc::g_tuning[key].store(value, std::memory_order_relaxed);
  return IVC_OK;
}

int ivc_tuning(int key) {
  if (key < 0 || key >= IVC_TUNE_COUNT) return fail(IVC_E_ARG, "ivc_tuning: unknown key");
  return ivc::g_tuning[key].load(std::memory_order_relaxed);
}

int ivc_set_store_pace(double total_gbps) {
  if (!(total_gbps >= 0)) return fail(IVC_E_ARG, "ivc_set_store_pace: rate must be >= 0");
  set_store_pace_gbps(total_gbps);
  return IVC_OK;
}

double ivc_store_pace(void) { return store_pace_gbps(); }

double ivc_store_pace_late(void) { return store_pace_late_fraction(); }

int ivc_store_pace_stats(int encoder, double* out, int n) {
  if (encoder < 0 || encoder > 2 || n < 0 || (n > 0 && !out))
    return fail(IVC_E_ARG, "ivc_store_pace_stats: encoder must be 0, 1 or 2, out must hold n values");
  return store_pace_stats(encoder, out, n);
}

int ivc_store_pace_reset_stats(void) {
  store_pace_reset_stats();
  return IVC_OK;
}

int ivc_store_pace_trace(int encoder, double* out, int max_records) {
  if (encoder < 0 || encoder > 2 || max_records < 0 || (max_records > 0 && !out))
    return fail(IVC_E_ARG, "ivc_store_pace_trace: encoder must be 0, 1 or 2, out must hold "
                           "7 * max_records values");
  return store_pace_trace(encoder, out, max_records);
}

int ivc_store_pace_settle(double margin) {
  if (!(margin >= 0 && margin < 0.5))
    return fail(IVC_E_ARG, "ivc_store_pace_settle: margin must be in [0, 0.5)");
  store_pace_settle(margin);
  return IVC_OK;
}

int ivc_set_histogram_occupancy(int wg_per_cu) {
  if (wg_per_cu < 0 || wg_per_cu > 16)
    return fail(IVC_E_ARG, "ivc_set_histogram_occupancy: wg_per_cu must be in [0, 16]");
  set_histogram_wg_per_cu(wg_per_cu);
  return IVC_OK;
}

int ivc_histogram_occupancy(void) { return histogram_wg_per_cu(); }

int ivc_release_scratch(void) {
  int dev = 0;
  TRY(current_device(&dev));
  DevCtx& c = g_ctx[dev];
  std::lock_guard<std::mutex> g(c.mu);
  for (int i = 0; i < kSlots; ++i) {
    if (c.slot[i]) (void)hipFree(c.slot[i]);
    c.slot[i] = nullptr;
    c.cap[i] = 0;
  }
  host_cache_drain();
  return IVC_OK;
}

// ---------------------------------------------------------------- DCT -----------------
int ivc_dct8x8_dev(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
                   int inverse, int norm, void* stream) {
  TRY(check_dct(src_dtype, nblk, dst_dtype, norm));
  CHECK(aligned16(src) && aligned16(dst), IVC_E_ARG, "dct8x8_dev: pointers must be 16-byte aligned");
  return dev_launch(launch_dct8x8(src, src_dtype, nblk, dst, dst_dtype, inverse, norm,
                                  (hipStream_t)stream), "dct8x8");
}

int ivc_dct8x8(const void* src, int src_dtype, int64_t nblk, void* dst, int dst_dtype,
               int inverse, int norm) {
  TRY(check_dct(src_dtype, nblk, dst_dtype, norm));
  if (nblk == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)nblk * 64 * dtype_size(src_dtype);
  const size_t ob = (size_t)nblk * 64 * dtype_size(dst_dtype);
  if (nblk == 1 && (dst_dtype == IVC_F64 || src_dtype == IVC_F32) &&
      !(dst_dtype == IVC_F64 && src_dtype == IVC_F32)) {
    // scipy's normalisation (as launch_dct8x8): inverse transforms use 2 - norm
    const int inorm = inverse ? 2 - norm : norm;
    const double fct = inorm == 0 ? 1.0 : (inorm == 1 ? 0.25 : 0.0625);
    if (st.server(SRV_DCT, src_dtype, dst_dtype, inverse, norm == IVC_NORM_ORTHO, fct, 0, nullptr, src, ib,
                  dst, ob))
      return st.status;
  }
  if (st.tiny(src, ib, dst, ob, "dct8x8", [&](const void* i, void* o, hipStream_t s, const TinyDone* d) {
        return launch_dct8x8(i, src_dtype, nblk, o, dst_dtype, inverse, norm, s, d);
      }))
    return st.status;
  if (st.pipelined(src, 64 * dtype_size(src_dtype), dst, 64 * dtype_size(dst_dtype), nblk, "dct8x8",
                   [&](const void* i, void* o, int64_t n, hipStream_t s) {
                     return launch_dct8x8(i, src_dtype, n, o, dst_dtype, inverse, norm, s);
                   }))
    return st.sync();
  void* d_in = st.in(src, ib);
  void* d_out = st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_dct8x8(d_in, src_dtype, nblk, d_out, dst_dtype, inverse, norm,
                                st.ctx->stream), "dct8x8"));
  TRY(st.out(dst, d_out, ob));
  return st.sync();
}

int ivc_dct8x8_image_dev(const void* img, int src_dtype, int64_t H, int64_t W, int64_t C, void* dst,
                         int dst_dtype, int inverse, int norm, void* stream) {
  TRY(check_dct(src_dtype, 0, dst_dtype, norm));
  TRY(check_frames(1, H, W, "dct8x8_image"));
  CHECK(C >= 1 && C <= 4096, IVC_E_SHAPE, "dct8x8_image: C must be in [1, 4096]");
  return dev_launch(launch_dct8x8_image(img, src_dtype, H / 8, W, C, dst, dst_dtype, inverse, norm,
                                        (hipStream_t)stream), "dct8x8_image");
}

int ivc_dct8x8_image(const void* img, int src_dtype, int64_t H, int64_t W, int64_t C, void* dst,
                     int dst_dtype, int inverse, int norm) {
  TRY(check_dct(src_dtype, 0, dst_dtype, norm));
  TRY(check_frames(1, H, W, "dct8x8_image"));
  CHECK(C >= 1 && C <= 4096, IVC_E_SHAPE, "dct8x8_image: C must be in [1, 4096]");
  const int64_t rows = H / 8;
  if (rows == 0 || W == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t rib = (size_t)(8 * W * C) * dtype_size(src_dtype);          // per block row
  const size_t rob = (size_t)(W / 8 * C) * 64 * dtype_size(dst_dtype);
  auto go = [&](const void* i, void* o, int64_t n, hipStream_t s) {
    return launch_dct8x8_image(i, src_dtype, n, W, C, o, dst_dtype, inverse, norm, s);
  };
  if (st.pipelined(img, rib, dst, rob, rows, "dct8x8_image", go)) return st.sync();
  void* d_in = st.in(img, rib * rows);
  void* d_out = st.alloc(rob * rows);
  if (st.status) return st.status;
  TRY(st.launched(go(d_in, d_out, rows, st.ctx->stream), "dct8x8_image"));
  TRY(st.out(dst, d_out, rob * rows));
  return st.sync();
}

// ---------------------------------------------------------------- quantisation --------
int ivc_quantize_dev(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                     int calc_dtype, int32_t* dst, void* stream) {
  TRY(check_quant(src_dtype, nblk, C, calc_dtype));
  CHECK(aligned16(dst), IVC_E_ARG, "quantize_dev: output must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_quantize(src, src_dtype, nblk, C, t, calc_dtype, dst,
                                    (hipStream_t)stream), "quantize");
}

int ivc_quantize(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                 int calc_dtype, int32_t* dst) {
  TRY(check_quant(src_dtype, nblk, C, calc_dtype));
  QTab t;
  TRY(load_table(table, &t));
  if (nblk == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)nblk * C * 64 * dtype_size(src_dtype), ob = (size_t)nblk * 192 * 4;
  // float32 arithmetic only for float32 or <= 16-bit integer inputs (as launch_quant_common)
  if (nblk == 1 && (calc_dtype == IVC_F64 || dtype_size(src_dtype) <= 2 || src_dtype == IVC_F32) &&
      st.server(SRV_QUANT, src_dtype, calc_dtype, 0, 0, 0.0, C, &t, src, ib, dst, ob))
    return st.status;
  if (st.tiny(src, ib, dst, ob, "quantize", [&](const void* i, void* o, hipStream_t s, const TinyDone* d) {
        return launch_quantize(i, src_dtype, nblk, C, t, calc_dtype, (int32_t*)o, s, d,
                               tiny_table(st.ctx, t));
      }))
    return st.status;
  if (st.pipelined(src, (size_t)C * 64 * dtype_size(src_dtype), dst, 192 * 4, nblk, "quantize",
                   [&](const void* i, void* o, int64_t n, hipStream_t s) {
                     return launch_quantize(i, src_dtype, n, C, t, calc_dtype, (int32_t*)o, s);
                   }))
    return st.sync();
  void* d_in = st.in(src, ib);
  int32_t* d_out = (int32_t*)st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_quantize(d_in, src_dtype, nblk, C, t, calc_dtype, d_out, st.ctx->stream),
                  "quantize"));
  TRY(st.out(dst, d_out, ob));
  return st.sync();
}

int ivc_dequantize_dev(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                       int calc_dtype, int32_t* dst, void* stream) {
  TRY(check_quant(src_dtype, nblk, C, calc_dtype));
  CHECK(aligned16(dst), IVC_E_ARG, "dequantize_dev: output must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_dequantize(src, src_dtype, nblk, C, t, calc_dtype, dst,
                                      (hipStream_t)stream), "dequantize");
}

int ivc_dequantize(const void* src, int src_dtype, int64_t nblk, int C, const double* table,
                   int calc_dtype, int32_t* dst) {
  TRY(check_quant(src_dtype, nblk, C, calc_dtype));
  QTab t;
  TRY(load_table(table, &t));
  if (nblk == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)nblk * C * 64 * dtype_size(src_dtype), ob = (size_t)nblk * 192 * 4;
  // float32 arithmetic only for float32 or <= 16-bit integer inputs (as launch_quant_common)
  if (nblk == 1 && (calc_dtype == IVC_F64 || dtype_size(src_dtype) <= 2 || src_dtype == IVC_F32) &&
      st.server(SRV_DEQUANT, src_dtype, calc_dtype, 0, 0, 0.0, C, &t, src, ib, dst, ob))
    return st.status;
  if (st.tiny(src, ib, dst, ob, "dequantize", [&](const void* i, void* o, hipStream_t s, const TinyDone* d) {
        return launch_dequantize(i, src_dtype, nblk, C, t, calc_dtype, (int32_t*)o, s, d,
                                 tiny_table(st.ctx, t));
      }))
    return st.status;
  if (st.pipelined(src, (size_t)C * 64 * dtype_size(src_dtype), dst, 192 * 4, nblk, "dequantize",
                   [&](const void* i, void* o, int64_t n, hipStream_t s) {
                     return launch_dequantize(i, src_dtype, n, C, t, calc_dtype, (int32_t*)o, s);
                   }))
    return st.sync();
  void* d_in = st.in(src, ib);
  int32_t* d_out = (int32_t*)st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_dequantize(d_in, src_dtype, nblk, C, t, calc_dtype, d_out,
                                    st.ctx->stream), "dequantize"));
  TRY(st.out(dst, d_out, ob));
  return st.sync();
}

// ---------------------------------------------------------------- zig-zag -------------
int ivc_zigzag_dev(const void* src, int64_t nrow, int64_t stride, int esize, int inverse,
                   void* dst, void* stream) {
  CHECK(esize == 1 || esize == 2 || esize == 4 || esize == 8, IVC_E_DTYPE, "zigzag: element size must be 1, 2, 4 or 8");
  CHECK(nrow >= 0 && stride >= 64, IVC_E_SHAPE, "zigzag: rows need at least 64 elements");
  return dev_launch(launch_zigzag(src, nrow, stride, esize, inverse, dst, (hipStream_t)stream),
                    "zigzag");
}

int ivc_zigzag(const void* src, int64_t nrow, int64_t stride, int esize, int inverse,
               void* dst) {
  CHECK(esize == 1 || esize == 2 || esize == 4 || esize == 8, IVC_E_DTYPE, "zigzag: element size must be 1, 2, 4 or 8");
  CHECK(nrow >= 0 && stride >= 64, IVC_E_SHAPE, "zigzag: rows need at least 64 elements");
  if (nrow == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)nrow * stride * esize, ob = (size_t)nrow * 64 * esize;
  if (st.tiny(src, ib, dst, ob, "zigzag", [&](const void* i, void* o, hipStream_t s, const TinyDone* d) {
        return launch_zigzag(i, nrow, stride, esize, inverse, o, s, d);
      }))
    return st.status;
  if (st.pipelined(src, (size_t)stride * esize, dst, 64 * (size_t)esize, nrow, "zigzag",
                   [&](const void* i, void* o, int64_t n, hipStream_t s) {
                     return launch_zigzag(i, n, stride, esize, inverse, o, s);
                   }))
    return st.sync();
  void* d_in = st.in(src, ib);
  void* d_out = st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_zigzag(d_in, nrow, stride, esize, inverse, d_out, st.ctx->stream), "zigzag"));
  TRY(st.out(dst, d_out, ob));
  return st.sync();
}

// ---------------------------------------------------------------- fused intra ---------
int ivc_intra_encode_dev(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                         int C, const double* table, int calc_dtype, int zigzag, int32_t* out,
                         int64_t* hist, int32_t hist_lo, int32_t nbins, void* stream) {
  TRY(check_frames(nframes, H, W, "intra_encode"));
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, "intra_encode: C must be 1 or 3");
  CHECK(aligned16(img) && aligned16(out), IVC_E_ARG, "intra_encode_dev: pointers must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  hipStream_t s = (hipStream_t)stream;
  TRY(dev_launch(launch_intra_encode(img, dtype, nframes, H, W, C, t, calc_dtype, zigzag, out, s),
                 "intra_encode"));
  if (hist) {
    CHECK(nbins > 0, IVC_E_ARG, "intra_encode: nbins must be positive");
    TRY(dev_launch(launch_histogram(out, nframes * (H / 8) * (W / 8) * 192, hist_lo, nbins, hist, s),
                   "histogram"));
  }
  return IVC_OK;
}

int ivc_intra_encode(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W, int C,
                     const double* table, int calc_dtype, int zigzag, int32_t* out) {
  TRY(check_frames(nframes, H, W, "intra_encode"));
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, "intra_encode: C must be 1 or 3");
  CHECK(valid_dtype(dtype), IVC_E_DTYPE, "intra_encode: invalid dtype");
  QTab t;
  TRY(load_table(table, &t));
  if (nframes * H * W == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)(nframes * H * W * C) * dtype_size(dtype);
  const size_t ob = (size_t)(nframes * (H / 8) * (W / 8)) * 192 * 4;
  // pipelined by frames, or by block rows of a single frame
  const bool by_rows = nframes == 1;
  const int64_t units = by_rows ? H / 8 : nframes;
  const size_t uib = ib / (size_t)units, uob = ob / (size_t)units;
  if (st.pipelined(img, uib, out, uob, units, "intra_encode",
                   [&](const void* i, void* o, int64_t n, hipStream_t s) {
                     return by_rows ? launch_intra_encode(i, dtype, 1, 8 * n, W, C, t, calc_dtype, zigzag,
                                                          (int32_t*)o, s)
                                    : launch_intra_encode(i, dtype, n, H, W, C, t, calc_dtype, zigzag,
                                                          (int32_t*)o, s);
                   }))
    return st.sync();
  void* d_in = st.in(img, ib);
  int32_t* d_out = (int32_t*)st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_intra_encode(d_in, dtype, nframes, H, W, C, t, calc_dtype, zigzag, d_out,
                                      st.ctx->stream), "intra_encode"));
  TRY(st.out(out, d_out, ob));
  return st.sync();
}

int ivc_intra_encode_luma_dev(const uint8_t* img, int64_t nframes, int64_t H, int64_t W,
                              const double* table, int zigzag, int32_t* out, void* stream) {
  TRY(check_frames(nframes, H, W, "intra_encode_luma"));
  CHECK(aligned16(img) && aligned16(out), IVC_E_ARG, "intra_encode_luma_dev: pointers must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_intra_encode_luma(img, nframes, H, W, t, zigzag, out, (hipStream_t)stream),
                    "intra_encode_luma");
}

int ivc_intra_decode_dev(const int32_t* q, int64_t nblk, const double* table, int calc_dtype,
                         int unzigzag, double* out, void* stream) {
  CHECK(nblk >= 0, IVC_E_SHAPE, "intra_decode: negative block count");
  CHECK(calc_dtype == IVC_F64, IVC_E_DTYPE, "intra_decode: int32 symbols dequantise in float64");
  CHECK(aligned16(q) && aligned16(out), IVC_E_ARG, "intra_decode_dev: pointers must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_intra_decode(q, nblk, t, unzigzag, out, (hipStream_t)stream),
                    "intra_decode");
}

int ivc_intra_decode(const int32_t* q, int64_t nblk, const double* table, int calc_dtype,
                     int unzigzag, double* out) {
  CHECK(nblk >= 0, IVC_E_SHAPE, "intra_decode: negative block count");
  CHECK(calc_dtype == IVC_F64, IVC_E_DTYPE, "intra_decode: int32 symbols dequantise in float64");
  QTab t;
  TRY(load_table(table, &t));
  if (nblk == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)nblk * 192 * 4, ob = (size_t)nblk * 192 * 8;
  void* d_in = st.in(q, ib);
  double* d_out = (double*)st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_intra_decode((const int32_t*)d_in, nblk, t, unzigzag, d_out,
                                      st.ctx->stream), "intra_decode"));
  TRY(st.out(out, d_out, ob));
  return st.sync();
}

static int check_zr_dec(int64_t nsym, int64_t nblk, int32_t B) {
  CHECK(nsym >= 0 && nsym < (1LL << 32), IVC_E_ARG, "zerorun_decode: need 0 <= nsym < 2^32");
  CHECK(nblk >= 0, IVC_E_ARG, "zerorun_decode: nblk must be >= 0");
  CHECK(B >= 0 && B <= 64, IVC_E_SHAPE, "zerorun_decode: block_size must be in [0, 64]");
  return IVC_OK;
}

static int check_decode_image(int64_t nframes, int64_t H, int64_t W, int C, const char* what) {
  TRY(check_frames(nframes, H, W, what));
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, std::string(what) + ": C must be 1 or 3 (the dequantiser "
                                       "broadcasts the channel axis against 3 table planes)");
  return IVC_OK;
}

int ivc_intra_decode_image_dev(const int32_t* q, int64_t nframes, int64_t H, int64_t W, int C,
                               const double* table, int unzigzag, int to_rgb, double* out,
                               void* stream) {
  TRY(check_decode_image(nframes, H, W, C, "intra_decode_image"));
  CHECK(aligned16(q) && aligned16(out), IVC_E_ARG, "intra_decode_image_dev: pointers must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_intra_decode_image(q, nframes, H, W, C, t, unzigzag, to_rgb, out,
                                              (hipStream_t)stream), "intra_decode_image");
}

int ivc_intra_decode_image(const int32_t* q, int64_t nframes, int64_t H, int64_t W, int C,
                           const double* table, int unzigzag, int to_rgb, double* out) {
  TRY(check_decode_image(nframes, H, W, C, "intra_decode_image"));
  QTab t;
  TRY(load_table(table, &t));
  const int64_t npx = nframes * H * W;
  if (npx == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t ib = (size_t)npx / 64 * C * 64 * 4, ob = (size_t)npx * 3 * 8;
  void* d_in = st.in(q, ib);
  double* d_out = (double*)st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_intra_decode_image((const int32_t*)d_in, nframes, H, W, C, t, unzigzag,
                                            to_rgb, d_out, st.ctx->stream), "intra_decode_image"));
  TRY(st.out(out, d_out, ob));
  return st.sync();
}

// symbols -> zero-run decode (zerorun.py:46-88, errors as results in err[3]) -> the image
// decode above, on the device without host hops
static int symbols2image_enqueue(const int32_t* sym, int64_t nsym, int64_t nframes, int64_t H,
                                 int64_t W, int C, const QTab& t, int32_t eob, int to_rgb,
                                 double* out, int64_t* err, void* coef, void* scratch,
                                 hipStream_t s) {
  return dev_launch(launch_symbols2image(sym, nsym, nframes, H, W, C, t, eob, to_rgb, out,
                                         (int32_t*)coef, scratch, err, s), "symbols2image");
}
static int64_t s2i_scratch_bytes(int64_t nsym, int64_t nframes, int64_t H, int64_t W) {
  return sym_image_scratch_bytes(nsym, nframes * (H / 8) * ((W / 8 + 7) / 8));
}

int ivc_symbols2image_dev(const int32_t* sym, int64_t nsym, int64_t nframes, int64_t H, int64_t W,
                          int C, const double* table, int32_t eob, int to_rgb, double* out,
                          int64_t* err, void* stream) {
  TRY(check_decode_image(nframes, H, W, C, "symbols2image"));
  TRY(check_zr_dec(nsym, nframes * (H / 8) * (W / 8) * C, 64));
  CHECK(err, IVC_E_ARG, "symbols2image: err is NULL");
  CHECK(aligned16(out), IVC_E_ARG, "symbols2image_dev: output must be 16-byte aligned");
  QTab t;
  TRY(load_table(table, &t));
  hipStream_t s = (hipStream_t)stream;
  const int64_t nblk = nframes * (H / 8) * (W / 8) * C;
  void *coef = nullptr, *scratch = nullptr;
  hipError_t e = scratch_alloc(&coef, (size_t)nblk * 256, s);
  if (e == hipSuccess) e = scratch_alloc(&scratch, (size_t)s2i_scratch_bytes(nsym, nframes, H, W), s);
  if (e != hipSuccess) {
    if (coef) (void)hipFreeAsync(coef, s);
    return fail(IVC_E_NOMEM, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  }
  const int rc = symbols2image_enqueue(sym, nsym, nframes, H, W, C, t, eob, to_rgb, out, err, coef,
                                       scratch, s);
  (void)hipFreeAsync(scratch, s);
  (void)hipFreeAsync(coef, s);
  return rc;
}

int ivc_symbols2image(const int32_t* sym, int64_t nsym, int64_t nframes, int64_t H, int64_t W,
                      int C, const double* table, int32_t eob, int to_rgb, double* out,
                      int64_t* err) {
  TRY(check_decode_image(nframes, H, W, C, "symbols2image"));
  const int64_t nblk = nframes * (H / 8) * (W / 8) * C;
  TRY(check_zr_dec(nsym, nblk, 64));
  CHECK(err, IVC_E_ARG, "symbols2image: err is NULL");
  QTab t;
  TRY(load_table(table, &t));
  Staging st;
  TRY(st.open());
  const size_t ob = (size_t)(nframes * H * W) * 3 * 8;
  const int32_t* d_sym = (const int32_t*)st.in(sym, (size_t)nsym * 4);
  void* scratch = st.alloc((size_t)s2i_scratch_bytes(nsym, nframes, H, W));
  void* coef = st.alloc((size_t)nblk * 256);
  double* d_out = (double*)st.alloc(ob);
  int64_t* d_err = (int64_t*)st.alloc(3 * 8);
  if (st.status) return st.status;
  TRY(symbols2image_enqueue(d_sym, nsym, nframes, H, W, C, t, eob, to_rgb, d_out, d_err, coef,
                            scratch, st.ctx->stream));
  TRY(st.out(out, d_out, ob));
  TRY(st.out(err, d_err, 3 * 8));
  return st.sync();
}

// ---------------------------------------------------------------- motion --------------
int ivc_motion_estimate_dev(const void* ref, const void* cur, int dtype, int64_t nframes,
                            int64_t H, int64_t W, int sr, int mode, int64_t* mv, void* stream) {
  TRY(check_frames(nframes, H, W, "motion_estimate"));
  TRY(check_sr(sr));
  CHECK(valid_dtype(dtype), IVC_E_DTYPE, "motion_estimate: invalid dtype");
  return dev_launch(launch_motion_estimate(ref, cur, dtype, nframes, H, W, sr, mode, mv,
                                           (hipStream_t)stream), "motion_estimate");
}

int ivc_motion_estimate(const void* ref, const void* cur, int dtype, int64_t nframes, int64_t H,
                        int64_t W, int sr, int mode, int64_t* mv) {
  TRY(check_frames(nframes, H, W, "motion_estimate"));
  TRY(check_sr(sr));
  CHECK(valid_dtype(dtype), IVC_E_DTYPE, "motion_estimate: invalid dtype");
  const int64_t nblk = nframes * (H / 8) * (W / 8);
  if (nblk == 0) return IVC_OK;
  Staging st;
  TRY(st.open());
  const size_t fb = (size_t)(nframes * H * W) * dtype_size(dtype), ob = (size_t)nblk * 8;
  void* d_ref = st.in(ref, fb);
  void* d_cur = st.in(cur, fb);
  int64_t* d_mv = (int64_t*)st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_motion_estimate(d_ref, d_cur, dtype, nframes, H, W, sr, mode, d_mv,
                                         st.ctx->stream), "motion_estimate"));
  TRY(st.out(mv, d_mv, ob));
  return st.sync();
}

int ivc_motion_compensate_dev(const void* ref, int esize, int64_t nframes, int64_t H, int64_t W,
                              int64_t C, const int64_t* mv, int sr, void* out, void* stream) {
  TRY(check_frames(nframes, H, W, "motion_compensate"));
  TRY(check_sr(sr));
  CHECK(esize == 1 || esize == 2 || esize == 4 || esize == 8, IVC_E_DTYPE, "motion_compensate: element size must be 1, 2, 4 or 8");
  CHECK(C >= 1, IVC_E_SHAPE, "motion_compensate: C must be >= 1");
  return dev_launch(launch_motion_compensate(ref, esize, nframes, H, W, C, mv, sr, out,
                                             (hipStream_t)stream), "motion_compensate");
}

int ivc_motion_compensate(const void* ref, int esize, int64_t nframes, int64_t H, int64_t W,
                          int64_t C, const int64_t* mv, int sr, void* out) {
  TRY(check_frames(nframes, H, W, "motion_compensate"));
  TRY(check_sr(sr));
  CHECK(esize == 1 || esize == 2 || esize == 4 || esize == 8, IVC_E_DTYPE, "motion_compensate: element size must be 1, 2, 4 or 8");
  CHECK(C >= 1, IVC_E_SHAPE, "motion_compensate: C must be >= 1");
  const size_t fb = (size_t)(nframes * H * W * C) * esize;
  if (fb == 0) return IVC_OK;
  const size_t mb = (size_t)(nframes * (H / 8) * (W / 8)) * 8;
  Staging st;
  TRY(st.open());
  void* d_ref = st.in(ref, fb);
  int64_t* d_mv = (int64_t*)st.in(mv, mb);
  void* d_out = st.alloc(fb);
  if (st.status) return st.status;
  TRY(st.launched(launch_motion_compensate(d_ref, esize, nframes, H, W, C, d_mv, sr, d_out,
                                           st.ctx->stream), "motion_compensate"));
  TRY(st.out(out, d_out, fb));
  return st.sync();
}

// ---------------------------------------------------------------- fused inter ---------
// ME then the residual encoder.  Long sequences are pipelined over K chunks of frame pairs: the
// search of chunk j + 1 on the caller's stream beside the residual encode of chunk j on the
// second stream (ME is latency-bound, the residual encoder HBM-bound).
#ifndef IVC_INTER_CHUNKS
#define IVC_INTER_CHUNKS 1
#endif
static int inter_encode_enqueue(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W, int sr,
                                const QTab& t, int zigzag, int64_t* mv, int32_t* out, int64_t* hist,
                                int32_t hist_lo, int32_t hist_n, hipStream_t s) {
  const int64_t HW = H * W, npairs = nframes - 1, hw = (H / 8) * (W / 8);
  int K = IVC_INTER_CHUNKS;
  if (const int f = tuning(IVC_TUNE_INTER_CHUNKS)) K = f;               // ivc_set_tuning
  if (K > PIPE_EVENTS - 2) K = PIPE_EVENTS - 2;
  if (K > npairs) K = (int)npairs;
  auto residual = [&](int64_t p0, int64_t p1, hipStream_t st) {
    return launch_inter_residual(frames + p0 * HW, p1 - p0, H, W, sr, mv + p0 * hw, t, zigzag,
                                 out + p0 * hw * 192, st, hist, hist_lo, hist_n);
  };
  if (K <= 1) {
    TRY(dev_launch(launch_motion_estimate(frames, frames + HW, IVC_U8, npairs, H, W, sr,
                                          IVC_ME_EXACT_U8, mv, s), "motion_estimate"));
    return dev_launch(residual(0, npairs, s), "inter_residual");
  }
  PipeCtx* pp = nullptr;
  TRY(dev_launch(pipe_ctx(&pp), "inter_encode"));
  PipeCtx& P = *pp;
  std::lock_guard<std::mutex> lock(P.mu);
  TRY(dev_launch(hipEventRecord(P.ev[PIPE_EVENTS - 2], s), "inter_encode"));
  TRY(dev_launch(hipStreamWaitEvent(P.aux, P.ev[PIPE_EVENTS - 2], 0), "inter_encode"));
  PipeJoin join{P, s, true};
  const int64_t per = (npairs + K - 1) / K;
  for (int j = 0; j < K; ++j) {
    const int64_t p0 = std::min<int64_t>((int64_t)j * per, npairs), p1 = std::min<int64_t>(p0 + per, npairs);
    if (p1 <= p0) break;
    TRY(dev_launch(launch_motion_estimate(frames + p0 * HW, frames + (p0 + 1) * HW, IVC_U8, p1 - p0,
                                          H, W, sr, IVC_ME_EXACT_U8, mv + p0 * hw, s),
                   "motion_estimate"));
    TRY(dev_launch(hipEventRecord(P.ev[j], s), "inter_encode"));
    TRY(dev_launch(hipStreamWaitEvent(P.aux, P.ev[j], 0), "inter_encode"));
    TRY(dev_launch(residual(p0, p1, P.aux), "inter_residual"));
  }
  join.armed = false;
  TRY(dev_launch(hipEventRecord(P.ev[PIPE_EVENTS - 1], P.aux), "inter_encode"));
  return dev_launch(hipStreamWaitEvent(s, P.ev[PIPE_EVENTS - 1], 0), "inter_encode");
}

int ivc_inter_encode_dev(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W, int sr,
                         const double* table, int calc_dtype, int zigzag, int64_t* mv,
                         int32_t* out, void* stream) {
  TRY(check_frames(nframes, H, W, "inter_encode"));
  TRY(check_sr(sr));
  CHECK(calc_dtype == IVC_F64, IVC_E_DTYPE, "inter_encode: float64 residual DCT needs float64 quantisation");
  CHECK(aligned16(out), IVC_E_ARG, "inter_encode_dev: output must be 16-byte aligned");
  CHECK(((uintptr_t)frames & 7u) == 0, IVC_E_ARG, "inter_encode_dev: frames must be 8-byte aligned");
  if (nframes < 2) return IVC_OK;
  QTab t;
  TRY(load_table(table, &t));
  return inter_encode_enqueue(frames, nframes, H, W, sr, t, zigzag, mv, out, nullptr, 0, 0,
                              (hipStream_t)stream);
}

int ivc_inter_encode_hist_dev(const uint8_t* frames, int64_t nframes, int64_t H, int64_t W, int sr,
                              const double* table, int calc_dtype, int zigzag, int64_t* mv,
                              int32_t* out, int64_t* hist, int32_t hist_lo, int32_t hist_n,
                              void* stream) {
  TRY(check_frames(nframes, H, W, "inter_encode"));
  TRY(check_sr(sr));
  CHECK(calc_dtype == IVC_F64, IVC_E_DTYPE, "inter_encode: float64 residual DCT needs float64 quantisation");
  CHECK(aligned16(out), IVC_E_ARG, "inter_encode_dev: output must be 16-byte aligned");
  CHECK(((uintptr_t)frames & 7u) == 0, IVC_E_ARG, "inter_encode_dev: frames must be 8-byte aligned");
  CHECK(hist && hist_n > 0, IVC_E_ARG, "inter_encode_hist: need a histogram of hist_n > 0 bins");
  if (nframes < 2) return IVC_OK;
  QTab t;
  TRY(load_table(table, &t));
  return inter_encode_enqueue(frames, nframes, H, W, sr, t, zigzag, mv, out, hist, hist_lo, hist_n,
                              (hipStream_t)stream);
}

// ---------------------------------------------------------------- histogram -----------
int ivc_histogram_i32_dev(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins, int64_t* hist,
                          void* stream) {
  CHECK(n >= 0 && nbins > 0, IVC_E_ARG, "histogram: need n >= 0 and nbins > 0");
  return dev_launch(launch_histogram(sym, n, lo, nbins, hist, (hipStream_t)stream), "histogram");
}

int ivc_histogram_i32(const int32_t* sym, int64_t n, int32_t lo, int32_t nbins, int64_t* hist) {
  CHECK(n >= 0 && nbins > 0, IVC_E_ARG, "histogram: need n >= 0 and nbins > 0");
  Staging st;
  TRY(st.open());
  const size_t hb = (size_t)nbins * 8;
  void* d_sym = st.in(sym, (size_t)n * 4);
  int64_t* d_hist = (int64_t*)st.in(hist, hb);  // accumulate onto the caller's counts
  if (st.status) return st.status;
  TRY(st.launched(launch_histogram((const int32_t*)d_sym, n, lo, nbins, d_hist, st.ctx->stream),
                  "histogram"));
  TRY(st.out(hist, d_hist, hb));
  return st.sync();
}

// ---------------------------------------------------------------- Huffman (host) ------
int ivc_huffman_lengths(const double* probs, int32_t n, uint8_t* lengths) {
  CHECK(n >= 0 && probs && lengths, IVC_E_ARG, "huffman: bad arguments");
  for (int32_t i = 0; i < n; ++i)
    CHECK(probs[i] > 0, IVC_E_ARG,
          "Zero-probability symbols found in PMF. All symbols must have non-zero probability.");
  CHECK(huffman_lengths(probs, n, lengths) == 0, IVC_E_ARG, "huffman: code longer than 64 bits");
  return IVC_OK;
}

int ivc_huffman_encode(const int32_t* sym, int64_t n, int32_t lower_bound,
                       const uint8_t* lengths, int32_t nalpha, uint32_t* words,
                       int64_t cap_words, int64_t* nbits) {
  CHECK(n >= 0 && nalpha > 0 && nbits, IVC_E_ARG, "huffman_encode: bad arguments");
  const int rc = huffman_encode(sym, n, lower_bound, lengths, nalpha, words, cap_words, nbits);
  CHECK(rc != -1, IVC_E_ARG, "huffman_encode: invalid code lengths");
  CHECK(rc != -2, IVC_E_ARG, "Message contains symbols outside the trained range.");
  CHECK(rc != -3, IVC_E_SHAPE, "huffman_encode: output buffer too small");
  return IVC_OK;
}

int ivc_huffman_decode(const uint32_t* words, int64_t nwords, int64_t count, int32_t lower_bound,
                       const uint8_t* lengths, int32_t nalpha, int32_t* out) {
  CHECK(nwords >= 0 && count >= 0 && nalpha > 0, IVC_E_ARG, "huffman_decode: bad arguments");
  const int rc = huffman_decode(words, nwords, count, lower_bound, lengths, nalpha, out);
  CHECK(rc != -1, IVC_E_ARG, "huffman_decode: invalid code lengths");
  CHECK(rc == 0, IVC_E_ARG, "huffman_decode: the bitstream ends before message_length symbols");
  return IVC_OK;
}

// ---------------------------------------------------------------- colour --------------
static size_t color_out_size(int dtype) { return dtype == IVC_F32 ? 4 : 8; }

int ivc_rgb2ycbcr_dev(const void* src, int src_dtype, int64_t npix, double* dst, void* stream) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "rgb2ycbcr: unsupported dtype");
  CHECK(npix >= 0, IVC_E_ARG, "rgb2ycbcr: negative size");
  return dev_launch(launch_rgb2ycbcr(src, src_dtype, npix, dst, (hipStream_t)stream), "rgb2ycbcr");
}

int ivc_rgb2ycbcr(const void* src, int src_dtype, int64_t npix, double* dst) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "rgb2ycbcr: unsupported dtype");
  CHECK(npix >= 0, IVC_E_ARG, "rgb2ycbcr: negative size");
  Staging st;
  TRY(st.open());
  const void* d_src = st.in(src, (size_t)npix * 3 * dtype_size(src_dtype));
  double* d_dst = (double*)st.alloc((size_t)npix * 3 * 8);
  if (st.status) return st.status;
  TRY(st.launched(launch_rgb2ycbcr(d_src, src_dtype, npix, d_dst, st.ctx->stream), "rgb2ycbcr"));
  TRY(st.out(dst, d_dst, (size_t)npix * 3 * 8));
  return st.sync();
}

int ivc_ycbcr2rgb_dev(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst,
                      void* stream) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "ycbcr2rgb: unsupported dtype");
  CHECK(npix >= 0 && channels >= 3, IVC_E_SHAPE, "ycbcr2rgb: need >= 3 channels");
  return dev_launch(launch_ycbcr2rgb(src, src_dtype, npix, channels, dst, (hipStream_t)stream),
                    "ycbcr2rgb");
}

int ivc_ycbcr2rgb(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "ycbcr2rgb: unsupported dtype");
  CHECK(npix >= 0 && channels >= 3, IVC_E_SHAPE, "ycbcr2rgb: need >= 3 channels");
  Staging st;
  TRY(st.open());
  const void* d_src = st.in(src, (size_t)(npix * channels) * dtype_size(src_dtype));
  const size_t ob = (size_t)npix * 3 * color_out_size(src_dtype);
  void* d_dst = st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_ycbcr2rgb(d_src, src_dtype, npix, channels, d_dst, st.ctx->stream),
                  "ycbcr2rgb"));
  TRY(st.out(dst, d_dst, ob));
  return st.sync();
}

int ivc_rgb2gray_dev(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst,
                     void* stream) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "rgb2gray: unsupported dtype");
  CHECK(npix >= 0 && channels >= 1 && channels < 8, IVC_E_SHAPE, "rgb2gray: 1..7 channels");
  return dev_launch(launch_rgb2gray(src, src_dtype, npix, (int)channels, dst, (hipStream_t)stream),
                    "rgb2gray");
}

int ivc_rgb2gray(const void* src, int src_dtype, int64_t npix, int64_t channels, void* dst) {
  CHECK(valid_dtype(src_dtype), IVC_E_DTYPE, "rgb2gray: unsupported dtype");
  CHECK(npix >= 0 && channels >= 1 && channels < 8, IVC_E_SHAPE, "rgb2gray: 1..7 channels");
  Staging st;
  TRY(st.open());
  const void* d_src = st.in(src, (size_t)(npix * channels) * dtype_size(src_dtype));
  const size_t ob = (size_t)npix * color_out_size(src_dtype);
  void* d_dst = st.alloc(ob);
  if (st.status) return st.status;
  TRY(st.launched(launch_rgb2gray(d_src, src_dtype, npix, (int)channels, d_dst, st.ctx->stream),
                  "rgb2gray"));
  TRY(st.out(dst, d_dst, ob));
  return st.sync();
}

// ---------------------------------------------------------------- zero-run coding -----
static int check_zr(int64_t nblk, int32_t stride, int32_t B) {
  CHECK(nblk >= 0, IVC_E_ARG, "zerorun: nblk must be >= 0");
  CHECK(B >= 0 && B <= 64, IVC_E_SHAPE, "zerorun: block_size must be in [0, 64]");
  CHECK(stride >= B && stride >= 1, IVC_E_SHAPE, "zerorun: row_stride must be >= block_size");
  return IVC_OK;
}

int ivc_zerorun_encode_dev(const int32_t* src, int64_t nblk, int32_t row_stride,
                           int32_t block_size, int32_t eob, int64_t* offsets, int32_t* out,
                           int64_t capacity, void* stream) {
  TRY(check_zr(nblk, row_stride, block_size));
  CHECK(capacity >= 0, IVC_E_ARG, "zerorun: capacity must be >= 0");
  hipStream_t s = (hipStream_t)stream;
  void* scratch = nullptr;
  if (nblk > 0) {
    hipError_t e = scratch_alloc(&scratch, (size_t)zerorun_scratch_bytes(nblk), s);
    if (e != hipSuccess) return fail(IVC_E_NOMEM, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  }
  const int rc = dev_launch(launch_zerorun_encode(src, nblk, row_stride, block_size, eob, scratch,
                                                  offsets, out, capacity, s),
                            "zerorun_encode");
  if (scratch) (void)hipFreeAsync(scratch, s);
  return rc;
}

int ivc_zerorun_encode(const int32_t* src, int64_t nblk, int32_t row_stride, int32_t block_size,
                       int32_t eob, int32_t* out, int64_t capacity, int64_t* nsym) {
  TRY(check_zr(nblk, row_stride, block_size));
  CHECK(nsym, IVC_E_ARG, "zerorun: nsym is NULL");
  CHECK(capacity >= 0, IVC_E_ARG, "zerorun: capacity must be >= 0");
  Staging st;
  TRY(st.open());
  const int32_t* d_src = (const int32_t*)st.in(src, (size_t)nblk * row_stride * 4);
  void* scratch = st.alloc((size_t)zerorun_scratch_bytes(nblk));
  int64_t* off = (int64_t*)st.alloc((size_t)(nblk + 1) * 8);
  if (st.status) return st.status;
  TRY(st.launched(launch_zerorun_offsets(d_src, nblk, row_stride, block_size, scratch, off,
                                         st.ctx->stream), "zerorun_encode"));
  int64_t total = 0;
  TRY(st.out(&total, off + nblk, 8));
  TRY(st.sync());
  *nsym = total;
  if (total > capacity)
    return fail(IVC_E_SHAPE, "zerorun_encode: the stream holds " + std::to_string(total) +
                                 " symbols, more than capacity " + std::to_string(capacity));
  int32_t* d_out = (int32_t*)st.alloc((size_t)total * 4);
  if (st.status) return st.status;
  TRY(st.launched(launch_zerorun_emit(d_src, nblk, row_stride, block_size, eob, scratch, off, d_out, total,
                                      st.ctx->stream), "zerorun_encode"));
  TRY(st.out(out, d_out, (size_t)total * 4));
  return st.sync();
}


int ivc_zerorun_decode_dev(const int32_t* sym, int64_t nsym, int64_t nblk, int32_t block_size,
                           int32_t eob, int32_t* out, int64_t* err, void* stream) {
  TRY(check_zr_dec(nsym, nblk, block_size));
  hipStream_t s = (hipStream_t)stream;
  void* scratch = nullptr;
  hipError_t e = scratch_alloc(&scratch, (size_t)zr_decode_scratch_bytes(nsym), s);
  if (e != hipSuccess) return fail(IVC_E_NOMEM, std::string("hipMallocAsync: ") + hipGetErrorString(e));
  const int rc = dev_launch(launch_zerorun_decode(sym, nsym, nblk, block_size, eob, out, scratch, err, s),
                            "zerorun_decode");
  (void)hipFreeAsync(scratch, s);
  return rc;
}

int ivc_zerorun_decode(const int32_t* sym, int64_t nsym, int64_t nblk, int32_t block_size,
                       int32_t eob, int32_t* out, int64_t* err) {
  TRY(check_zr_dec(nsym, nblk, block_size));
  CHECK(err, IVC_E_ARG, "zerorun_decode: err is NULL");
  Staging st;
  TRY(st.open());
  const int32_t* d_sym = (const int32_t*)st.in(sym, (size_t)nsym * 4);
  void* scratch = st.alloc((size_t)zr_decode_scratch_bytes(nsym));
  int32_t* d_out = (int32_t*)st.alloc((size_t)nblk * block_size * 4);
  int64_t* d_err = (int64_t*)st.alloc(3 * 8);
  if (st.status) return st.status;
  TRY(st.launched(launch_zerorun_decode(d_sym, nsym, nblk, block_size, eob, d_out, scratch, d_err,
                                        st.ctx->stream), "zerorun_decode"));
  TRY(st.out(out, d_out, (size_t)nblk * block_size * 4));
  TRY(st.out(err, d_err, 3 * 8));
  return st.sync();
}

int ivc_intra_symbols_dev(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                          int C, const double* table, int32_t eob, int32_t* out,
                          int64_t capacity, int64_t* nsym, void* stream) {
  TRY(check_frames(nframes, H, W, "intra_symbols"));
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, "intra_symbols: C must be 1 or 3");
  CHECK(dtype == IVC_U8, IVC_E_DTYPE, "intra_symbols: uint8 frames only");
  CHECK(capacity >= 0 && nsym, IVC_E_ARG, "intra_symbols: need capacity >= 0 and nsym");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_intra_symbols(img, dtype, nframes, H, W, C, t, eob, out, capacity, nsym,
                                         (hipStream_t)stream), "intra_symbols");
}

int ivc_intra_symbols_hist_dev(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W,
                               int C, const double* table, int32_t eob, int32_t* out,
                               int64_t capacity, int64_t* nsym, int64_t* hist, int32_t hist_lo,
                               int32_t hist_n, void* stream) {
  TRY(check_frames(nframes, H, W, "intra_symbols_hist"));
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, "intra_symbols_hist: C must be 1 or 3");
  CHECK(dtype == IVC_U8, IVC_E_DTYPE, "intra_symbols_hist: uint8 frames only");
  CHECK(capacity >= 0 && nsym, IVC_E_ARG, "intra_symbols_hist: need capacity >= 0 and nsym");
  CHECK(hist && hist_n >= 1, IVC_E_ARG, "intra_symbols_hist: need a histogram of >= 1 bin");
  QTab t;
  TRY(load_table(table, &t));
  return dev_launch(launch_intra_symbols(img, dtype, nframes, H, W, C, t, eob, out, capacity, nsym,
                                         (hipStream_t)stream, hist, hist_lo, hist_n),
                    "intra_symbols_hist");
}

int ivc_intra_symbols(const void* img, int dtype, int64_t nframes, int64_t H, int64_t W, int C,
                      const double* table, int32_t eob, int32_t* out, int64_t capacity,
                      int64_t* nsym) {
  TRY(check_frames(nframes, H, W, "intra_symbols"));
  CHECK(C == 1 || C == 3, IVC_E_SHAPE, "intra_symbols: C must be 1 or 3");
  CHECK(dtype == IVC_U8, IVC_E_DTYPE, "intra_symbols: uint8 frames only");
  CHECK(capacity >= 0 && nsym, IVC_E_ARG, "intra_symbols: need capacity >= 0 and nsym");
  QTab t;
  TRY(load_table(table, &t));
  Staging st;
  TRY(st.open());
  const void* d_img = st.in(img, (size_t)(nframes * H * W * C));
  int64_t* d_n = (int64_t*)st.alloc(8);
  if (st.status) return st.status;
  TRY(st.launched(launch_intra_symbols(d_img, dtype, nframes, H, W, C, t, eob, nullptr, 0, d_n,
                                       st.ctx->stream), "intra_symbols"));
  int64_t total = 0;
  TRY(st.out(&total, d_n, 8));
  TRY(st.sync());
  *nsym = total;
  if (total > capacity)
    return fail(IVC_E_SHAPE, "intra_symbols: the stream holds " + std::to_string(total) +
                                 " symbols, more than capacity " + std::to_string(capacity));
  int32_t* d_out = (int32_t*)st.alloc((size_t)total * 4);
  if (st.status) return st.status;
  TRY(st.launched(launch_intra_symbols(d_img, dtype, nframes, H, W, C, t, eob, d_out, total, d_n,
                                       st.ctx->stream), "intra_symbols"));
  TRY(st.out(out, d_out, (size_t)total * 4));
  return st.sync();
}

int ivc_minmax_i32_dev(const int32_t* sym, int64_t n, int32_t* mm, void* stream) {
  CHECK(n >= 0 && mm, IVC_E_ARG, "minmax: need n >= 0 and an output");
  return dev_launch(launch_minmax_i32(sym, n, mm, (hipStream_t)stream), "minmax");
}

int ivc_minmax_i32(const int32_t* sym, int64_t n, int32_t* mm) {
  CHECK(n >= 0 && mm, IVC_E_ARG, "minmax: need n >= 0 and an output");
  Staging st;
  TRY(st.open());
  const int32_t* d_sym = (const int32_t*)st.in(sym, (size_t)n * 4);
  int32_t* d_mm = (int32_t*)st.alloc(8);
  if (st.status) return st.status;
  TRY(st.launched(launch_minmax_i32(d_sym, n, d_mm, st.ctx->stream), "minmax"));
  TRY(st.out(mm, d_mm, 8));
  return st.sync();
}

int ivc_histogram_i64_dev(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins, int64_t* hist,
                          void* stream) {
  CHECK(n >= 0 && nbins > 0, IVC_E_ARG, "histogram: need n >= 0 and nbins > 0");
  return dev_launch(launch_histogram_i64(sym, n, lo, nbins, hist, (hipStream_t)stream),
                    "histogram");
}

int ivc_histogram_i64(const int64_t* sym, int64_t n, int64_t lo, int32_t nbins, int64_t* hist) {
  CHECK(n >= 0 && nbins > 0, IVC_E_ARG, "histogram: need n >= 0 and nbins > 0");
  Staging st;
  TRY(st.open());
  const size_t hb = (size_t)nbins * 8;
  void* d_sym = st.in(sym, (size_t)n * 8);
  int64_t* d_hist = (int64_t*)st.in(hist, hb);
  if (st.status) return st.status;
  TRY(st.launched(launch_histogram_i64((const int64_t*)d_sym, n, lo, nbins, d_hist,
                                       st.ctx->stream), "histogram"));
  TRY(st.out(hist, d_hist, hb));
  return st.sync();
}

int ivc_histogram_f64_edges(const double* x, int64_t n, const double* edges, int32_t nedges,
                            int64_t* counts) {
  CHECK(n >= 0 && nedges >= 2, IVC_E_ARG, "histogram_f64_edges: need n >= 0 and >= 2 edges");
  for (int32_t i = 0; i + 1 < nedges; ++i)
    CHECK(!(edges[i] > edges[i + 1]), IVC_E_ARG, "`bins` must increase monotonically, when an array");
  Staging st;
  TRY(st.open());
  const size_t cb = (size_t)(nedges - 1) * 8;
  void* d_x = st.in(x, (size_t)n * 8);
  void* d_e = st.in(edges, (size_t)nedges * 8);
  int64_t* d_c = (int64_t*)st.in(counts, cb);
  if (st.status) return st.status;
  TRY(st.launched(launch_edge_histogram((const double*)d_x, n, (const double*)d_e, nedges, d_c,
                                        st.ctx->stream), "histogram_f64_edges"));
  TRY(st.out(counts, d_c, cb));
  return st.sync();
}

int ivc_histogram_f64_edges_dev(const double* x, int64_t n, const double* edges, int32_t nedges,
                                int64_t* counts, void* stream) {
  CHECK(n >= 0 && nedges >= 2, IVC_E_ARG, "histogram_f64_edges: need n >= 0 and >= 2 edges");
  return dev_launch(launch_edge_histogram(x, n, edges, nedges, counts, (hipStream_t)stream),
                    "histogram_f64_edges");
}

}  // extern "C"
