// Latency breakdown of a tiny host-buffer call (one 8x8 block, the reference's per-block loops,
// exercises/ch3/E3-1_claude.py:47-60): what a launch, the completion wait and the mapped-memory
// access each cost, against the whole C-ABI call (ivc_dct8x8 on a u8 block).
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/tiny_call.hip -Iinclude -Livclab_amd/_lib -livc \
//         -Wl,-rpath,$PWD/ivclab_amd/_lib -o /tmp/tiny_call && /tmp/tiny_call
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>
#include "ivc.h"

__global__ void empty_k() {}
__global__ void flag_k(unsigned* flag, unsigned seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// 64 lanes read 8 bytes each of a mapped input and write 8 doubles each to a mapped output
__global__ void io_k(const uint8_t* in, double* out, unsigned* flag, unsigned seq) {
  const int t = threadIdx.x;
  double v = (double)in[t];
  out[t] = v * 0.5;
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the same with the input block passed by value in the kernel arguments (no device read of
// host memory): 64 B of u8, and 512 B of float64
struct Blk8 { uint8_t v[64]; };
struct Blk64 { double v[64]; };
__global__ void io_arg_k(Blk8 in, double* out, unsigned* flag, unsigned seq) {
  const int t = threadIdx.x;
  out[t] = (double)in.v[t] * 0.5;
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void io_arg64_k(Blk64 in, double* out, unsigned* flag, unsigned seq) {
  const int t = threadIdx.x;
  out[t] = in.v[t] * 0.5;
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void io64_k(const double* in, double* out, unsigned* flag, unsigned seq) {
  const int t = threadIdx.x;
  out[t] = in[t] * 0.5;
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the same, completion without the system fence: each lane's payload store is a system-scope
// (sc0 sc1) store, the wave waits for its stores (vmcnt 0), then lane 0 stores the flag
__global__ void io_arg_nofence_k(Blk64 in, double* out, unsigned* flag, unsigned seq) {
  const int t = threadIdx.x;
  __hip_atomic_store(out + t, in.v[t] * 0.5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 4 waves, with the system fence (the library's op kernels are 256 threads)
__global__ void io_arg_256_k(Blk64 in, double* out, unsigned* flag, unsigned seq) {
  const int t = threadIdx.x;
  if (t < 64) out[t] = in.v[t] * 0.5;
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <typename F>
static void run(const char* name, F&& f, int n = 3000) {
  std::vector<double> t(n);
  for (int i = 0; i < 200; ++i) f(i);
  for (int i = 0; i < n; ++i) {
    const double a = now_us();
    f(i);
    t[i] = now_us() - a;
  }
  std::sort(t.begin(), t.end());
  double s = 0;
  for (double x : t) s += x;
  printf("%-58s median %7.2f us  p10 %7.2f  p90 %7.2f  mean %7.2f\n", name, t[n / 2], t[n / 10],
         t[9 * n / 10], s / n);
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);   // a crash keeps the lines before it
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  unsigned* flag;
  (void)hipHostMalloc((void**)&flag, 4096, hipHostMallocDefault);
  uint8_t* min;
  double* mout;
  (void)hipHostMalloc((void**)&min, 4096, hipHostMallocDefault);
  (void)hipHostMalloc((void**)&mout, 4096, hipHostMallocDefault);
  *flag = 0;
  run("hipStreamSynchronize, idle stream", [&](int) { (void)hipStreamSynchronize(s); });
  run("launch empty kernel (host API only)", [&](int) { empty_k<<<1, 64, 0, s>>>(); });
  (void)hipStreamSynchronize(s);
  run("launch empty kernel + hipStreamSynchronize", [&](int) {
    empty_k<<<1, 64, 0, s>>>();
    (void)hipStreamSynchronize(s);
  });
  run("launch empty kernel + event record + hipEventSynchronize", [&](int) {
    empty_k<<<1, 64, 0, s>>>();
    (void)hipEventRecord(ev, s);
    (void)hipEventSynchronize(ev);
  });
  run("launch empty kernel + hipStreamQuery spin", [&](int) {
    empty_k<<<1, 64, 0, s>>>();
    while (hipStreamQuery(s) == hipErrorNotReady) {}
  });
  unsigned seq = 1;
  run("launch flag kernel + host spin on mapped flag", [&](int) {
    const unsigned q = ++seq;
    flag_k<<<1, 64, 0, s>>>(flag, q);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
  });
  (void)hipStreamSynchronize(s);
  run("launch io kernel (64 B in, 512 B out, mapped) + spin", [&](int) {
    const unsigned q = ++seq;
    io_k<<<1, 64, 0, s>>>(min, mout, flag, q);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
  });
  (void)hipStreamSynchronize(s);
  {
    Blk8 b8;
    memcpy(b8.v, min, 64);
    run("launch io kernel, input in kernel args (64 B) + spin", [&](int) {
      const unsigned q = ++seq;
      b8.v[0] = (uint8_t)q;
      io_arg_k<<<1, 64, 0, s>>>(b8, mout, flag, q);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
    });
    (void)hipStreamSynchronize(s);
    Blk64 b64;
    for (int i = 0; i < 64; ++i) b64.v[i] = i;
    run("launch io kernel, f64 input mapped (512 B) + spin", [&](int) {
      const unsigned q = ++seq;
      io64_k<<<1, 64, 0, s>>>((const double*)(min + 1024), mout, flag, q);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
    });
    (void)hipStreamSynchronize(s);
    run("launch io kernel, f64 input in kernel args (512 B) + spin", [&](int) {
      const unsigned q = ++seq;
      b64.v[0] = q;
      io_arg64_k<<<1, 64, 0, s>>>(b64, mout, flag, q);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
    });
    (void)hipStreamSynchronize(s);
    run("  same, 256 threads", [&](int) {
      const unsigned q = ++seq;
      b64.v[0] = q;
      io_arg_256_k<<<1, 256, 0, s>>>(b64, mout, flag, q);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
    });
    (void)hipStreamSynchronize(s);
    run("  same, 64 threads, no fence (sc1 stores + vmcnt(0))", [&](int) {
      const unsigned q = ++seq;
      b64.v[0] = q;
      io_arg_nofence_k<<<1, 64, 0, s>>>(b64, mout, flag, q);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
    });
    (void)hipStreamSynchronize(s);
    for (int i = 0; i < 64; ++i)
      if (mout[i] != (i ? i * 0.5 : b64.v[0] * 0.5)) { printf("nofence: out[%d] = %g\n", i, mout[i]); break; }
  }
  run("launch io kernel + hipStreamWriteValue32 + spin", [&](int) {
    const unsigned q = ++seq;
    io_k<<<1, 64, 0, s>>>(min, mout, flag + 16, q);
    (void)hipStreamWriteValue32(s, flag, q, 0);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
  });
  (void)hipStreamSynchronize(s);
  run("launch empty kernel + hipStreamWriteValue32 + spin", [&](int) {
    const unsigned q = ++seq;
    empty_k<<<1, 64, 0, s>>>();
    (void)hipStreamWriteValue32(s, flag, q, 0);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) __builtin_ia32_pause();
  });
  (void)hipStreamSynchronize(s);
  run("launch io kernel + hipStreamSynchronize", [&](int) {
    const unsigned q = ++seq;
    io_k<<<1, 64, 0, s>>>(min, mout, flag, q);
    (void)hipStreamSynchronize(s);
  });
  uint8_t blk[64];
  double out[64];
  for (int i = 0; i < 64; ++i) blk[i] = (uint8_t)(i * 7);
  run("ivc_dct8x8 u8 (8,8) -> f64 host call (the C-ABI tiny path)", [&](int) {
    if (ivc_dct8x8(blk, IVC_U8, 1, out, IVC_F64, 0, IVC_NORM_ORTHO) != 0) printf("err %s\n", ivc_last_error());
  });
  double q3[192], tb[192];
  int32_t qo[192];
  for (int i = 0; i < 192; ++i) { q3[i] = i * 3.7 - 300; tb[i] = 16 + i % 40; }
  run("ivc_quantize f64 (3,8,8) host call", [&](int) {
    if (ivc_quantize(q3, IVC_F64, 1, 3, tb, IVC_F64, qo) != 0) printf("err %s\n", ivc_last_error());
  });
  double bd[64];
  for (int i = 0; i < 64; ++i) bd[i] = i * 1.37 - 40;
  for (int srv = 0; srv < 2; ++srv) {
    ivc_set_tuning(IVC_TUNE_TINY_SERVER, srv);
    printf("-- tiny-call server %s\n", srv ? "off (one launch per call)" : "on");
    run("  ivc_dct8x8 u8 (8,8) -> f64", [&](int) {
      if (ivc_dct8x8(blk, IVC_U8, 1, out, IVC_F64, 0, IVC_NORM_ORTHO) != 0) printf("err %s\n", ivc_last_error());
    });
    run("  ivc_dct8x8 f64 (8,8) -> f64", [&](int) {
      if (ivc_dct8x8(bd, IVC_F64, 1, out, IVC_F64, 0, IVC_NORM_ORTHO) != 0) printf("err %s\n", ivc_last_error());
    });
    run("  ivc_quantize f64 (3,8,8)", [&](int) {
      if (ivc_quantize(q3, IVC_F64, 1, 3, tb, IVC_F64, qo) != 0) printf("err %s\n", ivc_last_error());
    });
    run("  ivc_quantize f64 (1,8,8)", [&](int) {
      if (ivc_quantize(q3, IVC_F64, 1, 1, tb, IVC_F64, qo) != 0) printf("err %s\n", ivc_last_error());
    });
  }
  ivc_set_tuning(IVC_TUNE_TINY_SERVER, 0);
  return 0;
}
