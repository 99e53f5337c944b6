// Does an s_barrier order one wave's in-flight LDS writes before another wave's LDS reads
// issued after it, with no s_waitcnt lgkmcnt(0) in between?  (The compiler omits that wait at
// some loop-header barriers, e.g. me_mfma16x2_kernel's first barrier: DESIGN.md §5c.)
// Each iteration every wave queues a burst of LDS writes, then writes the iteration number to
// its tag slot, then crosses a bare s_barrier (or one preceded by the wait) and reads the
// other waves' tags; a tag older than the iteration is a stale read, counted with a vector
// atomic.  Usage: lds_barrier_order [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <bool WAIT>
__global__ __launch_bounds__(256) void probe(int iters, unsigned long long* stale) {
  __shared__ int tag[4 * 64];
  __shared__ int junk[4][2048];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 256; i += 256) tag[i] = -1;
  __syncthreads();
  unsigned long long bad = 0;
  for (int it = 0; it < iters; ++it) {
    // a queue of writes ahead of the tag (the search's LDS traffic before red[] is written)
#pragma unroll
    for (int k = 0; k < 16; ++k) junk[wave][(k * 64 + lane * 5 + it) & 2047] = it + k;
    tag[wave * 64 + lane] = it;
    if (WAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // read another wave's tag (the merge reading red[])
    const int other = (wave + 1 + (it & 1) * 2) & 3;
    const int v = __hip_atomic_load(&tag[other * 64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    bad += v < it;
    // keep the next iteration's writes behind every wave's read of this one
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (bad) atomicAdd(stale, bad);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  unsigned long long* d;
  (void)hipMalloc(&d, 16);
  for (int wait = 0; wait < 2; ++wait) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipMemset(d, 0, 8);
      if (wait) probe<true><<<256 * 8, 256>>>(iters, d);
      else probe<false><<<256 * 8, 256>>>(iters, d);
      if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
      unsigned long long h = 0;
      (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
      printf("%-22s rep %d: %llu stale reads of %llu\n", wait ? "wait before barrier" : "bare barrier", rep, h,
             (unsigned long long)iters * 256 * 8 * 256);
      fflush(stdout);
    }
  }
  return 0;
}
