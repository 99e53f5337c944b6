// Microbenchmark: wave64 issue cost of v_dot4_u32_u8, v_alignbyte_b32, v_add_u32 and
// v_add_f64 / v_mul_f64 on gfx950 (8 independent chains per lane, all CUs busy).
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, int iters, unsigned seed) {
  unsigned a[CHAINS];
  double d[CHAINS];
  for (int c = 0; c < CHAINS; ++c) { a[c] = seed * (threadIdx.x + c + 1); d[c] = (double)a[c]; }
  const unsigned b = seed ^ threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (OP == 0) a[c] = __builtin_amdgcn_udot4(a[c], b, a[c], false);
      if (OP == 1) a[c] = __builtin_amdgcn_alignbyte(a[c], b, a[c]);
      if (OP == 2) a[c] = a[c] + b;
      if (OP == 3) d[c] = d[c] + 1.0000001;
      if (OP == 4) d[c] = d[c] * 1.0000001;
    }
  }
  unsigned r = 0;
  for (int c = 0; c < CHAINS; ++c) r += a[c] + (unsigned)d[c];
  if (r == 0x12345678u) out[0] = r;
}
int main() {
  unsigned* o; (void)hipMalloc(&o, 4);
  const char* names[] = {"v_dot4_u32_u8", "v_alignbyte_b32", "v_add_u32", "v_add_f64", "v_mul_f64"};
  int dev; (void)hipGetDevice(&dev); hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, dev);
  const int grid = p.multiProcessorCount * 8, iters = 4096;
  for (int op = 0; op < 5; ++op) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0, 0);
      switch (op) {
        case 0: k<0><<<grid, 256>>>(o, iters, 7); break;
        case 1: k<1><<<grid, 256>>>(o, iters, 7); break;
        case 2: k<2><<<grid, 256>>>(o, iters, 7); break;
        case 3: k<3><<<grid, 256>>>(o, iters, 7); break;
        case 4: k<4><<<grid, 256>>>(o, iters, 7); break;
      }
      (void)hipEventRecord(e1, 0); (void)hipEventSynchronize(e1);
    }
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double waves = (double)grid * 4, instr = waves * iters * CHAINS;
    // wave-instructions per second per SIMD -> cycles per wave-instruction at the given clock
    const double per_simd = instr / (p.multiProcessorCount * 4.0) / (ms * 1e-3);
    printf("%-18s %8.3f ms  %.3e wave-instr/s/SIMD  (%.2f cycles at 2.1 GHz)\n", names[op], ms,
           per_simd, 2.1e9 / per_simd);
  }
  return 0;
}
