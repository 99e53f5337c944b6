// Probe: launches a kernel whose by-value argument struct grows (pointers + a 16-byte aligned
// byte array), printing each size before it is launched.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int N>
struct Arg {
  uint32_t* flag;
  uint32_t* count;
  uint32_t seq;
  alignas(16) unsigned char in[N];
};
template <int N>
__global__ void k(const uint8_t* src, double* out, Arg<N> a) {
  const int t = threadIdx.x;
  out[t] = (double)a.in[t % N] + (src ? 1.0 : 0.0);
}
template <int N>
static void run(double* out) {
  printf("arg %d B ... ", (int)sizeof(Arg<N>));
  Arg<N> a{};
  for (int i = 0; i < N; ++i) a.in[i] = (unsigned char)i;
  k<N><<<1, 64>>>(nullptr, out, a);
  hipError_t e = hipDeviceSynchronize();
  double h[64];
  (void)hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  printf("%s, out[5] = %g\n", hipGetErrorString(e), h[5]);
}
int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  double* out;
  (void)hipMalloc(&out, 4096);
  run<64>(out);
  run<512>(out);
  run<1008>(out);
  run<1024>(out);
  run<1536>(out);
  run<2048>(out);
  run<3072>(out);
  return 0;
}
