// Lane maps of v_mfma_i32_16x16x64_i8 on gfx950, checked with exact integer data: the
// tiled ME search (ivc_me_mfma.hip) assumes lane l holds A[l & 15][16 (l >> 4) + t] and
// B[16 (l >> 4) + t][l & 15] in byte t = 0..15 of its 4-VGPR operand, and C[4 (l >> 4) + i][l & 15]
// in accumulator register i.  Prints OK or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const signed char* A, const signed char* B, int* C) {
  const int l = threadIdx.x;
  v4i a, b;
  signed char* pa = reinterpret_cast<signed char*>(&a);
  signed char* pb = reinterpret_cast<signed char*>(&b);
  for (int t = 0; t < 16; ++t) {
    pa[t] = A[(l & 15) * 64 + 16 * (l >> 4) + t];          // A[m][k], row-major 16 x 64
    pb[t] = B[(16 * (l >> 4) + t) * 16 + (l & 15)];        // B[k][n], row-major 64 x 16
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
  signed char hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (signed char)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (signed char)(rand() % 256 - 128);
  signed char *dA, *dB;
  int* dC;
  int hC[256];
  if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dC, sizeof hC)) return 2;
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(dA, dB, dC);
  if (hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      int want = 0;
      for (int k = 0; k < 64; ++k) want += hA[m * 64 + k] * hB[k * 16 + n];
      if (hC[m * 16 + n] != want) {
        printf("MISMATCH at C[%d][%d]: got %d want %d\n", m, n, hC[m * 16 + n], want);
        return 1;
      }
    }
  printf("OK: v_mfma_i32_16x16x64_i8 lane maps as assumed\n");
  return 0;
}
