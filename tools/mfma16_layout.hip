// Check the operand/result maps of v_mfma_f64_16x16x4_f64 assumed by the fused
// bootstrap kernels: A[i][k] at lane i + 16k, B[k][j] at lane j + 16k,
// C[row][col] at lane col + 16*(row % 4), reg row / 4  (i.e. row = (l>>4) + 4 reg).
// Exact small integers, asymmetric A and B; prints "ok" or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double *A, const double *B, double *C) {
  const int l = threadIdx.x;
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int g = 0; g < 4; ++g) C[((l >> 4) + 4 * g) * 16 + (l & 15)] = acc[g];
}
int main() {
  double hA[64], hB[64], hC[256];
  for (int i = 0; i < 16; ++i) for (int kk = 0; kk < 4; ++kk) hA[i * 4 + kk] = (i * 7 + kk * 3) % 11 - 5;
  for (int kk = 0; kk < 4; ++kk) for (int j = 0; j < 16; ++j) hB[kk * 16 + j] = (kk * 5 + j * 2) % 13 - 6;
  double *A, *B, *C;
  hipMalloc(&A, 512); hipMalloc(&B, 512); hipMalloc(&C, 2048);
  hipMemcpy(A, hA, 512, hipMemcpyHostToDevice); hipMemcpy(B, hB, 512, hipMemcpyHostToDevice);
  k<<<1, 64>>>(A, B, C);
  hipMemcpy(hC, C, 2048, hipMemcpyDeviceToHost);
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int kk = 0; kk < 4; ++kk) s += hA[i * 4 + kk] * hB[kk * 16 + j];
    if (s != hC[i * 16 + j]) { printf("mismatch at %d %d: %g vs %g\n", i, j, hC[i * 16 + j], s); return 1; }
  }
  printf("ok\n");
  return 0;
}
