// Probe: f64 MFMA operand/result layout and throughput on gfx950 (v_mfma_f64_16x16x4_f64),
// plus the v_fma_f64 vector rate, so the Gram kernel's roofline peak is measured, not assumed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)

__global__ void layout_k(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  // hypothesis: lane l holds A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];  // raw dump, decode on host
}

__global__ void __launch_bounds__(256) mfma_rate_k(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  d4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ void __launch_bounds__(256) fma_rate_k(double* out, int iters, double seed) {
  double x[8];
  for (int j = 0; j < 8; ++j) x[j] = seed + j + threadIdx.x;
  double m = 1.0000001, ad = 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = fma(x[j], m, ad);
  }
  double s = 0; for (int j = 0; j < 8; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


template<int NACC>
__global__ void __launch_bounds__(256) mfma_rate_n(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  d4 c[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) c[j] = (d4){0,0,0,0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < NACC; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) mfma4_rate(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3;
}

int main() {
  std::vector<double> A(64), B(64), D(256);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = (i + 1) * 10 + k;
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = (k + 1) * 100 + j * 3 + (k == 2 ? 7 : 0);
  double *dA, *dB, *dD; CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dD, 2048));
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  layout_k<<<1, 64>>>(dA, dB, dD); CK(hipDeviceSynchronize());
  CK(hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) + 4 * r, col = l & 15;
    double ref = 0; for (int k = 0; k < 4; ++k) ref += A[row * 4 + k] * B[k * 16 + col];
    if (ref != D[l * 4 + r]) ++bad;
  }
  printf("layout hypothesis (row=(l>>4)+4r, col=l&15): %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
  int nblk = 256 * 8, iters = 20000;
  double* out; CK(hipMalloc(&out, nblk * 256 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    mfma_rate_k<<<nblk, 256>>>(out, 100, 1.0);
    CK(hipEventRecord(e0)); mfma_rate_k<<<nblk, 256>>>(out, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * 4 /*waves*/ * iters * 4 * 2048.0;
    printf("f64 MFMA 16x16x4: %.2f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
    fma_rate_k<<<nblk, 256>>>(out, 100, 1.0);
    CK(hipEventRecord(e0)); fma_rate_k<<<nblk, 256>>>(out, iters, 1.0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    flops = (double)nblk * 256 * iters * 8 * 2.0;
    printf("v_fma_f64: %.2f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
  }

  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    #define RUNV(KER, NB, FLOPS_PER_WAVE_ITER, NAME) \
      KER<<<NB, 256>>>(out, 100, 1.0); CK(hipEventRecord(e0)); KER<<<NB, 256>>>(out, iters, 1.0); CK(hipEventRecord(e1)); \
      CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1)); \
      printf("%-28s nblk=%5d: %.2f TFLOP/s\n", NAME, NB, (double)NB*4*iters*(FLOPS_PER_WAVE_ITER)/ms/1e9);
    RUNV(mfma_rate_n<8>, 256, 8*2048.0, "mfma16 8acc 1WG/CU")
    RUNV(mfma_rate_n<8>, 512, 8*2048.0, "mfma16 8acc 2WG/CU")
    RUNV(mfma_rate_n<8>, 2048, 8*2048.0, "mfma16 8acc 8WG/CU")
    RUNV(mfma_rate_n<2>, 2048, 2*2048.0, "mfma16 2acc 8WG/CU")
    RUNV(mfma_rate_n<1>, 2048, 1*2048.0, "mfma16 1acc 8WG/CU")
    RUNV(mfma4_rate, 2048, 4*512.0, "mfma4x4x4(16blk) 4acc")
  }
  return 0;
}