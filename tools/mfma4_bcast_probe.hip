// Probe: v_mfma_f64_4x4x4_4b with the A-block broadcast (cbsz = 2, abid = 0..3):
// (1) semantics — C[blk] += A[abid] B[blk] for every block (lane layout of
//     dfm_common.h: A[blk][i][k] at 16k+4blk+i, B[blk][k][j] at 16k+4blk+j,
//     C[blk][i][j] at 16i+4blk+j);
// (2) throughput of the broadcast form (4 MFMAs per A/B register pair) with
//     operands re-read from LDS, vs the k-split 8x8 form of dfm_gemm.hip.
// Result (round 2): the f64 4x4x4_4b form ignores cbsz/abid -- every block
// multiplies its own A (192 of 256 outputs differ from the broadcast
// hypothesis, all match the plain per-block product); the loop runs at
// 62-67 TF/s like the k-split form.  No broadcast GEMM on f64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
template <int ABID>
__device__ double mf(double a, double b, double c) { return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 2, ABID, 0); }
__global__ void sem_k(const double *A, const double *B, double *D) {
  const int l = threadIdx.x;
  double a = A[l], b = B[l];
  D[0 * 64 + l] = mf<0>(a, b, 0.0);
  D[1 * 64 + l] = mf<1>(a, b, 0.0);
  D[2 * 64 + l] = mf<2>(a, b, 0.0);
  D[3 * 64 + l] = mf<3>(a, b, 0.0);
}
// wave tile 64 x 64 over k: per k=4 step A regs 4 (row groups of 16), B regs 4
// (col groups of 16), 64 MFMAs; acc[ra][cb][abid] = 64 doubles per lane
__global__ void __launch_bounds__(256) bc_lds(double *out, int iters, double seed) {
  __shared__ double l[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) l[i] = seed + i * 1e-6;
  __syncthreads();
  double acc[4][4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int z = 0; z < 4; ++z) acc[i][q][z] = 0;
  const int lane = threadIdx.x & 63;
  for (int it = 0; it < iters; ++it) {
    const int o = (it & 3) * 512;
    double af[4], bf[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) { af[f] = l[o + f * 64 + lane]; bf[f] = l[2048 + o + f * 64 + lane]; }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[i][q][0] = mf<0>(af[i], bf[q], acc[i][q][0]);
        acc[i][q][1] = mf<1>(af[i], bf[q], acc[i][q][1]);
        acc[i][q][2] = mf<2>(af[i], bf[q], acc[i][q][2]);
        acc[i][q][3] = mf<3>(af[i], bf[q], acc[i][q][3]);
      }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int z = 0; z < 4; ++z) s += acc[i][q][z];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  std::vector<double> A(64), B(64), D(256);
  for (int l = 0; l < 64; ++l) { A[l] = 1 + l; B[l] = 1000 + 3 * l + (l % 7); }
  double *dA, *dB, *dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
  hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice); hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice);
  sem_k<<<1, 64>>>(dA, dB, dD); hipDeviceSynchronize();
  hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int ab = 0; ab < 4; ++ab)
    for (int blk = 0; blk < 4; ++blk)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          double ref = 0;
          for (int k = 0; k < 4; ++k) ref += A[16 * k + 4 * ab + i] * B[16 * k + 4 * blk + j];
          if (ref != D[ab * 64 + 16 * i + 4 * blk + j]) ++bad;
        }
  printf("broadcast semantics C[blk] = A[abid] B[blk]: %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
  if (bad) {
    for (int l = 0; l < 16; ++l) printf("lane %d: %g (abid0)\n", l, D[l]);
  }
  double *out; hipMalloc(&out, 2048 * 256 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms; int iters = 2000;
  for (int nb : {256, 512, 768, 1024}) {
    bc_lds<<<nb, 256>>>(out, 100, 1.0); hipEventRecord(e0); bc_lds<<<nb, 256>>>(out, iters, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("bcast 64x64 lds nblk=%5d %.2f TF/s\n", nb, (double)nb * 4 * iters * 64 * 512.0 / ms / 1e9);
  }
  return 0;
}
