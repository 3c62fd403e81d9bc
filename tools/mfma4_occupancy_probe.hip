// Probe: v_mfma_f64_4x4x4_4b throughput vs waves per SIMD and accumulator count,
// and the GEMM inner-loop form (8x8 fragment outer product, operands from LDS)
// with and without fragment double-buffering.
// Measured on MI355X (round 2), TF/s at 1..4 workgroups of 4 waves per CU:
//   independent accumulators, operands in registers: 16 acc 68-76, 64 acc 72-77;
//   8x8 outer product, operands in registers: 74-76 (0.95 of 78.6);
//   8x8 from LDS, one register set: 65-66 (0.84) at every occupancy;
//   8x8 from LDS, two alternating register sets: 72-73 (0.92);
//   8x8 from LDS, next set loaded then moved into place: 63-64.
// v_mfma_f64_16x16x4 tops out at 49.7 TF/s with any accumulator count
// (tools/mfma_f64_probe.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
template<int NACC>
__global__ void __launch_bounds__(256) mfma4_n(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  double c[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) c[j] = 0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) c[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[j], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < NACC; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// DB = 0: load 16 fragments, then 64 MFMAs; DB = 1: next iteration's fragments
// loaded before this iteration's MFMAs (two register sets)
template <int DB>
__global__ void __launch_bounds__(256) mfma4_lds(double* out, int iters, double seed) {
  __shared__ double l[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) l[i] = seed + i * 1e-6;
  __syncthreads();
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0;
  const int lane = threadIdx.x & 63;
  const double *la = l + lane, *lb = l + 2048 + lane;
  double af[8], bf[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) { af[f] = la[f * 64]; bf[f] = lb[f * 64]; }
  for (int it = 0; it < iters; ++it) {
    const int o = (it & 3) * 512;
    double an[8], bn[8];
    if (DB) {
#pragma unroll
      for (int f = 0; f < 8; ++f) { an[f] = la[o + f * 64]; bn[f] = lb[o + f * 64]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = __builtin_amdgcn_mfma_f64_4x4x4f64(af[i], bf[q], acc[i][q], 0, 0, 0);
    if (DB) {
#pragma unroll
      for (int f = 0; f < 8; ++f) { af[f] = an[f]; bf[f] = bn[f]; }
    } else {
#pragma unroll
      for (int f = 0; f < 8; ++f) { af[f] = la[o + f * 64]; bf[f] = lb[o + f * 64]; }
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) s += acc[i][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// operands varying over the 8x8 outer product but register-resident (no LDS in the loop)
// V = 1: A operands for the 4 blocks broadcast-shuffled each iteration (cheap VALU)
template <int V>
__global__ void __launch_bounds__(256) mfma4_reg(double* out, int iters, double seed) {
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0;
  const int lane = threadIdx.x & 63;
  double af[8], bf[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) { af[f] = seed + lane * 1e-3 + f; bf[f] = seed - lane * 1e-3 - f; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = __builtin_amdgcn_mfma_f64_4x4x4f64(af[i], bf[q], acc[i][q], 0, 0, 0);
    if (V) {
#pragma unroll
      for (int f = 0; f < 8; ++f) af[f] = af[f] * 0.5 + 1.0;
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) s += acc[i][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// fragment double-buffering without register moves: the loop body is two
// iterations with alternating register sets; set Y's loads are issued before
// set X's 64 MFMAs
__global__ void __launch_bounds__(256) mfma4_lds2(double* out, int iters, double seed) {
  __shared__ double l[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) l[i] = seed + i * 1e-6;
  __syncthreads();
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0;
  const int lane = threadIdx.x & 63;
  const double *la = l + lane, *lb = l + 2048 + lane;
  double ax[8], bx[8], ay[8], by[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) { ax[f] = la[f * 64]; bx[f] = lb[f * 64]; }
  for (int it = 0; it < iters; it += 2) {
    const int o = (it & 3) * 512;
#pragma unroll
    for (int f = 0; f < 8; ++f) { ay[f] = la[o + 512 + f * 64]; by[f] = lb[o + 512 + f * 64]; }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = __builtin_amdgcn_mfma_f64_4x4x4f64(ax[i], bx[q], acc[i][q], 0, 0, 0);
#pragma unroll
    for (int f = 0; f < 8; ++f) { ax[f] = la[((o + 1024) & 2047) + f * 64]; bx[f] = lb[((o + 1024) & 2047) + f * 64]; }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = __builtin_amdgcn_mfma_f64_4x4x4f64(ay[i], by[q], acc[i][q], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) s += acc[i][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  double* out; hipMalloc(&out, 2048 * 256 * 8 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms; int iters = 20000;
#define RUN(KER, NB, FL, NAME) KER<<<NB,256>>>(out, 100, 1.0); hipEventRecord(e0); KER<<<NB,256>>>(out, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms,e0,e1); printf("%-24s nblk=%5d %.2f TF/s\n", NAME, NB, (double)NB*4*iters*(FL)/ms/1e9);
  for (int nb : {256, 512, 768, 1024}) {
    RUN(mfma4_n<16>, nb, 16*512.0, "mfma4 16acc")
    RUN(mfma4_n<64>, nb, 64*512.0, "mfma4 64acc")
  }
  iters = 2000;
  for (int nb : {256, 512, 768, 1024}) { RUN(mfma4_lds<0>, nb, 64*512.0, "lds 8x8 single") RUN(mfma4_lds<1>, nb, 64*512.0, "lds 8x8 double-buf") RUN(mfma4_lds2, nb, 64*512.0, "lds 8x8 2-set") RUN(mfma4_reg<0>, nb, 64*512.0, "reg 8x8") RUN(mfma4_reg<1>, nb, 64*512.0, "reg 8x8 + valu") }
  return 0;
}
