// Does the layout of the factored solver's per-replicate blocks Z / HZ
// (T rows x pz columns per replicate) limit the per-replicate passes
// (boot_y2 / ap2 / cheb / cheb_mid: one workgroup per replicate, 16-row
// tiles per wave)?  Today Z is ONE row-major T x (nb pz) matrix (the H.Z
// GEMM's B operand): a replicate's row is a 96-byte segment (pz = 12) and
// its consecutive rows are nb pz 8 bytes apart (960 KB at C3).  Tiled, the
// columns are grouped in 64-column blocks stored block after block (T x 64
// each, rows 512 B apart), which the GEMM can read just as well.  The probe
// times a copy-like pass (read Z rows, write HZ rows; the same bytes and the
// same per-wave tile loop as the real passes) over both layouts.
//
// build: hipcc -O3 --offload-arch=gfx950 tools/zlayout_probe.hip -o tools/zlayout_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int T = 500, PZ = 12, NB = 9999, BW = 4;

__device__ __forceinline__ int64_t ix_flat(int s, int rep, int c) { return (int64_t)s * NB * PZ + (int64_t)rep * PZ + c; }
__device__ __forceinline__ int64_t ix_tiled(int s, int rep, int c) {
  const int64_t col = (int64_t)rep * PZ + c;
  return (col >> 6) * ((int64_t)T * 64) + (int64_t)s * 64 + (col & 63);
}

__device__ __forceinline__ int64_t ix_rep(int s, int rep, int c) { return ((int64_t)rep * T + s) * PZ + c; }
__device__ __forceinline__ int64_t ix(int L, int s, int rep, int c) {
  return L == 0 ? ix_flat(s, rep, c) : (L == 1 ? ix_tiled(s, rep, c) : ix_rep(s, rep, c));
}

// layouts 0 flat, 1 tiled, 2 replicate-major [rep][T][pz]; all with the real
// passes' (row lane >> 4 + 4 g, column lane & 15) mapping
template <int L>
__global__ __launch_bounds__(64 * BW, 4) void pass(const double *__restrict__ Z, double *__restrict__ HZ, double a) {
  const int rep = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  for (int tile = wave; tile < (T + 15) / 16; tile += BW) {
    double v[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = tile * 16 + 4 * g + lk;
      v[g] = (s < T && li < PZ) ? Z[ix(L, s, rep, li)] : 0.0;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = tile * 16 + 4 * g + lk;
      if (s < T && li < PZ) HZ[ix(L, s, rep, li)] = a * v[g] + 1.0;
    }
  }
}
// layout 2 read lane-linearly: a tile's 16 x pz doubles are contiguous
template <int L>
__global__ __launch_bounds__(64 * BW, 4) void pass_lin(const double *__restrict__ Z, double *__restrict__ HZ, double a) {
  const int rep = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int tile = wave; tile < (T + 15) / 16; tile += BW) {
    const int64_t base = ((int64_t)rep * T + tile * 16) * PZ;
    const int n = (min(T, tile * 16 + 16) - tile * 16) * PZ;
    double v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = lane + 64 * j < n ? Z[base + lane + 64 * j] : 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (lane + 64 * j < n) HZ[base + lane + 64 * j] = a * v[j] + 1.0;
  }
}

int main() {
  const size_t n = (size_t)T * NB * PZ + 64 * T;   // (tiled: the last block padded)
  double *Z, *HZ;
  if (hipMalloc(&Z, n * 8) || hipMalloc(&HZ, n * 8)) return 2;
  hipMemset(Z, 0, n * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = 2.0 * T * NB * PZ * 8;
  const char *names[4] = {"flat T x nb pz", "tiled 64-col blocks", "replicate-major [rep][T][pz]",
                          "replicate-major, lane-linear"};
  auto launch = [&](int L) {
    if (L == 0) pass<0><<<NB, 64 * BW>>>(Z, HZ, 0.5);
    else if (L == 1) pass<1><<<NB, 64 * BW>>>(Z, HZ, 0.5);
    else if (L == 2) pass<2><<<NB, 64 * BW>>>(Z, HZ, 0.5);
    else pass_lin<2><<<NB, 64 * BW>>>(Z, HZ, 0.5);
  };
  for (int rnd = 0; rnd < 2; ++rnd)
    for (int tiled = 0; tiled < 4; ++tiled) {
      for (int w = 0; w < 2; ++w) launch(tiled);
      hipEventRecord(e0);
      for (int it = 0; it < 10; ++it) launch(tiled);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      printf("round %d %s: %.3f ms per pass, %.2f TB/s (%.0f MB moved)\n", rnd, names[tiled],
             ms / 10, bytes / (ms / 10 * 1e-3) / 1e12, bytes / 1e6);
    }
  return 0;
}
