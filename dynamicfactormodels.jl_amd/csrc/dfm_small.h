// dfm_small.h — workgroup-level small dense linear algebra in LDS (n <= 64).
// Every thread of the block must call these (they contain __syncthreads()).
#pragma once
#include "dfm_common.h"

namespace dfm {

// Inverse of an SPD matrix A (n x n, LDS, row stride S) via Cholesky:
// A = L L', Ai = L^-T L^-1.  Lw, Tw: LDS scratch n x S.  *bad |= 1 on a
// non-positive pivot (the reference's inv() would return Inf/garbage).
DFM_DEV void block_spd_inverse(const double *A, double *Ai, double *Lw, double *Tw, int n, int S,
                               int *bad) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < n * S; e += nt) Lw[e] = 0.0;
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (tid == 0) {
      double s = A[j * S + j];
      for (int p = 0; p < j; ++p) s -= Lw[j * S + p] * Lw[j * S + p];
      if (!(s > 0.0)) { *bad = 1; s = 1.0; }
      Lw[j * S + j] = sqrt(s);
    }
    __syncthreads();
    for (int i = j + 1 + tid; i < n; i += nt) {
      double s = A[i * S + j];
      for (int p = 0; p < j; ++p) s -= Lw[i * S + p] * Lw[j * S + p];
      Lw[i * S + j] = s / Lw[j * S + j];
    }
    __syncthreads();
  }
  for (int c = tid; c < n; c += nt)
    for (int i = 0; i < n; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int p = c; p < i; ++p) s -= Lw[i * S + p] * Tw[p * S + c];
      Tw[i * S + c] = i < c ? 0.0 : s / Lw[i * S + i];
    }
  __syncthreads();
  for (int e = tid; e < n * n; e += nt) {
    const int a = e / n, c = e % n;
    double s = 0.0;
    for (int p = (a > c ? a : c); p < n; ++p) s = fma(Tw[p * S + a], Tw[p * S + c], s);
    Ai[a * S + c] = s;
  }
  __syncthreads();
}

// block_spd_inverse on ONE wave (lanes, no barriers: every LDS write is
// waited for before the lanes that read it issue their reads) — the same
// operations in the same order, so several small inverses run side by side
// on different waves of a workgroup.  A, Ai, Lw, Tw MUST be LDS (__shared__)
// memory: they are cast to the LDS address space here, so every access is a
// ds_* instruction and `s_waitcnt lgkmcnt(0)` is the complete wait (a flat or
// global pointer would need vmcnt too — and is undefined after the cast).
// `bad` (LDS) is raised with an atomic OR: several waves may report at once.
typedef __attribute__((address_space(3))) double lds_double;
DFM_DEV void wave_spd_inverse(const double *A_, double *Ai_, double *Lw_, double *Tw_, int n, int S, int *bad) {
  const lds_double *A = (const lds_double *)A_;
  lds_double *Ai = (lds_double *)Ai_, *Lw = (lds_double *)Lw_, *Tw = (lds_double *)Tw_;
  const int lane = threadIdx.x & 63;
  auto sync = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  for (int e = lane; e < n * S; e += 64) Lw[e] = 0.0;
  sync();
  for (int j = 0; j < n; ++j) {
    if (lane == 0) {
      double s = A[j * S + j];
      for (int p = 0; p < j; ++p) s -= Lw[j * S + p] * Lw[j * S + p];
      if (!(s > 0.0)) { atomicOr(bad, 1); s = 1.0; }
      Lw[j * S + j] = sqrt(s);
    }
    sync();
    for (int i = j + 1 + lane; i < n; i += 64) {
      double s = A[i * S + j];
      for (int p = 0; p < j; ++p) s -= Lw[i * S + p] * Lw[j * S + p];
      Lw[i * S + j] = s / Lw[j * S + j];
    }
    sync();
  }
  for (int c = lane; c < n; c += 64)
    for (int i = 0; i < n; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int p = c; p < i; ++p) s -= Lw[i * S + p] * Tw[p * S + c];
      Tw[i * S + c] = i < c ? 0.0 : s / Lw[i * S + i];
    }
  sync();
  for (int e = lane; e < n * n; e += 64) {
    const int a = e / n, c = e % n;
    double s = 0.0;
    for (int p = (a > c ? a : c); p < n; ++p) s = fma(Tw[p * S + a], Tw[p * S + c], s);
    Ai[a * S + c] = s;
  }
  sync();
}

}  // namespace dfm
