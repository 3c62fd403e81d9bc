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

}  // namespace dfm
