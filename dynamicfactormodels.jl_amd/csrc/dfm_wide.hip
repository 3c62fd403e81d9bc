// dfm_wide.hip — the fit at ANY number of factors.  The register/LDS-sized
// kernels of dfm_model.hip cover k <= 32 factors and q + k <= 32 regressors
// (every bootstrap and window fit at the benchmarked configs); the reference
// allows r up to ceil(m/2) — its default constructor uses exactly that
// (src/DynamicFactorModel.jl:101, D2; test/DynamicFactorModel.jl:24 fits r =
// ceil(min(T,N)/2) with q = 5).  This file is the single-fit path for wider
// shapes, built from one strided fp64 GEMM:
//   * factors / loadings of a block (src/DynamicFactorModel.jl:77-92);
//   * OLS + HC2 on D = [w F_r] (:40-48) with inv(D'D) formed explicitly, as
//     the reference's `inv` does.
#include "dfm_common.h"
#include <algorithm>

namespace dfm {

// C(m, n) = alpha * sum_k A(m, k) B(k, n); element (i, j) of X at
// X[i * sXr + j * sXc].  64 x 64 tiles, 16-deep k slabs, 4 x 4 per thread.
__global__ __launch_bounds__(256) void gemm_strided_kernel(int M, int Nc, int K, double alpha,
                                                           const double *__restrict__ A, int64_t sAr, int64_t sAc,
                                                           const double *__restrict__ B, int64_t sBr, int64_t sBc,
                                                           double beta, double *C, int64_t sCr, int64_t sCc,
                                                           int64_t sAb, int64_t sBb, int64_t sCb) {
  __shared__ double As[16][65], Bs[16][65];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  A += blockIdx.z * sAb;
  B += blockIdx.z * sBb;
  C += blockIdx.z * sCb;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  double acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int e = tid; e < 1024; e += 256) {
      const int kk = e & 15, i = e >> 4;   // A: 64 rows x 16 k
      const int gm = m0 + i, gk = k0 + kk;
      As[kk][i] = (gm < M && gk < K) ? A[(int64_t)gm * sAr + (int64_t)gk * sAc] : 0.0;
      const int j = e & 63, kb = e >> 6;   // B: 16 k x 64 cols
      const int gn = n0 + j, gk2 = k0 + kb;
      Bs[kb][j] = (gn < Nc && gk2 < K) ? B[(int64_t)gk2 * sBr + (int64_t)gn * sBc] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gm = m0 + ty + 16 * i, gn = n0 + tx + 16 * j;
      if (gm < M && gn < Nc) {
        double *c = C + (int64_t)gm * sCr + (int64_t)gn * sCc;
        *c = beta == 0.0 ? alpha * acc[i][j] : fma(alpha, acc[i][j], beta * *c);
      }
    }
}

// C = alpha A B + beta C (beta == 0: C not read).  C may share an allocation
// with A or B when the elements touched are disjoint.
// Batched: problem z reads A + z sAb, B + z sBb, writes C + z sCb.
hipError_t gemm_batched(int nb, int M, int Nc, int K, double alpha, const double *A, int64_t sAr, int64_t sAc,
                        int64_t sAb, const double *B, int64_t sBr, int64_t sBc, int64_t sBb, double beta, double *C,
                        int64_t sCr, int64_t sCc, int64_t sCb, hipStream_t st) {
  if (nb < 1 || M < 1 || Nc < 1) return hipSuccess;
  hipLaunchKernelGGL(gemm_strided_kernel, dim3((Nc + 63) / 64, (M + 63) / 64, nb), dim3(256), 0, st, M, Nc, K, alpha,
                     A, sAr, sAc, B, sBr, sBc, beta, C, sCr, sCc, sAb, sBb, sCb);
  return hipGetLastError();
}
hipError_t gemm_strided(int M, int Nc, int K, double alpha, const double *A, int64_t sAr, int64_t sAc,
                        const double *B, int64_t sBr, int64_t sBc, double beta, double *C, int64_t sCr,
                        int64_t sCc, hipStream_t st) {
  return gemm_batched(1, M, Nc, K, alpha, A, sAr, sAc, 0, B, sBr, sBc, 0, beta, C, sCr, sCc, 0, st);
}
static void gemm_s(int M, int Nc, int K, double alpha, const double *A, int64_t sAr, int64_t sAc, const double *B,
                   int64_t sBr, int64_t sBc, double *C, int64_t sCr, int64_t sCc, hipStream_t st) {
  gemm_strided(M, Nc, K, alpha, A, sAr, sAc, B, sBr, sBc, 0.0, C, sCr, sCc, st);
}

__global__ void scale_copy_kernel(const double *__restrict__ x, int64_t n, double s, double *__restrict__ y) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = s * x[i];
}
// y[rep][i] = s x[rep][i] for strided batches (rows of n elements)
__global__ void scale_copy_batched_kernel(const double *__restrict__ x, int64_t sx, int64_t n, double s,
                                          double *__restrict__ y, int64_t sy) {
  const int rep = blockIdx.y;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[rep * sy + i] = s * x[rep * sx + i];
}

// per-variable SSR of the factor residual, N > T branch: ||x_n||^2 - Ts ||l_n||^2
__global__ void colssr_rows_fix_kernel(int N, int k, double Ts, const double *__restrict__ L,
                                       double *__restrict__ colssr) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double l2 = 0.0;
  for (int j = 0; j < k; ++j) { const double l = L[(int64_t)n * k + j]; l2 = fma(l, l, l2); }
  colssr[n] -= Ts * l2;
}
__global__ void col_ssq_plain_kernel(const double *__restrict__ P, int64_t ld, int T, int N,
                                     double *__restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int t = 0; t < T; ++t) { const double v = P[(int64_t)t * ld + n]; s = fma(v, v, s); }
  out[n] = s;
}

// X*_rep = C + eta_rep * E[idx_rep] (rows 0..T-1 of the PanelSrc), T x ld per replicate
__global__ void materialize_kernel(PanelSrc src, int T, int N, int64_t ld, double *__restrict__ X) {
  const int rep = blockIdx.z, t = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= ld) return;
  double v = 0.0;
  if (n < N) {
    const int er = src.idx ? src.idx[(int64_t)rep * src.rs + t] : t;
    const double ev = src.eta ? src.eta[(int64_t)rep * src.rs + t] : 1.0;
    v = src.E[(int64_t)er * src.ld + n] * ev;
    if (src.C) v += src.C[(int64_t)t * src.ld + n];
  }
  X[((int64_t)rep * T + t) * ld + n] = v;
}
hipError_t launch_materialize(const PanelSrc &src, int T, int N, int64_t ld, int nb, double *X, hipStream_t st) {
  hipLaunchKernelGGL(materialize_kernel, dim3((unsigned)((ld + 255) / 256), T, nb), dim3(256), 0, st, src, T, N, ld,
                     X);
  return hipGetLastError();
}

// Factors and loadings of one block at any k (the layouts of launch_factors),
// for nb panels X + rep * sX (row-major T x ld): orient 0 (N > T): F = sqrt(Ts) U,
// L = X' F / Ts; orient 1: L = sqrt(N) V, F = X V / sqrt(N).  U/V of replicate
// rep at Uk + rep * m * k, F at F + rep * fstride, L at L + rep * N * k.
int launch_factors_wide(int orient, const double *X, int64_t ld, int T, int N, int k, const double *Uk,
                        double *F, double *L, double *colssr, hipStream_t st, double Ts, int nb, int64_t sX,
                        int64_t fstride) {
  if (Ts <= 0) Ts = T;
  if (fstride <= 0) fstride = (int64_t)T * k;
  const int64_t sL = (int64_t)N * k;
  if (orient == 0) {
    const int64_t sU = (int64_t)T * k;
    hipLaunchKernelGGL(scale_copy_batched_kernel, dim3((unsigned)std::min<int64_t>(1024, (sU + 255) / 256), nb),
                       dim3(256), 0, st, Uk, sU, sU, sqrt(Ts), F, fstride);
    gemm_batched(nb, N, k, T, 1.0 / Ts, X, 1, ld, sX, F, k, 1, fstride, 0.0, L, k, 1, sL, st);
    if (colssr && nb == 1) {
      hipLaunchKernelGGL(col_ssq_plain_kernel, dim3((N + 255) / 256), dim3(256), 0, st, X, ld, T, N, colssr);
      hipLaunchKernelGGL(colssr_rows_fix_kernel, dim3((N + 255) / 256), dim3(256), 0, st, N, k, Ts, L, colssr);
    }
  } else {
    hipLaunchKernelGGL(scale_copy_batched_kernel, dim3((unsigned)std::min<int64_t>(1024, (sL + 255) / 256), nb),
                       dim3(256), 0, st, Uk, sL, sL, sqrt((double)N), L, sL);
    gemm_batched(nb, T, k, N, 1.0 / sqrt((double)N), X, ld, 1, sX, Uk, k, 1, sL, 0.0, F, k, 1, fstride, st);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ------------------------------------------------------------- wide OLS
// D = [w F] (T x d, row-major) per replicate; F of replicate rep at
// F + rep * Tphys * kF (row stride kF, first k columns used), rows t >= Tn[rep]
// zeroed (expanding windows) — they then drop out of D'D, D'y and the meat.
__global__ void design_kernel(const double *__restrict__ w, int q, const double *__restrict__ F, int T, int kF,
                              int k, const int *__restrict__ Tn, double *__restrict__ D) {
  const int d = q + k, rep = blockIdx.y;
  const int Tr = Tn ? Tn[rep] : T;
  const double *Fr = F + (int64_t)rep * T * kF;
  double *Dr = D + (int64_t)rep * T * d;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < (int64_t)T * d; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e / d), c = (int)(e % d);
    Dr[e] = t >= Tr ? 0.0 : (c < q ? w[(int64_t)c * T + t] : Fr[(int64_t)t * kF + (c - q)]);
  }
}

// In-place Cholesky of the row-major d x d M (lower), then Linv = L^-1
// (rows of Linv' per thread: Lt[c][i] = Linv[i][c]).  One workgroup per
// replicate (blockIdx.x).
__global__ __launch_bounds__(1024) void chol_inv_kernel(double *__restrict__ Mb, int d, double *__restrict__ Ltb,
                                                        int *__restrict__ status) {
  __shared__ int bad;
  __shared__ double piv;
  const int tid = threadIdx.x, rep = blockIdx.x;
  double *M = Mb + (int64_t)rep * d * d, *Lt = Ltb + (int64_t)rep * d * d;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int j = 0; j < d; ++j) {
    if (tid == 0) {
      double s = M[(int64_t)j * d + j];
      if (!(s > 0.0)) { bad = 1; s = 1.0; }
      piv = sqrt(s);
      M[(int64_t)j * d + j] = piv;
    }
    __syncthreads();
    const double pj = piv;
    for (int i = j + 1 + tid; i < d; i += 1024) M[(int64_t)i * d + j] /= pj;
    __syncthreads();
    // trailing lower triangle: M[i][c] -= L[i][j] L[c][j], j < c <= i
    const int n = d - j - 1;
    const int64_t tot = (int64_t)n * (n + 1) / 2;
    for (int64_t e = tid; e < tot; e += 1024) {
      // e -> (i, c) with i >= c, row-wise packed: i' = floor((sqrt(8e+1)-1)/2)
      int ip = (int)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
      while ((int64_t)ip * (ip + 1) / 2 > e) --ip;
      while ((int64_t)(ip + 1) * (ip + 2) / 2 <= e) ++ip;
      const int cp = (int)(e - (int64_t)ip * (ip + 1) / 2);
      const int i = j + 1 + ip, c = j + 1 + cp;
      M[(int64_t)i * d + c] -= M[(int64_t)i * d + j] * M[(int64_t)c * d + j];
    }
    __syncthreads();
  }
  // Linv column c by forward substitution, stored as row c of Lt
  for (int c = tid; c < d; c += 1024) {
    double *x = Lt + (int64_t)c * d;
    for (int i = 0; i < c; ++i) x[i] = 0.0;
    for (int i = c; i < d; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      const double *Li = M + (int64_t)i * d;
      for (int p = c; p < i; ++p) s -= Li[p] * x[p];
      x[i] = s / Li[i];
    }
  }
  if (tid == 0 && status) status[rep] = bad ? 2 : 0;
}

// Per row t (one wave): fit, leverage h_t = sum_c H1[t][c] D[t][c] with
// H1 = D inv(D'D), u_t, sigma2_t = u_t^2 / (1 - h_t), Ds = sigma2_t * D[t].
__global__ void hc2_rows_kernel(const double *__restrict__ Db, const double *__restrict__ H1b,
                                const double *__restrict__ y, const double *__restrict__ betab, int T, int d,
                                const int *__restrict__ Tn, double *__restrict__ Dsb, double *__restrict__ resid) {
  const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6), rep = blockIdx.y;
  if (t >= T) return;
  const int64_t o = ((int64_t)rep * T + t) * d;
  const double *Dt = Db + o, *Ht = H1b + o, *beta = betab + (int64_t)rep * d;
  const bool in = !Tn || t < Tn[rep];
  double fit = 0.0, h = 0.0;
  for (int c = lane; c < d; c += 64) { fit = fma(Dt[c], beta[c], fit); h = fma(Ht[c], Dt[c], h); }
  fit = wave_sum(fit);
  h = wave_sum(h);
  const double u = y[t] - fit, s2 = in ? u * u / (1.0 - h) : 0.0;
  if (lane == 0 && resid && in) resid[(int64_t)rep * T + t] = u;
  for (int c = lane; c < d; c += 64) Dsb[o + c] = s2 * Dt[c];
}

// coef / t rows of stride dstr (NaN past d), optional covariance (nb == 1)
__global__ void ols_finish_kernel(const double *__restrict__ betab, const double *__restrict__ Sigb, int d, int dstr,
                                  double *__restrict__ coef, double *__restrict__ tstat, double *__restrict__ cov) {
  const int rep = blockIdx.y;
  const double *beta = betab + (int64_t)rep * d, *Sig = Sigb + (int64_t)rep * d * d;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < d * d; e += gridDim.x * 256) {
    const int a = e / d, c = e % d;
    if (cov) cov[(int64_t)c * d + a] = Sig[e];
    if (a == c) {
      coef[(int64_t)rep * dstr + a] = beta[a];
      tstat[(int64_t)rep * dstr + a] = beta[a] / sqrt(Sig[e]);
    }
  }
  for (int a = d + blockIdx.x * 256 + threadIdx.x; a < dstr; a += gridDim.x * 256) {
    coef[(int64_t)rep * dstr + a] = NAN;
    tstat[(int64_t)rep * dstr + a] = NAN;
  }
}

int64_t ols_wide_work(int T, int d) { return 3 * (int64_t)T * d + 6 * (int64_t)d * d + 2 * (int64_t)d; }

// src/DynamicFactorModel.jl:40-48 for nb fits of any width d = q + k: F of
// replicate rep at F + rep * T * kF (first k of kF columns), optional sample
// sizes Tn; coef / tstat rows of stride q + kF; work: nb * ols_wide_work(T, d).
hipError_t launch_ols_wide_batched(int nb, const double *y, const double *w, int q, const double *F, int T, int kF,
                                   int k, const int *Tn, double *coef, double *tstat, double *cov_out,
                                   double *resid_out, int *status, double *work, hipStream_t st) {
  const int d = q + k, dstr = q + kF;
  const int64_t Td = (int64_t)T * d, dd = (int64_t)d * d;
  double *D = work, *H1 = D + nb * Td, *Ds = H1 + nb * Td, *DtD = Ds + nb * Td;
  double *Lt = DtD + nb * dd, *Inv = Lt + nb * dd, *Meat = Inv + nb * dd;
  double *Tmp = Meat + nb * dd, *Sig = Tmp + nb * dd, *Dty = Sig + nb * dd, *beta = Dty + (int64_t)nb * d;
  hipLaunchKernelGGL(design_kernel, dim3((unsigned)std::min<int64_t>(1024, (Td + 255) / 256), nb), dim3(256), 0, st,
                     w, q, F, T, kF, k, Tn, D);
  gemm_batched(nb, d, d, T, 1.0, D, 1, d, Td, D, d, 1, Td, 0.0, DtD, d, 1, dd, st);       // D'D
  gemm_batched(nb, d, 1, T, 1.0, D, 1, d, Td, y, 1, 0, 0, 0.0, Dty, 1, 0, d, st);         // D'y
  hipLaunchKernelGGL(chol_inv_kernel, dim3(nb), dim3(1024), 0, st, DtD, d, Lt, status);
  gemm_batched(nb, d, d, d, 1.0, Lt, d, 1, dd, Lt, 1, d, dd, 0.0, Inv, d, 1, dd, st);      // Linv' Linv
  gemm_batched(nb, d, 1, d, 1.0, Inv, d, 1, dd, Dty, 1, 0, d, 0.0, beta, 1, 0, d, st);     // beta
  gemm_batched(nb, T, d, d, 1.0, D, d, 1, Td, Inv, d, 1, dd, 0.0, H1, d, 1, Td, st);       // D inv(D'D)
  hipLaunchKernelGGL(hc2_rows_kernel, dim3((T + 3) / 4, nb), dim3(256), 0, st, D, H1, y, beta, T, d, Tn, Ds,
                     resid_out);
  gemm_batched(nb, d, d, T, 1.0, D, 1, d, Td, Ds, d, 1, Td, 0.0, Meat, d, 1, dd, st);     // sum sigma2_t d_t d_t'
  gemm_batched(nb, d, d, d, 1.0, Meat, d, 1, dd, Inv, d, 1, dd, 0.0, Tmp, d, 1, dd, st);
  gemm_batched(nb, d, d, d, 1.0, Inv, d, 1, dd, Tmp, d, 1, dd, 0.0, Sig, d, 1, dd, st);
  hipLaunchKernelGGL(ols_finish_kernel, dim3((unsigned)std::min<int64_t>(64, (dd + 255) / 256), nb), dim3(256), 0,
                     st, beta, Sig, d, dstr, coef, tstat, nb == 1 ? cov_out : nullptr);
  return hipGetLastError();
}
hipError_t launch_ols_wide(const double *y, const double *w, int q, const double *F, int T, int k, double *coef,
                           double *tstat, double *cov_out, double *resid_out, int *status, double *work,
                           hipStream_t st) {
  return launch_ols_wide_batched(1, y, w, q, F, T, k, k, nullptr, coef, tstat, cov_out, resid_out, status, work, st);
}

}  // namespace dfm
