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
                                const int *__restrict__ Tn, double *__restrict__ Dsb, double *__restrict__ resid,
                                int hc0) {
  const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6), rep = blockIdx.y;
  if (t >= T) return;
  const int64_t o = ((int64_t)rep * T + t) * d;
  const double *Dt = Db + o, *Ht = H1b + o, *beta = betab + (int64_t)rep * d;
  const bool in = !Tn || t < Tn[rep];
  double fit = 0.0, h = 0.0;
  for (int c = lane; c < d; c += 64) { fit = fma(Dt[c], beta[c], fit); if (!hc0) h = fma(Ht[c], Dt[c], h); }
  fit = wave_sum(fit);
  h = wave_sum(h);
  const double u = y[t] - fit, s2 = in ? u * u / (1.0 - h) : 0.0;
  if (lane == 0 && resid && in) resid[(int64_t)rep * T + t] = u;
  for (int c = lane; c < d; c += 64) Dsb[o + c] = s2 * Dt[c];
}

// coef / t rows of stride dstr (NaN past d), optional covariance (nb == 1)
__global__ void ols_finish_kernel(const double *__restrict__ betab, const double *__restrict__ Sigb, int d, int dstr,
                                  double *__restrict__ coef, double *__restrict__ tstat, double *__restrict__ cov,
                                  int flip) {
  const int rep = blockIdx.y;
  const double *beta = betab + (int64_t)rep * d, *Sig = Sigb + (int64_t)rep * d * d;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < d * d; e += gridDim.x * 256) {
    const int a = e / d, c = e % d;
    if (cov) cov[(int64_t)c * d + a] = Sig[e];
    if (a == c) {
      coef[(int64_t)rep * dstr + a] = beta[a];
      tstat[(int64_t)rep * dstr + a] = beta[a] / sqrt(flip ? fabs(Sig[e]) : Sig[e]);
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
// hc0: White (1980) HC0 meat instead of HC2 and negative variances flipped
// (targeted_predictors, src/targeted_predictors.jl:13-24).
hipError_t launch_ols_wide_batched(int nb, const double *y, const double *w, int q, const double *F, int T, int kF,
                                   int k, const int *Tn, double *coef, double *tstat, double *cov_out,
                                   double *resid_out, int *status, double *work, hipStream_t st, int hc0) {
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
  if (!hc0) gemm_batched(nb, T, d, d, 1.0, D, d, 1, Td, Inv, d, 1, dd, 0.0, H1, d, 1, Td, st);   // D inv(D'D)
  hipLaunchKernelGGL(hc2_rows_kernel, dim3((T + 3) / 4, nb), dim3(256), 0, st, D, H1, y, beta, T, d, Tn, Ds,
                     resid_out, hc0);
  gemm_batched(nb, d, d, T, 1.0, D, 1, d, Td, Ds, d, 1, Td, 0.0, Meat, d, 1, dd, st);     // sum sigma2_t d_t d_t'
  gemm_batched(nb, d, d, d, 1.0, Meat, d, 1, dd, Inv, d, 1, dd, 0.0, Tmp, d, 1, dd, st);
  gemm_batched(nb, d, d, d, 1.0, Inv, d, 1, dd, Tmp, d, 1, dd, 0.0, Sig, d, 1, dd, st);
  hipLaunchKernelGGL(ols_finish_kernel, dim3((unsigned)std::min<int64_t>(64, (dd + 255) / 256), nb), dim3(256), 0,
                     st, beta, Sig, d, dstr, coef, tstat, nb == 1 ? cov_out : nullptr, hc0);
  return hipGetLastError();
}
hipError_t launch_ols_wide(const double *y, const double *w, int q, const double *F, int T, int k, double *coef,
                           double *tstat, double *cov_out, double *resid_out, int *status, double *work,
                           hipStream_t st) {
  return launch_ols_wide_batched(1, y, w, q, F, T, k, k, nullptr, coef, tstat, cov_out, resid_out, status, work, st,
                                 0);
}

__global__ void tp_mask_kernel(const double *__restrict__ t, int q, int N, double cv, double *__restrict__ tx,
                               uint8_t *__restrict__ mask) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const double v = t[q + i];
  tx[i] = v;
  mask[i] = fabs(v) > cv ? 1 : 0;
}
// JOINT hard thresholding at any width (src/targeted_predictors.jl:9-30):
// OLS of y on [w x] with HC0, |diag| flip, |t_x| > cv.  X: row-major T x ld.
hipError_t launch_targeted_joint_wide(const double *y, const double *w, int q, const double *X, int64_t ld, int T,
                                      int N, double cv, double *tx, uint8_t *mask, int *status, double *work,
                                      hipStream_t st) {
  const int d = q + N, dstr = q + (int)ld;
  double *coef = work, *tst = coef + dstr, *wk = tst + dstr;
  hipError_t e = launch_ols_wide_batched(1, y, w, q, X, T, (int)ld, N, nullptr, coef, tst, nullptr, nullptr, status,
                                         wk, st, 1);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tp_mask_kernel, dim3((N + 255) / 256), dim3(256), 0, st, tst, q, N, cv, tx, mask);
  (void)d;
  return hipGetLastError();
}
int64_t targeted_joint_wide_work(int T, int q, int N, int64_t ld) {
  return 2 * (q + ld) + ols_wide_work(T, q + N);
}

// ------------------------------------------------------------ wide Chow
// LR / LM / Wald for every variable at any r (src/chowtest.jl:4-42), for nb
// panels, built from strided GEMMs; every residual is formed explicitly, as
// the reference's projections do (no ||x||^2 - b'A^-1 b cancellation):
//   LR   : T (ln ||E_i||^2 - ln(SSR1_i + SSR2_i)), SSR_j from x_i on F_j (:4-23)
//   LM   : T (1 - ||M_D E_i||^2 / ||E_i||^2), D = [F, F o d]           (:35-42)
//   Wald : b2' [Q2 (sum_t u_ti^2 d_t d_t') Q2']^-1 b2, Q2 = rows r..2r-1 of
//          inv(D'D): the HC0 block = sum_t u_ti^2 g_t g_t', g_t = Q2 d_t, all
//          variables at once as (U o U)' [g_t (x) g_t]                  (:25-33)
__global__ void copy_panel_kernel(const double *__restrict__ X, int64_t ld, int64_t sX, int T, int N,
                                  double *__restrict__ Y) {
  const int rep = blockIdx.y;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < (int64_t)T * N; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e / N), n = (int)(e % N);
    Y[(int64_t)rep * T * N + e] = X[rep * sX + (int64_t)t * ld + n];
  }
}
__global__ void col_ssq_batched_kernel(const double *__restrict__ Y, int T, int N, double *__restrict__ out) {
  const int rep = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const double *Yr = Y + (int64_t)rep * T * N;
  double s = 0.0;
  for (int t = 0; t < T; ++t) { const double v = Yr[(int64_t)t * N + n]; s = fma(v, v, s); }
  out[(int64_t)rep * N + n] = s;
}
__global__ void chow_design_kernel(const double *__restrict__ F, int64_t sF, int T, int r, int bp,
                                   double *__restrict__ D) {
  const int rep = blockIdx.y;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < (int64_t)T * 2 * r; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e / (2 * r)), c = (int)(e % (2 * r));
    const double f = F[rep * sF + (int64_t)t * r + (c < r ? c : c - r)];
    D[(int64_t)rep * T * 2 * r + e] = (c < r || t >= bp) ? f : 0.0;
  }
}
__global__ void square_kernel(double *__restrict__ U, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) U[i] *= U[i];
}
__global__ void outer_rows_kernel(const double *__restrict__ Gm, int T, int r, double *__restrict__ Pm) {
  const int rep = blockIdx.y;
  const int64_t rr = (int64_t)r * r;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < (int64_t)T * rr; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e / rr), a = (int)((e % rr) / r), b = (int)(e % r);
    const double *g = Gm + ((int64_t)rep * T + t) * r;
    Pm[(int64_t)rep * T * rr + e] = g[a] * g[b];
  }
}
// per (replicate, variable): LR, LM and the Wald quadratic form ||Linv b2||^2
__global__ void chow_finish_kernel(int nb, int T, int N, int r, const double *__restrict__ eE,
                                   const double *__restrict__ ssr, const double *__restrict__ vv,
                                   const double *__restrict__ Bx, const double *__restrict__ Lt,
                                   const int *__restrict__ cst, double *__restrict__ LR, double *__restrict__ LM,
                                   double *__restrict__ WD, int64_t ostr, double *__restrict__ scr) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (int64_t)nb * N) return;
  const int rep = (int)(g / N), i = (int)(g % N);
  const double e2 = eE[g];
  const double lr = T * (log(e2) - log(ssr[g]));
  const double lm = T * (1.0 - vv[g] / e2);
  const double *b2 = Bx + (int64_t)rep * 2 * r * N + (int64_t)r * N + i;   // rows r..2r-1, column i
  const double *Li = Lt + g * r * r;                                        // Lt[p][a] = Linv[a][p]
  double wd = 0.0;
  for (int a = 0; a < r; ++a) {
    double z = 0.0;
    for (int p = 0; p <= a; ++p) z = fma(Li[(int64_t)p * r + a], b2[(int64_t)p * N], z);
    wd = fma(z, z, wd);
  }
  if (cst[g]) wd = NAN;
  if (LR) LR[rep * ostr + i] = lr;
  if (LM) LM[rep * ostr + i] = lm;
  if (WD) WD[rep * ostr + i] = wd;
  if (scr) {
    scr[g] = lr;
    scr[(int64_t)nb * N + g] = lm;
    scr[2 * (int64_t)nb * N + g] = wd;
  }
}

int64_t chow_wide_work(int T, int N, int r) {   // doubles per panel
  const int64_t TN = (int64_t)T * N, rN = (int64_t)r * N, rr = (int64_t)r * r;
  return 2 * TN + 3 * (int64_t)N + 6 * rr + 2 * rN + 2 * (int64_t)T * r + 12 * rr + 6 * rN + (int64_t)T * r +
         (int64_t)T * rr + 2 * (int64_t)N * rr + 8 + 2 * (int64_t)N;
}

// nb panels X + rep sX (T x ld row-major), factors F + rep sF (T x r), loadings
// L + rep sL (N x r); E (the factor residuals, same layout as X) or nullptr
// (then E = X - F L').  Outputs: rows rep * ostr of LR / LM / WD (any may be
// null) and, if scr != nullptr, [3][nb][N] scratch rows.
// Break models (nblk > 1, E == nullptr): E = X - F_j L_j' per block j, rows
// brow[j] .. brow[j+1]-1, block j's loadings at L + j * lbs.
hipError_t launch_chow_wide(int nb, const double *X, int64_t ld, int64_t sX, const double *E, int T, int N, int r,
                            int bp, const double *F, int64_t sF, const double *L, int64_t sL, double *LR, double *LM,
                            double *WD, int64_t ostr, double *scr, double *work, hipStream_t st, int nblk,
                            const int *brow, int64_t lbs) {
  const int64_t TN = (int64_t)T * N, rN = (int64_t)r * N, rr = (int64_t)r * r, r2 = 2 * (int64_t)r;
  double *Eb = work, *R = Eb + nb * TN, *eE = R + nb * TN, *ssr = eE + (int64_t)nb * N, *vv = ssr + (int64_t)nb * N;
  double *A1 = vv + (int64_t)nb * N, *A2 = A1 + nb * rr, *Lt1 = A2 + nb * rr, *Lt2 = Lt1 + nb * rr;
  double *A1i = Lt2 + nb * rr, *A2i = A1i + nb * rr, *B1 = A2i + nb * rr, *C1 = B1 + nb * rN;
  double *D = C1 + nb * rN, *DtD = D + nb * r2 * T, *LtD = DtD + nb * 4 * rr, *Di = LtD + nb * 4 * rr;
  double *G = Di + nb * 4 * rr, *G2 = G + nb * r2 * N, *Bx = G2 + nb * r2 * N, *Gm = Bx + nb * r2 * N;
  double *Pm = Gm + (int64_t)nb * T * r, *Sig = Pm + nb * (int64_t)T * rr, *LtS = Sig + nb * (int64_t)N * rr;
  int *cst = (int *)(LtS + nb * (int64_t)N * rr);
  const dim3 g1((unsigned)std::min<int64_t>(1024, (TN + 255) / 256), nb);
  hipError_t e;
#define GB(...) if ((e = gemm_batched(__VA_ARGS__)) != hipSuccess) return e
  // ||E_i||^2
  hipLaunchKernelGGL(copy_panel_kernel, g1, dim3(256), 0, st, E ? E : X, ld, sX, T, N, Eb);
  if (!E) {
    for (int j = 0; j < nblk; ++j) {
      const int a = nblk > 1 ? brow[j] : 0, b = (nblk > 1 && j + 1 < nblk) ? brow[j + 1] : T;
      GB(nb, b - a, N, r, -1.0, F + (int64_t)a * r, r, 1, sF, L + j * lbs, 1, r, sL, 1.0, Eb + (int64_t)a * N, N, 1,
         TN, st);
    }
  }
  hipLaunchKernelGGL(col_ssq_batched_kernel, dim3((N + 255) / 256, nb), dim3(256), 0, st, Eb, T, N, eE);
  // LR: x_i on F within each subperiod, residuals explicit
  hipLaunchKernelGGL(copy_panel_kernel, g1, dim3(256), 0, st, X, ld, sX, T, N, R);
  const int rows[2] = {bp, T - bp}, row0[2] = {0, bp};
  double *Aj[2] = {A1, A2}, *Ltj[2] = {Lt1, Lt2}, *Aij[2] = {A1i, A2i};
  for (int j = 0; j < 2; ++j) {
    const double *Fj = F + (int64_t)row0[j] * r;
    GB(nb, r, r, rows[j], 1.0, Fj, 1, r, sF, Fj, r, 1, sF, 0.0, Aj[j], r, 1, rr, st);
    hipLaunchKernelGGL(chol_inv_kernel, dim3(nb), dim3(1024), 0, st, Aj[j], r, Ltj[j], (int *)nullptr);
    GB(nb, r, r, r, 1.0, Ltj[j], r, 1, rr, Ltj[j], 1, r, rr, 0.0, Aij[j], r, 1, rr, st);
    GB(nb, r, N, rows[j], 1.0, Fj, 1, r, sF, X + (int64_t)row0[j] * ld, ld, 1, sX, 0.0, B1, N, 1, rN, st);
    GB(nb, r, N, r, 1.0, Aij[j], r, 1, rr, B1, N, 1, rN, 0.0, C1, N, 1, rN, st);
    GB(nb, rows[j], N, r, -1.0, Fj, r, 1, sF, C1, N, 1, rN, 1.0, R + (int64_t)row0[j] * N, N, 1, TN, st);
  }
  hipLaunchKernelGGL(col_ssq_batched_kernel, dim3((N + 255) / 256, nb), dim3(256), 0, st, R, T, N, ssr);
  // D = [F, F o d], inv(D'D)
  hipLaunchKernelGGL(chow_design_kernel, dim3((unsigned)std::min<int64_t>(1024, (T * r2 + 255) / 256), nb), dim3(256),
                     0, st, F, sF, T, r, bp, D);
  GB(nb, 2 * r, 2 * r, T, 1.0, D, 1, r2, r2 * T, D, r2, 1, r2 * T, 0.0, DtD, r2, 1, 4 * rr, st);
  hipLaunchKernelGGL(chol_inv_kernel, dim3(nb), dim3(1024), 0, st, DtD, 2 * r, LtD, (int *)nullptr);
  GB(nb, 2 * r, 2 * r, 2 * r, 1.0, LtD, r2, 1, 4 * rr, LtD, 1, r2, 4 * rr, 0.0, Di, r2, 1, 4 * rr, st);
  // LM: v = E - D inv(D'D) D'E
  GB(nb, 2 * r, N, T, 1.0, D, 1, r2, r2 * T, Eb, N, 1, TN, 0.0, G, N, 1, r2 * N, st);
  GB(nb, 2 * r, N, 2 * r, 1.0, Di, r2, 1, 4 * rr, G, N, 1, r2 * N, 0.0, G2, N, 1, r2 * N, st);
  GB(nb, T, N, 2 * r, -1.0, D, r2, 1, r2 * T, G2, N, 1, r2 * N, 1.0, Eb, N, 1, TN, st);   // Eb := V
  hipLaunchKernelGGL(col_ssq_batched_kernel, dim3((N + 255) / 256, nb), dim3(256), 0, st, Eb, T, N, vv);
  // Wald: beta = inv(D'D) D'x, U = X - D beta, HC0 block of every variable
  GB(nb, 2 * r, N, T, 1.0, D, 1, r2, r2 * T, X, ld, 1, sX, 0.0, G, N, 1, r2 * N, st);
  GB(nb, 2 * r, N, 2 * r, 1.0, Di, r2, 1, 4 * rr, G, N, 1, r2 * N, 0.0, Bx, N, 1, r2 * N, st);
  hipLaunchKernelGGL(copy_panel_kernel, g1, dim3(256), 0, st, X, ld, sX, T, N, R);
  GB(nb, T, N, 2 * r, -1.0, D, r2, 1, r2 * T, Bx, N, 1, r2 * N, 1.0, R, N, 1, TN, st);    // R := U
  hipLaunchKernelGGL(square_kernel, dim3((unsigned)std::min<int64_t>(2048, (nb * TN + 255) / 256)), dim3(256), 0, st, R,
                     nb * TN);
  GB(nb, T, r, 2 * r, 1.0, D, r2, 1, r2 * T, Di + r * r2, 1, r2, 4 * rr, 0.0, Gm, r, 1, (int64_t)T * r, st);
  hipLaunchKernelGGL(outer_rows_kernel, dim3((unsigned)std::min<int64_t>(2048, (T * rr + 255) / 256), nb), dim3(256),
                     0, st, Gm, T, r, Pm);
  GB(nb, N, (int)rr, T, 1.0, R, 1, N, TN, Pm, rr, 1, (int64_t)T * rr, 0.0, Sig, rr, 1, (int64_t)N * rr, st);
  hipLaunchKernelGGL(chol_inv_kernel, dim3(nb * N), dim3(1024), 0, st, Sig, r, LtS, cst);
  hipLaunchKernelGGL(chow_finish_kernel, dim3((unsigned)(((int64_t)nb * N + 255) / 256)), dim3(256), 0, st, nb, T, N,
                     r, eE, ssr, vv, Bx, LtS, cst, LR, LM, WD, ostr, scr);
#undef GB
  return hipGetLastError();
}

}  // namespace dfm
