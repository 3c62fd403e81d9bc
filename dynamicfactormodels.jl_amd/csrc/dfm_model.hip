// dfm_model.hip — K3: the fused, HBM-bound kernels around the eigensolver:
// factor/loading passes, common-component / factor-residual panels, the
// OLS + HC2 regression of y on [w F_r], and the per-replicate statistics.
#include "dfm_common.h"

namespace dfm {

// Column-major T x N (ld ldx) -> row-major panel T x ld, zero padding.
__global__ void panel_from_colmajor_kernel(const double *__restrict__ X, int64_t ldx, int T, int N,
                                           double *__restrict__ P, int64_t ld) {
  __shared__ double tile[32][33];
  const int n0 = blockIdx.x * 32, t0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r, t = t0 + tx;
    tile[r][tx] = (n < N && t < T) ? X[(int64_t)n * ldx + t] : 0.0;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int t = t0 + r, n = n0 + tx;
    if (t < T && n < ld) P[(int64_t)t * ld + n] = tile[tx][r];
  }
}

// Row-major (rep x rows x ld) -> column-major host layout helper on device.
__global__ void colmajor_from_rows_kernel(const double *__restrict__ P, int64_t ld, int T, int N,
                                          double *__restrict__ X) {
  __shared__ double tile[32][33];
  const int n0 = blockIdx.x * 32, t0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int t = t0 + r, n = n0 + tx;
    tile[r][tx] = (t < T && n < N) ? P[(int64_t)t * ld + n] : 0.0;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r, t = t0 + tx;
    if (n < N && t < T) X[(int64_t)n * T + t] = tile[tx][r];
  }
}

// ----------------------------------------------------------------- factors
// N > T branch (src/DynamicFactorModel.jl:87-90): F = sqrt(T) U, L = X*' F / T.
// One thread per variable n; F rows staged in LDS.  Also ||x*_n||^2 and the
// per-variable factor-residual SSR ||x_n - F l_n||^2 = ||x_n||^2 - T ||l_n||^2.
template <int KM, bool HAS_C, bool HAS_ETA, bool HAS_IDX>
__global__ __launch_bounds__(256) void factors_rows_kernel(PanelSrc src, int T, int N, int k,
                                                           const double *__restrict__ Uk,
                                                           double *__restrict__ F,
                                                           double *__restrict__ L,
                                                           double *__restrict__ colssr, double Ts,
                                                           int64_t fstride) {
  constexpr int TR = 64;
  __shared__ double sF[TR * KM];
  __shared__ double sE[TR];
  __shared__ int sI[TR];
  const int rep = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
  const double sT = sqrt(Ts);
  const double *U = Uk + (int64_t)rep * T * k;
  double *Fr = F + (int64_t)rep * fstride;
  if (blockIdx.x == 0)
    for (int e = threadIdx.x; e < T * k; e += 256) Fr[e] = sT * U[e];
  const int32_t *idx = HAS_IDX ? src.idx + (int64_t)rep * src.rs : nullptr;
  const double *eta = HAS_ETA ? src.eta + (int64_t)rep * src.rs : nullptr;
  double acc[KM];
#pragma unroll
  for (int j = 0; j < KM; ++j) acc[j] = 0.0;
  double ss = 0.0;
  const bool ok = n < N;
  for (int t0 = 0; t0 < T; t0 += TR) {
    __syncthreads();
    for (int e = threadIdx.x; e < TR * KM; e += 256) {
      const int r = e / KM, j = e % KM;
      sF[e] = (t0 + r < T && j < k) ? sT * U[(int64_t)(t0 + r) * k + j] : 0.0;
    }
    if (threadIdx.x < TR) {
      const int t = t0 + threadIdx.x;
      sE[threadIdx.x] = (HAS_ETA && t < T) ? eta[t] : 1.0;
      sI[threadIdx.x] = (t < T) ? (HAS_IDX ? idx[t] : t) : 0;
    }
    __syncthreads();
    const int tn = min(TR, T - t0);
    if (ok) {
      for (int r = 0; r < tn; ++r) {
        const int t = t0 + r;
        double x = src.E[(int64_t)sI[r] * src.ld + n];
        if (HAS_ETA) x *= sE[r];
        if (HAS_C) x += src.C[(int64_t)t * src.ld + n];
        ss = fma(x, x, ss);
#pragma unroll
        for (int j = 0; j < KM; ++j) acc[j] = fma(x, sF[r * KM + j], acc[j]);
      }
    }
  }
  if (ok) {
    double l2 = 0.0;
    double *Lr = L + (int64_t)rep * N * k + (int64_t)n * k;
#pragma unroll
    for (int j = 0; j < KM; ++j)
      if (j < k) { const double l = acc[j] / Ts; Lr[j] = l; l2 = fma(l, l, l2); }
    if (colssr) colssr[(int64_t)rep * N + n] = ss - Ts * l2;
  }
}

// T >= N branch (src/DynamicFactorModel.jl:78-81): L = sqrt(N) V, F = X* L / N.
// One wave per time row t.
template <int KM, bool HAS_C, bool HAS_ETA, bool HAS_IDX>
__global__ __launch_bounds__(256) void factors_cols_kernel(PanelSrc src, int T, int N, int k,
                                                           const double *__restrict__ Uk,
                                                           double *__restrict__ F,
                                                           double *__restrict__ L,
                                                           int64_t fstride) {
  const int rep = blockIdx.y, lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const double sN = sqrt((double)N);
  const double *U = Uk + (int64_t)rep * N * k;
  if (blockIdx.x == 0) {
    double *Lr = L + (int64_t)rep * N * k;
    for (int e = threadIdx.x; e < N * k; e += 256) Lr[e] = sN * U[e];
  }
  if (t >= T) return;
  const int er = HAS_IDX ? src.idx[(int64_t)rep * src.rs + t] : t;
  const double ev = HAS_ETA ? src.eta[(int64_t)rep * src.rs + t] : 1.0;
  double acc[KM];
#pragma unroll
  for (int j = 0; j < KM; ++j) acc[j] = 0.0;
  for (int n = lane; n < N; n += 64) {
    double x = src.E[(int64_t)er * src.ld + n] * ev;
    if (HAS_C) x += src.C[(int64_t)t * src.ld + n];
#pragma unroll
    for (int j = 0; j < KM; ++j)
      if (j < k) acc[j] = fma(x, U[(int64_t)n * k + j], acc[j]);
  }
  double *Fr = F + (int64_t)rep * fstride + (int64_t)t * k;
#pragma unroll
  for (int j = 0; j < KM; ++j) {
    const double s = wave_sum(acc[j]);
    if (j < k && lane == 0) Fr[j] = s * sN / N;   // X (sqrt(N) V) / N
  }
}

// Per-variable SSR in the T >= N branch: ||x_n||^2 - sum_j lambda_j U[n][j]^2
// (G_nn from the Gram diagonal).
__global__ void colssr_cols_kernel(const double *__restrict__ G, int64_t ldg, int64_t strideG, int N,
                                   int k, const double *__restrict__ lam,
                                   const double *__restrict__ Uk, double *__restrict__ colssr) {
  const int rep = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double s = G[(int64_t)rep * strideG + (int64_t)n * ldg + n];
  for (int j = 0; j < k; ++j) {
    const double u = Uk[(int64_t)rep * N * k + (int64_t)n * k + j];
    s -= lam[(int64_t)rep * k + j] * u * u;
  }
  colssr[(int64_t)rep * N + n] = s;
}

// Common component C = F L' and factor residuals E = X - C
// (src/DynamicFactorModel.jl:33), row-major panels with zero padding.
__global__ void common_residual_kernel(const double *__restrict__ X, int64_t ld, int T, int N, int k,
                                       const double *__restrict__ F, const double *__restrict__ L,
                                       double *__restrict__ C, double *__restrict__ E) {
  const int t = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= ld) return;
  double c = 0.0;
  if (n < N)
    for (int j = 0; j < k; ++j) c = fma(F[(int64_t)t * k + j], L[(int64_t)n * k + j], c);
  const double x = X[(int64_t)t * ld + n];
  C[(int64_t)t * ld + n] = c;
  E[(int64_t)t * ld + n] = (n < N) ? x - c : 0.0;
}

// ||E||_F^2 of a row-major panel (T x ld, zero padding): per-row partial sums
// then a fixed-order sum — the brute-force sum(E.^2) of src/criteria.jl:5.
__global__ void panel_row_ssq_kernel(const double *__restrict__ E, int64_t ld, int T,
                                     double *__restrict__ rows) {
  __shared__ double red[256];
  const int t = blockIdx.x, tid = threadIdx.x;
  double s = 0.0;
  for (int64_t n = tid; n < ld; n += 256) { const double v = E[(int64_t)t * ld + n]; s = fma(v, v, s); }
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) { if (tid < o) red[tid] += red[tid + o]; __syncthreads(); }
  if (tid == 0) rows[t] = red[0];
}
__global__ void ordered_sum_kernel(const double *__restrict__ v, int n, double *__restrict__ out) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int i = tid; i < n; i += 256) s += v[i];
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) { if (tid < o) red[tid] += red[tid + o]; __syncthreads(); }
  if (tid == 0) *out = red[0];
}

// ------------------------------------------------------------------- OLS
// src/DynamicFactorModel.jl:40-48: D = [w F_r], beta = (D'D)^-1 D'y,
// u = y - D beta, h_t = d_t'(D'D)^-1 d_t, sigma2_t = u_t^2 / (1 - h_t) (HC2),
// Sigma = (D'D)^-1 (sum_t sigma2_t d_t d_t') (D'D)^-1, t = beta / sqrt(diag).
// One 256-thread workgroup per replicate; d = q + k <= 32.
constexpr int OLS_DMAX = 32;
constexpr int OLS_TR = 128;
// Per-replicate sample sizes Tn[rep] (rows 0..Tn-1 used) and factor counts
// kr[rep] <= kF are optional (expanding windows, src/utils.jl:59-65); F rows
// have stride kF, coefficient rows stride q + kF (unused tail = NaN).
template <int DMAX>
__global__ __launch_bounds__(256) void ols_hc2_kernel_t(const double *__restrict__ y,
                                                      const double *__restrict__ w, int q,
                                                      const double *__restrict__ F, int Tphys, int kF,
                                                      const int *__restrict__ Tn,
                                                      const int *__restrict__ kr,
                                                      double *__restrict__ coef,
                                                      double *__restrict__ tstat,
                                                      double *__restrict__ cov_out,
                                                      double *__restrict__ resid_out,
                                                      int *__restrict__ status,
                                                      const int *__restrict__ R0) {
  constexpr int S = DMAX + 1;
  __shared__ double sD[OLS_TR * S];
  __shared__ double sy[OLS_TR], ssig[OLS_TR];
  __shared__ double M[DMAX * S], Li[DMAX * S], Inv[DMAX * S], Meat[DMAX * S],
      Tmp[DMAX * S];
  __shared__ double sb[DMAX], sDy[DMAX];
  __shared__ int sbad;
  const int tid = threadIdx.x, rep = blockIdx.x;
  const int T = Tn ? Tn[rep] : Tphys;
  const int k = kr ? kr[rep] : kF;
  const int d = q + k, dstr = q + kF;
  const double *Fr = F + (int64_t)rep * Tphys * kF;
  if (R0) { y += R0[rep]; w += R0[rep]; }   // rolling windows: rows R0 .. R0 + T - 1 of y, w
  auto stage = [&](int t0) {
    for (int e = tid; e < OLS_TR * d; e += 256) {
      const int r = e / d, c = e % d, t = t0 + r;
      double v = 0.0;
      if (t < T) v = c < q ? w[(int64_t)c * Tphys + t] : Fr[(int64_t)t * kF + (c - q)];
      sD[r * S + c] = v;
    }
    for (int r = tid; r < OLS_TR; r += 256) sy[r] = (t0 + r < T) ? y[t0 + r] : 0.0;
  };
  // pass 1: D'D, D'y
  double accm[4] = {0, 0, 0, 0}, accy = 0.0;
  for (int t0 = 0; t0 < T; t0 += OLS_TR) {
    __syncthreads();
    stage(t0);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      if (e < d * d) {
        const int a = e / d, c = e % d;
        double s = accm[u];
        for (int r = 0; r < OLS_TR; ++r) s = fma(sD[r * S + a], sD[r * S + c], s);
        accm[u] = s;
      }
    }
    if (tid < d) {
      double s = accy;
      for (int r = 0; r < OLS_TR; ++r) s = fma(sD[r * S + tid], sy[r], s);
      accy = s;
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + 256 * u;
    if (e < d * d) M[(e / d) * S + e % d] = accm[u];
  }
  if (tid < d) sDy[tid] = accy;
  if (tid == 0) sbad = 0;
  __syncthreads();
  // Cholesky D'D = L L' (all threads step through j), then Inv = L^-T L^-1
  for (int e = tid; e < DMAX * S; e += 256) Li[e] = 0.0;
  __syncthreads();
  for (int j = 0; j < d; ++j) {
    if (tid == 0) {
      double s = M[j * S + j];
      for (int p = 0; p < j; ++p) s -= Li[j * S + p] * Li[j * S + p];
      if (!(s > 0.0)) { sbad = 1; s = 1.0; }
      Li[j * S + j] = sqrt(s);
    }
    __syncthreads();
    for (int i = j + 1 + tid; i < d; i += 256) {
      double s = M[i * S + j];
      for (int p = 0; p < j; ++p) s -= Li[i * S + p] * Li[j * S + p];
      Li[i * S + j] = s / Li[j * S + j];
    }
    __syncthreads();
  }
  // Tmp = L^-1 (column c per thread, forward substitution on e_c)
  for (int c = tid; c < d; c += 256)
    for (int i = 0; i < d; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int p = c; p < i; ++p) s -= Li[i * S + p] * Tmp[p * S + c];
      Tmp[i * S + c] = i < c ? 0.0 : s / Li[i * S + i];
    }
  __syncthreads();
  for (int e = tid; e < d * d; e += 256) {
    const int a = e / d, c = e % d;
    double s = 0.0;
    for (int p = max(a, c); p < d; ++p) s = fma(Tmp[p * S + a], Tmp[p * S + c], s);
    Inv[a * S + c] = s;
  }
  __syncthreads();
  if (tid < d) {
    double s = 0.0;
    for (int p = 0; p < d; ++p) s = fma(Inv[tid * S + p], sDy[p], s);
    sb[tid] = s;
  }
  __syncthreads();
  // pass 2: residuals, leverages, HC2 meat
  double accq[4] = {0, 0, 0, 0};
  for (int t0 = 0; t0 < T; t0 += OLS_TR) {
    __syncthreads();
    stage(t0);
    __syncthreads();
    for (int r = tid; r < OLS_TR; r += 256) {
      const int t = t0 + r;
      if (t >= T) { ssig[r] = 0.0; continue; }
      double fit = 0.0, h = 0.0;
      for (int a = 0; a < d; ++a) {
        const double da = sD[r * S + a];
        fit = fma(da, sb[a], fit);
        double ia = 0.0;
        for (int c = 0; c < d; ++c) ia = fma(Inv[a * S + c], sD[r * S + c], ia);
        h = fma(da, ia, h);
      }
      const double u = sy[r] - fit;
      if (resid_out) resid_out[t] = u;
      ssig[r] = u * u / (1.0 - h);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      if (e < d * d) {
        const int a = e / d, c = e % d;
        double s = accq[u];
        for (int r = 0; r < OLS_TR; ++r) s = fma(ssig[r] * sD[r * S + a], sD[r * S + c], s);
        accq[u] = s;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + 256 * u;
    if (e < d * d) Meat[(e / d) * S + e % d] = accq[u];
  }
  __syncthreads();
  for (int e = tid; e < d * d; e += 256) {
    const int a = e / d, c = e % d;
    double s = 0.0;
    for (int p = 0; p < d; ++p) s = fma(Meat[a * S + p], Inv[p * S + c], s);
    Tmp[a * S + c] = s;
  }
  __syncthreads();
  for (int e = tid; e < d * d; e += 256) {
    const int a = e / d, c = e % d;
    double s = 0.0;
    for (int p = 0; p < d; ++p) s = fma(Inv[a * S + p], Tmp[p * S + c], s);
    M[a * S + c] = s;   // coefficient covariance
  }
  __syncthreads();
  if (tid < dstr) {
    coef[(int64_t)rep * dstr + tid] = tid < d ? sb[tid] : NAN;
    tstat[(int64_t)rep * dstr + tid] = tid < d ? sb[tid] / sqrt(M[tid * S + tid]) : NAN;
  }
  if (cov_out)
    for (int e = tid; e < d * d; e += 256) cov_out[(int64_t)rep * d * d + (e % d) * d + e / d] = M[(e / d) * S + e % d];
  if (tid == 0 && status) status[rep] = sbad ? 2 : 0;
}

// One-wave form of the same regression for d + 1 <= 16 (every bootstrap fit
// at r <= 14 with one regressor): the augmented design [D y] (T x 16, zero
// columns past d) runs through v_mfma_f64_16x16x4 chains instead of 256
// threads of LDS dot products, so a replicate is one wave and a CU holds
// ~14 of them.
//   pass 1  [D y]'[D y] over 4-row chunks: lane l holds element (t0 + (l >> 4),
//           l & 15), which is its own A and B operand; four accumulators
//           summed in fixed order -> D'D, D'y (column d), y'y;
//   Cholesky D'D = L L', Inv = L^-T L^-1, beta = Inv D'y (as ols_hc2_kernel_t);
//   pass 2  per 16-row tile D [Inv | beta] on MFMA (A: row l & 15, column
//           4s + (l >> 4)); h_t = sum_j (D Inv)_tj D_tj by xor shuffles over the
//           16 lanes of a row, u_t = y_t - D_t beta, sigma2_t = u_t^2 / (1 - h_t);
//           the meat D' diag(sigma2) D on MFMA in the pass-1 layout (the tile's
//           accumulator register g holds rows t0 + 4g + (l >> 4)).
// The row sums run in MFMA order (not ols_hc2_kernel_t's serial order):
// results agree to rounding, and are per-replicate (batch-invariant).
__global__ __launch_bounds__(64, 3) void ols_hc2_wave_kernel(const double *__restrict__ y, const double *__restrict__ w,
                                                         int q, const double *__restrict__ F, int Tphys, int kF,
                                                         const int *__restrict__ Tn, const int *__restrict__ kr,
                                                         double *__restrict__ coef, double *__restrict__ tstat,
                                                         double *__restrict__ cov_out, double *__restrict__ resid_out,
                                                         int *__restrict__ status, const int *__restrict__ R0) {
  constexpr int S = 17;
  __shared__ double M[16 * S], Li[16 * S], Inv[16 * S], Tmp[16 * S];
  __shared__ double sb[16];
  __shared__ int sbad;
  const int tid = threadIdx.x, rep = blockIdx.x, li = tid & 15, lk = tid >> 4;
  const int T = Tn ? Tn[rep] : Tphys;
  const int k = kr ? kr[rep] : kF;
  const int d = q + k, dstr = q + kF;
  const double *Fr = F + (int64_t)rep * Tphys * kF;
  if (R0) { y += R0[rep]; w += R0[rep]; }   // rolling windows: rows R0 .. R0 + T - 1 of y, w
  // column j of [D y] as (base, row stride); columns past d read nothing
  struct Col { const double *p; int st; bool on; };
  auto col = [&](int j) -> Col {
    if (j < q) return {w + (int64_t)j * Tphys, 1, true};
    if (j < d) return {Fr + (j - q), kF, true};
    return {y, 1, j == d};
  };
  auto ld = [&](const Col &c, int t) -> double { return (c.on && t < T) ? c.p[(int64_t)t * c.st] : 0.0; };
  const Col cl = col(li);
  // ---- pass 1
  dv4 a4[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a4[u] = dv4{0.0, 0.0, 0.0, 0.0};
  for (int t0 = 0; t0 < T; t0 += 64) {   // 16 loads in flight per lane
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = ld(cl, t0 + 4 * u + lk);
#pragma unroll
    for (int u = 0; u < 16; ++u) a4[u & 3] = mfma16(v[u], v[u], a4[u & 3]);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) M[(4 * g + lk) * S + li] = ((a4[0][g] + a4[1][g]) + a4[2][g]) + a4[3][g];
  for (int e = tid; e < 16 * S; e += 64) Li[e] = 0.0;
  if (tid == 0) sbad = 0;
  __syncthreads();
  // ---- Cholesky, inverse, beta (ols_hc2_kernel_t's arithmetic)
  for (int j = 0; j < d; ++j) {
    if (tid == 0) {
      double s = M[j * S + j];
      for (int p = 0; p < j; ++p) s -= Li[j * S + p] * Li[j * S + p];
      if (!(s > 0.0)) { sbad = 1; s = 1.0; }
      Li[j * S + j] = sqrt(s);
    }
    __syncthreads();
    for (int i = j + 1 + tid; i < d; i += 64) {
      double s = M[i * S + j];
      for (int p = 0; p < j; ++p) s -= Li[i * S + p] * Li[j * S + p];
      Li[i * S + j] = s / Li[j * S + j];
    }
    __syncthreads();
  }
  for (int c = tid; c < d; c += 64)
    for (int i = 0; i < d; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int p = c; p < i; ++p) s -= Li[i * S + p] * Tmp[p * S + c];
      Tmp[i * S + c] = i < c ? 0.0 : s / Li[i * S + i];
    }
  __syncthreads();
  for (int e = tid; e < 16 * 16; e += 64) {
    const int a = e >> 4, c = e & 15;
    double s = 0.0;
    if (a < d && c < d)
      for (int p = max(a, c); p < d; ++p) s = fma(Tmp[p * S + a], Tmp[p * S + c], s);
    Inv[a * S + c] = s;   // zero outside d x d
  }
  __syncthreads();
  if (tid < d) {
    double s = 0.0;
    for (int p = 0; p < d; ++p) s = fma(Inv[tid * S + p], M[p * S + d], s);
    sb[tid] = s;
  }
  __syncthreads();
  // ---- pass 2: B operand [Inv | beta] (row k = 4s + (l >> 4), column l & 15)
  double Bm[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int kk = 4 * s + lk;
    Bm[s] = li < d ? Inv[kk * S + li] : ((li == d && kk < d) ? sb[kk] : 0.0);
  }
  Col ca[4];   // A-operand columns 4s + (l >> 4) of D (the y column excluded)
#pragma unroll
  for (int s = 0; s < 4; ++s) { ca[s] = col(4 * s + lk); ca[s].on = 4 * s + lk < d; }
  dv4 mt[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) mt[u] = dv4{0.0, 0.0, 0.0, 0.0};
  const int src = (tid & 48) | d;   // lane of this row group holding column d
  for (int tb = 0; tb < T; tb += 32) {   // two 16-row tiles, 16 loads in flight per lane
    double av[2][4], dgt[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int s = 0; s < 4; ++s) av[h][s] = ld(ca[s], tb + 16 * h + li);
#pragma unroll
      for (int g = 0; g < 4; ++g) dgt[h][g] = ld(cl, tb + 16 * h + 4 * g + lk);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
    const int t0 = tb + 16 * h;
    const double *dg = dgt[h];
    dv4 out = dv4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s) out = mfma16(av[h][s], Bm[s], out);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int t = t0 + 4 * g + lk;
      double h = li < d ? out[g] * dg[g] : 0.0;
      h += __shfl_xor(h, 8);
      h += __shfl_xor(h, 4);
      h += __shfl_xor(h, 2);
      h += __shfl_xor(h, 1);
      const double u = __shfl(dg[g] - out[g], src);   // y_t - D_t beta (lane d of the row)
      const double sig = t < T ? u * u / (1.0 - h) : 0.0;
      if (resid_out && li == d && t < T) resid_out[t] = u;
      const double dm = li < d ? dg[g] : 0.0;
      mt[g] = mfma16(dm * sig, dm, mt[g]);
    }
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) Tmp[(4 * g + lk) * S + li] = ((mt[0][g] + mt[1][g]) + mt[2][g]) + mt[3][g];
  __syncthreads();
  // ---- sandwich Inv Meat Inv, outputs (ols_hc2_kernel_t's arithmetic)
  for (int e = tid; e < d * d; e += 64) {
    const int a = e / d, c = e % d;
    double s = 0.0;
    for (int p = 0; p < d; ++p) s = fma(Tmp[a * S + p], Inv[p * S + c], s);
    Li[a * S + c] = s;
  }
  __syncthreads();
  for (int e = tid; e < d * d; e += 64) {
    const int a = e / d, c = e % d;
    double s = 0.0;
    for (int p = 0; p < d; ++p) s = fma(Inv[a * S + p], Li[p * S + c], s);
    M[a * S + c] = s;   // coefficient covariance
  }
  __syncthreads();
  if (tid < dstr) {
    coef[(int64_t)rep * dstr + tid] = tid < d ? sb[tid] : NAN;
    tstat[(int64_t)rep * dstr + tid] = tid < d ? sb[tid] / sqrt(M[tid * S + tid]) : NAN;
  }
  if (cov_out)
    for (int e = tid; e < d * d; e += 64) cov_out[(int64_t)rep * d * d + (e % d) * d + e / d] = M[(e / d) * S + e % d];
  if (tid == 0 && status) status[rep] = sbad ? 2 : 0;
}

// d + 1 <= 16: one wave per replicate (ols_hc2_wave_kernel); else LDS sized
// to the design width: d <= 16 fits 5 workgroups per CU instead of 2.
hipError_t launch_ols(int nb, hipStream_t st, const double *y, const double *w, int q, const double *F, int Tphys,
                      int kF, const int *Tn, const int *kr, double *coef, double *tstat, double *cov_out,
                      double *resid_out, int *status, const int *R0) {
  if (q + kF + 1 <= 16)
    hipLaunchKernelGGL(ols_hc2_wave_kernel, dim3(nb), dim3(64), 0, st, y, w, q, F, Tphys, kF, Tn, kr, coef, tstat,
                       cov_out, resid_out, status, R0);
  else if (q + kF <= 16)
    hipLaunchKernelGGL(ols_hc2_kernel_t<16>, dim3(nb), dim3(256), 0, st, y, w, q, F, Tphys, kF, Tn, kr, coef, tstat,
                       cov_out, resid_out, status, R0);
  else
    hipLaunchKernelGGL(ols_hc2_kernel_t<OLS_DMAX>, dim3(nb), dim3(256), 0, st, y, w, q, F, Tphys, kF, Tn, kr, coef,
                       tstat, cov_out, resid_out, status, R0);
  return hipGetLastError();
}

// ---------------------------------------------------------------- stats
// Criteria, src/criteria.jl:17-53 (V from the trace identity).
DFM_DEV double criterion_dev(int code, double V, int k, int T, int N, double sigma2) {
  const double c = (double)(N + T) / ((double)N * (double)T);
  const double m = (double)min(T, N);
  switch (code) {
    case 0: return V + k * sigma2 * c * log(1.0 / c);
    case 1: return V + k * sigma2 * c * log(m);
    case 2: return V + k * sigma2 * log(m) / m;
    case 3: return log(V) + k * c * log(1.0 / c);
    case 4: return log(V) + k * c * log(m);
    case 5: return log(V) + k * log(m) / m;
    case 6: return V + k * log((double)T) / T;
  }
  return NAN;
}

struct StatDesc { int kind, arg0, arg1, off; };

// PCp's sigma^2 of each replicate's unrestricted fit (src/criteria.jl:18):
// V(h) = sum_{j >= h} lambda_j / (N T), h = ceil(m/2), from its full spectrum
// (descending), summed in a fixed order.
__global__ void tail_sigma2_kernel(const double *__restrict__ ev, int m, int h, int nb, double NT,
                                   double *__restrict__ sig2) {
  const int rep = blockIdx.x * blockDim.x + threadIdx.x;
  if (rep >= nb) return;
  double s = 0.0;
  for (int j = m - 1; j >= h; --j) s += ev[(int64_t)rep * m + j];
  sig2[rep] = s / NT;
}

// One thread per replicate.  out row stride = width.
__global__ void stats_kernel(int nb, int T, int N, int r, int q, int crit, double sigma2,
                             const double *__restrict__ sig2v,
                             const double *__restrict__ lam, const double *__restrict__ trace,
                             const double *__restrict__ coef, const double *__restrict__ tstat,
                             const int *__restrict__ iters, const StatDesc *__restrict__ sd, int ns,
                             double *__restrict__ out, int64_t width, const int *__restrict__ st1,
                             const int *__restrict__ st2, int *__restrict__ flag) {
  const int rep = blockIdx.x * blockDim.x + threadIdx.x;
  if (rep >= nb) return;
  if (flag) {   // the replicates' solver / OLS status into the job's flag (or_status_kernel's work, one launch fewer)
    if (st1[rep]) atomicOr(flag, 1);
    if (st2[rep]) atomicOr(flag, 2);
  }
  double s = trace[rep];
  for (int j = 0; j < r; ++j) s -= lam[(int64_t)rep * r + j];
  const double V = s / ((double)N * (double)T);
  const int d = q + r;
  for (int i = 0; i < ns; ++i) {
    const StatDesc st = sd[i];
    double v = NAN;
    switch (st.kind) {
      case 0: v = V; break;
      case 1: v = criterion_dev(st.arg0 >= 0 ? st.arg0 : crit, V, r, T, N, sig2v ? sig2v[rep] : sigma2); break;
      case 2: v = st.arg0 < r ? lam[(int64_t)rep * r + st.arg0] : NAN; break;
      case 3: v = st.arg0 < d ? coef[(int64_t)rep * d + st.arg0] : NAN; break;
      case 4: v = st.arg0 < d ? tstat[(int64_t)rep * d + st.arg0] : NAN; break;
      case 5: v = trace[rep]; break;
      case 12: v = iters ? (double)iters[rep] : NAN; break;   // DFM_STAT_ITERS (diagnostic)
      default: continue;   // per-variable stats are written by the Chow kernel
    }
    out[(int64_t)rep * width + st.off] = v;
  }
}

template <int KM>
static void launch_factors_km(int orient, const PanelSrc &src, int T, int N, int k, int nb,
                              const double *Uk, double *F, double *L, double *colssr, hipStream_t st,
                              double Ts, int64_t fs) {
  const bool c = src.C, e = src.eta, x = src.idx;
#define DFM_FR(C_, E_, X_)                                                                         \
  if (orient == 0)                                                                                 \
    hipLaunchKernelGGL((factors_rows_kernel<KM, C_, E_, X_>), dim3((N + 255) / 256, nb), dim3(256), \
                       0, st, src, T, N, k, Uk, F, L, colssr, Ts, fs);                                     \
  else                                                                                             \
    hipLaunchKernelGGL((factors_cols_kernel<KM, C_, E_, X_>), dim3((T + 3) / 4, nb), dim3(256), 0, \
                       st, src, T, N, k, Uk, F, L, fs);
  // every PanelSrc form the callers build (as launch_gram): wild / residual
  // replicates, plain panels, and masked relocated windows (no C; idx, eta)
  if (c && e && x) { DFM_FR(true, true, true) }
  else if (c && !e && x) { DFM_FR(true, false, true) }
  else if (!c && e && x) { DFM_FR(false, true, true) }
  else if (!c && !e && x) { DFM_FR(false, false, true) }
  else { DFM_FR(false, false, false) }
#undef DFM_FR
}
// T = rows of the panel block; Ts = the T of the sqrt(T) / (1/T) scaling
// (the full-sample T for a break block, defect D7); F of replicate b starts at
// F + b * fstride (the block's rows inside a stacked T x k factor matrix).
int launch_factors(int orient, const PanelSrc &src, int T, int N, int k, int nb,
                   const double *Uk, double *F, double *L, double *colssr, hipStream_t st,
                   double Ts, int64_t fstride) {
  if (Ts <= 0) Ts = T;
  if (fstride <= 0) fstride = (int64_t)T * k;
  if (k <= 8) launch_factors_km<8>(orient, src, T, N, k, nb, Uk, F, L, colssr, st, Ts, fstride);
  else if (k <= 16) launch_factors_km<16>(orient, src, T, N, k, nb, Uk, F, L, colssr, st, Ts, fstride);
  else if (k <= 32) launch_factors_km<32>(orient, src, T, N, k, nb, Uk, F, L, colssr, st, Ts, fstride);
  else return -1;
  return 0;
}



// T >= N bootstrap factors by the same identity as the replicate Grams
// (dfm_gram.hip gram_wk_*): with X* = C + D P E, C = F L' (base fit) and the
// replicate loadings L* = sqrt(N) U*,
//   F* = X* L* / N = ( F (L' L*) + D P (E L*) ) / N,
// so a replicate needs E L* (T x N x k, E shared and L2-resident) and the
// k x k block L' L* instead of a pass over its resampled panel.
// Two launches:
//  fact_el_kernel — E L* for the whole batch as ONE MFMA product
//    E (T x N) . [L*_1 .. L*_nb] (N x nb k), one wave per 32 x 16 output tile
//    (8 x 4 v_mfma_f64_4x4x4 fragments, N in chunks of 16), operands read
//    straight from L2 into the fragments (E rows: 4 x 128 B segments per
//    load; a replicate's U is n-major, so its k columns are contiguous),
//    written replicate-major G[rep][s][j].  (Round 4 computed it per
//    replicate, one thread per row s walking E's row: 64 rows per load
//    instruction, L1 thrashed — 0.29 ms per C2 lane, now ~0.01 ms.)
//  fact_gather_kernel — per replicate: L = L*, M = L' L*, and
//    F*[t] = (F[t] M + eta_t G[rep][idx_t]) / N.
// Per replicate the sums run in a fixed order (no dependence on the batch).
__global__ __launch_bounds__(256) void fact_el_kernel(const double *__restrict__ Ep, int64_t ld, int T, int N, int k,
                                                      int nb, const double *__restrict__ Uk, double *__restrict__ G) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrt = (T + 31) / 32, ncols = nb * k, nct = (ncols + 15) / 16;
  const int tile = blockIdx.x * 4 + wave;
  if (tile >= nrt * nct) return;   // wave-uniform; the kernel has no barriers
  // consecutive waves: the row tiles of one column tile (its U columns re-read from L1)
  const int rt = tile % nrt, ct = tile / nrt, rbase = rt * 32, cbase = ct * 16;
  const double sN = sqrt((double)N);
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const double *ea[8], *ub[4];
#pragma unroll
  for (int f = 0; f < 8; ++f) ea[f] = Ep + (int64_t)min(rbase + 4 * f + fi, T - 1) * ld;   // past T: discarded
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = min(cbase + 4 * q + fi, ncols - 1), rep = c / k;   // past the batch: discarded
    ub[q] = Uk + (int64_t)rep * N * k + (c - rep * k);
  }
  double acc[8][4];
#pragma unroll
  for (int f = 0; f < 8; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[f][q] = 0.0;
  // the next 16-deep chunk's loads issue before this chunk's MFMAs; the k
  // tail (n >= N) reads row N - 1 (finite), zeroed on the A side
  auto load = [&](int k0, double (&af)[8], double (&bf)[4]) {
    const int nc = min(k0 + fkc, N - 1);
#pragma unroll
    for (int f = 0; f < 8; ++f) af[f] = ea[f][nc];
#pragma unroll
    for (int q = 0; q < 4; ++q) bf[q] = ub[q][(int64_t)nc * k];
  };
  double af[8], bf[4];
  load(0, af, bf);
  for (int k0 = 0; k0 < N; k0 += 16) {
    double an[8], bn[4];
    if (k0 + 16 < N) load(k0 + 16, an, bn);
    const bool okn = k0 + fkc < N;
#pragma unroll
    for (int f = 0; f < 8; ++f) af[f] = okn ? af[f] : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) bf[q] = sN * bf[q];   // L* = sqrt(N) U*, rounded as L is
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[f][q] = mfma4(af[f], bf[q], acc[f][q]);
#pragma unroll
    for (int f = 0; f < 8; ++f) af[f] = an[f];
#pragma unroll
    for (int q = 0; q < 4; ++q) bf[q] = bn[q];
  }
  // the four k-blocks summed and transposed into (row, column) lanes (dfm_gemm.hip's epilogue)
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa) {
    const double a0 = acc[fa][0], a1 = acc[fa][1], a2 = acc[fa][2], a3 = acc[fa][3];
    const double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
    const double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
    const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
    const int row = rbase + 4 * fa + oi, col = cbase + 4 * blk + oj;
    if (row < T && col < ncols) {
      const int rep = col / k;
      G[((int64_t)rep * T + row) * k + (col - rep * k)] = v;
    }
  }
}

template <int KM>
__global__ __launch_bounds__(256) void fact_gather_kernel(int T, int N, int k, const double *__restrict__ Fb,
                                                          const double *__restrict__ Lb, int rb,
                                                          const int32_t *__restrict__ idx,
                                                          const double *__restrict__ eta, int64_t rs,
                                                          const double *__restrict__ Uk,
                                                          const double *__restrict__ G, double *__restrict__ F,
                                                          double *__restrict__ L, int64_t fstride) {
  extern __shared__ double fdyn[];
  double *sL = fdyn;                        // N x KM: L* = sqrt(N) U*
  double *sEt = sL + (size_t)N * KM;        // eta_t (T)
  int *sIx = (int *)(sEt + T);              // idx_t (T)
  __shared__ double sM[32 * KM];            // rb x k: L' L*
  __shared__ double sP[256];                // its partial sums
  const int rep = blockIdx.x, tid = threadIdx.x;
  const double sN = sqrt((double)N);
  const double *U = Uk + (int64_t)rep * N * k;
  double *Lr = L + (int64_t)rep * N * k;
  {   // the replicate's draws, staged (the gather below then issues its G loads without waiting for idx)
    const int32_t *ix = idx + (int64_t)rep * rs;
    const double *et = eta ? eta + (int64_t)rep * rs : nullptr;
    for (int t = tid; t < T; t += 256) { sIx[t] = ix[t]; sEt[t] = et ? et[t] : 1.0; }
  }
  for (int e = tid; e < N * k; e += 256) {
    const int n = e / k, j = e - n * k;
    const double v = sN * U[e];
    sL[n * KM + j] = v;
    Lr[e] = v;
  }
  __syncthreads();
  // M = L' L* (rb x k <= 256 entries): np = 256 / (rb k) partial sums per
  // entry (partial q over n = q, q + np, ...), then summed in q order — a
  // single thread's N-long chain per entry was most of this kernel's time
  {
    const int ne = rb * k, np = 256 / ne, e = tid / np, q = tid - e * np;
    if (e < ne) {
      const int i = e / k, j = e - i * k;
      double acc = 0.0;
      for (int n = q; n < N; n += np) acc = fma(Lb[(int64_t)n * rb + i], sL[n * KM + j], acc);
      sP[tid] = acc;
    }
    __syncthreads();
    if (tid < ne) {
      double acc = 0.0;
      for (int u = 0; u < np; ++u) acc += sP[tid * np + u];
      sM[(tid / k) * KM + tid % k] = acc;
    }
  }
  __syncthreads();
  const double *Gr = G + (int64_t)rep * T * k;
  double *Fr = F + (int64_t)rep * fstride;
  const double invN = 1.0 / N;
  for (int e = tid; e < T * k; e += 256) {
    const int t = e / k, j = e - t * k;
    double c = 0.0;   // (F (L' L*))[t][j]
    for (int i = 0; i < rb; ++i) c = fma(Fb[(int64_t)t * rb + i], sM[i * KM + j], c);
    const double x = fma(sEt[t], Gr[(int64_t)sIx[t] * k + j], c);
    Fr[(int64_t)t * k + j] = x * invN;
  }
}
// nb replicates; G: nb T k doubles of scratch.  false when the shape does not
// fit (caller keeps launch_factors)
bool launch_factors_cols_fact(const double *Ep, int64_t ld, int T, int N, int k, const double *Fb, const double *Lb,
                              int rb, const int32_t *idx, const double *eta, int64_t rs, int nb, const double *Uk,
                              double *F, double *L, int64_t fstride, double *G, hipStream_t st) {
  if (k < 1 || k > 8 || rb < 1 || rb > 32 || T < 1 || N < 1) return false;
  const size_t lds = (size_t)N * 8 * 8 + (size_t)T * 12;
  if (lds > 64 * 1024) return false;
  const int64_t tiles = (int64_t)((T + 31) / 32) * (((int64_t)nb * k + 15) / 16);
  hipLaunchKernelGGL(fact_el_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, st, Ep, ld, T, N, k, nb, Uk, G);
  hipLaunchKernelGGL(fact_gather_kernel<8>, dim3(nb), dim3(256), lds, st, T, N, k, Fb, Lb, rb, idx, eta, rs, Uk, G, F,
                     L, fstride);
  return hipGetLastError() == hipSuccess;
}

// ------------------------------------------------------------ break blocks
// Per-variable ||E_n||^2 of a row-major residual panel, rows summed in order
// (the per-variable SSR the Chow LR test reads, for a model fitted per break
// block: src/DynamicFactorModel.jl:33 with break_indices).
__global__ void col_ssq_kernel(const double *__restrict__ E, int64_t ld, int T, int N,
                               double *__restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int t = 0; t < T; ++t) { const double v = E[(int64_t)t * ld + n]; s = fma(v, v, s); }
  out[n] = s;
}

// Break blocks of a batch of replicates: the criteria read V(k) = (sum_j
// trace(G_j) - sum_j sum_{i<=k} lambda_{j,i}) / (N T), so the per-block top-r
// eigenvalues and traces are summed into one (lambda, trace) row per replicate.
__global__ void block_accum_kernel(const double *__restrict__ lam_b, const double *__restrict__ tr_b,
                                   int nb, int r, double *__restrict__ lam, double *__restrict__ tr,
                                   int first) {
  const int rep = blockIdx.x * blockDim.x + threadIdx.x;
  if (rep >= nb) return;
  for (int j = 0; j < r; ++j)
    lam[(int64_t)rep * r + j] = (first ? 0.0 : lam[(int64_t)rep * r + j]) + lam_b[(int64_t)rep * r + j];
  tr[rep] = (first ? 0.0 : tr[rep]) + tr_b[rep];
}

}  // namespace dfm
