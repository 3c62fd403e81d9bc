// dfm_predict.hip — get_factors / predict of a fitted model on new rows
// (src/DynamicFactorModel.jl:125-128, :152-155), with defect D4 repaired.
//
// The reference's get_factors reads the non-existent field dfm.rotation; the
// local `rotation = dfm.loadings * inv(dfm.loadings'dfm.loadings)` of :126 is
// meant, with dfm.loadings the first break block's full loadings (D1).  Only
// its first r columns are used ("active", :127).  In both branches L'L is
// diagonal (T >= N: L = sqrt(N) V, L'L = N I; N > T: L = X'F/T, L'L = Lambda/T),
// so rotation[:, j] = L_j / |L_j|^2 for j < r — the same columns the full
// inverse gives, without inverting the (for a centred N > T panel singular)
// full L'L.  New rows are normalised by the SCALAR mean and sample std of all
// T N entries of the fitted x (Julia 0.3 mean(A) / std(A), :127); both
// moments in two fixed-order passes over the resident panel.
//
//   F_new[i, j] = sum_n ((x_new[i, n] - mu) / sd) L[n, j] / |L_j|^2
//   yhat[i]     = sum_k w_new[i, k] beta_k + sum_j F_new[i, j] beta_{q+j}
#include "dfm_common.h"

namespace dfm {

// per panel row: sum of the row's entries (pass 1) or of (x - mu)^2 (pass 2)
__global__ __launch_bounds__(256) void panel_row_moment_kernel(const double *__restrict__ P, int64_t ld, int N,
                                                               const double *__restrict__ mu, double *__restrict__ out) {
  __shared__ double red[256];
  const int t = blockIdx.x, tid = threadIdx.x;
  const double *row = P + (int64_t)t * ld;
  const double m = mu ? *mu : 0.0;
  double a = 0.0;
  for (int c = tid; c < N; c += 256) {
    const double v = row[c] - m;
    a = mu ? fma(v, v, a) : a + row[c];
  }
  red[tid] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) out[t] = red[0];
}

// ordered sum of n partials, scaled: out = scale * sum (one workgroup)
__global__ __launch_bounds__(256) void scaled_sum_kernel(const double *__restrict__ v, int n, double scale,
                                                         double *__restrict__ out) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int i = tid; i < n; i += 256) s += v[i];
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) *out = red[0] * scale;
}

// one workgroup per new row i: F_new[i, :] and (beta != null) yhat[i].
// L row-major N x r (the model's block-0 loadings); x_new column-major
// (n_new x N, leading dimension ldx); w_new column-major (n_new x q, ldw);
// mom = {mu, sum (x - mu)^2}; F_out n_new x r column-major (ld n_new).
__global__ __launch_bounds__(256) void predict_rows_kernel(const double *__restrict__ L, int N, int r,
                                                           const double *__restrict__ x, int64_t ldx, int64_t nn,
                                                           const double *__restrict__ w, int64_t ldw, int q,
                                                           const double *__restrict__ mom, double cnt,
                                                           const double *__restrict__ beta,
                                                           double *__restrict__ F_out, double *__restrict__ yhat) {
  __shared__ double red[256], red2[256];
  const int64_t i = blockIdx.x;
  const int tid = threadIdx.x;
  const double mu = mom[0], sd = sqrt(mom[1] / (cnt - 1.0));
  double acc = 0.0;   // only lane 0's is used
  for (int j = 0; j < r; ++j) {
    double p = 0.0, s2 = 0.0;
    for (int n = tid; n < N; n += 256) {
      const double l = L[(int64_t)n * r + j];
      p = fma((x[i + (int64_t)n * ldx] - mu) / sd, l, p);
      s2 = fma(l, l, s2);
    }
    red[tid] = p;
    red2[tid] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (tid < o) { red[tid] += red[tid + o]; red2[tid] += red2[tid + o]; }
      __syncthreads();
    }
    const double f = red[0] / red2[0];
    if (tid == 0) {
      if (F_out) F_out[i + (int64_t)j * nn] = f;
      if (beta) acc = fma(f, beta[q + j], acc);
    }
    __syncthreads();
  }
  if (tid == 0 && beta) {
    double yh = 0.0;
    for (int k = 0; k < q; ++k) yh = fma(w[i + (int64_t)k * ldw], beta[k], yh);
    yhat[i] = yh + acc;
  }
}

hipError_t launch_predict(const double *Xp, int64_t ld, int T, int N, const double *L, int r, const double *x_dev,
                          int64_t ldx, int64_t nn, const double *w_dev, int64_t ldw, int q, const double *beta_dev,
                          double *work, double *F_out, double *yhat, hipStream_t st) {
  double *part = work, *mom = work + T;   // T partials, {mu, ssq}
  hipLaunchKernelGGL(panel_row_moment_kernel, dim3(T), dim3(256), 0, st, Xp, ld, N, (const double *)nullptr, part);
  hipLaunchKernelGGL(scaled_sum_kernel, dim3(1), dim3(256), 0, st, part, T, 1.0 / ((double)T * N), mom);
  hipLaunchKernelGGL(panel_row_moment_kernel, dim3(T), dim3(256), 0, st, Xp, ld, N, (const double *)mom, part);
  hipLaunchKernelGGL(scaled_sum_kernel, dim3(1), dim3(256), 0, st, part, T, 1.0, mom + 1);
  hipLaunchKernelGGL(predict_rows_kernel, dim3((unsigned)nn), dim3(256), 0, st, L, N, r, x_dev, ldx, nn, w_dev, ldw,
                     q, (const double *)mom, (double)T * N, beta_dev, F_out, yhat);
  return hipGetLastError();
}

}  // namespace dfm
