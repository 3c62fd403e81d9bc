// dfm_spec.hip — the full spectrum (all eigenvalues) of symmetric m x m Grams
// of any size, for what the reference gets from the full `eig` of
// src/DynamicFactorModel.jl:78 / :87 and then reads past the top r:
//   * the PCp criteria's sigma^2 = V(ceil(m/2)) of the unrestricted fit
//     (src/criteria.jl:18, :23, :28), i.e. the tail sum of the spectrum;
//   * IC sweeps with kmax > 24 (src/DynamicFactorModel.jl:54, kmax = ceil(m/2)).
// m <= SPEC_MAX goes to the LDS-resident Jacobi kernel of dfm_eig.hip.
// Larger m: Householder tridiagonalisation (one workgroup per matrix, the
// trailing matrix in HBM, ONE read+write pass per reflector: the previous
// reflector's rank-2 update is applied lazily in the same pass that forms the
// next symmetric product), then Sturm-count bisection on the tridiagonal,
// one thread per eigenvalue.  Both are backward stable: eigenvalues to
// O(eps ||G||), as LAPACK's dsyevr the reference reaches.
#include "dfm_common.h"
#include <algorithm>

namespace dfm {

hipError_t launch_spectrum_jacobi(const double *G, int64_t ldg, int64_t strideG, int m, int m0, int dm, int nb,
                                  double *ev, hipStream_t st);
int spectrum_max();

constexpr int TRI_THREADS = 512;
constexpr int TRI_WAVES = TRI_THREADS / 64;
constexpr int SPEC_ANY_MAX = 4096;   // 4 LDS vectors of m doubles

DFM_DEV double block_sum(double v, double *red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < TRI_WAVES; ++i) s += red[i];
  return s;
}

// Householder reduction G = Q T Q' (LAPACK dsytd2 semantics, lower form).
// Work S: m x m per matrix, row-major upper triangle (S[a][b], b >= a), so
// that column k of the lower triangle — the reflector's source — is the
// contiguous row k.  Outputs d (m) and e (m-1, stored with stride m); with
// tout != nullptr also the reflectors for the eigenvector back-transform:
// v_k over S[k][k+1..m-1] (v_k[k+1] = 1, stored) and tau_k in tout[k].
__global__ __launch_bounds__(TRI_THREADS) void tridiag_kernel(const double *__restrict__ G, int64_t ldg,
                                                              int64_t strideG, int mst, int m0, int dm, int pad,
                                                              double *__restrict__ Sw,
                                                              double *__restrict__ dout,
                                                              double *__restrict__ eout,
                                                              double *__restrict__ tout) {
  extern __shared__ double sm[];
  double *vp = sm, *wp = sm + mst, *v = sm + 2 * mst, *p = sm + 3 * mst;
  __shared__ double red[TRI_WAVES];
  __shared__ double pcol[TRI_WAVES * 128];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rep = blockIdx.x;
  const double *g = G + (int64_t)rep * strideG;
  // this matrix's size m0 + dm * rep (buffers have stride mst); pad: the
  // matrix is the leading (m0 + dm * rep) block zero-padded to mst x mst
  const int mv = m0 + dm * rep, m = pad ? mst : mv;
  double *S = Sw + (int64_t)rep * mst * mst;
  double *d = dout + (int64_t)rep * mst, *e = eout + (int64_t)rep * mst;
  for (int a = wv; a < m; a += TRI_WAVES)
    for (int b = a + lane; b < m; b += 64)
      S[(int64_t)a * m + b] = (a < mv && b < mv) ? 0.5 * (g[(int64_t)a * ldg + b] + g[(int64_t)b * ldg + a]) : 0.0;
  for (int i = tid; i < m; i += TRI_THREADS) { vp[i] = 0.0; wp[i] = 0.0; }
  __syncthreads();
  for (int k = 0; k < m; ++k) {
    // 1. column k with the pending update (vp, wp) of reflector k-1 applied
    const double vpk = vp[k], wpk = wp[k];
    const double *Sk = S + (int64_t)k * m;
    double ss = 0.0;
    for (int i = k + tid; i < m; i += TRI_THREADS) {
      const double c = Sk[i] - vpk * wp[i] - wpk * vp[i];
      v[i] = c;
      if (i > k + 1) ss += c * c;
    }
    const double xn2 = block_sum(ss, red);   // (syncs: v[] visible)
    const double dk = v[k];
    double tau = 0.0, scale = 0.0;
    if (k + 1 < m) {
      const double alpha = v[k + 1];
      double beta = alpha;
      if (xn2 > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
        tau = (beta - alpha) / beta;
        scale = 1.0 / (alpha - beta);
      }
      if (tid == 0) e[k] = beta;
    }
    if (tid == 0) d[k] = dk;
    __syncthreads();
    for (int i = k + 1 + tid; i < m; i += TRI_THREADS) {
      const double vi = (i == k + 1) ? 1.0 : (tau != 0.0 ? v[i] * scale : 0.0);
      v[i] = vi;
      p[i] = 0.0;
      if (tout) S[(int64_t)k * m + i] = vi;   // row k is consumed: keep the reflector there
    }
    if (tout && tid == 0) tout[(int64_t)rep * mst + k] = tau;
    __syncthreads();
    if (k + 1 >= m) break;
    // 2. one pass over the trailing triangle in 128-column panels: apply the
    //    pending rank-2 update, store, and accumulate p = A v in a FIXED order
    //    (bit-reproducible, no float atomics): a row's part by one wave
    //    reduction per (row, panel), added by the row's owning wave in panel
    //    order; the mirrored column part per lane over the wave's rows, summed
    //    over the waves in wave order once the panel is done
    const bool refl = tau != 0.0;
    for (int b0 = (k + 1) & ~127; b0 < m; b0 += 128) {
      const int bA = b0 + lane, bB = b0 + 64 + lane;
      const int alast = min(m - 1, b0 + 127);
      double cA = 0.0, cB = 0.0;
      for (int a = k + 1 + wv; a <= alast; a += TRI_WAVES) {
        const double vpa = vp[a], wpa = wp[a], va = v[a];
        double *Sa = S + (int64_t)a * m;
        double rp = 0.0;
        if (bA >= a && bA < m) {
          const double s = Sa[bA] - (vpa * wp[bA] + wpa * vp[bA]);
          Sa[bA] = s;
          rp = s * v[bA];
          if (bA > a) cA = fma(s, va, cA);
        }
        if (bB >= a && bB < m) {
          const double s = Sa[bB] - (vpa * wp[bB] + wpa * vp[bB]);
          Sa[bB] = s;
          rp = fma(s, v[bB], rp);
          if (bB > a) cB = fma(s, va, cB);
        }
        if (refl) {
          rp = wave_sum(rp);
          if (lane == 0) p[a] += rp;
        }
      }
      if (refl) {
        pcol[wv * 128 + lane] = cA;
        pcol[wv * 128 + 64 + lane] = cB;
      }
      __syncthreads();
      if (refl && tid < 128 && b0 + tid < m) {
        double sum = 0.0;
        for (int w2 = 0; w2 < TRI_WAVES; ++w2) sum += pcol[w2 * 128 + tid];
        p[b0 + tid] += sum;
      }
      __syncthreads();
    }
    // 3. w = tau p - (tau^2/2)(p'v) v becomes the pending update
    double pv = 0.0;
    for (int i = k + 1 + tid; i < m; i += TRI_THREADS) pv += p[i] * v[i];
    pv = block_sum(pv, red) * tau;
    for (int i = k + 1 + tid; i < m; i += TRI_THREADS) {
      const double pi = tau * p[i];
      wp[i] = pi - 0.5 * tau * pv * v[i];
      vp[i] = v[i];
    }
    __syncthreads();
  }
}

// Eigenvalue j (descending) of the symmetric tridiagonal (d, e) by bisection
// on the Sturm count (LAPACK dlaebz's recurrence with its pivmin guard).
// Multisection (Sturm counts at BS_G points per eigenvalue, one per lane of
// a BS_G-lane group): the interval shrinks (BS_G + 1)-fold per count instead
// of 2-fold, so an eigenvalue needs ~13 sequential O(m) counts instead of
// ~53.  Every lane of a group computes the same new interval from the group's
// ballot (no data exchange beyond it): deterministic.  Same tolerance as the
// bisection it replaces: eps * ||T|| (+ 4 pivmin).
constexpr int BS_G = 16;
__global__ __launch_bounds__(256) void bisect_kernel(const double *__restrict__ din,
                                                     const double *__restrict__ ein, int mst, int m0, int dm,
                                                     int nev, double *__restrict__ ev) {
  extern __shared__ double sm[];
  const int tid = threadIdx.x, rep = blockIdx.y;
  const int m = m0 + dm * rep;   // nev == 0: all m of this matrix
  if (nev <= 0) nev = m;
  double *d = sm, *e2 = sm + m;
  __shared__ double bnd[2];
  const double *dg = din + (int64_t)rep * mst, *eg = ein + (int64_t)rep * mst;
  for (int i = tid; i < m; i += 256) {
    d[i] = dg[i];
    e2[i] = (i + 1 < m) ? eg[i] * eg[i] : 0.0;
  }
  __syncthreads();
  if (tid == 0) {   // Gershgorin interval, pivmin
    double lo = 1e308, hi = -1e308, emax = 0.0;
    for (int i = 0; i < m; ++i) {
      const double r = (i > 0 ? fabs(eg[i - 1]) : 0.0) + (i + 1 < m ? fabs(eg[i]) : 0.0);
      lo = fmin(lo, d[i] - r);
      hi = fmax(hi, d[i] + r);
      if (i + 1 < m) emax = fmax(emax, e2[i]);
    }
    const double nrm = fmax(fabs(lo), fabs(hi));
    lo -= 2.2e-16 * nrm * m + 1e-300;
    hi += 2.2e-16 * nrm * m + 1e-300;
    bnd[0] = lo; bnd[1] = hi;
    e2[m] = fmax(2.2e-308, emax * 2.2e-308);   // pivmin (slot m: LDS holds 2m+1)
  }
  __syncthreads();
  const int g = tid % BS_G, j = blockIdx.x * (256 / BS_G) + tid / BS_G;
  const bool live = j < nev;   // the whole group agrees (j is per group)
  const double pivmin = e2[m];
  const int kth = m - 1 - (live ? j : 0);   // ascending index of eigenvalue j (descending)
  double lo = bnd[0], hi = bnd[1];
  // absolute accuracy eps * ||T||: what the reduction itself guarantees
  const double tol = 2.2e-16 * fmax(fabs(lo), fabs(hi));
  const int gshift = (threadIdx.x & 63) & ~(BS_G - 1);
  for (int it = 0; it < 64; ++it) {
    if (hi - lo <= tol + 4.0 * pivmin) break;   // group-uniform
    const double w = (hi - lo) / (BS_G + 1);
    const double x = lo + w * (g + 1);
    // number of eigenvalues < x
    int cnt = 0;
    double q = d[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < m; ++i) {
      q = d[i] - x - e2[i - 1] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    // first point above eigenvalue kth: lanes with cnt > kth
    const unsigned long long above = (__ballot(cnt > kth) >> gshift) & ((1ull << BS_G) - 1);
    const int gs = above ? __builtin_ctzll(above) : BS_G;
    const double nlo = gs > 0 ? lo + w * gs : lo;
    const double nhi = gs < BS_G ? lo + w * (gs + 1) : hi;
    if (!(nlo > lo || nhi < hi)) break;   // no representable progress
    lo = fmax(lo, nlo);
    hi = fmin(hi, nhi);
  }
  if (live && g == 0) ev[(int64_t)rep * (dm ? mst : nev) + j] = 0.5 * (lo + hi);
}

// Jacobi (LDS-resident, 1 WG per CU) only for small matrices: from m ~ 40 on
// the tridiagonal path's O(m) barriers beat Jacobi's O(sweeps * m).
constexpr int JACOBI_MAX = 32;
int64_t spectrum_work(int m, int nb) {
  if (m <= JACOBI_MAX) return 0;
  return (int64_t)nb * m * m + 2 * (int64_t)nb * m;
}
int spectrum_any_max() { return SPEC_ANY_MAX; }

// Tridiagonal form (d, e) only, for m <= TRI_LDS_MAX: the whole symmetric
// matrix resident in LDS (row stride m + 1), LAPACK dsytd2 (lower) step by
// step: reflector of column k, p = tau A22 v with one thread per row (no
// cross-lane reductions per row), w = p - (tau/2)(p'v) v, A22 -= v w' + w v'.
// Single fits (C1's PCp sigma^2, m = 100): 529 -> 477 us per matrix — the
// step sequence (two block reductions and three barriers per reflector), not
// the memory level, bounds both forms.
constexpr int TRI_LDS_MAX = 128;
constexpr int TRL_THREADS = 256;
DFM_DEV double trl_sum(double v, double *red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < TRL_THREADS / 64; ++i) s += red[i];
  return s;
}
__global__ __launch_bounds__(TRL_THREADS) void tridiag_lds_kernel(const double *__restrict__ G, int64_t ldg,
                                                                  int64_t strideG, int mst, int m0, int dm,
                                                                  double *__restrict__ dout,
                                                                  double *__restrict__ eout) {
  extern __shared__ double sm[];
  __shared__ double red[TRL_THREADS / 64];
  const int tid = threadIdx.x, rep = blockIdx.x;
  const int m = m0 + dm * rep, S = m + 1;
  double *A = sm, *v = A + (size_t)m * S, *p = v + m;
  const double *g = G + (int64_t)rep * strideG;
  double *d = dout + (int64_t)rep * mst, *e = eout + (int64_t)rep * mst;
  for (int x = tid; x < m * m; x += TRL_THREADS) {
    const int a = x / m, b = x - a * m;
    A[a * S + b] = 0.5 * (g[(int64_t)a * ldg + b] + g[(int64_t)b * ldg + a]);
  }
  __syncthreads();
  for (int k = 0; k + 1 < m; ++k) {
    double ss = 0.0;
    for (int i = k + 2 + tid; i < m; i += TRL_THREADS) ss += A[i * S + k] * A[i * S + k];
    const double xn2 = trl_sum(ss, red);
    const double alpha = A[(k + 1) * S + k];
    double beta = alpha, tau = 0.0, scale = 0.0;
    if (xn2 > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
      tau = (beta - alpha) / beta;
      scale = 1.0 / (alpha - beta);
    }
    if (tid == 0) { d[k] = A[k * S + k]; e[k] = beta; }
    for (int i = k + 1 + tid; i < m; i += TRL_THREADS) v[i] = i == k + 1 ? 1.0 : A[i * S + k] * scale;
    __syncthreads();
    if (tau == 0.0) continue;   // column already reduced (uniform)
    double pv = 0.0;
    for (int a = k + 1 + tid; a < m; a += TRL_THREADS) {
      double acc = 0.0;
      for (int b = k + 1; b < m; ++b) acc = fma(A[a * S + b], v[b], acc);
      acc *= tau;
      p[a] = acc;
      pv += acc * v[a];
    }
    const double K = 0.5 * tau * trl_sum(pv, red);   // (syncs: p visible)
    for (int a = k + 1 + tid; a < m; a += TRL_THREADS) p[a] -= K * v[a];   // w
    __syncthreads();
    const int n2 = m - k - 1;
    for (int x = tid; x < n2 * n2; x += TRL_THREADS) {
      const int a = k + 1 + x / n2, b = k + 1 + x % n2;
      A[a * S + b] -= v[a] * p[b] + p[a] * v[b];
    }
    __syncthreads();
  }
  if (tid == 0) d[m - 1] = A[(m - 1) * S + m - 1];
}

// All eigenvalues (descending) of nb symmetric matrices G + rep * strideG;
// matrix rep has size m0 + dm * rep <= m (dm = 0: all m x m), ev rows stride m.
// work: spectrum_work(m, nb) doubles (none for m <= SPEC_MAX).
hipError_t launch_spectrum_var(const double *G, int64_t ldg, int64_t strideG, int m, int m0, int dm, int nb,
                               double *ev, double *work, hipStream_t st) {
  if (m0 < 1 || nb < 1 || dm < 0 || m0 + (int64_t)dm * (nb - 1) > m) return hipErrorInvalidValue;
  if (m <= JACOBI_MAX) return launch_spectrum_jacobi(G, ldg, strideG, m, m0, dm, nb, ev, st);
  if (m > SPEC_ANY_MAX || !work) return hipErrorInvalidValue;
  double *S = work, *d = work + (int64_t)nb * m * m, *e = d + (int64_t)nb * m;
  // the dynamic-LDS attribute is per device: set it on every call (cheap)
  const bool lds_attr = hipFuncSetAttribute((const void *)tridiag_lds_kernel,
                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (TRI_LDS_MAX * (TRI_LDS_MAX + 1) + 2 * TRI_LDS_MAX) * 8) == hipSuccess;
  // the LDS form holds one workgroup per CU: only when the matrices do not
  // outnumber the CUs (single fits); large batches keep the global-memory form
  if (m <= TRI_LDS_MAX && nb <= 256 && lds_attr)
    hipLaunchKernelGGL(tridiag_lds_kernel, dim3(nb), dim3(TRL_THREADS), (size_t)(m * (m + 1) + 2 * m) * sizeof(double),
                       st, G, ldg, strideG, m, m0, dm, d, e);
  else
    hipLaunchKernelGGL(tridiag_kernel, dim3(nb), dim3(TRI_THREADS), (size_t)4 * m * sizeof(double), st, G, ldg,
                       strideG, m, m0, dm, 0, S, d, e, (double *)nullptr);
  hipLaunchKernelGGL(bisect_kernel, dim3((m * BS_G + 255) / 256, nb), dim3(256), (size_t)(2 * m + 1) * sizeof(double),
                     st, d, e, m, m0, dm, 0, ev);
  return hipGetLastError();
}
hipError_t launch_spectrum(const double *G, int64_t ldg, int64_t strideG, int m, int nb, double *ev,
                           double *work, hipStream_t st) {
  return launch_spectrum_var(G, ldg, strideG, m, m, 0, nb, ev, work, st);
}

// ------------------------------------------------ dense top-k eigenpairs
// For k beyond the subspace eigensolver's block (k > 24; the reference's r
// may be anything up to ceil(m/2), src/DynamicFactorModel.jl:101, :116-119):
// tridiagonalise (reflectors kept), bisect the top k eigenvalues, then
//  1. inverse iteration on the tridiagonal, ONE THREAD PER EIGENVECTOR (LAPACK
//     dstein's partial-pivoting LU of T - sigma I with perturbed tiny pivots;
//     near-equal shifts separated by 10 eps ||T||; distinct pseudo-random
//     starts, so a (near-)degenerate cluster yields independent vectors of its
//     invariant subspace), LU and vectors interleaved [i * k + j] so a wave's
//     serial recurrences read coalesced rows;
//  2. orthonormalisation in eigenvalue order by block classical Gram-Schmidt
//     with re-orthogonalisation (BCGS2) and CholQR2 inside 32-column blocks,
//     all as strided GEMMs: every overlap it removes is O(eps ||T|| / gap), the
//     accuracy any backward-stable solver has;
//  3. U = H_0 H_1 ... H_{m-3} Z.
constexpr int SPEC_VEC_MAX = 4096;
constexpr int OB = 32;   // orthonormalisation block

hipError_t gemm_batched(int nb, int M, int Nc, int K, double alpha, const double *A, int64_t sAr, int64_t sAc,
                        int64_t sAb, const double *B, int64_t sBr, int64_t sBc, int64_t sBb, double beta, double *C,
                        int64_t sCr, int64_t sCc, int64_t sCb, hipStream_t st);

// ||T||_inf, and the shifts: sigma_j = lambda_j, pushed down so consecutive
// shifts differ by >= 10 eps ||T|| (dstein's perturbation of close shifts)
__global__ void stein_shifts_kernel(const double *__restrict__ db, const double *__restrict__ eb, int m,
                                    const double *__restrict__ lamb, int k, double *__restrict__ sigb,
                                    double *__restrict__ tnb) {
  if (threadIdx.x != 0) return;
  const int rep = blockIdx.x;
  const double *d = db + (int64_t)rep * m, *e = eb + (int64_t)rep * m, *lam = lamb + (int64_t)rep * k;
  double *sig = sigb + (int64_t)rep * k, *tn = tnb + rep;
  double nrm = 0.0;
  for (int i = 0; i < m; ++i)
    nrm = fmax(nrm, fabs(d[i]) + (i + 1 < m ? fabs(e[i]) : 0.0) + (i > 0 ? fabs(e[i - 1]) : 0.0));
  const double pertol = 10.0 * 2.2e-16 * nrm;
  double prev = 0.0;
  for (int j = 0; j < k; ++j) {
    double x = lam[j];
    if (j > 0 && x > prev - pertol) x = prev - pertol;
    sig[j] = x;
    prev = x;
  }
  *tn = nrm;
}

__global__ __launch_bounds__(64) void invit_kernel(const double *__restrict__ db, const double *__restrict__ eb,
                                                   int m, int k, const double *__restrict__ sigb,
                                                   const double *__restrict__ tnb, double *__restrict__ uab,
                                                   double *__restrict__ ubb, double *__restrict__ ucb,
                                                   double *__restrict__ udb, unsigned char *__restrict__ pivb,
                                                   double *__restrict__ Zb) {
  const int j = blockIdx.x * 64 + threadIdx.x, rep = blockIdx.y;
  if (j >= k) return;
  const int64_t mk = (int64_t)m * k;
  const double *d = db + (int64_t)rep * m, *e = eb + (int64_t)rep * m, *sig = sigb + (int64_t)rep * k,
               *tn = tnb + rep;
  double *ua = uab + rep * mk, *ub = ubb + rep * mk, *uc = ucb + rep * mk, *ud = udb + rep * mk, *Z = Zb + rep * mk;
  unsigned char *piv = pivb + rep * mk;
  const double xj = sig[j], tiny = 2.2e-16 * *tn;
#define IX(i) ((int64_t)(i) * k + j)
  for (int i = 0; i < m; ++i) { ua[IX(i)] = d[i] - xj; ub[IX(i)] = (i + 1 < m) ? e[i] : 0.0; ud[IX(i)] = 0.0; }
  for (int i = 0; i + 1 < m; ++i) {
    const double a = ua[IX(i)], c = e[i];
    if (fabs(a) >= fabs(c)) {
      const double aa = fabs(a) < tiny ? copysign(tiny, a) : a;
      const double mult = c / aa;
      ua[IX(i)] = aa;
      uc[IX(i)] = mult;
      ua[IX(i + 1)] -= mult * ub[IX(i)];
      piv[IX(i)] = 0;
    } else {
      const double mult = a / c;
      const double t = ua[IX(i + 1)];
      ua[IX(i)] = c;
      ua[IX(i + 1)] = ub[IX(i)] - mult * t;
      if (i + 2 < m) { const double b1 = ub[IX(i + 1)]; ud[IX(i)] = b1; ub[IX(i + 1)] = -mult * b1; }
      ub[IX(i)] = t;
      uc[IX(i)] = mult;
      piv[IX(i)] = 1;
    }
  }
  for (int i = 0; i < m; ++i) {
    const double a = ua[IX(i)];
    if (fabs(a) < tiny) ua[IX(i)] = copysign(tiny, a);
  }
  double nn = 0.0;
  for (int i = 0; i < m; ++i) { const double v = hash_unit(0x5eed, (uint64_t)j, (uint64_t)i); Z[IX(i)] = v; nn += v * v; }
  double sc = 1.0 / sqrt(nn);
  for (int it = 0; it < 3; ++it) {
    // forward: the row interchanges and multipliers of L
    double xi = Z[IX(0)] * sc;
    for (int i = 0; i + 1 < m; ++i) {
      const double xn = Z[IX(i + 1)] * sc;
      double a, b;
      if (piv[IX(i)]) { a = xn; b = xi - uc[IX(i)] * xn; }
      else { a = xi; b = xn - uc[IX(i)] * xi; }
      Z[IX(i)] = a;
      xi = b;
    }
    Z[IX(m - 1)] = xi;
    // back substitution with U (diagonal ua, superdiagonals ub, ud)
    double x1 = Z[IX(m - 1)] / ua[IX(m - 1)], x2 = 0.0;
    Z[IX(m - 1)] = x1;
    nn = x1 * x1;
    for (int i = m - 2; i >= 0; --i) {
      const double x0 = (Z[IX(i)] - ub[IX(i)] * x1 - ud[IX(i)] * x2) / ua[IX(i)];
      Z[IX(i)] = x0;
      nn += x0 * x0;
      x2 = x1; x1 = x0;
    }
    sc = 1.0 / sqrt(nn);
  }
  for (int i = 0; i < m; ++i) Z[IX(i)] *= sc;
#undef IX
}

// CholQR step on a b-column block: W = R'R (Cholesky, b <= OB), Rinv = R^-1.
__global__ void small_chol_inv_kernel(const double *__restrict__ Wb, int b, double *__restrict__ Rinvb,
                                      int *__restrict__ status) {
  __shared__ double R[OB][OB + 1], X[OB][OB + 1];
  const int tid = threadIdx.x, rep = blockIdx.x;
  const double *W = Wb + (int64_t)rep * OB * OB;
  double *Rinv = Rinvb + (int64_t)rep * OB * OB;
  for (int e = tid; e < OB * OB; e += blockDim.x) {
    const int a = e / OB, c = e % OB;
    R[a][c] = (a < b && c < b) ? W[a * b + c] : 0.0;
    X[a][c] = 0.0;
  }
  __syncthreads();
  if (tid == 0) {
    int bad = 0;
    for (int j = 0; j < b; ++j) {   // upper R: W = R'R
      double s = R[j][j];
      for (int p = 0; p < j; ++p) s -= R[p][j] * R[p][j];
      if (!(s > 0.0)) { bad = 1; s = 1.0; }
      R[j][j] = sqrt(s);
      for (int c = j + 1; c < b; ++c) {
        double t = R[j][c];
        for (int p = 0; p < j; ++p) t -= R[p][j] * R[p][c];
        R[j][c] = t / R[j][j];
      }
    }
    for (int c = 0; c < b; ++c)   // X = R^-1 (upper), column by column
      for (int i = c; i >= 0; --i) {
        double t = (i == c) ? 1.0 : 0.0;
        for (int p = i + 1; p <= c; ++p) t -= R[i][p] * X[p][c];
        X[i][c] = t / R[i][i];
      }
    if (bad) status[rep] = 1;
  }
  __syncthreads();
  for (int e = tid; e < b * b; e += blockDim.x) Rinv[e] = X[e / b][e % b];
}

__global__ void copy_cols_kernel(const double *__restrict__ srcb, int b, int m, double *__restrict__ Zb, int k,
                                 int j0) {
  const int rep = blockIdx.y;
  const double *src = srcb + (int64_t)rep * m * OB;
  double *Z = Zb + (int64_t)rep * m * k;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < (int64_t)m * b; e += (int64_t)gridDim.x * 256)
    Z[(e / b) * k + j0 + e % b] = src[e];
}

// U(:, j) = H_0 H_1 ... H_{m-3} z_j, one workgroup per vector; then the sign
// convention of eig_final_kernel (largest |entry|, first on ties, positive)
// and the m x k row-major layout of the subspace eigensolver's output.
__global__ __launch_bounds__(256) void backtransform_kernel(const double *S, const double *taus,
                                                            const double *__restrict__ Z, int m, int k,
                                                            double *__restrict__ Uk) {
  extern __shared__ double x[];
  __shared__ double red[4];
  __shared__ int redi[4];
  const int tid = threadIdx.x, j = blockIdx.x, rep = blockIdx.y;
  S += (int64_t)rep * m * m;
  taus += (int64_t)rep * m;
  Z += (int64_t)rep * m * k;
  Uk += (int64_t)rep * m * k;
  for (int i = tid; i < m; i += 256) x[i] = Z[(int64_t)i * k + j];
  __syncthreads();
  for (int q = m - 3; q >= 0; --q) {
    const double tau = taus[q];
    if (tau == 0.0) continue;
    const double *v = S + (int64_t)q * m;
    double s = 0.0;
    for (int i = q + 1 + tid; i < m; i += 256) s += v[i] * x[i];
    s = wave_sum(s);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    s = tau * (red[0] + red[1] + red[2] + red[3]);
    for (int i = q + 1 + tid; i < m; i += 256) x[i] -= s * v[i];
    __syncthreads();
  }
  double best = -1.0;
  int bi = 0;
  for (int i = tid; i < m; i += 256)
    if (fabs(x[i]) > best) { best = fabs(x[i]); bi = i; }
  for (int o = 32; o >= 1; o >>= 1) {
    const double ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if ((tid & 63) == 0) { red[tid >> 6] = best; redi[tid >> 6] = bi; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (red[w] > red[0] || (red[w] == red[0] && redi[w] < redi[0])) { red[0] = red[w]; redi[0] = redi[w]; }
  }
  __syncthreads();
  const double sg = x[redi[0]] < 0.0 ? -1.0 : 1.0;
  for (int i = tid; i < m; i += 256) Uk[(int64_t)i * k + j] = sg * x[i];
}

__global__ void diag_sum_kernel(const double *__restrict__ G, int64_t ldg, int64_t strideG, int m0, int dm,
                                double *__restrict__ trb) {
  const int rep = blockIdx.x, m = m0 + dm * rep;
  G += (int64_t)rep * strideG;
  double *tr = trb + rep;
  double s = 0.0;
  for (int i = threadIdx.x; i < m; i += 256) s += G[(int64_t)i * ldg + i];
  s = wave_sum(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *tr = red[0] + red[1] + red[2] + red[3];
}

int dense_eig_max() { return SPEC_VEC_MAX; }
int64_t dense_eig_work(int m, int k) {   // per matrix
  return (int64_t)m * m + 3 * (int64_t)m + 8 + 5 * (int64_t)m * k + ((int64_t)m * k + 7) / 8 + 2 * (int64_t)k +
         (int64_t)k * OB + 2 * OB * OB + (int64_t)m * OB;
}

// Top-k eigenpairs of nb symmetric matrices G + rep * strideG, each the
// leading (mv0 + dmv * rep) block zero-padded to m x m (dmv = 0, mv0 = m: plain
// m x m).  lam: nb x k, Uk: nb x m x k (row-major m x k each), trace: nb (of
// the valid block), status: nb (1 = an orthonormalisation block numerically
// rank deficient).  work: nb * dense_eig_work(m, k) doubles.
hipError_t launch_dense_eig_batched(const double *G, int64_t ldg, int64_t strideG, int m, int mv0, int dmv, int nb,
                                    int k, double *lam, double *Uk, double *trace, int *status, double *work,
                                    hipStream_t st) {
  if (m < 2 || m > SPEC_VEC_MAX || k < 1 || k > m || nb < 1 || !work || !status) return hipErrorInvalidValue;
  const int64_t mk = (int64_t)m * k;
  double *S = work, *d = S + nb * (int64_t)m * m, *e = d + (int64_t)nb * m, *taus = e + (int64_t)nb * m;
  double *tn = taus + (int64_t)nb * m, *ua = tn + 8 * (int64_t)nb, *ub = ua + nb * mk, *uc = ub + nb * mk;
  double *ud = uc + nb * mk, *Z = ud + nb * mk;
  unsigned char *piv = (unsigned char *)(Z + nb * mk);
  double *sig = Z + nb * mk + (nb * mk + 7) / 8, *Sm = sig + 2 * (int64_t)nb * k, *W = Sm + (int64_t)nb * k * OB;
  double *Ri = W + (int64_t)nb * OB * OB, *Tmp = Ri + (int64_t)nb * OB * OB;
  const int pad = (dmv != 0 || mv0 != m) ? 1 : 0;
  hipLaunchKernelGGL(tridiag_kernel, dim3(nb), dim3(TRI_THREADS), (size_t)4 * m * sizeof(double), st, G, ldg,
                     strideG, m, mv0, dmv, pad, S, d, e, taus);
  hipLaunchKernelGGL(bisect_kernel, dim3((k * BS_G + 255) / 256, nb), dim3(256), (size_t)(2 * m + 1) * sizeof(double),
                     st, d, e, m, m, 0, k, lam);
  hipLaunchKernelGGL(stein_shifts_kernel, dim3(nb), dim3(64), 0, st, d, e, m, lam, k, sig, tn);
  hipLaunchKernelGGL(invit_kernel, dim3((k + 63) / 64, nb), dim3(64), 0, st, d, e, m, k, sig, tn, ua, ub, uc, ud, piv,
                     Z);
  hipError_t er = hipMemsetAsync(status, 0, sizeof(int) * nb, st);
  if (er != hipSuccess) return er;
  // BCGS2 + CholQR2 in eigenvalue order; Z(i, j) = Z[i * k + j]
  const int64_t sS = (int64_t)k * OB, sW = OB * OB, sT = (int64_t)m * OB;
  for (int j0 = 0; j0 < k; j0 += OB) {
    const int b = std::min(OB, k - j0);
    double *Bj = Z + j0;
    for (int pass = 0; pass < 2 && j0 > 0; ++pass) {
      if ((er = gemm_batched(nb, j0, b, m, 1.0, Z, 1, k, mk, Bj, k, 1, mk, 0.0, Sm, b, 1, sS, st)) != hipSuccess)
        return er;
      if ((er = gemm_batched(nb, m, b, j0, -1.0, Z, k, 1, mk, Sm, b, 1, sS, 1.0, Bj, k, 1, mk, st)) != hipSuccess)
        return er;
    }
    for (int pass = 0; pass < 2; ++pass) {
      if ((er = gemm_batched(nb, b, b, m, 1.0, Bj, 1, k, mk, Bj, k, 1, mk, 0.0, W, b, 1, sW, st)) != hipSuccess)
        return er;
      hipLaunchKernelGGL(small_chol_inv_kernel, dim3(nb), dim3(64), 0, st, W, b, Ri, status);
      if ((er = gemm_batched(nb, m, b, b, 1.0, Bj, k, 1, mk, Ri, b, 1, sW, 0.0, Tmp, b, 1, sT, st)) != hipSuccess)
        return er;
      hipLaunchKernelGGL(copy_cols_kernel, dim3(std::min(1024, (m * b + 255) / 256), nb), dim3(256), 0, st, Tmp, b, m,
                         Z, k, j0);
    }
  }
  hipLaunchKernelGGL(backtransform_kernel, dim3(k, nb), dim3(256), (size_t)m * sizeof(double), st, S, taus, Z, m, k,
                     Uk);
  if (trace)
    hipLaunchKernelGGL(diag_sum_kernel, dim3(nb), dim3(256), 0, st, G, ldg, strideG, mv0, dmv, trace);
  return hipGetLastError();
}
hipError_t launch_dense_eig(const double *G, int64_t ldg, int m, int k, double *lam, double *Uk, double *trace,
                            int *status, double *work, hipStream_t st) {
  return launch_dense_eig_batched(G, ldg, 0, m, m, 0, 1, k, lam, Uk, trace, status, work, st);
}

}  // namespace dfm
