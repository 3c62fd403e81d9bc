// dfm_soft.hip — soft-threshold targeted predictors: the glmnetcv lasso path.
//
// Replaces src/targeted_predictors.jl:31-36 (GLMNet.glmnetcv(Z, y) on
// Z = [w x], keep the x columns whose coefficient at the CV-optimal lambda is
// nonzero).  GLMNet is never imported by the reference (defect D5); the
// algorithm is glmnet's gaussian lasso (Friedman, Hastie & Tibshirani 2010),
// the same restatement the parity tests' CPU checker holds: standardised coordinate descent with covariance
// updates on the active set, KKT scan appending violators in index order,
// warm starts along the lambda grid, early path exit on the full fit.
//
// Device work per call, K folds + the full fit = K + 1 "problems":
//   soft_stats_kernel   per (problem, column): training-row mean / population
//                       sd / constant flag (two passes), the standardised
//                       panel of every problem stacked in one tall panel, and
//                       c = Zs'ys / n                          (HBM-bound)
//   gram_kernel (K1)    G_f = Zs_f' Zs_f over each problem's training rows,
//                       gathered by row index (zero row pads ragged folds):
//                       (K+1) p^2 n MACs on MFMA              (MFMA-bound)
//   lasso_path_kernel   one workgroup per problem: the whole lambda path in
//                       one launch; g_A updates against an LDS-cached G_AA
//                       (latency-bound: sequential coordinate updates)
//   soft_loss_kernel    hold-out SSE per (fold, lambda)        (HBM-bound)
#include "dfm_common.h"
#include "../../include/dfm.h"
#include <algorithm>
#include <cmath>
#include <vector>

namespace dfm {
hipError_t launch_gram(int orient, const PanelSrc &src, int m, int K, int T, double *G, int64_t ldg,
                       int64_t strideG, int nrep, hipStream_t st);
__global__ void panel_from_colmajor_kernel(const double *, int64_t, int, int, double *, int64_t);

constexpr int LS_AMAX = 1024;   // active-set capacity (glmnet's pmax analogue)
constexpr int LS_GC = 126;      // G_AA cached in LDS while the active set is this small (124 KB of the 160)
// development timing of lasso_path_kernel phases (DFM_SOFT_PROF=1): problem
// 0's thread 0 accumulates s_memrealtime ticks (100 MHz) per phase
__device__ unsigned long long g_soft_prof[8];
#define SPROF_START() unsigned long long sp_t0 = wall_clock64()
#define SPROF(i) do { if (f == 0 && tid == 0) { const unsigned long long sp_t1 = wall_clock64(); g_soft_prof[i] += sp_t1 - sp_t0; sp_t0 = sp_t1; } } while (0)

// y mean / population sd over each problem's training rows (fold != f; f = 0: all).
__global__ void soft_ystats_kernel(const double *__restrict__ y, const int32_t *__restrict__ fold, int n,
                                   int nprob, double *__restrict__ ystat) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nprob) return;
  double s = 0.0;
  int nf = 0;
  for (int i = 0; i < n; ++i)
    if (fold[i] != f) { s += y[i]; ++nf; }
  const double yb = s / nf;
  double v = 0.0;
  for (int i = 0; i < n; ++i)
    if (fold[i] != f) { const double d = y[i] - yb; v = fma(d, d, v); }
  ystat[3 * f + 0] = yb;
  ystat[3 * f + 1] = sqrt(v / nf);
  ystat[3 * f + 2] = (double)nf;
}

// Column statistics and the standardised stacked panel.  Problem f's rows
// occupy rows f*(n+1) .. f*(n+1)+n of Zs (row n of each block stays zero:
// the pad target of the ragged training-row gather).  Every row of a block
// is standardised with the problem's training statistics (hold-out rows are
// read by the loss kernel).
__global__ void soft_stats_kernel(const double *__restrict__ Z, int64_t ld, int n, int p,
                                  const double *__restrict__ y, const int32_t *__restrict__ fold,
                                  const double *__restrict__ ystat, double *__restrict__ Zs,
                                  double *__restrict__ mu, double *__restrict__ sd,
                                  uint8_t *__restrict__ ju, double *__restrict__ c) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, f = blockIdx.y;
  if (j >= p) return;
  const double nf = ystat[3 * f + 2], yb = ystat[3 * f + 0], ys = ystat[3 * f + 1];
  double s = 0.0, lo = INFINITY, hi = -INFINITY;
  for (int i = 0; i < n; ++i)
    if (fold[i] != f) {
      const double v = Z[(int64_t)i * ld + j];
      s += v; lo = fmin(lo, v); hi = fmax(hi, v);
    }
  const double m = s / nf;
  double v2 = 0.0;
  for (int i = 0; i < n; ++i)
    if (fold[i] != f) { const double d = Z[(int64_t)i * ld + j] - m; v2 = fma(d, d, v2); }
  const bool keep = hi > lo;                    // glmnet chkvars: constant columns excluded
  const double sdv = keep ? sqrt(v2 / nf) : 1.0;
  double cy = 0.0;
  double *Zf = Zs + (int64_t)f * (n + 1) * ld;
  for (int i = 0; i < n; ++i) {
    const double z = keep ? (Z[(int64_t)i * ld + j] - m) / sdv : 0.0;
    Zf[(int64_t)i * ld + j] = z;
    if (fold[i] != f) cy = fma(z, (y[i] - yb) / ys, cy);
  }
  mu[(int64_t)f * p + j] = m;
  sd[(int64_t)f * p + j] = sdv;
  ju[(int64_t)f * p + j] = keep ? 1 : 0;
  c[(int64_t)f * p + j] = cy / nf;
}

// G_f /= n_f (the Gram kernel leaves Zs_f' Zs_f)
__global__ void soft_scale_kernel(double *__restrict__ G, int64_t strideG, int64_t count,
                                  const double *__restrict__ ystat) {
  const int f = blockIdx.y;
  const double inv = 1.0 / ystat[3 * f + 2];
  double *Gf = G + (int64_t)f * strideG;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (int64_t)gridDim.x * blockDim.x)
    Gf[e] *= inv;
}

// One workgroup per problem: the lasso path over lambdas alm[0..nlam-1]
// (standardised units), warm-started, by coordinate descent on the active
// set.  Per pass the active list is walked in entry order (the serial
// dependency of coordinate descent) and every coordinate change applied to
// g_A (wave 0 alone while G_AA sits in LDS, else all threads); after a converged pass the non-active
// gradients are refreshed with the pass's accumulated changes (rows of G for
// the active variables, coalesced along j) and the KKT scan appends every
// violator |g_j| > lambda in index order.  status[f]: 0 ok, 1 no convergence,
// 2 active set over LS_AMAX; status[nprob + f]: the lambda index of the failure.
// early = 1: problem 0 (the full fit) applies glmnet's early path exit and
// publishes its path length in nlam_out[0] (zeroed before the launch); the
// other problems stop when they reach it.
__global__ __launch_bounds__(256) void lasso_path_kernel(
    const double *__restrict__ Gall, int64_t strideG, int p, const double *__restrict__ call,
    const uint8_t *__restrict__ juall, const double *__restrict__ almall, int nlam, int prob0, int early, int cdmode,
    double thr, int maxit, double *__restrict__ gws, int *__restrict__ actws, double *__restrict__ gaaws,
    double *__restrict__ bpath,
    double *__restrict__ rsq_out, int *__restrict__ nlam_out, int *__restrict__ status) {
  const int f = prob0 + blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double *G = Gall + (int64_t)f * strideG;
  const double *c = call + (int64_t)f * p;
  const uint8_t *ju = juall + (int64_t)f * p;
  const double *alm = almall + (int64_t)f * nlam;
  double *g = gws + (int64_t)f * p;
  int *act = actws + (int64_t)f * p;
  // G_AA compacted in entry order (row stride LS_AMAX) for active sets past
  // LS_GC: one coalesced 8 na-byte row per coordinate step instead of a
  // gather that touches nearly every cache line of a p-wide G row
  double *GAA = gaaws + (int64_t)f * LS_AMAX * LS_AMAX;
  double *bp = bpath + (int64_t)f * nlam * p;
  __shared__ int ia[LS_AMAX], rows[LS_AMAX];
  __shared__ double bA[LS_AMAX], gA[LS_AMAX], dA[LS_AMAX];
  __shared__ double GC[LS_GC * LS_GC];
  __shared__ double s_red[4];
  __shared__ int s_flag, s_cnt[4];
  for (int j = tid; j < p; j += 256) { g[j] = c[j]; act[j] = 0; }
  __syncthreads();
  int na = 0, L = nlam, st = 0, fail_m = nlam;
  double rsq_prev = 0.0;
  for (int m = 0; m < nlam && !st; ++m) {
    const double lam = alm[m];
    for (;;) {
      SPROF_START();
      // ---- passes over the active set until max delta^2 < thr
      // Small active sets (G_AA cached in LDS): wave 0 alone runs the passes —
      // every lane reads gA[k], bA[k] (an LDS broadcast) and computes the same
      // d, so no cross-wave barrier per coordinate; the wave's LDS accesses
      // complete in program order and the wavefront fences keep the compiler
      // from reordering them across steps.  Larger sets (G_AA rows gathered
      // from HBM) keep all four waves on the update, thread 0 broadcasting d.
      // Same arithmetic in the same order either way.
      int it = 0;
      if (na <= LS_GC) {
        if (wave == 0) {
          for (; it < maxit; ++it) {
            double dlx = 0.0;
            for (int k = 0; k < na; ++k) {
              const double bk = bA[k];
              const double u = gA[k] + bk, v = fabs(u) - lam;
              const double nb = v > 0.0 ? copysign(v, u) : 0.0;
              const double d = nb - bk;
              if (d != 0.0) {   // uniform over the wave
                dlx = fmax(dlx, d * d);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) { bA[k] = nb; dA[k] += d; }
                for (int t = lane; t < na; t += 64) gA[t] -= GC[k * LS_GC + t] * d;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
              }
            }
            if (dlx < thr) break;
          }
          if (lane == 0) s_flag = it;
        }
        __syncthreads();
        it = s_flag;
        __syncthreads();
      } else if (cdmode == 1) {
        if (wave == 0) {
          for (; it < maxit; ++it) {
            double dlx = 0.0;
            for (int k = 0; k < na; ++k) {
              const double bk = bA[k];
              const double u = gA[k] + bk, v = fabs(u) - lam;
              const double nb = v > 0.0 ? copysign(v, u) : 0.0;
              const double d = nb - bk;
              if (d != 0.0) {   // uniform over the wave
                dlx = fmax(dlx, d * d);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) { bA[k] = nb; dA[k] += d; }
                const double *Gk = GAA + (int64_t)k * LS_AMAX;
                for (int t = lane; t < na; t += 64)
                  gA[t] -= __hip_atomic_load(Gk + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * d;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
              }
            }
            if (dlx < thr) break;
          }
          if (lane == 0) s_flag = it;
        }
        __syncthreads();
        it = s_flag;
        __syncthreads();
      } else if (cdmode == 0) {
        // all four waves; row k + 1 of G_AA prefetched into registers (4 per
        // thread: na <= LS_AMAX = 1024) while step k runs — it does not
        // depend on d — so a step waits on no global-memory latency
        constexpr int RV = LS_AMAX / 256;
        for (; it < maxit; ++it) {
          double dlx = 0.0;
          double cur[RV], nxt[RV];
#pragma unroll
          for (int i = 0; i < RV; ++i) {
            const int t = tid + 256 * i;
            cur[i] = t < na ? __hip_atomic_load(GAA + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
          }
          for (int k = 0; k < na; ++k) {
            const double *Gn = GAA + (int64_t)min(k + 1, na - 1) * LS_AMAX;
#pragma unroll
            for (int i = 0; i < RV; ++i) {
              const int t = tid + 256 * i;
              nxt[i] = t < na ? __hip_atomic_load(Gn + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
            }
            if (tid == 0) {
              const double u = gA[k] + bA[k], v = fabs(u) - lam;
              const double nb = v > 0.0 ? copysign(v, u) : 0.0;
              const double d = nb - bA[k];
              if (d != 0.0) { bA[k] = nb; dA[k] += d; dlx = fmax(dlx, d * d); }
              s_red[0] = d;
            }
            __syncthreads();
            const double d = s_red[0];
            if (d != 0.0) {
#pragma unroll
              for (int i = 0; i < RV; ++i) {
                const int t = tid + 256 * i;
                if (t < na) gA[t] -= cur[i] * d;
              }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < RV; ++i) cur[i] = nxt[i];
          }
          if (tid == 0) s_flag = dlx < thr;
          __syncthreads();
          const bool done = s_flag;
          __syncthreads();
          if (done) break;
        }
      } else {
        for (; it < maxit; ++it) {
          double dlx = 0.0;
          for (int k = 0; k < na; ++k) {
            if (tid == 0) {
              const double u = gA[k] + bA[k], v = fabs(u) - lam;
              const double nb = v > 0.0 ? copysign(v, u) : 0.0;
              const double d = nb - bA[k];
              if (d != 0.0) { bA[k] = nb; dA[k] += d; dlx = fmax(dlx, d * d); }
              s_red[0] = d;
            }
            __syncthreads();
            const double d = s_red[0];
            if (d != 0.0) {
              // (L1-bypassing loads: the rows were written by this workgroup)
              const double *Gk = GAA + (int64_t)k * LS_AMAX;
              for (int t = tid; t < na; t += 256)
                gA[t] -= __hip_atomic_load(Gk + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * d;
            }
            __syncthreads();
          }
          if (tid == 0) s_flag = dlx < thr;
          __syncthreads();
          const bool done = s_flag;
          __syncthreads();
          if (done) break;
        }
      }
      SPROF(na <= LS_GC ? 0 : 4);
      if (it == maxit) { st = 1; fail_m = m; break; }
      // ---- refresh the non-active gradients with this round's changes:
      // row-outer, so each thread keeps SEG loads in flight per row (one per
      // owned j), RU rows at a time (RU x SEG independent loads before their
      // FMAs: the pass is latency-bound on one CU otherwise); rows with no
      // change are compacted out first (adding 0 * G leaves the sum
      // unchanged), t ascending as before, so the sums are bit-identical
      {
        int nr = 0;
        for (int t0 = 0; t0 < na; t0 += 256) {
          const int t = t0 + tid;
          const bool v = t < na && dA[t] != 0.0;
          const unsigned long long bal = __ballot(v);
          if (lane == 0) s_cnt[wave] = __popcll(bal);
          __syncthreads();
          int off = nr;
          for (int w2 = 0; w2 < wave; ++w2) off += s_cnt[w2];
          if (v) rows[off + __popcll(bal & ((1ull << lane) - 1ull))] = t;
          nr += s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
          __syncthreads();
        }
        constexpr int SEG = 8, RU = 8;
        for (int j0 = 0; j0 < p; j0 += 256 * SEG) {
          double acc[SEG];
#pragma unroll
          for (int u = 0; u < SEG; ++u) acc[u] = 0.0;
          int q = 0;
          for (; q + RU <= nr; q += RU) {
            double gv[RU][SEG], dt[RU];
#pragma unroll
            for (int h = 0; h < RU; ++h) {
              const int t = rows[q + h];
              dt[h] = dA[t];
              const double *Gt = G + (int64_t)ia[t] * p;
#pragma unroll
              for (int u = 0; u < SEG; ++u) {
                const int j = j0 + tid + 256 * u;
                gv[h][u] = j < p ? Gt[j] : 0.0;
              }
            }
#pragma unroll
            for (int h = 0; h < RU; ++h)
#pragma unroll
              for (int u = 0; u < SEG; ++u) acc[u] = fma(gv[h][u], dt[h], acc[u]);
          }
          for (; q < nr; ++q) {
            const int t = rows[q];
            const double dt = dA[t];
            const double *Gt = G + (int64_t)ia[t] * p;
#pragma unroll
            for (int u = 0; u < SEG; ++u) {
              const int j = j0 + tid + 256 * u;
              if (j < p) acc[u] = fma(Gt[j], dt, acc[u]);
            }
          }
#pragma unroll
          for (int u = 0; u < SEG; ++u) {
            const int j = j0 + tid + 256 * u;
            if (j < p && !act[j]) g[j] -= acc[u];
          }
        }
      }
      __syncthreads();
      SPROF(1);
      for (int t = tid; t < na; t += 256) dA[t] = 0.0;
      // ---- KKT scan: append violators in index order
      const int na0 = na;
      int base = na;
      for (int j0 = 0; j0 < p; j0 += 256) {
        const int j = j0 + tid;
        const bool v = j < p && ju[j] && !act[j] && fabs(g[j]) > lam;
        const unsigned long long bal = __ballot(v);
        if (lane == 0) s_cnt[wave] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int w2 = 0; w2 < wave; ++w2) off += s_cnt[w2];
        const int tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        if (v) {
          const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
          if (pos < LS_AMAX) { ia[pos] = j; bA[pos] = 0.0; gA[pos] = g[j]; dA[pos] = 0.0; act[j] = 1; }
        }
        base += tot;
        __syncthreads();
      }
      SPROF(2);
      if (base > LS_AMAX) { st = 2; fail_m = m; break; }
      na = base;
      if (na == na0) break;
      // G_AA entries of the new variables (G symmetric): LDS while small,
      // and always the compacted global copy (read once the set outgrows LDS)
      for (int e = tid; e < (na - na0) * na; e += 256) {
        const int k = na0 + e / na, t = e % na;
        const double v = G[(int64_t)ia[k] * p + ia[t]];
        if (na <= LS_GC) {
          GC[k * LS_GC + t] = v;
          GC[t * LS_GC + k] = v;
        }
        __hip_atomic_store(GAA + (int64_t)k * LS_AMAX + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(GAA + (int64_t)t * LS_AMAX + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __threadfence();
      __syncthreads();
      SPROF(3);
    }
    if (st) break;
    // ---- record: dense beta_m, R^2 = beta'(c + g)
    double part = 0.0;
    for (int t = tid; t < na; t += 256) part = fma(bA[t], c[ia[t]] + gA[t], part);
    part = wave_sum(part);
    if (lane == 0) s_red[wave] = part;
    double *bm = bp + (int64_t)m * p;
    for (int j = tid; j < p; j += 256) bm[j] = 0.0;
    __syncthreads();
    for (int t = tid; t < na; t += 256) bm[ia[t]] = bA[t];
    const double rsq = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    if (tid == 0) rsq_out[(int64_t)f * nlam + m] = rsq;
    __syncthreads();
    if (early && f == 0 && m + 1 >= min(5, nlam) && (rsq - rsq_prev < 1e-5 * rsq || rsq > 0.999)) {
      L = m + 1;
      break;
    }
    rsq_prev = rsq;
    // folds stop once the full fit (running concurrently) has published a
    // path length they have reached
    if (early && f > 0) {
      const int Lp = __hip_atomic_load(nlam_out, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (Lp > 0 && m + 1 >= Lp) { L = m + 1; break; }
    }
  }
  if (tid == 0) {
    status[f] = st;
    status[gridDim.x + prob0 + f] = st ? fail_m : nlam;   // lambda index of a failure
    if (f == 0) __hip_atomic_store(nlam_out, L, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else nlam_out[f] = L;
  }
}

// Hold-out SSE of fold f (problem f >= 1) at lambda m: one workgroup per (m, f).
__global__ __launch_bounds__(256) void soft_loss_kernel(const double *__restrict__ Zs, int64_t ld, int n, int p,
                                                        const double *__restrict__ y,
                                                        const int32_t *__restrict__ fold,
                                                        const double *__restrict__ ystat,
                                                        const double *__restrict__ bpath, int nlam,
                                                        double *__restrict__ sse) {
  const int m = blockIdx.x, f = blockIdx.y + 1, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __shared__ double red[4];
  const double *b = bpath + ((int64_t)f * nlam + m) * p;
  const double *Zf = Zs + (int64_t)f * (n + 1) * ld;
  const double yb = ystat[3 * f], ys = ystat[3 * f + 1];
  double acc = 0.0;
  for (int i = 0; i < n; ++i) {
    if (fold[i] != f) continue;
    double s = 0.0;
    for (int j = tid; j < p; j += 256) s = fma(b[j], Zf[(int64_t)i * ld + j], s);
    s = wave_sum(s);
    __syncthreads();
    if (lane == 0) red[wave] = s;
    __syncthreads();
    const double e = y[i] - (yb + ys * ((red[0] + red[1]) + (red[2] + red[3])));
    acc = fma(e, e, acc);
  }
  if (tid == 0) sse[(int64_t)(f - 1) * nlam + m] = acc;
}

}  // namespace dfm

using namespace dfm;

// Context internals shared with dfm_api.hip (error text, stream, device).
namespace dfm {
int ctx_fail(dfm_ctx *ctx, int code, const char *msg);
hipStream_t ctx_stream(dfm_ctx *ctx);
int ctx_device(dfm_ctx *ctx);
}  // namespace dfm

extern "C" int dfm_targeted_soft(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                                 const double *X, int64_t T64, int64_t N64, int64_t ldx,
                                 const int32_t *folds, int nlambda, double lmr, int *nlam_out,
                                 int *best_out, double *lambda_out, double *meanloss_out,
                                 double *beta_out, double *a0_out, uint8_t *mask) {
  if (!ctx) return -1;
  auto fail = [&](int code, const char *msg) { return ctx_fail(ctx, code, msg); };
  if (!y || !X || !folds || T64 < 3 || N64 < 1 || q < 0 || ldx < T64 || (q > 0 && (!w || ldw < T64)))
    return fail(-2, "dfm_targeted_soft: bad arguments");
  if (nlambda < 2 || nlambda > 1000) return fail(-2, "dfm_targeted_soft: nlambda must be in 2..1000");
  const int n = (int)T64, N = (int)N64, p = q + N;
  int K = 0;
  std::vector<int> hold(n + 2, 0);
  for (int i = 0; i < n; ++i) {
    if (folds[i] < 1 || folds[i] > n) return fail(-2, "dfm_targeted_soft: fold ids must be 1..K");
    K = std::max(K, folds[i]);
    hold[folds[i]]++;
  }
  if (K < 2) return fail(-2, "dfm_targeted_soft: need at least 2 folds");
  for (int f = 1; f <= K; ++f)
    if (hold[f] == 0 || hold[f] > n - 2) return fail(-2, "dfm_targeted_soft: every fold id 1..K needs rows");
  const int nprob = K + 1;
  const int64_t ld = (p + 15) / 16 * 16;
  const int64_t strideG = (int64_t)p * p;
  const double gbytes = (double)nprob * strideG * 8;
  if (gbytes > 64e9) return fail(-2, "dfm_targeted_soft: (K+1) p^2 Gram workspace above 64 GB");
  if (lmr <= 0) lmr = n < p ? 1e-2 : 1e-4;   // GLMNet.jl lambda_min_ratio default
  hipSetDevice(ctx_device(ctx));
  hipStream_t st = ctx_stream(ctx);
  // ---- device buffers
  std::vector<void *> bufs;
  bool oom = false;
  auto alloc = [&](size_t bytes) -> void * {
    void *p_ = nullptr;
    if (hipMalloc(&p_, std::max<size_t>(bytes, 8)) != hipSuccess) { oom = true; return nullptr; }
    bufs.push_back(p_);
    return p_;
  };
  auto cleanup = [&]() { hipStreamSynchronize(st); for (void *b : bufs) hipFree(b); bufs.clear(); };
  double *Zraw = (double *)alloc((size_t)n * p * 8);
  double *Zp = (double *)alloc((size_t)n * ld * 8);
  double *Zs = (double *)alloc((size_t)nprob * (n + 1) * ld * 8);
  double *yd = (double *)alloc((size_t)n * 8);
  int32_t *fd = (int32_t *)alloc((size_t)n * 4);
  int32_t *tidx = (int32_t *)alloc((size_t)nprob * n * 4);
  double *ystat = (double *)alloc((size_t)nprob * 3 * 8);
  double *mu = (double *)alloc((size_t)nprob * p * 8), *sd = (double *)alloc((size_t)nprob * p * 8);
  double *cc = (double *)alloc((size_t)nprob * p * 8);
  uint8_t *ju = (uint8_t *)alloc((size_t)nprob * p);
  double *G = (double *)alloc((size_t)nprob * strideG * 8);
  double *alm = (double *)alloc((size_t)nprob * nlambda * 8);
  double *gws = (double *)alloc((size_t)nprob * p * 8);
  int *actws = (int *)alloc((size_t)nprob * p * 4);
  double *gaaws = (double *)alloc((size_t)nprob * LS_AMAX * LS_AMAX * 8);
  double *bpath = (double *)alloc((size_t)nprob * nlambda * p * 8);
  double *rsq = (double *)alloc((size_t)nprob * nlambda * 8);
  int *nl = (int *)alloc((size_t)nprob * 4), *sts = (int *)alloc((size_t)nprob * 8);
  double *sse = (double *)alloc((size_t)K * nlambda * 8);
  if (oom) { cleanup(); return fail(1002, "dfm_targeted_soft: out of device memory"); }
  // ---- inputs: Z = [w x] column-major on the host side of the copy
  hipError_t e = hipSuccess;
  if (q > 0) e = hipMemcpy2DAsync(Zraw, (size_t)n * 8, w, (size_t)ldw * 8, (size_t)n * 8, q, hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpy2DAsync(Zraw + (size_t)q * n, (size_t)n * 8, X, (size_t)ldx * 8, (size_t)n * 8, N,
                         hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(yd, y, (size_t)n * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(fd, folds, (size_t)n * 4, hipMemcpyHostToDevice, st);
  // training-row lists per problem, padded with the block's zero row n
  std::vector<int32_t> tl((size_t)nprob * n);
  for (int f = 0; f < nprob; ++f) {
    int c = 0;
    for (int i = 0; i < n; ++i)
      if (folds[i] != f) tl[(size_t)f * n + c++] = f * (n + 1) + i;
    for (; c < n; ++c) tl[(size_t)f * n + c] = f * (n + 1) + n;
  }
  if (e == hipSuccess) e = hipMemcpyAsync(tidx, tl.data(), tl.size() * 4, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemsetAsync(Zs, 0, (size_t)nprob * (n + 1) * ld * 8, st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: upload failed"); }
  hipLaunchKernelGGL(panel_from_colmajor_kernel, dim3((unsigned)((ld + 31) / 32), (n + 31) / 32), dim3(256), 0, st,
                     Zraw, (int64_t)n, n, p, Zp, ld);
  hipLaunchKernelGGL(soft_ystats_kernel, dim3(1), dim3(64), 0, st, yd, fd, n, nprob, ystat);
  hipLaunchKernelGGL(soft_stats_kernel, dim3((p + 255) / 256, nprob), dim3(256), 0, st, Zp, ld, n, p, yd, fd,
                     ystat, Zs, mu, sd, ju, cc);
  // ---- standardised Grams of every problem on MFMA: G_f = Zs_f' Zs_f / n_f
  PanelSrc src{nullptr, Zs, tidx, nullptr, ld, (int64_t)n};
  e = launch_gram(1, src, p, n, n, G, p, strideG, nprob, st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: Gram launch failed"); }
  hipLaunchKernelGGL(soft_scale_kernel, dim3(2048, nprob), dim3(256), 0, st, G, strideG, strideG, ystat);
  // ---- lambda grid of the full fit: lambda_max = max_j |c_j| over non-constant columns
  std::vector<double> hc(p), hys(3 * nprob);
  std::vector<uint8_t> hju(p);
  e = hipMemcpyAsync(hc.data(), cc, (size_t)p * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hju.data(), ju, (size_t)p, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hys.data(), ystat, hys.size() * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: stats failed"); }
  double lam_max = 0.0;
  for (int j = 0; j < p; ++j)
    if (hju[j]) lam_max = std::max(lam_max, std::fabs(hc[j]));
  if (!(lam_max > 0.0) || !(hys[1] > 0.0)) { cleanup(); return fail(-2, "dfm_targeted_soft: degenerate y or Z"); }
  const double alf = std::pow(lmr, 1.0 / (nlambda - 1));
  std::vector<double> halm((size_t)nprob * nlambda);
  for (int m = 0; m < nlambda; ++m) halm[m] = lam_max * std::pow(alf, (double)m);
  const double thr = 1e-7;   // glmnet's default convergence threshold
  const int maxit = 100000;
  e = hipMemcpyAsync(alm, halm.data(), (size_t)nlambda * 8, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: upload failed"); }
  // ---- every problem's path in ONE launch (one workgroup each).  The full
  // fit (problem 0) exits early at L; the folds use the same lambdas in
  // original units, alm_f = alm_0 ys_0 / ys_f, and run the whole grid (user
  // lambdas: no early exit) — their first L path points are the ones used,
  // so they need not wait for L.
  for (int f = 1; f < nprob; ++f)
    for (int m = 0; m < nlambda; ++m) halm[(size_t)f * nlambda + m] = halm[m] * hys[1] / hys[3 * f + 1];
  e = hipMemcpyAsync(alm, halm.data(), halm.size() * 8, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: upload failed"); }
  e = hipMemsetAsync(nl, 0, (size_t)nprob * 4, st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: memset failed"); }
  static const bool sprof = getenv("DFM_SOFT_PROF") != nullptr;
  static const int cdmode = [] { const char *e_ = getenv("DFM_SOFT_CD"); return e_ ? atoi(e_) : 0; }();
  if (sprof) {
    unsigned long long z[8] = {};
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_soft_prof), z, sizeof z, 0, hipMemcpyHostToDevice, st);
  }
  hipLaunchKernelGGL(lasso_path_kernel, dim3(nprob), dim3(256), 0, st, G, strideG, p, cc, ju, alm, nlambda, 0, 1, cdmode,
                     thr, maxit, gws, actws, gaaws, bpath, rsq, nl, sts);
  std::vector<int> hnl(nprob), hst(2 * nprob);
  e = hipMemcpyAsync(hnl.data(), nl, (size_t)nprob * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hst.data(), sts, (size_t)nprob * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: path kernel failed"); }
  const int L = hnl[0];
  if (sprof) {
    unsigned long long z[8];
    hipMemcpyFromSymbol(z, HIP_SYMBOL(g_soft_prof), sizeof z, 0, hipMemcpyDeviceToHost);
    fprintf(stderr, "[soft prof] ms: passes (LDS G_AA) %.2f passes (global G_AA) %.2f refresh %.2f kkt %.2f fill %.2f\n",
            z[0] * 1e-5, z[4] * 1e-5, z[1] * 1e-5, z[2] * 1e-5, z[3] * 1e-5);
  }
  for (int f = 0; f < nprob; ++f)   // a fold's failure past L concerns lambdas the CV never reads
    if (hst[f] && (f == 0 || hst[nprob + f] < L))
      { cleanup(); return fail(2, hst[f] == 1 ? "lasso coordinate descent did not converge"
                                              : "lasso active set above 1024 variables"); }
  hipLaunchKernelGGL(soft_loss_kernel, dim3(L, K), dim3(256), 0, st, Zs, ld, n, p, yd, fd, ystat, bpath, nlambda,
                     sse);
  std::vector<double> hsse((size_t)K * nlambda), hb(p), hmu(p), hsd(p);
  e = hipMemcpyAsync(hsse.data(), sse, hsse.size() * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: loss kernel failed"); }
  // ---- meanloss = sum_f SSE_f / n (fold-size-weighted hold-out MSE), first argmin
  std::vector<double> ml(L, 0.0);
  for (int f = 0; f < K; ++f)
    for (int m = 0; m < L; ++m) ml[m] += hsse[(size_t)f * nlambda + m];
  int best = 0;
  for (int m = 0; m < L; ++m) {
    ml[m] /= n;
    if (ml[m] < ml[best]) best = m;
  }
  e = hipMemcpyAsync(hb.data(), bpath + (size_t)best * p, (size_t)p * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hmu.data(), mu, (size_t)p * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hsd.data(), sd, (size_t)p * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  cleanup();
  if (e != hipSuccess) return fail(1000 + (int)e, "dfm_targeted_soft: read-back failed");
  const double yb = hys[0], ys = hys[1];
  double a0 = yb;
  for (int j = 0; j < p; ++j) {
    const double bo = hb[j] * ys / hsd[j];
    if (beta_out) beta_out[j] = bo;
    a0 -= bo * hmu[j];
    if (j >= q && mask) mask[j - q] = hb[j] != 0.0 ? 1 : 0;
  }
  if (a0_out) *a0_out = a0;
  if (nlam_out) *nlam_out = L;
  if (best_out) *best_out = best;
  for (int m = 0; m < L; ++m) {
    if (lambda_out) lambda_out[m] = halm[m] * ys;
    if (meanloss_out) meanloss_out[m] = ml[m];
  }
  return 0;
}
