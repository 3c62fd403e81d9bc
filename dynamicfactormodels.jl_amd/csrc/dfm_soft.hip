// dfm_soft.hip — soft-threshold targeted predictors: the glmnetcv lasso path.
//
// Replaces src/targeted_predictors.jl:31-36 (GLMNet.glmnetcv(Z, y) on
// Z = [w x], keep the x columns whose coefficient at the CV-optimal lambda is
// nonzero).  GLMNet is never imported by the reference (defect D5); the
// algorithm is glmnet's gaussian lasso (Friedman, Hastie & Tibshirani 2010),
// the same restatement the parity tests' CPU checker holds: elnet1's
// covariance-updating coordinate descent in its loop order (full cyclic
// passes with in-pass entry, active-set passes, gradient refresh), warm
// starts along the lambda grid, early path exit on the full fit.
//
// Device work per call, K folds + the full fit = K + 1 "problems":
//   soft_stats_kernel   per (problem, column): training-row mean / population
//                       sd / constant flag (two passes), the standardised
//                       panel of every problem stacked in one tall panel, and
//                       c = Zs'ys / n                          (HBM-bound)
//   gram_kernel (K1)    G_f = Zs_f' Zs_f over each problem's training rows,
//                       gathered by row index (zero row pads ragged folds):
//                       (K+1) p^2 n MACs on MFMA              (MFMA-bound)
//   lasso_coop_kernel   one co-resident launch, 1 leader + H helper
//                       workgroups per problem: glmnet's elnet1 path (the
//                       serial coordinate descent over the active set on the
//                       leader, the O(p |A|) full-pass replays and gradient
//                       refreshes spread over the helpers)
//   soft_loss_kernel    hold-out SSE per (fold, lambda)        (HBM-bound)
#include "dfm_common.h"
#include "../../include/dfm.h"
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <utility>
#include <cmath>
#include <vector>

namespace dfm {
hipError_t launch_gram(int orient, const PanelSrc &src, int m, int K, int T, double *G, int64_t ldg,
                       int64_t strideG, int nrep, hipStream_t st);
hipError_t launch_gram_plain_scaled(const double *X, int64_t ld, int m, int K, double *G, int64_t ldg, double alpha,
                                    hipStream_t st);
__global__ void panel_from_colmajor_kernel(const double *, int64_t, int, int, double *, int64_t);

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

// Problem f's standardised training rows, transposed: Zt_f[j][c] =
// Zs[tidx[f n + c]][j] for c < n (tidx's pad entries point at the block's zero
// row) and 0 for n <= c < ldk — a p x ldk row-major panel per problem, the
// plain operand of the LDS-DMA Gram G_f = Zt_f Zt_f' (gram_dma_kernel).  The
// training rows keep their order, so every G_f entry sums the same products
// in the same order as the fused-gather K1 Gram it replaces.  32 x 32 tiles
// through LDS: gathered rows read along j, panel rows written along c.
__global__ __launch_bounds__(256) void soft_transpose_kernel(const double *__restrict__ Zs, int64_t ld,
                                                             const int32_t *__restrict__ tidx, int n, int p,
                                                             int64_t ldk, double *__restrict__ Zt) {
  __shared__ double tile[32][33];
  const int f = blockIdx.z, c0 = blockIdx.x * 32, j0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int32_t *tl = tidx + (int64_t)f * n;
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, j = j0 + tx;
    tile[k][tx] = (c < n && j < p) ? Zs[(int64_t)tl[c] * ld + j] : 0.0;
  }
  __syncthreads();
  double *Zf = Zt + (int64_t)f * p * ldk;
  for (int k = ty; k < 32; k += 8) {
    const int j = j0 + k, c = c0 + tx;
    if (j < p && c < ldk) Zf[(int64_t)j * ldk + c] = tile[tx][k];
  }
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

// ------------------------------------------------------------- lasso path
// glmnet's elnet1 (covariance updating) for K + 1 problems in ONE co-resident
// launch.  The loop order is elnet1's (the parity checker's lasso_path_cd):
// per lambda a full cyclic pass over every variable in index order with
// in-pass entry and eager gradient updates g_j -= c_jk d, then passes over
// the active set in entry order until max d^2 < thr, the non-active
// gradients refreshed by dot(da, c_j,A), and back to the full pass; from the
// second lambda on a lambda starts with the active-set passes.  Every
// product and difference is rounded separately (this file is compiled with
// -ffp-contract=off): given the same G and c the path is bit-identical to
// the restatement (tests/test_gpu_soft.py).
//
// Parallel form.  Problem f owns 1 + H workgroups:
//   leader  (role 0): the serial coordinate descent over the ACTIVE set, on
//           wave 0 in blocks of 64 coordinates (lane t = one coordinate, its
//           column of the 64 x 64 block of G_AA in registers, deltas
//           broadcast by readlane: no barrier per coordinate); each block's
//           changes are applied to every other active gradient by all four
//           waves, in the same order as elnet1's eager updates;
//   helpers (roles 1..H): the O(p |A|) work over the NON-active variables,
//           each on a contiguous slice of the p columns:
//           FULL:    a full pass is run speculatively — the leader visits the
//                    active coordinates in index order assuming no entry; the
//                    helpers replay its change list against every non-active
//                    gradient (the value at the variable's own visit, and the
//                    final one), and report the first variable that enters.
//                    The leader then adds it and re-runs the pass from the
//                    pass-start state (identical up to the entry), until a
//                    replay finds no entry: exactly elnet1's pass;
//           REFRESH: g_j -= dot(da, c_j,A) after the active-set passes.
// Leader and helpers meet through per-problem 8-byte granules in global
// memory, each on a line of its own (cdna_hip_programming.md §6 Guideline
// 16): the producer drains its stores (s_waitcnt vmcnt(0) in every storing
// wave, barrier), ONE lane issues an agent release fence and stores the
// granule {tag = task number, value}; the consumer polls the granule relaxed
// with s_sleep, then ONE agent acquire before the barrier.  Task granule value:
// type | gcur | nc; a helper's done granule carries its first entering
// variable.  Every spin is bounded by a wall-clock timeout, so every wave
// reaches the exit.
constexpr int LP_LMAX = 4096;   // active-set capacity (leader LDS state; glmnet's pmax)
constexpr int LP_B = 64;        // coordinate block = one wave
constexpr int LP_NT = 512;      // threads per workgroup
constexpr int LP_PROF = 32;     // diagnostics slots per problem
constexpr int LP_U = 32;        // helper change-list chunk (replay snapshots at every chunk boundary)
constexpr int LP_NCH = LP_LMAX / LP_U + 2;   // chunk snapshots per column
constexpr int LP_NBL = LP_LMAX / LP_B + 2;   // block snapshots of the leader's full sweep
constexpr int LP_PF = (LP_B * LP_B + LP_NT - 64 - 1) / (LP_NT - 64);   // next-block loads per thread of waves 1..7
enum { LP_FULL = 1, LP_REFRESH = 2, LP_EXIT = 3 };

struct alignas(256) LpLine {   // one granule per 256-B line
  unsigned long long v;
  unsigned long long pad[31];
};
struct LassoCtl {   // per problem, zeroed before the launch
  LpLine task;      // {tag = task number, value = type | gcur << 2 | c0 << 3 | nc << 11}
  LpLine lam;       // the task's lambda (payload)
  LpLine done[64];  // helper h: {tag = task number, value = first entering variable (or INT_MAX)}
};

// Per-workgroup launch record (always on; 128 B, zeroed before every
// attempt).  Every bounded spin that runs out reports itself here — which
// wait, the tag it expected and the granule it last saw — and re-reads the
// granule after an agent acquire and by an atomic read-modify-write; the
// host turns the records into the counters of dfm_lasso_stats and an
// error / stderr line.
enum { LD_NONE = 0, LD_TASK = 1, LD_DONE = 2, LD_PIPE = 3, LD_BUDGET = 4 };
struct alignas(128) LassoDiag {
  long long t_start, t_end;    // wall clock (100 MHz) at the workgroup's entry / exit
  long long t_pub_exit;        // leader: when it published LP_EXIT
  long long t_to;              // first timed-out spin: when it gave up
  long long t_rec;             // ... when a re-read found the granule (0: never)
  unsigned long long seen;     // ... the granule its relaxed polls last returned
  unsigned long long seen_inv; // ... re-read after fence(acquire, agent)
  unsigned long long seen_rmw; // ... read by an agent-scope fetch_or(0)
  int kind, expect, xcc, hwid; // first timeout's kind (LD_*), the tag it waited for; placement
  int m, seq, lane, ntmo;      // lambda index / task number / the polled helper; timeouts in all
  int wend[8];                 // per wave: exit - entry, wall-clock ticks
};

struct LassoArgs {
  const double *G;
  int64_t strideG;
  int p, nlam, early, maxit, H, ldaa;
  double thr;
  const double *c, *alm;
  const uint8_t *ju;
  LassoCtl *ctl;
  double *g2;       // [nprob][2][p]  gradients: the current buffer and the FULL replay's output
  int *isact;       // [nprob][p]
  int *klist;       // [nprob][LP_LMAX] task payload: coordinates
  double *dlist;    // [nprob][LP_LMAX]              deltas
  double *save;     // [nprob][2][LP_LMAX] pass-start a, g (by entry position)
  double *GAA;      // [nprob][ldaa][ldaa] G over the active set, entry order
  double *snapC;    // [nprob][LP_NCH][p]  FULL replay: gradient of column j after the first LP_U c changes
  double *snapL;    // [nprob][LP_NBL][2][ldaa] full sweep: active (g, a) at each block start (entry order)
  double *snapR;    // [nprob][LP_NBL][4]  full sweep: {R^2, changes, active count} at each block start
  double *bpath, *rsq_out;
  int *nlam_out, *status;
  long long tmo;    // spin timeout, wall-clock ticks (100 MHz)
  long long tmo_path;   // whole-path budget of a leader, wall-clock ticks
  long long *prof;  // diagnostics (nullable): [nprob][8] leader wall-clock ticks per phase + counts
  LassoDiag *diag;  // [gridDim.x] launch records
};

DFM_DEV double lp_ld(const double *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DFM_DEV unsigned long long lp_ldu(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DFM_DEV void lp_stu(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DFM_DEV unsigned long long lp_gran(int tag, unsigned int val) { return ((unsigned long long)(unsigned)tag << 32) | val; }
// drain this wave's stores (the producer side of the hand-off; every storing wave)
DFM_DEV void lp_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// ONE lane: agent release, then its own wait (ROCm 7.2 can drop the fence's, Guideline 16)
DFM_DEV void lp_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
DFM_DEV void lp_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
DFM_DEV int lp_xcc() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x;
}
DFM_DEV int lp_hwid() {
  int h;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
  return h;
}
// a timed-out spin: count it, and fill the record if it is the workgroup's first
DFM_DEV bool lp_note(LassoDiag *d, int kind, int want, unsigned long long seen, int m, int seq, int lane) {
  atomicAdd(&d->ntmo, 1);
  if (atomicCAS(&d->kind, 0, kind) != 0) return false;
  d->t_to = wall_clock64();
  d->expect = want; d->seen = seen; d->m = m; d->seq = seq; d->lane = lane;
  return true;
}
// A relaxed poll of granule g ran out at `seen` (tag < want): record it,
// re-read g after an agent acquire (seen_inv) and by an agent-scope atomic
// read-modify-write (seen_rmw), then keep polling by RMW for one more
// timeout.  Returns the granule once its tag reaches `want`, else the last
// value read (the hand-off failed).
DFM_DEV unsigned long long lp_recheck(LassoDiag *d, int kind, int want, unsigned long long *g,
                                      unsigned long long seen, int m, int seq, int lane, long long tmo) {
  const bool first = lp_note(d, kind, want, seen, m, seq, lane);
  const long long t0 = wall_clock64();
  lp_acquire();
  const unsigned long long vi = lp_ldu(g);
  unsigned long long v = __hip_atomic_fetch_or(g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (first) { d->seen_inv = vi; d->seen_rmw = v; }
  if ((int)(vi >> 32) >= want) v = vi;
  while ((int)(v >> 32) < want && wall_clock64() - t0 <= tmo) {
    __builtin_amdgcn_s_sleep(2);
    v = __hip_atomic_fetch_or(g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (first && (int)(v >> 32) >= want) d->t_rec = wall_clock64();
  return v;
}
DFM_DEV int lp_ldi(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DFM_DEV void lp_st(double *p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DFM_DEV void lp_sti(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DFM_DEV double lp_rdlane(double x, int l) {   // l: a compile-time constant inside unrolled loops
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The helpers' share of a task over columns [j0, j1) of problem f.  hk / hd:
// the task's change list, padded past nc with a valid row and a zero delta
// (g - G * 0 == g), so that every load is unconditional and two chunks of
// LP_U loads stay in flight.  FULL: the list is in coordinate order, so the
// variable's own visit falls after the pos = #{k < j} first changes.  A FULL
// task resumes at change LP_U c0 from the column's chunk snapshot (the list
// before it is the one the snapshot was taken on: a restarted pass keeps its
// prefix) and snapshots every further complete chunk.  A visit inside the
// kept prefix precedes the entering variable that caused the restart, so it
// was found not entering and is not checked again.
DFM_DEV int lp_task_cols(const LassoArgs &A, int f, int type, int nc, int c0, double lam, int gcur, int j0, int j1,
                         const int *hk, const double *hd) {
  const int p = A.p;
  const double *G = A.G + (int64_t)f * A.strideG;
  const uint8_t *ju = A.ju + (int64_t)f * p;
  const int *isact = A.isact + (int64_t)f * p;
  double *gin = A.g2 + ((int64_t)f * 2 + gcur) * p;
  double *gout = A.g2 + ((int64_t)f * 2 + (gcur ^ 1)) * p;
  double *sc = A.snapC + (int64_t)f * LP_NCH * p;
  const bool full = type == LP_FULL;
  const int i0s = full ? LP_U * c0 : 0;
  int first = INT_MAX;   // this thread's first entering variable
  const int lane = threadIdx.x & 63;
  // wave-uniform trip count: every lane runs the body (the readlane
  // broadcasts read all 64 lanes); lanes without a live column compute on a
  // valid one and store nothing
  for (int jb = j0 + (int)(threadIdx.x & ~63); jb < j1; jb += blockDim.x) {
    const int jr = jb + lane, j = min(jr, j1 - 1);
    const bool live = jr < j1 && ju[j] && !lp_ldi(isact + j);
    int pos = 0;   // FULL: changes before j's visit (hk ascending)
    if (full) {
      int lo = 0, hi = nc;
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (hk[mid] < j) lo = mid + 1; else hi = mid; }
      pos = lo;
    }
    double s = full ? lp_ld(c0 == 0 ? gin + j : sc + (int64_t)c0 * p + j) : 0.0, sv = s;
    // 64 changes at a time, lane u holding change i0 + u: the row and delta of
    // change u are broadcast by readlane (scalar row base, no LDS round trip
    // per change); two halves of 32 loads in flight
    double ga[LP_U], gb[LP_U];
    auto ld = [&](double *gv, int kv, int h0) {
#pragma unroll
      for (int u = 0; u < LP_U; ++u) {
        const double *row = G + (int64_t)__builtin_amdgcn_readlane(kv, h0 + u) * p;
        gv[u] = row[j];
      }
    };
    auto use = [&](const double *gv, double dv, int i0, int h0) {
#pragma unroll
      for (int u = 0; u < LP_U; ++u) {
        const double d = lp_rdlane(dv, h0 + u);
        if (full) {   // elnet1's eager updates in visit order
          s = s - gv[u] * d;
          sv = i0 + h0 + u < pos ? s : sv;
        } else {      // REFRESH: dot(da, c_j,A), a sequential sum in entry order
          s = s + d * gv[u];
        }
      }
      if (full && live && i0 + h0 + LP_U <= nc) sc[(int64_t)((i0 + h0 + LP_U) / LP_U) * p + j] = s;
    };
    if (i0s < nc) {
      int kv = hk[i0s + lane];
      double dv = hd[i0s + lane];
      ld(ga, kv, 0);
      ld(gb, kv, LP_U);
      for (int i0 = i0s; i0 < nc; i0 += 2 * LP_U) {
        const bool more = i0 + 2 * LP_U < nc;
        const int kn = more ? hk[i0 + 2 * LP_U + lane] : kv;
        const double dn = more ? hd[i0 + 2 * LP_U + lane] : 0.0;
        use(ga, dv, i0, 0);
        if (more) ld(ga, kn, 0);
        use(gb, dv, i0, LP_U);
        if (more) ld(gb, kn, LP_U);
        kv = kn;
        dv = dn;
      }
    }
    if (!live) continue;
    if (full) {
      if (pos >= i0s && fabs(sv) - lam > 0.0) first = min(first, j);
      gout[j] = s;
    } else {
      gin[j] = lp_ld(gin + j) - s;
    }
  }
  return first;
}

// entry position at sweep position x: index order (ORD, ord = s_srt) or entry order
template <bool ORD>
DFM_DEV int lp_at(const int *ord, int x) { return ORD ? ord[x] : x; }

// s_gb := the 64 x 64 block of G_AA at sweep positions [b, b + 64) (zero outside n)
template <bool ORD>
DFM_DEV void lp_gblock_load(const int *ord, int b, int n, const double *GAA, int ldaa, double *s_gb) {
  const int nb = min(LP_B, n - b);
  for (int e = threadIdx.x; e < LP_B * LP_B; e += blockDim.x) {
    const int s = e >> 6, t = e & 63;
    s_gb[e] = (s < nb && t < nb) ? GAA[(int64_t)lp_at<ORD>(ord, b + s) * ldaa + lp_at<ORD>(ord, b + t)] : 0.0;
  }
}

// S serial coordinate steps on wave 0 (lane t = coordinate t of the block,
// Gr = its column of the block's G_AA, a0 = its coefficient at the block
// start).  Every step is branch-free: an unchanged coordinate gives d = +0,
// and g - G * 0 == g (a gradient of exactly -0 becomes +0, which no later
// step can tell apart).  Lanes past the block hold g = a0 = 0 and Gr = 0, so
// their steps are no-ops.  Lane s keeps its gradient at its own visit (gm,
// written from the broadcast value): its delta and new coefficient are
// recomputed from it off the chain, with the same operations.
template <int L>
DFM_DEV double lp_wrlane(double x, double v) {   // x with lane L := v (v uniform)
  const long long b = __double_as_longlong(x), c = __double_as_longlong(v);
  int lo = (int)b, hi = (int)(b >> 32);
  asm("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"((int)c), "i"(L));
  asm("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"((int)(c >> 32)), "i"(L));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int s, int S>
DFM_DEV void lp_chain_step(double &g, double &gm, const double a0, const double *Gr, double lam) {
  if constexpr (s < S) {
    const double gk = lp_rdlane(g, s), ak = lp_rdlane(a0, s);
    const double uu = gk + ak;
    const double v = fabs(uu) - lam;
    const double na = v > 0.0 ? copysign(v, uu) : 0.0;
    const double d = na - ak;
    g = g - Gr[s] * d;
    gm = lp_wrlane<s>(gm, gk);
    lp_chain_step<s + 1, S>(g, gm, a0, Gr, lam);
  }
}
template <int S>
DFM_DEV void lp_chain(double &g, double &gm, const double a0, const double *Gr, double lam) {
  lp_chain_step<0, S>(g, gm, a0, Gr, lam);
}

// Wave-pipeline state of a sweep (LDS; monotone counters of blocks).
struct LpPipe {
  int rdy;                 // wave 1: blocks whose gradients are complete (the next chain may start)
  int grc;                 // wave 0: blocks whose chain has ended (their s_gb block is no longer read)
  int pub;                 // wave 0: blocks whose deltas it has published (s_dr / s_gmr slot k & 1)
  int gbw;                 // waves 2..7: s_gb fills (6 per block)
  int cons[LP_NT / 64];    // per wave: published blocks it has finished with
  int nch[2];              // changes in the published block (slot)
  int stop;                // wave 0: 1 + the index of the last block (entry-order passes: dlx < thr or budget)
  int nsw;                 // wave 0: sweeps done
  int err;                 // a spin timed out (1) or the leader's path budget ran out (2)
  int errw, errt, errv;    // the first timed-out wait: 16 wave + counter (int offset in LpPipe), target, value seen
};
DFM_DEV void lp_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// a pipeline wait timed out: fail the sweep, recording which wait (the first)
DFM_DEV void lp_pipe_fail(LpPipe *pp, const int *f, int target, int seen) {
  volatile int *e = &pp->err;
  if (*e == 0) {
    ((volatile int *)&pp->errw)[0] = 16 * (threadIdx.x >> 6) + (int)(f - reinterpret_cast<const int *>(pp));
    ((volatile int *)&pp->errt)[0] = target;
    ((volatile int *)&pp->errv)[0] = seen;
  }
  *e = 1;
}
// spin (every lane of the wave) until *f >= target; LDS reads are in order per wave
DFM_DEV void lp_wait(const int *f, int target, LpPipe *pp, long long tmo) {
  const volatile int *vf = f;
  const volatile int *ve = &pp->err;
  if (*vf < target) {
    const long long t0 = wall_clock64();
    while (*vf < target) {
      __builtin_amdgcn_s_sleep(1);
      if (*ve) break;   // another wave timed out: the launch is failing, do not wait out a timeout per spin
      if (wall_clock64() - t0 > tmo) { lp_pipe_fail(pp, f, target, *vf); break; }
    }
  }
  asm volatile("" ::: "memory");
}
DFM_DEV void lp_post(int *f, int v) {   // after this wave's LDS writes
  lp_lds_fence();
  if ((threadIdx.x & 63) == 0) *(volatile int *)f = v;
}
// waves 1..7 leave a sweep at the block wave 0 stopped at (pp->stop, set
// before pub(k + 1)) — at or past it, never only AT it: once a spin has timed
// out (pp->err) the waits return at once and these waves can run ahead of
// wave 0, and an equality test they have passed would keep them in the
// unbounded (!ORD) loop with nothing left to wait on — or as soon as the
// launch is failing
template <bool ORD>
DFM_DEV bool lp_sweep_over(const LpPipe *pp, int k) {
  if (((const volatile int *)&pp->err)[0]) return true;
  const int stp = ((const volatile int *)&pp->stop)[0];
  return !ORD && stp > 0 && stp <= k + 1;
}
DFM_DEV int lp_min_cons(const LpPipe *pp, int w0) {
  const volatile int *c = pp->cons;
  int m = INT_MAX;
  for (int w = w0; w < LP_NT / 64; ++w) m = min(m, c[w]);
  return m;
}
DFM_DEV void lp_wait_cons(LpPipe *pp, int w0, int target, long long tmo) {
  if (lp_min_cons(pp, w0) < target) {
    const long long t0 = wall_clock64();
    while (lp_min_cons(pp, w0) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (((const volatile int *)&pp->err)[0]) break;
      if (wall_clock64() - t0 > tmo) { lp_pipe_fail(pp, pp->cons + w0, target, lp_min_cons(pp, w0)); break; }
    }
  }
  asm volatile("" ::: "memory");
}

// One pass over n active positions from block bstart on, in entry order
// (!ORD) or in coordinate-index order (ORD, ord = s_srt: elnet1's full pass,
// which appends every change (coordinate, delta) to kl / dl in visit order
// and snapshots (g, a) of the active set and {R^2, changes, n} at every
// block start, the restart points of the pass).  All threads call it.
//
// Blocks of 64 sweep positions run as a wave pipeline with LDS counters
// instead of workgroup barriers:
//   wave 0     the serial coordinate steps of block k (lane t = one
//              coordinate, its column of the block's G_AA in registers from
//              the LDS copy s_gb, deltas broadcast by readlane), then
//              publishes the block's deltas and visit gradients;
//   wave 1     applies block k's deltas to the 64 gradients of block k + 1
//              first (their G_AA rows prefetched during the chain), which
//              releases wave 0 into block k + 1, then the R^2 bookkeeping;
//   waves 2..7 refill s_gb with block k + 1's G_AA block as soon as wave 0's
//              chain of block k ends, and apply block k's deltas to every
//              other active gradient (rows prefetched) while wave 0 runs
//              block k + 1.
// Every gradient receives the blocks' changes in visit order (wave 1 waits
// for waves 2..7 to finish block k - 1 before it applies block k), so the
// arithmetic is elnet1's.  G_AA is private to this workgroup: plain loads
// (its L1 lines are invalidated after every update of G_AA, see the entry
// step).  s_gb holds the first block of the sweep order `key` when
// gkey == key (the last block prefetches the next sweep's first).
template <bool ORD>
DFM_DEV void lp_sweep(const int *ord, int n, int bstart, double lam, int key, int &gkey, const double *GAA, int ldaa,
                      const int *s_ia, double *s_g, double *s_a, const int *s_rank, double *s_dr, double *s_gmr,
                      double *s_gb, LpPipe *pp, double *s_sc, int *s_nc, int *kl, double *dl, double *snapL,
                      double *snapR, long long tmo, long long *tk, int maxsw = 1, double thr = 0.0,
                      long long tpath0 = 0, long long tmo_path = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (n <= 0) return;
  if (gkey != key || bstart != 0) {
    lp_gblock_load<ORD>(ord, LP_B * bstart, n, GAA, ldaa, s_gb);
    gkey = key;
  }
  if (tid < (int)(sizeof(LpPipe) / 4)) reinterpret_cast<int *>(pp)[tid] = 0;
  __syncthreads();
  // ORD: one pass from block bstart.  !ORD: elnet1's passes over the active
  // set back to back, the pipeline running on across pass boundaries (block
  // k is block k mod nbk of pass k / nbk), until wave 0 finds a pass with
  // max d^2 < thr or maxsw passes are done
  const int nbk = (n + LP_B - 1) / LP_B, K = ORD ? nbk - bstart : INT_MAX;
  const bool nxt = ORD ? false : nbk > 1;   // !ORD: the next block always exists (and differs)
  double *snG = snapL, *snA = snapL + ldaa;   // + bn * 2 ldaa
  if (wave == 0) {
    // ------------------------------------------------ the serial chain
    double dlx_s = 0.0;   // !ORD: this pass's max d^2 per lane
    int sw = 0;
    for (int k = 0; k < K; ++k) {
      const int bk = (bstart + k) % nbk, b0 = LP_B * bk, nb = min(LP_B, n - b0), bn = bk + 1;
      long long t0 = tk && tid == 0 ? wall_clock64() : 0;
      if (k > 0) {
        if (ORD || nxt) lp_wait(&pp->rdy, k, pp, tmo);
        lp_wait(&pp->gbw, 6 * k, pp, tmo);
      }
      long long t1 = 0;
      if (tk && tid == 0) { t1 = wall_clock64(); tk[0] += t1 - t0; }
      const bool on = lane < nb;
      const int pt = on ? lp_at<ORD>(ord, b0 + lane) : 0;
      double g = on ? s_g[pt] : 0.0;
      const double a0 = on ? s_a[pt] : 0.0;
      double Gr[LP_B];
#pragma unroll
      for (int s = 0; s < LP_B; ++s) Gr[s] = s_gb[s * LP_B + lane];
      if (tk && tid == 0) { lp_lds_fence(); t0 = wall_clock64(); tk[4] += t0 - t1; }
      double gm = 0.0;
      switch ((nb + 15) >> 4) {
        case 1: lp_chain<16>(g, gm, a0, Gr, lam); break;
        case 2: lp_chain<32>(g, gm, a0, Gr, lam); break;
        case 3: lp_chain<48>(g, gm, a0, Gr, lam); break;
        default: lp_chain<64>(g, gm, a0, Gr, lam); break;
      }
      lp_post(&pp->grc, k + 1);   // (the chain has consumed every Gr read: s_gb may be refilled)
      if (tk && tid == 0) { t1 = wall_clock64(); tk[5] += t1 - t0; }
      // this lane's step, recomputed from its gradient at the visit (same operations)
      const double uu = gm + a0;
      const double vv = fabs(uu) - lam;
      const double na = vv > 0.0 ? copysign(vv, uu) : 0.0;
      const double dv = on ? na - a0 : 0.0;
      const bool ch = dv != 0.0;
      const double a = ch ? na : a0;
      if (on) { s_g[pt] = g; s_a[pt] = a; }
      const unsigned long long bal = __ballot(ch);
      if (k >= 2) lp_wait_cons(pp, 1, k - 1, tmo);   // slot k & 1 free: block k - 2 consumed by waves 1..7
      s_dr[(k & 1) * LP_B + lane] = dv;
      s_gmr[(k & 1) * LP_B + lane] = gm;
      if (lane == 0) pp->nch[k & 1] = __popcll(bal);
      if (ORD) {   // changes in visit order; this block's coordinates at the next block start
        const int base = *s_nc;
        if (ch) {
          const int o = base + __popcll(bal & ((1ull << lane) - 1ull));
          kl[o] = s_ia[pt];
          dl[o] = dv;
        }
        if (lane == 0) {
          *s_nc = base + __popcll(bal);
          snapR[bn * 4 + 1] = (double)(base + __popcll(bal));
          snapR[bn * 4 + 2] = (double)n;
        }
        if (on) {
          snG[(int64_t)bn * 2 * ldaa + pt] = g;
          snA[(int64_t)bn * 2 * ldaa + pt] = a;
        }
      }
      bool last = false;
      if (!ORD) {
        dlx_s = fmax(dlx_s, dv * dv);
        if (bk == nbk - 1) {   // end of a pass: converged, or the pass budget spent?
          double mx = dlx_s;
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
          ++sw;
          // the leader's whole-path budget (tmo_path): fail like a timed-out hand-off
          const bool over = tmo_path > 0 &&
                            __builtin_amdgcn_readfirstlane((int)(wall_clock64() - tpath0 > tmo_path)) != 0;
          last = mx < thr || sw >= maxsw || over;
          if (lane == 0) {
            s_sc[1] = mx; pp->nsw = sw;
            if (last) pp->stop = k + 1;
            if (over) ((volatile int *)&pp->err)[0] = 2;
          }
          dlx_s = 0.0;
        }
      }
      lp_post(&pp->pub, k + 1);
      if (tk && tid == 0) { tk[6] += wall_clock64() - t1; tk[2] += 1; }
      if (last) break;
      if (*(volatile int *)&pp->err) {   // a spin timed out: the launch is failing (status 3)
        if (lane == 0) *(volatile int *)&pp->stop = k + 1;
        break;
      }
    }
  } else if (wave == 1) {
    // ------------------------------------------------ next block first, R^2
    double rsq = s_sc[0], dlx_l = 0.0;
    for (int k = 0; k < K; ++k) {
      const int bk = (bstart + k) % nbk, b0 = LP_B * bk, nb = min(LP_B, n - b0), bn = bk + 1;
      const bool urg = ORD ? k + 1 < K : nxt;
      const int b1 = LP_B * ((bk + 1) % nbk), nb1 = urg ? min(LP_B, n - b1) : 0;
      const bool qon = lane < nb1;
      const int qq = urg ? lp_at<ORD>(ord, b1 + min(lane, nb1 - 1)) : 0;   // block k + 1's gradient (entry position)
      double pv[LP_B];
      if (urg) {
#pragma unroll
        for (int s = 0; s < LP_B; ++s) {
          const double *row = GAA + (int64_t)__builtin_amdgcn_readfirstlane(lp_at<ORD>(ord, b0 + min(s, nb - 1))) * ldaa;
          pv[s] = (qon && s < nb) ? row[qq] : 0.0;
        }
      }
      long long w0 = tk && tid == 64 ? wall_clock64() : 0;
      lp_wait(&pp->pub, k + 1, pp, tmo);
      if (tk && tid == 64) { const long long w1 = wall_clock64(); tk[16] += w1 - w0; w0 = w1; }
      const int nch = pp->nch[k & 1];
      const double *dr = s_dr + (k & 1) * LP_B;
      if (urg) {
        lp_wait_cons(pp, 2, k, tmo);   // waves 2..7 have applied block k - 1 to these gradients
        if (tk && tid == 64) { const long long w1 = wall_clock64(); tk[17] += w1 - w0; w0 = w1; }
        if (qon) {
          double gq = s_g[qq];
          if (nch) {
            const double2 *d2 = reinterpret_cast<const double2 *>(dr);
#pragma unroll
            for (int c = 0; c < LP_B / 16; ++c) {
              double2 dd[8];
#pragma unroll
              for (int i = 0; i < 8; ++i) dd[i] = d2[8 * c + i];
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                pv[16 * c + 2 * i] = pv[16 * c + 2 * i] * dd[i].x;
                pv[16 * c + 2 * i + 1] = pv[16 * c + 2 * i + 1] * dd[i].y;
              }
            }
#pragma unroll
            for (int s = 0; s < LP_B; ++s) gq = gq - pv[s];
            s_g[qq] = gq;
          }
          if (ORD) {
            snG[(int64_t)bn * 2 * ldaa + qq] = gq;
            snA[(int64_t)bn * 2 * ldaa + qq] = s_a[qq];
          }
        }
        lp_post(&pp->rdy, k + 1);
        if (tk && tid == 64) tk[20] += wall_clock64() - w0;
      }
      // R^2, a sequential sum in visit order (an unchanged coordinate adds
      // t = 0 * x = +-0: rsq >= 0 is unchanged), and max d^2 per lane
      const double dv = dr[lane];
      dlx_l = fmax(dlx_l, dv * dv);
      if (nch) {
        const double t = dv * (2.0 * s_gmr[(k & 1) * LP_B + lane] - dv);
        const unsigned long long bal = __ballot(dv != 0.0);
        const int last = 63 - __builtin_clzll(bal);
#pragma unroll
        for (int s0 = 0; s0 < LP_B; s0 += 16) {
          if (s0 > last) break;
#pragma unroll
          for (int s = s0; s < s0 + 16; ++s) rsq = rsq + lp_rdlane(t, s);
        }
      }
      if (ORD && lane == 0) snapR[bn * 4 + 0] = rsq;
      lp_post(&pp->cons[1], k + 1);
      if (lp_sweep_over<ORD>(pp, k)) break;
    }
    if (ORD) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) dlx_l = fmax(dlx_l, __shfl_xor(dlx_l, o));
    }
    if (lane == 0) { s_sc[0] = rsq; if (ORD) s_sc[1] = fmax(s_sc[1], dlx_l); }
  } else {
    // ------------------------------------------------ s_gb refill, the other gradients
    constexpr int NW = LP_NT - 128, PF = (LP_B * LP_B + NW - 1) / NW;
    const int v = tid - 128;
    for (int k = 0; k < K; ++k) {
      const int bk = (bstart + k) % nbk, b0 = LP_B * bk, nb = min(LP_B, n - b0), bn = bk + 1;
      const int b1 = LP_B * ((bk + 1) % nbk), nb1 = min(LP_B, n - b1);   // (wraps to the next sweep's first)
      const bool urg = ORD ? k + 1 < K : nxt;
      const int u0 = urg ? b1 : n, u1 = urg ? b1 + nb1 : n;   // wave 1's block
      double nx[PF], pv[LP_B];
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int e = v + NW * i, s = e >> 6, t = e & 63;
        nx[i] = (e < LP_B * LP_B && s < nb1 && t < nb1)
                    ? GAA[(int64_t)lp_at<ORD>(ord, b1 + s) * ldaa + lp_at<ORD>(ord, b1 + t)] : 0.0;
      }
      const int q = v, qq = min(q, n - 1);   // gradient (entry position) q
      bool qon = false;
      if (q < n) {
        const int rq = ORD ? s_rank[q] : q;
        qon = (rq < b0 || rq >= b0 + nb) && (rq < u0 || rq >= u1);
      }
#pragma unroll
      for (int s = 0; s < LP_B; ++s) {
        const double *row = GAA + (int64_t)__builtin_amdgcn_readfirstlane(lp_at<ORD>(ord, b0 + min(s, nb - 1))) * ldaa;
        pv[s] = (qon && s < nb) ? row[qq] : 0.0;
      }
      lp_wait(&pp->grc, k + 1, pp, tmo);   // wave 0's chain of block k has ended
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int e = v + NW * i;
        if (e < LP_B * LP_B) s_gb[e] = nx[i];
      }
      lp_lds_fence();
      if (lane == 0) atomicAdd(&pp->gbw, 1);
      lp_wait(&pp->pub, k + 1, pp, tmo);
      const int nch = pp->nch[k & 1];
      const double *dr = s_dr + (k & 1) * LP_B;
      if (qon) {
        double gq = s_g[q];
        if (nch) {   // elnet1's eager updates, in visit order (d = 0: g - G * 0 == g)
          const double2 *d2 = reinterpret_cast<const double2 *>(dr);
#pragma unroll
          for (int c = 0; c < LP_B / 16; ++c) {
            double2 dd[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) dd[i] = d2[8 * c + i];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              pv[16 * c + 2 * i] = pv[16 * c + 2 * i] * dd[i].x;
              pv[16 * c + 2 * i + 1] = pv[16 * c + 2 * i + 1] * dd[i].y;
            }
          }
#pragma unroll
          for (int s = 0; s < LP_B; ++s) gq = gq - pv[s];
          s_g[q] = gq;
        }
        if (ORD) {
          snG[(int64_t)bn * 2 * ldaa + q] = gq;
          snA[(int64_t)bn * 2 * ldaa + q] = s_a[q];
        }
      }
      for (int q2 = NW + v; q2 < n; q2 += NW) {   // gradients past the prefetched ones
        const int rq = ORD ? s_rank[q2] : q2;
        if ((rq >= b0 && rq < b0 + nb) || (rq >= u0 && rq < u1)) continue;
        double gq = s_g[q2];
        if (nch) {
          for (int s0 = 0; s0 < nb; s0 += 32) {
            double gv[32];
#pragma unroll
            for (int w = 0; w < 32; ++w) {
              const double *row =
                  GAA + (int64_t)__builtin_amdgcn_readfirstlane(lp_at<ORD>(ord, b0 + min(s0 + w, nb - 1))) * ldaa;
              gv[w] = row[q2];
            }
#pragma unroll
            for (int w = 0; w < 32; ++w) gq = gq - gv[w] * dr[s0 + w];   // dr = 0 past the block
          }
          s_g[q2] = gq;
        }
        if (ORD) {
          snG[(int64_t)bn * 2 * ldaa + q2] = gq;
          snA[(int64_t)bn * 2 * ldaa + q2] = s_a[q2];
        }
      }
      lp_post(&pp->cons[wave], k + 1);
      if (lp_sweep_over<ORD>(pp, k)) break;
    }
  }
  long long te = tk && tid == 0 ? wall_clock64() : 0;
  __syncthreads();
  if (tk && tid == 0) tk[1] += wall_clock64() - te;
}

__global__ __launch_bounds__(LP_NT, 1) void lasso_coop_kernel(LassoArgs A) {
  __shared__ __attribute__((aligned(16))) char lds[3 * LP_LMAX * 4 + 2 * LP_LMAX * 8];
  __shared__ __attribute__((aligned(16))) double s_d[2 * LP_B];   // sweeps: the delta ring
  __shared__ double s_sc[4], s_gb[LP_B * LP_B], s_log[2 * LP_B];  // sweeps: s_log = the visit-gradient ring
  __shared__ LpPipe s_pp;
  __shared__ int s_i[8], s_cnt[LP_NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = blockIdx.x / (A.H + 1), role = blockIdx.x % (A.H + 1), f = grp, p = A.p, H = A.H;
  LassoCtl *ctl = A.ctl + f;
  LassoDiag *dg = A.diag + blockIdx.x;
  const long long t_wave = wall_clock64();   // this wave's entry (its exit stamp: wend)
  if (tid == 0) { dg->t_start = t_wave; dg->xcc = lp_xcc(); dg->hwid = lp_hwid(); }
  int *kl = A.klist + (int64_t)f * LP_LMAX;
  double *dl = A.dlist + (int64_t)f * LP_LMAX;
  if (role > 0) {   // ------------------------------------------------ helper
    int *hk = (int *)lds;
    double *hd = (double *)(lds + (LP_LMAX + 2 * LP_U) * 4);   // hk padded by < 2 LP_U
    const int h = role - 1, j0 = (int)((int64_t)h * p / H), j1 = (int)((int64_t)(h + 1) * p / H);
    long long hb[6] = {0, 0, 0, 0, 0, 0};   // helper 0 diagnostics: busy (FULL), FULL tasks, changes, busy (REFRESH), staging, replayed changes
    for (int q = 1;; ++q) {
      if (tid == 0) {   // ONE lane polls the task granule, then ONE acquire
        const long long t0 = wall_clock64();
        unsigned long long gv;
        int ok = 1;
        while ((int)((gv = lp_ldu(&ctl->task.v)) >> 32) < q) {
          if (wall_clock64() - t0 > A.tmo) { ok = 0; break; }
          __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) {   // reported, re-read; the task may still be found
          gv = lp_recheck(dg, LD_TASK, q, &ctl->task.v, gv, -1, q, h, A.tmo);
          ok = (int)(gv >> 32) >= q;
        }
        lp_acquire();
        s_i[0] = ok ? (int)(unsigned)gv : -1;
        s_i[1] = INT_MAX;
      }
      __syncthreads();
      const int tv = s_i[0];
      if (tv < 0) break;
      const int type = tv & 3, gcur = (tv >> 2) & 1, c0 = (tv >> 3) & 255, nc = tv >> 11;
      if (type == LP_EXIT) break;
      const long long tb = A.prof && h == 0 && tid == 0 ? wall_clock64() : 0;
      const double lam = __longlong_as_double((long long)lp_ldu(&ctl->lam.v));
      const int i0s = type == LP_FULL ? LP_U * c0 : 0;   // the replay's first change
      const int ncp = nc > i0s ? i0s + (nc - i0s + 2 * LP_U - 1) / (2 * LP_U) * (2 * LP_U) : nc;
      for (int i = tid; i < nc; i += blockDim.x) { hk[i] = lp_ldi(kl + i); hd[i] = lp_ld(dl + i); }
      __syncthreads();
      for (int i = nc + tid; i < ncp; i += blockDim.x) { hk[i] = hk[nc - 1]; hd[i] = 0.0; }
      __syncthreads();
      if (A.prof && h == 0 && tid == 0) { hb[4] += wall_clock64() - tb; hb[5] += nc - i0s; }
      const int first = lp_task_cols(A, f, type, nc, c0, lam, gcur, j0, j1, hk, hd);
      if (first != INT_MAX) atomicMin(&s_i[1], first);   // LDS
      lp_drain();
      __syncthreads();
      if (A.prof && h == 0 && tid == 0) {
        const long long dt = wall_clock64() - tb;
        if (type == LP_FULL) { hb[0] += dt; hb[1] += 1; hb[2] += nc; } else hb[3] += dt;
      }
      if (tid == 0) {
        lp_release();
        lp_stu(&ctl->done[h].v, lp_gran(q, (unsigned)s_i[1]));
      }
    }
    if (A.prof && h == 0 && tid == 0)
      for (int i = 0; i < 4; ++i) A.prof[(int64_t)f * LP_PROF + 20 + i] = hb[i];
    if (A.prof && h == 0 && tid == 0) { A.prof[(int64_t)f * LP_PROF + 26] = hb[4]; A.prof[(int64_t)f * LP_PROF + 27] = hb[5]; }
    if (tid == 0) dg->t_end = wall_clock64();
    if (lane == 0) dg->wend[wave] = (int)(wall_clock64() - t_wave);
    return;
  }
  // ----------------------------------------------------------------- leader
  int *s_ia = (int *)lds, *s_srt = s_ia + LP_LMAX, *s_rank = s_srt + LP_LMAX;
  double *s_g = (double *)(s_rank + LP_LMAX), *s_a = s_g + LP_LMAX;
  const double *G = A.G + (int64_t)f * A.strideG;
  const double *c = A.c + (int64_t)f * p;
  const double *alm = A.alm + (int64_t)f * A.nlam;
  const int ldaa = A.ldaa, cap = min(ldaa, LP_LMAX), nlam = A.nlam;
  double *g2 = A.g2 + (int64_t)f * 2 * p;
  int *isact = A.isact + (int64_t)f * p;
  double *sv = A.save + (int64_t)f * 2 * LP_LMAX;
  double *GAA = A.GAA + (int64_t)f * ldaa * ldaa;
  double *snL = A.snapL + (int64_t)f * LP_NBL * 2 * ldaa, *snR = A.snapR + (int64_t)f * LP_NBL * 4;
  const double *snC = A.snapC + (int64_t)f * LP_NCH * p;
  double *bp = A.bpath + (int64_t)f * nlam * p;
  for (int j = tid; j < p; j += blockDim.x) { lp_st(g2 + j, c[j]); lp_sti(isact + j, 0); }
  if (tid == 0) { s_sc[0] = 0.0; s_sc[1] = 0.0; s_i[1] = 0; s_i[2] = 0; s_pp.err = 0; }
  int seq = 0, gcur = 0, nlp = 0, iz = 0, L = nlam, st = 0, fail_m = nlam, nin = 0, cur_m = 0;
  int ver = 0, gkey = -1;   // active-set version (entries); the sweep order s_gb's block belongs to
  // publish a task to the helpers and wait for all of them (H == 0: run it here)
  // publish a task to the helpers (payload: kl, dl, isact, g2, lam) and wait
  // for every helper's done granule; s_i[3] = the first entering variable
  auto run_task = [&](int type, int nc, double lam, int c0) -> bool {   // (H >= 1: the host guarantees it)
    ++seq;
    if (tid == 0) lp_stu(&ctl->lam.v, (unsigned long long)__double_as_longlong(lam));
    lp_drain();
    __syncthreads();
    if (tid == 0) {
      lp_release();
      lp_stu(&ctl->task.v, lp_gran(seq, (unsigned)(type | gcur << 2 | c0 << 3 | nc << 11)));
    }
    if (type == LP_EXIT) return true;
    if (wave == 0) {   // lane h polls helper h's granule
      const long long t0 = wall_clock64();
      int ok = 1;
      unsigned int v = INT_MAX;
      bool mine = true;
      for (;;) {
        mine = true;
        if (lane < H) {
          const unsigned long long gv = lp_ldu(&ctl->done[lane].v);
          mine = (int)(gv >> 32) >= seq;
          v = (unsigned)gv;
        }
        if (__all(mine)) break;
        if (wall_clock64() - t0 > A.tmo) { ok = 0; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      if (!ok) {   // reported, re-read by every lane still waiting
        if (!mine) {
          const unsigned long long gv = lp_recheck(dg, LD_DONE, seq, &ctl->done[lane].v,
                                                   lp_ldu(&ctl->done[lane].v), cur_m, seq, lane, A.tmo);
          mine = (int)(gv >> 32) >= seq;
          v = (unsigned)gv;
        }
        ok = __all(mine) ? 1 : 0;
      }
      lp_acquire();
      int first = lane < H ? (int)v : INT_MAX;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) first = min(first, __shfl_xor(first, o));
      if (lane == 0) { s_i[3] = first; s_i[4] = ok; }
    }
    __syncthreads();
    return s_i[4] != 0;
  };
  long long pt = wall_clock64();
  const long long tstart = pt;
  // diagnostics accumulators (A.prof) in LDS: a private array whose address
  // is taken (tk) would put the kernel on scratch
  __shared__ long long s_prof[LP_PROF];
  long long *pacc = s_prof;
  if (tid < LP_PROF) pacc[tid] = 0;
  __syncthreads();
  long long *tk = A.prof ? pacc + 8 : nullptr;
  auto ptick = [&](int i) {   // leader phase timing (A.prof): thread 0 only
    if (A.prof && tid == 0) { const long long t = wall_clock64(); pacc[i] += t - pt; pt = t; }
  };
  // a pipeline wait of the last sweep timed out (1) or the path budget ran out (2): record it
  auto sweep_failed = [&]() -> int {
    const int e = s_pp.err;
    if (e && tid == 0)
      lp_note(dg, e == 2 ? LD_BUDGET : LD_PIPE, s_pp.errt, (unsigned long long)(unsigned)s_pp.errv, cur_m, seq,
              s_pp.errw);
    return e == 0 ? 0 : e == 2 ? 4 : 3;
  };
  for (int m = 0; m < nlam && !st; ++m) {
    const double lam = alm[m];
    cur_m = m;
    __syncthreads();
    const double rsq0 = s_sc[0];
    int jz = 1;
    for (;;) {
      // a whole-path wall-clock budget (A.tmo_path): a launch that has not
      // finished by then fails as a timed-out hand-off does (status 3, the
      // host relaunches) instead of running out elnet1's 1e5 passes
      if (tid == 0) s_i[7] = wall_clock64() - tstart > A.tmo_path;
      __syncthreads();
      if (s_i[7]) {
        if (tid == 0) lp_note(dg, LD_BUDGET, 0, 0, m, seq, -1);
        st = 4; fail_m = m; break;
      }
      if (!(iz && jz)) {
        // ---------------- full pass (speculative: see the header comment)
        for (int t = tid; t < nin; t += blockDim.x) { lp_st(sv + t, s_a[t]); lp_st(sv + LP_LMAX + t, s_g[t]); }
        const double rsq_save = s_sc[0];
        const int n_pass = nin;   // active count at the pass start (sv's entries)
        int rsb = 0, c0 = 0;      // the restart's first block (sweep) and chunk (replay)
        lp_drain();
        ++nlp;
        if (tid == 0) s_i[1] = 0;
        for (;;) {
          __syncthreads();
          ptick(6);
          lp_sweep<true>(s_srt, nin, rsb, lam, 2 * ver + 1, gkey, GAA, ldaa, s_ia, s_g, s_a, s_rank, s_d, s_log, s_gb,
                         &s_pp, s_sc, &s_i[1], kl, dl, snL, snR, A.tmo, tk);
          ptick(0);
          if (tid == 0) { pacc[16] += 1; pacc[17] += nin - LP_B * rsb; }
          if (const int e = sweep_failed()) { st = e; fail_m = m; break; }
          if (!run_task(LP_FULL, s_i[1], lam, c0)) { st = 3; fail_m = m; break; }
          ptick(1);
          const int v = s_i[3];
          if (v == INT_MAX) break;
          if (nin >= cap) { st = 2; fail_m = m; break; }
          const long long te0 = A.prof && tid == 0 ? wall_clock64() : 0;
          // ---- variable v enters at entry position nin; the pass restarts
          // from the block holding v's slot (the pass up to that block is
          // unchanged).  Its snapshot (block 0: the pass start) gives the
          // entries visited before; an entry not in the snapshot (v, or one
          // that entered later than it was taken) sits past the block start,
          // so it has a = 0 and the gradient after the first nc_b changes: its
          // chunk snapshot (chunk 0: the pass-start gradient) plus the changes
          // left, in visit order.  Three rounds of global loads: (1) v's row
          // of G, the change list (counts below v and below the restart
          // block's first coordinate) and the block record; (2) the
          // snapshots and the changes past the chunk snapshot; (3) their G
          // entries.
          const int pos = nin, nc = s_i[1];
          int below = 0;   // v's slot in the index order: active indices below v (LDS only)
          for (int t = tid; t < pos; t += blockDim.x) below += s_ia[t] < v ? 1 : 0;
          below = (int)wave_sum((double)below);
          if (lane == 0) s_d[wave] = below;
          __syncthreads();
          int ins = 0;
          for (int w2 = 0; w2 < LP_NT / 64; ++w2) ins += (int)s_d[w2];
          const int bi = ins / LP_B;
          // the restart block's first coordinate (v's slot at the end of a full block: past every change)
          const int cbi = bi == 0 ? 0 : (LP_B * bi < pos ? s_ia[s_srt[LP_B * bi]] : INT_MAX);
          double rsq_b = rsq_save;
          int n_snap = n_pass;
          if (bi > 0) { rsq_b = lp_ld(snR + bi * 4 + 0); n_snap = (int)lp_ld(snR + bi * 4 + 2); }
          int cbelow = 0, cblk = 0;
          for (int t = tid; t <= pos || t < nc; t += blockDim.x) {
            const double val = t <= pos ? G[(int64_t)v * p + (t == pos ? v : s_ia[t])] : 0.0;
            const int kk = t < nc ? lp_ldi(kl + t) : INT_MAX;
            if (t <= pos) {
              GAA[(int64_t)pos * ldaa + t] = val;
              GAA[(int64_t)t * ldaa + pos] = val;
            }
            cbelow += kk < v ? 1 : 0;
            cblk += bi > 0 && kk < cbi ? 1 : 0;
          }
          cbelow = (int)wave_sum((double)cbelow);
          cblk = (int)wave_sum((double)cblk);
          if (lane == 0) { s_log[wave] = cbelow; s_log[8 + wave] = cblk; }
          __syncthreads();
          int pos_v = 0, nc_b = 0;   // changes before v's visit / before the restart block
          for (int w2 = 0; w2 < LP_NT / 64; ++w2) { pos_v += (int)s_log[w2]; nc_b += (int)s_log[8 + w2]; }
          int tmp[LP_LMAX / LP_NT];
#pragma unroll
          for (int i = 0; i < LP_LMAX / LP_NT; ++i) {
            const int t = tid + LP_NT * i;
            tmp[i] = (t >= ins && t < pos) ? s_srt[t] : 0;
          }
          __syncthreads();
#pragma unroll
          for (int i = 0; i < LP_LMAX / LP_NT; ++i) {
            const int t = tid + LP_NT * i;
            if (t >= ins && t < pos) s_srt[t + 1] = tmp[i];
          }
          if (tid == 0) {
            s_srt[ins] = pos;
            s_ia[pos] = v;
            lp_sti(isact + v, 1);
          }
          nin = pos + 1;
          ++ver;
          const double *snG = bi == 0 ? sv + LP_LMAX : snL + (int64_t)bi * 2 * ldaa;
          const double *snA = bi == 0 ? sv : snL + ((int64_t)bi * 2 + 1) * ldaa;
          const double *gin = g2 + (int64_t)gcur * p;
          const int cb = nc_b / LP_U, nt = nc_b - LP_U * cb;   // chunk snapshot, changes past it (< LP_U)
          double *s_pd = s_log;                                  // (s_log is free between sweeps)
          int *s_pk = reinterpret_cast<int *>(s_log + LP_U);
          __syncthreads();
          // (2) the snapshots, the entries past them, the changes past the chunk snapshot
          double ra = 0.0, rg = 0.0;
          const int t1 = tid < nin ? tid : nin - 1;   // nin <= LP_NT here: one entry per thread, else the loop below
          if (tid < nt) { s_pk[tid] = lp_ldi(kl + LP_U * cb + tid); s_pd[tid] = lp_ld(dl + LP_U * cb + tid); }
          if (t1 < n_snap) { ra = lp_ld(snA + t1); rg = lp_ld(snG + t1); }
          else rg = lp_ld(cb == 0 ? gin + s_ia[t1] : snC + (int64_t)cb * p + s_ia[t1]);
          for (int t = tid + LP_NT; t < nin; t += blockDim.x) {   // (more than LP_NT active)
            if (t < n_snap) { s_a[t] = lp_ld(snA + t); s_g[t] = lp_ld(snG + t); }
            else { s_a[t] = 0.0; s_g[t] = lp_ld(cb == 0 ? gin + s_ia[t] : snC + (int64_t)cb * p + s_ia[t]); }
          }
          __syncthreads();
          // (3) the entries past the snapshot: the changes left, in visit order
          for (int t = tid; t < nin; t += blockDim.x) {
            double g = t == tid ? rg : s_g[t];
            const bool fresh = t >= n_snap;
            if (fresh && nt > 0) {
              const int j = s_ia[t];
              double gv[LP_U];
#pragma unroll
              for (int i = 0; i < LP_U; ++i) gv[i] = G[(int64_t)s_pk[min(i, nt - 1)] * p + j];
#pragma unroll
              for (int i = 0; i < LP_U; ++i)
                if (i < nt) g = g - gv[i] * s_pd[i];
            }
            if (t == tid) s_a[t] = fresh ? 0.0 : ra;
            else if (fresh) s_a[t] = 0.0;
            s_g[t] = g;
          }
          for (int t = tid; t <= nin - 1; t += blockDim.x) s_rank[s_srt[t]] = t;
          lp_drain();
          __syncthreads();
          lp_acquire();   // this CU's L1 drops its G_AA lines (plain loads read the new row / column)
          if (tid == 0) { s_sc[0] = rsq_b; s_i[1] = nc_b; }
          rsb = bi;
          c0 = pos_v / LP_U;   // the replay's changes before v's visit are unchanged
          if (A.prof && tid == 0) { pacc[29] += wall_clock64() - te0; pacc[30] += 1; }
        }
        if (st) break;
        {   // the pass's max d^2: over its changes
          const int nc = s_i[1];
          double mx = 0.0;
          for (int i = tid; i < nc; i += blockDim.x) { const double d = lp_ld(dl + i); mx = fmax(mx, d * d); }
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
          __syncthreads();
          if (lane == 0) s_d[wave] = mx;
          __syncthreads();
          if (tid == 0) {
            double r = 0.0;
            for (int w2 = 0; w2 < LP_NT / 64; ++w2) r = fmax(r, s_d[w2]);
            s_sc[1] = r;
          }
        }
        if (st) break;
        gcur ^= 1;                     // the replay's non-active gradients are current
        __syncthreads();
        const double dlx = s_sc[1];
        if (dlx < A.thr) break;        // lambda converged
        if (nlp > A.maxit) { st = 1; fail_m = m; break; }
      }
      iz = 1;
      // ---------------- passes over the active set (entry order)
      for (int t = tid; t < nin; t += blockDim.x) lp_st(sv + t, s_a[t]);   // da start
      lp_drain();
      {   // the passes until max d^2 < thr, as one pipelined run (nlp: elnet1's pass count)
        __syncthreads();
        if (tid == 0) s_sc[1] = 0.0;
        ptick(6);
        if (nin > 0) {
          lp_sweep<false>(nullptr, nin, 0, lam, 2 * ver, gkey, GAA, ldaa, s_ia, s_g, s_a, s_rank, s_d, s_log, s_gb,
                          &s_pp, s_sc, &s_i[1], kl, dl, nullptr, nullptr, A.tmo, tk, A.maxit + 1 - nlp, A.thr,
                          tstart, A.tmo_path);
        } else {
          if (tid == 0) s_pp.nsw = 1;   // (no active variable: one empty pass, max d^2 = 0)
          __syncthreads();
        }
        ptick(2);
        const int nsw = s_pp.nsw;
        nlp += nsw;
        if (tid == 0) { pacc[18] += nsw; pacc[19] += (long long)nsw * nin; }
        if (const int e = sweep_failed()) { st = e; fail_m = m; break; }
        if (!(s_sc[1] < A.thr) && nlp > A.maxit) { st = 1; fail_m = m; break; }
      }
      // ---------------- refresh: g_j -= dot(da, c_j,A) over the non-active j
      if (tid == 0) s_i[1] = 0;
      __syncthreads();
      for (int t0 = 0; t0 < nin; t0 += blockDim.x) {   // nonzero da in entry order
        const int t = t0 + tid;
        const double d = t < nin ? s_a[t] - lp_ld(sv + t) : 0.0;
        const bool ch = d != 0.0;
        const unsigned long long bal = __ballot(ch);
        if (lane == 0) s_cnt[wave] = __popcll(bal);
        __syncthreads();
        int off = s_i[1];
        for (int w2 = 0; w2 < wave; ++w2) off += s_cnt[w2];
        if (ch) {
          const int o = off + __popcll(bal & ((1ull << lane) - 1ull));
          lp_sti(kl + o, s_ia[t]);
          lp_st(dl + o, d);
        }
        __syncthreads();
        if (tid == 0) for (int w2 = 0; w2 < LP_NT / 64; ++w2) s_i[1] += s_cnt[w2];
        __syncthreads();
      }
      ptick(6);
      if (!run_task(LP_REFRESH, s_i[1], lam, 0)) { st = 3; fail_m = m; break; }
      ptick(3);
      jz = 0;
    }
    if (st) break;
    // ---- record beta_m (dense) and R^2
    __syncthreads();
    double *bm = bp + (int64_t)m * p;
    for (int j = tid; j < p; j += blockDim.x) bm[j] = 0.0;
    __syncthreads();
    for (int t = tid; t < nin; t += blockDim.x) bm[s_ia[t]] = s_a[t];
    const double rsq = s_sc[0];
    if (tid == 0) A.rsq_out[(int64_t)f * nlam + m] = rsq;
    if (A.early && f == 0 && m + 1 >= min(5, nlam) && (rsq - rsq0 < 1e-5 * rsq || rsq > 0.999)) {
      L = m + 1;
      break;
    }
    // folds stop once the full fit (running concurrently) has published a
    // path length they have reached.  ONE thread reads the published length
    // and the workgroup decides on that one value: read by every thread (as
    // in round 3), waves could see it on different sides of its publication,
    // wave 0 then left for the exit while waves 1..7 ran into the next lambda
    // and waited on wave 0's pipeline counters until the spin timeout — the
    // 2 s stalls of round 3 (the kernel's workgroups done, these waves not;
    // tools/soft_repeat.py)
    if (A.early && f > 0) {
      __syncthreads();
      if (tid == 0) s_i[6] = __hip_atomic_load(A.nlam_out, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int Lp = s_i[6];
      if (Lp > 0 && m + 1 >= Lp) { L = m + 1; break; }
    }
  }
  run_task(LP_EXIT, 0, 0.0, 0);
  if (tid == 0) dg->t_pub_exit = wall_clock64();
  ptick(6);
  if (A.prof && tid == 64) {
    A.prof[(int64_t)f * LP_PROF + 24] = pacc[24];
    A.prof[(int64_t)f * LP_PROF + 25] = pacc[25];
    A.prof[(int64_t)f * LP_PROF + 28] = pacc[28];
  }
  if (A.prof && tid == 0) { A.prof[(int64_t)f * LP_PROF + 29] = pacc[29]; A.prof[(int64_t)f * LP_PROF + 30] = pacc[30]; }
  if (A.prof && tid == 0) {
    pacc[7] = nin;
    for (int i = 0; i < 20; ++i) A.prof[(int64_t)f * LP_PROF + i] = pacc[i];
  }
  if (tid == 0) {
    A.status[f] = st;
    A.status[gridDim.x / (H + 1) + f] = st ? fail_m : nlam;   // lambda index of a failure
    if (f == 0) __hip_atomic_store(A.nlam_out, L, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else A.nlam_out[f] = L;
    dg->t_end = wall_clock64();
  }
  if (lane == 0) dg->wend[wave] = (int)(wall_clock64() - t_wave);
}

// G_f's diagonal := 1 over the non-constant columns (elnet1's c(k,k) = xv(k) = 1)
__global__ void soft_unit_diag_kernel(double *__restrict__ G, int64_t strideG, int p, const uint8_t *__restrict__ ju) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, f = blockIdx.y;
  if (j < p && ju[(int64_t)f * p + j]) G[(int64_t)f * strideG + (int64_t)j * p + j] = 1.0;
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

// Process-wide record of the lasso launches (dfm_lasso_stats): every
// timed-out spin is counted and reported, so a test can assert there were
// none.  Slots: DFM_LASSO_STAT_* in include/dfm.h.
static std::atomic<long long> g_lasso_stats[DFM_LASSO_NSTATS];
static void lasso_stat_add(int i, long long v) { g_lasso_stats[i].fetch_add(v, std::memory_order_relaxed); }
static void lasso_stat_max(int i, long long v) {
  long long o = g_lasso_stats[i].load(std::memory_order_relaxed);
  while (v > o && !g_lasso_stats[i].compare_exchange_weak(o, v, std::memory_order_relaxed)) {}
}
static long long env_ms(const char *name, long long dflt) {
  const char *v = getenv(name);
  if (!v || !*v) return dflt;
  const long long x = atoll(v);
  return x > 0 ? x : dflt;
}
static const char *lasso_diag_kind(int k) {
  switch (k) {
    case LD_TASK: return "helper task poll";
    case LD_DONE: return "leader done poll";
    case LD_PIPE: return "leader pipeline wait";
    case LD_BUDGET: return "leader path budget";
    default: return "none";
  }
}

// Every problem's path in one co-resident launch (lasso_coop_kernel): nprob
// groups of 1 leader + H helper workgroups, H as large as the chip's
// co-resident workgroups allow (<= one per 256 columns, <= 64).  Scratch is
// allocated here; outputs: bpath [nprob][nlam][p], rsq [nprob][nlam], nl
// [nprob] path lengths, sts [2 nprob] (status, failing lambda).
static hipError_t launch_lasso(const double *G, int64_t strideG, int p, const double *c, const uint8_t *ju,
                               const double *alm, int nlam, int nprob, int early, double thr, int maxit, double *bpath,
                               double *rsq, int *nl, int *sts, hipStream_t st, const char **why) {
  int dev = 0, ncu = 0, per_cu = 0;
  hipGetDevice(&dev);
  hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lasso_coop_kernel, LP_NT, 0);
  if (e != hipSuccess) return e;
  const int maxb = per_cu * ncu;
  int H = std::min(std::min(maxb / nprob - 1, std::max(1, (p + 255) / 256)), 64);
  if (H < 1) { *why = "more lasso problems than co-resident workgroup pairs"; return hipErrorInvalidConfiguration; }
  const int nblk = nprob * (H + 1);
  if (nblk > maxb) { *why = "lasso grid above the co-resident capacity"; return hipErrorInvalidConfiguration; }
  // The grid fills the chip: no other libdfm work may hold CUs while it
  // runs.  The device gate (dfm_common.h) waits for every library call on the
  // device to return and holds new ones off until this launch is done; the
  // device's queued work is then drained.  (Another process on the same GPU
  // is outside the gate: its kernels can still delay workgroups, which the
  // hand-off timeouts and the relaunch below then report.)
  DeviceSolo solo(dev);
  if (!solo.held) { *why = "lasso path launched from inside another libdfm call on the device"; return hipErrorInvalidConfiguration; }
  if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
  const int ldaa = std::min(p, LP_LMAX);
  std::vector<void *> bufs;
  auto alloc = [&](size_t bytes) -> void * {
    void *q_ = nullptr;
    if (hipMalloc(&q_, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
    bufs.push_back(q_);
    return q_;
  };
  LassoArgs A{};
  A.G = G; A.strideG = strideG; A.p = p; A.nlam = nlam; A.early = early; A.maxit = maxit; A.H = H; A.ldaa = ldaa;
  A.thr = thr; A.c = c; A.alm = alm; A.ju = ju;
  A.ctl = (LassoCtl *)alloc((size_t)nprob * sizeof(LassoCtl));
  A.g2 = (double *)alloc((size_t)nprob * 2 * p * 8);
  A.isact = (int *)alloc((size_t)nprob * p * 4);
  A.klist = (int *)alloc((size_t)nprob * LP_LMAX * 4);
  A.dlist = (double *)alloc((size_t)nprob * LP_LMAX * 8);
  A.save = (double *)alloc((size_t)nprob * 2 * LP_LMAX * 8);
  A.GAA = (double *)alloc((size_t)nprob * ldaa * ldaa * 8);
  A.snapC = (double *)alloc((size_t)nprob * LP_NCH * p * 8);
  A.snapL = (double *)alloc((size_t)nprob * LP_NBL * 2 * ldaa * 8);
  A.snapR = (double *)alloc((size_t)nprob * LP_NBL * 4 * 8);
  A.diag = (LassoDiag *)alloc((size_t)nblk * sizeof(LassoDiag));
  A.bpath = bpath; A.rsq_out = rsq; A.nlam_out = nl; A.status = sts;
  // Spin timeout: 2 s of the 100 MHz wall clock (every legitimate wait is
  // microseconds to milliseconds).  Whole-path budget of a leader: 10 s plus
  // 2 us per (variable, lambda) — C4 (p 5002, 100 lambdas) 11 s against the
  // 49 ms it takes.  DFM_LASSO_TMO_MS / DFM_LASSO_BUDGET_MS override both.
  A.tmo = env_ms("DFM_LASSO_TMO_MS", 2000) * 100000LL;
  A.tmo_path = env_ms("DFM_LASSO_BUDGET_MS", 10000 + (long long)p * nlam / 500) * 100000LL;
  // DFM_LASSO_PROF (diagnostic, stderr): the leaders' per-phase wall time
  static const bool prof = getenv("DFM_LASSO_PROF") != nullptr;
  if (prof) A.prof = (long long *)alloc((size_t)nprob * LP_PROF * 8);
  auto cleanup = [&]() { hipStreamSynchronize(st); for (void *b : bufs) hipFree(b); };
  if (!A.ctl || !A.g2 || !A.isact || !A.klist || !A.dlist || !A.save || !A.GAA || !A.snapC || !A.snapL || !A.snapR ||
      !A.diag) {
    cleanup();
    *why = "out of device memory";
    return hipErrorOutOfMemory;
  }
  // Every scratch buffer starts zeroed before EVERY attempt, as on a fresh
  // allocation (a second call in one process gets recycled pool memory, and
  // round 3 saw such calls stall; a relaunch must not start from a failed
  // attempt's state either).
  auto zero_all = [&]() -> hipError_t {
    hipError_t z = hipSuccess;
    for (auto b : {std::make_pair((void *)A.ctl, (size_t)nprob * sizeof(LassoCtl)),
                   std::make_pair((void *)A.g2, (size_t)nprob * 2 * p * 8),
                   std::make_pair((void *)A.isact, (size_t)nprob * p * 4),
                   std::make_pair((void *)A.klist, (size_t)nprob * LP_LMAX * 4),
                   std::make_pair((void *)A.dlist, (size_t)nprob * LP_LMAX * 8),
                   std::make_pair((void *)A.save, (size_t)nprob * 2 * LP_LMAX * 8),
                   std::make_pair((void *)A.GAA, (size_t)nprob * ldaa * ldaa * 8),
                   std::make_pair((void *)A.snapC, (size_t)nprob * LP_NCH * p * 8),
                   std::make_pair((void *)A.snapL, (size_t)nprob * LP_NBL * 2 * ldaa * 8),
                   std::make_pair((void *)A.snapR, (size_t)nprob * LP_NBL * 4 * 8),
                   std::make_pair((void *)A.diag, (size_t)nblk * sizeof(LassoDiag)),
                   std::make_pair((void *)nl, (size_t)nprob * 4), std::make_pair((void *)sts, (size_t)nprob * 8)})
      if (z == hipSuccess) z = hipMemsetAsync(b.first, 0, b.second, st);
    return z;
  };
  // A plain launch sized to the co-resident capacity (occupancy API above,
  // checked: nblk <= maxb): the kernel needs every workgroup resident
  // (leader/helper hand-offs), not a grid barrier, and every spin is bounded
  // by the wall-clock timeout.  A cooperative launch
  // (hipLaunchCooperativeKernel) adds only the same size check and makes
  // rocprofv3 (ROCm 7.2) fault in its exit path: a bare cooperative launch
  // of a trivial kernel reproduces that SIGSEGV while the same kernel
  // launched plainly exits cleanly (tools/coop_exit_probe.hip,
  // profiles/r03_coop_exit_probe.txt).  Residency is measured instead: every
  // workgroup stamps its entry and exit, and a workgroup that entered after
  // another had exited is reported.
  // A launch in which a hand-off failed (status 3) is run again (<= 3
  // launches; the path is deterministic, so a completed relaunch returns
  // the same bits); a path-budget overrun (status 4) is not.
  std::vector<LassoDiag> hd(nblk);
  static char msg[512];
  for (int attempt = 0; e == hipSuccess; ++attempt) {
    e = zero_all();
    if (e != hipSuccess) break;
    e = hipStreamSynchronize(st);   // (the launch's own wall time below: the memsets and earlier work done)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (e == hipSuccess) e = hipEventCreate(&ev0);
    if (e == hipSuccess) e = hipEventCreate(&ev1);
    const auto h0 = std::chrono::steady_clock::now();
    if (e == hipSuccess) e = hipEventRecord(ev0, st);
    if (e == hipSuccess) hipLaunchKernelGGL(lasso_coop_kernel, dim3(nblk), dim3(LP_NT), 0, st, A);
    if (e == hipSuccess) e = hipEventRecord(ev1, st);
    if (e == hipSuccess) e = hipGetLastError();
    const auto h1 = std::chrono::steady_clock::now();
    static const bool poll = getenv("DFM_LASSO_SYNC_POLL") != nullptr;   // diagnostic: query instead of a blocking wait
    if (e == hipSuccess && poll) {
      while ((e = hipStreamQuery(st)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    const auto h2 = std::chrono::steady_clock::now();
    const long long host_us = std::chrono::duration_cast<std::chrono::microseconds>(h2 - h0).count();
    const long long launch_us = std::chrono::duration_cast<std::chrono::microseconds>(h1 - h0).count();
    float ev_ms = -1.0f;
    if (e == hipSuccess && ev0 && ev1) hipEventElapsedTime(&ev_ms, ev0, ev1);
    if (ev0) hipEventDestroy(ev0);
    if (ev1) hipEventDestroy(ev1);
    if (e != hipSuccess) break;
    lasso_stat_add(DFM_LASSO_STAT_LAUNCHES, 1);
    if (attempt > 0) lasso_stat_add(DFM_LASSO_STAT_RELAUNCHES, 1);
    std::vector<int> hs(2 * nprob);
    if ((e = hipMemcpy(hs.data(), sts, hs.size() * 4, hipMemcpyDeviceToHost)) != hipSuccess) break;
    if ((e = hipMemcpy(hd.data(), A.diag, hd.size() * sizeof(LassoDiag), hipMemcpyDeviceToHost)) != hipSuccess) break;
    // residency: the latest entry against the earliest exit
    long long t0 = LLONG_MAX, t1 = 0, e0 = LLONG_MAX, e1 = 0, w1 = 0;
    int wb = 0, ww = 0;   // the last wave to leave: workgroup, wave
    long long split = 0;  // widest spread of one workgroup's wave exits
    for (int b = 0; b < nblk; ++b) {
      const LassoDiag &d = hd[b];
      t0 = std::min(t0, d.t_start); t1 = std::max(t1, d.t_start);
      e0 = std::min(e0, d.t_end); e1 = std::max(e1, d.t_end);
      int lo = INT_MAX, hi = 0;
      for (int wv = 0; wv < LP_NT / 64; ++wv) {   // (waves enter together)
        lo = std::min(lo, d.wend[wv]); hi = std::max(hi, d.wend[wv]);
        if (d.t_start + d.wend[wv] > w1) { w1 = d.t_start + d.wend[wv]; wb = b; ww = wv; }
      }
      split = std::max(split, (long long)(hi - lo));
    }
    // a workgroup's waves leave together; 1 ms apart means they took
    // different paths (round 3's lost wake-up was that: see the folds' exit)
    if (split > 100000) lasso_stat_add(DFM_LASSO_STAT_WAVE_SPLITS, 1);
    lasso_stat_max(DFM_LASSO_STAT_MAX_SKEW_US, (t1 - t0) / 100);
    lasso_stat_max(DFM_LASSO_STAT_MAX_KERNEL_US, (e1 - t0) / 100);
    lasso_stat_max(DFM_LASSO_STAT_MAX_HOST_US, host_us);
    if (t1 > e0) lasso_stat_add(DFM_LASSO_STAT_LATE_ENTRIES, 1);
    if (host_us > 2 * (e1 - t0) / 100 + 50000) {   // the launch, not the kernel, took the time
      lasso_stat_add(DFM_LASSO_STAT_SLOW_LAUNCHES, 1);
      fprintf(stderr, "[dfm] lasso launch %d: %lld us on the host (launch call %lld us, events %.0f us) for a %lld us "
              "kernel (last wave exit +%lld us: problem %d %s %d wave %d, its workgroup's tid 0 left at +%lld us; "
              "waves' exits there:", attempt + 1, host_us, launch_us, ev_ms * 1e3, (e1 - t0) / 100, (w1 - t0) / 100,
              wb / (H + 1), wb % (H + 1) ? "helper" : "leader", wb % (H + 1), ww, (hd[wb].t_end - t0) / 100);
      for (int wv = 0; wv < LP_NT / 64; ++wv) fprintf(stderr, " %d", hd[wb].wend[wv] / 100);
      fprintf(stderr, " us; %d workgroups)\n", nblk);
    }
    for (int b = 0; b < nblk; ++b) {
      const LassoDiag &d = hd[b];
      if (!d.ntmo) continue;
      lasso_stat_add(DFM_LASSO_STAT_TIMEOUTS, d.ntmo);
      lasso_stat_add(d.kind == LD_TASK ? DFM_LASSO_STAT_TASK_TMO
                     : d.kind == LD_DONE ? DFM_LASSO_STAT_DONE_TMO
                     : d.kind == LD_PIPE ? DFM_LASSO_STAT_PIPE_TMO : DFM_LASSO_STAT_BUDGET, 1);
      if (d.t_rec) lasso_stat_add(DFM_LASSO_STAT_RECOVERED, 1);
      const int f = b / (H + 1), role = b % (H + 1);
      const LassoDiag &ld = hd[(size_t)f * (H + 1)];
      snprintf(msg, sizeof msg,
               "lasso launch %d: problem %d %s %d (xcc %d hwid %#x): %s timed out %d time(s), waiting for tag %d "
               "(lambda %d, task %d, lane/wave %d); polls saw %#llx, after acquire %#llx, by RMW %#llx; %s; entry +%lld "
               "us, timeout +%lld us, leader (xcc %d) exit published +%lld us, exited +%lld us",
               attempt + 1, f, role ? "helper" : "leader", role ? role - 1 : 0, d.xcc, d.hwid, lasso_diag_kind(d.kind),
               d.ntmo, d.expect, d.m, d.seq, d.lane, d.seen, d.seen_inv, d.seen_rmw,
               d.t_rec ? "a re-read found it" : "no re-read found it", (d.t_start - t0) / 100, (d.t_to - t0) / 100,
               ld.xcc, ld.t_pub_exit ? (ld.t_pub_exit - t0) / 100 : -1, (ld.t_end - t0) / 100);
      fprintf(stderr, "[dfm] %s\n", msg);
      *why = msg;
    }
    if (attempt == 2 || std::find(hs.begin(), hs.begin() + nprob, 3) == hs.begin() + nprob) break;
    fprintf(stderr, "[dfm] lasso path launch %d failed in a hand-off; relaunching\n", attempt + 1);
  }
  if (e == hipSuccess && A.prof) {
    std::vector<long long> hp((size_t)nprob * LP_PROF);
    hipMemcpy(hp.data(), A.prof, hp.size() * 8, hipMemcpyDeviceToHost);
    for (int f = 0; f < nprob; ++f) {
      const long long *q = hp.data() + f * LP_PROF;
      fprintf(stderr, "[lasso prof] problem %2d H %d: full-pass sweeps %.2f ms, FULL replays %.2f, active passes %.2f, "
              "REFRESH %.2f, other %.2f; final |A| %lld | full sweeps %lld (sum n %lld), active sweeps %lld (sum n %lld), "
              "blocks %lld: wave 0 wait %.2f ms, Gr %.2f, chain %.2f, post %.2f, drain %.2f | helper 0: FULL %lld "
              "tasks, %lld changes (%lld replayed), busy %.2f ms (staging %.2f), REFRESH busy %.2f ms | wave 1: wait pub %.2f, "
              "wait bulk %.2f, urgent %.2f | entries %lld: %.2f ms\n", f, H,
              q[0] * 1e-5, q[1] * 1e-5, q[2] * 1e-5, q[3] * 1e-5, q[6] * 1e-5, q[7], q[16], q[17], q[18], q[19], q[10],
              q[8] * 1e-5, q[12] * 1e-5, q[13] * 1e-5, q[14] * 1e-5, q[9] * 1e-5, q[21], q[22], q[27], q[20] * 1e-5,
              q[26] * 1e-5, q[23] * 1e-5, q[24] * 1e-5, q[25] * 1e-5, q[28] * 1e-5, q[30], q[29] * 1e-5);
    }
  }
  cleanup();
  return e;
}

static const char *lasso_status_text(int code) {
  switch (code) {
    case 1: return "lasso coordinate descent did not converge";
    case 2: return "lasso active set above 4096 variables";
    case 3: return "lasso path kernel: a leader/helper hand-off timed out in every launch";
    case 4: return "lasso path kernel: a leader ran past its path time budget (DFM_LASSO_BUDGET_MS)";
    default: return "lasso path failed";
  }
}

// the status text, with the launch record's report of a timed-out spin
static const char *lasso_fail_text(int code, const char *why) {
  static char buf[768];
  if (code < 3) return lasso_status_text(code);
  snprintf(buf, sizeof buf, "%s [%s]", lasso_status_text(code), why);
  return buf;
}

extern "C" int dfm_lasso_stats(int64_t *out, int n, int reset) {
  if (!out && !reset) return -2;
  for (int i = 0; i < n && i < DFM_LASSO_NSTATS; ++i) out[i] = g_lasso_stats[i].load(std::memory_order_relaxed);
  if (reset)
    for (auto &x : g_lasso_stats) x.store(0, std::memory_order_relaxed);
  return DFM_LASSO_NSTATS;
}

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
  const int64_t ldk = ((int64_t)n + 15) / 16 * 16;
  double *Zt = (double *)alloc((size_t)nprob * p * ldk * 8);
  double *alm = (double *)alloc((size_t)nprob * nlambda * 8);
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
  std::vector<int> ntrain(nprob);
  for (int f = 0; f < nprob; ++f) {
    int c = 0;
    for (int i = 0; i < n; ++i)
      if (folds[i] != f) tl[(size_t)f * n + c++] = f * (n + 1) + i;
    ntrain[f] = c;
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
  // each problem's training rows as a transposed plain panel, then one
  // LDS-DMA Gram per problem (C4: 3 160 lower 64 x 64 tiles each)
  hipLaunchKernelGGL(soft_transpose_kernel, dim3((unsigned)((ldk + 31) / 32), (p + 31) / 32, nprob), dim3(256), 0,
                     st, Zs, ld, tidx, n, p, ldk, Zt);
  // G_f = Zt_f Zt_f' / n_f: the 1/n_f (the same double soft_ystats_kernel
  // forms) applied in the Gram's epilogue, no pass over the (K+1) p^2 Grams
  const bool scaled = p >= 64;
  for (int f = 0; f < nprob && e == hipSuccess; ++f) {
    if (scaled) {
      e = launch_gram_plain_scaled(Zt + (size_t)f * p * ldk, ldk, p, n, G + (size_t)f * strideG, p,
                                   1.0 / (double)ntrain[f], st);
    } else {
      PanelSrc src{nullptr, Zt + (size_t)f * p * ldk, nullptr, nullptr, ldk, 0};
      e = launch_gram(0, src, p, n, n, G + (size_t)f * strideG, p, strideG, 1, st);
    }
  }
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: Gram launch failed"); }
  if (!scaled) hipLaunchKernelGGL(soft_scale_kernel, dim3(2048, nprob), dim3(256), 0, st, G, strideG, strideG, ystat);
  hipLaunchKernelGGL(soft_unit_diag_kernel, dim3((p + 255) / 256, nprob), dim3(256), 0, st, G, strideG, p, ju);
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
  // elnet1's grid: lambda_2 = alf lambda_max, lambda_m = lambda_{m-1} alf
  // (lambda_1: the all-zero fit, reported as lambda_max)
  const double alf = std::pow(lmr, 1.0 / (nlambda - 1));
  std::vector<double> halm((size_t)nprob * nlambda);
  halm[0] = lam_max;
  if (nlambda > 1) halm[1] = alf * lam_max;
  for (int m = 2; m < nlambda; ++m) halm[m] = halm[m - 1] * alf;
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
  const char *why = "lasso path launch failed";
  e = launch_lasso(G, strideG, p, cc, ju, alm, nlambda, nprob, 1, thr, maxit, bpath, rsq, nl, sts, st, &why);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, why); }
  std::vector<int> hnl(nprob), hst(2 * nprob);
  e = hipMemcpyAsync(hnl.data(), nl, (size_t)nprob * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hst.data(), sts, (size_t)nprob * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) { cleanup(); return fail(1000 + (int)e, "dfm_targeted_soft: path kernel failed"); }
  const int L = hnl[0];
  for (int f = 0; f < nprob; ++f)   // a fold's failure past L concerns lambdas the CV never reads
    if (hst[f] && (f == 0 || hst[nprob + f] < L)) { cleanup(); return fail(2, lasso_fail_text(hst[f], why)); }
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

// glmnet's elnet1 path on a standardised covariance (the core of
// dfm_targeted_soft, exposed for parity tests and direct use): G p x p
// symmetric with unit diagonal over ju, c = Zs'ys / n, lambdas alms[nlam]
// (standardised units), early = glmnet's early path exit.  Outputs: betas
// (nlam x p, row-major; rows past *L_out untouched), rsq (nlam), *L_out.
extern "C" int dfm_lasso_path(dfm_ctx *ctx, const double *G, const double *c, const uint8_t *ju, int p,
                              const double *alms, int nlam, int early, double thr, double *betas, double *rsq,
                              int *L_out) {
  if (!ctx) return -1;
  if (!G || !c || !ju || !alms || p < 1 || nlam < 1 || !(thr > 0.0) || !L_out)
    return ctx_fail(ctx, -2, "dfm_lasso_path: bad arguments");
  hipSetDevice(ctx_device(ctx));
  hipStream_t st = ctx_stream(ctx);
  const int64_t pp = (int64_t)p * p;
  double *dG = nullptr, *dc = nullptr, *da = nullptr, *db = nullptr, *dr = nullptr;
  uint8_t *dj = nullptr;
  int *dn = nullptr, *ds = nullptr;
  auto freeall = [&]() {
    hipStreamSynchronize(st);
    for (void *q : {(void *)dG, (void *)dc, (void *)da, (void *)db, (void *)dr, (void *)dj, (void *)dn, (void *)ds})
      hipFree(q);
  };
  hipError_t e = hipMalloc(&dG, pp * 8);
  if (e == hipSuccess) e = hipMalloc(&dc, (size_t)p * 8);
  if (e == hipSuccess) e = hipMalloc(&da, (size_t)nlam * 8);
  if (e == hipSuccess) e = hipMalloc(&db, (size_t)nlam * p * 8);
  if (e == hipSuccess) e = hipMalloc(&dr, (size_t)nlam * 8);
  if (e == hipSuccess) e = hipMalloc(&dj, (size_t)p);
  if (e == hipSuccess) e = hipMalloc(&dn, 8);
  if (e == hipSuccess) e = hipMalloc(&ds, 16);
  if (e == hipSuccess) e = hipMemcpyAsync(dG, G, pp * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(dc, c, (size_t)p * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(da, alms, (size_t)nlam * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(dj, ju, (size_t)p, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) { freeall(); return ctx_fail(ctx, 1000 + (int)e, "dfm_lasso_path: upload failed"); }
  const char *why = "lasso path launch failed";
  e = launch_lasso(dG, pp, p, dc, dj, da, nlam, 1, early ? 1 : 0, thr, 100000, db, dr, dn, ds, st, &why);
  if (e != hipSuccess) { freeall(); return ctx_fail(ctx, 1000 + (int)e, why); }
  int hn = 0, hs[2] = {0, 0};
  e = hipMemcpyAsync(&hn, dn, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hs, ds, 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess && !hs[0] && betas) e = hipMemcpyAsync(betas, db, (size_t)hn * p * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && !hs[0] && rsq) e = hipMemcpyAsync(rsq, dr, (size_t)hn * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  freeall();
  if (e != hipSuccess) return ctx_fail(ctx, 1000 + (int)e, "dfm_lasso_path: read-back failed");
  if (hs[0]) return ctx_fail(ctx, 2, lasso_fail_text(hs[0], why));
  *L_out = hn;
  return 0;
}
