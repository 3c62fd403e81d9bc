/*
 * dfm_threads.c — the library's host-side threading under a sanitizer build
 * (csrc Makefile `san` / `tsan` targets: ASan + UBSan or TSan on the host code
 * of libdfm.so and of this program; GPU code is not instrumented).
 *
 * It drives every path where libdfm runs host threads of its own or is
 * called from several threads at once:
 *   1. the two-lane bootstrap (dfm_bootstrap_dev: 512..6000 replicates run as
 *      two lanes, the second on a persistent LaneWorker thread with its own
 *      context made by dfm_model_clone on the first call), first and later
 *      calls, against the one-lane result of the same draws (bit-identical);
 *   2. dfm_bootstrap_multi over three contexts (one host thread per shard);
 *   3. two caller threads, each with its own context and model, fitting and
 *      bootstrapping at the same time (the C ABI's threading contract:
 *      different contexts may run concurrently);
 *   4. teardown of a model with a live lane (LaneWorker join, lane context
 *      release);
 *   5. the device gate: the lasso path (a grid that must own the whole chip)
 *      on one thread while another thread's context bootstraps — every path
 *      bit-identical to the first.
 * Exit 0: all results consistent; 1: a call failed or results differ;
 * 3: no GPU.  The sanitizer reports go to stderr.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "dfm.h"

#define T_ 96
#define N_ 150
#define B_ 600

static uint64_t lcg(uint64_t *s) {
  *s = *s * 6364136223846793005ull + 1442695040888963407ull;
  return *s >> 11;
}
static double unif(uint64_t *s) { return (double)lcg(s) * (1.0 / 9007199254740992.0); }
static double gauss(uint64_t *s) {   /* sum of 12 uniforms: plenty for a test panel */
  double a = -6.0;
  int i;
  for (i = 0; i < 12; ++i) a += unif(s);
  return a;
}

static void panel(uint64_t seed, double *y, double *X, int32_t *idx, double *eta) {
  uint64_t s = seed;
  double f[T_ * 3], l[N_ * 3];   /* (stack: per thread) */
  int t, n, j;
  for (j = 0; j < T_ * 3; ++j) f[j] = gauss(&s);
  for (j = 0; j < N_ * 3; ++j) l[j] = gauss(&s);
  for (n = 0; n < N_; ++n)
    for (t = 0; t < T_; ++t) {
      double v = gauss(&s);
      for (j = 0; j < 3; ++j) v += f[t * 3 + j] * l[n * 3 + j];
      X[(int64_t)n * T_ + t] = v;   /* column-major, as Julia */
    }
  for (t = 0; t < T_; ++t) y[t] = f[t * 3] + gauss(&s);
  for (j = 0; j < B_ * T_; ++j) {
    idx[j] = (int32_t)(lcg(&s) % T_);
    eta[j] = gauss(&s);
  }
}

#define CK(ctx, call)                                                                         \
  do {                                                                                        \
    int rc_ = (call);                                                                         \
    if (rc_ != 0) {                                                                           \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_, dfm_last_error(ctx)); \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)

static dfm_stat stats[4];
static int nst = 4;

static int lanes_vs_one(uint64_t seed, int mode) {
  /* per call: two caller threads run this at once */
  double *y = calloc(T_, 8), *X = calloc((size_t)T_ * N_, 8), *w = calloc(T_, 8), *eta = calloc((size_t)B_ * T_, 8);
  int32_t *idx = calloc((size_t)B_ * T_, 4);
  dfm_ctx *ctx = NULL;
  dfm_model *m = NULL;
  double *a, *b, *c;
  int64_t width, i;
  int t;
  panel(seed, y, X, idx, eta);
  for (t = 0; t < T_; ++t) w[t] = 1.0;
  if (dfm_ctx_create(0, &ctx)) return 3;
  CK(ctx, dfm_model_fit(ctx, y, w, 1, T_, X, T_, N_, T_, 3, DFM_CRIT_ICP2, 0, &m));
  CK(ctx, dfm_model_set_mode(m, mode));
  width = dfm_stats_width(m, stats, nst);
  a = calloc((size_t)(B_ * width), 8);
  b = calloc((size_t)(B_ * width), 8);
  c = calloc((size_t)(B_ * width), 8);
  CK(ctx, dfm_bootstrap(m, DFM_BOOT_WILD, B_, idx, eta, stats, nst, a));   /* first call: makes the lane */
  CK(ctx, dfm_bootstrap(m, DFM_BOOT_WILD, B_, idx, eta, stats, nst, b));   /* the lane again */
  CK(ctx, dfm_model_set_batch(m, B_));
  CK(ctx, dfm_bootstrap(m, DFM_BOOT_WILD, B_, idx, eta, stats, nst, c));   /* one lane */
  for (i = 0; i < B_ * width; ++i)
    if (memcmp(&a[i], &c[i], 8) || memcmp(&b[i], &c[i], 8)) {
      fprintf(stderr, "mode %d: lanes differ from one lane at value %lld\n", mode, (long long)i);
      return 1;
    }
  free(a); free(b); free(c);
  dfm_model_destroy(m);   /* joins the LaneWorker, releases the lane context */
  dfm_ctx_destroy(ctx);
  free(y); free(X); free(w); free(eta); free(idx);
  return 0;
}

static int multi(uint64_t seed) {
  double *y = calloc(T_, 8), *X = calloc((size_t)T_ * N_, 8), *w = calloc(T_, 8), *eta = calloc((size_t)B_ * T_, 8);
  int32_t *idx = calloc((size_t)B_ * T_, 4);
  dfm_ctx *cx[3] = {NULL, NULL, NULL};
  dfm_model *ms[3] = {NULL, NULL, NULL};
  double *a, *b;
  int64_t width, i, B = 90;
  int t, g;
  panel(seed, y, X, idx, eta);
  for (t = 0; t < T_; ++t) w[t] = 1.0;
  for (g = 0; g < 3; ++g)
    if (dfm_ctx_create(0, &cx[g])) return 3;
  CK(cx[0], dfm_model_fit(cx[0], y, w, 1, T_, X, T_, N_, T_, 3, DFM_CRIT_ICP2, 0, &ms[0]));
  for (g = 1; g < 3; ++g) CK(cx[g], dfm_model_clone(ms[0], cx[g], &ms[g]));
  width = dfm_stats_width(ms[0], stats, nst);
  a = calloc((size_t)(B * width), 8);
  b = calloc((size_t)(B * width), 8);
  CK(cx[0], dfm_bootstrap_multi(ms, 3, DFM_BOOT_WILD, B, idx, eta, stats, nst, a));
  CK(cx[0], dfm_bootstrap(ms[0], DFM_BOOT_WILD, B, idx, eta, stats, nst, b));
  for (i = 0; i < B * width; ++i)
    if (memcmp(&a[i], &b[i], 8)) {
      fprintf(stderr, "multi: shard rows differ at value %lld\n", (long long)i);
      return 1;
    }
  free(a); free(b);
  for (g = 2; g >= 0; --g) dfm_model_destroy(ms[g]);
  for (g = 0; g < 3; ++g) dfm_ctx_destroy(cx[g]);
  free(y); free(X); free(w); free(eta); free(idx);
  return 0;
}

/* a standardised lasso problem: G = Z'Z / n with unit diagonal, c = Z'y / n */
#define LP_ 40
#define LN_ 80
#define LL_ 30
static void lasso_problem(double *G, double *c, uint8_t *ju, double *alm) {
  uint64_t s = 99;
  double Z[LN_ * LP_], y[LN_], lmax = 0.0;
  int i, j, k;
  for (i = 0; i < LN_ * LP_; ++i) Z[i] = gauss(&s);
  for (i = 0; i < LN_; ++i) y[i] = Z[i * LP_] - 0.5 * Z[i * LP_ + 3] + gauss(&s);
  for (j = 0; j < LP_; ++j) {   /* standardise column j (population sd, as glmnet) */
    double mu = 0.0, v = 0.0;
    for (i = 0; i < LN_; ++i) mu += Z[i * LP_ + j];
    mu /= LN_;
    for (i = 0; i < LN_; ++i) { Z[i * LP_ + j] -= mu; v += Z[i * LP_ + j] * Z[i * LP_ + j]; }
    v = 1.0 / __builtin_sqrt(v / LN_);
    for (i = 0; i < LN_; ++i) Z[i * LP_ + j] *= v;
  }
  for (j = 0; j < LP_; ++j) {
    double a = 0.0;
    for (i = 0; i < LN_; ++i) a += Z[i * LP_ + j] * y[i];
    c[j] = a / LN_;
    ju[j] = 1;
    if (__builtin_fabs(c[j]) > lmax) lmax = __builtin_fabs(c[j]);
    for (k = 0; k < LP_; ++k) {
      double g = 0.0;
      for (i = 0; i < LN_; ++i) g += Z[i * LP_ + j] * Z[i * LP_ + k];
      G[j * LP_ + k] = j == k ? 1.0 : g / LN_;
    }
  }
  alm[0] = lmax;
  for (k = 1; k < LL_; ++k) alm[k] = alm[k - 1] * 0.85;
}

struct gate_job { int stop, rc, runs; };   /* stop: __atomic loads / stores */
static void *boot_loop(void *p) {
  struct gate_job *g = (struct gate_job *)p;
  while (!__atomic_load_n(&g->stop, __ATOMIC_ACQUIRE) && !g->rc) {
    g->rc = lanes_vs_one(21 + g->runs, g->runs & 1);
    ++g->runs;
  }
  return NULL;
}

static int gate(void) {
  static double G[LP_ * LP_], c[LP_], alm[LL_], b0[LL_ * LP_], r0[LL_], b1[LL_ * LP_], r1[LL_];
  static uint8_t ju[LP_];
  dfm_ctx *ctx = NULL;
  struct gate_job g = {0, 0, 0};
  pthread_t th;
  int L0 = 0, L1 = 0, k;
  lasso_problem(G, c, ju, alm);
  if (dfm_ctx_create(0, &ctx)) return 3;
  CK(ctx, dfm_lasso_path(ctx, G, c, ju, LP_, alm, LL_, 0, 1e-7, b0, r0, &L0));
  pthread_create(&th, NULL, boot_loop, &g);
  for (k = 0; k < 8; ++k) {
    int rc = dfm_lasso_path(ctx, G, c, ju, LP_, alm, LL_, 0, 1e-7, b1, r1, &L1);
    if (rc) { fprintf(stderr, "gate: lasso call %d -> %d: %s\n", k, rc, dfm_last_error(ctx)); __atomic_store_n(&g.stop, 1, __ATOMIC_RELEASE); pthread_join(th, NULL); return 1; }
    if (L1 != L0 || memcmp(b0, b1, (size_t)L0 * LP_ * 8) || memcmp(r0, r1, (size_t)L0 * 8)) {
      fprintf(stderr, "gate: lasso call %d differs from the solo path\n", k);
      __atomic_store_n(&g.stop, 1, __ATOMIC_RELEASE); pthread_join(th, NULL); return 1;
    }
  }
  __atomic_store_n(&g.stop, 1, __ATOMIC_RELEASE);
  pthread_join(th, NULL);
  dfm_ctx_destroy(ctx);
  if (g.rc) return g.rc;
  fprintf(stderr, "gate: 8 lasso paths alongside %d bootstrap jobs\n", g.runs);
  return 0;
}

struct job { uint64_t seed; int mode, rc; };
static void *worker(void *p) {
  struct job *j = (struct job *)p;
  j->rc = lanes_vs_one(j->seed, j->mode);
  return NULL;
}

int main(void) {
  int rc;
  struct job jobs[2] = {{11, 0, -1}, {12, 1, -1}};
  pthread_t th[2];
  int i;
  stats[0].kind = DFM_STAT_V; stats[0].arg0 = 0; stats[0].arg1 = 0; stats[0].pad = 0;
  stats[1].kind = DFM_STAT_EIGVAL; stats[1].arg0 = 0; stats[1].arg1 = 0; stats[1].pad = 0;
  stats[2].kind = DFM_STAT_LR_ALL; stats[2].arg0 = T_ / 2; stats[2].arg1 = 0; stats[2].pad = 0;
  stats[3].kind = DFM_STAT_ITERS; stats[3].arg0 = 0; stats[3].arg1 = 0; stats[3].pad = 0;
  /* 1. two lanes, factored (mode 0 = auto) and direct (1) */
  if ((rc = lanes_vs_one(7, 0))) return rc;
  if ((rc = lanes_vs_one(8, 1))) return rc;
  /* 2. shards over three contexts */
  if ((rc = multi(9))) return rc;
  /* 3. two caller threads at once, each its own context (and each spawning a lane) */
  for (i = 0; i < 2; ++i) pthread_create(&th[i], NULL, worker, &jobs[i]);
  for (i = 0; i < 2; ++i) pthread_join(th[i], NULL);
  for (i = 0; i < 2; ++i)
    if (jobs[i].rc) return jobs[i].rc;
  /* 5. the lasso's device gate against a bootstrapping context */
  if ((rc = gate())) return rc;
  printf("dfm_threads OK\n");
  fflush(stdout);
  /* leave without the ROCm runtimes' exit-time teardown: under ASan its
   * device-allocator hooks abort there (sanitizer_allocator_device.h
   * dev_runtime_unloaded_ CHECK), after every libdfm call has returned */
  _exit(0);
}
