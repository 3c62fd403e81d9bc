/*
 * dfm_harness.c — a plain-C (C99) caller of include/dfm.h that makes the same
 * calls as the Julia ccall shim of INTEGRATION.md, independently of the
 * Python ctypes table (_lib.py), so header / ABI drift is caught here.
 *
 *   dfm_harness IN OUT
 *
 * IN  (raw, little endian): int64 T, N, B; double y[T]; double X[T*N]
 *     (column-major, Julia's layout); int32 idx[B*T] (0-based); double eta[B*T].
 * OUT (text): one line per result, "name v0 v1 ..." with %.17g values.
 * Exit: 0 ok, 3 no usable GPU (dfm_ctx_create failed cleanly), 1 any error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dfm.h"

static FILE *out;

static void put(const char *name, const double *v, int64_t n) {
  int64_t i;
  fprintf(out, "%s", name);
  for (i = 0; i < n; ++i) fprintf(out, " %.17g", v[i]);
  fprintf(out, "\n");
}

static void puti(const char *name, const int64_t *v, int64_t n) {
  int64_t i;
  fprintf(out, "%s", name);
  for (i = 0; i < n; ++i) fprintf(out, " %lld", (long long)v[i]);
  fprintf(out, "\n");
}

#define CHECK(ctx, call)                                                                 \
  do {                                                                                   \
    int rc_ = (call);                                                                    \
    if (rc_ != 0) {                                                                      \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_, dfm_last_error(ctx)); \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

static void *xmalloc(size_t n) {
  void *p = calloc(n ? n : 1, 1);
  if (!p) {
    fprintf(stderr, "out of memory\n");
    exit(1);
  }
  return p;
}

int main(int argc, char **argv) {
  FILE *in;
  int64_t T, N, B, t, width, r = 0, kmax = 0, n_eig = 0;
  double *y, *X, *eta, *w, *ev, *coef, *tst, *bo, *bm, *LR, *LM, *WD, *ic, *Xn, *F, *L, *tstat, tr;
  double V, cv, trace, pred[4], truev[4];
  int32_t *idx;
  uint8_t *mask;
  int64_t rw[4], brk[1];
  dfm_ctx *ctx = NULL, *ctx2 = NULL;
  dfm_model *m = NULL, *m2 = NULL, *mb = NULL;
  dfm_model *pair[2];
  dfm_stat st[3];
  size_t got = 0;
  if (argc != 3) {
    fprintf(stderr, "usage: %s IN OUT\n", argv[0]);
    return 1;
  }
  in = fopen(argv[1], "rb");
  if (!in) return 1;
  got += fread(&T, 8, 1, in);
  got += fread(&N, 8, 1, in);
  got += fread(&B, 8, 1, in);
  if (got != 3 || T < 8 || N < 2 || B < 2) return 1;
  y = xmalloc(8 * T);
  X = xmalloc(8 * T * N);
  idx = xmalloc(4 * B * T);
  eta = xmalloc(8 * B * T);
  got = fread(y, 8, T, in) + fread(X, 8, T * N, in) + fread(idx, 4, B * T, in) + fread(eta, 8, B * T, in);
  fclose(in);
  if ((int64_t)got != T + T * N + 2 * B * T) return 1;
  out = fopen(argv[2], "w");
  if (!out) return 1;

  if (dfm_ctx_create(0, &ctx) != 0) {
    fprintf(out, "NO_GPU\n");
    fclose(out);
    return 3;
  }
  w = xmalloc(8 * T);
  for (t = 0; t < T; ++t) w[t] = 1.0;

  /* DynamicFactorModel(y, w, x, "ICp2") with kmax 8: src/DynamicFactorModel.jl:53 */
  CHECK(ctx, dfm_model_fit(ctx, y, w, 1, T, X, T, N, T, 0, DFM_CRIT_ICP2, 8, &m));
  CHECK(ctx, dfm_model_dims(m, &r, &kmax, &n_eig));
  CHECK(ctx, dfm_model_scalars(m, &r, &V, &cv, &trace));
  ev = xmalloc(8 * n_eig);
  coef = xmalloc(8 * (1 + r));
  tst = xmalloc(8 * (1 + r));
  ic = xmalloc(8 * 7 * kmax);
  CHECK(ctx, dfm_model_read(m, ev, coef, tst, NULL, NULL, NULL, NULL, NULL, ic));
  {
    double s[4];
    s[0] = (double)r; s[1] = V; s[2] = cv; s[3] = trace;
    put("fit_scalars", s, 4);
  }
  put("fit_eigvals", ev, n_eig);
  put("fit_coef", coef, 1 + r);
  put("fit_tstat", tst, 1 + r);
  put("fit_ic", ic, 7 * kmax);

  /* criterion_* for k = 1..kmax from the eigenvalues (src/criteria.jl:17-53) */
  {
    double *crit = xmalloc(8 * 7 * kmax);
    CHECK(ctx, dfm_ic_sweep(ev, (int)n_eig, (int)kmax, trace, T, N, 1.0 /* PCp sigma^2 given */, crit));
    put("ic_sweep_sigma1", crit, 7 * kmax);
    free(crit);
  }

  /* wild_bootstrap(dfm, B, stat) (src/bootstrap.jl:41-51) */
  st[0].kind = DFM_STAT_V; st[0].arg0 = 0; st[0].arg1 = 0; st[0].pad = 0;
  st[1].kind = DFM_STAT_CRIT; st[1].arg0 = -1; st[1].arg1 = 0; st[1].pad = 0;
  st[2].kind = DFM_STAT_LR_ALL; st[2].arg0 = (int32_t)(T / 2); st[2].arg1 = 0; st[2].pad = 0;
  width = dfm_stats_width(m, st, 3);
  bo = xmalloc(8 * B * width);
  bm = xmalloc(8 * B * width);
  CHECK(ctx, dfm_bootstrap(m, DFM_BOOT_WILD, B, idx, eta, st, 3, bo));
  put("wild", bo, B * width);
  /* residual_bootstrap (src/bootstrap.jl:21-39) */
  CHECK(ctx, dfm_bootstrap(m, DFM_BOOT_RESIDUAL, B, idx, NULL, st, 1, bm));
  put("residual_V", bm, B);

  /* the host-closure escape: every replicate's factors and loadings (T r and
   * N r values per row) for a stat::Function run on the host */
  {
    dfm_stat fl[2];
    double *fo;
    int64_t wf;
    fl[0].kind = DFM_STAT_FACTORS; fl[0].arg0 = 0; fl[0].arg1 = 0; fl[0].pad = 0;
    fl[1].kind = DFM_STAT_LOADINGS; fl[1].arg0 = 0; fl[1].arg1 = 0; fl[1].pad = 0;
    wf = dfm_stats_width(m, fl, 2);
    fo = xmalloc(8 * B * wf);
    CHECK(ctx, dfm_bootstrap(m, DFM_BOOT_WILD, B, idx, eta, fl, 2, fo));
    put("wild_factors_loadings", fo, B * wf);
    free(fo);
  }

  /* the replicate loop sharded over two contexts (dfm_model_clone + multi) */
  CHECK(ctx, dfm_ctx_create(0, &ctx2));
  CHECK(ctx2, dfm_model_clone(m, ctx2, &m2));
  pair[0] = m;
  pair[1] = m2;
  memset(bm, 0, 8 * B * width);
  CHECK(ctx, dfm_bootstrap_multi(pair, 2, DFM_BOOT_WILD, B, idx, eta, st, 3, bm));
  put("wild_multi", bm, B * width);

  /* LR_test / LM_test / Wald_test for every variable (src/chowtest.jl) */
  LR = xmalloc(8 * N);
  LM = xmalloc(8 * N);
  WD = xmalloc(8 * N);
  CHECK(ctx, dfm_chow_all(m, T / 2, LR, LM, WD));
  put("chow_LR", LR, N);
  put("chow_LM", LM, N);
  put("chow_Wald", WD, N);

  /* the same with break_indices = [T/2 + 1] (1-based): rows split at T/2 */
  brk[0] = T / 2;
  CHECK(ctx, dfm_model_fit_breaks(ctx, y, w, 1, T, X, T, N, T, 2, DFM_CRIT_BIC, 0, brk, 1, &mb));
  CHECK(ctx, dfm_chow_all(mb, T / 2 + 1, LR, NULL, WD));
  put("break_chow_LR", LR, N);
  put("break_chow_Wald", WD, N);

  /* calculate_factors / principal_components (src/DynamicFactorModel.jl:71-121) */
  F = xmalloc(8 * T * 3);
  L = xmalloc(8 * N * 3);
  CHECK(ctx, dfm_pca(ctx, X, T, N, T, 3, ev, F, L, &tr));
  put("pca_eigvals", ev, 3);
  put("pca_F", F, T * 3);

  /* targeted_predictors(..., "hard"), per-candidate (D8 extension) */
  tstat = xmalloc(8 * N);
  mask = xmalloc(N);
  CHECK(ctx, dfm_targeted_hard(ctx, y, w, 1, T, X, T, N, T, DFM_TP_PER_CANDIDATE, 1.96, tstat, mask));
  put("tp_hard_t", tstat, N);

  /* normalize (src/utils.jl:33) */
  Xn = xmalloc(8 * T * N);
  CHECK(ctx, dfm_normalize(ctx, X, T, N, T, Xn, T));
  put("normalize_col0", Xn, T);

  /* pseudo_out_of_sample_forecasts (src/utils.jl:54-72), 4 windows */
  CHECK(ctx, dfm_windows_forecast(ctx, y, w, 1, T, X, T, N, T, 4, DFM_CRIT_ICP2, 4, rw, pred, truev));
  puti("windows_r", rw, 4);
  put("windows_pred", pred, 4);

  /* predict / get_factors on the last two rows (src/DynamicFactorModel.jl:125-128,
   * :152-155, D4 repaired): the model fitted on rows 0..T-3 */
  {
    dfm_model *mp = NULL;
    double pr[2], Fn[2 * 8], lr1, lm1, wd1, cr[7];
    int c;
    CHECK(ctx, dfm_model_fit(ctx, y, w, 1, T, X, T - 2, N, T, 3, DFM_CRIT_ICP2, 0, &mp));
    CHECK(ctx, dfm_predict(mp, 2, w + T - 2, T, X + T - 2, T, pr));
    CHECK(ctx, dfm_get_factors(mp, 2, X + T - 2, T, Fn));
    put("predict", pr, 2);
    put("get_factors", Fn, 2 * 3);
    /* one variable's Chow statistics (cached all-variables pass) */
    CHECK(ctx, dfm_chow(mp, (T - 2) / 2, 4, &lr1, &lm1, &wd1));
    {
      double c3[3];
      c3[0] = lr1; c3[1] = lm1; c3[2] = wd1;
      put("chow_one", c3, 3);
    }
    /* criterion_<name>(dfm) for every name on the fitted model */
    for (c = 0; c < 7; ++c) CHECK(ctx, dfm_model_criterion(mp, c, &cr[c]));
    put("model_criteria", cr, 7);
    dfm_model_destroy(mp);
  }

  /* rolling windows (len T/2) of the workhorse at r = 2 with BIC, forecasts */
  {
    dfm_window_spec sp;
    int64_t rr[4];
    double Vw[4], cw[4], ew[4 * 2], co[4 * 3], tw[4 * 3], pw[4], tv[4];
    sp.kind = DFM_WIN_ROLLING; sp.length = (int32_t)(T / 2); sp.r = 2; sp.crit = DFM_CRIT_BIC; sp.kmax = 0;
    sp.nbreaks = 0; sp.breaks = NULL;
    CHECK(ctx, dfm_windows_ex(ctx, y, w, 1, T, X, T, N, T, 4, &sp, 0, rr, Vw, cw, ew, co, tw, pw, tv));
    puti("rolling_r", rr, 4);
    put("rolling_V", Vw, 4);
    put("rolling_crit", cw, 4);
    put("rolling_pred", pw, 4);
  }

  /* error behaviour: a status code and a message, nothing thrown */
  {
    int rc = dfm_chow_all(m, 0, LR, LM, WD);
    double e[1];
    e[0] = (double)rc;
    put("error_rc", e, 1);
    fprintf(out, "error_msg_nonempty %d\n", (int)(strlen(dfm_last_error(ctx)) > 0));
  }

  /* the lasso path kernel's launch record (no lasso ran: all zero) */
  {
    int64_t ls[DFM_LASSO_NSTATS];
    double d[DFM_LASSO_NSTATS];
    int i, n = dfm_lasso_stats(ls, DFM_LASSO_NSTATS, 0);
    for (i = 0; i < n; ++i) d[i] = (double)ls[i];
    put("lasso_stats", d, n);
  }

  dfm_model_destroy(mb);
  dfm_model_destroy(m2);
  dfm_model_destroy(m);
  dfm_ctx_destroy(ctx2);
  dfm_ctx_destroy(ctx);
  fclose(out);
  return 0;
}
