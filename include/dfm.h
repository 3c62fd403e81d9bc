/*
 * dfm.h — C ABI of libdfm, the MI355X-native engine for the data-parallel core
 * of DynamicFactorModels.jl (joidegn/DynamicFactorModels.jl).
 *
 * The reference has no FFI: its boundary is the exported Julia API
 * (src/DynamicFactorModels.jl:16-20).  Each entry point below replaces the
 * reference function cited next to it; the Julia `ccall` shim and the Python
 * ctypes mirror that bind them are shown in INTEGRATION.md.
 *
 * Conventions
 *   - Return codes: 0 ok; <0 invalid argument / shape; >0 HIP or numerical
 *     error (singular design, eigensolver not converged).  No exception,
 *     abort or exit crosses the ABI; dfm_last_error() has the message.
 *   - Host arrays are caller-owned; the library copies in/out and never
 *     retains host pointers.  Matrices passed from the host are COLUMN-major
 *     (Julia) with a leading dimension; vectors are contiguous.
 *   - *_dev entry points take DEVICE pointers on the context's device and run
 *     on the context's stream (dfm_ctx_set_stream lets the caller supply its
 *     own, e.g. PyTorch's current stream).  They never synchronise the host
 *     except where a convergence poll needs a 4-byte read-back.
 *   - Indices are 0-based int32 (the Julia shim subtracts 1).
 *   - One context per GPU, used by one host thread at a time.  Different
 *     contexts (of one device or several) may be used from different threads
 *     at once, except that the lasso path (dfm_targeted_soft, dfm_lasso_path)
 *     runs alone on its device: it waits for every other libdfm call on that
 *     device to return, drains the device, and holds new calls off until it
 *     is done (its grid must own every CU).  Called from inside another
 *     libdfm call on the same device it fails instead of waiting.
 */
#ifndef DFM_H
#define DFM_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct dfm_ctx dfm_ctx;
typedef struct dfm_model dfm_model; /* a fitted base model resident in HBM */

/* Information criteria, src/criteria.jl:17-53 (name-based dispatch at
 * src/DynamicFactorModel.jl:138 becomes this code). */
enum dfm_criterion {
  DFM_CRIT_NONE = -1,
  DFM_CRIT_PCP1 = 0, DFM_CRIT_PCP2 = 1, DFM_CRIT_PCP3 = 2,
  DFM_CRIT_ICP1 = 3, DFM_CRIT_ICP2 = 4, DFM_CRIT_ICP3 = 5,
  DFM_CRIT_BIC = 6
};

/* Replicate statistics.  The reference's `stat::Function` callback
 * (src/bootstrap.jl:21, :41) cannot run on the device, so it is this fixed
 * menu.  Each dfm_stat yields ONE double per replicate, except the *_ALL
 * kinds (N doubles, one per variable), FACTORS (T r) and LOADINGS (N r):
 * with those (plus COEF/TSTAT/EIGVAL) a host binding rebuilds each
 * replicate's fit and runs an arbitrary closure on it. */
enum dfm_stat_kind {
  DFM_STAT_V = 0,          /* factor_residual_variance, src/criteria.jl:5       */
  DFM_STAT_CRIT = 1,       /* criterion value (arg0 = dfm_criterion code)       */
  DFM_STAT_EIGVAL = 2,     /* eigenvalue arg0 (0-based, descending)             */
  DFM_STAT_COEF = 3,       /* OLS coefficient arg0, src/DynamicFactorModel.jl:41 */
  DFM_STAT_TSTAT = 4,      /* HC2 t-stat arg0, src/DynamicFactorModel.jl:48     */
  DFM_STAT_TRACE = 5,      /* trace of the Gram (= ||X*||_F^2)                  */
  DFM_STAT_LR = 6,         /* LR_test(dfm, bp=arg0, i=arg1), src/chowtest.jl:19 */
  DFM_STAT_LM = 7,         /* LM_test, src/chowtest.jl:35                       */
  DFM_STAT_WALD = 8,       /* Wald_test, src/chowtest.jl:25                     */
  DFM_STAT_LR_ALL = 9,     /* LR for every variable i (N values), bp = arg0     */
  DFM_STAT_LM_ALL = 10,
  DFM_STAT_WALD_ALL = 11,
  DFM_STAT_ITERS = 12,     /* diagnostic: Rayleigh-Ritz steps of the replicate's eigensolve
                              (NaN on the dense path); an eigenvalue-only stat */
  DFM_STAT_FACTORS = 13,   /* the replicate's factors vcat(F_j) (T x r row-major: T r values),
                              src/DynamicFactorModel.jl:18, :131 — the fields a host-side
                              stat::Function closure reads (src/bootstrap.jl:21, :41) */
  DFM_STAT_LOADINGS = 14   /* break block arg0's loadings L_j (N x r row-major: N r values), :19 */
};
typedef struct dfm_stat { int32_t kind, arg0, arg1, pad; } dfm_stat;

enum dfm_boot_kind { DFM_BOOT_WILD = 0, DFM_BOOT_RESIDUAL = 1 };
enum dfm_tp_mode { DFM_TP_JOINT = 0, DFM_TP_PER_CANDIDATE = 1 };

/* ---------------------------------------------------------------- context */
int dfm_ctx_create(int device, dfm_ctx **out);
int dfm_ctx_destroy(dfm_ctx *ctx);
const char *dfm_last_error(const dfm_ctx *ctx);
int dfm_ctx_set_stream(dfm_ctx *ctx, void *hip_stream); /* NULL = own stream */
int dfm_ctx_synchronize(dfm_ctx *ctx);
/* Eigensolver controls: relative residual tolerance (default 1e-12), maximum
 * subspace iterations (default 400), block width (0 = auto; a block below
 * r + 1 is raised to r + 1: the filtered subspace iteration needs a guard
 * vector beyond the r wanted ones). */
int dfm_ctx_set_eig_params(dfm_ctx *ctx, double tol, int max_iter, int block);
/* Per-kernel HIP-event timing on the context stream (bench/roofline use). */
/* Bootstrap calls whose statistics are all eigenvalue functions (V, CRIT,
   EIGVAL, TRACE) stop the eigensolver when every returned eigenvalue and the
   residual energy trace - sum(theta) are within `tol` relative by the
   Kato-Temple bound (default 1e-12); tol <= 0 always uses the eigenvector
   residual rule of dfm_ctx_set_eig_params. */
int dfm_ctx_set_value_tol(dfm_ctx *ctx, double tol);
int dfm_ctx_enable_timing(dfm_ctx *ctx, int enable);
/* ms accumulated per kernel class (see DFM_KCLASS_* in the implementation);
 * returns the number of classes written into ms_out/launches_out. */
int dfm_ctx_read_timing(dfm_ctx *ctx, double *ms_out, int64_t *launches_out, int cap);
int dfm_ctx_reset_timing(dfm_ctx *ctx);
/* Eigensolver statistics since the last reset: batches solved, total and
 * maximum subspace iterations per batch. */
int dfm_ctx_eig_stats(dfm_ctx *ctx, int64_t *batches, int64_t *iters_total, int64_t *iters_max);
/* Replicate-iterations of the eigensolver's dominant product (the H.Z GEMM in
   the factored bootstrap, G.Q otherwise) summed over the calls since the last
   dfm_ctx_reset_timing: each counts one unconverged replicate in one
   iteration (2 m^2 P flop).  Instrumentation for the roofline figure. */
/* Replicate-products H . Z run by the factored bootstrap's GEMMs since the
 * last reset (two per Rayleigh-Ritz iteration with the Chebyshev filter):
 * the GEMM's algorithmic work is 2 T^2 p per product. */
int dfm_ctx_gemm_products(dfm_ctx *ctx, int64_t *products);
int dfm_ctx_rep_iters(dfm_ctx *ctx, int64_t *rep_iters);
const char *dfm_kernel_class_name(int cls);

/* ------------------------------------------------ principal components
 * principal_components (src/DynamicFactorModel.jl:75-95), no breaks:
 *   T >= N: G = X'X, L = sqrt(N) V, F = X L / N
 *   N >  T: G = XX', F = sqrt(T) U, L = X' F / T
 * Top-k eigenpairs only (the reference consumes [:,1:r]; :33, :131).
 * X column-major T x N (ldx >= T).  Outputs: eigvals[k] descending,
 * F (T x k, col-major, ld T), L (N x k, col-major, ld N), trace_G (may be NULL).
 * Eigenvectors are sign-canonicalised (largest-|.| entry positive). */
int dfm_pca(dfm_ctx *ctx, const double *X, int64_t T, int64_t N, int64_t ldx,
            int k, double *eigvals, double *F, double *L, double *trace_G);

/* Full spectrum of the Gram (eigenvalues only, descending) for
 * min(T,N) <= dfm_full_spectrum_max(); used by PCp's unrestricted sigma^2
 * (src/criteria.jl:18) and full IC sweeps. */
int dfm_full_spectrum_max(void);
int dfm_gram_spectrum(dfm_ctx *ctx, const double *X, int64_t T, int64_t N,
                      int64_t ldx, double *eigvals_m, double *trace_G);

/* normalize (src/utils.jl:33): out = (X .- mean(X, 1)) ./ std(X, 1), the
 * column z-score with the sample (n - 1) std.  X and out column-major T x N
 * (ldx, ldo >= T); out may alias X.  dfm_normalize_dev: both on the device,
 * asynchronous on the context stream. */
int dfm_normalize(dfm_ctx *ctx, const double *X, int64_t T, int64_t N, int64_t ldx, double *out, int64_t ldo);
int dfm_normalize_dev(dfm_ctx *ctx, const double *X_dev, int64_t T, int64_t N, int64_t ldx, double *out_dev,
                      int64_t ldo);

/* ----------------------------------------------------- IC sweep (host math)
 * Criteria for k = 1..kmax from the eigenvalues (identity ||E_k||_F^2 =
 * trace(G) - sum_{j<=k} lambda_j).  sigma2 < 0 means "compute
 * V(ceil(m/2)) from eigvals" (needs ceil(m/2) eigenvalues).  crit_out is
 * 7 x kmax row-major in dfm_criterion order.  Pure arithmetic; no device. */
int dfm_ic_sweep(const double *eigvals, int n_eig, int kmax, double trace_G,
                 int64_t T, int64_t N, double sigma2, double *crit_out);

/* ------------------------------------------------------------ model fit
 * Workhorse constructor (src/DynamicFactorModel.jl:28-51) at fixed r, and
 * the IC-sweep constructor (:53-66) when r <= 0: r is then chosen by
 * criterion `crit` over k = 1..kmax (kmax <= 0 -> ceil(m/2), defect D11).
 * y (T), w (T x q col-major, ldw >= T), X (T x N col-major).  The fitted
 * model (factors, loadings, common component, factor residuals) stays in HBM
 * for the bootstrap and Chow entry points. */
int dfm_model_fit(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                  const double *X, int64_t T, int64_t N, int64_t ldx,
                  int r, int crit, int kmax, dfm_model **out);
/* The same with structural breaks (src/DynamicFactorModel.jl:73, :98): the
 * rows split into blocks at `breaks` (0-based first rows of blocks 2..nbreaks+1,
 * strictly increasing inside 1..T-1 — the reference's 1-based break_indices
 * minus 1).  Each block gets its own principal components with the FULL-sample
 * T, N for branch choice and scaling (:72, defect D7); E = X - vcat(F_j L_j')
 * (:33); the design matrix stacks the blocks' factors (:131).  The IC sweep
 * reads V(k) = (sum_j trace G_j - sum_j sum_{i<=k} lambda_{j,i}) / (N T); PCp's
 * sigma^2 is the no-break unrestricted fit (src/criteria.jl:18).  A block needs
 * at least r (sweep: kmax) eigenpairs: -9 otherwise (the reference's
 * F_j[:, 1:r] would raise).  Reported eigenvalue i is sum_j lambda_{j,i};
 * per-block values and loadings via dfm_model_block.  nbreaks = 0 is
 * dfm_model_fit. */
int dfm_model_fit_breaks(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                         const double *X, int64_t T, int64_t N, int64_t ldx, int r, int crit,
                         int kmax, const int64_t *breaks, int nbreaks, dfm_model **out);
int dfm_model_destroy(dfm_model *m);
/* Number of break blocks (1 without breaks), and block j's first row, rows,
 * top-r eigenvalues (r) and loadings L_j (N x r col-major); NULL skips. */
int dfm_model_blocks(const dfm_model *m);
int dfm_model_block(const dfm_model *m, int j, int64_t *row0, int64_t *rows, double *eigvals,
                    double *L);
/* Sizes of the arrays dfm_model_read fills: r, the IC-sweep kmax (0 when r was
 * given), n_eig = number of eigenvalues returned (max(r, kmax)). */
int dfm_model_dims(const dfm_model *m, int64_t *r, int64_t *kmax, int64_t *n_eig);
/* Scalars: [r, V(r), criterion value, trace_G]. */
int dfm_model_scalars(const dfm_model *m, int64_t *r_out, double *V, double *crit_value,
                      double *trace_G);
/* Host copies (any pointer may be NULL): eigvals (kmax), coefficients and
 * t-stats (q+r), coefficient covariance ((q+r)^2 col-major), OLS residuals
 * (T), F (T x r col-major), L (N x r col-major), factor residuals E (T x N
 * col-major, ld T), criteria for k=1..kmax (7 x kmax, row-major) when the IC
 * sweep ran.  eigvals holds n_eig values (dfm_model_dims). */
int dfm_model_read(const dfm_model *m, double *eigvals, double *coef, double *tstat,
                   double *coef_cov, double *ols_resid, double *F, double *L,
                   double *E, double *ic_values);

/* get_factors (src/DynamicFactorModel.jl:125-128) and predict (:152-155) of a
 * fitted model on n_new new rows, defect D4 repaired: rotation = L (L'L)^-1 of
 * the first break block's loadings (D1), first r columns ("active"); the new
 * rows normalised by the scalar mean and sample std of all T N entries of the
 * fitted x (:127).  x_new: n_new x N column-major (ldx >= n_new), w_new: n_new x q
 * column-major (ldw >= n_new; unused when q = 0); host or device memory.
 * F_out: n_new x r column-major (host); out: n_new predictions (host). */
int dfm_get_factors(dfm_model *m, int64_t n_new, const double *x_new, int64_t ldx, double *F_out);
int dfm_predict(dfm_model *m, int64_t n_new, const double *w_new, int64_t ldw, const double *x_new, int64_t ldx,
                double *out);

/* ------------------------------------------------------------- bootstrap
 * wild_bootstrap (src/bootstrap.jl:41-51) / residual_bootstrap (:21-39):
 * for b < B: X*_b = F_r L_r' + diag(eta_b) E[idx_b, :]  (eta == NULL for
 * RESIDUAL), refit at the model's r and criterion, emit the stats.  A model
 * fitted with breaks refits per break block (:36, :48 pass break_indices);
 * the common component is the blockwise vcat(F_j L_j'); the residual
 * bootstrap's block-wise draws (:23-28) are the caller's idx.  Chow stats of
 * such models read F = vcat(F_j) and the blockwise factor residuals (D1).
 * idx: B x T int32 (row-major, 0-based), eta: B x T.  out: B rows of
 * sum(width(stat)) doubles (row-major). */
int dfm_bootstrap(dfm_model *m, int kind, int64_t B, const int32_t *idx,
                  const double *eta, const dfm_stat *stats, int nstats, double *out);
/* Same, all pointers on the device (inputs resident in HBM). */
int dfm_bootstrap_dev(dfm_model *m, int kind, int64_t B, const int32_t *idx_dev,
                      const double *eta_dev, const dfm_stat *stats, int nstats,
                      double *out_dev);
/* The replicate loop (src/bootstrap.jl:43) sharded over n models, one per
 * context (typically one per GPU; contexts must be distinct), each a
 * dfm_model_clone of the same fit: replicate b runs on model floor(b n / B)
 * (contiguous shards), every shard on its own host thread and stream, rows
 * written in order into the caller's out (B x width, host).  Same arguments and
 * results as dfm_bootstrap: rows are bit-identical to a one-model call. */
int dfm_bootstrap_multi(dfm_model *const *models, int n, int kind, int64_t B, const int32_t *idx,
                        const double *eta, const dfm_stat *stats, int nstats, double *out);
/* Copy of a fitted model on another context (device buffers and host fields),
 * for dfm_bootstrap_multi.  Destroy it with dfm_model_destroy. */
int dfm_model_clone(const dfm_model *m, dfm_ctx *ctx, dfm_model **out);
/* Width of one replicate's output row for a stat list. */
int64_t dfm_stats_width(const dfm_model *m, const dfm_stat *stats, int nstats);
/* Replicates per device batch (0 = auto). */
int dfm_model_set_batch(dfm_model *m, int64_t batch);
/* Bootstrap algorithm for N > T panels: 0 auto (= factored), 1 direct (per-
 * replicate fused-gather Gram + eigensolver on it), 2 factored (the replicate
 * Gram is never formed: every eigen-iteration is one MFMA GEMM of the shared
 * H = E E' against the batch's iterates).  Results agree to rounding. */
int dfm_model_set_mode(dfm_model *m, int mode);
/* Block of the factored bootstrap solver for this model: p eigen-iterate
 * columns per replicate, pz = p rounded up to even = the columns each
 * replicate contributes to the batched H.Z GEMM (its flop per
 * replicate-product is 2 T^2 pz).  Returns 0, or 1 (p = pz = 0) when the
 * model's bootstrap never takes the factored path (T >= N, breaks, r > 16).
 * The answer ignores the statistics of a particular call: a stat list with a
 * PCp criterion (which reads each replicate's full spectrum) or mode 1 sends
 * that call down the direct path even when this returns 0. */
int dfm_model_fact_block(const dfm_model *m, int *p, int *pz);

/* ------------------------------------------------------------ Chow tests
 * LR_test / LM_test / Wald_test (src/chowtest.jl:19-42) for EVERY variable
 * i = 0..N-1 of the fitted model at break period bp (rows 0..bp-1 | bp..T-1).
 * Any output pointer may be NULL. */
int dfm_chow_all(dfm_model *m, int64_t bp, double *LR, double *LM, double *Wald);

/* One variable's LR_test / LM_test / Wald_test (src/chowtest.jl:19-42), i
 * 0-based.  The model keeps the all-variables results of the last break
 * period asked for, so a loop over i = 0..N-1 costs one dfm_chow_all. */
int dfm_chow(dfm_model *m, int64_t bp, int64_t i, double *LR, double *LM, double *Wald);

/* criterion_<name>(dfm) (src/criteria.jl:17-53) of a fitted model at its r,
 * for any criterion code (not only the one it was fitted with).  PCp's sigma^2
 * = V(ceil(m/2)) of the unrestricted fit DynamicFactorModel(y, w, x)
 * (:18, :23, :28) comes from the resident panel's full spectrum (min(T,N) <=
 * dfm_full_spectrum_max()), computed once per model. */
int dfm_model_criterion(dfm_model *m, int crit, double *value);

/* ---------------------------------------------------- expanding windows
 * The refits of pseudo_out_of_sample_forecasts (src/utils.jl:54-72): window
 * w = 0..P-1 refits the IC-sweep constructor (src/DynamicFactorModel.jl:53)
 * on rows 0..T-P+w-1 with criterion crit (any of the 7) over k = 1..kmax_w,
 * kmax_w = ceil(min(T-P+w, N)/2) (the constructor's default, :54), capped by
 * kmax when kmax > 0 (D11).  N > T uses the prefix-Gram identity (one Gram for
 * all windows).  Outputs per window: r (P), V(r) (P), criterion value (P),
 * eigenvalues (P x K, row-major), OLS coefficients and HC2 t-stats
 * (P x (q + K), row-major, NaN past q + r), K = kmax_{P-1} =
 * min(kmax, ceil(min(T-1, N)/2)) (kmax <= 0: no cap).  The forecast step:
 * dfm_windows_forecast. */
int dfm_windows(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                const double *X, int64_t T, int64_t N, int64_t ldx, int P, int crit,
                int kmax, int64_t *r_out, double *V_out, double *crit_out, double *eig_out,
                double *coef_out, double *tstat_out);

/* pseudo_out_of_sample_forecasts (src/utils.jl:54-72) in full: the refits of
 * dfm_windows, then window w predicts row n = T-P+w from its own fit:
 * predict (src/DynamicFactorModel.jl:152-155) with get_factors repaired
 * (defect D4: rotation = L (L'L)^-1 of :126, L = the window's loadings; the
 * new row normalised by the scalar mean / sample std of the window's X).
 * Outputs per window: r (P), prediction (P), true value y[n] (P). */
int dfm_windows_forecast(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                         const double *X, int64_t T, int64_t N, int64_t ldx, int P, int crit,
                         int kmax, int64_t *r_out, double *pred_out, double *true_out);
/* dfm_windows with the inputs already resident in HBM (y_dev: T, w_dev: ldw x q
 * column-major, X_dev: column-major T x N with leading dimension ldx, all on the
 * context's device); outputs as dfm_windows, in host memory (a few hundred
 * bytes per window).  A multi-GPU caller shards the windows by truncating the
 * panel: windows [w0, w1) of (T, P) are windows 0..w1-w0-1 of the leading
 * T - P + w1 rows with P' = w1 - w0 (window w only reads rows < T - P + w). */
int dfm_windows_dev(dfm_ctx *ctx, const double *y_dev, const double *w_dev, int q, int64_t ldw,
                    const double *X_dev, int64_t T, int64_t N, int64_t ldx, int P, int crit,
                    int kmax, int64_t *r_out, double *V_out, double *crit_out, double *eig_out,
                    double *coef_out, double *tstat_out);

/* pseudo_out_of_sample_forecasts(model, y, w, x, model_args...) (src/utils.jl:54-72)
 * for every model_args form of the DynamicFactorModel constructors, and rolling
 * windows (BASELINE configs[4]: "rolling-window factor re-estimation").
 *   kind DFM_WIN_EXPANDING: window w = rows 0 .. T-P+w-1 (the reference's loop);
 *   kind DFM_WIN_ROLLING:   window w = the `length` rows T-P+w-length .. T-P+w-1.
 *   r > 0:  the workhorse constructor at fixed r (src/DynamicFactorModel.jl:28),
 *           r_w = min(r, ceil(m_w/2)) (:116-119), criterion value of crit at r_w
 *           (crit = DFM_CRIT_NONE: NaN, D3);
 *   r == 0: the IC-sweep constructor (:53-66) by crit over k = 1..kmax_w (as dfm_windows);
 *   r < 0:  the 3-arg constructor's default r_w = ceil(m_w/2) (D2).
 *   breaks (nbreaks > 0, expanding windows only): model_args' break_indices
 *           (0-based first rows of blocks 2..; all inside the first window), the
 *           same rows in every refit; each window is then a break-aware fit
 *           (dfm_model_fit_breaks on its rows, D7) and forecasts through dfm_predict.
 * dev != 0: y, w, X are device pointers (as dfm_windows_dev).  Outputs as
 * dfm_windows with K = the widest window's r_w bound; pred_out / true_out (P
 * each, both or neither) add the forecast step (as dfm_windows_forecast). */
enum dfm_window_kind { DFM_WIN_EXPANDING = 0, DFM_WIN_ROLLING = 1 };
typedef struct dfm_window_spec {
  int32_t kind, length, r, crit, kmax, nbreaks;
  const int64_t *breaks;
} dfm_window_spec;
int dfm_windows_ex(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                   const double *X, int64_t T, int64_t N, int64_t ldx, int P,
                   const dfm_window_spec *spec, int dev, int64_t *r_out, double *V_out,
                   double *crit_out, double *eig_out, double *coef_out, double *tstat_out,
                   double *pred_out, double *true_out);

/* --------------------------------------------------- targeted predictors
 * targeted_predictors(..., thresholding="hard") (src/targeted_predictors.jl:9-30).
 * JOINT: OLS of y on [w x], White HC0, |t_x| > crit_value (the reference's
 * t_{0.975}(T-q-N) is passed in by the caller: no quantile code on device).
 * PER_CANDIDATE: y on [w x_i] for each i (extension, defect D8).
 * tstat (N) and mask (N, 0/1) are host outputs. */
int dfm_targeted_hard(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                      const double *X, int64_t T, int64_t N, int64_t ldx, int mode,
                      double crit_value, double *tstat, uint8_t *mask);

/* targeted_predictors(..., thresholding="soft") (src/targeted_predictors.jl:31-36):
 * GLMNet.glmnetcv(Z = [w x], y), gaussian lasso (alpha = 1) with standardised
 * columns and an intercept; keep the x columns with a nonzero coefficient at
 * the CV-optimal lambda.  GLMNet is never imported by the reference (D5): the
 * algorithm is glmnet's Fortran elnet1 in its loop order (covariance updates,
 * full cyclic passes with in-pass entry, active-set passes, threshold 1e-7,
 * warm starts over `nlambda` log-spaced lambdas from lambda_max down to
 * lambda_min_ratio * lambda_max (<= 0: 1e-2 if T < q + N else 1e-4), early
 * path exit on the full fit after 5 lambdas when R^2 gains < 1e-5 relative or
 * R^2 > 0.999; no cap on the active set below 4096).  folds: T fold ids 1..K (host-drawn, as the
 * bootstrap draws).  Outputs: path length L, best (0-based argmin of the
 * fold-size-weighted hold-out MSE), lambda (L, original units), meanloss (L),
 * beta (q + N, original scale, at best), intercept a0, mask (N, 0/1).  Any
 * output pointer may be NULL. */
int dfm_targeted_soft(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                      const double *X, int64_t T, int64_t N, int64_t ldx, const int32_t *folds,
                      int nlambda, double lambda_min_ratio, int *nlam_out, int *best_out,
                      double *lambda_out, double *meanloss_out, double *beta_out, double *a0_out,
                      uint8_t *mask);

/* glmnet's elnet1 lasso path (the core of dfm_targeted_soft, for direct use
 * and parity tests): G p x p symmetric (row-major) with unit diagonal over the
 * non-constant columns ju, c = Zs'ys/n, lambdas alms[nlam] in standardised
 * units (decreasing), early = glmnet's early path exit (5 lambdas, R^2 gain
 * < 1e-5 R^2 or R^2 > 0.999), thr = glmnet's threshold (1e-7).  Outputs: the
 * path length *L_out, betas (L x p row-major), rsq (L); NULL skips. */
int dfm_lasso_path(dfm_ctx *ctx, const double *G, const double *c, const uint8_t *ju, int p,
                   const double *alms, int nlam, int early, double thr, double *betas, double *rsq,
                   int *L_out);

/* Launch record of the lasso path kernel (process-wide, every context).  Its
 * leader and helper workgroups meet through bounded spins; each spin that
 * runs out is counted here (and described on stderr and in dfm_last_error)
 * instead of passing silently.  out[i] for i < n (slots below); reset != 0
 * zeroes the record after reading.  Returns DFM_LASSO_NSTATS. */
enum {
  DFM_LASSO_STAT_LAUNCHES = 0,   /* kernel launches, relaunches included */
  DFM_LASSO_STAT_RELAUNCHES,     /* launches after a failed hand-off */
  DFM_LASSO_STAT_TIMEOUTS,       /* timed-out spins, all kinds */
  DFM_LASSO_STAT_TASK_TMO,       /* workgroups whose first timeout was a helper's task poll */
  DFM_LASSO_STAT_DONE_TMO,       /* ... a leader's wait for its helpers */
  DFM_LASSO_STAT_PIPE_TMO,       /* ... a leader's in-workgroup pipeline wait */
  DFM_LASSO_STAT_BUDGET,         /* ... a leader's whole-path time budget */
  DFM_LASSO_STAT_RECOVERED,      /* timed-out polls whose re-read then found the granule */
  DFM_LASSO_STAT_MAX_SKEW_US,    /* max spread of the workgroups' entry times in one launch (us) */
  DFM_LASSO_STAT_LATE_ENTRIES,   /* launches where a workgroup entered after another had exited */
  DFM_LASSO_STAT_MAX_KERNEL_US,  /* longest kernel: first entry to last exit (us) */
  DFM_LASSO_STAT_MAX_HOST_US,    /* longest launch + synchronisation seen by the host (us) */
  DFM_LASSO_STAT_SLOW_LAUNCHES,  /* launches whose host time exceeded 2x the kernel + 50 ms */
  DFM_LASSO_STAT_WAVE_SPLITS,    /* launches where one workgroup's waves left > 1 ms apart */
  DFM_LASSO_NSTATS
};
int dfm_lasso_stats(int64_t *out, int n, int reset);

#ifdef __cplusplus
}
#endif
#endif /* DFM_H */
