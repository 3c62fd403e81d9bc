// dfm_api.hip — the C ABI of include/dfm.h: context, model fit, bootstrap.
// Host-side orchestration only; all arithmetic runs in the kernels of
// dfm_gram.hip (K1), dfm_eig.hip (K2), dfm_model.hip / dfm_chow.hip (K3).
#include "dfm_common.h"
#include "../../include/dfm.h"
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dfm {
hipError_t launch_gram(int orient, const PanelSrc &src, int m, int K, int T, double *G, int64_t ldg,
                       int64_t strideG, int nrep, hipStream_t st);
typedef void (*timer_fn)(void *ctx, int cls, int begin);
int eig_run(const double *G, int64_t ldg, int64_t strideG, int m, int nb, int k, int p,
            const double *warm, int kw, double tol, int maxit, int poll, char *ws, double *lam,
            double *Uk, double *trace_out, int *status, int *iters_host, hipStream_t st,
            timer_fn tf, void *tctx, int64_t rep0, int subspace = 0);
size_t eig_workspace_bytes_padded(int m, int nb, int P, int maxit);
const int *eig_iters_ptr(char *ws, int m, int nb, int P, int maxit);
int eig_block_p(int m, int k, int req);
int fact_block_p(int m, int k, int req);
extern thread_local int g_last_iters;   // per host thread: dfm_bootstrap_multi's shards run concurrently
extern thread_local int64_t g_last_rep_iters;
extern thread_local int64_t g_last_gemm_products;
int spectrum_max();
int spectrum_any_max();
int64_t spectrum_work(int m, int nb);
int dense_eig_max();
int launch_factors_wide(int orient, const double *X, int64_t ld, int T, int N, int k, const double *Uk,
                        double *F, double *L, double *colssr, hipStream_t st, double Ts, int nb = 1, int64_t sX = 0,
                        int64_t fstride = 0);
hipError_t launch_materialize(const PanelSrc &src, int T, int N, int64_t ld, int nb, double *X, hipStream_t st);
int64_t chow_wide_work(int T, int N, int r);
hipError_t launch_chow_wide(int nb, const double *X, int64_t ld, int64_t sX, const double *E, int T, int N, int r,
                            int bp, const double *F, int64_t sF, const double *L, int64_t sL, double *LR, double *LM,
                            double *WD, int64_t ostr, double *scr, double *work, hipStream_t st, int nblk = 1,
                            const int *brow = nullptr, int64_t lbs = 0);
hipError_t launch_ols_wide_batched(int nb, const double *y, const double *w, int q, const double *F, int T, int kF,
                                   int k, const int *Tn, double *coef, double *tstat, double *cov_out,
                                   double *resid_out, int *status, double *work, hipStream_t st, int hc0 = 0);
hipError_t launch_targeted_joint_wide(const double *y, const double *w, int q, const double *X, int64_t ld, int T,
                                      int N, double cv, double *tx, uint8_t *mask, int *status, double *work,
                                      hipStream_t st);
int64_t targeted_joint_wide_work(int T, int q, int N, int64_t ld);
int64_t ols_wide_work(int T, int d);
hipError_t launch_ols_wide(const double *y, const double *w, int q, const double *F, int T, int k, double *coef,
                           double *tstat, double *cov_out, double *resid_out, int *status, double *work,
                           hipStream_t st);
int64_t dense_eig_work(int m, int k);
hipError_t launch_dense_eig(const double *G, int64_t ldg, int m, int k, double *lam, double *Uk, double *trace,
                            int *status, double *work, hipStream_t st);
hipError_t launch_dense_eig_batched(const double *G, int64_t ldg, int64_t strideG, int m, int mv0, int dmv, int nb,
                                    int k, double *lam, double *Uk, double *trace, int *status, double *work,
                                    hipStream_t st);
hipError_t launch_spectrum_var(const double *G, int64_t ldg, int64_t strideG, int m, int m0, int dm, int nb,
                               double *ev, double *work, hipStream_t st);
hipError_t launch_spectrum(const double *G, int64_t ldg, int64_t strideG, int m, int nb, double *ev, double *work,
                           hipStream_t st);
// dfm_model.hip
__global__ void panel_from_colmajor_kernel(const double *, int64_t, int, int, double *, int64_t);
__global__ void colmajor_from_rows_kernel(const double *, int64_t, int, int, double *);
bool launch_factors_cols_fact(const double *Ep, int64_t ld, int T, int N, int k, const double *Fb, const double *Lb,
                              int rb, const int32_t *idx, const double *eta, int64_t rs, int nb, const double *Uk,
                              double *F, double *L, int64_t fstride, double *G, hipStream_t st);
double *gram_wk_scratch(double *work, int T, int N, int r, int nb);
int launch_factors(int orient, const PanelSrc &src, int T, int N, int k, int nb, const double *Uk,
                   double *F, double *L, double *colssr, hipStream_t st, double Ts = 0, int64_t fstride = 0);
__global__ void colssr_cols_kernel(const double *, int64_t, int64_t, int, int, const double *,
                                   const double *, double *);
__global__ void common_residual_kernel(const double *, int64_t, int, int, int, const double *,
                                       const double *, double *, double *);
__global__ void panel_row_ssq_kernel(const double *, int64_t, int, double *);
__global__ void col_ssq_kernel(const double *, int64_t, int, int, double *);
__global__ void block_accum_kernel(const double *, const double *, int, int, double *, double *, int);
__global__ void ordered_sum_kernel(const double *, int, double *);
hipError_t launch_ols(int nb, hipStream_t st, const double *y, const double *w, int q, const double *F, int Tphys,
                      int kF, const int *Tn, const int *kr, double *coef, double *tstat, double *cov_out,
                      double *resid_out, int *status,
                      const int *R0 = nullptr);
struct StatDesc { int kind, arg0, arg1, off; };
__global__ void stats_kernel(int, int, int, int, int, int, double, const double *, const double *, const double *,
                             const double *, const double *, const int *, const StatDesc *, int, double *, int64_t,
                             const int *, const int *, int *);
__global__ void tail_sigma2_kernel(const double *, int, int, int, double, double *);
// dfm_chow.hip
hipError_t launch_chow(int orient, const PanelSrc &src, int T, int N, int r, int bp, int nb,
                       const double *F, const double *Lm, double *LR, double *LM, double *Wald,
                       int64_t out_stride, char *ws, size_t ws_bytes, hipStream_t st, int nblk = 1,
                       const int *brow = nullptr, int64_t lbs = 0);
size_t chow_workspace_bytes(int T, int N, int r, int nb);
struct FactBase {   // layout shared with dfm_eig.hip's definition
  int T, r;
  int64_t ldH;
  const double *F, *EL, *S, *H, *cF, *hd;
  const double *FtF = nullptr;
};
__global__ void eig_trace_kernel(const double *__restrict__ G, int64_t ldg, int64_t strideG, int m,
                                 double *__restrict__ trace);
int eig_run_factored(const FactBase &fb, const int32_t *idx, const double *eta, int nb, int k, int p,
                     const double *warm, int kw, double tol, int maxit, int poll, char *ws, char *fws,
                     double *lam, double *Uk, double *trace_out, int *status, hipStream_t st,
                     timer_fn tf, void *tctx, int *off, int *lst, long long *cnt = nullptr, int subspace = 0,
                     double spread = 0.0, const PollBuf *pb = nullptr);
size_t fact_workspace_bytes(int T, int nb, int P);
int fact_t_max();
int fact_loadings(const FactBase &fb, const double *Ep, int64_t ld, int N, const double *Lb,
                  const double *Uk, const double *eta, const int *off, const int *lst, int nb,
                  double *Fout, double *Lout, char *ws, hipStream_t st);
size_t fact_loadings_bytes(int T, int N, int r, int nb);
hipError_t gram_wk_precompute(const double *Ep, int64_t ld, int T, int N, int r, const double *F, const double *L,
                              double *K, double *A0, hipStream_t st);
size_t gram_wk_work(int T, int N, int r, int nb);
int64_t gram_wk_ldk(int N);
int gram_wk_tp(int T);
size_t gram_wk_prep_lds(int T, int r);
hipError_t launch_gram_wk(const double *Ep, int64_t ld, int T, int N, int r, const double *F, const double *L,
                          const double *K, const double *A0, const int32_t *idx, const double *eta, int64_t rs,
                          int nb, double *work, double *G, hipStream_t st);
hipError_t launch_fact_fsf(int T, int r, const double *Fb, const double *S, double *FSF, int64_t ldH, hipStream_t st);
hipError_t launch_gram_fact(const FactBase &fb, const double *FSF, const int32_t *idx, const double *eta, int nb,
                            double *G, int64_t ldg, int64_t strideG, hipStream_t st);
hipError_t launch_predict(const double *Xp, int64_t ld, int T, int N, const double *L, int r, const double *x_dev,
                          int64_t ldx, int64_t nn, const double *w_dev, int64_t ldw, int q, const double *beta_dev,
                          double *work, double *F_out, double *yhat, hipStream_t st);
int fact_precompute(const double *Ep, int64_t ld, int T, int N, int r, const double *Lb, const double *Fb,
                    const double *H, int64_t ldH, double *EL, double *S, double *cF, double *hd, hipStream_t st);
hipError_t launch_fact_ftf(const FactBase &fb, double *FtF, hipStream_t st);
hipError_t launch_targeted(int mode, const double *y, const double *w, int q, const double *Xp,
                           int64_t ld, int T, int N, double cv, double *tstat, uint8_t *mask,
                           char *ws, size_t ws_bytes, hipStream_t st, int *bad);
size_t targeted_workspace_bytes(int mode, int T, int N, int q);
}  // namespace dfm

using namespace dfm;

static const char *kclass_names[DFM_KC_COUNT] = {"gram", "eig_gq", "eig_small", "eig_apply",
                                                 "eig_other", "factors", "ols", "stats", "chow",
                                                 "misc", "gemm"};

struct dfm_ctx {
  int device = 0;
  int refs = 1;            // the caller's handle + one per live dfm_model
  bool closed = false;
  hipStream_t own = nullptr, stream = nullptr;
  std::string err;
  double tol = 1e-12;   // residual <= tol * eigen-gap (see eig_gq_kernel)
  // bootstrap calls whose statistics depend on eigenvalues only: Ritz values
  // within this relative bound (Kato-Temple, check_converged); <= 0 = strict
  double tol_values = 1e-12;
  int maxit = 400, block = 0, poll = 4;
  bool timing = false;
  std::vector<hipEvent_t> pool;
  struct Pend { int cls; hipEvent_t a, b; };
  std::vector<Pend> pend;
  hipEvent_t cur_a[DFM_KC_COUNT] = {};
  double ms[DFM_KC_COUNT] = {};
  int64_t launches[DFM_KC_COUNT] = {};
  int64_t eig_batches = 0, eig_iters = 0, eig_iters_max = 0, rep_iters = 0, gemm_products = 0;
  // factored runs accumulate {replicate-iterations, GEMM replicate-products}
  // here on the device (no host sync after the eigen loop); read on query
  long long *cnt_dev = nullptr;
  // expanding-windows scratch: one arena reused call to call (stream-ordered),
  // grown to the largest call's need — no per-call pool malloc/free on the host
  char *warena = nullptr;
  size_t warena_cap = 0, warena_need = 0;
  hipEvent_t gate = nullptr;   // bootstrap_lanes: the second lane starts behind the caller's prior work
  hipMemPool_t mpool = nullptr;  // this context's stream-ordered scratch (stream_malloc)
  PollBuf pollbuf;               // pinned convergence read-backs of the factored solver (host == nullptr: none)
  // the bootstrap lanes' contexts whose kernel timings this context reports:
  // merged when the timings are read (harvesting a lane's events after every
  // call put ~30 hipEventElapsedTime calls between a timed job's steps)
  std::vector<dfm_ctx *> kids;
};
static const PollBuf *ctx_poll(const dfm_ctx *c) { return c->pollbuf.host ? &c->pollbuf : nullptr; }

// stream -> the owning context's pool (stream_malloc); guarded: contexts are
// created, re-streamed and destroyed from any host thread.  One entry per
// context (a context re-registers after dfm_ctx_set_stream).  A stream that
// several contexts are bound to (dfm_ctx_set_stream with a shared external
// stream) is served by the device's default pool instead of either context's
// own: a context's pool then never holds blocks another context allocated,
// so destroying one context (hipMemPoolDestroy) cannot free memory still in
// flight on the other's calls.
static std::mutex g_pool_mu;
static std::vector<std::pair<hipStream_t, hipMemPool_t>> g_pools;
static void pool_register(hipStream_t st, hipMemPool_t pool) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  g_pools.emplace_back(st, pool);
}
static void pool_unregister(hipMemPool_t pool) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  g_pools.erase(std::remove_if(g_pools.begin(), g_pools.end(), [&](const auto &e) { return e.second == pool; }),
                g_pools.end());
}
namespace dfm {
hipError_t stream_malloc(void **p, size_t bytes, hipStream_t st) {
  hipMemPool_t pool = nullptr;
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    int owners = 0;
    for (auto &e : g_pools)
      if (e.first == st) { pool = e.second; ++owners; }
    if (owners > 1) pool = nullptr;   // a shared stream: the default pool
  }
  const hipError_t e = pool ? hipMallocFromPoolAsync(p, bytes, pool, st) : hipMallocAsync(p, bytes, st);
  if (e == hipSuccess) DFM_POISON_ASYNC(*p, bytes, st);
  return e;
}

// The device gate (dfm_common.h): per device, a count of library calls in
// progress and a solo flag.  Shares wait only while a solo section runs
// (reader-preferring, so a call holding a share can always start more shared
// calls on other threads — dfm_bootstrap_multi's shards — without deadlocking
// behind a waiting solo); a solo section waits for the count to reach zero.
namespace {
struct DevGate {
  std::mutex mu;
  std::condition_variable cv;
  int shares = 0;
  bool solo = false;
};
constexpr int kGateDevs = 64;
DevGate g_gate[kGateDevs];
thread_local int t_shares[kGateDevs];   // this thread's nesting depth per device
}  // namespace
DeviceShare::DeviceShare(int device) : dev(device >= 0 && device < kGateDevs ? device : -1) {
  if (dev < 0 || t_shares[dev]++ > 0) return;
  DevGate &g = g_gate[dev];
  std::unique_lock<std::mutex> lk(g.mu);
  g.cv.wait(lk, [&] { return !g.solo; });
  ++g.shares;
}
DeviceShare::~DeviceShare() {
  if (dev < 0 || --t_shares[dev] > 0) return;
  DevGate &g = g_gate[dev];
  {
    std::lock_guard<std::mutex> lk(g.mu);
    --g.shares;
  }
  g.cv.notify_all();
}
DeviceSolo::DeviceSolo(int device) : dev(device >= 0 && device < kGateDevs ? device : -1) {
  if (dev < 0 || t_shares[dev] > 0) { dev = -1; return; }   // (nested in a shared call: would never drain)
  DevGate &g = g_gate[dev];
  std::unique_lock<std::mutex> lk(g.mu);
  g.cv.wait(lk, [&] { return !g.solo && g.shares == 0; });
  g.solo = true;
  held = true;
}
DeviceSolo::~DeviceSolo() {
  if (!held) return;
  DevGate &g = g_gate[dev];
  {
    std::lock_guard<std::mutex> lk(g.mu);
    g.solo = false;
  }
  g.cv.notify_all();
}
}  // namespace dfm

// The host thread of a model's second bootstrap lane (bootstrap_lanes):
// persistent, so a call costs a hand-off, not a thread start.  Both sides of
// the hand-off spin briefly (kSpin) before blocking: in a run of jobs the next
// job, and the lane's finish, come within microseconds, and a condition
// variable wake-up (~10-20 us) sat in front of the lane's first kernel and
// behind its last one on every call.
struct LaneWorker {
  static constexpr std::chrono::microseconds kSpin{200};
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;   // guarded by mu
  std::atomic<bool> has{false}, done{false}, quit{false};
  std::thread th;   // last: starts after the members it uses
  LaneWorker() : th([this] { loop(); }) {}
  template <class F>
  static void spin(F ready) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!ready() && std::chrono::steady_clock::now() - t0 < kSpin) __builtin_ia32_pause();
  }
  void loop() {
    for (;;) {
      spin([&] { return has.load(std::memory_order_acquire) || quit.load(std::memory_order_acquire); });
      std::function<void()> j;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return has.load() || quit.load(); });
        if (quit.load()) return;
        j = std::move(job);
        has.store(false);
      }
      j();
      {
        std::lock_guard<std::mutex> g(mu);
        done.store(true, std::memory_order_release);
      }
      cv.notify_all();
    }
  }
  void run(std::function<void()> j) {
    {
      std::lock_guard<std::mutex> g(mu);
      job = std::move(j);
      done.store(false);
      has.store(true, std::memory_order_release);
    }
    cv.notify_all();
  }
  void wait() {
    spin([&] { return done.load(std::memory_order_acquire); });
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done.load(); });
  }
  ~LaneWorker() {
    {
      std::lock_guard<std::mutex> g(mu);
      quit.store(true);
    }
    cv.notify_all();
    th.join();
  }
};

struct dfm_model {
  dfm_ctx *ctx = nullptr;
  int T = 0, N = 0, q = 0, r = 0, crit = -1, kmax = 0, m = 0, orient = 0, k_eig = 0;
  bool swept = false;   // IC sweep ran (r chosen by criterion)
  int64_t ld = 0;
  double *Xp = nullptr, *Cp = nullptr, *Ep = nullptr, *y = nullptr, *w = nullptr;
  double *F = nullptr, *L = nullptr, *Ub = nullptr, *colssr = nullptr;
  std::vector<double> lam, coef, tstat, cov, resid, ic;
  double trace = 0, V = 0, critval = NAN, sigma2 = NAN;
  int64_t batch = 0;
  char *ws = nullptr;
  size_t ws_bytes = 0;
  StatDesc *sd_dev = nullptr;
  int sd_cap = 0;
  std::vector<StatDesc> sd_host;   // what sd_dev holds (uploaded only when a call's descriptors differ)
  int *flag_dev = nullptr;
  // factored bootstrap (N > T): H = E E', EL = E L, S = L'L, cF, hd
  int mode = 0;   // 0 auto, 1 direct Gram, 2 factored
  bool fact_ready = false;
  int64_t ldH = 0;
  double *H = nullptr, *EL = nullptr, *S = nullptr, *cF = nullptr, *hd = nullptr;
  double *FtF = nullptr;   // F'F (16 x 16): the factored solver's middle Horner steps
  double *FSF = nullptr;   // F S F' (T x ldH): the direct path's identity-based replicate Grams
  // T >= N bootstrap Grams by one weighted-outer-product GEMM (gram_wk_*):
  // K = [E_s' E_s] lower-triangle pairs (Tp x ldk) and A0 = C'C (N x N)
  double *Kwk = nullptr, *A0wk = nullptr;
  // break blocks (src/DynamicFactorModel.jl:73, :98): first row, rows, Gram
  // size, per-block eigenvectors (Gram size x r) and loadings (N x r); block 0's
  // are aliased by Ub and L
  int nblk = 1;
  std::vector<int> ba, bt, bm;
  std::vector<double *> Ubs, Ls;   // Ls[j] = Lall + j N r (contiguous: the Chow kernels index blocks)
  double *Lall = nullptr;
  std::vector<std::vector<double>> blam;
  // dfm_chow: the all-variables statistics of the last break period asked for
  int64_t chow_bp = -1;
  std::vector<double> chow_cache;   // LR (N), LM (N), Wald (N)
  // the extra lanes of small factored bootstrap jobs (dfm_bootstrap_dev):
  // clones of this fit, each on its own context / stream of the same device
  // and driven by its own host thread, made on first use
  static constexpr int kMaxLanes = 4;
  dfm_model *lane[kMaxLanes - 1] = {};
  LaneWorker *lane_worker[kMaxLanes - 1] = {};
  bool is_lane = false;
  dfm_ctx *count_ctx = nullptr;   // a lane counts its GEMM products into its parent's context
};

static int fail(dfm_ctx *ctx, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}
#define HIPCHK(ctx, x)                                                                            \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      return fail(ctx, 1000 + (int)e_, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                                      \
  } while (0)

static void timer_cb(void *p, int cls, int begin) {
  dfm_ctx *ctx = (dfm_ctx *)p;
  if (!ctx->timing) return;
  auto get = [&]() {
    hipEvent_t e;
    if (!ctx->pool.empty()) { e = ctx->pool.back(); ctx->pool.pop_back(); }
    else hipEventCreate(&e);
    return e;
  };
  if (begin) {
    ctx->cur_a[cls] = get();
    hipEventRecord(ctx->cur_a[cls], ctx->stream);
  } else {
    hipEvent_t b = get();
    hipEventRecord(b, ctx->stream);
    ctx->pend.push_back({cls, ctx->cur_a[cls], b});
    ctx->launches[cls]++;
  }
}
static void harvest(dfm_ctx *ctx) {
  if (ctx->pend.empty()) return;
  hipEventSynchronize(ctx->pend.back().b);
  for (auto &p : ctx->pend) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, p.a, p.b);
    ctx->ms[p.cls] += ms;
    ctx->pool.push_back(p.a);
    ctx->pool.push_back(p.b);
  }
  ctx->pend.clear();
}
// a lane context's timings into its parent's (read / reset time, lane teardown)
static void merge_kid(dfm_ctx *ctx, dfm_ctx *kid) {
  harvest(kid);
  for (int i = 0; i < DFM_KC_COUNT; ++i) {
    ctx->ms[i] += kid->ms[i]; ctx->launches[i] += kid->launches[i];
    kid->ms[i] = 0; kid->launches[i] = 0;
  }
}
static void merge_kids(dfm_ctx *ctx) {
  for (dfm_ctx *k : ctx->kids) merge_kid(ctx, k);
}
struct Scope {
  dfm_ctx *c; int cls;
  Scope(dfm_ctx *c_, int k) : c(c_), cls(k) { timer_cb(c, cls, 1); }
  ~Scope() { timer_cb(c, cls, 0); }
};

namespace dfm {
int ctx_fail(dfm_ctx *ctx, int code, const char *msg) { return fail(ctx, code, "%s", msg); }
hipStream_t ctx_stream(dfm_ctx *ctx) { return ctx->stream; }
int ctx_device(dfm_ctx *ctx) { return ctx->device; }
}  // namespace dfm

static int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }
static bool chow_stat(int k) { return k >= DFM_STAT_LR && k <= DFM_STAT_WALD_ALL; }
static bool all_var_stat(int k) { return k >= DFM_STAT_LR_ALL && k <= DFM_STAT_WALD_ALL; }
// values a stat adds to a replicate's row
static int64_t stat_width(const dfm_model *m, int k) {
  if (all_var_stat(k)) return m->N;
  if (k == DFM_STAT_FACTORS) return (int64_t)m->T * m->r;
  if (k == DFM_STAT_LOADINGS) return (int64_t)m->N * m->r;
  return 1;
}
static int ceil_half(int m) { return (m + 1) / 2; }
// src/criteria.jl:17-53 at k factors: V(k), PCp's sigma^2 (V of the
// unrestricted fit), c = (N + T) / (N T), m = min(T, N)
static double crit_formula(int crit, double V, int k, double sigma2, int T, int N) {
  const double NT = (double)N * (double)T, c = (double)(N + T) / NT, m = (double)std::min(T, N);
  switch (crit) {
    case 0: return V + k * sigma2 * c * std::log(1.0 / c);
    case 1: return V + k * sigma2 * c * std::log(m);
    case 2: return V + k * sigma2 * std::log(m) / m;
    case 3: return std::log(V) + k * c * std::log(1.0 / c);
    case 4: return std::log(V) + k * c * std::log(m);
    case 5: return std::log(V) + k * std::log(m) / m;
    case 6: return V + k * std::log((double)T) / T;
  }
  return NAN;
}

template <class T>
static hipError_t dalloc(T **p, size_t n) {
  const hipError_t e = hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T));
  if (e == hipSuccess) DFM_POISON_SYNC(*p, std::max<size_t>(n, 1) * sizeof(T));
  return e;
}

extern "C" {

int dfm_ctx_create(int device, dfm_ctx **out) {
  if (!out) return -1;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return -2;
  dfm_ctx *c = new dfm_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) { delete c; return -3; }
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) { delete c; return -4; }
  c->stream = c->own;
  if (hipMalloc((void **)&c->cnt_dev, 2 * sizeof(long long)) != hipSuccess ||
      hipMemsetAsync(c->cnt_dev, 0, 2 * sizeof(long long), c->stream) != hipSuccess) {
    hipStreamDestroy(c->own);
    delete c;
    return -4;
  }
  {   // stream-ordered scratch (split-K Gram partials, eigen workspaces) from
      // the context's own pool, kept mapped between calls
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    uint64_t keep = UINT64_MAX;
    if (hipMemPoolCreate(&c->mpool, &props) == hipSuccess) {
      hipMemPoolSetAttribute(c->mpool, hipMemPoolAttrReleaseThreshold, &keep);
      pool_register(c->stream, c->mpool);
    } else {
      c->mpool = nullptr;   // the default pool then serves this context (stream_malloc's fallback)
    }
    hipMemPool_t dp;
    if (hipDeviceGetDefaultMemPool(&dp, device) == hipSuccess) hipMemPoolSetAttribute(dp, hipMemPoolAttrReleaseThreshold, &keep);
  }
  {   // the factored solver's look-ahead polls (without them it polls blocking)
    PollBuf &pb = c->pollbuf;
    constexpr int kCap = 4096;
    if (hipHostMalloc((void **)&pb.host, kCap * sizeof(int), hipHostMallocDefault) == hipSuccess &&
        hipEventCreateWithFlags(&pb.ev[0], hipEventDisableTiming) == hipSuccess &&
        hipEventCreateWithFlags(&pb.ev[1], hipEventDisableTiming) == hipSuccess) {
      pb.cap = kCap;
    } else {
      if (pb.ev[0]) hipEventDestroy(pb.ev[0]);
      if (pb.host) hipHostFree(pb.host);
      pb = PollBuf{};
    }
  }
  *out = c;
  return 0;
}

static void ctx_release(dfm_ctx *ctx);
int dfm_ctx_destroy(dfm_ctx *ctx) {
  if (!ctx || ctx->closed) return -1;
  ctx->closed = true;
  ctx_release(ctx);
  return 0;
}
static void ctx_release(dfm_ctx *ctx) {
  if (--ctx->refs > 0) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  harvest(ctx);
  for (auto e : ctx->pool) hipEventDestroy(e);
  hipFree(ctx->cnt_dev);
  hipFree(ctx->warena);
  if (ctx->gate) hipEventDestroy(ctx->gate);
  if (ctx->pollbuf.host) {
    hipEventDestroy(ctx->pollbuf.ev[0]);
    hipEventDestroy(ctx->pollbuf.ev[1]);
    hipHostFree(ctx->pollbuf.host);
  }
  if (ctx->mpool) {
    pool_unregister(ctx->mpool);
    hipMemPoolDestroy(ctx->mpool);
  }
  if (ctx->own) hipStreamDestroy(ctx->own);
  delete ctx;
}

const char *dfm_last_error(const dfm_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dfm_ctx_set_stream(dfm_ctx *ctx, void *s) {
  if (!ctx) return -1;
  if (ctx->mpool) pool_unregister(ctx->mpool);
  ctx->stream = s ? (hipStream_t)s : ctx->own;
  if (ctx->mpool) pool_register(ctx->stream, ctx->mpool);
  return 0;
}
int dfm_ctx_synchronize(dfm_ctx *ctx) {
  if (!ctx) return -1;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}
int dfm_ctx_set_eig_params(dfm_ctx *ctx, double tol, int max_iter, int block) {
  if (!ctx) return -1;
  if (tol > 0) ctx->tol = tol;
  if (max_iter > 0) ctx->maxit = max_iter;
  if (block >= 0) ctx->block = block;
  return 0;
}
int dfm_ctx_set_value_tol(dfm_ctx *ctx, double tol) {
  if (!ctx) return -1;
  ctx->tol_values = tol;
  return 0;
}
int dfm_ctx_enable_timing(dfm_ctx *ctx, int enable) {
  if (!ctx) return -1;
  ctx->timing = enable != 0;
  if (ctx->timing) {   // events made up front, not one hipEventCreate per timed launch inside the jobs
    hipSetDevice(ctx->device);
    auto fill = [](dfm_ctx *c) {
      while (c->pool.size() < 1024) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) break;
        c->pool.push_back(e);
      }
    };
    fill(ctx);
    for (dfm_ctx *c : ctx->kids) fill(c);
  }
  return 0;
}
int dfm_ctx_read_timing(dfm_ctx *ctx, double *ms_out, int64_t *launches_out, int cap) {
  if (!ctx) return -1;
  harvest(ctx);
  merge_kids(ctx);
  const int n = std::min(cap, (int)DFM_KC_COUNT);
  for (int i = 0; i < n; ++i) {
    if (ms_out) ms_out[i] = ctx->ms[i];
    if (launches_out) launches_out[i] = ctx->launches[i];
  }
  return n;
}
int dfm_ctx_reset_timing(dfm_ctx *ctx) {
  if (!ctx) return -1;
  harvest(ctx);
  merge_kids(ctx);
  for (int i = 0; i < DFM_KC_COUNT; ++i) { ctx->ms[i] = 0; ctx->launches[i] = 0; }
  ctx->eig_batches = ctx->eig_iters = ctx->eig_iters_max = ctx->rep_iters = ctx->gemm_products = 0;
  hipMemsetAsync(ctx->cnt_dev, 0, 2 * sizeof(long long), ctx->stream);
  return 0;
}
// host totals + the device-side counters of factored runs (one sync, on query)
static void read_counts(dfm_ctx *ctx, int64_t *rep_iters, int64_t *products) {
  long long c[2] = {0, 0};
  hipMemcpyAsync(c, ctx->cnt_dev, sizeof(c), hipMemcpyDeviceToHost, ctx->stream);
  hipStreamSynchronize(ctx->stream);
  if (rep_iters) *rep_iters = ctx->rep_iters + c[0];
  if (products) *products = ctx->gemm_products + c[1];
}
int dfm_ctx_eig_stats(dfm_ctx *ctx, int64_t *batches, int64_t *iters_total, int64_t *iters_max) {
  if (!ctx) return -1;
  if (batches) *batches = ctx->eig_batches;
  if (iters_total) *iters_total = ctx->eig_iters;
  if (iters_max) *iters_max = ctx->eig_iters_max;
  return 0;
}
static void note_iters(dfm_ctx *ctx) {
  ctx->eig_batches++;
  ctx->eig_iters += g_last_iters;
  ctx->eig_iters_max = std::max<int64_t>(ctx->eig_iters_max, g_last_iters);
  ctx->rep_iters += g_last_rep_iters;
  ctx->gemm_products += g_last_gemm_products;
}
int dfm_ctx_gemm_products(dfm_ctx *ctx, int64_t *products) {
  if (!ctx || !products) return -1;
  read_counts(ctx, nullptr, products);
  return 0;
}
int dfm_ctx_rep_iters(dfm_ctx *ctx, int64_t *rep_iters) {
  if (!ctx || !rep_iters) return -1;
  read_counts(ctx, rep_iters, nullptr);
  return 0;
}
const char *dfm_kernel_class_name(int cls) {
  return (cls >= 0 && cls < DFM_KC_COUNT) ? kclass_names[cls] : "?";
}
int dfm_full_spectrum_max(void) { return spectrum_any_max(); }

int dfm_ic_sweep(const double *eig, int n_eig, int kmax, double trace, int64_t T, int64_t N,
                 double sigma2, double *out) {
  if (!eig || !out || kmax < 1 || n_eig < kmax || T < 1 || N < 1) return -1;
  const int m = (int)std::min(T, N);
  if (sigma2 < 0) {
    const int kh = ceil_half(m);
    if (n_eig < kh) return -2;
    double s = trace;
    for (int j = 0; j < kh; ++j) s -= eig[j];
    sigma2 = s / ((double)N * (double)T);
  }
  const double c = (double)(N + T) / ((double)N * (double)T);
  double cum = trace;
  for (int k = 1; k <= kmax; ++k) {
    cum -= eig[k - 1];
    const double V = cum / ((double)N * (double)T);
    out[0 * kmax + k - 1] = V + k * sigma2 * c * std::log(1.0 / c);
    out[1 * kmax + k - 1] = V + k * sigma2 * c * std::log((double)m);
    out[2 * kmax + k - 1] = V + k * sigma2 * std::log((double)m) / m;
    out[3 * kmax + k - 1] = std::log(V) + k * c * std::log(1.0 / c);
    out[4 * kmax + k - 1] = std::log(V) + k * c * std::log((double)m);
    out[5 * kmax + k - 1] = std::log(V) + k * std::log((double)m) / m;
    out[6 * kmax + k - 1] = V + k * std::log((double)T) / T;
  }
  return 0;
}

}  // extern "C"

// device buffer freed on every return path
struct DevBuf {
  double *p = nullptr;
  ~DevBuf() { hipFree(p); }
};

#ifdef DFM_DEBUG_MEM
// Debug build: a device buffer inside 64 KB guard bands of 0xA5 bytes, its
// body poisoned (0xFF).  check() reports guard bytes that changed (offsets
// relative to the body: negative = the front band) and, given the host copy
// the body was loaded from, body rows that no longer match it (row = `rowb`
// bytes: a replicate's draws).
struct GuardBuf {
  static constexpr size_t kG = 65536;
  char *raw = nullptr;
  void *p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t bytes) {
    n = std::max<size_t>(bytes, 8);
    hipError_t e = hipMalloc((void **)&raw, n + 2 * kG);
    if (e != hipSuccess) return e;
    (void)hipMemset(raw, 0xA5, kG);
    (void)hipMemset(raw + kG, 0xFF, n);
    (void)hipMemset(raw + kG + n, 0xA5, kG);
    (void)hipDeviceSynchronize();
    p = raw + kG;
    return hipSuccess;
  }
  int check(const char *name, const void *host, int64_t rowb) {
    if (!raw) return 0;
    std::vector<unsigned char> h(n + 2 * kG);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h.data(), raw, h.size(), hipMemcpyDeviceToHost);
    int bad = 0;
    int64_t first = 0, last = 0, cnt = 0;
    for (size_t i = 0; i < h.size(); ++i) {
      if (i >= kG && i < kG + n) continue;
      if (h[i] != 0xA5) {
        const int64_t o = (int64_t)i - (int64_t)kG;
        if (!cnt) first = o;
        last = o;
        ++cnt;
      }
    }
    if (cnt) {
      fprintf(stderr, "[dfm debug] %s: %lld guard bytes changed, body offsets %lld .. %lld (body %zu bytes)\n", name,
              (long long)cnt, (long long)first, (long long)last, n);
      ++bad;
    }
    if (host && rowb > 0) {
      const unsigned char *b = h.data() + kG, *q = (const unsigned char *)host;
      int64_t nrow = (int64_t)n / rowb, rbad = 0, r0 = -1, r1 = -1;
      for (int64_t r = 0; r < nrow; ++r)
        if (memcmp(b + r * rowb, q + r * rowb, (size_t)rowb) != 0) {
          if (r0 < 0) r0 = r;
          r1 = r;
          ++rbad;
        }
      if (rbad) {
        fprintf(stderr, "[dfm debug] %s: %lld of %lld rows changed on the device during the call (rows %lld .. %lld)\n",
                name, (long long)rbad, (long long)nrow, (long long)r0, (long long)r1);
        ++bad;
      }
    }
    hipFree(raw);
    raw = nullptr;
    return bad;
  }
  ~GuardBuf() { if (raw) hipFree(raw); }
};
// DFM_LANE_SKEW_US (debug build): hold one bootstrap lane back this long on the
// device (> 0: the second lane, < 0: the caller's), so a cross-lane ordering
// hazard shows up deterministically instead of at the mercy of scheduling
__global__ void dbg_spin_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
static int dbg_lane_skew_us() {
  const char *e = getenv("DFM_LANE_SKEW_US");
  return e ? atoi(e) : 0;
}
#endif

#if defined(DFM_LANE_SKEW_AB) && !defined(DFM_DEBUG_MEM)
// (A/B builds only: the debug build's lane skew as a timing experiment, no poisoning)
__global__ void dbg_spin_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
static int dbg_lane_skew_us() {
  static const int v = [] { const char *e = getenv("DFM_LANE_SKEW_US"); return e ? atoi(e) : 0; }();
  return v;
}
#endif

// ---------------------------------------------------------------- internals
// Top-k eigen-decomposition of nb Grams + trace; G workspace provided.
static int run_eig(dfm_ctx *ctx, const double *G, int m, int nb, int k, const double *warm, int kw,
                   double *lam, double *Uk, double *trace, int *status_dev) {
  const int p = eig_block_p(m, k, ctx->block);
  if ((p > 32 || p < k) && nb == 1 && m >= 2 && m <= dense_eig_max()) {
    // k beyond the subspace block: tridiagonalisation + inverse iteration (dfm_spec.hip)
    double *wk = nullptr;
    HIPCHK(ctx, hipMalloc(&wk, (size_t)dense_eig_work(m, k) * 8));
    hipError_t e;
    {
      Scope sc(ctx, DFM_KC_EIG_OTHER);
      e = launch_dense_eig(G, m, m, k, lam, Uk, trace, status_dev, wk, ctx->stream);
    }
    hipStreamSynchronize(ctx->stream);
    hipFree(wk);
    if (e != hipSuccess) return fail(ctx, 1000 + (int)e, "dense eigensolver: %s", hipGetErrorString(e));
    return 0;
  }
  if (p > 32 || p < k) return fail(ctx, -20, "eigensolver block %d unsupported for k=%d m=%d", p, k, m);
  const int P = p <= 16 ? 16 : 32;
  const size_t bytes = eig_workspace_bytes_padded(m, nb, P, ctx->maxit);
  char *ws = nullptr;   // stream-ordered pool memory: no device-wide sync in the free
  HIPCHK(ctx, stream_malloc((void **)&ws, bytes, ctx->stream));
  // a single fit's eigenvectors are polished to the rounding floor (the
  // residual rule at 1e-14; the floor and stagnation tests end it): statistics
  // of the fit with a near-zero value (an LR of ~0.4 between two nearly equal
  // SSRs) move by ~1e-10 relative when its eigenvectors stop at 1e-12 of the
  // gap (a break fit's LR in tests/test_gpu_breaks.py: 4e-10 off the oracle;
  // the tridiagonal path's inverse-iteration vectors: 9e-10)
  const double tol = nb == 1 ? std::min(ctx->tol, 1e-14) : ctx->tol;
  int rc = eig_run(G, m, (int64_t)m * m, m, nb, k, p, warm, kw, tol, ctx->maxit, ctx->poll, ws,
                   lam, Uk, trace, status_dev, nullptr, ctx->stream, timer_cb, ctx, 0);
  hipFreeAsync(ws, ctx->stream);
  hipStreamSynchronize(ctx->stream);
  if (rc != 0) return fail(ctx, rc > 0 ? rc : -21, "eigensolver failed (%d)", rc);
  return 0;
}

extern "C" {

int dfm_model_destroy(dfm_model *m) {
  if (!m) return -1;
  for (int j = 0; j < dfm_model::kMaxLanes - 1; ++j) {
    delete m->lane_worker[j];
    m->lane_worker[j] = nullptr;
    if (m->lane[j]) {   // the lane model, then its context (the model held the last reference but one)
      dfm_ctx *lc = m->lane[j]->ctx;
      hipSetDevice(lc->device);
      hipStreamSynchronize(lc->stream);
      merge_kid(m->ctx, lc);   // its unread kernel timings
      auto &kd = m->ctx->kids;
      kd.erase(std::remove(kd.begin(), kd.end(), lc), kd.end());
      dfm_model_destroy(m->lane[j]);
      dfm_ctx_destroy(lc);
      m->lane[j] = nullptr;
    }
  }
  hipSetDevice(m->ctx->device);
  hipStreamSynchronize(m->ctx->stream);
  for (double *p : {m->Xp, m->Cp, m->Ep, m->y, m->w, m->F, m->Lall, m->Ub, m->colssr, m->H, m->EL, m->S,
                    m->cF, m->hd, m->FtF, m->FSF, m->Kwk, m->A0wk})
    hipFree(p);
  for (size_t j = 1; j < m->Ubs.size(); ++j) hipFree(m->Ubs[j]);
  hipFree(m->ws);
  hipFree(m->sd_dev);
  hipFree(m->flag_dev);
  dfm_ctx *ctx = m->ctx;
  delete m;
  ctx_release(ctx);
  return 0;
}

int dfm_model_fit(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                  const double *X, int64_t T64, int64_t N64, int64_t ldx, int r, int crit, int kmax,
                  dfm_model **out) {
  return dfm_model_fit_breaks(ctx, y, w, q, ldw, X, T64, N64, ldx, r, crit, kmax, nullptr, 0, out);
}

int dfm_model_fit_breaks(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                         const double *X, int64_t T64, int64_t N64, int64_t ldx, int r, int crit,
                         int kmax, const int64_t *breaks, int nbreaks, dfm_model **out) {
  if (!ctx || !out) return -1;
  DeviceShare gate(ctx->device);
  *out = nullptr;
  if (!y || !X || T64 < 2 || N64 < 1 || ldx < T64 || q < 0 || (q > 0 && (!w || ldw < T64)))
    return fail(ctx, -2, "dfm_model_fit: bad arguments");
  if (T64 > (1 << 24) || N64 > (1 << 24)) return fail(ctx, -2, "panel too large");
  if (crit < -1 || crit > 6) return fail(ctx, -3, "unknown criterion %d", crit);
  if (r <= 0 && crit < 0) return fail(ctx, -3, "IC sweep needs a criterion");
  if (nbreaks < 0 || (nbreaks > 0 && !breaks)) return fail(ctx, -2, "dfm_model_fit: bad break list");
  for (int j = 0; j < nbreaks; ++j)   // src/DynamicFactorModel.jl:73: vcat(1, breaks, T+1)
    if (breaks[j] <= (j ? breaks[j - 1] : 0) || breaks[j] >= T64)
      return fail(ctx, -9, "break indices must increase strictly inside 1..T-1 (0-based rows)");
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  const int T = (int)T64, N = (int)N64, m = std::min(T, N);
  const int mfn = ceil_half(m);  // max_factor_number, src/DynamicFactorModel.jl:101
  dfm_model *M = new dfm_model();
  ++ctx->refs;
  M->ctx = ctx; M->T = T; M->N = N; M->q = q; M->crit = crit; M->m = m;
  // src/DynamicFactorModel.jl:77 (T >= N) vs :86 (N > T), with the FULL-sample
  // T and N for every break block (:72, defect D7)
  M->orient = (N > T) ? 0 : 1;
  M->ld = round_up(N, 16);
  const int nblk = nbreaks + 1;
  M->nblk = nblk;
  for (int j = 0; j < nblk; ++j) {
    const int a = j ? (int)breaks[j - 1] : 0, e = j < nbreaks ? (int)breaks[j] : T;
    M->ba.push_back(a);
    M->bt.push_back(e - a);
    M->bm.push_back(M->orient == 0 ? e - a : N);   // size of the block's Gram
  }
  const bool nob = nblk == 1;
  std::vector<double *> Gb(nblk, nullptr), lamd(nblk, nullptr), Ukd(nblk, nullptr);
  std::vector<double *> tmp;   // freed on every exit path below
  auto tfree = [&]() {
    for (int j = 0; j < nblk; ++j) {
      if (!nob) hipFree(Gb[j]);
      hipFree(lamd[j]); hipFree(Ukd[j]);
      Gb[j] = lamd[j] = Ukd[j] = nullptr;
    }
    for (double *p : tmp) hipFree(p);
    tmp.clear();
  };
  auto bail = [&](int code) { tfree(); dfm_model_destroy(M); return code; };
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return bail(fail(ctx, 1000 + (int)e_, "HIP %s line %d", hipGetErrorString(e_), __LINE__)); } while (0)
#define LCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail(ctx, 1000 + (int)e_, "HIP %s line %d", hipGetErrorString(e_), __LINE__); } while (0)
#define CKB(x) do { int r_ = (x); if (r_) return bail(r_); } while (0)
#define TALLOC(p, n) do { CK(dalloc(&(p), (n))); tmp.push_back((double *)(p)); } while (0)
  const size_t panel = (size_t)T * M->ld;
  CK(dalloc(&M->Xp, panel));
  CK(dalloc(&M->Cp, panel));
  CK(dalloc(&M->Ep, panel));
  CK(dalloc(&M->y, T));
  CK(dalloc(&M->w, (size_t)T * std::max(q, 1)));
  double *Xraw = nullptr;
  TALLOC(Xraw, (size_t)T * N);
  // host or device inputs (hipMemcpyDefault: the windows driver refits from a resident panel)
  CK(hipMemcpy2DAsync(Xraw, (size_t)T * 8, X, (size_t)ldx * 8, (size_t)T * 8, N, hipMemcpyDefault, st));
  CK(hipMemcpyAsync(M->y, y, (size_t)T * 8, hipMemcpyDefault, st));
  if (q > 0) CK(hipMemcpy2DAsync(M->w, (size_t)T * 8, w, (size_t)ldw * 8, (size_t)T * 8, q, hipMemcpyDefault, st));
  {
    Scope sc(ctx, DFM_KC_MISC);
    hipLaunchKernelGGL(panel_from_colmajor_kernel, dim3((unsigned)((M->ld + 31) / 32), (T + 31) / 32),
                       dim3(256), 0, st, Xraw, (int64_t)T, T, N, M->Xp, M->ld);
  }
  CK(hipGetLastError());
  // block j's panel: rows ba[j] .. ba[j] + bt[j] - 1 of X
  auto block_src = [&](int j) { return PanelSrc{nullptr, M->Xp + (size_t)M->ba[j] * M->ld, nullptr, nullptr, M->ld, 0}; };
  auto block_gram = [&](int j, double *G) -> hipError_t {
    Scope sc(ctx, DFM_KC_GRAM);
    return launch_gram(M->orient, block_src(j), M->bm[j], M->orient == 0 ? N : M->bt[j], M->bt[j], G,
                       M->bm[j], (int64_t)M->bm[j] * M->bm[j], 1, st);
  };
  auto spectrum = [&](const double *G, int mm, std::vector<double> &sp) -> int {
    double *ev = nullptr;
    LCK(dalloc(&ev, mm));
    tmp.push_back(ev);
    double *wk = nullptr;
    if (spectrum_work(mm, 1) > 0) {
      LCK(dalloc(&wk, (size_t)spectrum_work(mm, 1)));
      tmp.push_back(wk);
    }
    {
      Scope sc(ctx, DFM_KC_EIG_OTHER);
      LCK(launch_spectrum(G, mm, (int64_t)mm * mm, mm, 1, ev, wk, st));
    }
    sp.resize(mm);
    LCK(hipMemcpyAsync(sp.data(), ev, (size_t)mm * 8, hipMemcpyDeviceToHost, st));
    LCK(hipStreamSynchronize(st));
    return 0;
  };
  const bool pcp = crit >= 0 && crit <= 2;
  if (kmax <= 0) kmax = mfn;  // src/DynamicFactorModel.jl:54 (D11)
  kmax = std::min(kmax, mfn);
  M->kmax = kmax;
  const double NT = (double)N * (double)T;
  // --- PCp's sigma^2 = V(ceil(m/2)) of the UNRESTRICTED fit DynamicFactorModel(y, w, x):
  // full sample, no breaks (src/criteria.jl:18, :23, :28)
  double *Gfull = nullptr;
  std::vector<double> spec_full;
  // the sweep reports all 7 criteria: PCp rows need sigma^2 (NaN when the full
  // spectrum is out of reach and the chosen criterion is not a PCp one)
  const bool full_spec = pcp || (nob && r <= 0 && (kmax > 24 || m <= spectrum_max()));
  if (full_spec && m > spectrum_any_max()) {
    return bail(fail(ctx, -30, "PCp criteria / kmax > 24 need the full spectrum; supported for "
                               "min(T,N) <= %d (got %d)", spectrum_any_max(), m));
  }
  if (nob || full_spec) {
    TALLOC(Gfull, (size_t)m * m);
    PanelSrc src{nullptr, M->Xp, nullptr, nullptr, M->ld, 0};
    Scope sc(ctx, DFM_KC_GRAM);
    CK(launch_gram(M->orient, src, m, M->orient == 0 ? N : T, T, Gfull, m, (int64_t)m * m, 1, st));
  }
  if (full_spec) {
    CKB(spectrum(Gfull, m, spec_full));
    double s = 0.0;
    for (double v : spec_full) s += v;
    for (int j = 0; j < mfn; ++j) s -= spec_full[j];
    M->sigma2 = s / NT;
  }
  // --- per block: Gram, the eigenvalues the sweep needs, trace
  std::vector<int> kk(nblk, 0);
  std::vector<std::vector<double>> bev(nblk), blam(nblk);
  std::vector<double> btr(nblk, 0.0);
  double *tr_d = nullptr;
  int *st_d = nullptr;
  TALLOC(tr_d, 1);
  CK(dalloc(&st_d, 1));
  tmp.push_back((double *)st_d);
  auto top_eig = [&](int j, int k) -> int {
    hipFree(lamd[j]); hipFree(Ukd[j]);
    lamd[j] = Ukd[j] = nullptr;
    LCK(dalloc(&lamd[j], k)); LCK(dalloc(&Ukd[j], (size_t)M->bm[j] * k));
    kk[j] = k;
    int rc2 = run_eig(ctx, Gb[j], M->bm[j], 1, k, nullptr, 0, lamd[j], Ukd[j], tr_d, st_d);
    if (rc2) return rc2;
    int est = 0;
    blam[j].resize(k);
    LCK(hipMemcpyAsync(blam[j].data(), lamd[j], (size_t)k * 8, hipMemcpyDeviceToHost, st));
    LCK(hipMemcpyAsync(&btr[j], tr_d, 8, hipMemcpyDeviceToHost, st));
    LCK(hipMemcpyAsync(&est, st_d, 4, hipMemcpyDeviceToHost, st));
    LCK(hipStreamSynchronize(st));
    if (est) return fail(ctx, 2, "eigensolver did not converge");
    return 0;
  };
  const int r_req = (r <= 0) ? kmax : std::min(r, mfn);
  for (int j = 0; j < nblk; ++j) {
    // the reference slices F_j[:, 1:k] (:33, :131): a block needs >= k eigenpairs
    if (M->bm[j] < r_req)
      CKB(fail(ctx, -9, "break block %d has %d rows: fewer than the %d factors requested", j, M->bt[j], r_req));
    if (nob) Gb[j] = Gfull;
    else {
      CKB(dalloc(&Gb[j], (size_t)M->bm[j] * M->bm[j]) == hipSuccess ? 0 : fail(ctx, 1002, "out of memory"));
      CKB(block_gram(j, Gb[j]) == hipSuccess ? 0 : fail(ctx, 1001, "block Gram failed"));
    }
    if (r <= 0) {   // the sweep's eigenvalues of this block
      if (nob && full_spec) bev[j] = spec_full;
      else if (!nob && M->bm[j] <= spectrum_any_max() && (kmax > 24 || pcp)) {
        std::vector<double> sp;
        CKB(spectrum(Gb[j], M->bm[j], sp));
        bev[j] = sp;
      } else if (kmax > 24) {
        CKB(fail(ctx, -30, "kmax > 24 needs the full spectrum of every block; supported for Gram "
                           "size <= %d (block %d: %d)", spectrum_any_max(), j, M->bm[j]));
      }
      if (bev[j].empty()) {   // top-k pairs: the sweep's eigenvalues and the trace
        CKB(top_eig(j, kmax));
        bev[j] = blam[j];
      } else {                // a spectrum gave the eigenvalues: only the trace (the Gram's diagonal)
        hipLaunchKernelGGL(eig_trace_kernel, dim3(1), dim3(64), 0, st, Gb[j], (int64_t)M->bm[j],
                           (int64_t)M->bm[j] * M->bm[j], M->bm[j], tr_d);
        CK(hipMemcpyAsync(&btr[j], tr_d, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
      }
    } else {
      CKB(top_eig(j, r_req));
      bev[j] = blam[j];
    }
  }
  double trace = 0.0;
  for (int j = 0; j < nblk; ++j) trace += btr[j];
  // eigenvalue i summed over blocks: V(k) = (trace - sum_{i<=k} ev[i]) / (N T)
  const int n_ev = (int)bev[0].size();
  std::vector<double> ev(n_ev, 0.0);
  for (int j = 0; j < nblk; ++j)
    for (int i = 0; i < n_ev && i < (int)bev[j].size(); ++i) ev[i] += bev[j][i];
  if (r <= 0) {
    M->swept = true;
    M->ic.assign(7 * kmax, 0.0);
    dfm_ic_sweep(ev.data(), (int)ev.size(), kmax, trace, T, N, full_spec ? M->sigma2 : NAN, M->ic.data());
    int best = 0;
    for (int k = 1; k < kmax; ++k)   // first argmin, indmin (src/DynamicFactorModel.jl:65)
      if (M->ic[crit * kmax + k] < M->ic[crit * kmax + best]) best = k;
    r = best + 1;
  }
  r = std::min(r, mfn);   // src/DynamicFactorModel.jl:116-119
  M->r = r;
  for (int j = 0; j < nblk; ++j)
    if (r > kk[j]) CKB(top_eig(j, r));   // the sweep used spectra: now the r eigenvectors
  // eigenvalues reported: kmax of the sweep (when it ran) or r; per block summed
  {
    const size_t ne = (size_t)(M->swept ? std::max(kmax, r) : r);
    M->lam.assign(ne, NAN);
    for (size_t j = 0; j < ne && j < ev.size(); ++j) M->lam[j] = ev[j];
    for (int i = 0; i < r; ++i) {
      double s = 0.0;
      for (int j = 0; j < nblk; ++j) s += blam[j][i];
      M->lam[i] = s;
    }
    M->blam.resize(nblk);
    for (int j = 0; j < nblk; ++j) M->blam[j].assign(blam[j].begin(), blam[j].begin() + r);
  }
  M->k_eig = kk[0];
  // --- factors, loadings per block for r (first r canonical eigenvectors)
  CK(dalloc(&M->F, (size_t)T * r));
  CK(dalloc(&M->colssr, N));
  M->Ubs.assign(nblk, nullptr);
  M->Ls.assign(nblk, nullptr);
  CK(dalloc(&M->Lall, (size_t)nblk * N * r));
  for (int j = 0; j < nblk; ++j) {
    const int mj = M->bm[j];
    CK(dalloc(&M->Ubs[j], (size_t)mj * r));
    M->Ls[j] = M->Lall + (size_t)j * N * r;
    if (j == 0) { M->Ub = M->Ubs[0]; M->L = M->Ls[0]; }
    CK(hipMemcpy2DAsync(M->Ubs[j], (size_t)r * 8, Ukd[j], (size_t)kk[j] * 8, (size_t)r * 8, mj,
                        hipMemcpyDeviceToDevice, st));
  }
  for (int j = 0; j < nblk; ++j) {
    Scope sc(ctx, DFM_KC_FACTORS);
    if (r <= 32) {
      if (launch_factors(M->orient, block_src(j), M->bt[j], N, r, 1, M->Ubs[j], M->F + (size_t)M->ba[j] * r,
                         M->Ls[j], nob ? M->colssr : nullptr, st, (double)T, 0))
        CKB(fail(ctx, -4, "r=%d too large", r));
    } else if (launch_factors_wide(M->orient, M->Xp + (size_t)M->ba[j] * M->ld, M->ld, M->bt[j], N, r, M->Ubs[j],
                                   M->F + (size_t)M->ba[j] * r, M->Ls[j], nob ? M->colssr : nullptr, st,
                                   (double)T)) {
      CKB(fail(ctx, 1001, "factor kernels failed"));
    }
    if (nob && M->orient == 1) {
      double *lr = nullptr;
      CK(dalloc(&lr, r));
      CK(hipMemcpyAsync(lr, lamd[0], (size_t)r * 8, hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL(colssr_cols_kernel, dim3((N + 255) / 256, 1), dim3(256), 0, st, Gfull, m,
                         (int64_t)m * m, N, r, lr, M->Ub, M->colssr);
      CK(hipStreamSynchronize(st));
      hipFree(lr);
    }
  }
  for (int j = 0; j < nblk; ++j) {   // :33 per subperiod
    Scope sc(ctx, DFM_KC_MISC);
    const size_t o = (size_t)M->ba[j] * M->ld;
    hipLaunchKernelGGL(common_residual_kernel, dim3((unsigned)((M->ld + 255) / 256), M->bt[j]), dim3(256), 0,
                       st, M->Xp + o, M->ld, M->bt[j], N, r, M->F + (size_t)M->ba[j] * r, M->Ls[j], M->Cp + o,
                       M->Ep + o);
  }
  CK(hipGetLastError());
  if (!nob)
    hipLaunchKernelGGL(col_ssq_kernel, dim3((N + 255) / 256), dim3(256), 0, st, M->Ep, M->ld, T, N, M->colssr);
  // --- V(r) by brute force over the explicit residual panel (src/criteria.jl:5)
  double essq = 0.0;
  {
    double *rows = nullptr, *tot = nullptr;
    TALLOC(rows, T); TALLOC(tot, 1);
    hipLaunchKernelGGL(panel_row_ssq_kernel, dim3(T), dim3(256), 0, st, M->Ep, M->ld, T, rows);
    hipLaunchKernelGGL(ordered_sum_kernel, dim3(1), dim3(256), 0, st, rows, T, tot);
    CK(hipMemcpyAsync(&essq, tot, 8, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
  }
  // --- OLS + HC2 on [w vcat(F_j)] (:40-48, :130-133)
  const int d = q + r;
  if (d > T) return bail(fail(ctx, -5, "q + r = %d regressors exceed the %d observations", d, T));
  double *coef = nullptr, *tst = nullptr, *cov = nullptr, *res = nullptr;
  int *ost = nullptr;
  TALLOC(coef, d); TALLOC(tst, d); TALLOC(cov, (size_t)d * d); TALLOC(res, T);
  CK(dalloc(&ost, 1));
  tmp.push_back((double *)ost);
  if (d <= 32) {
    Scope sc(ctx, DFM_KC_OLS);
    launch_ols(1, st, M->y, M->w, q, M->F, T, r, nullptr, nullptr, coef,
                       tst, cov, res, ost);
  } else {   // wide design: GEMM-built OLS (dfm_wide.hip)
    double *wk = nullptr;
    TALLOC(wk, (size_t)ols_wide_work(T, d));
    Scope sc(ctx, DFM_KC_OLS);
    CK(launch_ols_wide(M->y, M->w, q, M->F, T, r, coef, tst, cov, res, ost, wk, st));
  }
  CK(hipGetLastError());
  M->coef.resize(d); M->tstat.resize(d); M->cov.resize((size_t)d * d); M->resid.resize(T);
  int ols_bad = 0;
  CK(hipMemcpyAsync(M->coef.data(), coef, (size_t)d * 8, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(M->tstat.data(), tst, (size_t)d * 8, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(M->cov.data(), cov, (size_t)d * d * 8, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(M->resid.data(), res, (size_t)T * 8, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(&ols_bad, ost, 4, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  tfree();
  if (ols_bad) return bail(fail(ctx, 3, "singular design matrix D'D"));
  M->trace = trace;
  M->V = essq / NT;
  if (crit >= 0) M->critval = crit_formula(crit, M->V, r, M->sigma2, T, N);
  CK(dalloc(&M->flag_dev, 4));
  *out = M;
  return 0;
#undef CKB
#undef LCK
#undef TALLOC
#undef CK
}

int dfm_model_blocks(const dfm_model *m) { return m ? m->nblk : -1; }

int dfm_model_block(const dfm_model *m, int j, int64_t *row0, int64_t *rows, double *eigvals, double *L) {
  if (!m) return -1;
  if (j < 0 || j >= m->nblk) return fail(m->ctx, -2, "block %d out of range", j);
  if (row0) *row0 = m->ba[j];
  if (rows) *rows = m->bt[j];
  if (eigvals) std::copy(m->blam[j].begin(), m->blam[j].end(), eigvals);
  if (L) {
    dfm_ctx *ctx = m->ctx;
    hipSetDevice(ctx->device);
    std::vector<double> tmp((size_t)m->N * m->r);
    HIPCHK(ctx, hipMemcpyAsync(tmp.data(), m->Ls[j], tmp.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < m->N; ++i)
      for (int c = 0; c < m->r; ++c) L[(size_t)c * m->N + i] = tmp[(size_t)i * m->r + c];
  }
  return 0;
}

int dfm_model_dims(const dfm_model *m, int64_t *r, int64_t *kmax, int64_t *n_eig) {
  if (!m) return -1;
  if (r) *r = m->r;
  if (kmax) *kmax = m->swept ? m->kmax : 0;
  if (n_eig) *n_eig = (int64_t)m->lam.size();
  return 0;
}

int dfm_model_scalars(const dfm_model *m, int64_t *r, double *V, double *cv, double *tr) {
  if (!m) return -1;
  if (r) *r = m->r;
  if (V) *V = m->V;
  if (cv) *cv = m->critval;
  if (tr) *tr = m->trace;
  return 0;
}

int dfm_model_read(const dfm_model *m, double *eigvals, double *coef, double *tstat, double *coef_cov,
                   double *ols_resid, double *F, double *L, double *E, double *ic_values) {
  if (!m) return -1;
  dfm_ctx *ctx = m->ctx;
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  const int d = m->q + m->r;
  if (eigvals) std::copy(m->lam.begin(), m->lam.end(), eigvals);
  if (coef) std::copy(m->coef.begin(), m->coef.end(), coef);
  if (tstat) std::copy(m->tstat.begin(), m->tstat.end(), tstat);
  if (coef_cov) std::copy(m->cov.begin(), m->cov.end(), coef_cov);
  if (ols_resid) std::copy(m->resid.begin(), m->resid.end(), ols_resid);
  if (ic_values && !m->ic.empty()) std::copy(m->ic.begin(), m->ic.end(), ic_values);
  (void)d;
  std::vector<double> tmp;
  auto rows_to_colmajor = [&](const double *src, int rows, int cols, double *dst) -> int {
    tmp.resize((size_t)rows * cols);
    if (hipMemcpyAsync(tmp.data(), src, tmp.size() * 8, hipMemcpyDeviceToHost, st) != hipSuccess) return 1;
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    for (int i = 0; i < rows; ++i)
      for (int j = 0; j < cols; ++j) dst[(size_t)j * rows + i] = tmp[(size_t)i * cols + j];
    return 0;
  };
  if (F && rows_to_colmajor(m->F, m->T, m->r, F)) return fail(ctx, 1001, "copy F");
  if (L && rows_to_colmajor(m->L, m->N, m->r, L)) return fail(ctx, 1001, "copy L");
  if (E) {
    double *d_out = nullptr;
    HIPCHK(ctx, dalloc(&d_out, (size_t)m->T * m->N));
    hipLaunchKernelGGL(colmajor_from_rows_kernel, dim3((m->N + 31) / 32, (m->T + 31) / 32), dim3(256), 0,
                       st, m->Ep, m->ld, m->T, m->N, d_out);
    HIPCHK(ctx, hipMemcpyAsync(E, d_out, (size_t)m->T * m->N * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    hipFree(d_out);
  }
  return 0;
}

int dfm_model_set_mode(dfm_model *m, int mode) {
  if (!m || mode < 0 || mode > 2) return -1;
  m->mode = mode;
  return 0;
}

int dfm_model_fact_block(const dfm_model *m, int *p, int *pz) {
  if (!m) return -1;
  const int b = (m->orient == 0 && m->mode != 1 && m->r >= 1 && m->r <= 16 && m->T <= fact_t_max() && m->nblk == 1)
                    ? fact_block_p(m->m, m->r, m->ctx->block) : 0;
  if (p) *p = b;
  if (pz) *pz = (b + 1) & ~1;
  return b > 0 ? 0 : 1;
}

int dfm_model_set_batch(dfm_model *m, int64_t batch) {
  if (!m || batch < 0) return -1;
  m->batch = batch;
  return 0;
}

int64_t dfm_stats_width(const dfm_model *m, const dfm_stat *stats, int nstats) {
  if (!m || (!stats && nstats)) return -1;
  int64_t w = 0;
  for (int i = 0; i < nstats; ++i) w += stat_width(m, stats[i].kind);
  return w;
}

// Per-batch device workspace layout for the bootstrap.
// T >= N, no breaks, small N: the batch's Grams by one weighted GEMM (gram_wk).
// Its prep kernel stages the replicate's draws and F (T x r) in LDS: only
// while that fits the default 64 KB dynamic-LDS launch; larger T r take the
// fused-gather K1 Gram (gram_kernel<COLS>).
static bool use_gram_wk(const dfm_model *M) {
  return M->orient == 1 && M->nblk == 1 && M->N <= 256 && M->r >= 1 && M->r <= 16 &&
         gram_wk_prep_lds(M->T, M->r) <= 65536;
}
struct BootWs {
  double *G, *lam, *Uk, *trace, *F, *L, *colssr, *coef, *tstat, *blam, *btr, *gwk;
  int *status, *ost, *off, *lst;
  char *eig, *chow, *fact, *fload;
  size_t eig_bytes, chow_bytes, fact_bytes, fload_bytes;
};
static size_t boot_ws_bytes(const dfm_model *M, int nb, int P, int maxit, bool chow, bool fact, BootWs *o,
                            char *base) {
  const int m = M->m, r = M->r, T = M->T, N = M->N, d = M->q + M->r;
  size_t off = 0;
  auto take = [&](size_t bytes) { char *p = base ? base + off : nullptr; off += (bytes + 255) & ~size_t(255); return p; };
  BootWs w{};
  w.G = (double *)take(fact ? 8 : (size_t)nb * m * m * 8);
  w.lam = (double *)take((size_t)nb * r * 8);
  w.Uk = (double *)take((size_t)nb * m * r * 8);
  w.trace = (double *)take((size_t)nb * 8);
  w.F = (double *)take((size_t)nb * T * r * 8);
  w.L = (double *)take((size_t)M->nblk * nb * N * r * 8);   // block j at w.L + j nb N r
  w.colssr = (double *)take((size_t)nb * N * 8);
  w.coef = (double *)take((size_t)nb * d * 8);
  w.tstat = (double *)take((size_t)nb * d * 8);
  w.blam = (double *)take(M->nblk > 1 ? (size_t)nb * r * 8 : 8);   // one break block's lambdas
  w.btr = (double *)take(M->nblk > 1 ? (size_t)nb * 8 : 8);
  w.status = (int *)take((size_t)nb * 4);
  w.ost = (int *)take((size_t)nb * 4);
  w.eig_bytes = eig_workspace_bytes_padded(m, nb, P, maxit);
  w.eig = take(w.eig_bytes);
  w.chow_bytes = chow ? chow_workspace_bytes(T, N, r, nb) : 0;
  w.chow = take(w.chow_bytes);
  w.fact_bytes = fact ? fact_workspace_bytes(T, nb, P) : 0;
  w.fact = take(w.fact_bytes);
  w.fload_bytes = fact ? fact_loadings_bytes(T, N, r, nb) : 0;
  w.fload = take(w.fload_bytes);
  w.off = (int *)take(fact ? (size_t)nb * (T + 1) * 4 : 4);
  w.lst = (int *)take(fact ? (size_t)nb * T * 4 : 4);
  w.gwk = (double *)take(use_gram_wk(M) ? gram_wk_work(T, N, r, nb) * 8 : 8);
  if (o) *o = w;
  return off;
}

__global__ void or_flag_kernel(const int *s, int nb, int *flag, int bit) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb && s[i]) atomicOr(flag, bit);
}

__global__ void or_status_kernel(const int *s1, const int *s2, int nb, int *flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb) {
    if (s1[i]) atomicOr(flag, 1);
    if (s2[i]) atomicOr(flag, 2);
  }
}

static int bootstrap_one(dfm_model *M, int kind, int64_t B, const int32_t *idx, const double *eta,
                         const dfm_stat *stats, int ns, double *out);

// Small jobs (a rank's shard of a multi-GPU bootstrap: C3 at 8 GPUs is 1 250
// replicates per device; C2's 999) leave the chip part-idle: the
// per-replicate passes (y2, Rayleigh-Ritz, ap2, Chebyshev, Chow: one
// workgroup or one wave per replicate) run ~1 round of the resident slots or
// less, and every launch gap and convergence poll is exposed.  Such jobs run
// as lanes — contiguous parts of the replicate range on their own streams,
// each driven by its own host thread — so one lane's latency-bound passes
// overlap another's GEMMs (measured at C3 with two Python-driven contexts:
// 1 250 replicates 4.12 -> 3.76 ms, 2 500: 6.96 -> 6.55 ms; 9 999 gains < 2 %
// and stays one lane, keeping its kernels' timings solo).  Every kernel is
// batch-invariant (a replicate's result never depends on its batch), so the
// rows are bit-identical to one lane (tests/test_gpu_multi.py).
constexpr int64_t kLaneMin = 512, kLaneMax = 6000;
static int lane_count(const dfm_model *M, int64_t B, const dfm_stat *stats, int ns) {
  // DFM_NO_LANES=1 (diagnostic): one lane, so a kernel trace shows solo durations;
  // DFM_LANES=n (A/B): n lanes (1..4) wherever lanes apply
  static const bool no_lanes = [] { const char *e = getenv("DFM_NO_LANES"); return e && atoi(e) != 0; }();
  static const int forced = [] { const char *e = getenv("DFM_LANES"); return e ? atoi(e) : 0; }();
  if (no_lanes) return 1;
  if (M->is_lane || M->batch != 0 || B < kLaneMin || B > kLaneMax || ns < 0 || (ns > 0 && !stats)) return 1;
  const int p = eig_block_p(M->m, M->r, M->ctx->block);
  if (p > 32 || p < M->r) return 1;
  for (int i = 0; i < ns; ++i)
    if (stats[i].kind < 0 || stats[i].kind > DFM_STAT_LOADINGS) return 1;
  if (M->r > 16) return 1;   // the subspace solver's paths (not the dense / GEMM-built wide ones)
  if (forced > 0) return std::min(forced, dfm_model::kMaxLanes);
  return 2;
}

static int bootstrap_lanes(dfm_model *M, int nl, int kind, int64_t B, const int32_t *idx, const double *eta,
                           const dfm_stat *stats, int ns, double *out) {
  dfm_ctx *ctx = M->ctx;
  hipSetDevice(ctx->device);
  for (int j = 0; j < nl - 1; ++j) {
    if (M->lane[j]) continue;
    dfm_ctx *lc = nullptr;
    int rc = dfm_ctx_create(ctx->device, &lc);
    if (rc) return fail(ctx, 1002, "bootstrap lane: no context (%d)", rc);
    dfm_model *L = nullptr;
    rc = dfm_model_clone(M, lc, &L);
    if (rc) {
      const std::string e = lc->err;
      dfm_ctx_destroy(lc);
      return fail(ctx, rc, "bootstrap lane: %s", e.c_str());
    }
    L->is_lane = true;
    L->count_ctx = ctx;
    ctx->kids.push_back(lc);
    M->lane[j] = L;
    M->lane_worker[j] = new LaneWorker();
  }
  // the lanes' work starts after the caller's work on the main stream (its
  // inputs).  Measured and rejected: starting the second lane half a step
  // late (an event after the first lane's first eigen-iteration product), so
  // the lanes' GEMMs and latency-bound passes alternate instead of running in
  // lock-step: C3 1 250 replicates 3.81 -> 3.93 ms, C2 283 k -> 265 k
  if (!ctx->gate) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->gate, hipEventDisableTiming));
  HIPCHK(ctx, hipEventRecord(ctx->gate, ctx->stream));
  for (int j = 0; j < nl - 1; ++j) {
    dfm_ctx *lc = M->lane[j]->ctx;
    lc->tol = ctx->tol; lc->tol_values = ctx->tol_values; lc->maxit = ctx->maxit;
    lc->block = ctx->block; lc->poll = ctx->poll; lc->timing = ctx->timing;
    M->lane[j]->mode = M->mode;
    HIPCHK(ctx, hipStreamWaitEvent(lc->stream, ctx->gate, 0));
  }
#if defined(DFM_DEBUG_MEM) || defined(DFM_LANE_SKEW_AB)
  if (const int sk = dbg_lane_skew_us()) {   // wall clock: 100 ticks per microsecond
    hipLaunchKernelGGL(dbg_spin_kernel, dim3(1), dim3(64), 0, sk > 0 ? M->lane[0]->ctx->stream : ctx->stream,
                       (long long)std::abs(sk) * 100);
#ifdef DFM_DEBUG_MEM
    fprintf(stderr, "[dfm debug] lane skew %d us\n", sk);
#endif
  }
#endif
  // lane j takes replicates [b_j, b_{j+1}), b_j = ceil(j B / nl) (lane 0 = this thread)
  const int64_t width = dfm_stats_width(M, stats, ns), T = M->T;
  auto b_at = [&](int j) { return (j * B + nl - 1) / nl; };
  int rcl[dfm_model::kMaxLanes] = {};
  for (int j = 1; j < nl; ++j) {
    dfm_model *L = M->lane[j - 1];
    const int64_t b0 = b_at(j), b1 = b_at(j + 1);
    int *rc = &rcl[j];
    M->lane_worker[j - 1]->run([=]() {
      hipSetDevice(L->ctx->device);
      *rc = bootstrap_one(L, kind, b1 - b0, idx + b0 * T, eta ? eta + b0 * T : nullptr, stats, ns,
                          out ? out + b0 * width : nullptr);
    });
  }
  rcl[0] = bootstrap_one(M, kind, b_at(1), idx, eta, stats, ns, out);
  for (int j = 1; j < nl; ++j) M->lane_worker[j - 1]->wait();
  // the lanes' host-side counters join the caller's context (their kernel
  // timings when the caller's are read: merge_kids; their device-side
  // GEMM-product counts went to ctx->cnt_dev directly)
  for (int j = 0; j < nl - 1; ++j) {
    dfm_ctx *lc = M->lane[j]->ctx;
    if (lc->pend.size() > 4096) merge_kid(ctx, lc);   // (bounded: a long timed run)
    ctx->eig_batches += lc->eig_batches;
    ctx->eig_iters += lc->eig_iters;
    ctx->eig_iters_max = std::max(ctx->eig_iters_max, lc->eig_iters_max);
    ctx->rep_iters += lc->rep_iters;
    ctx->gemm_products += lc->gemm_products;
    lc->eig_batches = lc->eig_iters = lc->eig_iters_max = lc->rep_iters = lc->gemm_products = 0;
  }
  if (rcl[0]) return rcl[0];
  for (int j = 1; j < nl; ++j)
    if (rcl[j]) return fail(ctx, rcl[j], "bootstrap lane %d: %s", j, M->lane[j - 1]->ctx->err.c_str());
  return 0;
}

int dfm_bootstrap_dev(dfm_model *M, int kind, int64_t B, const int32_t *idx, const double *eta,
                      const dfm_stat *stats, int ns, double *out) {
  if (!M) return -1;
  DeviceShare gate(M->ctx->device);
  const int nl = idx && (kind != DFM_BOOT_WILD || eta) ? lane_count(M, B, stats, ns) : 1;
  if (nl > 1) return bootstrap_lanes(M, nl, kind, B, idx, eta, stats, ns, out);
  return bootstrap_one(M, kind, B, idx, eta, stats, ns, out);
}

static int bootstrap_one(dfm_model *M, int kind, int64_t B, const int32_t *idx, const double *eta,
                         const dfm_stat *stats, int ns, double *out) {
  if (!M) return -1;
  dfm_ctx *ctx = M->ctx;
  if (B < 0 || !idx || (kind == DFM_BOOT_WILD && !eta) || (ns > 0 && (!stats || !out)) || ns < 0)
    return fail(ctx, -2, "dfm_bootstrap: bad arguments");
  if (kind != DFM_BOOT_WILD && kind != DFM_BOOT_RESIDUAL) return fail(ctx, -2, "bad bootstrap kind");
  if (B == 0) return 0;
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  const int m = M->m, r = M->r, T = M->T, N = M->N, q = M->q;
  // stat descriptors
  std::vector<StatDesc> sd(ns);
  int64_t width = 0;
  bool chow = false, pcp = false;
  int chow_bp = -1;
  for (int i = 0; i < ns; ++i) {
    const dfm_stat s = stats[i];
    if (s.kind < 0 || s.kind > DFM_STAT_LOADINGS) return fail(ctx, -6, "unknown stat kind %d", s.kind);
    if (s.kind == DFM_STAT_LOADINGS && (s.arg0 < 0 || s.arg0 >= M->nblk))
      return fail(ctx, -6, "loadings of break block %d outside 0..%d", s.arg0, M->nblk - 1);
    if (s.kind == DFM_STAT_CRIT) {
      const int c = s.arg0 >= 0 ? s.arg0 : M->crit;
      if (c < 0 || c > 6) return fail(ctx, -6, "criterion stat without a criterion");
      if (c <= 2) pcp = true;
    }
    if (s.kind == DFM_STAT_EIGVAL && (s.arg0 < 0 || s.arg0 >= r))
      return fail(ctx, -6, "eigenvalue index %d outside 0..%d", s.arg0, r - 1);
    if ((s.kind == DFM_STAT_COEF || s.kind == DFM_STAT_TSTAT) && (s.arg0 < 0 || s.arg0 >= q + r))
      return fail(ctx, -6, "coefficient index %d outside 0..%d", s.arg0, q + r - 1);
    if (chow_stat(s.kind)) {
      if (s.arg0 < r || s.arg0 > T - r) return fail(ctx, -7, "break period %d out of range", s.arg0);
      if (chow && s.arg0 != chow_bp) return fail(ctx, -7, "one break period per call");
      if (M->nblk > 64) return fail(ctx, -7, "Chow statistics support at most 64 break blocks");
      chow = true; chow_bp = s.arg0;
      if (s.kind <= DFM_STAT_WALD && (s.arg1 < 0 || s.arg1 >= N)) return fail(ctx, -7, "variable index");
    }
    sd[i] = {s.kind, s.arg0, s.arg1, (int)width};
    width += stat_width(M, s.kind);
  }
  // Statistics that read only the eigenvalues and the trace let the
  // eigensolver stop on the (quadratic) eigenvalue bound instead of the
  // eigenvector residual: same 1e-12-relative accuracy for what is returned.
  bool values_only = ns > 0;
  for (int i = 0; i < ns; ++i)
    values_only = values_only && (stats[i].kind == DFM_STAT_V || stats[i].kind == DFM_STAT_CRIT ||
                                  stats[i].kind == DFM_STAT_EIGVAL || stats[i].kind == DFM_STAT_TRACE ||
                                  stats[i].kind == DFM_STAT_ITERS);
  const double etol = (values_only && ctx->tol_values > 0) ? -ctx->tol_values : ctx->tol;
  // Statistics invariant to rotations within span(F_r) — the Chow tests
  // (src/chowtest.jl reads F only through projections on it), V, criteria,
  // eigenvalues, and the w-columns' coefficients / t-statistics (the factor
  // block of the design spans the same space) — need the wanted SUBSPACE, not
  // each eigenvector: the strict rule then measures every wanted residual
  // against the gap to the first unwanted Ritz value (EigWork::subspace).
  // Factor-column coefficients / t-statistics keep the per-vector gap.
  bool subspace_only = ns > 0;
  for (int i = 0; i < ns; ++i) {
    const int kd = stats[i].kind;
    subspace_only = subspace_only && (kd == DFM_STAT_V || kd == DFM_STAT_CRIT || kd == DFM_STAT_EIGVAL ||
                                      kd == DFM_STAT_TRACE || kd == DFM_STAT_ITERS || chow_stat(kd) ||
                                      ((kd == DFM_STAT_COEF || kd == DFM_STAT_TSTAT) && stats[i].arg0 < q));
  }
  const int esub = (subspace_only && !values_only) ? 1 : 0;
  // Fields the statistics read (demand-driven, as the stopping rule above):
  // V, the criteria, eigenvalues and the trace need only the eigensolve;
  // the replicate factors F* and loadings L* (the factored path's loadings
  // GEMM) are formed for coefficients / t-statistics, the Chow tests and the
  // host-closure fields, the OLS + HC2 pass for coefficients / t-statistics.
  bool need_fl = false, need_ols = false;
  for (int i = 0; i < ns; ++i) {
    const int kd = stats[i].kind;
    need_ols = need_ols || kd == DFM_STAT_COEF || kd == DFM_STAT_TSTAT;
    need_fl = need_fl || kd == DFM_STAT_COEF || kd == DFM_STAT_TSTAT || chow_stat(kd) || kd == DFM_STAT_FACTORS ||
              kd == DFM_STAT_LOADINGS;
  }
  const int p = eig_block_p(m, r, ctx->block);
  // r beyond the subspace eigensolver's block: dense batched eigenpairs,
  // materialised replicate panels for the factor GEMMs, GEMM-built OLS
  const bool wide = p > 32 || p < r;
  const int P = (p <= 16 || wide) ? 16 : 32;
  if (wide && (M->m > dense_eig_max()))
    return fail(ctx, -20, "bootstrap at r=%d > 24 needs min(T,N) <= %d", r, dense_eig_max());
  const bool chow_wide = chow && r > 16;   // GEMM-built Chow tests on materialised replicates
  // PCp reads each replicate's full spectrum, so its Gram is formed: direct path
  const bool fact = (M->orient == 0) && (M->mode != 1) && r <= 16 && T <= fact_t_max() && M->nblk == 1 && !pcp &&
                    !wide;
  // direct path, N > T, no breaks: the replicate Grams by the factored
  // identity (gram_fact_kernel, 2 T^2 r flop each) instead of the SYRK
  const bool gid = !fact && (M->orient == 0) && M->nblk == 1 && r >= 1 && r <= 16 && T <= 4096;
  // the factored solver's own block (k + 4 columns, fact_block_p) and the
  // register template it selects: its workspace layout (eig_iters_ptr) follows
  // pf, not the direct solvers' p
  const int pf = fact ? fact_block_p(m, r, ctx->block) : p;
  const int Pf = pf <= 16 ? 16 : 32;
  // T >= N, no breaks, small N: the batch's Grams by one weighted GEMM (gram_wk)
  const bool gwk = use_gram_wk(M);
  if (pcp && m > spectrum_any_max())
    return fail(ctx, -31, "PCp criteria inside the bootstrap need each replicate's full spectrum: "
                          "supported for min(T,N) <= %d", spectrum_any_max());
  int64_t nb = M->batch;
  if (nb <= 0) {
    if (fact) {
      // No per-replicate Gram: a replicate's workspace is O((T + N) P) (C3:
      // ~0.8 MB), so one batch holds the whole job up to a 16 GB budget —
      // the latency-bound per-replicate kernels then fill the chip.
      const double per = (double)boot_ws_bytes(M, 1024, P, ctx->maxit, chow, true, nullptr, nullptr) / 1024.0;
      nb = (int64_t)std::max(1.0, std::min(16384.0, std::floor(16e9 / per)));
    } else {
      double gbytes = (double)m * m * 8 * (pcp ? 3 : 1);
      if (gwk) gbytes += 8.0 * (double)gram_wk_work(T, N, r, 1);
      if (wide)
        gbytes += 8.0 * ((double)dense_eig_work(m, r) + (double)T * M->ld + (double)ols_wide_work(T, q + r));
      if (chow_wide) gbytes += 8.0 * ((double)chow_wide_work(T, N, r) + (double)T * M->ld + 3.0 * N);
      nb = (int64_t)std::max(1.0, std::min(4096.0, std::floor((wide ? 4e9 : 1.5e9) / gbytes)));
    }
    // equal batches (no small tail batch running the iterations half-empty)
    const int64_t nbat = (B + nb - 1) / nb;
    nb = (B + nbat - 1) / nbat;
  }
  nb = std::min<int64_t>(nb, B);
  if ((fact || gid) && !M->fact_ready) {
    // H = E E' by the MFMA Gram kernel (K1), then EL, S, cF, diag(H)
    M->ldH = round_up(T, 16);
    HIPCHK(ctx, dalloc(&M->H, (size_t)T * M->ldH));
    HIPCHK(ctx, dalloc(&M->EL, (size_t)T * r));
    HIPCHK(ctx, dalloc(&M->S, (size_t)r * r));
    HIPCHK(ctx, dalloc(&M->cF, T));
    HIPCHK(ctx, dalloc(&M->hd, T));
    HIPCHK(ctx, hipMemsetAsync(M->H, 0, (size_t)T * M->ldH * 8, st));
    PanelSrc es{nullptr, M->Ep, nullptr, nullptr, M->ld, 0};
    {
      Scope sc(ctx, DFM_KC_GRAM);
      HIPCHK(ctx, launch_gram(0, es, T, N, T, M->H, M->ldH, 0, 1, st));
    }
    int rc0 = fact_precompute(M->Ep, M->ld, T, N, r, M->L, M->F, M->H, M->ldH, M->EL, M->S, M->cF, M->hd, st);
    if (rc0) return fail(ctx, rc0, "factored precompute failed");
    // F'F once per model (it was one launch per solve on every lane's stream)
    HIPCHK(ctx, dalloc(&M->FtF, 256));
    HIPCHK(ctx, launch_fact_ftf(FactBase{T, r, M->ldH, M->F, M->EL, M->S, M->H, M->cF, M->hd}, M->FtF, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    M->fact_ready = true;
  }
  if (gwk && !M->Kwk) {
    HIPCHK(ctx, dalloc(&M->Kwk, (size_t)gram_wk_tp(T) * gram_wk_ldk(N)));
    HIPCHK(ctx, dalloc(&M->A0wk, (size_t)N * N));
    HIPCHK(ctx, gram_wk_precompute(M->Ep, M->ld, T, N, r, M->F, M->L, M->Kwk, M->A0wk, st));
  }
  if (gid && !M->FSF) {
    HIPCHK(ctx, dalloc(&M->FSF, (size_t)T * M->ldH));
    HIPCHK(ctx, launch_fact_fsf(T, r, M->F, M->S, M->FSF, M->ldH, st));
  }
  const size_t need = boot_ws_bytes(M, (int)nb, P, ctx->maxit, chow && !chow_wide, fact, nullptr, nullptr);
  if (need > M->ws_bytes) {
    hipFree(M->ws);
    M->ws = nullptr; M->ws_bytes = 0;
#ifdef DFM_DEBUG_MEM
    // debug build: a 64 KB guard band of 0xA5 after the workspace, checked at the end of the call
    HIPCHK(ctx, hipMalloc(&M->ws, need + GuardBuf::kG));
    DFM_POISON_SYNC(M->ws, need);
    (void)hipMemset(M->ws + need, 0xA5, GuardBuf::kG);
    (void)hipStreamSynchronize(nullptr);
#else
    HIPCHK(ctx, hipMalloc(&M->ws, need));
#endif
    M->ws_bytes = need;
  }
  if (ns > M->sd_cap) {
    hipFree(M->sd_dev);
    HIPCHK(ctx, dalloc(&M->sd_dev, ns));
    M->sd_cap = ns;
    M->sd_host.clear();
  }
  // the descriptors go up only when they change: a pageable upload per call
  // was a host round trip in front of every small job's first kernel
  if (ns && (M->sd_host.size() != (size_t)ns || memcmp(M->sd_host.data(), sd.data(), ns * sizeof(StatDesc)) != 0)) {
    M->sd_host.clear();
    HIPCHK(ctx, hipMemcpyAsync(M->sd_dev, sd.data(), ns * sizeof(StatDesc), hipMemcpyHostToDevice, st));
    M->sd_host = sd;
  }
  BootWs w;
  boot_ws_bytes(M, (int)nb, P, ctx->maxit, chow && !chow_wide, fact, &w, M->ws);
  {   // the status flag, and the OLS status rows no OLS pass writes: one launch
    ZeroSpans zs{};
    zs.p[0] = M->flag_dev; zs.n[0] = 1;
    if (!need_ols) { zs.p[1] = w.ost; zs.n[1] = nb; }
    HIPCHK(ctx, launch_zero_spans(zs, st));
  }
  // PCp: the unrestricted full-sample Gram of every replicate (no breaks,
  // src/criteria.jl:18), its spectrum, sigma^2 per replicate
  DevBuf pG, pEv, pWk, pSig, wDe, wX, wOls, wCh, wSc;
  if (wide) {
    HIPCHK(ctx, dalloc(&wDe.p, (size_t)nb * dense_eig_work(m, r)));
    if (q + r > 32) HIPCHK(ctx, dalloc(&wOls.p, (size_t)nb * ols_wide_work(T, q + r)));
  }
  if (r > 32 || chow_wide) HIPCHK(ctx, dalloc(&wX.p, (size_t)nb * T * M->ld));
  if (chow_wide) {
    HIPCHK(ctx, dalloc(&wCh.p, (size_t)nb * chow_wide_work(T, N, r)));
    HIPCHK(ctx, dalloc(&wSc.p, (size_t)3 * nb * N));
  }
  // top-r eigenpairs of n Grams (stride mm*mm): subspace iteration or dense
  auto eig_any = [&](const double *G, int mm, int n, const double *warm, double *lam, double *Uk, double *tr,
                     int64_t b0) -> int {
    if (!wide) {
      const int pj = eig_block_p(mm, r, ctx->block);
      int rc = eig_run(G, mm, (int64_t)mm * mm, mm, n, r, pj, warm, r, etol, ctx->maxit, ctx->poll, w.eig, lam, Uk,
                       tr, w.status, nullptr, st, timer_cb, ctx, b0, esub);
      if (rc) return fail(ctx, rc > 0 ? rc : -21, "eigensolver failed (%d)", rc);
      note_iters(ctx);
      return 0;
    }
    Scope sc(ctx, DFM_KC_EIG_OTHER);
    hipError_t e = launch_dense_eig_batched(G, mm, (int64_t)mm * mm, mm, mm, 0, n, r, lam, Uk, tr, w.status, wDe.p,
                                            st);
    return e == hipSuccess ? 0 : fail(ctx, 1000 + (int)e, "dense eigensolver: %s", hipGetErrorString(e));
  };
  // factors of n replicate panels (rows T_rows of src) into F (+ row offset)
  auto factors_any = [&](const PanelSrc &ps, int Trows, int n, double *Fo, const double *Uk, double *Lo) -> int {
    Scope sc(ctx, DFM_KC_FACTORS);
    if (r <= 32) {
      launch_factors(M->orient, ps, Trows, N, r, n, Uk, Fo, Lo, nullptr, st, (double)T, (int64_t)T * r);
      return 0;
    }
    HIPCHK(ctx, launch_materialize(ps, Trows, N, M->ld, n, wX.p, st));
    if (launch_factors_wide(M->orient, wX.p, M->ld, Trows, N, r, Uk, Fo, Lo, nullptr, st, (double)T, n,
                            (int64_t)Trows * M->ld, (int64_t)T * r))
      return fail(ctx, 1001, "factor kernels failed");
    return 0;
  };
  if (pcp) {
    HIPCHK(ctx, dalloc(&pG.p, (size_t)nb * m * m));
    HIPCHK(ctx, dalloc(&pEv.p, (size_t)nb * m));
    HIPCHK(ctx, dalloc(&pSig.p, (size_t)nb));
    if (spectrum_work(m, (int)nb) > 0) HIPCHK(ctx, dalloc(&pWk.p, (size_t)spectrum_work(m, (int)nb)));
  }
  FactBase fb{T, r, M->ldH, M->F, M->EL, M->S, M->H, M->cF, M->hd, M->FtF};
  for (int64_t b0 = 0; b0 < B; b0 += nb) {
    const int n = (int)std::min<int64_t>(nb, B - b0);
    PanelSrc src{M->Cp, M->Ep, idx + b0 * T, kind == DFM_BOOT_WILD ? eta + b0 * T : nullptr, M->ld, T};
    if (fact) {
      const double *et = kind == DFM_BOOT_WILD ? eta + b0 * T : nullptr;
      // the base fit's wanted-eigenvalue spread lambda_1 / lambda_r bounds the
      // warm first filter's degree (eig_run_fact2_t)
      const double spread = (M->lam.size() >= (size_t)r && r > 0 && M->lam[r - 1] > 0.0) ? M->lam[0] / M->lam[r - 1]
                                                                                        : 0.0;
      int rc = eig_run_factored(fb, idx + b0 * T, et, n, r, pf, M->Ub, r, etol,
                                ctx->maxit, ctx->poll,
                                w.eig, w.fact, w.lam, need_fl ? w.Uk : nullptr, w.trace, w.status, st, timer_cb,
                                ctx, w.off, w.lst,
                                (M->count_ctx ? M->count_ctx : ctx)->cnt_dev, esub, spread, ctx_poll(ctx));
      if (rc) return fail(ctx, rc > 0 ? rc : -21, "eigensolver failed (%d)", rc);
      note_iters(ctx);
      if (need_fl) {
        Scope sc(ctx, DFM_KC_FACTORS);
        rc = fact_loadings(fb, M->Ep, M->ld, N, M->L, w.Uk, et, w.off, w.lst, n, w.F, w.L, w.fload, st);
        if (rc) return fail(ctx, rc, "factored loadings failed");
      }
    } else if (M->nblk > 1) {
      // refit per break block (src/bootstrap.jl:36, :48 pass dfm.break_indices):
      // block j of X*_b is rows a..a+t_j-1 of C + diag(eta_b) E[idx_b, :]
      for (int j = 0; j < M->nblk; ++j) {
        const int a = M->ba[j], tj = M->bt[j], mj = M->bm[j];
        PanelSrc sj{M->Cp + (size_t)a * M->ld, M->Ep, idx + b0 * T + a,
                    kind == DFM_BOOT_WILD ? eta + b0 * T + a : nullptr, M->ld, T};
        {
          Scope sc(ctx, DFM_KC_GRAM);
          HIPCHK(ctx, launch_gram(M->orient, sj, mj, M->orient == 0 ? N : tj, tj, w.G, mj, (int64_t)mj * mj, n, st));
        }
        int rc = eig_any(w.G, mj, n, M->Ubs[j], w.blam, w.Uk, w.btr, b0);
        if (rc) return rc;
        hipLaunchKernelGGL(or_flag_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.status, n, M->flag_dev, 1);
        if (need_fl && (rc = factors_any(sj, tj, n, w.F + (size_t)a * r, w.Uk, w.L + (size_t)j * nb * N * r)))
          return rc;
        hipLaunchKernelGGL(block_accum_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.blam, w.btr, n, r,
                           w.lam, w.trace, j == 0 ? 1 : 0);
      }
    } else {
      {
        Scope sc(ctx, DFM_KC_GRAM);
        if (gid)
          HIPCHK(ctx, launch_gram_fact(fb, M->FSF, idx + b0 * T, kind == DFM_BOOT_WILD ? eta + b0 * T : nullptr, n,
                                       w.G, m, (int64_t)m * m, st));
        else if (gwk)
          HIPCHK(ctx, launch_gram_wk(M->Ep, M->ld, T, N, r, M->F, M->L, M->Kwk, M->A0wk, idx + b0 * T,
                                     kind == DFM_BOOT_WILD ? eta + b0 * T : nullptr, T, n, w.gwk, w.G, st));
        else
          HIPCHK(ctx, launch_gram(M->orient, src, m, M->orient == 0 ? N : T, T, w.G, m, (int64_t)m * m, n, st));
      }
      int rc = eig_any(w.G, m, n, M->Ub, w.lam, w.Uk, w.trace, b0);
      if (rc) return rc;
      bool done_f = !need_fl;
      if (gwk && need_fl) {   // T >= N: F* = (F (L' L*) + D P (E L*)) / N, no pass over the resampled panel
        Scope sc(ctx, DFM_KC_FACTORS);
        done_f = launch_factors_cols_fact(M->Ep, M->ld, T, N, r, M->F, M->L, r, idx + b0 * T,
                                          kind == DFM_BOOT_WILD ? eta + b0 * T : nullptr, T, n, w.Uk, w.F, w.L,
                                          (int64_t)T * r, gram_wk_scratch(w.gwk, T, N, r, n), st);
      }
      if (!done_f && (rc = factors_any(src, T, n, w.F, w.Uk, w.L))) return rc;
    }
    if (!need_ols) {
      // (no design to be singular: w.ost zeroed at the top of the call)
    } else if (q + r <= 32) {
      Scope sc(ctx, DFM_KC_OLS);
      launch_ols(n, st, M->y, M->w, q, w.F, T, r, nullptr, nullptr, w.coef,
                         w.tstat, nullptr, nullptr, w.ost);
    } else {
      Scope sc(ctx, DFM_KC_OLS);
      HIPCHK(ctx, launch_ols_wide_batched(n, M->y, M->w, q, w.F, T, r, r, nullptr, w.coef, w.tstat, nullptr, nullptr,
                                          w.ost, wOls.p, st));
    }
    if (pcp) {
      const double *Gp = w.G;
      if (M->nblk > 1) {   // the blocks' Grams are not the full-sample one
        Scope sc(ctx, DFM_KC_GRAM);
        HIPCHK(ctx, launch_gram(M->orient, src, m, M->orient == 0 ? N : T, T, pG.p, m, (int64_t)m * m, n, st));
        Gp = pG.p;
      }
      Scope sc(ctx, DFM_KC_EIG_OTHER);
      HIPCHK(ctx, launch_spectrum(Gp, m, (int64_t)m * m, m, n, pEv.p, pWk.p, st));
      hipLaunchKernelGGL(tail_sigma2_kernel, dim3((n + 255) / 256), dim3(256), 0, st, pEv.p, m, (m + 1) / 2, n,
                         (double)N * (double)T, pSig.p);
    }
    {
      Scope sc(ctx, DFM_KC_STATS);
      if (ns)
      {
        // the eigensolver's per-replicate step counts (DFM_STAT_ITERS): the
        // workspace of this batch's (last block's) subspace solve
        // (the factored solver carves its workspace for ITS block pf, which
        // can select a narrower template than the direct solvers' P)
        const int *iters = wide ? nullptr
                                : eig_iters_ptr(w.eig, M->nblk > 1 ? M->bm.back() : m, n, fact ? Pf : P, ctx->maxit);
        hipLaunchKernelGGL(stats_kernel, dim3((n + 127) / 128), dim3(128), 0, st, n, T, N, r, q,
                           M->crit, M->sigma2, pcp ? pSig.p : nullptr, w.lam, w.trace, w.coef, w.tstat, iters,
                           M->sd_dev, ns, out + b0 * width, width, w.status, w.ost, M->flag_dev);
      } else {
        hipLaunchKernelGGL(or_status_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w.status, w.ost,
                           n, M->flag_dev);
      }
      // the replicates' factors / a block's loadings, row by row (host closures)
      for (int i = 0; i < ns; ++i) {
        if (sd[i].kind != DFM_STAT_FACTORS && sd[i].kind != DFM_STAT_LOADINGS) continue;
        const bool fk = sd[i].kind == DFM_STAT_FACTORS;
        const int64_t cnt = fk ? (int64_t)T * r : (int64_t)N * r;
        const double *srcp = fk ? w.F : w.L + (size_t)sd[i].arg0 * nb * N * r;
        HIPCHK(ctx, hipMemcpy2DAsync(out + b0 * width + sd[i].off, (size_t)width * 8, srcp, (size_t)cnt * 8,
                                     (size_t)cnt * 8, n, hipMemcpyDeviceToDevice, st));
      }
    }
    if (chow) {
      Scope sc(ctx, DFM_KC_CHOW);
      // per-variable statistics for every requested Chow stat share one pass
      double *LR = nullptr, *LM = nullptr, *WD = nullptr;
      int64_t ostride = width;
      for (int i = 0; i < ns; ++i) {
        double *base = out + b0 * width + sd[i].off;
        switch (sd[i].kind) {
          case DFM_STAT_LR_ALL: LR = base; break;
          case DFM_STAT_LM_ALL: LM = base; break;
          case DFM_STAT_WALD_ALL: WD = base; break;
          default: break;
        }
      }
      // single-variable Chow stats are served by a full pass too (cheap); they
      // are copied out of a scratch row afterwards.
      const double *scr;
      if (!chow_wide) {
        HIPCHK(ctx, launch_chow(M->orient, src, T, N, r, chow_bp, n, w.F, w.L, LR, LM, WD, ostride,
                                w.chow, w.chow_bytes, st, M->nblk, M->ba.data(), (int64_t)nb * N * r));
        // scratch rows live at the end of the chow workspace: [3][nb][N]
        scr = (const double *)(w.chow + w.chow_bytes) - (size_t)3 * n * N;   // launch_chow's [3][n][N]
      } else {
        // the whole replicate panel (r > 32 without breaks: factors_any already did)
        if (r <= 32 || M->nblk > 1) HIPCHK(ctx, launch_materialize(src, T, N, M->ld, n, wX.p, st));
        HIPCHK(ctx, launch_chow_wide(n, wX.p, M->ld, (int64_t)T * M->ld, nullptr, T, N, r, chow_bp, w.F,
                                     (int64_t)T * r, w.L, (int64_t)N * r, LR, LM, WD, ostride, wSc.p, wCh.p, st,
                                     M->nblk, M->ba.data(), (int64_t)nb * N * r));
        scr = wSc.p;
      }
      for (int i = 0; i < ns; ++i) {
        if (sd[i].kind < DFM_STAT_LR || sd[i].kind > DFM_STAT_WALD) continue;
        const int which = sd[i].kind - DFM_STAT_LR;
        HIPCHK(ctx, hipMemcpy2DAsync(out + b0 * width + sd[i].off, (size_t)width * 8,
                                     scr + ((size_t)which * n) * N + sd[i].arg1, (size_t)N * 8, 8, n,
                                     hipMemcpyDeviceToDevice, st));
      }
    }
  }
  // the status flag through the context's pinned slot (a pageable read-back
  // is a staging copy kernel and ~25 us of host time at the end of every job)
  int flag = 0;
  int *fl = ctx->pollbuf.host ? ctx->pollbuf.host + ctx->pollbuf.cap - 1 : &flag;
  HIPCHK(ctx, hipMemcpyAsync(fl, M->flag_dev, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  flag = *fl;
#ifdef DFM_DEBUG_MEM
  {
    std::vector<unsigned char> g(GuardBuf::kG);
    (void)hipMemcpy(g.data(), M->ws + M->ws_bytes, g.size(), hipMemcpyDeviceToHost);
    int64_t cnt = 0, first = -1;
    for (size_t i = 0; i < g.size(); ++i)
      if (g[i] != 0xA5) { if (first < 0) first = (int64_t)i; ++cnt; }
    if (cnt) {
      fprintf(stderr, "[dfm debug] bootstrap workspace (%s, %zu bytes, batch %lld): %lld guard bytes written past "
              "its end, first at +%lld\n", M->is_lane ? "lane" : "main", M->ws_bytes, (long long)nb, (long long)cnt,
              (long long)first);
      return fail(ctx, 9001, "debug build: bootstrap workspace overrun");
    }
  }
#endif
  if (flag & 1) return fail(ctx, 2, "eigensolver did not converge for some replicate");
  if (flag & 2) return fail(ctx, 3, "singular design matrix in some replicate");
  return 0;
}

int dfm_bootstrap(dfm_model *M, int kind, int64_t B, const int32_t *idx, const double *eta,
                  const dfm_stat *stats, int ns, double *out) {
  if (!M) return -1;
  dfm_ctx *ctx = M->ctx;
  if (B < 0 || !idx || (kind == DFM_BOOT_WILD && !eta)) return fail(ctx, -2, "dfm_bootstrap: bad arguments");
  if (B == 0) return 0;
  for (int64_t i = 0; i < B * M->T; ++i)
    if (idx[i] < 0 || idx[i] >= M->T) return fail(ctx, -8, "resample index out of range at %lld", (long long)i);
  // the whole call under the device gate — the uploads and the result copy
  // too, not only dfm_bootstrap_dev's kernels (nested: that share is this one)
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  const int64_t width = dfm_stats_width(M, stats, ns);
  int32_t *di = nullptr;
  double *de = nullptr, *dout = nullptr;
#ifdef DFM_DEBUG_MEM
  // debug build: the draws and the output rows inside guard bands, checked
  // (with the draws themselves) after the call
  GuardBuf gi, ge, go;
  HIPCHK(ctx, gi.alloc((size_t)B * M->T * 4));
  if (eta) HIPCHK(ctx, ge.alloc((size_t)B * M->T * 8));
  HIPCHK(ctx, go.alloc((size_t)B * std::max<int64_t>(width, 1) * 8));
  di = (int32_t *)gi.p; de = (double *)ge.p; dout = (double *)go.p;
#else
  HIPCHK(ctx, dalloc(&di, (size_t)B * M->T));
  if (eta) HIPCHK(ctx, dalloc(&de, (size_t)B * M->T));
  HIPCHK(ctx, dalloc(&dout, (size_t)B * std::max<int64_t>(width, 1)));
#endif
  HIPCHK(ctx, hipMemcpyAsync(di, idx, (size_t)B * M->T * 4, hipMemcpyHostToDevice, st));
  if (eta) HIPCHK(ctx, hipMemcpyAsync(de, eta, (size_t)B * M->T * 8, hipMemcpyHostToDevice, st));
  int rc = dfm_bootstrap_dev(M, kind, B, di, kind == DFM_BOOT_WILD ? de : nullptr, stats, ns, dout);
  if (rc == 0 && width > 0)
    rc = hipMemcpyAsync(out, dout, (size_t)B * width * 8, hipMemcpyDeviceToHost, st) == hipSuccess ? 0 : 1001;
  hipStreamSynchronize(st);
#ifdef DFM_DEBUG_MEM
  {
    const int bad = gi.check("idx", idx, M->T * 4) + (eta ? ge.check("eta", eta, M->T * 8) : 0) +
                    go.check("out", nullptr, width * 8);
    if (bad && rc == 0) rc = fail(ctx, 9001, "debug build: %d guard / input violations (stderr)", bad);
  }
#else
  hipFree(di); hipFree(de); hipFree(dout);
#endif
  return rc;
}

}  // extern "C"

// --------------------------------------------------------- stand-alone entry points
namespace {
struct DevPanel {   // stream-ordered (pool) allocations: no device-wide sync in hipFree
  double *raw = nullptr, *P = nullptr;
  int64_t ld = 0;
  hipStream_t st = nullptr;
  ~DevPanel() {
    if (raw) hipFreeAsync(raw, st);
    if (P) hipFreeAsync(P, st);
  }
};
// X column-major T x N (leading dimension ldx) in host memory, or already in
// HBM when dev (then it is transposed in place of the copy, never duplicated)
int upload_panel(dfm_ctx *ctx, const double *X, int T, int N, int64_t ldx, DevPanel &dp, bool dev = false) {
  hipStream_t st = ctx->stream;
  dp.ld = round_up(N, 16);
  dp.st = st;
  HIPCHK(ctx, stream_malloc((void **)&dp.P, (size_t)T * dp.ld * 8, st));
  const double *src = X;
  int64_t lds = ldx;
  if (!dev) {
    HIPCHK(ctx, stream_malloc((void **)&dp.raw, (size_t)T * N * 8, st));
    HIPCHK(ctx, hipMemcpy2DAsync(dp.raw, (size_t)T * 8, X, (size_t)ldx * 8, (size_t)T * 8, N,
                                 hipMemcpyHostToDevice, st));
    src = dp.raw;
    lds = T;
  }
  hipLaunchKernelGGL(panel_from_colmajor_kernel, dim3((unsigned)((dp.ld + 31) / 32), (T + 31) / 32),
                     dim3(256), 0, st, src, lds, T, N, dp.P, dp.ld);
  HIPCHK(ctx, hipGetLastError());
  return 0;
}
void rows_to_colmajor_host(const std::vector<double> &src, int rows, int cols, double *dst) {
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) dst[(size_t)j * rows + i] = src[(size_t)i * cols + j];
}
}  // namespace

extern "C" {

int dfm_pca(dfm_ctx *ctx, const double *X, int64_t T64, int64_t N64, int64_t ldx, int k,
            double *eigvals, double *F, double *L, double *trace_G) {
  if (!ctx) return -1;
  if (!X || T64 < 1 || N64 < 1 || ldx < T64 || k < 1) return fail(ctx, -2, "dfm_pca: bad arguments");
  const int T = (int)T64, N = (int)N64, m = std::min(T, N);
  if (k > m) return fail(ctx, -2, "dfm_pca: k=%d > min(T,N)=%d", k, m);
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  DevPanel dp;
  int rc = upload_panel(ctx, X, T, N, ldx, dp);
  if (rc) return rc;
  const int orient = (N > T) ? 0 : 1;
  double *G = nullptr, *lam = nullptr, *Uk = nullptr, *tr = nullptr, *Fd = nullptr, *Ld = nullptr;
  int *sd = nullptr;
  HIPCHK(ctx, dalloc(&G, (size_t)m * m));
  HIPCHK(ctx, dalloc(&lam, k)); HIPCHK(ctx, dalloc(&Uk, (size_t)m * k)); HIPCHK(ctx, dalloc(&tr, 1));
  HIPCHK(ctx, dalloc(&Fd, (size_t)T * k)); HIPCHK(ctx, dalloc(&Ld, (size_t)N * k)); HIPCHK(ctx, dalloc(&sd, 1));
  PanelSrc src{nullptr, dp.P, nullptr, nullptr, dp.ld, 0};
  {
    Scope sc(ctx, DFM_KC_GRAM);
    HIPCHK(ctx, launch_gram(orient, src, m, orient == 0 ? N : T, T, G, m, (int64_t)m * m, 1, st));
  }
  rc = run_eig(ctx, G, m, 1, k, nullptr, 0, lam, Uk, tr, sd);
  int est = 0;
  if (!rc) {
    Scope sc(ctx, DFM_KC_FACTORS);
    if (k <= 32 ? launch_factors(orient, src, T, N, k, 1, Uk, Fd, Ld, nullptr, st)
                : launch_factors_wide(orient, dp.P, dp.ld, T, N, k, Uk, Fd, Ld, nullptr, st, (double)T))
      rc = fail(ctx, 1001, "factor kernels failed");
  }
  std::vector<double> hF((size_t)T * k), hL((size_t)N * k);
  if (!rc) {
    if (eigvals) HIPCHK(ctx, hipMemcpyAsync(eigvals, lam, (size_t)k * 8, hipMemcpyDeviceToHost, st));
    if (trace_G) HIPCHK(ctx, hipMemcpyAsync(trace_G, tr, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(hF.data(), Fd, hF.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(hL.data(), Ld, hL.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(&est, sd, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    if (F) rows_to_colmajor_host(hF, T, k, F);
    if (L) rows_to_colmajor_host(hL, N, k, L);
  }
  for (double *p : {G, lam, Uk, tr, Fd, Ld}) hipFree(p);
  hipFree(sd);
  if (rc) return rc;
  if (est) return fail(ctx, 2, "eigensolver did not converge");
  return 0;
}

int dfm_gram_spectrum(dfm_ctx *ctx, const double *X, int64_t T64, int64_t N64, int64_t ldx,
                      double *eigvals_m, double *trace_G) {
  if (!ctx) return -1;
  if (!X || !eigvals_m || T64 < 1 || N64 < 1 || ldx < T64) return fail(ctx, -2, "bad arguments");
  const int T = (int)T64, N = (int)N64, m = std::min(T, N);
  if (m > spectrum_any_max()) return fail(ctx, -30, "full spectrum supported for min(T,N) <= %d", spectrum_any_max());
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  DevPanel dp;
  int rc = upload_panel(ctx, X, T, N, ldx, dp);
  if (rc) return rc;
  const int orient = (N > T) ? 0 : 1;
  DevBuf Gb, evb, wk;
  HIPCHK(ctx, dalloc(&Gb.p, (size_t)m * m));
  HIPCHK(ctx, dalloc(&evb.p, m));
  double *G = Gb.p, *ev = evb.p;
  if (spectrum_work(m, 1) > 0) HIPCHK(ctx, dalloc(&wk.p, (size_t)spectrum_work(m, 1)));
  PanelSrc src{nullptr, dp.P, nullptr, nullptr, dp.ld, 0};
  {
    Scope sc(ctx, DFM_KC_GRAM);
    HIPCHK(ctx, launch_gram(orient, src, m, orient == 0 ? N : T, T, G, m, (int64_t)m * m, 1, st));
  }
  {
    Scope sc(ctx, DFM_KC_EIG_OTHER);
    HIPCHK(ctx, launch_spectrum(G, m, (int64_t)m * m, m, 1, ev, wk.p, st));
  }
  HIPCHK(ctx, hipMemcpyAsync(eigvals_m, ev, (size_t)m * 8, hipMemcpyDeviceToHost, st));
  if (trace_G) {
    std::vector<double> g((size_t)m * m);
    HIPCHK(ctx, hipMemcpyAsync(g.data(), G, g.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    double s = 0;
    for (int i = 0; i < m; ++i) s += g[(size_t)i * m + i];
    *trace_G = s;
  }
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

// criterion_<name>(dfm) of a fitted model (src/criteria.jl:17-53) at its r:
// V(r) is the model's; PCp's sigma^2 is V(ceil(m/2)) of the unrestricted
// 3-arg fit DynamicFactorModel(y, w, x) (:18, :23, :28; no breaks, D2): the
// spectral tail of the resident panel's full Gram spectrum, computed once.
int dfm_model_criterion(dfm_model *M, int crit, double *value) {
  if (!M || !value) return -1;
  dfm_ctx *ctx = M->ctx;
  if (crit < 0 || crit > 6) return fail(ctx, -31, "unknown criterion %d", crit);
  DeviceShare gate(ctx->device);
  if (crit <= 2 && std::isnan(M->sigma2)) {
    const int m = M->m;
    if (m > spectrum_any_max())
      return fail(ctx, -30, "PCp criteria need the full spectrum: supported for min(T,N) <= %d", spectrum_any_max());
    hipSetDevice(ctx->device);
    hipStream_t st = ctx->stream;
    DevBuf Gb, evb, wk;
    HIPCHK(ctx, dalloc(&Gb.p, (size_t)m * m));
    HIPCHK(ctx, dalloc(&evb.p, m));
    if (spectrum_work(m, 1) > 0) HIPCHK(ctx, dalloc(&wk.p, (size_t)spectrum_work(m, 1)));
    PanelSrc src{nullptr, M->Xp, nullptr, nullptr, M->ld, 0};
    {
      Scope sc(ctx, DFM_KC_GRAM);
      HIPCHK(ctx, launch_gram(M->orient, src, m, M->orient == 0 ? M->N : M->T, M->T, Gb.p, m, (int64_t)m * m, 1, st));
    }
    {
      Scope sc(ctx, DFM_KC_EIG_OTHER);
      HIPCHK(ctx, launch_spectrum(Gb.p, m, (int64_t)m * m, m, 1, evb.p, wk.p, st));
    }
    std::vector<double> ev(m);
    HIPCHK(ctx, hipMemcpyAsync(ev.data(), evb.p, (size_t)m * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    double s = 0.0;   // trace minus the top ceil(m/2), as the fit's sigma^2
    for (double v : ev) s += v;
    for (int j = 0; j < ceil_half(m); ++j) s -= ev[j];
    M->sigma2 = s / ((double)M->N * M->T);
  }
  *value = crit_formula(crit, M->V, M->r, M->sigma2, M->T, M->N);
  return 0;
}

// One variable's LR / LM / Wald (src/chowtest.jl:19-42): the all-variables
// kernel runs once per break period and the model keeps its N x 3 results,
// so a caller's loop over the variables costs one pass over the panel.
int dfm_chow(dfm_model *M, int64_t bp, int64_t i, double *LR, double *LM, double *Wald) {
  if (!M) return -1;
  if (i < 0 || i >= M->N) return fail(M->ctx, -2, "variable index %lld out of range", (long long)i);
  if (M->chow_bp != bp) {
    std::vector<double> c((size_t)3 * M->N);
    int rc = dfm_chow_all(M, bp, c.data(), c.data() + M->N, c.data() + 2 * M->N);
    if (rc) return rc;
    M->chow_cache.swap(c);
    M->chow_bp = bp;
  }
  if (LR) *LR = M->chow_cache[(size_t)i];
  if (LM) *LM = M->chow_cache[(size_t)M->N + i];
  if (Wald) *Wald = M->chow_cache[(size_t)2 * M->N + i];
  return 0;
}

int dfm_chow_all(dfm_model *M, int64_t bp, double *LR, double *LM, double *Wald) {
  if (!M) return -1;
  dfm_ctx *ctx = M->ctx;
  if (bp < M->r || bp > M->T - M->r) return fail(ctx, -7, "break period %lld out of range", (long long)bp);
  if (M->nblk > 64) return fail(ctx, -7, "Chow statistics support at most 64 break blocks");
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  if (M->r > 16) {   // any r: the GEMM-built tests (dfm_wide.hip)
    DevBuf wk, sc3;
    HIPCHK(ctx, dalloc(&wk.p, (size_t)chow_wide_work(M->T, M->N, M->r)));
    HIPCHK(ctx, dalloc(&sc3.p, (size_t)3 * M->N));
    {
      Scope sc(ctx, DFM_KC_CHOW);
      HIPCHK(ctx, launch_chow_wide(1, M->Xp, M->ld, 0, M->Ep, M->T, M->N, M->r, (int)bp, M->F, 0, M->L, 0, nullptr,
                                   nullptr, nullptr, M->N, sc3.p, wk.p, st));
    }
    double *outs[3] = {LR, LM, Wald};
    for (int i = 0; i < 3; ++i)
      if (outs[i]) HIPCHK(ctx, hipMemcpyAsync(outs[i], sc3.p + (size_t)i * M->N, (size_t)M->N * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    return 0;
  }
  const size_t bytes = chow_workspace_bytes(M->T, M->N, M->r, 1);
  char *ws = nullptr;
  HIPCHK(ctx, hipMalloc(&ws, bytes));
  PanelSrc src{nullptr, M->Xp, nullptr, nullptr, M->ld, 0};
  {
    Scope sc(ctx, DFM_KC_CHOW);
    HIPCHK(ctx, launch_chow(M->orient, src, M->T, M->N, M->r, (int)bp, 1, M->F, M->L, nullptr, nullptr,
                            nullptr, M->N, ws, bytes, st, M->nblk, M->ba.data(), (int64_t)M->N * M->r));
  }
  const double *scr = (const double *)(ws + bytes) - (size_t)3 * M->N;
  double *outs[3] = {LR, LM, Wald};
  for (int i = 0; i < 3; ++i)
    if (outs[i]) HIPCHK(ctx, hipMemcpyAsync(outs[i], scr + (size_t)i * M->N, (size_t)M->N * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  hipFree(ws);
  return 0;
}

int dfm_targeted_hard(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                      const double *X, int64_t T64, int64_t N64, int64_t ldx, int mode,
                      double crit_value, double *tstat, uint8_t *mask) {
  if (!ctx) return -1;
  if (!y || !X || !tstat || !mask || T64 < 2 || N64 < 1 || ldx < T64 || q < 0 || (q > 0 && (!w || ldw < T64)))
    return fail(ctx, -2, "dfm_targeted_hard: bad arguments");
  if (mode != DFM_TP_JOINT && mode != DFM_TP_PER_CANDIDATE) return fail(ctx, -2, "bad mode");
  const int T = (int)T64, N = (int)N64;
  if (mode == DFM_TP_JOINT && q + N >= T)
    return fail(ctx, 3, "joint hard thresholding is singular for q + N >= T (defect D8); use PER_CANDIDATE");

  if (mode == DFM_TP_PER_CANDIDATE && (q < 1 || q > 16)) return fail(ctx, -32, "PER_CANDIDATE needs 1 <= q <= 16");
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  DevPanel dp;
  int rc = upload_panel(ctx, X, T, N, ldx, dp);
  if (rc) return rc;
  double *dy = nullptr, *dw = nullptr, *dt = nullptr;
  uint8_t *dm = nullptr;
  int *bad = nullptr;
  char *ws = nullptr;
  const size_t wsb = targeted_workspace_bytes(mode, T, N, q);
  HIPCHK(ctx, dalloc(&dy, T)); HIPCHK(ctx, dalloc(&dw, (size_t)T * std::max(q, 1)));
  HIPCHK(ctx, dalloc(&dt, N)); HIPCHK(ctx, hipMalloc(&dm, N)); HIPCHK(ctx, dalloc(&bad, 1));
  HIPCHK(ctx, hipMalloc(&ws, wsb));
  HIPCHK(ctx, hipMemcpyAsync(dy, y, (size_t)T * 8, hipMemcpyHostToDevice, st));
  if (q > 0) HIPCHK(ctx, hipMemcpy2DAsync(dw, (size_t)T * 8, w, (size_t)ldw * 8, (size_t)T * 8, q, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemsetAsync(bad, 0, 4, st));
  if (mode == DFM_TP_JOINT && q + N > 64) {   // any width: GEMM-built OLS with HC0 (dfm_wide.hip)
    DevBuf wk;
    HIPCHK(ctx, dalloc(&wk.p, (size_t)targeted_joint_wide_work(T, q, N, dp.ld)));
    Scope sc(ctx, DFM_KC_MISC);
    HIPCHK(ctx, launch_targeted_joint_wide(dy, dw, q, dp.P, dp.ld, T, N, crit_value, dt, dm, bad, wk.p, st));
  } else {
    Scope sc(ctx, DFM_KC_MISC);
    HIPCHK(ctx, launch_targeted(mode, dy, dw, q, dp.P, dp.ld, T, N, crit_value, dt, dm, ws, wsb, st, bad));
  }
  int hb = 0;
  HIPCHK(ctx, hipMemcpyAsync(tstat, dt, (size_t)N * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(mask, dm, (size_t)N, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  hipFree(dy); hipFree(dw); hipFree(dt); hipFree(dm); hipFree(bad); hipFree(ws);
  if (hb) return fail(ctx, 3, "singular design matrix");
  return 0;
}

}  // extern "C"

// ----------------------------------------------------------- expanding windows
// pseudo_out_of_sample_forecasts, refit part (src/utils.jl:54-72): for
// date_index = T-P+1..T (1-based) the model is refit on rows 1..date_index-1,
// i.e. window w = 0..P-1 uses the first n_w = T-P+w rows.  Every window is a
// masked replicate of the full panel (idx = identity, eta_t = 1{t < n_w}):
//  N > T : the window Gram is the leading n_w x n_w block of H = X X' (the
//          prefix-Gram identity) -> ONE Gram for all windows,
//          then the factored batched eigensolver (H . Z GEMMs);
//  T >= N: per-window Grams X_w' X_w from the masked fused-gather Gram kernel.
// Each window runs the IC sweep k = 1..kmax (the refit is the IC-sweep
// constructor, :53-66), picks r_w, and fits OLS+HC2 on [w F_r] over its rows.
__global__ void window_scale_kernel(const double *__restrict__ Uk, int T, int k, int Tfirst, int dn,
                                    double *__restrict__ F) {
  const int rep = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)T * k) return;
  const int t = (int)(e / k), n = Tfirst + dn * rep;
  F[(int64_t)rep * T * k + e] = t < n ? sqrt((double)n) * Uk[(int64_t)rep * T * k + e] : 0.0;
}

// ---- forecast step of pseudo_out_of_sample_forecasts (src/utils.jl:54-72)
// with get_factors repaired (defect D4: the local rotation = L (L'L)^-1 of
// src/DynamicFactorModel.jl:126, L = block 1's full loadings).  For the
// window's first r columns rotation is L_j n / lambda_j (N > T: L'L =
// Lambda / n) or L_j / N (T >= N: L'L = N I), so with the new row
// x~ = (x_n - mean(X_w)) / std(X_w) (scalar moments of all window entries,
// Julia 0.3 mean/std of a matrix):
//   N > T : F_new_j = sum_{s<n} (x~ . x_s) F_j[s] / lambda_j,
//           x~ . x_s = (H[n][s] - mean * rowsum_s) / std   (H = X X', prefix Gram)
//   T >= N: F_new_j = x~ . V_j / sqrt(N)
// and the forecast is [w_n F_new] beta (src/DynamicFactorModel.jl:152-155).
__global__ void panel_row_sums_kernel(const double *__restrict__ P, int64_t ld, int N, double *__restrict__ rs,
                                      double *__restrict__ ss) {
  __shared__ double r1[256], r2[256];
  const int t = blockIdx.x, tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int c = tid; c < N; c += 256) { const double v = P[(int64_t)t * ld + c]; a += v; b = fma(v, v, b); }
  r1[tid] = a; r2[tid] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) { r1[tid] += r1[tid + o]; r2[tid] += r2[tid + o]; }
    __syncthreads();
  }
  if (tid == 0) { rs[t] = r1[0]; ss[t] = r2[0]; }
}

__global__ void window_forecast_kernel(int orient, const double *__restrict__ Xp, int64_t ld, int T, int N, int n0,
                                       int len, int q, int kmax, const double *__restrict__ H, int64_t ldH,
                                       const double *__restrict__ F, const double *__restrict__ Uk,
                                       const double *__restrict__ lam, const double *__restrict__ rs,
                                       const double *__restrict__ ss, const int *__restrict__ kr,
                                       const double *__restrict__ coef, const double *__restrict__ y,
                                       const double *__restrict__ w, double *__restrict__ pred,
                                       double *__restrict__ truev) {
  __shared__ double red[256];
  __shared__ double smom[2];
  // the window's rows a0 .. n - 1 (expanding: a0 = 0; rolling: the last len
  // rows before n, relocated to rows 0 .. len - 1 of F)
  const int wi = blockIdx.x, tid = threadIdx.x, n = n0 + wi, a0 = len > 0 ? n - len : 0, r = kr[wi], d = q + kmax;
  if (tid == 0) {   // scalar moments of the window's (n - a0) x N entries (fixed order)
    double a = 0.0, b = 0.0;
    for (int s = a0; s < n; ++s) { a += rs[s]; b += ss[s]; }
    const double cnt = (double)(n - a0) * N, mu = a / cnt;
    smom[0] = mu;
    smom[1] = sqrt((b - cnt * mu * mu) / (cnt - 1.0));
  }
  __syncthreads();
  const double mu = smom[0], sd = smom[1];
  double yhat = 0.0;
  for (int j = 0; j < r; ++j) {
    double part = 0.0;
    if (orient == 0) {
      const double *Hn = H + (int64_t)n * ldH;
      const double *Fw = F + (int64_t)wi * T * kmax;
      for (int s = a0 + tid; s < n; s += 256)
        part = fma((Hn[s] - mu * rs[s]) / sd, Fw[(int64_t)(s - a0) * kmax + j], part);
    } else {
      const double *xn = Xp + (int64_t)n * ld;
      const double *V = Uk + (int64_t)wi * N * kmax;
      for (int c = tid; c < N; c += 256) part = fma((xn[c] - mu) / sd, V[(int64_t)c * kmax + j], part);
    }
    red[tid] = part;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (tid < o) red[tid] += red[tid + o];
      __syncthreads();
    }
    const double fnew = orient == 0 ? red[0] / lam[(int64_t)wi * kmax + j] : red[0] / sqrt((double)N);
    yhat = fma(fnew, coef[(int64_t)wi * d + q + j], yhat);
    __syncthreads();
  }
  if (tid == 0) {
    for (int i = 0; i < q; ++i) yhat = fma(w[(int64_t)i * T + n], coef[(int64_t)wi * d + i], yhat);
    pred[wi] = yhat;
    truev[wi] = y[n];
  }
}

// window wi as a masked "replicate" of the panel: rows t < n_w are panel rows
// a_w + t (expanding: a_w = 0, n_w = n0 + wi; rolling: n_w = len, a_w = n0 +
// wi - len), rows past n_w carry eta = 0
__global__ void window_draws_kernel(int T, int n0, int len, int32_t *__restrict__ idx, double *__restrict__ eta) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, wi = blockIdx.y;
  if (t >= T) return;
  const int nw = len > 0 ? len : n0 + wi, aw = len > 0 ? n0 + wi - len : 0;
  idx[(int64_t)wi * T + t] = t < nw ? aw + t : t;
  eta[(int64_t)wi * T + t] = t < nw ? 1.0 : 0.0;
}
// The refit of each window (pseudo_out_of_sample_forecasts' model_args,
// src/utils.jl:64-65): len = 0 expanding windows (rows 0 .. T-P+w-1), len > 0
// rolling windows of len rows ending at T-P+w-1; r > 0 the workhorse
// constructor at fixed r (:28, clamped to ceil(m_w/2), :116-119), r = 0 the
// IC-sweep constructor (:53) by crit over k <= kmax_w, r < 0 the 3-arg default
// r = ceil(m_w/2) (D2); breaks: model_args' break_indices, the same rows for
// every (expanding) window.
struct WinSpec {
  int len = 0, r = 0, crit = -1, kmax = 0;
  const int64_t *breaks = nullptr;
  int nbreaks = 0;
};
static int windows_impl(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw, const double *X,
                        int64_t T64, int64_t N64, int64_t ldx, int P, const WinSpec &ws, int64_t *r_out,
                        double *V_out, double *crit_out, double *eig_out, double *coef_out, double *tstat_out,
                        double *pred_out, double *true_out, bool dev);
static int windows_breaks_impl(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw, const double *X,
                               int T, int N, int64_t ldx, int P, const WinSpec &ws, int K, int64_t *r_out,
                               double *V_out, double *crit_out, double *eig_out, double *coef_out,
                               double *tstat_out, double *pred_out, double *true_out);
#define LCKW(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail(ctx, 1000 + (int)e_, "%s", hipGetErrorString(e_)); } while (0)

extern "C" int dfm_windows(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                           const double *X, int64_t T64, int64_t N64, int64_t ldx, int P, int crit,
                           int kmax, int64_t *r_out, double *V_out, double *crit_out, double *eig_out,
                           double *coef_out, double *tstat_out) {
  WinSpec ws;
  ws.crit = crit; ws.kmax = kmax;
  return windows_impl(ctx, y, w, q, ldw, X, T64, N64, ldx, P, ws, r_out, V_out, crit_out, eig_out,
                      coef_out, tstat_out, nullptr, nullptr, false);
}

extern "C" int dfm_windows_dev(dfm_ctx *ctx, const double *y_dev, const double *w_dev, int q, int64_t ldw,
                               const double *X_dev, int64_t T64, int64_t N64, int64_t ldx, int P, int crit,
                               int kmax, int64_t *r_out, double *V_out, double *crit_out, double *eig_out,
                               double *coef_out, double *tstat_out) {
  WinSpec ws;
  ws.crit = crit; ws.kmax = kmax;
  return windows_impl(ctx, y_dev, w_dev, q, ldw, X_dev, T64, N64, ldx, P, ws, r_out, V_out, crit_out,
                      eig_out, coef_out, tstat_out, nullptr, nullptr, true);
}

extern "C" int dfm_windows_forecast(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw,
                                    const double *X, int64_t T64, int64_t N64, int64_t ldx, int P, int crit,
                                    int kmax, int64_t *r_out, double *pred_out, double *true_out) {
  if (!pred_out || !true_out) return fail(ctx, -2, "dfm_windows_forecast: output pointers required");
  WinSpec ws;
  ws.crit = crit; ws.kmax = kmax;
  return windows_impl(ctx, y, w, q, ldw, X, T64, N64, ldx, P, ws, r_out, nullptr, nullptr, nullptr,
                      nullptr, nullptr, pred_out, true_out, false);
}

extern "C" int dfm_windows_ex(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw, const double *X,
                              int64_t T64, int64_t N64, int64_t ldx, int P, const dfm_window_spec *spec, int dev,
                              int64_t *r_out, double *V_out, double *crit_out, double *eig_out, double *coef_out,
                              double *tstat_out, double *pred_out, double *true_out) {
  if (!ctx) return -1;
  if (!spec) return fail(ctx, -2, "dfm_windows_ex: spec required");
  if (spec->kind != DFM_WIN_EXPANDING && spec->kind != DFM_WIN_ROLLING)
    return fail(ctx, -2, "dfm_windows_ex: unknown window kind %d", spec->kind);
  if ((pred_out == nullptr) != (true_out == nullptr))
    return fail(ctx, -2, "dfm_windows_ex: pred_out and true_out go together");
  WinSpec ws;
  ws.len = spec->kind == DFM_WIN_ROLLING ? spec->length : 0;
  if (spec->kind == DFM_WIN_ROLLING && spec->length < 2) return fail(ctx, -2, "dfm_windows_ex: rolling length < 2");
  ws.r = spec->r; ws.crit = spec->crit; ws.kmax = spec->kmax;
  ws.breaks = spec->breaks; ws.nbreaks = spec->nbreaks;
  return windows_impl(ctx, y, w, q, ldw, X, T64, N64, ldx, P, ws, r_out, V_out, crit_out, eig_out, coef_out,
                      tstat_out, pred_out, true_out, dev != 0);
}

// Masked explicit window Grams for N > T windows past the factored solver's
// T range: G_w[i][j] = eta_i eta_j H[idx_i][idx_j] (H = X X', the prefix Gram)
__global__ void window_gram_kernel(const double *__restrict__ H, int64_t ldH, const int32_t *__restrict__ idx,
                                   const double *__restrict__ eta, int T, double *__restrict__ G) {
  const int i = blockIdx.y, wi = blockIdx.z;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= T) return;
  const int32_t *ix = idx + (int64_t)wi * T;
  const double *et = eta + (int64_t)wi * T;
  const double ei = et[i], ej = et[j];
  G[((int64_t)wi * T + i) * T + j] = (ei != 0.0 && ej != 0.0) ? ei * ej * H[(int64_t)ix[i] * ldH + ix[j]] : 0.0;
}

static int windows_impl(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw, const double *X,
                        int64_t T64, int64_t N64, int64_t ldx, int P, const WinSpec &ws, int64_t *r_out,
                        double *V_out, double *crit_out, double *eig_out, double *coef_out, double *tstat_out,
                        double *pred_out, double *true_out, bool dev) {
  if (!ctx) return -1;
  DeviceShare gate(ctx->device);
  const int T = (int)T64, N = (int)N64;
  if (!y || !X || T < 4 || N < 1 || ldx < T || P < 1 || T - P < 2 || q < 0 || (q > 0 && (!w || ldw < T)) ||
      !r_out)
    return fail(ctx, -2, "dfm_windows: bad arguments");
  const int crit = ws.crit, len = ws.len;
  if (crit < -1 || crit > 6 || (ws.r == 0 && crit < 0))
    return fail(ctx, -31, "dfm_windows: unknown criterion %d (the IC sweep needs one)", crit);
  const bool pcp = crit >= 0 && crit <= 2;
  const int n0 = T - P;
  if (len > n0) return fail(ctx, -2, "dfm_windows: rolling length %d exceeds the %d rows before the first window", len, n0);
  if (ws.nbreaks < 0 || (ws.nbreaks > 0 && !ws.breaks)) return fail(ctx, -2, "dfm_windows: bad break list");
  if (ws.nbreaks > 0 && len > 0)
    return fail(ctx, -2, "dfm_windows: break_indices apply to expanding windows (the same rows in every refit, "
                         "src/utils.jl:64)");
  // window wi: rows aw(wi) .. aw(wi) + nw(wi) - 1 (relocated to rows 0 .. nw - 1)
  auto nw = [&](int wi) { return len > 0 ? len : n0 + wi; };
  auto aw = [&](int wi) { return len > 0 ? n0 + wi - len : 0; };
  const int orient = len > 0 ? (N > len ? 0 : 1) : (N > T ? 0 : 1);
  if (orient == 1 && len == 0 && N > n0)
    return fail(ctx, -2, "dfm_windows: windows straddle the T >= N / N > T branches");
  // window w's factor count: the sweep k = 1..kmax_w, kmax_w = ceil(m_w / 2)
  // (the IC-sweep constructor's default, src/DynamicFactorModel.jl:54) capped
  // by the caller's kmax (D11); fixed r clamped to ceil(m_w/2) (:116-119);
  // the 3-arg default ceil(m_w/2) (D2); m_w = min(n_w, N)
  auto kd_w = [&](int wi) { return (std::min(nw(wi), N) + 1) / 2; };
  auto kmax_w = [&](int wi) {
    const int kd = kd_w(wi);
    if (ws.r > 0) return std::min(ws.r, kd);
    if (ws.r < 0) return kd;
    return ws.kmax > 0 ? std::min(ws.kmax, kd) : kd;
  };
  int kmax = kmax_w(P - 1);   // the widest window's: row stride of eig_out / coef_out
  if (ws.nbreaks > 0)
    return windows_breaks_impl(ctx, y, w, q, ldw, X, T, N, ldx, P, ws, kmax, r_out, V_out, crit_out, eig_out,
                               coef_out, tstat_out, pred_out, true_out);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  const int m = orient == 0 ? T : N;
  // kmax beyond the subspace block (or a design wider than 32): each window's
  // sweep reads its full spectrum, the r_w eigenvectors come from the dense
  // batched eigensolver (diagonal blocks of H zero-padded to T x T for N > T)
  const int p = eig_block_p(m, kmax, ctx->block);
  const bool wide = p > 32 || p < kmax || q + kmax > 32;
  if ((pcp || wide) && m > std::min(spectrum_any_max(), dense_eig_max()))
    return fail(ctx, -31, "dfm_windows: PCp / kmax > 24 need each window's full spectrum: supported for "
                          "min(T,N) <= %d", std::min(spectrum_any_max(), dense_eig_max()));
  const int Pb = (p <= 16 || wide) ? 16 : 32;
  // N > T past the factored solver's T range: per-window masked Grams, explicit-Gram solver
  const bool explicit_gram = orient == 0 && !wide && T > fact_t_max();
  DevPanel dp;
  int rc = upload_panel(ctx, X, T, N, ldx, dp, dev);
  if (rc) return rc;
  std::vector<int> hTn(P), hkr(P), hR0(P);
  // scratch: bump allocation from the context's arena (sized by the largest
  // earlier call; stream-ordered reuse), overflow from the stream-ordered pool
  if (ctx->warena_need > ctx->warena_cap) {
    hipStreamSynchronize(st);
    hipFree(ctx->warena);
    ctx->warena = nullptr;
    ctx->warena_cap = 0;
    if (hipMalloc((void **)&ctx->warena, ctx->warena_need) == hipSuccess) ctx->warena_cap = ctx->warena_need;
  }
  std::vector<void *> frees;
  size_t aoff = 0, aneed = 0;
  auto dal = [&](size_t bytes) -> void * {
    const size_t b = (std::max<size_t>(bytes, 8) + 255) & ~size_t(255);
    aneed += b;
    if (aoff + b <= ctx->warena_cap) { void *ptr = ctx->warena + aoff; aoff += b; return ptr; }
    void *ptr = nullptr;
    if (stream_malloc(&ptr, b, st) != hipSuccess) return nullptr;
    frees.push_back(ptr);
    return ptr;
  };
  struct Freer {
    std::vector<void *> &v; hipStream_t s; dfm_ctx *c; size_t &need;
    ~Freer() { for (void *x : v) hipFreeAsync(x, s); c->warena_need = std::max(c->warena_need, need); }
  } freer{frees, st, ctx, aneed};
  // window w as a "replicate" of the panel: relocated rows, row mask t < n_w
  int32_t *didx = (int32_t *)dal((size_t)P * T * 4);
  double *deta = (double *)dal((size_t)P * T * 8);
  double *dy = (double *)dal((size_t)T * 8), *dw = (double *)dal((size_t)T * std::max(q, 1) * 8);
  double *tr = (double *)dal((size_t)P * 8);
  int *stt = (int *)dal((size_t)P * 4), *ost = (int *)dal((size_t)P * 4);
  int *dTn = (int *)dal((size_t)P * 4), *dkr = (int *)dal((size_t)P * 4), *dR0 = (int *)dal((size_t)P * 4);
  if (!didx || !deta || !dy || !dw || !tr || !stt || !ost || !dTn || !dkr || !dR0)
    return fail(ctx, 1002, "dfm_windows: out of device memory");
  hipLaunchKernelGGL(window_draws_kernel, dim3((unsigned)((T + 255) / 256), P), dim3(256), 0, st, T, n0, len, didx,
                     deta);
  const hipMemcpyKind yk = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIPCHK(ctx, hipMemcpyAsync(dy, y, (size_t)T * 8, yk, st));
  if (q > 0) HIPCHK(ctx, hipMemcpy2DAsync(dw, (size_t)T * 8, w, (size_t)ldw * 8, (size_t)T * 8, q, yk, st));
  PanelSrc msrc{nullptr, dp.P, didx, deta, dp.ld, T};   // window w = its rows of X, relocated
  // ---- the windows' Grams: N > T one Gram H = X X' (every window's Gram is a
  // diagonal block of it); T >= N per-window G
  double *H = nullptr, *G = nullptr;
  int64_t ldH = 0;
  if (orient == 0) {
    ldH = round_up(T, 16);
    H = (double *)dal((size_t)T * ldH * 8);
    if (!H) return fail(ctx, 1002, "dfm_windows: out of device memory");
    HIPCHK(ctx, hipMemsetAsync(H, 0, (size_t)T * ldH * 8, st));
    PanelSrc es{nullptr, dp.P, nullptr, nullptr, dp.ld, 0};
    Scope sc(ctx, DFM_KC_GRAM);
    HIPCHK(ctx, launch_gram(0, es, T, N, T, H, ldH, 0, 1, st));   // ONE Gram for every window
  } else {
    G = (double *)dal((size_t)P * N * N * 8);
    if (!G) return fail(ctx, 1002, "dfm_windows: out of device memory");
    Scope sc(ctx, DFM_KC_GRAM);
    HIPCHK(ctx, launch_gram(1, msrc, N, T, T, G, N, (int64_t)N * N, P, st));
  }
  // N > T windows as diagonal blocks of H: expanding = leading (n0 + w) blocks,
  // rolling = the len x len block at row/column n0 + w - len
  const double *Hb = H ? (len > 0 ? H + (int64_t)(n0 - len) * (ldH + 1) : H) : nullptr;
  const int64_t sHb = len > 0 ? ldH + 1 : 0;
  const int mv0 = len > 0 ? len : n0, dmv = len > 0 ? 0 : 1;
  // ---- full spectra (PCp's sigma^2, and the whole sweep when wide)
  double *pev = nullptr;   // P x pst
  const int pst = orient == 0 ? (len > 0 ? len : T - 1) : N;
  if (pcp || wide) {
    pev = (double *)dal((size_t)P * pst * 8);
    double *pwk = spectrum_work(pst, P) > 0 ? (double *)dal((size_t)spectrum_work(pst, P) * 8) : nullptr;
    if (!pev || (spectrum_work(pst, P) > 0 && !pwk)) return fail(ctx, 1002, "dfm_windows: out of device memory");
    Scope sc(ctx, DFM_KC_EIG_OTHER);
    if (orient == 0) HIPCHK(ctx, launch_spectrum_var(Hb, ldH, sHb, pst, mv0, dmv, P, pev, pwk, st));
    else HIPCHK(ctx, launch_spectrum(G, N, (int64_t)N * N, N, P, pev, pwk, st));
  }
  std::vector<double> hev;
  if (pev) {
    hev.resize((size_t)P * pst);
    HIPCHK(ctx, hipMemcpyAsync(hev.data(), pev, hev.size() * 8, hipMemcpyDeviceToHost, st));
  }
  // ---- narrow: top-kmax pairs of every window by the batched subspace solver
  int kv = kmax;   // eigenvectors kept per window (stride of F, Uk, lam, coef)
  double *lam = nullptr, *Uk = nullptr, *F = nullptr;
  std::vector<double> hl((size_t)P * kmax), ht(P);
  if (!wide) {
    lam = (double *)dal((size_t)P * kmax * 8); Uk = (double *)dal((size_t)P * m * kmax * 8);
    F = (double *)dal((size_t)P * T * kmax * 8);
    if (!lam || !Uk || !F) return fail(ctx, 1002, "dfm_windows: out of device memory");
    if (orient == 0 && !explicit_gram) {
      char *ews = (char *)dal(eig_workspace_bytes_padded(m, P, Pb, ctx->maxit));
      double *zero = (double *)dal((size_t)T * 8), *hd = (double *)dal((size_t)T * 8);
      char *fws = (char *)dal(fact_workspace_bytes(T, P, Pb));
      int *off = (int *)dal((size_t)P * (T + 1) * 4), *lst = (int *)dal((size_t)P * T * 4);
      if (!ews || !zero || !hd || !fws || !off || !lst) return fail(ctx, 1002, "dfm_windows: out of device memory");
      HIPCHK(ctx, hipMemsetAsync(zero, 0, (size_t)T * 8, st));
      rc = fact_precompute(dp.P, dp.ld, T, N, 0, nullptr, nullptr, H, ldH, zero, zero, zero, hd, st);
      if (rc) return fail(ctx, rc, "precompute");
      HIPCHK(ctx, hipMemsetAsync(zero, 0, (size_t)T * 8, st));
      FactBase fb{T, 0, ldH, zero, zero, zero, H, zero, hd};
      rc = eig_run_factored(fb, didx, deta, P, kmax, p, nullptr, 0, ctx->tol, ctx->maxit, ctx->poll, ews, fws,
                            lam, Uk, tr, stt, st, timer_cb, ctx, off, lst, nullptr, 0, 0.0, ctx_poll(ctx));
      if (rc) return fail(ctx, rc > 0 ? rc : -21, "eigensolver failed (%d)", rc);
    } else if (orient == 0) {
      // T > the factored solver's range: the windows' masked T x T Grams in
      // chunks (<= 2 GB), each chunk by the explicit-Gram subspace solver
      const int64_t per = (int64_t)T * T * 8;
      const int Pc = (int)std::max<int64_t>(1, std::min<int64_t>(P, (int64_t)(2LL << 30) / per));
      double *Gc = (double *)dal((size_t)Pc * per);
      char *ews = (char *)dal(eig_workspace_bytes_padded(m, Pc, Pb, ctx->maxit));
      if (!Gc || !ews) return fail(ctx, 1002, "dfm_windows: out of device memory");
      for (int c0 = 0; c0 < P; c0 += Pc) {
        const int pc = std::min(Pc, P - c0);
        {
          Scope sc(ctx, DFM_KC_GRAM);
          hipLaunchKernelGGL(window_gram_kernel, dim3((unsigned)((T + 255) / 256), T, pc), dim3(256), 0, st, H, ldH,
                             didx + (size_t)c0 * T, deta + (size_t)c0 * T, T, Gc);
          HIPCHK(ctx, hipGetLastError());
        }
        rc = eig_run(Gc, T, (int64_t)T * T, T, pc, kmax, p, nullptr, 0, ctx->tol, ctx->maxit, ctx->poll, ews,
                     lam + (size_t)c0 * kmax, Uk + (size_t)c0 * T * kmax, tr + c0, stt + c0, nullptr, st, timer_cb,
                     ctx, 0);
        if (rc) return fail(ctx, rc > 0 ? rc : -21, "eigensolver failed (%d)", rc);
      }
    } else {
      char *ews = (char *)dal(eig_workspace_bytes_padded(m, P, Pb, ctx->maxit));
      double *Ld = (double *)dal((size_t)P * N * kmax * 8);
      if (!ews || !Ld) return fail(ctx, 1002, "dfm_windows: out of device memory");
      rc = eig_run(G, N, (int64_t)N * N, N, P, kmax, p, nullptr, 0, ctx->tol, ctx->maxit, ctx->poll, ews, lam, Uk,
                   tr, stt, nullptr, st, timer_cb, ctx, 0);
      if (rc) return fail(ctx, rc > 0 ? rc : -21, "eigensolver failed (%d)", rc);
      Scope sc(ctx, DFM_KC_FACTORS);
      launch_factors(1, msrc, T, N, kmax, P, Uk, F, Ld, nullptr, st);
    }
    if (orient == 0) {
      Scope sc(ctx, DFM_KC_FACTORS);
      hipLaunchKernelGGL(window_scale_kernel, dim3((unsigned)(((int64_t)T * kmax + 255) / 256), P), dim3(256), 0,
                         st, Uk, T, kmax, mv0, dmv, F);
    }
    std::vector<int> hs(P);
    HIPCHK(ctx, hipMemcpyAsync(hl.data(), lam, hl.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(ht.data(), tr, (size_t)P * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(hs.data(), stt, (size_t)P * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    for (int wi = 0; wi < P; ++wi)
      if (hs[wi]) return fail(ctx, 2, "eigensolver did not converge for window %d", wi);
  } else {
    HIPCHK(ctx, hipStreamSynchronize(st));
    for (int wi = 0; wi < P; ++wi) {   // eigenvalues and trace from the window's spectrum
      const int mw = orient == 0 ? nw(wi) : N;
      double s = 0.0;
      for (int j = mw - 1; j >= 0; --j) s += hev[(size_t)wi * pst + j];
      ht[wi] = s;
      for (int j = 0; j < kmax; ++j) hl[(size_t)wi * kmax + j] = hev[(size_t)wi * pst + j];
    }
  }
  // ---- per window on the host (arithmetic only): the IC sweep and r_w, or
  // the fixed / default r_w and its criterion value
  std::vector<double> ic(7 * (size_t)kmax);
  for (int wi = 0; wi < P; ++wi) {
    const int n = nw(wi);
    double s2 = NAN;
    if (pcp) {   // src/criteria.jl:18: V(ceil(m_w/2)) of the window's unrestricted fit = spectral tail
      const int mw = std::min(n, N), h = (mw + 1) / 2;
      double s = 0.0;
      for (int j = mw - 1; j >= h; --j) s += hev[(size_t)wi * pst + j];
      s2 = s / ((double)N * n);
    }
    const int kw = kmax_w(wi);
    int rsel = kw;
    double cv = NAN;
    if (ws.r == 0) {
      dfm_ic_sweep(&hl[(size_t)wi * kmax], kw, kw, ht[wi], n, N, s2, ic.data());
      int best = 0;
      for (int k = 1; k < kw; ++k)
        if (ic[(size_t)crit * kw + k] < ic[(size_t)crit * kw + best]) best = k;
      rsel = best + 1;
      cv = ic[(size_t)crit * kw + best];
    } else if (crit >= 0) {   // the workhorse constructor's criterion at r_w (:50)
      dfm_ic_sweep(&hl[(size_t)wi * kmax], kw, kw, ht[wi], n, N, s2, ic.data());
      cv = ic[(size_t)crit * kw + kw - 1];
    }
    hTn[wi] = n;
    hkr[wi] = rsel;
    hR0[wi] = aw(wi);
    r_out[wi] = rsel;
    if (crit_out) crit_out[wi] = cv;
    if (V_out) {
      double sacc = ht[wi];
      for (int j = 0; j < rsel; ++j) sacc -= hl[(size_t)wi * kmax + j];
      V_out[wi] = sacc / ((double)N * n);
    }
  }
  if (eig_out) std::copy(hl.begin(), hl.end(), eig_out);
  HIPCHK(ctx, hipMemcpyAsync(dTn, hTn.data(), (size_t)P * 4, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(dkr, hkr.data(), (size_t)P * 4, hipMemcpyHostToDevice, st));
  HIPCHK(ctx, hipMemcpyAsync(dR0, hR0.data(), (size_t)P * 4, hipMemcpyHostToDevice, st));
  // ---- wide: the r_w eigenvectors (kv = max_w r_w) and factors of every window
  if (wide) {
    kv = *std::max_element(hkr.begin(), hkr.end());
    lam = (double *)dal((size_t)P * kv * 8); Uk = (double *)dal((size_t)P * m * kv * 8);
    F = (double *)dal((size_t)P * T * kv * 8);
    double *dwk = (double *)dal((size_t)P * dense_eig_work(m, kv) * 8);
    if (!lam || !Uk || !F || !dwk) return fail(ctx, 1002, "dfm_windows: out of device memory");
    hipError_t e;
    {
      Scope sc(ctx, DFM_KC_EIG_OTHER);
      e = orient == 0 ? launch_dense_eig_batched(Hb, ldH, sHb, T, mv0, dmv, P, kv, lam, Uk, tr, stt, dwk, st)
                      : launch_dense_eig_batched(G, N, (int64_t)N * N, N, N, 0, P, kv, lam, Uk, tr, stt, dwk, st);
    }
    if (e != hipSuccess) return fail(ctx, 1000 + (int)e, "dense eigensolver: %s", hipGetErrorString(e));
    Scope sc(ctx, DFM_KC_FACTORS);
    if (orient == 0) {
      hipLaunchKernelGGL(window_scale_kernel, dim3((unsigned)(((int64_t)T * kv + 255) / 256), P), dim3(256), 0, st,
                         Uk, T, kv, mv0, dmv, F);
    } else {
      double *Ld = (double *)dal((size_t)P * N * kv * 8);
      if (!Ld) return fail(ctx, 1002, "dfm_windows: out of device memory");
      if (kv <= 32) {
        launch_factors(1, msrc, T, N, kv, P, Uk, F, Ld, nullptr, st);
      } else {
        double *Xw = (double *)dal((size_t)P * T * dp.ld * 8);
        if (!Xw) return fail(ctx, 1002, "dfm_windows: out of device memory");
        HIPCHK(ctx, launch_materialize(msrc, T, N, dp.ld, P, Xw, st));
        if (launch_factors_wide(1, Xw, dp.ld, T, N, kv, Uk, F, Ld, nullptr, st, (double)T, P, (int64_t)T * dp.ld,
                                (int64_t)T * kv))
          return fail(ctx, 1001, "factor kernels failed");
      }
    }
  }
  // ---- OLS + HC2 of every window on [w F_{r_w}] over its rows
  const int dv = q + kv;
  double *coef = (double *)dal((size_t)P * dv * 8), *tst = (double *)dal((size_t)P * dv * 8);
  if (!coef || !tst) return fail(ctx, 1002, "dfm_windows: out of device memory");
  if (dv <= 32) {
    Scope sc(ctx, DFM_KC_OLS);
    launch_ols(P, st, dy, dw, q, F, T, kv, dTn, dkr, coef, tst, nullptr, nullptr, ost, len > 0 ? dR0 : nullptr);
  } else {   // per window: its own width q + r_w
    const int dmax = q + kv;
    double *owk = (double *)dal((size_t)ols_wide_work(T, dmax) * 8);
    if (!owk) return fail(ctx, 1002, "dfm_windows: out of device memory");
    Scope sc(ctx, DFM_KC_OLS);
    for (int wi = 0; wi < P; ++wi)
      HIPCHK(ctx, launch_ols_wide_batched(1, dy + hR0[wi], dw + hR0[wi], q, F + (size_t)wi * T * kv, T, kv, hkr[wi],
                                          dTn + wi, coef + (size_t)wi * dv, tst + (size_t)wi * dv, nullptr, nullptr,
                                          ost + wi, owk, st));
  }
  {
    std::vector<int> ho(P);
    HIPCHK(ctx, hipMemcpyAsync(ho.data(), ost, (size_t)P * 4, hipMemcpyDeviceToHost, st));
    std::vector<int> hs2(P, 0);
    if (wide) HIPCHK(ctx, hipMemcpyAsync(hs2.data(), stt, (size_t)P * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    for (int wi = 0; wi < P; ++wi) {
      if (hs2[wi]) return fail(ctx, 2, "dense eigensolver: window %d lost orthogonality", wi);
      if (ho[wi]) return fail(ctx, 3, "singular design matrix in window %d", wi);
    }
  }
  // outputs keep the q + kmax row stride of the header (NaN past q + r_w)
  auto restride = [&](const double *dsrc, double *out) -> int {
    std::vector<double> h((size_t)P * dv);
    LCKW(hipMemcpyAsync(h.data(), dsrc, h.size() * 8, hipMemcpyDeviceToHost, st));
    LCKW(hipStreamSynchronize(st));
    const int dk = q + kmax;
    for (int wi = 0; wi < P; ++wi)
      for (int c = 0; c < dk; ++c)
        out[(size_t)wi * dk + c] = (c < dv && c < q + hkr[wi]) ? h[(size_t)wi * dv + c] : NAN;
    return 0;
  };
  if (coef_out && (rc = restride(coef, coef_out))) return rc;
  if (tstat_out && (rc = restride(tst, tstat_out))) return rc;
  if (pred_out) {   // forecast step: predict row n = n0 + w from window w's fit
    double *rs = (double *)dal((size_t)T * 8), *ss = (double *)dal((size_t)T * 8);
    double *dp_ = (double *)dal((size_t)P * 8), *dt_ = (double *)dal((size_t)P * 8);
    if (!rs || !ss || !dp_ || !dt_) return fail(ctx, 1002, "dfm_windows: out of device memory");
    Scope sc(ctx, DFM_KC_MISC);
    hipLaunchKernelGGL(panel_row_sums_kernel, dim3(T), dim3(256), 0, st, dp.P, dp.ld, N, rs, ss);
    hipLaunchKernelGGL(window_forecast_kernel, dim3(P), dim3(256), 0, st, orient, dp.P, dp.ld, T, N, n0, len, q, kv,
                       H, ldH, F, Uk, lam, rs, ss, dkr, coef, dy, dw, dp_, dt_);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(pred_out, dp_, (size_t)P * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(true_out, dt_, (size_t)P * 8, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

// Expanding windows of a model with structural breaks (model_args'
// break_indices, src/utils.jl:64 -> src/DynamicFactorModel.jl:73, :98): each
// window is the break-aware fit of dfm_model_fit_breaks on its leading rows
// (per-block PCA with the window's full-sample T, N, D7), read back, and —
// for the forecast step — dfm_predict on the next row.  X, y, w host or
// device memory (the fit copies with hipMemcpyDefault).
static int windows_breaks_impl(dfm_ctx *ctx, const double *y, const double *w, int q, int64_t ldw, const double *X,
                               int T, int N, int64_t ldx, int P, const WinSpec &ws, int K, int64_t *r_out,
                               double *V_out, double *crit_out, double *eig_out, double *coef_out,
                               double *tstat_out, double *pred_out, double *true_out) {
  const int n0 = T - P;
  for (int j = 0; j < ws.nbreaks; ++j)
    if (ws.breaks[j] >= n0)
      return fail(ctx, -9, "dfm_windows: break row %lld is not inside the first window (%d rows)",
                  (long long)ws.breaks[j], n0);
  for (int wi = 0; wi < P; ++wi) {
    const int n = n0 + wi;
    const int kd = (std::min(n, N) + 1) / 2;
    const int rarg = ws.r > 0 ? ws.r : (ws.r < 0 ? kd : 0);
    dfm_model *M = nullptr;
    int rc = dfm_model_fit_breaks(ctx, y, w, q, ldw, X, n, N, ldx, rarg, ws.crit, ws.kmax, ws.breaks, ws.nbreaks,
                                  &M);
    if (rc) return rc;
    struct Kill { dfm_model *m; ~Kill() { dfm_model_destroy(m); } } kill{M};
    int64_t r = 0, kmx = 0, ne = 0;
    double V = 0, cv = 0, tr = 0;
    dfm_model_scalars(M, &r, &V, &cv, &tr);
    dfm_model_dims(M, &r, &kmx, &ne);
    const int d = q + (int)r;
    std::vector<double> ev(ne), co(d), ts(d);
    if ((rc = dfm_model_read(M, ev.data(), co.data(), ts.data(), nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr)))
      return rc;
    r_out[wi] = r;
    if (V_out) V_out[wi] = V;
    if (crit_out) crit_out[wi] = ws.crit >= 0 ? cv : NAN;
    if (eig_out)
      for (int j = 0; j < K; ++j) eig_out[(size_t)wi * K + j] = j < ne ? ev[j] : NAN;
    const int dk = q + K;
    for (int c = 0; c < dk; ++c) {
      if (coef_out) coef_out[(size_t)wi * dk + c] = c < d ? co[c] : NAN;
      if (tstat_out) tstat_out[(size_t)wi * dk + c] = c < d ? ts[c] : NAN;
    }
    if (pred_out) {   // predict row n from this window's fit (D4-repaired get_factors)
      if ((rc = dfm_predict(M, 1, q > 0 ? w + n : nullptr, ldw, X + n, ldx, pred_out + wi))) return rc;
      HIPCHK(ctx, hipMemcpy(true_out + wi, y + n, 8, hipMemcpyDefault));
    }
  }
  return 0;
}

// ---- get_factors / predict on new rows (src/DynamicFactorModel.jl:125-128,
// :152-155; D4 repaired, dfm_predict.hip).  x_new (nn x N) and w_new (nn x q)
// column-major, host or device memory (hipMemcpyDefault); outputs host.
static int predict_impl(dfm_model *M, int64_t nn, const double *w_new, int64_t ldw, const double *x_new,
                        int64_t ldx, double *F_out, double *yhat) {
  if (!M) return -1;
  dfm_ctx *ctx = M->ctx;
  const int q = M->q, r = M->r, N = M->N, T = M->T;
  if (nn < 1 || !x_new || ldx < nn || (yhat && q > 0 && (!w_new || ldw < nn)) || (!F_out && !yhat))
    return fail(ctx, -2, "dfm_predict: bad arguments");
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  double *xd = nullptr, *wd = nullptr, *bd = nullptr, *wk = nullptr, *Fd = nullptr, *yd = nullptr;
  struct Fr { std::vector<double *> v; ~Fr() { for (double *p : v) hipFree(p); } } fr;
  auto al = [&](double **p, size_t n) { hipError_t e = dalloc(p, n); if (e == hipSuccess) fr.v.push_back(*p); return e; };
  HIPCHK(ctx, al(&xd, (size_t)nn * N));
  HIPCHK(ctx, al(&wd, (size_t)nn * std::max(q, 1)));
  HIPCHK(ctx, al(&bd, (size_t)q + r));
  HIPCHK(ctx, al(&wk, (size_t)T + 2));
  HIPCHK(ctx, al(&Fd, (size_t)nn * std::max(r, 1)));
  HIPCHK(ctx, al(&yd, (size_t)nn));
  HIPCHK(ctx, hipMemcpy2DAsync(xd, (size_t)nn * 8, x_new, (size_t)ldx * 8, (size_t)nn * 8, N, hipMemcpyDefault, st));
  if (yhat && q > 0)
    HIPCHK(ctx, hipMemcpy2DAsync(wd, (size_t)nn * 8, w_new, (size_t)ldw * 8, (size_t)nn * 8, q, hipMemcpyDefault, st));
  HIPCHK(ctx, hipMemcpyAsync(bd, M->coef.data(), (size_t)(q + r) * 8, hipMemcpyHostToDevice, st));
  {
    Scope sc(ctx, DFM_KC_MISC);
    HIPCHK(ctx, launch_predict(M->Xp, M->ld, T, N, M->L, r, xd, nn, nn, wd, nn, q, yhat ? bd : nullptr, wk, Fd, yd,
                               st));
  }
  if (F_out) HIPCHK(ctx, hipMemcpyAsync(F_out, Fd, (size_t)nn * r * 8, hipMemcpyDeviceToHost, st));
  if (yhat) HIPCHK(ctx, hipMemcpyAsync(yhat, yd, (size_t)nn * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

extern "C" int dfm_get_factors(dfm_model *m, int64_t n_new, const double *x_new, int64_t ldx, double *F_out) {
  if (!F_out) return m ? fail(m->ctx, -2, "dfm_get_factors: output required") : -1;
  return predict_impl(m, n_new, nullptr, 0, x_new, ldx, F_out, nullptr);
}

extern "C" int dfm_predict(dfm_model *m, int64_t n_new, const double *w_new, int64_t ldw, const double *x_new,
                           int64_t ldx, double *out) {
  if (!out) return m ? fail(m->ctx, -2, "dfm_predict: output required") : -1;
  return predict_impl(m, n_new, w_new, ldw, x_new, ldx, nullptr, out);
}

// ------------------------------------------------------------------ normalize
// normalize (src/utils.jl:33): (A .- mean(A, 1)) ./ std(A, 1) — column z-score
// with the sample std (n - 1 denominator), two passes over the column (mean,
// then the centred sum of squares), then the scaled write.  One wave per
// column of the column-major panel (contiguous in Julia's layout: coalesced);
// Y may alias X.
__global__ __launch_bounds__(256) void normalize_cols_kernel(const double *X, int64_t ldx, int T, int N, double *Y,
                                                             int64_t ldy) {
  const int lane = threadIdx.x & 63, c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= N) return;
  const double *x = X + (int64_t)c * ldx;
  double s = 0.0;
  for (int t = lane; t < T; t += 64) s += x[t];
  const double mu = wave_sum(s) / T;
  double v = 0.0;
  for (int t = lane; t < T; t += 64) { const double d = x[t] - mu; v = fma(d, d, v); }
  const double sd = sqrt(wave_sum(v) / (T - 1));
  double *y = Y + (int64_t)c * ldy;
  for (int t = lane; t < T; t += 64) y[t] = (x[t] - mu) / sd;
}

extern "C" int dfm_normalize_dev(dfm_ctx *ctx, const double *X, int64_t T, int64_t N, int64_t ldx, double *out,
                                 int64_t ldo) {
  if (!ctx) return -1;
  if (!X || !out || T < 2 || N < 1 || ldx < T || ldo < T || T > INT32_MAX || N > INT32_MAX)
    return fail(ctx, -2, "dfm_normalize: bad arguments");
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  Scope sc(ctx, DFM_KC_MISC);
  hipLaunchKernelGGL(normalize_cols_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, ctx->stream, X, ldx, (int)T,
                     (int)N, out, ldo);
  HIPCHK(ctx, hipGetLastError());
  return 0;
}

extern "C" int dfm_normalize(dfm_ctx *ctx, const double *X, int64_t T, int64_t N, int64_t ldx, double *out,
                             int64_t ldo) {
  if (!ctx) return -1;
  if (!X || !out || T < 2 || N < 1 || ldx < T || ldo < T) return fail(ctx, -2, "dfm_normalize: bad arguments");
  DeviceShare gate(ctx->device);
  hipSetDevice(ctx->device);
  hipStream_t st = ctx->stream;
  DevBuf d;
  HIPCHK(ctx, dalloc(&d.p, (size_t)T * N));
  HIPCHK(ctx, hipMemcpy2DAsync(d.p, (size_t)T * 8, X, (size_t)ldx * 8, (size_t)T * 8, N, hipMemcpyHostToDevice, st));
  int rc = dfm_normalize_dev(ctx, d.p, T, N, T, d.p, T);
  if (rc) return rc;
  HIPCHK(ctx, hipMemcpy2DAsync(out, (size_t)ldo * 8, d.p, (size_t)T * 8, (size_t)T * 8, N, hipMemcpyDeviceToHost, st));
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

// ------------------------------------------------------------ multi-device
// A fitted model copied onto another context (another GPU, or a second
// context of the same GPU): every device buffer and host field, so the copy's
// bootstrap replicates are bit-identical to the original's.
extern "C" int dfm_model_clone(const dfm_model *S, dfm_ctx *ctx, dfm_model **out) {
  if (!S || !ctx || !out) return -1;
  *out = nullptr;
  dfm_ctx *sc = S->ctx;
  DeviceShare gate_src(sc->device), gate_dst(ctx->device);
  hipSetDevice(sc->device);
  HIPCHK(ctx, hipStreamSynchronize(sc->stream));
  dfm_model *M = new dfm_model();
  ++ctx->refs;
  M->ctx = ctx;
  M->T = S->T; M->N = S->N; M->q = S->q; M->r = S->r; M->crit = S->crit; M->kmax = S->kmax; M->m = S->m;
  M->orient = S->orient; M->k_eig = S->k_eig; M->swept = S->swept; M->ld = S->ld;
  M->lam = S->lam; M->coef = S->coef; M->tstat = S->tstat; M->cov = S->cov; M->resid = S->resid; M->ic = S->ic;
  M->trace = S->trace; M->V = S->V; M->critval = S->critval; M->sigma2 = S->sigma2;
  M->batch = S->batch; M->mode = S->mode;
  M->nblk = S->nblk; M->ba = S->ba; M->bt = S->bt; M->bm = S->bm; M->blam = S->blam;
  // device-to-device (peer) copies: no staging through host memory.  They are
  // issued on the NEW context's stream and completed before the clone is
  // returned: hipMemcpyPeer would run them on the legacy null stream, which
  // returns before a device-to-device copy lands and which the context's
  // non-blocking stream does not wait for — round 4's intermittent wrong
  // two-lane rows were the second lane's first kernels (H = E E', EL = E L,
  // F S F', the warm start) reading a partly copied fit
  // (tests/test_gpu_multi.py::test_clone_is_complete_before_its_first_bootstrap)
  auto dup = [&](const double *src, size_t n, double **dst) -> int {
    hipSetDevice(ctx->device);
    if (dalloc(dst, n) != hipSuccess) return 1;
    if (!src || n == 0) return 0;
    return hipMemcpyPeerAsync(*dst, ctx->device, src, sc->device, n * 8, ctx->stream) == hipSuccess ? 0 : 1;
  };
  const size_t T = S->T, N = S->N, r = S->r, panel = T * S->ld;
  int bad = 0;
  bad |= dup(S->Xp, panel, &M->Xp);
  bad |= dup(S->Cp, panel, &M->Cp);
  bad |= dup(S->Ep, panel, &M->Ep);
  bad |= dup(S->y, T, &M->y);
  bad |= dup(S->w, T * std::max(S->q, 1), &M->w);
  bad |= dup(S->F, T * r, &M->F);
  bad |= dup(S->colssr, N, &M->colssr);
  bad |= dup(S->Lall, (size_t)S->nblk * N * r, &M->Lall);
  M->Ubs.assign(S->nblk, nullptr);
  M->Ls.assign(S->nblk, nullptr);
  for (int j = 0; j < S->nblk && !bad; ++j) {
    bad |= dup(S->Ubs[j], (size_t)S->bm[j] * r, &M->Ubs[j]);
    M->Ls[j] = M->Lall + (size_t)j * N * r;
  }
  M->Ub = M->Ubs.empty() ? nullptr : M->Ubs[0];
  M->L = M->Lall;
  hipSetDevice(ctx->device);
  if (!bad) bad = dalloc(&M->flag_dev, 4) != hipSuccess;
  if (!bad) bad = hipStreamSynchronize(ctx->stream) != hipSuccess;   // every copy landed
  if (bad) {
    dfm_model_destroy(M);
    return fail(ctx, 1002, "dfm_model_clone: device copy failed");
  }
  *out = M;
  return 0;
}

// wild_bootstrap / residual_bootstrap (src/bootstrap.jl:21-51) with the
// replicate loop (:43) sharded over n models (one per context, typically one
// per GPU, each a dfm_model_clone of the same fit): replicate b runs on model
// floor(b n / B), i.e. contiguous shards, each driven by its own host thread
// on its own stream; rows land in order in the caller's out (B x width).
// No collective: the shards are independent and the host buffer is the
// gather.  Contexts must be distinct (one host thread per context).
extern "C" int dfm_bootstrap_multi(dfm_model *const *models, int n, int kind, int64_t B, const int32_t *idx,
                                   const double *eta, const dfm_stat *stats, int ns, double *out) {
  if (!models || n < 1 || !models[0]) return -1;
  dfm_ctx *c0 = models[0]->ctx;
  for (int g = 0; g < n; ++g) {
    if (!models[g]) return fail(c0, -2, "dfm_bootstrap_multi: model %d is NULL", g);
    const dfm_model *a = models[g], *b = models[0];
    if (a->T != b->T || a->N != b->N || a->r != b->r || a->q != b->q || a->nblk != b->nblk || a->crit != b->crit)
      return fail(c0, -2, "dfm_bootstrap_multi: model %d is not a copy of model 0", g);
    for (int h = 0; h < g; ++h)
      if (models[h]->ctx == a->ctx) return fail(c0, -2, "dfm_bootstrap_multi: models %d and %d share a context", h, g);
  }
  if (B < 0 || !idx || (kind == DFM_BOOT_WILD && !eta)) return fail(c0, -2, "dfm_bootstrap_multi: bad arguments");
  if (B == 0) return 0;
  const int64_t width = dfm_stats_width(models[0], stats, ns);
  if (width < 0) return fail(c0, -2, "dfm_bootstrap_multi: bad stat list");
  const int64_t T = models[0]->T;
  std::vector<int> rcs(n, 0);
  std::vector<std::thread> th;
  for (int g = 0; g < n; ++g) {
    const int64_t b0 = ((int64_t)g * B + n - 1) / n, b1 = ((int64_t)(g + 1) * B + n - 1) / n;
    if (b1 <= b0) continue;
    th.emplace_back([=, &rcs]() {
      rcs[g] = dfm_bootstrap(models[g], kind, b1 - b0, idx + b0 * T, eta ? eta + b0 * T : nullptr, stats, ns,
                             out ? out + b0 * width : nullptr);
    });
  }
  for (auto &t : th) t.join();
  for (int g = 0; g < n; ++g)
    if (rcs[g]) {
      const std::string msg = models[g]->ctx->err;
      return fail(c0, rcs[g], "shard %d: %s", g, msg.c_str());
    }
  return 0;
}
