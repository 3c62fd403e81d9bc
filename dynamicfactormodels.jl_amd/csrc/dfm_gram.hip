// dfm_gram.hip — K1: batched fp64 Gram of resampled panels, fused gather, MFMA.
//
// Replaces the Gram + LAPACK front of principal_components
// (src/DynamicFactorModel.jl:78 `x'x` for T >= N, :87 `x*x'` for N > T),
// evaluated on the bootstrap panel X* = F_r L_r' + diag(eta) E[idx, :]
// (src/bootstrap.jl:44-45) without materialising X*.
//
// Orientation ROWS (N > T): G = X* X*'  (m = T, reduction over n = 0..N-1)
// Orientation COLS (T >= N): G = X*' X* (m = N, reduction over t = 0..T-1)
//
// Tiling: one 256-thread workgroup per 64x64 lower-triangular output tile of
// one replicate; 4 waves each own a 32x32 sub-tile = 8x8 fragments of 4x4.
// Each 16-deep k-step issues 64 v_mfma_f64_4x4x4_4b_f64 per wave: the four
// MFMA blocks split the 16-deep reduction 4 ways and are summed once in the
// epilogue (transpose-reduce: 3 shuffles per 4 accumulators).  Operands are
// gathered + fused (C + eta*E[idx]) while staged through a double-buffered,
// XOR-swizzled LDS image (conflict-free ds_read_b64 for the MFMA lane maps,
// conflict-free ds_write_b128 for the staging rows).  One barrier per k-step.
//
// Requirements: panels C/E have zero-filled padding columns N..ld-1 and
// ld % 16 == 0.  Output G is the full symmetric m x m matrix (row-major, ldg).
#include <algorithm>
#include <cstdlib>

#include "dfm_common.h"

namespace dfm {

constexpr int GT = 64;  // workgroup output tile
constexpr int KS = 16;  // k per stage == one MFMA k-step
enum { ORIENT_ROWS = 0, ORIENT_COLS = 1 };

// LDS image of one 64 x 16 operand tile (1024 doubles).
template <int ORIENT>
DFM_DEV int lds_off(int a, int kc) {
  if constexpr (ORIENT == ORIENT_ROWS) return a * KS + (kc ^ (((a >> 1) & 1) << 3));
  else return kc * GT + (a ^ ((kc & 7) << 2));
}

template <int ORIENT, bool HAS_C, bool HAS_ETA, bool HAS_IDX>
__global__ __launch_bounds__(256, 2) void gram_kernel(PanelSrc src, int m, int K, int T,
                                                      double *__restrict__ G, int64_t ldg,
                                                      int64_t strideG, int ksteps, int64_t strideZ, int kpre) {
  __shared__ __attribute__((aligned(16))) double lds[2][2][GT * KS];
  // COLS with kpre = K: the replicate's eta / idx rows staged in dynamic LDS
  // up front, so a k-row's gather is one load (E[idx_t]) instead of two
  // dependent ones (idx_t, then the row) per stage
  extern __shared__ double s_pre[];
  double *s_et = s_pre;
  int *s_ix = (int *)(s_pre + kpre);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int rep = blockIdx.y;
  // lower-triangular tile enumeration: t -> (I, J), I >= J
  const int tt = blockIdx.x;
  int I = (int)((sqrt(8.0 * tt + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= tt) ++I;
  while (I * (I + 1) / 2 > tt) --I;
  const int J = tt - I * (I + 1) / 2;
  const bool diag = (I == J);
  const int abase = I * GT, bbase = J * GT;

  const int32_t *idx = HAS_IDX ? src.idx + (int64_t)rep * src.rs : nullptr;
  const double *eta = HAS_ETA ? src.eta + (int64_t)rep * src.rs : nullptr;
  const int64_t ld = src.ld;

  // ---------------- staging state: each thread moves 2 x 16-B chunks per operand
  double2 rc[2][2], re[2][2];  // [operand][chunk] raw C and E values
  double ev[2][2];             // ROWS: per-row eta for [operand][chunk]
  const double *pC[2][2], *pE[2][2];
  bool rowok[2][2];

  if constexpr (ORIENT == ORIENT_ROWS) {
    // chunk c = tid + 256*h: row a = c >> 3, 16-B column pair j = c & 7
#pragma unroll
    for (int op = 0; op < 2; ++op)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int a = (tid >> 3) + 32 * h;
        const int row = (op == 0 ? abase : bbase) + a;
        rowok[op][h] = row < m;
        const int rr = rowok[op][h] ? row : 0;
        const int er = HAS_IDX ? idx[rr] : rr;
        ev[op][h] = HAS_ETA ? eta[rr] : 1.0;
        pC[op][h] = HAS_C ? src.C + (int64_t)rr * ld + 2 * (tid & 7) : nullptr;
        pE[op][h] = src.E + (int64_t)er * ld + 2 * (tid & 7);
      }
  }

  auto load_stage = [&](int k0) {
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      if (op == 1 && diag) break;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr (ORIENT == ORIENT_ROWS) {
          if (rowok[op][h]) {
            re[op][h] = *reinterpret_cast<const double2 *>(pE[op][h] + k0);
            if (HAS_C) rc[op][h] = *reinterpret_cast<const double2 *>(pC[op][h] + k0);
          }
        } else {
          // chunk c: k-row kc = c >> 5 (t = k0 + kc), column pair j = c & 31
          const int kc = (tid >> 5) + 8 * h;
          const int t = k0 + kc;
          const int col = (op == 0 ? abase : bbase) + 2 * (tid & 31);
          const bool ok = (t < K) && (col < ld);
          rowok[op][h] = ok;
          if (ok) {
            const int er = HAS_IDX ? (kpre ? s_ix[t] : idx[t]) : t;
            ev[op][h] = HAS_ETA ? (kpre ? s_et[t] : eta[t]) : 1.0;
            re[op][h] = *reinterpret_cast<const double2 *>(src.E + (int64_t)er * ld + col);
            if (HAS_C) rc[op][h] = *reinterpret_cast<const double2 *>(src.C + (int64_t)t * ld + col);
          }
        }
      }
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      if (op == 1 && diag) break;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double2 v = {0.0, 0.0};
        if (rowok[op][h]) {
          const double e = ev[op][h];
          v.x = HAS_C ? fma(e, re[op][h].x, rc[op][h].x) : (HAS_ETA ? e * re[op][h].x : re[op][h].x);
          v.y = HAS_C ? fma(e, re[op][h].y, rc[op][h].y) : (HAS_ETA ? e * re[op][h].y : re[op][h].y);
        }
        int off;
        if constexpr (ORIENT == ORIENT_ROWS) off = lds_off<ORIENT>((tid >> 3) + 32 * h, 2 * (tid & 7));
        else off = lds_off<ORIENT>(2 * (tid & 31), (tid >> 5) + 8 * h);
        *reinterpret_cast<double2 *>(&lds[buf][op][off]) = v;
      }
    }
  };

  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0;

  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  // split-K: this workgroup reduces k-steps [s0, s1) (blockIdx.z) into its
  // own partial image (strideZ apart); launch_gram sums them in fixed order
  const int s0 = blockIdx.z * ksteps;
  const int nst = min((K + KS - 1) / KS, s0 + ksteps);
  if (ORIENT == ORIENT_COLS && kpre) {
    for (int e = tid; e < kpre; e += 256) {
      if (HAS_ETA) s_et[e] = eta[e];
      if (HAS_IDX) s_ix[e] = idx[e];
    }
    __syncthreads();
  }
  load_stage(s0 * KS);
  store_stage(0);
  __syncthreads();
  for (int s = s0; s < nst; ++s) {
    const int buf = (s - s0) & 1;
    if (s + 1 < nst) load_stage((s + 1) * KS);
    const double *la = lds[buf][0];
    const double *lb = diag ? lds[buf][0] : lds[buf][1];
    double af[8], bf[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = la[lds_off<ORIENT>(wr * 32 + 4 * f + fi, fkc)];
      bf[f] = lb[lds_off<ORIENT>(wc * 32 + 4 * f + fi, fkc)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma4(af[i], bf[j], acc[i][j]);
    if (s + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue: transpose-reduce over the 4 MFMA blocks, store
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
  double *Gr = G + (int64_t)rep * strideG + (int64_t)blockIdx.z * strideZ;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double a0 = acc[fa][4 * q + 0], a1 = acc[fa][4 * q + 1];
      const double a2 = acc[fa][4 * q + 2], a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int row = abase + wr * 32 + 4 * fa + oi;
      const int col = bbase + wc * 32 + 16 * q + 4 * blk + oj;
      if (row < m && col < m) {
        Gr[(int64_t)row * ldg + col] = v;
        if (!diag) Gr[(int64_t)col * ldg + row] = v;
      }
    }
}

// Fixed-order sum of the split-K partial images: G[r] = sum_z W[r][z].
__global__ void gram_splitk_sum_kernel(const double *__restrict__ W, int S, int m, int64_t ldg,
                                       int64_t elems, double *__restrict__ G, int64_t strideG, double alpha) {
  const int r = blockIdx.y;
  const double *w = W + (int64_t)r * S * elems;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < elems; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / ldg, j = e - i * ldg;
    if (j >= m) continue;
    double a = 0.0;
    for (int z = 0; z < S; ++z) a += w[(int64_t)z * elems + e];
    G[(int64_t)r * strideG + i * ldg + j] = a * alpha;
  }
}

// K-split of one Gram: a function of (m, K) only — never of the batch — so a
// replicate's Gram is bit-identical however the replicates are batched.  A
// lone large Gram (C5's prefix Gram: m = 2000, 528 tiles of 64 x 64 over 20000
// columns) otherwise runs 1.03 rounds of a 512-slot chip; split over the
// reduction it fills ~13 rounds at 96 %.
int gram_ksplit(int m, int K) {
  const int nt = (m + GT - 1) / GT, tiles = nt * (nt + 1) / 2;
  if (tiles < 64 || K < 4096) return 1;
  return std::max(1, std::min(16, K / 1536));
}

hipError_t launch_gram_dma(const double *X, int64_t ld, int m, int K, int S, int ksteps, double *G, int64_t ldg,
                           int64_t strideZ, hipStream_t st, double alpha);
int gram_dma_slots(int m);
// K-split of ONE plain-panel Gram (no replicate batch, so no batch
// invariance to keep): enough (tile, split) workgroups to fill the chip's
// resident slots (gram_dma_slots) several times over with a last round >= 90 % full, each
// split >= 256 deep.  C5's prefix Gram (528 tiles, K = 20000): S = 7.
int gram_ksplit_single(int m, int K) {
  const int nt = (m + GT - 1) / GT, tiles = nt * (nt + 1) / 2, slots = gram_dma_slots(m);
  const int smax = std::max(1, std::min(32, K / 256));
  for (int S = 1; S <= smax; ++S) {
    const int64_t items = (int64_t)tiles * S, rounds = (items + slots - 1) / slots;
    if (items >= 4 * slots && items * 10 >= rounds * slots * 9) return S;
  }
  if ((int64_t)tiles * smax <= slots) return smax;   // small Gram: one partial round, deepest split
  int best = 1;
  double beff = 0.0;
  for (int S = 1; S <= smax; ++S) {
    const int64_t items = (int64_t)tiles * S, rounds = (items + slots - 1) / slots;
    const double eff = (double)items / (double)(rounds * slots);
    if (items >= slots && eff > beff + 1e-9) { beff = eff; best = S; }
  }
  return best;
}

static hipError_t launch_gram_a(int orient, const PanelSrc &src, int m, int K, int T, double *G, int64_t ldg,
                                int64_t strideG, int nrep, hipStream_t st, double alpha);
// Dispatch.  Returns hipError of the launch.
hipError_t launch_gram(int orient, const PanelSrc &src, int m, int K, int T, double *G,
                       int64_t ldg, int64_t strideG, int nrep, hipStream_t st) {
  return launch_gram_a(orient, src, m, K, T, G, ldg, strideG, nrep, st, 1.0);
}
// G = alpha X X' of ONE plain row-major panel (m >= 64, ld % 16 == 0, zero
// columns K..ld-1) on the LDS-DMA SYRK, alpha applied in the epilogue (or in
// the split-K sum): the soft-threshold Grams' 1/n_f without a pass over G.
// hipErrorInvalidValue when the panel does not take the LDS-DMA path.
hipError_t launch_gram_plain_scaled(const double *X, int64_t ld, int m, int K, double *G, int64_t ldg, double alpha,
                                    hipStream_t st) {
  if (m < GT || ld % 16 != 0) return hipErrorInvalidValue;
  PanelSrc src{nullptr, X, nullptr, nullptr, ld, 0};
  return launch_gram_a(ORIENT_ROWS, src, m, K, K, G, ldg, 0, 1, st, alpha);
}
static hipError_t launch_gram_a(int orient, const PanelSrc &src, int m, int K, int T, double *G, int64_t ldg,
                                int64_t strideG, int nrep, hipStream_t st, double alpha) {
  const int nt = (m + GT - 1) / GT;
  const int nsteps = (K + KS - 1) / KS;
  const bool plain = orient == ORIENT_ROWS && !src.C && !src.eta && !src.idx && src.ld % 16 == 0 && nrep == 1 &&
                     m >= GT;
  const int S0 = plain ? gram_ksplit_single(m, K) : gram_ksplit(m, K);
  const int ksteps = (nsteps + S0 - 1) / S0, S = (nsteps + ksteps - 1) / ksteps;
  double *Gk = G, *W = nullptr;
  int64_t sG = strideG, sZ = 0;
  const int64_t elems = (int64_t)m * ldg;
  int nrc = nrep;   // replicates per launch (bounds the partial images to ~1 GB)
  if (S > 1) {
    nrc = (int)std::max<int64_t>(1, std::min<int64_t>(nrep, ((int64_t)1 << 27) / (elems * S)));
    hipError_t e = stream_malloc((void **)&W, (size_t)nrc * S * elems * 8, st);
    if (e != hipSuccess) return e;
    Gk = W; sZ = elems; sG = elems * S;
  }
  const bool c = src.C != nullptr, e = src.eta != nullptr, x = src.idx != nullptr;
  // a plain row-major panel (no fused gather): LDS-DMA SYRK (dfm_gemm.hip).
  // The k-split counts 16-deep steps of both kernels alike, so the partial
  // sums (and the result bits) do not depend on which kernel ran.
  if (plain) {
    hipError_t er = launch_gram_dma(src.E, src.ld, m, K, S, ksteps, Gk, ldg, sZ, st, S > 1 ? 1.0 : alpha);
    if (er == hipSuccess && S > 1)
      hipLaunchKernelGGL(gram_splitk_sum_kernel, dim3((unsigned)std::min<int64_t>((elems + 255) / 256, 4096), 1),
                         dim3(256), 0, st, W, S, m, ldg, elems, G, strideG, alpha);
    if (W) hipFreeAsync(W, st);
    return er != hipSuccess ? er : hipGetLastError();
  }
  for (int r0 = 0; r0 < nrep; r0 += nrc) {
  const int nr = std::min(nrc, nrep - r0);
  PanelSrc sub = src;
  if (x) sub.idx = src.idx + (int64_t)r0 * src.rs;
  if (e) sub.eta = src.eta + (int64_t)r0 * src.rs;
  double *Gout = S > 1 ? Gk : G + (int64_t)r0 * strideG;
  dim3 grid(nt * (nt + 1) / 2, nr, S), block(256);
  // COLS gather rows staged in LDS when they fit (C2: K = 600, 7.2 KB)
  const int kpre = (orient == ORIENT_COLS && (e || x) && K <= 2048) ? K : 0;
  const size_t dyn = (size_t)kpre * 12;
#define DFM_GRAM_L(O, C_, E_, X_) \
  hipLaunchKernelGGL((gram_kernel<O, C_, E_, X_>), grid, block, dyn, st, sub, m, K, T, Gout, ldg, sG, ksteps, sZ, \
                     kpre)
  if (orient == ORIENT_ROWS) {
    if (c && e && x) DFM_GRAM_L(ORIENT_ROWS, true, true, true);
    else if (c && !e && x) DFM_GRAM_L(ORIENT_ROWS, true, false, true);
    else if (!c && !e && !x) DFM_GRAM_L(ORIENT_ROWS, false, false, false);
    else if (!c && e && x) DFM_GRAM_L(ORIENT_ROWS, false, true, true);
    else if (!c && !e && x) DFM_GRAM_L(ORIENT_ROWS, false, false, true);
    else return hipErrorInvalidValue;
  } else {
    if (c && e && x) DFM_GRAM_L(ORIENT_COLS, true, true, true);
    else if (c && !e && x) DFM_GRAM_L(ORIENT_COLS, true, false, true);
    else if (!c && !e && !x) DFM_GRAM_L(ORIENT_COLS, false, false, false);
    else if (!c && e && x) DFM_GRAM_L(ORIENT_COLS, false, true, true);
    else if (!c && !e && x) DFM_GRAM_L(ORIENT_COLS, false, false, true);
    else return hipErrorInvalidValue;
  }
#undef DFM_GRAM_L
  if (S > 1) {
    hipLaunchKernelGGL(gram_splitk_sum_kernel, dim3((unsigned)std::min<int64_t>((elems + 255) / 256, 4096), nr),
                       dim3(256), 0, st, W, S, m, ldg, elems, G + (int64_t)r0 * strideG, strideG, 1.0);
  }
  }
  if (W) hipFreeAsync(W, st);
  return hipGetLastError();
}

}  // namespace dfm

namespace dfm {

// ---------------------------------------------------------------------------
// T >= N bootstrap Grams without the per-replicate SYRK (C2: 130 x 130 Grams
// of 600 resampled rows, where 64 x 64 tiles waste 65 % of the MFMA work).
// With X* = C + D P E (C = F L' the base common component, D = diag(eta),
// P the row selection idx):
//   X*'X* = C'C + L B + (L B)' + E' diag(w) E,
//   B = F' D P E (r x N),  w_s = sum_{t : idx_t = s} eta_t^2,
// and E' diag(w) E = sum_s w_s vec(E_s' E_s): for the whole batch ONE MFMA
// GEMM  Q (nb x NP) = W (nb x T) K (T x NP), K[s][(n, m)] = E[s][n] E[s][m]
// over the NP = N(N+1)/2 lower-triangle pairs (precomputed once per model).
// Every replicate's Gram is then A0 + L B + (L B)' + unpack(Q), each lower
// tile computed once and stored with its transpose (exactly symmetric).
// Per-replicate sums run in a fixed order: results are batch-invariant.

// K[s][n(n+1)/2 + m] = E[s][n] E[s][m] (m <= n); rows T..Tp-1 and pad column zero
__global__ void gram_wk_kmat_kernel(const double *__restrict__ Ep, int64_t ld, int T, int N, int64_t ldk,
                                    double *__restrict__ K) {
  const int s = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= ldk) return;
  double v = 0.0;
  const int64_t NP = (int64_t)N * (N + 1) / 2;
  if (s < T && e < NP) {
    int n = (int)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
    while ((int64_t)(n + 1) * (n + 2) / 2 <= e) ++n;
    while ((int64_t)n * (n + 1) / 2 > e) --n;
    const int m = (int)(e - (int64_t)n * (n + 1) / 2);
    v = Ep[(int64_t)s * ld + n] * Ep[(int64_t)s * ld + m];
  }
  K[(int64_t)s * ldk + e] = v;
}

// A0 = L (F'F) L' (the common-component Gram C'C), lower triangle mirrored
__global__ void gram_wk_a0_kernel(const double *__restrict__ F, const double *__restrict__ L, int T, int N, int r,
                                  double *__restrict__ A0) {
  __shared__ double FF[32 * 32];
  for (int e = threadIdx.x; e < r * r; e += 256) {
    const int i = e / r, j = e % r;
    double acc = 0.0;
    for (int t = 0; t < T; ++t) acc = fma(F[(int64_t)t * r + i], F[(int64_t)t * r + j], acc);
    FF[e] = acc;
  }
  __syncthreads();
  const int n = blockIdx.x;
  for (int m = threadIdx.x; m <= n; m += 256) {
    double acc = 0.0;
    for (int i = 0; i < r; ++i) {
      double u = 0.0;
      for (int j = 0; j < r; ++j) u = fma(FF[i * r + j], L[(int64_t)m * r + j], u);
      acc = fma(L[(int64_t)n * r + i], u, acc);
    }
    A0[(int64_t)n * N + m] = acc;
    A0[(int64_t)m * N + n] = acc;
  }
}

// Per replicate: w (row rep of W, zero-padded to Tp) and the bucket sums
// Ft[s][j] = sum_{t : idx_t = s} eta_t F[t][j] (At: rows rep*r + j, Tp
// columns, zero-padded), so that B = F' D P E = Ft' E for the whole batch is
// ONE MFMA GEMM At (nb r x T) . E (T x N) — the per-replicate gather of T
// rows of E (a serial 600-step chain per column) is gone.
// idx / eta of the replicate staged in LDS.  w_s = sum of eta_t^2 over the
// t with idx_t = s, ascending t: a counting sort of t by idx_t (bucket
// counts, a block scan, slots handed out by LDS atomics in any order, each
// bucket then insertion-sorted by t), O(T) per replicate — the same sums in
// the same order as a scan over every t (round 3's O(T^2) form, which added
// +0 for the t outside the bucket), so bit-identical to it.
__global__ __launch_bounds__(256) void gram_wk_prep_kernel(int T, int r, const double *__restrict__ F,
                                                           const int32_t *__restrict__ idx,
                                                           const double *__restrict__ eta, int64_t rs, int Tp,
                                                           double *__restrict__ W, double *__restrict__ At) {
  extern __shared__ double pdyn[];
  __shared__ int scan[256];
  double *se = pdyn;                 // eta_t
  double *sF = pdyn + T;             // F (T x r)
  int *sx = (int *)(sF + (int64_t)T * r);   // idx_t
  int *cnt = sx + ((T + 7) & ~7);           // bucket starts, then ends (T + 1)
  int *lst = cnt + ((T + 8) & ~7);          // t by bucket (T)
  const int rep = blockIdx.x, tid = threadIdx.x;
  const int32_t *ix = idx + (int64_t)rep * rs;
  const double *et = eta ? eta + (int64_t)rep * rs : nullptr;
  for (int t = tid; t < T; t += 256) { sx[t] = ix[t]; se[t] = et ? et[t] : 1.0; }
  for (int e = tid; e < T * r; e += 256) sF[e] = F[e];
  for (int s = tid; s <= T; s += 256) cnt[s] = 0;
  __syncthreads();
  for (int t = tid; t < T; t += 256) atomicAdd(&cnt[sx[t] + 1], 1);
  __syncthreads();
  {   // inclusive scan of cnt[0..T]: per-thread chunks, then a 256-wide scan of the chunk sums
    const int per = (T + 1 + 255) / 256, c0 = min(T + 1, tid * per), c1 = min(T + 1, c0 + per);
    int run = 0;
    for (int q = c0; q < c1; ++q) run += cnt[q];
    scan[tid] = run;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const int v = tid >= o ? scan[tid - o] : 0;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    run = scan[tid] - run;
    for (int q = c0; q < c1; ++q) { run += cnt[q]; cnt[q] = run; }   // cnt[s] = start of bucket s
  }
  __syncthreads();
  for (int t = tid; t < T; t += 256) lst[atomicAdd(&cnt[sx[t]], 1)] = t;
  __syncthreads();   // cnt[s] is now the END of bucket s
  double *Wr = W + (int64_t)rep * Tp;
  for (int s = tid; s < Tp; s += 256) {
    double acc = 0.0;
    if (s < T) {
      const int b0 = s ? cnt[s - 1] : 0, b1 = cnt[s];
      for (int i = b0 + 1; i < b1; ++i) {   // insertion sort of the bucket by t (Poisson(1) sized)
        const int v = lst[i];
        int j = i - 1;
        while (j >= b0 && lst[j] > v) { lst[j + 1] = lst[j]; --j; }
        lst[j + 1] = v;
      }
      for (int i = b0; i < b1; ++i) { const double e = se[lst[i]]; acc = __dadd_rn(acc, __dmul_rn(e, e)); }
    }
    Wr[s] = acc;
  }
  __syncthreads();   // every bucket sorted by t
  double *Ar = At + (int64_t)rep * r * Tp;
  for (int e = tid; e < r * Tp; e += 256) {
    const int j = e / Tp, s = e - j * Tp;
    double acc = 0.0;
    if (s < T) {
      const int b0 = s ? cnt[s - 1] : 0, b1 = cnt[s];
      for (int i = b0; i < b1; ++i) { const int t = lst[i]; acc = fma(se[t], sF[t * r + j], acc); }
    }
    Ar[e] = acc;
  }
}

// B = At . E (nb r x N): the 64 x 64 tiles of the batched GEMM left C2's
// 130 columns in 3 column blocks (one holding 2 columns) and 96 tiles with a
// 600-deep serial K loop each — latency-bound on a quarter of the chip
// (61 us per lane).  Here one wave per 32 x 16 output tile (8 x 4
// v_mfma_f64_4x4x4 fragments, operands read straight from L2 into the
// fragments, the next 16-deep chunk's loads issued before this chunk's
// MFMAs) and split-K over WK_BS fixed k-ranges: partial images Bo[z], summed
// in z order where they are read (gram_wk_combine_kernel).
constexpr int WK_BS = 4;
__global__ __launch_bounds__(256) void gram_wk_b_kernel(const double *__restrict__ At, int Tp, const double *__restrict__ Ep,
                                                        int64_t ld, int T, int N, int rows, int nch,
                                                        double *__restrict__ Bo) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nrt = (rows + 31) / 32, nct = (N + 15) / 16;
  const int item = blockIdx.x * 4 + wave;
  if (item >= nrt * nct * WK_BS) return;   // wave-uniform; the kernel has no barriers
  const int z = item % WK_BS, tile = item / WK_BS;
  const int ct = tile % nct, rt = tile / nct, rbase = rt * 32, cbase = ct * 16;
  const int c0 = z * nch, c1 = min(c0 + nch, Tp / 16);   // this split's 16-deep chunks
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const double *pa[8];
  int col[4];
#pragma unroll
  for (int f = 0; f < 8; ++f) pa[f] = At + (int64_t)min(rbase + 4 * f + fi, rows - 1) * Tp + fkc;   // past rows: discarded
#pragma unroll
  for (int q = 0; q < 4; ++q) col[q] = min(cbase + 4 * q + fi, N - 1);                         // past N: discarded
  double acc[8][4];
#pragma unroll
  for (int f = 0; f < 8; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[f][q] = 0.0;
  // At's columns T..Tp-1 are zero: the k tail reads E's last row (finite)
  auto load = [&](int c, double (&af)[8], double (&bf)[4]) {
    const int k = 16 * c;
    const double *eb = Ep + (int64_t)min(k + fkc, T - 1) * ld;
#pragma unroll
    for (int f = 0; f < 8; ++f) af[f] = pa[f][k];
#pragma unroll
    for (int q = 0; q < 4; ++q) bf[q] = eb[col[q]];
  };
  double af[8], bf[4];
  if (c0 < c1) load(c0, af, bf);
  for (int c = c0; c < c1; ++c) {
    double an[8], bn[4];
    if (c + 1 < c1) load(c + 1, an, bn);
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[f][q] = mfma4(af[f], bf[q], acc[f][q]);
#pragma unroll
    for (int f = 0; f < 8; ++f) af[f] = an[f];
#pragma unroll
    for (int q = 0; q < 4; ++q) bf[q] = bn[q];
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
  double *Bz = Bo + (int64_t)z * rows * N;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa) {
    const double a0 = acc[fa][0], a1 = acc[fa][1], a2 = acc[fa][2], a3 = acc[fa][3];
    const double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
    const double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
    const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
    const int row = rbase + 4 * fa + oi, cc = cbase + 4 * blk + oj;
    if (row < rows && cc < N) Bz[(int64_t)row * N + cc] = v;
  }
}

// G[rep] (N x N, row-major, stride N*N) = A0 + L B + (L B)' + unpack(Q[rep]),
// one workgroup per (lower 32 x 32 tile (I, J), replicate): the L rows and B
// columns of blocks I and J staged in LDS first (every entry's two r-term
// dot products then read LDS broadcasts instead of 4 r global loads), the
// tile computed once (rows n of block I read their contiguous packed Q
// ranges), staged in LDS, and written as tile (I, J) and, transposed,
// (J, I) — both coalesced, G exactly symmetric.  Same operations in the same
// order as before (x, y as r-term fma chains, then A0 + (x + y) + Q).
#ifndef DFM_WK_TILE   // (A/B builds: combine tile edge)
#define DFM_WK_TILE 32
#endif
constexpr int WK_TILE = DFM_WK_TILE, WK_RMAX = 16;
__global__ __launch_bounds__(256) void gram_wk_combine_kernel(const double *__restrict__ A0,
                                                              const double *__restrict__ L,
                                                              const double *__restrict__ Bo,
                                                              const double *__restrict__ Q, int64_t ldk, int N, int r,
                                                              int64_t bstride, double *__restrict__ G) {
  __shared__ double tile[WK_TILE][WK_TILE + 1];
  __shared__ double sLI[WK_TILE][WK_RMAX + 1], sLJ[WK_TILE][WK_RMAX + 1];   // L rows of blocks I, J
  __shared__ double sBI[WK_RMAX][WK_TILE + 1], sBJ[WK_RMAX][WK_TILE + 1];   // B columns of blocks I, J
  const int rep = blockIdx.y, tid = threadIdx.x;
  int I = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= (int)blockIdx.x) ++I;
  while (I * (I + 1) / 2 > (int)blockIdx.x) --I;
  const int J = blockIdx.x - I * (I + 1) / 2;
  const double *Br = Bo + (int64_t)rep * r * N;
  const double *Qr = Q + (int64_t)rep * ldk;
  double *Gr = G + (int64_t)rep * N * N;
  // this thread's A0 and Q entries, loaded before the staging below (their
  // latency overlaps it instead of following the barrier)
  constexpr int EPT = WK_TILE * WK_TILE / 256;
  double a0v[EPT], qv[EPT];
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = tid + 256 * u, a = e / WK_TILE, b = e % WK_TILE, n = I * WK_TILE + a, m = J * WK_TILE + b;
    const bool in = n < N && m <= n;
    a0v[u] = in ? A0[(int64_t)n * N + m] : 0.0;
    qv[u] = in ? Qr[(int64_t)n * (n + 1) / 2 + m] : 0.0;
  }
  for (int e = tid; e < WK_TILE * r; e += 256) {
    const int a = e / r, j = e % r, nI = I * WK_TILE + a, nJ = J * WK_TILE + a;
    sLI[a][j] = nI < N ? L[(int64_t)nI * r + j] : 0.0;
    sLJ[a][j] = nJ < N ? L[(int64_t)nJ * r + j] : 0.0;
  }
  for (int e = tid; e < WK_TILE * r; e += 256) {
    const int j = e / WK_TILE, a = e % WK_TILE, nI = I * WK_TILE + a, nJ = J * WK_TILE + a;
    double bi = 0.0, bj = 0.0;   // the split-K partial images, in z order
#pragma unroll
    for (int z = 0; z < WK_BS; ++z) {
      if (nI < N) bi += Br[z * bstride + (int64_t)j * N + nI];
      if (nJ < N) bj += Br[z * bstride + (int64_t)j * N + nJ];
    }
    sBI[j][a] = bi;
    sBJ[j][a] = bj;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < EPT; ++u) {
    const int e = tid + 256 * u, a = e / WK_TILE, b = e % WK_TILE, n = I * WK_TILE + a, m = J * WK_TILE + b;
    double v = 0.0;
    if (n < N && m <= n) {
      double x = 0.0, y = 0.0;   // x: L[n] . B[:, m],  y: L[m] . B[:, n]
      for (int j = 0; j < r; ++j) {
        x = fma(sLI[a][j], sBJ[j][b], x);
        y = fma(sLJ[b][j], sBI[j][a], y);
      }
      v = (a0v[u] + (x + y)) + qv[u];
    }
    tile[a][b] = v;
  }
  __syncthreads();
  for (int e = tid; e < WK_TILE * WK_TILE; e += 256) {
    const int a = e / WK_TILE, b = e % WK_TILE;
    const int n = I * WK_TILE + a, m = J * WK_TILE + b;
    if (n < N && m <= n) Gr[(int64_t)n * N + m] = tile[a][b];
    const int n2 = J * WK_TILE + a, m2 = I * WK_TILE + b;   // transposed tile (J, I): entry (n2, m2) = (m2, n2)
    if (m2 < N && n2 < m2) Gr[(int64_t)n2 * N + m2] = tile[b][a];
  }
}

hipError_t launch_gemm(bool a_trans, const double *A, int64_t lda, const double *B, int64_t ldb,
                       double *C, int64_t ldc, int M, int Nc, int K, hipStream_t st,
                       const int *col_done, int col_group, bool b_padded, const int *clist, const int *ccount);

// gram_wk_prep_kernel's dynamic LDS: se (T), sF (T x r), sx (round_up(T, 8) ints), the
// bucket bounds (round_up(T + 1, 8) ints) and the bucketed t (T ints)
size_t gram_wk_prep_lds(int T, int r) {
  const size_t T8 = (size_t)((T + 7) & ~7), T18 = (size_t)((T + 8) & ~7);
  return (size_t)T * 8 + (size_t)T * r * 8 + T8 * 4 + T18 * 4 + (size_t)T * 4;
}
int64_t gram_wk_ldk(int N) { return ((int64_t)N * (N + 1) / 2 + 1) / 2 * 2; }
int gram_wk_tp(int T) { return (T + 15) / 16 * 16; }
// model-level: K (Tp x ldk) and A0 (N x N)
hipError_t gram_wk_precompute(const double *Ep, int64_t ld, int T, int N, int r, const double *F, const double *L,
                              double *K, double *A0, hipStream_t st) {
  const int64_t ldk = gram_wk_ldk(N);
  hipLaunchKernelGGL(gram_wk_kmat_kernel, dim3((unsigned)((ldk + 255) / 256), gram_wk_tp(T)), dim3(256), 0, st, Ep,
                     ld, T, N, ldk, K);
  hipLaunchKernelGGL(gram_wk_a0_kernel, dim3(N), dim3(256), 0, st, F, L, T, N, r, A0);
  return hipGetLastError();
}
// workspace doubles for nb replicates: W (nb x Tp), B (WK_BS x nb x r x N), Q (nb x ldk), At (nb x r x Tp)
size_t gram_wk_work(int T, int N, int r, int nb) {
  return (size_t)nb * ((size_t)gram_wk_tp(T) + (size_t)WK_BS * r * N + (size_t)gram_wk_ldk(N) + (size_t)r * gram_wk_tp(T));
}
// the At region (nb r Tp >= nb T r doubles): free once the batch's Grams are
// formed — the factored F* pass (dfm_model.hip fact_el_kernel) writes E L* there
double *gram_wk_scratch(double *work, int T, int N, int r, int nb) {
  return work + (size_t)nb * ((size_t)gram_wk_tp(T) + (size_t)WK_BS * r * N + (size_t)gram_wk_ldk(N));
}
// nb replicate Grams X*'X* (N x N each, stride N*N) of src (C + diag(eta) E[idx]).
hipError_t launch_gram_wk(const double *Ep, int64_t ld, int T, int N, int r, const double *F, const double *L,
                          const double *K, const double *A0, const int32_t *idx, const double *eta, int64_t rs,
                          int nb, double *work, double *G, hipStream_t st) {
  const int Tp = gram_wk_tp(T);
  const int64_t ldk = gram_wk_ldk(N);
  double *W = work, *Bo = W + (size_t)nb * Tp, *Q = Bo + (size_t)WK_BS * nb * r * N, *At = Q + (size_t)nb * ldk;
  hipLaunchKernelGGL(gram_wk_prep_kernel, dim3(nb), dim3(256), gram_wk_prep_lds(T, r), st, T, r, F, idx, eta, rs, Tp,
                     W, At);
  // B (nb r x N) = At . E, then Q (nb x ldk) = W K
  {
    const int rows = nb * r, nch = (Tp / 16 + WK_BS - 1) / WK_BS;
    const int64_t items = (int64_t)((rows + 31) / 32) * ((N + 15) / 16) * WK_BS;
    hipLaunchKernelGGL(gram_wk_b_kernel, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, st, At, Tp, Ep, ld, T, N,
                       rows, nch, Bo);
  }
  hipError_t e = launch_gemm(false, W, Tp, K, ldk, Q, ldk, nb, (int)ldk, T, st, nullptr, 1, true, nullptr, nullptr);
  if (e != hipSuccess) return e;
  const int nt = (N + WK_TILE - 1) / WK_TILE;
  hipLaunchKernelGGL(gram_wk_combine_kernel, dim3(nt * (nt + 1) / 2, nb), dim3(256), 0, st, A0, L, Bo, Q, ldk, N, r,
                     (int64_t)nb * r * N, G);
  return hipGetLastError();
}

}  // namespace dfm
