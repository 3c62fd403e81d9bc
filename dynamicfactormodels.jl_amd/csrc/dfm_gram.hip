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
                                       int64_t elems, double *__restrict__ G, int64_t strideG) {
  const int r = blockIdx.y;
  const double *w = W + (int64_t)r * S * elems;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < elems; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / ldg, j = e - i * ldg;
    if (j >= m) continue;
    double a = 0.0;
    for (int z = 0; z < S; ++z) a += w[(int64_t)z * elems + e];
    G[(int64_t)r * strideG + i * ldg + j] = a;
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
                           int64_t strideZ, hipStream_t st);
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

// Dispatch.  Returns hipError of the launch.
hipError_t launch_gram(int orient, const PanelSrc &src, int m, int K, int T, double *G,
                       int64_t ldg, int64_t strideG, int nrep, hipStream_t st) {
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
    hipError_t e = hipMallocAsync((void **)&W, (size_t)nrc * S * elems * 8, st);
    if (e != hipSuccess) return e;
    Gk = W; sZ = elems; sG = elems * S;
  }
  const bool c = src.C != nullptr, e = src.eta != nullptr, x = src.idx != nullptr;
  // a plain row-major panel (no fused gather): LDS-DMA SYRK (dfm_gemm.hip).
  // The k-split counts 16-deep steps of both kernels alike, so the partial
  // sums (and the result bits) do not depend on which kernel ran.
  if (plain) {
    hipError_t er = launch_gram_dma(src.E, src.ld, m, K, S, ksteps, Gk, ldg, sZ, st);
    if (er == hipSuccess && S > 1)
      hipLaunchKernelGGL(gram_splitk_sum_kernel, dim3((unsigned)std::min<int64_t>((elems + 255) / 256, 4096), 1),
                         dim3(256), 0, st, W, S, m, ldg, elems, G, strideG);
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
                       dim3(256), 0, st, W, S, m, ldg, elems, G + (int64_t)r0 * strideG, strideG);
  }
  }
  if (W) hipFreeAsync(W, st);
  return hipGetLastError();
}

}  // namespace dfm
