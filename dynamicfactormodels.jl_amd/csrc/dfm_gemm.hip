// dfm_gemm.hip — batched-replicate fp64 GEMM on MFMA (v_mfma_f64_4x4x4_4b).
//
//   C[M x Nc] = op(A) B,  op(A) = A (M x K row-major)  or  A^T (A stored K x M)
//   B: K x Nc row-major (the k-rows of every replicate's skinny operand laid
//   side by side: column block = one replicate's p columns).
//
// This is the compute core of the factored bootstrap (dfm_eig.hip): one
// fixed, cache-resident left operand (H = E E' or E') shared by every
// replicate of a batch, so the per-replicate eigen-iterations and the
// loadings pass become single large MFMA GEMMs instead of nb memory-bound
// skinny products.  Tiling, fragment maps and the swizzled LDS images are
// those of the Gram kernel (dfm_gram.hip); grid order is XCD-aware: the row
// blocks of one column block are issued to one XCD so a B tile is fetched
// from HBM once and re-read from that XCD's L2.
#include "dfm_common.h"
#include <cstdlib>

namespace dfm {

namespace {
// 32-deep stages: two MFMA k-steps (128 MFMA per wave) between barriers.
// [a][k] image: 256-B rows, k XOR-swizzled by 8*(a&3) -> the 4x4x4 A/B
// fragment reads (lanes: 4 rows x 8 k per half-wave) hit 32 distinct bank
// pairs, and the 16-B staging writes stay conflict-free.
// [k][a] image: 512-B rows, a XOR-swizzled by 4*(k&7) (as in dfm_gram.hip).
constexpr int GT = 64, KS = 32;
DFM_DEV int off_rows(int a, int kc) { return a * KS + (kc ^ ((a & 3) << 3)); }  // [a][k]
DFM_DEV int off_cols(int a, int kc) { return kc * GT + (a ^ ((kc & 7) << 2)); }  // [k][a]
}  // namespace

// Ring/occupancy choice of the LDS-DMA kernels by output height: rows >= 1024
// run the 3-deep ring at 3 workgroups per CU (more resident waves beat a
// deeper ring there: tools/gemm_bench.hip, M = 2000).
static bool gemm_ring3(int M) { return M >= 1024; }

// One stage of staging registers (4 A chunks + 4 B chunks of 16 B per
// thread) kept as a plain struct of scalars: no lambdas capturing arrays by
// reference and no conditional loads, both of which make the compiler route
// the staging through scratch and wait on every load.
struct Stage {
  double2 a0, a1, a2, a3, b0, b1, b2, b3;
  unsigned ok;
};

template <bool A_TRANS>
DFM_DEV void stage_offsets(int h, int tid, int k0, int abase, int bbase, int M, int Nc, int K, int64_t lda,
                           int64_t ldb, int64_t &offa, int64_t &offb, unsigned &ok) {
  bool oka;
  if constexpr (!A_TRANS) {   // A rows: chunk -> (row a = tid>>4 + 16h, k pair 2*(tid&15))
    const int a = abase + (tid >> 4) + 16 * h, k = k0 + 2 * (tid & 15);
    oka = (a < M) && (k < K);
    offa = oka ? (int64_t)a * lda + k : 0;
  } else {                    // A^T: k-rows of A (contiguous in a)
    const int kc = k0 + (tid >> 5) + 8 * h, a = abase + 2 * (tid & 31);
    oka = (kc < K) && (a < M);
    offa = oka ? (int64_t)kc * lda + a : 0;
  }
  const int kb = k0 + (tid >> 5) + 8 * h, col = bbase + 2 * (tid & 31);
  const bool okb = (kb < K) && (col < Nc);
  offb = okb ? (int64_t)kb * ldb + col : 0;
  ok |= ((oka ? 1u : 0u) << h) | ((okb ? 16u : 0u) << h);
}

template <bool A_TRANS>
DFM_DEV void load_stage(Stage &sg, const double *__restrict__ A, const double *__restrict__ B, int tid,
                        int k0, int abase, int bbase, int M, int Nc, int K, int64_t lda, int64_t ldb) {
  int64_t oa0, oa1, oa2, oa3, ob0, ob1, ob2, ob3;
  unsigned ok = 0;
  stage_offsets<A_TRANS>(0, tid, k0, abase, bbase, M, Nc, K, lda, ldb, oa0, ob0, ok);
  stage_offsets<A_TRANS>(1, tid, k0, abase, bbase, M, Nc, K, lda, ldb, oa1, ob1, ok);
  stage_offsets<A_TRANS>(2, tid, k0, abase, bbase, M, Nc, K, lda, ldb, oa2, ob2, ok);
  stage_offsets<A_TRANS>(3, tid, k0, abase, bbase, M, Nc, K, lda, ldb, oa3, ob3, ok);
  sg.a0 = *reinterpret_cast<const double2 *>(A + oa0);
  sg.a1 = *reinterpret_cast<const double2 *>(A + oa1);
  sg.a2 = *reinterpret_cast<const double2 *>(A + oa2);
  sg.a3 = *reinterpret_cast<const double2 *>(A + oa3);
  sg.b0 = *reinterpret_cast<const double2 *>(B + ob0);
  sg.b1 = *reinterpret_cast<const double2 *>(B + ob1);
  sg.b2 = *reinterpret_cast<const double2 *>(B + ob2);
  sg.b3 = *reinterpret_cast<const double2 *>(B + ob3);
  sg.ok = ok;
}

template <bool A_TRANS>
DFM_DEV void store_one(double *la, double *lb, int h, int tid, const double2 &va, const double2 &vb,
                       unsigned ok) {
  // component-wise selects: a select of whole double2 values is lowered
  // through a dynamically indexed stack slot (scratch)
  int oa;
  if constexpr (!A_TRANS) oa = off_rows((tid >> 4) + 16 * h, 2 * (tid & 15));
  else oa = off_cols(2 * (tid & 31), (tid >> 5) + 8 * h);
  const bool ka = (ok >> h) & 1u, kb = (ok >> (4 + h)) & 1u;
  double2 wa, wb;
  wa.x = ka ? va.x : 0.0;
  wa.y = ka ? va.y : 0.0;
  wb.x = kb ? vb.x : 0.0;
  wb.y = kb ? vb.y : 0.0;
  *reinterpret_cast<double2 *>(la + oa) = wa;
  *reinterpret_cast<double2 *>(lb + off_cols(2 * (tid & 31), (tid >> 5) + 8 * h)) = wb;
}

template <bool A_TRANS>
DFM_DEV void store_stage(const Stage &sg, double *la, double *lb, int tid) {
  store_one<A_TRANS>(la, lb, 0, tid, sg.a0, sg.b0, sg.ok);
  store_one<A_TRANS>(la, lb, 1, tid, sg.a1, sg.b1, sg.ok);
  store_one<A_TRANS>(la, lb, 2, tid, sg.a2, sg.b2, sg.ok);
  store_one<A_TRANS>(la, lb, 3, tid, sg.a3, sg.b3, sg.ok);
}

template <bool A_TRANS>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const double *__restrict__ A, int64_t lda,
                                                      const double *__restrict__ B, int64_t ldb,
                                                      double *__restrict__ C, int64_t ldc, int M,
                                                      int Nc, int K, int nrb, int ncb,
                                                      const int *__restrict__ col_done, int col_group) {
  __shared__ __attribute__((aligned(16))) double lds[2][2][GT * KS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  // XCD-aware mapping: blocks b and b+8 share an XCD (round-robin dispatch)
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int rb = j % nrb, cb = (j / nrb) * 8 + xcd;
  if (cb >= ncb) return;
  const int abase = rb * GT, bbase = cb * GT;
  if (col_done) {   // skip column blocks whose replicates have all converged
    bool all = true;
    const int r0 = bbase / col_group, r1 = min(Nc - 1, bbase + GT - 1) / col_group;
    for (int q = r0; q <= r1; ++q) all = all && col_done[q];
    if (all) return;
  }

  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0.0;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int nst = (K + KS - 1) / KS;
  Stage sg;
  load_stage<A_TRANS>(sg, A, B, tid, 0, abase, bbase, M, Nc, K, lda, ldb);
  store_stage<A_TRANS>(sg, lds[0][0], lds[0][1], tid);
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) load_stage<A_TRANS>(sg, A, B, tid, (s + 1) * KS, abase, bbase, M, Nc, K, lda, ldb);
#pragma unroll
    for (int sub = 0; sub < KS / 16; ++sub) {
      const int kc = 16 * sub + fkc;
      double af[8], bf[8];
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        const int a = wr * 32 + 4 * f + fi;
        af[f] = A_TRANS ? lds[buf][0][off_cols(a, kc)] : lds[buf][0][off_rows(a, kc)];
        bf[f] = lds[buf][1][off_cols(wc * 32 + 4 * f + fi, kc)];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
    }
    if (s + 1 < nst) store_stage<A_TRANS>(sg, lds[buf ^ 1][0], lds[buf ^ 1][1], tid);
    __syncthreads();
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int row = abase + wr * 32 + 4 * fa + oi;
      const int col = bbase + wc * 32 + 16 * q + 4 * blk + oj;
      if (row < M && col < Nc) C[(int64_t)row * ldc + col] = v;
    }
}

// ---------------------------------------------------------------------------
// gemmh_kernel: C = A B for the eigen-iteration product H.Z, staged by LDS-DMA
// (global_load_lds_dwordx4: no VGPR staging, no ds_write pass) through a
// 4-deep ring of 16-deep stages, two stages in flight across each barrier:
// every wave waits only for its own DMAs of the stage about to be read
// (counted vmcnt, never 0 inside the loop), then ONE raw s_barrier orders
// them for every reader and retires the ring slot being refilled (read one
// iteration earlier).  All LDS is one __shared__ array (a second object makes
// hipcc drain vmcnt before ds_reads).  LDS images as dfm_gram.hip's 16-deep
// ones; DMA writes are lane-linear, so the XOR swizzle is applied to the
// per-lane SOURCE address.  Out-of-range rows/columns read clamped (finite)
// data that only reaches discarded outputs; the k tail reads A's zero
// padding (requirement: lda >= round_up(K, 16), A[i][K..lda) = 0).
namespace {
constexpr int G2_KS = 16, G2_STAGE = 2 * GT * G2_KS;   // doubles per stage (A + B)
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
DFM_DEV int g2_offA(int a, int kc) { return a * G2_KS + (kc ^ (((a >> 1) & 1) << 3)); }   // [a][k]
DFM_DEV int g2_offB(int kc, int a) { return kc * GT + (a ^ ((kc & 7) << 2)); }           // [k][a]
}  // namespace

// Per-lane DMA sources, fixed for the whole K loop: A chunk rows 8c..8c+7
// (lane pair lane & 7), B chunk k-rows 2c, 2c+1 (lane pair lane & 31), with
// the LDS images' XOR swizzle applied to the source column.
struct G2Src {
  int64_t a[2], b[2];   // element offsets at k0 = 0
  int kb[2];            // B k-row within the stage
};
// clist (optional): column compaction by indirection — compact column x of
// B / C is physical column clist[x / cg] * cg + x % cg (x / cg < ccount);
// pairs (x, x+1) never straddle a group (x even, cg even).
DFM_DEV int64_t g2_phys_col(int x, const int *__restrict__ clist, int ccount, int cg) {
  const int slot = min(x / cg, ccount - 1);   // past the list: finite data, discarded outputs
  return (int64_t)clist[slot] * cg + (x - (x / cg) * cg);
}
DFM_DEV G2Src g2_sources(int64_t lda, int64_t ldb, int abase, int bbase, int M, int Nc, int wave, int lane,
                         const int *__restrict__ clist = nullptr, int ccount = 0, int cg = 1) {
  G2Src s;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 2 * wave + h;
    const int a = 8 * c + (lane >> 3);
    const int ka = (2 * (lane & 7)) ^ (((a >> 1) & 1) << 3);
    s.a[h] = (int64_t)min(abase + a, M - 1) * lda + ka;
    const int kc = 2 * c + (lane >> 5);
    s.kb[h] = kc;
    const int x = bbase + ((2 * (lane & 31)) ^ ((kc & 7) << 2));
    s.b[h] = (int64_t)kc * ldb + (clist ? g2_phys_col(x, clist, ccount, cg) : (int64_t)min(x, Nc - 2));
  }
  return s;
}
DFM_DEV void g2_issue(double *stage, const double *__restrict__ A, const double *__restrict__ B, int64_t ldb,
                      const G2Src &src, int k0, int K) {
  double *la = stage, *lb = stage + GT * G2_KS;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c_off = (2 * (threadIdx.x >> 6) + h) * 128;
    __builtin_amdgcn_global_load_lds((gbl_void_t *)(A + src.a[h] + k0), (lds_void_t *)(la + c_off), 16, 0, 0);
    // k rows past K (last stage only) re-read row K-1: finite, multiplied by A's zero k-padding
    const int64_t over = (int64_t)max(0, k0 + src.kb[h] - (K - 1)) * ldb;
    __builtin_amdgcn_global_load_lds((gbl_void_t *)(B + src.b[h] + (int64_t)k0 * ldb - over),
                                     (lds_void_t *)(lb + c_off), 16, 0, 0);
  }
}

template <int NBUF, int MINB, bool RUN = false>
__global__ __launch_bounds__(256, MINB) void gemmh_kernel_t(const double *__restrict__ A, int64_t lda,
                                                       const double *__restrict__ B, int64_t ldb,
                                                       double *__restrict__ C, int64_t ldc, int M, int Nc, int K,
                                                       int nrb, int ncb, const int *__restrict__ col_done,
                                                       int col_group, const int *__restrict__ clist = nullptr,
                                                       const int *__restrict__ ccount_p = nullptr) {
  __shared__ __attribute__((aligned(16))) double lds[NBUF * G2_STAGE];
  constexpr int AHEAD = NBUF - 2;   // stages in flight across a barrier
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int rb = j % nrb, cb = (j / nrb) * 8 + xcd;
  if (cb >= ncb) return;
  const int abase = rb * GT, bbase = cb * GT;
  // compacted launch (straggler phase): column block cb of the listed
  // replicates' column groups only.  The list is rebuilt on the device after
  // every convergence check; compaction applies once it holds < 1/8 of the
  // batch (Nc / col_group replicates), decided here from its device-side
  // count, so the host never waits for it.  Either way a column's sum runs in
  // the same order: the bits do not depend on the mode.
  const int ccount = clist ? *ccount_p : 0;
  const bool compact = clist && (int64_t)ccount * 8 < Nc / col_group;
  clist = compact ? clist : nullptr;
  if (compact) {
    if (bbase >= ccount * col_group) return;
    if (col_done) {   // every listed replicate of the block retired since the list was built
      bool all = true;
      const int s0 = bbase / col_group, s1 = min(ccount - 1, (bbase + GT - 1) / col_group);
      for (int q = s0; q <= s1; ++q) all = all && col_done[clist[q]];
      if (all) return;
    }
  } else if (col_done) {
    bool all = true;
    const int r0 = bbase / col_group, r1 = min(Nc - 1, bbase + GT - 1) / col_group;
    for (int q = r0; q <= r1; ++q) all = all && col_done[q];
    if (all) return;
  }
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0.0;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int nst = (K + G2_KS - 1) / G2_KS;
  const G2Src src = g2_sources(lda, ldb, abase, bbase, M, Nc, wave, lane, clist, ccount, col_group);
  // RUN: the DMA sources are running pointers advanced by one stage per
  // issue (no per-stage 64-bit address arithmetic, no k-tail clamp: B holds
  // zero rows up to round_up(K, 16), as A holds zero k-columns)
  const double *pa0 = A + src.a[0], *pa1 = A + src.a[1], *pb0 = B + src.b[0], *pb1 = B + src.b[1];
  const int64_t bstep = (int64_t)G2_KS * ldb;
  auto issue = [&](int s) {
    double *stage = lds + (s % NBUF) * G2_STAGE;
    if (RUN) {
      double *la = stage, *lb = stage + GT * G2_KS;
      const int c0 = (2 * wave) * 128, c1 = c0 + 128;
#if defined(DFM_GEMM_DIAG_AONLY)   // (timing diagnostic, WRONG results: B tiles not re-staged after the first stages)
      const bool fb = s < NBUF;
#else
      const bool fb = true;
#endif
#if defined(DFM_GEMM_DIAG_BONLY)   // (timing diagnostic, WRONG results: A tiles not re-staged after the first stages)
      const bool fa = s < NBUF;
#else
      const bool fa = true;
#endif
      if (fa) __builtin_amdgcn_global_load_lds((gbl_void_t *)pa0, (lds_void_t *)(la + c0), 16, 0, 0);
      if (fb) __builtin_amdgcn_global_load_lds((gbl_void_t *)pb0, (lds_void_t *)(lb + c0), 16, 0, 0);
      if (fa) __builtin_amdgcn_global_load_lds((gbl_void_t *)pa1, (lds_void_t *)(la + c1), 16, 0, 0);
      if (fb) __builtin_amdgcn_global_load_lds((gbl_void_t *)pb1, (lds_void_t *)(lb + c1), 16, 0, 0);
      pa0 += G2_KS; pa1 += G2_KS; pb0 += bstep; pb1 += bstep;
    } else {
      g2_issue(stage, A, B, ldb, src, s * G2_KS, K);
    }
  };
  for (int s = 0; s < NBUF - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    const int ahead = min(AHEAD, nst - 1 - s);   // later stages already issued (4 DMAs each per wave)
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NBUF - 1 < nst) issue(s + NBUF - 1);   // ring slot (s-1)%NBUF: its readers all passed this barrier
    const double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    double af[8], bf[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = la[g2_offA(wr * 32 + 4 * f + fi, fkc)];
      bf[f] = lb[g2_offB(fkc, wc * 32 + 4 * f + fi)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
#if defined(DFM_GEMM_SC1)
  // A/B: HZ leaves through write-through (sc1) 16-B stores, which drop the
  // line from this XCD's L2 (MI355X_MICROARCH.md, store flavours) — the
  // 360 MB output stream then no longer evicts the L2-resident H (2 MB) that
  // every workgroup re-reads.  Lane pairs (oj, oj ^ 1) combine two adjacent
  // columns; the even lane stores both.
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(C, 0, (int)((int64_t)M * ldc * 8), 0x00020000);
#endif
#pragma unroll
  for (int fa = 0; fa < 8; ++fa)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int row = abase + wr * 32 + 4 * fa + oi;
      const int col = bbase + wc * 32 + 16 * q + 4 * blk + oj;
#if defined(DFM_GEMM_SC1)
      if (RUN) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const double vn = __shfl_xor(v, 1);
        const bool ok = row < M && (clist ? col < ccount * col_group : col < Nc);
        if (!(oj & 1) && ok) {
          const int64_t pc = clist ? g2_phys_col(col, clist, ccount, col_group) : (int64_t)col;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, double2{v, vn}), crs,
                                                 (int)(((int64_t)row * ldc + pc) * 8), 0, 16);
        }
        continue;
      }
#endif
      if (clist) {
        if (row < M && col < ccount * col_group) C[(int64_t)row * ldc + g2_phys_col(col, clist, ccount, col_group)] = v;
      } else if (row < M && col < Nc) {
        C[(int64_t)row * ldc + col] = v;
      }
    }
}

// the production configuration
#define gemmh_kernel gemmh_kernel_t<4, 2>

// ---------------------------------------------------------------------------
// gemmh_zrm_kernel: the factored solver's H.Z with Z replicate-major (round 6).
// Z holds replicate rep's T x pz block as 16-row chunks, each chunk column-
// major: element (s, c) at rep zrs + (s >> 4) 16 pz + 16 c + (s & 15)
// (zrs = round_up(T, 16) pz, the chunk rows past T zero).  A 16-deep k stage
// of one B column is then ONE 128-B line, so the B operand is staged like A
// (and like gram_dma_kernel's second operand): an [a][k] LDS image, 8 columns
// per DMA instruction, each column's 16 k values one line — a 64-column tile
// spanning 5.33 replicates reads whole lines, where the column-interleaved
// T x nb pz layout read one 512-B k-row segment and a replicate-major
// [rep][T][pz] layout six 96-B pieces per k-row (round 5: +5.6 % GEMM).
// The passes that write Z (zscatter_tail, boot_cheb_mid_kernel) then write
// each replicate's 16-row tile as one contiguous 16 pz x 8-B chunk.  The
// fragments hold the same elements as gemmh_kernel_t's, so HZ is
// bit-identical; C (HZ) keeps the column-interleaved layout (its rows are
// gathered by idx).  A = H as gemmh_kernel_t<3, 3, true> (lda >= round_up(K,
// 16), zero k-padding); 3-deep ring at 3 workgroups per CU; column
// compaction by clist as gemmh_kernel_t.
__global__ __launch_bounds__(256, 3) void gemmh_zrm_kernel(const double *__restrict__ A, int64_t lda,
                                                          const double *__restrict__ Z, int pz, int64_t zrs,
                                                          double *__restrict__ C, int64_t ldc, int M, int Nc, int K,
                                                          int nrb, int ncb, const int *__restrict__ col_done,
                                                          const int *__restrict__ clist, const int *__restrict__ ccount_p) {
  constexpr int NBUF = 3;
  __shared__ __attribute__((aligned(16))) double lds[NBUF * G2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int rb = j % nrb, cb = (j / nrb) * 8 + xcd;
  if (cb >= ncb) return;
  const int abase = rb * GT, bbase = cb * GT, col_group = pz;
  const int ccount = clist ? *ccount_p : 0;
  const bool compact = clist && (int64_t)ccount * 8 < Nc / col_group;
  clist = compact ? clist : nullptr;
  if (compact) {
    if (bbase >= ccount * col_group) return;
    if (col_done) {
      bool all = true;
      const int s0 = bbase / col_group, s1 = min(ccount - 1, (bbase + GT - 1) / col_group);
      for (int q = s0; q <= s1; ++q) all = all && col_done[clist[q]];
      if (all) return;
    }
  } else if (col_done) {
    bool all = true;
    const int r0 = bbase / col_group, r1 = min(Nc - 1, bbase + GT - 1) / col_group;
    for (int q = r0; q <= r1; ++q) all = all && col_done[q];
    if (all) return;
  }
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0.0;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int nst = (K + G2_KS - 1) / G2_KS;
  // per-lane DMA sources: rows a of the A block and columns a of the B block,
  // 16 k per row in 8 lane pairs (the [a][k] images' XOR swizzle on the source k)
  const double *pa[2], *pb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 2 * wave + h;
    const int a = 8 * c + (lane >> 3);
    const int ka = (2 * (lane & 7)) ^ (((a >> 1) & 1) << 3);
    pa[h] = A + (int64_t)min(abase + a, M - 1) * lda + ka;
    const int x = bbase + a;
    int rep, cc;
    if (clist) {   // compact column x: replicate clist[x / pz] (past the list: finite, discarded)
      const int slot = min(x / pz, ccount - 1);
      rep = clist[slot];
      cc = x - (x / pz) * pz;
    } else {
      const int xc = min(x, Nc - 1);   // past Nc: finite data, discarded outputs
      rep = xc / pz;
      cc = xc - rep * pz;
    }
    pb[h] = Z + (int64_t)rep * zrs + 16 * cc + ka;
  }
  const int64_t bstep = (int64_t)G2_KS * pz;
  const int c0 = (2 * wave) * 128, c1 = c0 + 128;
  auto issue = [&](int s) {
    double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pa[0], (lds_void_t *)(la + c0), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pb[0], (lds_void_t *)(lb + c0), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pa[1], (lds_void_t *)(la + c1), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pb[1], (lds_void_t *)(lb + c1), 16, 0, 0);
    pa[0] += G2_KS; pa[1] += G2_KS; pb[0] += bstep; pb[1] += bstep;
  };
  for (int s = 0; s < NBUF - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    const int ahead = min(NBUF - 2, nst - 1 - s);
    if (ahead >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NBUF - 1 < nst) issue(s + NBUF - 1);
    const double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    double af[8], bf[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = la[g2_offA(wr * 32 + 4 * f + fi, fkc)];
      bf[f] = lb[g2_offA(wc * 32 + 4 * f + fi, fkc)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int row = abase + wr * 32 + 4 * fa + oi;
      const int col = bbase + wc * 32 + 16 * q + 4 * blk + oj;
      if (clist) {
        if (row < M && col < ccount * col_group) C[(int64_t)row * ldc + g2_phys_col(col, clist, ccount, col_group)] = v;
      } else if (row < M && col < Nc) {
        C[(int64_t)row * ldc + col] = v;
      }
    }
}

// H (M x K, lda >= round_up(K, 16), zero k-padding) times the replicate-major
// chunked Z of nb = Nc / pz replicates (gemmh_zrm_kernel) -> C (M x Nc, ldc)
hipError_t launch_gemm_zrm(const double *A, int64_t lda, const double *Z, int pz, int64_t zrs, double *C,
                           int64_t ldc, int M, int Nc, int K, hipStream_t st, const int *col_done, const int *clist,
                           const int *ccount) {
  if (lda < (K + G2_KS - 1) / G2_KS * G2_KS || pz < 2 || (pz & 1) || Nc % pz) return hipErrorInvalidValue;
  const int nrb = (M + GT - 1) / GT, ncb = (Nc + GT - 1) / GT;
  const int ncb8 = (ncb + 7) / 8 * 8;
  hipLaunchKernelGGL(gemmh_zrm_kernel, dim3(nrb * ncb8), dim3(256), 0, st, A, lda, Z, pz, zrs, C, ldc, M, Nc, K, nrb,
                     ncb, col_done, clist, ccount);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Loadings GEMM of the factored bootstrap:
//   L*[rep][n][j] = ( [E' | L] [ZF ; M1] )[n][rep rp + j] / T
// (src/DynamicFactorModel.jl:90 for every replicate: L* = X*' F* / T with
// X*' F* = E' P' D F* + L (F'F*)): the r x r blocks M1 = F'F* sit under ZF
// as r extra k-rows and L' under E, so the whole finish is K = T + r MFMA
// depth (+1.6 %) and the epilogue a plain scaled store.  A^T operand
// [E; L'] (Kpad x lda, Kpad = round_up(T + r, 16), zero rows past T + r).
// B operand replicate-major: replicate rep's [ZF; M1; 0] is one contiguous
// Kpad x rp block (rp = r rounded up to even, column r zero when r is odd),
// so boot_zf writes whole lines; column x of the GEMM is (rep, j) =
// (x / rp, x % rp), and a lane's 16-B DMA pair (x, x + 1), x even, never
// straddles two replicates.  Both operands staged by LDS-DMA into [k][a]
// images (4-deep ring as gemmh_kernel).  Grid: the row blocks (64 variables)
// are spread over the XCDs — XCD x owns row blocks x, x+8, ... whose E slabs
// (64 x T x 8 B each) stay in its L2 — and every XCD walks the column blocks
// in the same order, so a ZF tile is fetched from HBM once and served to the
// other XCDs from the Infinity Cache.
template <int NBUF, int MINB>
__global__ __launch_bounds__(256, MINB) void gemm_loadings_kernel(const double *__restrict__ A, int64_t lda,
                                                                  const double *__restrict__ B, int Kp, int rp, int M,
                                                                  int Nc, int K, int nrb, int ncb, int r, double invT,
                                                                  double *__restrict__ Lout, int nrep) {
  __shared__ __attribute__((aligned(16))) double lds[NBUF * G2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int nrb8 = (nrb + 7) / 8;
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int rb = (j % nrb8) * 8 + xcd, cb = j / nrb8;
  if (rb >= nrb || cb >= ncb) return;
  const int abase = rb * GT, bbase = cb * GT;
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0.0;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int nst = (K + G2_KS - 1) / G2_KS;
  // running DMA pointers (both operands hold zero k-rows up to
  // round_up(K, 16), so the last stage needs no clamp)
  const double *pa[2], *pb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kc = 2 * (2 * wave + h) + (lane >> 5);
    const int sw = (2 * (lane & 31)) ^ ((kc & 7) << 2);
    pa[h] = A + (int64_t)kc * lda + min(abase + sw, (int)lda - 2);
    const int x = min(bbase + sw, Nc - 2), rep = x / rp;   // past Nc: finite, discarded
    pb[h] = B + ((int64_t)rep * Kp + kc) * rp + (x - rep * rp);
  }
  const int64_t astep = (int64_t)G2_KS * lda, bstep = (int64_t)G2_KS * rp;
  auto issue = [&](int s) {
    double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 2 * wave + h;
      __builtin_amdgcn_global_load_lds((gbl_void_t *)pa[h], (lds_void_t *)(la + c * 128), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_t *)pb[h], (lds_void_t *)(lb + c * 128), 16, 0, 0);
      pa[h] += astep;
      pb[h] += bstep;
    }
  };
  for (int s = 0; s < NBUF - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    const int ahead = min(NBUF - 2, nst - 1 - s);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NBUF - 1 < nst) issue(s + NBUF - 1);
    const double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    double af[8], bf[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = la[g2_offB(fkc, wr * 32 + 4 * f + fi)];
      bf[f] = lb[g2_offB(fkc, wc * 32 + 4 * f + fi)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int n = abase + wr * 32 + 4 * fa + oi;
      const int col = bbase + wc * 32 + 16 * q + 4 * blk + oj;
      const int rep = col / rp, jj = col - rep * rp;
      if (n < M && rep < nrep && jj < r) Lout[((int64_t)rep * M + n) * r + jj] = v * invT;
    }
}

// ZF: nrep replicate blocks of Kp x rp (see gemm_loadings_kernel); K = T + r.
hipError_t launch_gemm_loadings(const double *Eaug, int64_t lda, const double *ZF, int Kp, int rp, int N, int nrep,
                                int K, int r, double invT, double *Lout, hipStream_t st) {
  const int Nc = nrep * rp;
  const int nrb = (N + GT - 1) / GT, ncb = (Nc + GT - 1) / GT;
  const int nrb8 = (nrb + 7) / 8;
  // (the 3-deep ring at 3 workgroups per CU measured 20 % slower here, with
  // running pointers still 23 % slower: 4-deep at 2 per CU stays)
  hipLaunchKernelGGL((gemm_loadings_kernel<4, 2>), dim3(8 * nrb8 * ncb), dim3(256), 0, st, Eaug, lda, ZF, Kp, rp, N,
                     Nc, K, nrb, ncb, r, invT, Lout, nrep);
  return hipGetLastError();
}

// resident gram_dma_kernel workgroups on the chip for an m-row Gram
int gram_dma_slots(int m) { return (gemm_ring3(m) ? 3 : 2) * 256; }

// ---------------------------------------------------------------------------
// gram_dma_kernel: G = X X' of a plain row-major panel (m x K, ld % 16 == 0,
// zero columns K..ld-1) — the N > T Gram of principal_components
// (src/DynamicFactorModel.jl:87 `x*x'`) when no resample gather is fused: the
// base fit's H = E E' and the expanding windows' one prefix Gram
// (src/utils.jl:59-65 through the prefix identity).  Both
// operands are row blocks of X in [a][k] images, staged by LDS-DMA through the
// 4-deep ring of gemmh_kernel; only lower-triangular 64 x 64 tiles run, the
// epilogue writes both halves.  Split-K over blockIdx-derived z (partial
// images summed in fixed order by the caller).  XCD-aware order: the work
// list (z-major, then column tile J, then row tile I >= J) is cut into 8
// contiguous spans, XCD x taking span x, so the workgroups resident on one XCD
// share one k-range and a few column blocks (operands re-read from its L2).

template <int NBUF, int MINB>
__global__ __launch_bounds__(256, MINB) void gram_dma_kernel(const double *__restrict__ X, int64_t ld, int m, int K,
                                                             int nt, int tiles, int items, int span, int ksteps,
                                                             double *__restrict__ G, int64_t ldg, int64_t strideZ,
                                                             double alpha) {
  __shared__ __attribute__((aligned(16))) double lds[NBUF * G2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int item = (blockIdx.x & 7) * span + (blockIdx.x >> 3);
  if (item >= items) return;
  const int z = item / tiles;
  int u = item - z * tiles, J = 0;
  while (u >= nt - J) { u -= nt - J; ++J; }
  const int I = J + u;
  const int abase = I * GT, bbase = J * GT;
  // per-lane DMA sources: A chunk rows of block I, B chunk rows of block J
  G2Src src;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 2 * wave + h;
    const int a = 8 * c + (lane >> 3);
    const int ka = (2 * (lane & 7)) ^ (((a >> 1) & 1) << 3);
    src.a[h] = (int64_t)min(abase + a, m - 1) * ld + ka;   // rows past m: finite, discarded outputs
    src.b[h] = (int64_t)min(bbase + a, m - 1) * ld + ka;
    src.kb[h] = 0;
  }
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0.0;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int s0 = z * ksteps;
  const int nst = min((K + G2_KS - 1) / G2_KS, s0 + ksteps) - s0;   // the k tail reads ld's zero padding
  const int kbase = s0 * G2_KS;
  // running DMA pointers: one 64-bit add per operand and stage
  const double *pa0 = X + src.a[0] + kbase, *pa1 = X + src.a[1] + kbase;
  const double *pb0 = X + src.b[0] + kbase, *pb1 = X + src.b[1] + kbase;
  const int c0 = (2 * wave) * 128, c1 = c0 + 128;
  auto issue = [&](int s) {
    double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pa0, (lds_void_t *)(la + c0), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pb0, (lds_void_t *)(lb + c0), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pa1, (lds_void_t *)(la + c1), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pb1, (lds_void_t *)(lb + c1), 16, 0, 0);
    pa0 += G2_KS; pa1 += G2_KS; pb0 += G2_KS; pb1 += G2_KS;
  };
  for (int s = 0; s < NBUF - 1 && s < nst; ++s) issue(s);
  for (int s = 0; s < nst; ++s) {
    const int ahead = min(NBUF - 2, nst - 1 - s);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NBUF - 1 < nst)
      issue(s + NBUF - 1);
    const double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    double af[8], bf[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = la[g2_offA(wr * 32 + 4 * f + fi, fkc)];
      bf[f] = lb[g2_offA(wc * 32 + 4 * f + fi, fkc)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
  const bool diag = I == J;
  double *Gz = G + (int64_t)z * strideZ;
#pragma unroll
  for (int fa = 0; fa < 8; ++fa)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = ((b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8)) * alpha;   // alpha = 1: exact
      const int row = abase + wr * 32 + 4 * fa + oi;
      const int col = bbase + wc * 32 + 16 * q + 4 * blk + oj;
      if (row < m && col < m) {
        Gz[(int64_t)row * ldg + col] = v;
        if (!diag) Gz[(int64_t)col * ldg + row] = v;
      }
    }
}

// One launch of gram_dma_kernel over split-K partial images: S images of
// strideZ elements at G (S == 1: G is the output itself).
hipError_t launch_gram_dma(const double *X, int64_t ld, int m, int K, int S, int ksteps, double *G, int64_t ldg,
                           int64_t strideZ, hipStream_t st, double alpha) {
  const int nt = (m + GT - 1) / GT, tiles = nt * (nt + 1) / 2, items = tiles * S;
  const int span = (items + 7) / 8;
  // 3-deep ring at 3 workgroups per CU for the large Grams (more resident
  // waves beat a deeper ring there: tools/gemm_bench.hip, M = 2000)
  if (gemm_ring3(m))
    hipLaunchKernelGGL((gram_dma_kernel<3, 3>), dim3(8 * span), dim3(256), 0, st, X, ld, m, K, nt, tiles, items, span,
                       ksteps, G, ldg, strideZ, alpha);
  else
    hipLaunchKernelGGL((gram_dma_kernel<4, 2>), dim3(8 * span), dim3(256), 0, st, X, ld, m, K, nt, tiles, items, span,
                       ksteps, G, ldg, strideZ, alpha);
  return hipGetLastError();
}

// Requirements: lda, ldb even (16-B aligned pairs); B/A padding beyond the
// logical size is never read (masked).  The LDS-DMA kernel additionally
// needs Nc even and A's zero k-padding (lda >= round_up(K, 16)); otherwise
// the register-staged kernel runs.
hipError_t launch_gemm(bool a_trans, const double *A, int64_t lda, const double *B, int64_t ldb,
                       double *C, int64_t ldc, int M, int Nc, int K, hipStream_t st,
                       const int *col_done = nullptr, int col_group = 1, bool b_padded = false,
                       const int *clist = nullptr, const int *ccount = nullptr) {
  const int nrb = (M + GT - 1) / GT, ncb = (Nc + GT - 1) / GT;
  const int ncb8 = (ncb + 7) / 8 * 8;
  dim3 grid(nrb * ncb8), block(256);
  if (!a_trans && lda >= (K + G2_KS - 1) / G2_KS * G2_KS && Nc % 2 == 0 && Nc >= 2)
  {
    // B zero-padded to round_up(K, 16) rows: running DMA pointers, 3-deep
    // ring at 3 workgroups per CU (tools/gemm_bench.hip: 0.62 of peak at the
    // C3 shape, 0.75 at M = K = 2000, vs 0.60 / 0.71 for the clamped kernels)
    if (b_padded)
      hipLaunchKernelGGL((gemmh_kernel_t<3, 3, true>), grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb,
                         ncb, col_done, col_group, clist, ccount);
    else if (gemm_ring3(M))
      hipLaunchKernelGGL((gemmh_kernel_t<3, 3>), grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb, ncb,
                         col_done, col_group);
    else
      hipLaunchKernelGGL(gemmh_kernel, grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb, ncb, col_done,
                         col_group);
  }
  else if (a_trans)
    hipLaunchKernelGGL(gemm_kernel<true>, grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb, ncb,
                       col_done, col_group);
  else
    hipLaunchKernelGGL(gemm_kernel<false>, grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb, ncb,
                       col_done, col_group);
  return hipGetLastError();
}

}  // namespace dfm
