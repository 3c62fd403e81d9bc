// dfm_gemm.hip — batched-replicate fp64 GEMM on MFMA (v_mfma_f64_4x4x4_4b).
//
//   C[M x Nc] = op(A) B,  op(A) = A (M x K row-major)  or  A^T (A stored K x M)
//   B: K x Nc row-major (the k-rows of every replicate's skinny operand laid
//   side by side: column block = one replicate's p columns).
//
// This is the compute core of the factored bootstrap (dfm_boot.hip): one
// fixed, cache-resident left operand (H = E E' or E') shared by every
// replicate of a batch, so the per-replicate eigen-iterations and the
// loadings pass become single large MFMA GEMMs instead of nb memory-bound
// skinny products.  Tiling, fragment maps and the swizzled LDS images are
// those of the Gram kernel (dfm_gram.hip); grid order is XCD-aware: the row
// blocks of one column block are issued to one XCD so a B tile is fetched
// from HBM once and re-read from that XCD's L2.
#include "dfm_common.h"

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

// Requirements: lda, ldb even (16-B aligned pairs); B/A padding beyond the
// logical size is never read (masked).
hipError_t launch_gemm(bool a_trans, const double *A, int64_t lda, const double *B, int64_t ldb,
                       double *C, int64_t ldc, int M, int Nc, int K, hipStream_t st,
                       const int *col_done = nullptr, int col_group = 1) {
  const int nrb = (M + GT - 1) / GT, ncb = (Nc + GT - 1) / GT;
  const int ncb8 = (ncb + 7) / 8 * 8;
  dim3 grid(nrb * ncb8), block(256);
  if (a_trans)
    hipLaunchKernelGGL(gemm_kernel<true>, grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb, ncb,
                       col_done, col_group);
  else
    hipLaunchKernelGGL(gemm_kernel<false>, grid, block, 0, st, A, lda, B, ldb, C, ldc, M, Nc, K, nrb, ncb,
                       col_done, col_group);
  return hipGetLastError();
}

}  // namespace dfm
