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
constexpr int GT = 64, KS = 16;
DFM_DEV int off_rows(int a, int kc) { return a * KS + (kc ^ (((a >> 1) & 1) << 3)); }  // [a][k]
DFM_DEV int off_cols(int a, int kc) { return kc * GT + (a ^ ((kc & 7) << 2)); }         // [k][a]
}  // namespace

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

  double2 ra[2], rbv[2];
  bool oka[2], okb[2];
  auto load_stage = [&](int k0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (!A_TRANS) {   // A rows: chunk -> (row a = c>>3, k pair 2*(c&7))
        const int a = (tid >> 3) + 32 * h, k = k0 + 2 * (tid & 7);
        oka[h] = (abase + a < M) && (k < K);
        if (oka[h]) ra[h] = *reinterpret_cast<const double2 *>(A + (int64_t)(abase + a) * lda + k);
      } else {                    // A^T: k-rows of A (contiguous in a)
        const int kc = (tid >> 5) + 8 * h, a = 2 * (tid & 31);
        oka[h] = (k0 + kc < K) && (abase + a < M);
        if (oka[h]) ra[h] = *reinterpret_cast<const double2 *>(A + (int64_t)(k0 + kc) * lda + abase + a);
      }
      const int kc = (tid >> 5) + 8 * h, col = 2 * (tid & 31);
      okb[h] = (k0 + kc < K) && (bbase + col < Nc);
      if (okb[h]) rbv[h] = *reinterpret_cast<const double2 *>(B + (int64_t)(k0 + kc) * ldb + bbase + col);
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double2 z = {0.0, 0.0};
      int oa;
      if constexpr (!A_TRANS) oa = off_rows((tid >> 3) + 32 * h, 2 * (tid & 7));
      else oa = off_cols(2 * (tid & 31), (tid >> 5) + 8 * h);
      *reinterpret_cast<double2 *>(&lds[buf][0][oa]) = oka[h] ? ra[h] : z;
      *reinterpret_cast<double2 *>(&lds[buf][1][off_cols(2 * (tid & 31), (tid >> 5) + 8 * h)]) =
          okb[h] ? rbv[h] : z;
    }
  };

  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[i][q] = 0.0;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int nst = (K + KS - 1) / KS;
  load_stage(0);
  store_stage(0);
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    if (s + 1 < nst) load_stage((s + 1) * KS);
    double af[8], bf[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      const int a = wr * 32 + 4 * f + fi;
      af[f] = A_TRANS ? lds[buf][0][off_cols(a, fkc)] : lds[buf][0][off_rows(a, fkc)];
      bf[f] = lds[buf][1][off_cols(wc * 32 + 4 * f + fi, fkc)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
    if (s + 1 < nst) store_stage(buf ^ 1);
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
