// Dev microbenchmark for dfm_gemm.hip: the H.Z kernels (register-staged
// gemm_kernel as the reference, the LDS-DMA running-pointer gemmh_kernel_t and
// the fragment-double-buffered gemmh_db_kernel at several ring depths /
// occupancies) and the A^T kernel over the bootstrap's shapes, with a
// max-abs-difference check against the register-staged kernel.
// Measured (round 2, M = K = 500, Nc = 160000): run3/3 0.695 of peak; the
// double-buffered kernel needs 219-226 VGPRs, so it runs at 2 workgroups per CU
// (db4/2, db3/2: 0.58) or spills at 3 (db3/3, db2/3: 0.09) -- rejected, kept
// here as the record.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gemm_bench tools/gemm_bench.hip
#include "../dynamicfactormodels.jl_amd/csrc/dfm_gemm.hip"
#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>
using namespace dfm;
namespace dfm {
// ---------------------------------------------------------------------------
// gemmh_db_kernel: gemmh_kernel_t<·,·,RUN> with the MFMA fragments double-
// buffered in two register sets.  A wave no longer waits on its own fragment
// reads at the top of every stage: the barrier that publishes stage s+1 (and
// retires every wave's reads of stage s, whose ring slot is refilled right
// after it) comes before stage s's MFMAs, and stage s+1's fragment reads are
// issued ahead of them.  The stage loop is unrolled by two so the sets
// alternate without register moves (tools/mfma4_occupancy_probe.hip: the 8x8
// fragment loop from LDS runs at 0.84 of peak with one set, 0.92 with two;
// operands in registers 0.95).  The prologue fills all NBUF ring slots.
DFM_DEV void g2_vmwait(int ahead) {   // own DMAs: at most `ahead` later stages (4 per stage) outstanding
  if (ahead >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The double-buffered stage loop shared by the LDS-DMA kernels: issue(s)
// starts stage s's DMAs into ring slot s % NBUF (4 per wave), frags(s, af, bf)
// reads this lane's 8 + 8 fragments of stage s.
template <int NBUF, class Issue, class Frags>
DFM_DEV void g2_db_mainloop(int nst, double (&acc)[8][8], Issue &issue, Frags &frags) {
  static_assert(NBUF >= 2 && NBUF <= 4, "ring depth");
  auto publish = [&](int s) {   // stage s+1 visible, every wave's reads of stage s retired
    g2_vmwait(min(NBUF - 2, nst - s - 2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NBUF < nst) issue(s + NBUF);
  };
  auto mma = [&](const double *af, const double *bf) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[i][q] = mfma4(af[i], bf[q], acc[i][q]);
  };
  for (int s = 0; s < NBUF && s < nst; ++s) issue(s);
  g2_vmwait(min(NBUF, nst) - 1);
  __builtin_amdgcn_s_barrier();
  double ax[8], bx[8], ay[8], by[8];
  frags(0, ax, bx);
  for (int s = 0; s < nst; s += 2) {
    if (s + 1 < nst) {
      publish(s);
      frags(s + 1, ay, by);
    }
    mma(ax, bx);
    if (s + 1 >= nst) break;
    if (s + 2 < nst) {
      publish(s + 1);
      frags(s + 2, ax, bx);
    }
    mma(ay, by);
  }
}

template <int NBUF, int MINB>
__global__ __launch_bounds__(256, MINB) void gemmh_db_kernel(const double *__restrict__ A, int64_t lda,
                                                          const double *__restrict__ B, int64_t ldb,
                                                          double *__restrict__ C, int64_t ldc, int M, int Nc, int K,
                                                          int nrb, int ncb, const int *__restrict__ col_done,
                                                          int col_group, const int *__restrict__ clist,
                                                          const int *__restrict__ ccount_p) {
  __shared__ __attribute__((aligned(16))) double lds[NBUF * G2_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int rb = j % nrb, cb = (j / nrb) * 8 + xcd;
  if (cb >= ncb) return;
  const int abase = rb * GT, bbase = cb * GT;
  const int ccount = clist ? *ccount_p : 0;
  if (clist && bbase >= ccount * col_group) return;
  if (col_done && !clist) {
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
  const double *pa0 = A + src.a[0], *pa1 = A + src.a[1], *pb0 = B + src.b[0], *pb1 = B + src.b[1];
  const int64_t bstep = (int64_t)G2_KS * ldb;
  const int c0 = (2 * wave) * 128, c1 = c0 + 128;
  auto issue = [&](int s) {
    double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pa0, (lds_void_t *)(la + c0), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pb0, (lds_void_t *)(lb + c0), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pa1, (lds_void_t *)(la + c1), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void_t *)pb1, (lds_void_t *)(lb + c1), 16, 0, 0);
    pa0 += G2_KS; pa1 += G2_KS; pb0 += bstep; pb1 += bstep;
  };
  auto frags = [&](int s, double *af, double *bf) {
    const double *la = lds + (s % NBUF) * G2_STAGE, *lb = la + GT * G2_KS;
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      af[f] = la[g2_offA(wr * 32 + 4 * f + fi, fkc)];
      bf[f] = lb[g2_offB(fkc, wc * 32 + 4 * f + fi)];
    }
  };
  g2_db_mainloop<NBUF>(nst, acc, issue, frags);
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

}  // namespace dfm
__global__ void fill(double *p, size_t n, double s, int64_t ld, int valid) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = ((int64_t)(i % ld) < valid) ? ((i * 2654435761ull) % 1000) * 1e-3 * s - 0.5 : 0.0;
}
__global__ void maxdiff(const double *a, const double *b, size_t n, unsigned long long *out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    const double d = fabs(a[i] - b[i]);
    atomicMax(out, (unsigned long long)__double_as_longlong(d));
  }
}

int main() {
  struct Cfg { bool at; int M, K, Nc; };
  std::vector<Cfg> cfgs = {{false, 500, 500, 160000}, {false, 512, 512, 160000}, {false, 500, 500, 40000},
                           {false, 1024, 1024, 40000}, {false, 2000, 2000, 16000}, {true, 2000, 500, 80000}};
  for (auto c : cfgs) {
    const int64_t lda = c.at ? ((c.M + 15) / 16 * 16) : ((c.K + 15) / 16 * 16);
    const size_t na = c.at ? (size_t)c.K * lda : (size_t)c.M * lda;
    const int64_t ldb = c.Nc, ldc = c.Nc;
    double *A, *B, *C, *C2;
    hipMalloc(&A, na * 8); hipMalloc(&B, (size_t)((c.K + 15) / 16 * 16) * ldb * 8); hipMemset(B, 0, (size_t)((c.K + 15) / 16 * 16) * ldb * 8);
    hipMalloc(&C, (size_t)c.M * ldc * 8); hipMalloc(&C2, (size_t)c.M * ldc * 8);
    fill<<<(na + 255) / 256, 256>>>(A, na, 1.0, lda, c.at ? c.M : c.K);
    fill<<<((size_t)c.K * ldb + 255) / 256, 256>>>(B, (size_t)c.K * ldb, 2.0, ldb, c.Nc);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int nrb = (c.M + GT - 1) / GT, ncb = (c.Nc + GT - 1) / GT, ncb8 = (ncb + 7) / 8 * 8;
    const dim3 grid(nrb * ncb8);
    const int variants = c.at ? 1 : 6;
    for (int v = 0; v < variants; ++v) {
      auto run = [&](double *Cout) {
        if (c.at) hipLaunchKernelGGL(gemm_kernel<true>, grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else if (v == 0) hipLaunchKernelGGL(gemm_kernel<false>, grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else if (v == 1) hipLaunchKernelGGL((gemmh_kernel_t<3, 3, true>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1, nullptr, nullptr);
        else if (v == 2) hipLaunchKernelGGL((gemmh_db_kernel<3, 3>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1, nullptr, nullptr);
        else if (v == 3) hipLaunchKernelGGL((gemmh_db_kernel<4, 2>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1, nullptr, nullptr);
        else if (v == 4) hipLaunchKernelGGL((gemmh_db_kernel<3, 2>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1, nullptr, nullptr);
        else hipLaunchKernelGGL((gemmh_db_kernel<2, 3>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1, nullptr, nullptr);
      };
      double *Cout = v == 0 ? C : C2;
      if (v > 0) hipMemset(C2, 0, (size_t)c.M * ldc * 8);
      for (int w = 0; w < 3; ++w) run(Cout);
      const int reps = 10;
      hipEventRecord(e0);
      for (int w = 0; w < reps; ++w) run(Cout);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double t = ms / reps * 1e-3, fl = 2.0 * c.M * (double)c.Nc * c.K;
      static const char *names[] = {"reg     ", "run3/3  ", "db3/3   ", "db4/2   ", "db3/2   ", "db2/3   "};
      printf("%s A%s M=%5d K=%5d Nc=%6d : %8.3f ms  %6.2f TF/s (%.1f%% of 78.6)\n", names[v],
             c.at ? "^T" : "  ", c.M, c.K, c.Nc, t * 1e3, fl / t / 1e12, fl / t / 1e12 / 78.6 * 100);
      if (v > 0) {
        unsigned long long *d, h = 0;
        hipMalloc(&d, 8); hipMemset(d, 0, 8);
        const size_t n = (size_t)c.M * ldc;
        maxdiff<<<(n + 255) / 256, 256>>>(C, C2, n, d);
        hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
        double md; memcpy(&md, &h, 8);
          printf("     max |reg - glds| = %.3e\n", md);
        hipFree(d);
    }
    }
    hipFree(A); hipFree(B); hipFree(C); hipFree(C2);
  }
  return 0;
}
