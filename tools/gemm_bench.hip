// Dev microbenchmark for dfm_gemm.hip: both H.Z kernels (register-staged
// gemm_kernel, LDS-DMA gemmh_kernel) and the A^T kernel over the bootstrap's
// shapes, with a max-abs-difference check between the two H.Z kernels.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gemm_bench tools/gemm_bench.hip
#include "../dynamicfactormodels.jl_amd/csrc/dfm_gemm.hip"
#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>
using namespace dfm;
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
    const int variants = c.at ? 1 : 5;
    for (int v = 0; v < variants; ++v) {
      auto run = [&](double *Cout) {
        if (c.at) hipLaunchKernelGGL(gemm_kernel<true>, grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else if (v == 0) hipLaunchKernelGGL(gemm_kernel<false>, grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else if (v == 1) hipLaunchKernelGGL((gemmh_kernel_t<4, 2>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else if (v == 2) hipLaunchKernelGGL((gemmh_kernel_t<3, 2>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else if (v == 3) hipLaunchKernelGGL((gemmh_kernel_t<3, 3>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1);
        else hipLaunchKernelGGL((gemmh_kernel_t<3, 3, true>), grid, dim3(256), 0, 0, A, lda, B, ldb, Cout, ldc, c.M, c.Nc, c.K, nrb, ncb, nullptr, 1, nullptr, nullptr);
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
      static const char *names[] = {"reg     ", "glds4/2 ", "glds4/2p", "glds3/2 ", "glds3/3 ", "glds3/3p", "run3/3  ", "run3/3p "};
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
