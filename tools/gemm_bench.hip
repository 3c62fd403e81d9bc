// Dev microbenchmark for dfm_gemm.hip: time launch_gemm over shapes/layouts.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gemm_bench tools/gemm_bench.hip
#include "../dynamicfactormodels.jl_amd/csrc/dfm_gemm.hip"
#include <cstdio>
#include <vector>
using namespace dfm;
__global__ void fill(double *p, size_t n, double s) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = ((i * 2654435761ull) % 1000) * 1e-3 * s - 0.5;
}
int main(int argc, char **argv) {
  struct Cfg { bool at; int M, K, Nc; };
  std::vector<Cfg> cfgs = {{false, 500, 500, 160000}, {true, 500, 500, 160000}, {false, 512, 512, 160000},
                           {false, 2000, 500, 80000}, {true, 2000, 500, 80000}, {false, 500, 500, 40000},
                           {false, 1024, 1024, 40000}};
  for (auto c : cfgs) {
    const int64_t lda = c.at ? ((c.M + 15) / 16 * 16) : ((c.K + 15) / 16 * 16);
    const size_t na = c.at ? (size_t)c.K * lda : (size_t)c.M * lda;
    const int64_t ldb = c.Nc, ldc = c.Nc;
    double *A, *B, *C;
    hipMalloc(&A, na * 8); hipMalloc(&B, (size_t)c.K * ldb * 8); hipMalloc(&C, (size_t)c.M * ldc * 8);
    fill<<<(na + 255) / 256, 256>>>(A, na, 1.0);
    fill<<<((size_t)c.K * ldb + 255) / 256, 256>>>(B, (size_t)c.K * ldb, 2.0);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) launch_gemm(c.at, A, lda, B, ldb, C, ldc, c.M, c.Nc, c.K, 0);
    const int reps = 10;
    hipEventRecord(e0);
    for (int w = 0; w < reps; ++w) launch_gemm(c.at, A, lda, B, ldb, C, ldc, c.M, c.Nc, c.K, 0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double t = ms / reps * 1e-3, fl = 2.0 * c.M * (double)c.Nc * c.K;
    printf("A%s M=%5d K=%5d Nc=%6d : %8.3f ms  %6.2f TF/s (%.1f%% of 78.6)\n", c.at ? "^T" : "  ", c.M, c.K, c.Nc,
           t * 1e3, fl / t / 1e12, fl / t / 1e12 / 78.6 * 100);
    hipFree(A); hipFree(B); hipFree(C);
  }
  return 0;
}
