// Probe the operand/result lane maps of v_mfma_f64_4x4x4_4b_f64 with one-hot experiments:
// wave w = (la, lb): A one-hot at lane la, B one-hot at lane lb; dump the 64 C values.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void onehot_k(double* out) {
  int w = blockIdx.x, la = w >> 6, lb = w & 63, l = threadIdx.x;
  double a = (l == la) ? 1.0 : 0.0, b = (l == lb) ? 1.0 : 0.0;
  double c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[w * 64 + l] = c;
}
int main() {
  double* d; hipMalloc(&d, 4096 * 64 * 8);
  onehot_k<<<4096, 64>>>(d); hipDeviceSynchronize();
  std::vector<double> h(4096 * 64); hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  // print, for each (la, lb) pair with a nonzero result, the output lane(s)
  int cnt = 0;
  for (int la = 0; la < 64; ++la) for (int lb = 0; lb < 64; ++lb)
    for (int l = 0; l < 64; ++l) if (h[(la * 64 + lb) * 64 + l] != 0.0) { printf("%d %d %d %g\n", la, lb, l, h[(la*64+lb)*64+l]); ++cnt; }
  fprintf(stderr, "nonzero=%d\n", cnt);
}
