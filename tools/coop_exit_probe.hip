// Does a bare cooperative launch followed by process exit crash under
// rocprofv3 --kernel-trace?  (Round-3 diagnosis of the exit-time SIGSEGV
// seen after C4's lasso_coop_kernel.)  Modes: 0 = cooperative launch,
// 1 = the same kernel by a plain launch, 2 = cooperative launch and an
// explicit hipDeviceReset before exit.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void coop_probe_kernel(double *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = 2.0 * i;
}

int main(int argc, char **argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const int n = 256 * 64;
  double *d = nullptr;
  if (hipMalloc(&d, n * 8) != hipSuccess) return 2;
  hipStream_t st;
  hipStreamCreate(&st);
  int nn = n;
  void *args[] = {&d, &nn};
  hipError_t e;
  if (mode == 1)
    e = hipLaunchKernel((const void *)coop_probe_kernel, dim3(64), dim3(256), args, 0, st);
  else
    e = hipLaunchCooperativeKernel((const void *)coop_probe_kernel, dim3(64), dim3(256), args, 0, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  double h = 0;
  hipMemcpy(&h, d + 7, 8, hipMemcpyDeviceToHost);
  printf("mode %d launch %s out[7] = %g\n", mode, hipGetErrorString(e), h);
  hipFree(d);
  hipStreamDestroy(st);
  if (mode == 2) hipDeviceReset();
  return e == hipSuccess ? 0 : 1;
}
