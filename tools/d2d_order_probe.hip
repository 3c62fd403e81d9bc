// Does hipMemcpyPeer (device-to-device, same device) return before the copy
// has landed, and is a kernel on a hipStreamNonBlocking stream launched right
// after it ordered behind it?  dfm_model_clone (dfm_api.hip) made the second
// bootstrap lane's copy of a fit with hipMemcpyPeer on the legacy null stream
// and the lane then ran on its own non-blocking stream with no event between
// them (VERDICT r04 Weak #1).  This probe copies a large buffer whose LAST
// element differs from the destination's old contents, launches at once a
// one-thread kernel on a non-blocking stream that reads that element, and
// reports what it saw and how long the host call took.
//
// build: hipcc -O2 --offload-arch=gfx950 tools/d2d_order_probe.hip -o tools/d2d_order_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void fill(double *p, size_t n, double v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void peek(const double *p, size_t n, double *out) { out[0] = p[0]; out[1] = p[n - 1]; }

int main() {
  const size_t n = (size_t)96 << 20;   // 768 MB per buffer
  double *src, *dst, *seen;
  if (hipMalloc(&src, n * 8) || hipMalloc(&dst, n * 8) || hipHostMalloc(&seen, 16)) return 2;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int late = 0;
  for (int trial = 0; trial < 3; ++trial) {
    fill<<<4096, 256>>>(src, n, 1.0 + trial);
    fill<<<4096, 256>>>(dst, n, -1.0);
    hipDeviceSynchronize();
    seen[0] = seen[1] = 0.0;
    const auto t0 = std::chrono::steady_clock::now();
    hipMemcpyPeer(dst, 0, src, 0, n * 8);
    const auto t1 = std::chrono::steady_clock::now();
    peek<<<1, 1, 0, s>>>(dst, n, seen);
    hipStreamSynchronize(s);
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    printf("trial %d: hipMemcpyPeer returned after %.1f us (768 MB); non-blocking-stream kernel saw first %.1f last %.1f"
           " (copied value %.1f, old -1.0)\n", trial, us, seen[0], seen[1], 1.0 + trial);
    if (seen[1] != 1.0 + trial || seen[0] != 1.0 + trial) late = 1;
    hipDeviceSynchronize();
  }
  printf(late ? "RESULT: the kernel ran before the copy landed (unordered)\n"
              : "RESULT: the copy had landed before the kernel read it\n");
  return 0;
}
