// Probe of the leader/helper hand-off used by lasso_coop_kernel (gfx950),
// following cdna_hip_programming.md §6 Guideline 16: producer = stores ->
// s_waitcnt vmcnt(0) -> barrier -> lane 0 release fence (agent) -> vmcnt(0)
// -> relaxed flag store / atomic add; consumer = ONE lane relaxed poll +
// s_sleep -> acquire fence (agent) -> vmcnt(0) -> barrier.  Flags on lines
// of their own.  variant 0: helper signals by a counter add, 1: flag store.
#include <hip/hip_runtime.h>
#include <cstdio>
struct alignas(256) Line { int v; int pad[63]; };
struct Ctl { Line seq, done, flag; long long t[8]; int err; };
__device__ __forceinline__ bool poll_ge(int *p, int target, long long tmo) {
  const long long t0 = wall_clock64();
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (wall_clock64() - t0 > tmo) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}
__device__ __forceinline__ void signal_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__global__ __launch_bounds__(256, 1) void k(Ctl *c, int variant, int ntask, long long tmo) {
  __shared__ char big[110 * 1024];
  __shared__ int s;
  big[threadIdx.x] = 0;
  const int tid = threadIdx.x;
  if (blockIdx.x == 1) {   // helper
    for (int q = 1;; ++q) {
      if (tid == 0) s = poll_ge(&c->seq.v, q, tmo) ? __hip_atomic_load(&c->seq.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
      __syncthreads();
      if (s < 0 || s > ntask) break;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        signal_release();
        if (variant == 1) __hip_atomic_store(&c->flag.v, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(&c->done.v, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  for (int q = 1; q <= ntask + 1; ++q) {   // leader
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const long long t0 = wall_clock64();
      signal_release();
      __hip_atomic_store(&c->seq.v, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (q <= ntask) {
        const bool ok = poll_ge(variant == 1 ? &c->flag.v : &c->done.v, q, tmo);
        if (!ok) c->err = q;
        if (q <= 8) c->t[q - 1] = ok ? wall_clock64() - t0 : -1;
        s = ok;
      }
    }
    __syncthreads();
    if (q <= ntask && !s) {   // abort: publish past the end
      if (tid == 0) __hip_atomic_store(&c->seq.v, ntask + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}
int main() {
  Ctl *c;
  hipMalloc(&c, sizeof(Ctl));
  for (int variant = 0; variant < 2; ++variant) {
    hipMemset(c, 0, sizeof(Ctl));
    int ntask = 1000;
    long long tmo = 50000000;   // 0.5 s
    void *args[] = {&c, &variant, &ntask, &tmo};
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipError_t e = hipLaunchCooperativeKernel((const void *)k, dim3(2), dim3(256), args, 0, 0);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    Ctl h; hipMemcpy(&h, c, sizeof h, hipMemcpyDeviceToHost);
    printf("variant %d launch %s: %.3f ms for %d round trips (%.2f us each); seq %d done %d flag %d err %d; first hops (ticks):",
           variant, hipGetErrorString(e), ms, ntask, ms * 1e3 / ntask, h.seq.v, h.done.v, h.flag.v, h.err);
    for (int i = 0; i < 8; ++i) printf(" %lld", h.t[i]);
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
