// Floor of the lasso leader's coordinate chain (C4 soft).
//
// lasso_coop_kernel's wave 0 visits the coordinates of a 64-coordinate block
// one after another (glmnet elnet1's cyclic order, src/targeted_predictors.jl
// :31-36 through GLMNet): for visit s, u = g_s + a_s, soft-threshold
// na = sign(u) max(|u| - lam, 0), d = na - a_s, then every gradient
// g_j -= G_js d.  The next visit needs g_{s+1} after that update, so the
// visits form one dependent chain.  This probe times, on one wave, 20 000
// blocks of 64 visits of:
//   prod   the production step (dfm_soft.hip lp_chain_step: readlane pair of
//          g and a0, the fp64 step, the vector update of g, writelane of gm);
//   nogm   the same without the off-chain writelane of gm;
//   pipe   the readlane of g taken off the chain: g_{s+1} is read from the
//          vector BEFORE d_s's update and d_s's term is applied to the scalar
//          copy with the same two operations (mul, sub) — bit-identical;
//   floor  the bare dependent fp64 chain of a visit, one chain per lane (no
//          cross-lane traffic at all; a_s, G_{s+1,s} in registers): mul, sub,
//          add, |.| - lam, compare + copysign select, sub — the minimum any
//          bit-exact elnet1 visit order needs on this hardware.
// Results (ns per visit, core cycles per visit) go to stdout; every variant's
// final state is summed to keep it live, and prod / nogm / pipe are checked
// bit-identical to each other.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/lcf tools/lasso_chain_floor.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int B = 64;

__device__ __forceinline__ double rdlane(double x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int L>
__device__ __forceinline__ double wrlane(double x, double v) {
  const long long b = __double_as_longlong(x), c = __double_as_longlong(v);
  int lo = (int)b, hi = (int)(b >> 32);
  asm("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"((int)c), "i"(L));
  asm("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"((int)(c >> 32)), "i"(L));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int V, int s>
__device__ __forceinline__ void step(double &g, double &gm, double &gk, const double a0, const double *Gr, double lam) {
  if constexpr (s < B) {
    if constexpr (V == 2) {   // pipe: gk (= g_s after every update) arrives from the previous step
      const double ak = rdlane(a0, s);
      const double uu = gk + ak;
      const double v = fabs(uu) - lam;
      const double na = v > 0.0 ? copysign(v, uu) : 0.0;
      const double d = na - ak;
      double gn = 0.0, gns = 0.0;
      if constexpr (s + 1 < B) { gn = rdlane(g, s + 1); gns = rdlane(Gr[s], s + 1); }   // before d's update
      g = g - Gr[s] * d;
      gk = gn - gns * d;   // lane s+1's own operations on its own operands
      step<V, s + 1>(g, gm, gk, a0, Gr, lam);
    } else {
      const double gk0 = rdlane(g, s), ak = rdlane(a0, s);
      const double uu = gk0 + ak;
      const double v = fabs(uu) - lam;
      const double na = v > 0.0 ? copysign(v, uu) : 0.0;
      const double d = na - ak;
      g = g - Gr[s] * d;
      if constexpr (V == 0) gm = wrlane<s>(gm, gk0);
      step<V, s + 1>(g, gm, gk, a0, Gr, lam);
    }
  }
}

// V: 0 prod, 1 nogm, 2 pipe
template <int V>
__global__ __launch_bounds__(64) void chain_kernel(const double *__restrict__ Gb, const double *__restrict__ g0,
                                                   const double *__restrict__ a0v, int nblk, double lam,
                                                   double *__restrict__ out, long long *__restrict__ tm) {
  __shared__ double s_gb[B * B];
  const int lane = threadIdx.x;
  for (int e = lane; e < B * B; e += 64) s_gb[e] = Gb[e];
  __syncthreads();
  double g = g0[lane];
  const double a0 = a0v[lane];
  double acc = 0.0, gm = 0.0;
  const long long w0 = wall_clock64(), c0 = clock64();
  for (int k = 0; k < nblk; ++k) {
    double Gr[B];
#pragma unroll
    for (int s = 0; s < B; ++s) Gr[s] = s_gb[s * B + lane];
    double gk = rdlane(g, 0);
    step<V, 0>(g, gm, gk, a0, Gr, lam);
    acc += gm;
    g = g * 0.5 + a0;   // keep the next block's values in range, data-dependent on this block
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = g + acc;
  if (lane == 0) { tm[0] = w1 - w0; tm[1] = c1 - c0; }
}

// floor: the bare dependent chain, one independent chain per lane (operands
// per lane in VGPRs, so no cross-lane instruction is needed at all)
__global__ __launch_bounds__(64) void floor_kernel(const double *__restrict__ Gb, const double *__restrict__ g0,
                                                   const double *__restrict__ a0v, int nblk, double lam,
                                                   double *__restrict__ out, long long *__restrict__ tm) {
  double gs[16], as[16];   // 16 operand pairs cycled (registers, not reloaded)
#pragma unroll
  for (int s = 0; s < 16; ++s) { gs[s] = Gb[s * B + threadIdx.x]; as[s] = a0v[(s + threadIdx.x) & 63]; }
  double d = g0[threadIdx.x], acc = 0.0;
  const long long w0 = wall_clock64(), c0 = clock64();
  for (int k = 0; k < nblk; ++k) {
#pragma unroll
    for (int s = 0; s < B; ++s) {
      const double gk = as[(s + 7) & 15] - gs[s & 15] * d;   // g_s after the previous visit's update
      const double uu = gk + as[s & 15];
      const double v = fabs(uu) - lam;
      const double na = v > 0.0 ? copysign(v, uu) : 0.0;
      d = na - as[s & 15];
    }
    acc += d;
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[threadIdx.x] = d + acc;
  if (threadIdx.x == 0) { tm[0] = w1 - w0; tm[1] = c1 - c0; }
}

int main(int argc, char **argv) {
  const int nblk = argc > 1 ? atoi(argv[1]) : 20000;
  double hG[B * B], hg[B], ha[B];
  srand(7);
  auto u = [] { return (double)rand() / RAND_MAX - 0.5; };
  for (int i = 0; i < B * B; ++i) hG[i] = 0.05 * u();
  for (int s = 0; s < B; ++s) hG[s * B + s] = 1.0;
  for (int i = 0; i < B; ++i) { hg[i] = u(); ha[i] = (i % 3) ? 0.0 : u(); }
  double *dG, *dg, *da, *dout;
  long long *dtm;
  CHK(hipMalloc(&dG, sizeof hG)); CHK(hipMalloc(&dg, sizeof hg)); CHK(hipMalloc(&da, sizeof ha));
  CHK(hipMalloc(&dout, 4 * B * sizeof(double))); CHK(hipMalloc(&dtm, 8 * sizeof(long long)));
  CHK(hipMemcpy(dG, hG, sizeof hG, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dg, hg, sizeof hg, hipMemcpyHostToDevice));
  CHK(hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice));
  const double lam = 0.1;
  const char *names[4] = {"prod", "nogm", "pipe", "floor"};
  double outs[4][B];
  for (int v = 0; v < 4; ++v) {
    for (int rep = 0; rep < 2; ++rep) {   // the first launch warms the code object
      switch (v) {
        case 0: chain_kernel<0><<<1, 64>>>(dG, dg, da, nblk, lam, dout + v * B, dtm + 2 * v); break;
        case 1: chain_kernel<1><<<1, 64>>>(dG, dg, da, nblk, lam, dout + v * B, dtm + 2 * v); break;
        case 2: chain_kernel<2><<<1, 64>>>(dG, dg, da, nblk, lam, dout + v * B, dtm + 2 * v); break;
        default: floor_kernel<<<1, 64>>>(dG, dg, da, nblk, lam, dout + v * B, dtm + 2 * v); break;
      }
      CHK(hipGetLastError());
      CHK(hipDeviceSynchronize());
    }
    long long tm[2];
    CHK(hipMemcpy(tm, dtm + 2 * v, sizeof tm, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(outs[v], dout + v * B, sizeof outs[v], hipMemcpyDeviceToHost));
    const double visits = 64.0 * nblk;
    printf("%-5s %8.2f ns/visit %8.1f cycles/visit  (%d blocks of 64 visits, wall %.3f ms)\n", names[v],
           tm[0] * 10.0 / visits, tm[1] / visits, nblk, tm[0] * 1e-5);
  }
  // prod (gm aside), nogm and pipe update g identically: the sums must agree bit for bit
  double s1 = 0, s2 = 0;
  for (int i = 0; i < B; ++i) { s1 += outs[1][i]; s2 += outs[2][i]; }
  printf("nogm == pipe (bit-identical g): %s\n", memcmp(outs[1], outs[2], sizeof outs[1]) == 0 ? "yes" : "NO");
  printf("checksums %.17g %.17g\n", s1, s2);
  return 0;
}
