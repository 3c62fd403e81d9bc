// dfm_eig.hip — K2: batched top-k symmetric eigensolver (block subspace
// iteration with Rayleigh–Ritz), replacing the full-spectrum LAPACK `eig` of
// principal_components (src/DynamicFactorModel.jl:78-79, :87-88) whose
// trailing columns the reference never consumes (only [:, 1:r], :33, :131).
//
// Per replicate b (G_b is m x m, row-major, ldg):
//   gq    : Y = G Q  (v_mfma_f64_4x4x4_4b, 64 rows / workgroup) + per-row-block
//           partials of Q'Y, Y'Y, Q'Q; first checks the previous iteration's
//           explicit residuals and retires converged replicates.
//   small : one wave per replicate.  Q'Q = LL' (the basis is re-orthonormalised
//           implicitly: CholQR folded into the Rayleigh–Ritz step), H~ =
//           L^-1 (Q'Y) L^-T, parallel cyclic Jacobi on p x p, A = L^-T S,
//           Z'Z = A'(Y'Y)A = L2 L2', Bm = A L2^-T.
//   apply : U = Q A (Ritz vectors), Q <- Y Bm (next orthonormal basis),
//           W = Y A - U diag(theta) -> per-block residual partials.
//   final : sign canonicalisation (largest-|.| entry positive, first index).
// Converged when ||G u_j - theta_j u_j|| <= tol * |theta_1| for j < k.
// Deterministic: fixed-order reductions only, no float atomics.
#include "dfm_common.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace dfm {

constexpr int EROWS = 64;  // rows per workgroup in gq/apply

struct EigWork {
  double *Q, *Y, *U;       // nb x m x P
  double *S;               // nb x m x P: the direct path's second Horner vector (filters of degree > 2)
  double *part;            // nb x nrb x 3 x P x P
  double *rpart;           // nb x nrb x P
  double *small;           // nb x SMALL_STRIDE (A, Bm, theta, dead)
  int *done, *iters, *active;
  double *trace;           // nb
  long long *dbg;          // phase stamps of replicate 0 (SMALL_STAMP) when a diagnostic build points it at a buffer; null
  // strict rule's gap: 0 = distance to the neighbouring Ritz values (every
  // wanted eigenVECTOR converged); 1 = distance to the first unwanted Ritz
  // value theta_k (the wanted SUBSPACE converged: for statistics invariant to
  // rotations within span(F_r) — Chow tests, V, criteria, eigenvalues)
  int subspace;
  int no_vectors;          // eigenvalue-only caller (Uk == nullptr): the Ritz vectors are never written
};
#define SMALL_STAMP(i) do { if (w.dbg && rep == 0 && lane == 0) w.dbg[i] = (long long)wall_clock64(); } while (0)
template <int P> constexpr int small_stride() { return 2 * P * P + 4 * P; }
constexpr int SMALL_CHOL1_DONE = 0x100;   // small_rr: R4 already holds chol(Q'Q)^-1 (eig_fused forms it during Y = G Q)
constexpr int SMALL_STAGE_A = 0x200;      // small_rr: stop once A (R2), theta and Z'Z (R3) are formed
constexpr int SMALL_STAGE_B = 0x400;      // small_rr: only chol(Z'Z) and Bm (eig_fused: beside the U pass)

// ----------------------------------------------------------------- init
template <int P>
__global__ void eig_init_kernel(double *__restrict__ Q, int m, int p, const double *__restrict__ warm,
                                int kw, int *__restrict__ done, uint64_t seed, int64_t rep0, int ps = P) {
  // ps: row stride (the factored solver's compact rows hold ps = pz <= P columns)
  const int rep = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)m * ps) return;
  const int row = (int)(e / ps), c = (int)(e % ps);
  double v = 0.0;
  if (c < kw) v = warm[(int64_t)row * kw + c];
  else if (c < p) v = hash_unit(seed, row, c);   // same start for every replicate: call/batch/shard-invariant
  Q[(int64_t)rep * m * ps + e] = v;
  if (e == 0) done[rep] = 0;
}

__global__ void eig_trace_kernel(const double *__restrict__ G, int64_t ldg, int64_t strideG, int m,
                                 double *__restrict__ trace) {
  const int rep = blockIdx.x, lane = threadIdx.x;
  const double *g = G + (int64_t)rep * strideG;
  double s = 0.0;
  for (int i = lane; i < m; i += 64) s += g[(int64_t)i * ldg + i];
  s = wave_sum(s);
  if (lane == 0) trace[rep] = s;
}

// Convergence test of iteration it-1's Ritz pairs (explicit residual partials
// written by eig_apply).  Every workgroup of a replicate evaluates it on the
// same data (so they agree); row block 0 records the verdict.  Called by one
// whole wave: lane (j, r) loads one partial, the sum over r is a fixed-order
// shuffle tree — no serial chain of dependent global loads.
// tail: the small record's tail (theta[P], dead[P], residual history 2 x P);
// rp: the nrb row-block residual partials (P apart); d: the replicate's done flag.
template <int P>
DFM_DEV int check_converged(EigWork &w, double *tail, const double *rp, double tr, int d, int rep, int rb,
                            int nrb, int k, int p, double tol, int it, int check_only) {
  const int lane = threadIdx.x & 63;
  if (!d && it > 0) {
    // Converged when every wanted Ritz pair j < k satisfies
    //   res_j <= tol * gap_j            (eigenvector error ~ res/gap <= tol)
    // or sits at the rounding floor: res_j <= 2e-14 |theta_1|, or
    //   res_j <= 1e-11 |theta_1| and stagnating (no 2x decrease).
    const double *th = tail;
    const double *prev = tail + 2 * P + ((it - 1) & 1) * P;
    double *next = tail + 2 * P + (it & 1) * P;
    const double th0 = fabs(th[0]);
    bool ok = true;
    if (tol < 0.0) {
      // Eigenvalue-only statistics (V, criteria, eigenvalues, trace): a Ritz
      // value's error is quadratic in its residual, |theta_j - lambda_j| <=
      // res_j^2 / gap_j (Kato-Temple; gap_j = distance to the neighbouring
      // Ritz values, halved for safety).  Converged when every wanted
      // eigenvalue is within -tol relative AND the summed bound moves the
      // residual energy trace - sum_j theta_j (the numerator of V(k),
      // src/criteria.jl:5) by at most -tol relative.
      const double tv = -tol;
      double bsum = 0.0, tsum = 0.0;
      bool okall = true, floor_ok = true;
      for (int j = lane; j < k; j += 64) {
        double rs = 0.0;
        for (int r = 0; r < nrb; ++r) rs += rp[r * P + j];
        double gap = INFINITY;
        if (j > 0) gap = fmin(gap, fabs(th[j] - th[j - 1]));
        if (j + 1 < p) gap = fmin(gap, fabs(th[j] - th[j + 1]));
        const double bnd = rs / (0.5 * gap);
        bsum += bnd;
        tsum += th[j];
        okall = okall && (bnd <= tv * fabs(th[j]) || sqrt(rs) <= 2e-14 * th0);
        floor_ok = floor_ok && sqrt(rs) <= 2e-14 * th0;
        if (rb == 0) next[j] = sqrt(rs);
      }
      bsum = wave_sum(bsum);
      tsum = wave_sum(tsum);
      // residual energy floored at 1e-6 trace: below that the reference's own
      // rounding of ||E||^2 already exceeds -tol relative (exact-rank panels)
      const double vnum = fmax(fabs(tr - tsum), 1e-6 * fabs(tr));
      ok = !__any(!okall) && (bsum <= tv * vnum || !__any(!floor_ok));
    } else
    for (int j0 = 0; j0 < k; j0 += 64) {
      // lanes: j = j0 + lane / G, r = lane % G   with G = power of two >= nrb
      // (capped at 64: past 64 row blocks — m > 4096 — lane r also sums
      // blocks r + 64, r + 128, ... in order before the shuffle tree)
      int G = 1;
      while (G < nrb && G < 64) G <<= 1;
      const int per = 64 / G;   // residual columns handled per pass
      for (int jj = 0; jj < 64 && j0 + jj < k; jj += per) {
        const int j = j0 + jj + lane / G, r = lane % G;
        double v = 0.0;
        if (j < k)
          for (int rr = r; rr < nrb; rr += G) v += rp[rr * P + j];
        for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        // lanes with r == 0 hold the column sums
        bool okj = true;
        if (j < k && r == 0) {
          const double res = sqrt(v);
          double gap = INFINITY;
          if (w.subspace && k < p) {   // (k == p: no unwanted Ritz value, the neighbour rule)
            gap = fabs(th[j] - th[k]);
          } else {
            if (j > 0) gap = fmin(gap, fabs(th[j] - th[j - 1]));
            if (j + 1 < p) gap = fmin(gap, fabs(th[j] - th[j + 1]));
          }
          const bool stagn = it > 2 && res <= 1e-11 * th0 && res > 0.5 * prev[j];
          okj = (res <= tol * gap || res <= 2e-14 * th0 || stagn);
          if (rb == 0) next[j] = res;
        }
        ok = ok && !__any(!okj);
      }
    }
    if (ok) {
      d = 1;
      if (rb == 0 && lane == 0) { w.done[rep] = 1; w.iters[rep] = it; }
    }
  }
  if (rb == 0 && lane == 0 && !d) atomicAdd(&w.active[it], 1);
  return d || check_only;
}

// Partial Q'Y, Y'Y, Q'Q over one 64-row block (fixed order), LDS images sQ/sY.
template <int P, int SQ>
DFM_DEV void emit_partials(const double *sQ, const double *sY, double *pp) {
  for (int e = threadIdx.x; e < 3 * P * P; e += blockDim.x) {
    const int which = e / (P * P), a = (e / P) % P, c = e % P;
    const double *X1 = (which == 1) ? sY : sQ;
    const double *X2 = (which == 2) ? sQ : sY;
    double s = 0.0;
    for (int r = 0; r < EROWS; ++r) s = fma(X1[r * SQ + a], X2[r * SQ + c], s);
    pp[e] = s;
  }
}

// ------------------------------------------------------------------- gq
template <int P>
__global__ __launch_bounds__(256) void eig_gq_kernel(const double *__restrict__ G, int64_t ldg,
                                                     int64_t strideG, EigWork w, int m, int k,
                                                     int p, double tol, int it, int check_only) {
  constexpr int SQ = P + 4;  // padded LDS row stride (conflict-free B-fragment reads)
  __shared__ __attribute__((aligned(16))) double sQ[EROWS * SQ];
  __shared__ __attribute__((aligned(16))) double sY[EROWS * SQ];
  __shared__ int s_skip;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rep = blockIdx.y, rb = blockIdx.x, nrb = gridDim.x;
  double *small = w.small + (int64_t)rep * small_stride<P>();
  if (tid < 64) {
    const int d = check_converged<P>(w, small + 2 * P * P, w.rpart + (int64_t)rep * nrb * P, w.trace[rep], w.done[rep],
                                     rep, rb, nrb, k, p, tol, it, check_only);
    if (tid == 0) s_skip = d;
  }
  __syncthreads();
  if (s_skip) return;

  const double *Gr = G + (int64_t)rep * strideG;
  const double *Qr = w.Q + (int64_t)rep * m * P;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int row0 = rb * EROWS + wave * 16;
  double acc[4][P / 4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < P / 4; ++b) acc[a][b] = 0.0;

  for (int kc0 = 0; kc0 < m; kc0 += EROWS) {
    for (int e = tid; e < EROWS * P; e += 256) {
      const int r = e / P, c = e % P;
      sQ[r * SQ + c] = (kc0 + r < m) ? Qr[(int64_t)(kc0 + r) * P + c] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < EROWS / 16; ++ks) {
      // wave-uniform: rows past m (m = 130: 3 of 12 waves) and k steps past m
      // only ever added zero products
      if (row0 >= m || kc0 + ks * 16 >= m) continue;
      const int kg = kc0 + ks * 16 + fkc;
      double af[4], bf[P / 4];
#pragma unroll
      for (int fa = 0; fa < 4; ++fa) {
        const int row = row0 + 4 * fa + fi;
        af[fa] = (row < m && kg < m) ? Gr[(int64_t)row * ldg + kg] : 0.0;
      }
#pragma unroll
      for (int fb = 0; fb < P / 4; ++fb) bf[fb] = sQ[(ks * 16 + fkc) * SQ + 4 * fb + fi];
#pragma unroll
      for (int fa = 0; fa < 4; ++fa)
#pragma unroll
        for (int fb = 0; fb < P / 4; ++fb) acc[fa][fb] = mfma4(af[fa], bf[fb], acc[fa][fb]);
    }
    __syncthreads();
  }
  // transpose-reduce, write Y (global + LDS)
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
  double *Yr = w.Y + (int64_t)rep * m * P;
#pragma unroll
  for (int fa = 0; fa < 4; ++fa)
#pragma unroll
    for (int q = 0; q < P / 16; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double v = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int lr = wave * 16 + 4 * fa + oi, col = 16 * q + 4 * blk + oj;
      const int row = rb * EROWS + lr;
      sY[lr * SQ + col] = v;
      if (row < m) Yr[(int64_t)row * P + col] = v;
    }
  // Q rows of this block
  for (int e = tid; e < EROWS * P; e += 256) {
    const int r = e / P, c = e % P, row = rb * EROWS + r;
    sQ[r * SQ + c] = row < m ? Qr[(int64_t)row * P + c] : 0.0;
  }
  __syncthreads();
  // partial Q'Y, Y'Y, Q'Q over this block's rows (fixed order)
  emit_partials<P, SQ>(sQ, sY, w.part + ((int64_t)rep * nrb + rb) * 3 * P * P);
}

// One Horner step of the direct path's Chebyshev filter (the factored path's
// boot_cheb_kernel on an explicit Gram): eig_apply leaves V0 = Q Bm in w.Q and
// S_{d-1} = (a_d/b) G V0 + a_{d-1} V0 in w.Y; step i reads S_{i+1} (Sin, every
// row) and writes S_i = G S_{i+1} / b + a_i V0 (Sout: w.S / w.Y alternately,
// w.Q for S_0, the next basis; a thread reads its V0 entry before it writes
// S_0 over it).  b = theta_p; dead (re-randomised) columns keep V0.  Rows of
// one 64-row block per workgroup.
template <int P>
__global__ __launch_bounds__(256) void eig_cheb_kernel(const double *__restrict__ G, int64_t ldg,
                                                       int64_t strideG, EigWork w, int m, int p,
                                                       const double *Sin, double *Sout, double fai) {
  constexpr int SQ = P + 4;
  __shared__ __attribute__((aligned(16))) double sV[EROWS * SQ];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rep = blockIdx.y, rb = blockIdx.x;
  if (w.done[rep]) return;
  const double *small = w.small + (int64_t)rep * small_stride<P>();
  const double b = small[2 * P * P + p - 1];
  // b <= 0 (a degenerate block): plain power steps
  const double cb = b > 0.0 ? 1.0 / b : 1.0, cv0 = b > 0.0 ? fai : 0.0;
  const double *Gr = G + (int64_t)rep * strideG;
  const double *Vr = Sin + (int64_t)rep * m * P;
  double *So = Sout + (int64_t)rep * m * P;
  const double *V0 = w.Q + (int64_t)rep * m * P;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int row0 = rb * EROWS + wave * 16;
  double acc[4][P / 4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int bb = 0; bb < P / 4; ++bb) acc[a][bb] = 0.0;
  for (int kc0 = 0; kc0 < m; kc0 += EROWS) {
    for (int e = tid; e < EROWS * P; e += 256) {
      const int r = e / P, c = e % P;
      sV[r * SQ + c] = (kc0 + r < m) ? Vr[(int64_t)(kc0 + r) * P + c] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < EROWS / 16; ++ks) {
      // wave-uniform: rows past m (m = 130: 3 of 12 waves) and k steps past m
      // only ever added zero products
      if (row0 >= m || kc0 + ks * 16 >= m) continue;
      const int kg = kc0 + ks * 16 + fkc;
      double af[4], bf[P / 4];
#pragma unroll
      for (int fa = 0; fa < 4; ++fa) {
        const int row = row0 + 4 * fa + fi;
        af[fa] = (row < m && kg < m) ? Gr[(int64_t)row * ldg + kg] : 0.0;
      }
#pragma unroll
      for (int fb = 0; fb < P / 4; ++fb) bf[fb] = sV[(ks * 16 + fkc) * SQ + 4 * fb + fi];
#pragma unroll
      for (int fa = 0; fa < 4; ++fa)
#pragma unroll
        for (int fb = 0; fb < P / 4; ++fb) acc[fa][fb] = mfma4(af[fa], bf[fb], acc[fa][fb]);
    }
    __syncthreads();
  }
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1, blk = (lane >> 2) & 3;
  const int oi = lane >> 4, oj = lane & 3;
#pragma unroll
  for (int fa = 0; fa < 4; ++fa)
#pragma unroll
    for (int q = 0; q < P / 16; ++q) {
      const double a0 = acc[fa][4 * q], a1 = acc[fa][4 * q + 1], a2 = acc[fa][4 * q + 2],
                   a3 = acc[fa][4 * q + 3];
      double k01 = (b1 ? a1 : a0) + __shfl_xor(b1 ? a0 : a1, 4);
      double k23 = (b1 ? a3 : a2) + __shfl_xor(b1 ? a2 : a3, 4);
      const double gv = (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
      const int lr = wave * 16 + 4 * fa + oi, col = 16 * q + 4 * blk + oj;
      const int row = rb * EROWS + lr;
      if (row < m) {
        const bool dead = small[2 * P * P + P + col] != 0.0;
        const double v0 = V0[(int64_t)row * P + col];
        double sn = dead ? v0 : fma(cb, gv, cv0 * v0);
        if (col >= p) sn = 0.0;
        So[(int64_t)row * P + col] = sn;
      }
    }
}

// ---------------------------------------------------------------- small
// One wave per replicate, all p x p algebra in LDS, written for latency:
// Cholesky + triangular inverse in registers (every solve becomes a parallel
// matrix product), and a parallel cyclic Jacobi whose round is ONE phase: with
// the pairs of a round disjoint, every 2x2 block (pair s1 rows, pair s2 cols)
// is rotated J1' B J2 by one lane.
template <int P>
struct SmallLds {
  static constexpr int S = P + 1;
  // four P x (P+1) regions, reused as the matrices' lifetimes end (the
  // kernel is latency-bound and one wave per workgroup, so the LDS image sets
  // the occupancy: 4 regions = 9.2 KB at P = 16, 16 waves per CU, where the 6
  // of the unshared layout held it to 11):
  //   R1  H~ (Q'Y, then Li Q'Y Li', Jacobi)      -> W = V[:, perm] -> Y'Y A -> Bm
  //   R2  Q'Q -> Li Q'Y -> V (Jacobi vectors)    -> A = Li' W
  //   R3  Y'Y                                    -> Z'Z = A' Y'Y A
  //   R4  Li = chol(Q'Q)^-1                      -> chol(Z'Z)^-1
  double R1[P * S], R2[P * S], R3[P * S], R4[P * S];
  double rc[P / 2], rs[P / 2];
  int ra[P / 2], rb[P / 2], perm[P];
  int dead[P];
};

// LDS hand-off inside the ONE wave that runs the p x p algebra (eig_small's
// single-wave workgroups; in eig_fused the other waves wait at a barrier):
// a wave's LDS accesses complete in issue order, so waiting for its own
// outstanding ones (and fencing the compiler) is the whole synchronisation.
DFM_DEV void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// reciprocal and reciprocal square root: hardware seed + two Newton steps
// (full double precision to within an ulp or so; the Jacobi rotations only
// need c^2 + s^2 = 1 to rounding, which c = rsq(1 + t^2), s = t c keep)
DFM_DEV double nr_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}
DFM_DEV double nr_rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  return y * fma(-hx * y, y, 1.5);
}

DFM_DEV double rl64(double x, int l) {   // lane l's x (l wave-uniform: a compile-time constant in unrolled loops)
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Li = Lo^-1 of the lower Cholesky factor M = Lo Lo' (p x p): lane i < P
// holds row i in registers.  Right-looking factorisation (step j: pivot by
// readlane, column j scaled by one reciprocal square root, the trailing rows
// updated), then lane c forward-substitutes column c of the inverse.  M is
// dead once its rows are in registers, so it holds the columns of Lo as they
// are formed (column j in M's row j): every lane reads the values it needs
// from there as same-address LDS broadcasts, one instruction per double
// where a readlane pair plus its hazard wait took three or four (this
// wave's own writes, in LDS order).  Tiny pivots -> dead (unit diagonal,
// zero column, zero row of Li).
template <int P>
DFM_DEV void wave_chol_inv(double *M, double *Li, int *dead, int p) {
  constexpr int S = P + 1;
  const int lane = threadIdx.x & 63;
  double mx = 0.0;
  for (int j = lane; j < p; j += 64) mx = fmax(mx, fabs(M[j * S + j]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  const double thresh = 1e-22 * mx;
  double r[P];
#pragma unroll
  for (int k = 0; k < P; ++k) r[k] = (lane < p && k < p) ? M[min(lane, P - 1) * S + k] : 0.0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // M's rows are in registers before M is overwritten
  double inv_l = 1.0;
  int dead_l = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (j < p) {
      const double sj = rl64(r[j], j);
      const bool dd = !(sj > thresh);
      const double inv = dd ? 1.0 : rsqrt(sj);
      double lij = (lane > j && lane < p) ? (dd ? 0.0 : r[j] * inv) : 0.0;
      if (lane == j) { lij = dd ? 1.0 : sj * inv; inv_l = inv; dead_l = dd; }
      r[j] = lij;
      if (lane < P) M[j * S + lane] = lij;          // column j of Lo
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = j + 1; k < P; ++k) r[k] = r[k] - lij * M[j * S + k];
    }
  }
  if (lane < P) dead[lane] = lane < p ? dead_l : 0;
  if (lane < P) M[(P - 1) * S + lane] = inv_l;   // 1 / Lo[i][i], over column P-1 of Lo (the substitution never reads it)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  double x[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    double sacc = (i == lane) ? 1.0 : 0.0;
#pragma unroll
    for (int q = 0; q < i; ++q) sacc = sacc - M[q * S + i] * x[q];
    x[i] = (i < p) ? sacc * M[(P - 1) * S + i] : 0.0;
  }
  const bool dl = lane < p;
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const bool di = dead[i] != 0;
    if (lane < P) Li[i * S + lane] = (i < p && dl && !di) ? x[i] : 0.0;
  }
  wave_lds_sync();
}

// C = op(A) op(B) for P x P LDS matrices (TA/TB transpose flags; C distinct
// from A and B); padded entries are zero so the full P x P product is exact.
// One wave of v_mfma_f64_16x16x4 per 16 x 16 output tile: A operand = row
// (lane & 15), k (lane >> 4); B operand = k (lane >> 4), column (lane & 15);
// accumulator register g = row 4g + (lane >> 4), column (lane & 15).
template <int P, bool TA, bool TB>
DFM_DEV void wave_mm(const double *A, const double *B, double *C) {
  constexpr int S = P + 1, NT = P / 16;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < NT; ++rt)
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      const int i = 16 * rt + li, j = 16 * ct + li;
      dv4 acc = dv4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < P / 4; ++kk) {
        const int q = 4 * kk + lk;
        acc = mfma16(TA ? A[q * S + i] : A[i * S + q], TB ? B[j * S + q] : B[q * S + j], acc);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) C[(16 * rt + 4 * g + lk) * S + 16 * ct + li] = acc[g];
    }
  wave_lds_sync();
}

template <int P>
DFM_DEV void wave_sym(double *M) {
  constexpr int S = P + 1;
  for (int e = threadIdx.x & 63; e < P * P; e += 64) {
    const int i = e / P, j = e % P;
    if (i < j) { const double v = 0.5 * (M[i * S + j] + M[j * S + i]); M[i * S + j] = v; M[j * S + i] = v; }
  }
  wave_lds_sync();
}

// The Rayleigh-Ritz step on ONE wave (any wave of the workgroup): in, R1 =
// Q'Y, R3 = Y'Y, R2 = Q'Q (entries >= p zero; with SMALL_CHOL1_DONE in
// jsweeps, R4 = chol(Q'Q)^-1 and sm.dead already formed instead); out, A in R2 and Bm in R1
// (also copied to ab[0, P^2) and ab[P^2, 2 P^2) when ab is given) and the
// small record's tail: theta[P], then the dead flags[P].
template <int P>
DFM_DEV void small_rr(SmallLds<P> &sm, EigWork &w, int rep, int p, int jsweeps, double *ab, double *tail) {
  constexpr int S = P + 1;
  double *const Hq = sm.R1, *const Yq = sm.R3;   // region map: SmallLds
  // opaque lane and p: called inside eig_fused's iteration loop, whose
  // optimiser would otherwise hoist this step's lane-derived indices out of
  // the loop and keep them live through every other phase
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  asm volatile("" : "+s"(p));
  SMALL_STAMP(1);
  if (!(jsweeps & SMALL_STAGE_B)) {
  wave_sym<P>(Hq);
  // 2. Q'Q = L L',  Li = L^-1;  H~ = Li (Q'Y) Li'
  if (!(jsweeps & SMALL_CHOL1_DONE)) wave_chol_inv<P>(sm.R2, sm.R4, sm.dead, p);
  SMALL_STAMP(2);
  SMALL_STAMP(3);
  wave_mm<P, false, false>(sm.R4, Hq, sm.R2);   // Q'Q is dead once Li is formed
  wave_mm<P, false, true>(sm.R2, sm.R4, Hq);
  wave_sym<P>(Hq);
  SMALL_STAMP(4);
  for (int e = lane; e < P * S; e += 64) sm.R2[e] = ((e / S) == (e % S)) ? 1.0 : 0.0;   // V
  wave_lds_sync();
  double *const V = sm.R2;
  // 3. parallel cyclic Jacobi (circle-method pairs; index p is a dummy when p is odd)
  const int n = p + (p & 1), h = n / 2;
  // A pair is rotated only while |h_ab| > 4 eps sqrt(|h_aa h_bb|) (the classic
  // Jacobi threshold: a smaller off-diagonal moves the eigenvalues by
  // O(eps^2)); the sweep loop ends at the first sweep that rotates nothing.
  // (A Frobenius off-diagonal test sits at the rounding floor for these
  // matrices and ran every sweep to the cap.)
  // every lane's 2x2 blocks and V entries are the same in every round: their
  // (s1, s2) and (k, sI) indices are computed once here, and the circle-method
  // positions advance by a wrapped increment (no integer division per round)
  constexpr int NHB = ((P / 2) * (P / 2) + 63) / 64, NVE = (P * (P / 2) + 63) / 64;
  int hb1[NHB], hb2[NHB], vk[NVE], vs[NVE];
#pragma unroll
  for (int u = 0; u < NHB; ++u) {
    const int e = lane + 64 * u;
    hb1[u] = (h > 0 && e < h * h) ? e / h : -1;
    hb2[u] = (h > 0 && e < h * h) ? e % h : 0;
  }
#pragma unroll
  for (int u = 0; u < NVE; ++u) {
    const int e = lane + 64 * u;
    vk[u] = (h > 0 && e < p * h) ? e / h : -1;
    vs[u] = (h > 0 && e < p * h) ? e % h : 0;
  }
  const int n1 = n - 1, pa = lane, pb = n - 1 - lane;
  for (int sweep = 0; sweep < (jsweeps & 0xff); ++sweep) {
    bool rotated = false;
    int xa = pa - 1, xb = pb - 1;   // position - 1 + r, wrapped into [0, n - 1)
    for (int r = 0; r < n1; ++r, ++xa, ++xb) {
      if (xa >= n1) xa -= n1;
      if (xb >= n1) xb -= n1;
      bool rot = false;
      if (lane < h) {
        int a = pa == 0 ? 0 : 1 + xa;
        int b = pb == 0 ? 0 : 1 + xb;
        if (a > b) { const int t = a; a = b; b = t; }
        double c = 1.0, sn = 0.0;
        if (b < p) {
          const double hab = Hq[a * S + b], haa = Hq[a * S + a], hbb = Hq[b * S + b];
          // |h_ab| > 4 eps sqrt(|h_aa h_bb|), squared; the rotation from the
          // hardware reciprocal / reciprocal-square-root seeds plus Newton
          // steps (the round's critical path: three divisions and three
          // square roots in correctly rounded form)
          if (fabs(hab) > 1e-300 && hab * hab > 7.921e-31 * fabs(haa * hbb)) {
            const double zeta = (hbb - haa) * nr_rcp(2.0 * hab), az = fabs(zeta);
            const double y = fma(zeta, zeta, 1.0);
            const double rt = az > 1e150 ? az : y * nr_rsq(y);   // sqrt(1 + zeta^2)
            const double t = (zeta >= 0.0 ? 1.0 : -1.0) * nr_rcp(az + rt);
            c = nr_rsq(fma(t, t, 1.0));
            sn = t * c;
            rot = true;
          }
        }
        sm.ra[lane] = a; sm.rb[lane] = b; sm.rc[lane] = c; sm.rs[lane] = sn;
      }
      const bool any = __any(rot);
      rotated = rotated || any;
      if (!any) continue;   // wave-uniform: nothing to apply this round
      wave_lds_sync();
      // H <- J' H J by 2x2 blocks; V <- V J
#pragma unroll
      for (int u = 0; u < NHB; ++u) {
        if (hb1[u] < 0) continue;
        const int s1 = hb1[u], s2 = hb2[u];
        const int i0 = sm.ra[s1], i1 = sm.rb[s1], j0 = sm.ra[s2], j1 = sm.rb[s2];
        const double c1 = sm.rc[s1], n1 = sm.rs[s1], c2 = sm.rc[s2], n2 = sm.rs[s2];
        const double b00 = Hq[i0 * S + j0], b01 = Hq[i0 * S + j1];
        const double b10 = Hq[i1 * S + j0], b11 = Hq[i1 * S + j1];
        const double t00 = c1 * b00 - n1 * b10, t01 = c1 * b01 - n1 * b11;
        const double t10 = n1 * b00 + c1 * b10, t11 = n1 * b01 + c1 * b11;
        Hq[i0 * S + j0] = c2 * t00 - n2 * t01;
        Hq[i0 * S + j1] = n2 * t00 + c2 * t01;
        Hq[i1 * S + j0] = c2 * t10 - n2 * t11;
        Hq[i1 * S + j1] = n2 * t10 + c2 * t11;
      }
#pragma unroll
      for (int u = 0; u < NVE; ++u) {
        if (vk[u] < 0) continue;
        const int k = vk[u], sI = vs[u];
        const int a = sm.ra[sI], b = sm.rb[sI];
        const double c = sm.rc[sI], sn = sm.rs[sI];
        const double va = V[k * S + a], vb = V[k * S + b];
        V[k * S + a] = c * va - sn * vb;
        V[k * S + b] = sn * va + c * vb;
      }
      wave_lds_sync();
    }
    if (w.dbg && rep == 0 && lane == 0) w.dbg[15] = sweep + 1;
    if (!rotated) break;
  }
  SMALL_STAMP(5);
  // 4. sort descending (stable): lane j computes the rank of diagonal j
  for (int j = lane; j < p; j += 64) {
    const double v = Hq[j * S + j];
    int rank = 0;
    for (int i = 0; i < p; ++i) {
      const double u = Hq[i * S + i];
      rank += (u > v || (u == v && i < j)) ? 1 : 0;
    }
    sm.perm[rank] = j;
  }
  wave_lds_sync();
  for (int j = lane; j < P; j += 64) tail[j] = j < p ? Hq[sm.perm[j] * S + sm.perm[j]] : 0.0;
  wave_lds_sync();   // the Ritz values are read from R1 before W overwrites it
  // W = V[:, perm] (zero-padded), into R1
  double *const W = sm.R1;
  for (int e = lane; e < P * P; e += 64) {
    const int i = e / P, c = e % P;
    W[i * S + c] = (i < p && c < p) ? V[i * S + sm.perm[c]] : 0.0;
  }
  wave_lds_sync();
  SMALL_STAMP(6);
  // 5. A = L^-T Vs = Li' W ;  Z'Z = A' (Y'Y) A ;  L2 = chol ;  Bm = A L2^-T
  double *const A = sm.R2;
  wave_mm<P, true, false>(sm.R4, W, A);       // V is dead once permuted
  wave_mm<P, false, false>(Yq, A, sm.R1);     // Y'Y A (W is dead)
  wave_mm<P, true, false>(A, sm.R1, sm.R3);   // Z'Z (Y'Y is dead)
  wave_sym<P>(sm.R3);
  SMALL_STAMP(7);
  }
  if (jsweeps & SMALL_STAGE_A) return;
  double *const A = sm.R2;
  wave_chol_inv<P>(sm.R3, sm.R4, sm.dead, p);
  SMALL_STAMP(8);
  SMALL_STAMP(9);
  wave_mm<P, false, true>(A, sm.R4, sm.R1);   // Bm = A Li'
  if (ab)
    for (int e = lane; e < P * P; e += 64) {
      const int a = e / P, c = e % P;
      ab[e] = (a < p && c < p) ? A[a * S + c] : 0.0;
      ab[P * P + e] = (a < p && c < p) ? sm.R1[a * S + c] : 0.0;
    }
  for (int j = lane; j < P; j += 64) tail[P + j] = (j < p && sm.dead[j]) ? 1.0 : 0.0;
  wave_lds_sync();
  SMALL_STAMP(10);
}

template <int P>
__global__ __launch_bounds__(64) void eig_small_kernel(EigWork w, int p, int nrb, int jsweeps) {
  constexpr int S = P + 1;
  __shared__ SmallLds<P> sm;
  const int lane = threadIdx.x, rep = blockIdx.x;
  if (w.done[rep]) return;
  SMALL_STAMP(0);
  // 1. sum partials in fixed order (entries >= p are zero: Q columns >= p are zero)
  const double *pp = w.part + (int64_t)rep * nrb * 3 * P * P;
  constexpr int PER = 3 * P * P / 64;   // entries per lane (12 for P = 16)
  {
    double acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = 0.0;
    for (int r = 0; r < nrb; ++r) {   // all PER loads of a block issue together
      double v[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) v[u] = pp[(int64_t)r * 3 * P * P + lane + 64 * u];
#pragma unroll
      for (int u = 0; u < PER; ++u) acc[u] += v[u];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = lane + 64 * u;
      const int which = e / (P * P), a = (e / P) % P, c = e % P;
      double *M = which == 0 ? sm.R1 : (which == 1 ? sm.R3 : sm.R2);
      M[a * S + c] = acc[u];
    }
  }
  wave_lds_sync();
  double *small = w.small + (int64_t)rep * small_stride<P>();
  small_rr<P>(sm, w, rep, p, jsweeps, small, small + 2 * P * P);
}

// ---------------------------------------------------------------- apply
template <int P>
// cheb = 1: the next basis is formed by eig_cheb_kernel; here V = Y Bm goes
// to w.Y and Q Bm to w.Q (both over this block's own rows, already staged).
__global__ __launch_bounds__(256) void eig_apply_kernel(EigWork w, int m, int p, int k, int it,
                                                        uint64_t seed, int64_t rep0, int cheb, double fa1,
                                                        double fa0) {
  constexpr int SQ = P + 1;
  __shared__ double sQ[EROWS * SQ], sY[EROWS * SQ], sW[EROWS * P];
  __shared__ double sA[P * P], sB[P * P], sT[2 * P];
  const int tid = threadIdx.x, rep = blockIdx.y, rb = blockIdx.x, nrb = gridDim.x;
  if (w.done[rep]) return;
  const double *small = w.small + (int64_t)rep * small_stride<P>();
  double *Qr = w.Q + (int64_t)rep * m * P;
  double *Yr = w.Y + (int64_t)rep * m * P;
  double *Ur = w.U + (int64_t)rep * m * P;
  for (int e = tid; e < EROWS * P; e += 256) {
    const int r = e / P, c = e % P, row = rb * EROWS + r;
    sQ[r * SQ + c] = row < m ? Qr[(int64_t)row * P + c] : 0.0;
    sY[r * SQ + c] = row < m ? Yr[(int64_t)row * P + c] : 0.0;
  }
  for (int e = tid; e < P * P; e += 256) { sA[e] = small[e]; sB[e] = small[P * P + e]; }
  for (int e = tid; e < 2 * P; e += 256) sT[e] = small[2 * P * P + e];
  __syncthreads();
  for (int e = tid; e < EROWS * P; e += 256) {
    const int r = e / P, c = e % P, row = rb * EROWS + r;
    double u = 0.0, ya = 0.0, qn = 0.0, qb = 0.0;
    for (int a = 0; a < p; ++a) {
      u = fma(sQ[r * SQ + a], sA[a * P + c], u);
      ya = fma(sY[r * SQ + a], sA[a * P + c], ya);
      qn = fma(sY[r * SQ + a], sB[a * P + c], qn);
      if (cheb) qb = fma(sQ[r * SQ + a], sB[a * P + c], qb);
    }
    if (c < p && sT[P + c] != 0.0) qn = hash_unit(seed, row, 1000003ull * (it + 1) + c);
    if (c >= p) { qn = 0.0; qb = 0.0; }
    if (c < k) { const double wv = ya - sT[c] * u; sW[r * P + c] = row < m ? wv * wv : 0.0; }
    if (row < m) {
      Ur[(int64_t)row * P + c] = u;
      if (cheb) {   // the filter's first Horner term S = (a_d/b) V + a_{d-1} Q Bm, and V0 = Q Bm (dead: V)
        const double bch = sT[p - 1];
        const bool dead = c < p && sT[P + c] != 0.0;
        const double sv = dead ? qn : (bch > 0.0 ? fma(fa1 / bch, qn, fa0 * qb) : qn);
        Yr[(int64_t)row * P + c] = c >= p ? 0.0 : sv;
        Qr[(int64_t)row * P + c] = c >= p ? 0.0 : (dead ? qn : qb);
      } else {
        Qr[(int64_t)row * P + c] = qn;
      }
    }
  }
  __syncthreads();
  if (tid < k) {
    double s = 0.0;
    for (int r = 0; r < EROWS; ++r) s += sW[r * P + tid];
    w.rpart[((int64_t)rep * nrb + rb) * P + tid] = s;
  }
}

// ---------------------------------------------------------------- final
// lam: nb x k, Uk: nb x m x k (row-major), status: nb (0 ok, 1 not converged)
// Ur: the replicate's Ritz vectors (m x P), theta its Ritz values; 256 threads.
template <int P>
DFM_DEV void eig_final_body(const double *Ur, const double *theta, int done, int rep, int m, int k,
                            double *__restrict__ lam, double *__restrict__ Uk, int *__restrict__ status) {
  if (!Uk) {   // eigenvalue-only statistics: no vectors wanted, no pass over U
    if (threadIdx.x < k) lam[(int64_t)rep * k + threadIdx.x] = theta[threadIdx.x];
    if (threadIdx.x == 0) status[rep] = done ? 0 : 1;
    return;
  }
  // one pass over U: each thread keeps the running max |U[r][j]| (first row
  // on ties) of its rows for every column j, then a shuffle reduction per
  // wave and a fixed-order combine of the four waves (smaller row index wins
  // ties: the same pick as a serial scan)
  __shared__ double sv[P][4];
  __shared__ int si[P][4];
  __shared__ double ssign[P];
  const int tid = threadIdx.x, wv = tid >> 6;
  double best[P];
  int bi[P];
#pragma unroll
  for (int j = 0; j < P; ++j) { best[j] = -1.0; bi[j] = 0; }
  for (int r = tid; r < m; r += 256) {
    double v[P];
#pragma unroll
    for (int j = 0; j < P; j += 2) {
      const double2 x = *reinterpret_cast<const double2 *>(Ur + (int64_t)r * P + j);
      v[j] = x.x; v[j + 1] = x.y;
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const double a = fabs(v[j]);
      if (j < k && a > best[j]) { best[j] = a; bi[j] = r; }
    }
  }
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (j >= k) continue;
    double a = best[j];
    int ai = bi[j];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double b = __shfl_xor(a, o);
      const int bj = __shfl_xor(ai, o);
      if (b > a || (b == a && bj < ai)) { a = b; ai = bj; }
    }
    if ((tid & 63) == 0) { sv[j][wv] = a; si[j][wv] = ai; }
  }
  __syncthreads();
  if (tid < k) {
    double a = sv[tid][0];
    int ai = si[tid][0];
    for (int q = 1; q < 4; ++q)
      if (sv[tid][q] > a || (sv[tid][q] == a && si[tid][q] < ai)) { a = sv[tid][q]; ai = si[tid][q]; }
    si[tid][0] = ai;
  }
  __syncthreads();
  if (tid < k) ssign[tid] = Ur[(int64_t)si[tid][0] * P + tid] < 0.0 ? -1.0 : 1.0;
  __syncthreads();
  if (tid < k) lam[(int64_t)rep * k + tid] = theta[tid];
  if (tid == 0) status[rep] = done ? 0 : 1;
  for (int64_t e = tid; e < (int64_t)m * k; e += 256) {
    const int r = (int)(e / k), j = (int)(e % k);
    Uk[(int64_t)rep * m * k + e] = ssign[j] * Ur[(int64_t)r * P + j];
  }
}

DFM_DEV void count_iters_body(const int *__restrict__ active, int last_gemm, int last_cheb, int nb, long long *cnt,
                              int cp0, int cp1);
template <int P>
__global__ __launch_bounds__(256) void eig_final_kernel(EigWork w, int m, int k, double *__restrict__ lam,
                                                        double *__restrict__ Uk, int *__restrict__ status,
                                                        double *__restrict__ trace_out, long long *cnt = nullptr,
                                                        int last_gemm = -1, int last_cheb = -1, int cp0 = 0,
                                                        int cp1 = 0) {
  const int rep = blockIdx.x;
  if (trace_out && threadIdx.x == 0) trace_out[rep] = w.trace[rep];   // (the caller's copy of trace(G))
  // the factored run's iteration / product counts (count_iters_kernel's work, one launch fewer)
  if (cnt && rep == 0 && threadIdx.x == 0) count_iters_body(w.active, last_gemm, last_cheb, gridDim.x, cnt, cp0, cp1);
  eig_final_body<P>(w.U + (int64_t)rep * m * P, w.small + (int64_t)rep * small_stride<P>() + 2 * P * P, w.done[rep],
                    rep, m, k, lam, Uk, status);
}

// ------------------------------------------------------------- host driver
size_t eig_workspace_bytes(int m, int nb, int P, int maxit) {
  const int nrb = (m + EROWS - 1) / EROWS;
  size_t s = 0;
  s += 4 * (size_t)nb * m * P * 8;               // Q, Y, U, S
  s += (size_t)nb * nrb * 3 * P * P * 8;         // part
  s += (size_t)nb * nrb * P * 8;                 // rpart
  s += (size_t)nb * (2 * P * P + 4 * P) * 8;     // small
  s += (size_t)nb * 8;                           // trace
  s += (size_t)(2 * nb + maxit + 2) * 4 + 256;   // done, iters, active
  return s;
}

static EigWork carve(char *base, int m, int nb, int P, int maxit) {
  const int nrb = (m + EROWS - 1) / EROWS;
  EigWork w;
  auto take = [&](size_t bytes) { char *p = base; base += (bytes + 255) & ~size_t(255); return p; };
  w.Q = (double *)take((size_t)nb * m * P * 8);
  w.Y = (double *)take((size_t)nb * m * P * 8);
  w.U = (double *)take((size_t)nb * m * P * 8);
  w.S = (double *)take((size_t)nb * m * P * 8);
  w.part = (double *)take((size_t)nb * nrb * 3 * P * P * 8);
  w.rpart = (double *)take((size_t)nb * nrb * P * 8);
  w.small = (double *)take((size_t)nb * (2 * P * P + 4 * P) * 8);
  w.trace = (double *)take((size_t)nb * 8);
  w.done = (int *)take((size_t)nb * 4);
  w.iters = (int *)take((size_t)nb * 4);
  w.active = (int *)take((size_t)(maxit + 2) * 4);
  w.dbg = nullptr;
  w.subspace = 0;
  w.no_vectors = 0;
  return w;
}

// per-replicate Rayleigh-Ritz steps of the last solve carved from ws (diagnostic stat)
const int *eig_iters_ptr(char *ws, int m, int nb, int P, int maxit) { return carve(ws, m, nb, P, maxit).iters; }

size_t eig_workspace_bytes_padded(int m, int nb, int P, int maxit) {
  return eig_workspace_bytes(m, nb, P, maxit) + 16 * 256;
}

typedef void (*timer_fn)(void *ctx, int cls, int begin);
// Jacobi sweeps per Rayleigh-Ritz step.  The projected matrix need not be
// diagonalised exactly at every outer iteration: the next iteration starts
// from the (nearly) rotated basis, so the inner sweeps accumulate across outer
// iterations, and the residual test of check_converged includes any leftover
// off-diagonal coupling.
constexpr int kJacobiSweeps = 2;
// Jacobi sweeps per Rayleigh-Ritz step of the fused solver: ONE (C2: the
// same 4.99 steps per replicate as two sweeps, 458k vs 423k rep/s — the
// inner sweeps accumulate across outer steps).  DFM_EIG_JSWEEPS overrides.
static int fused_sweeps() {
  static const int v = [] {
    const char *a = getenv("DFM_EIG_JSWEEPS");
    return a ? std::max(1, std::min(8, atoi(a))) : 1;
  }();
  return v;
}
thread_local int g_last_iters = 0;   // iterations run by the last eig_run / eig_run_factored (host stat)
// replicate-iterations of the last run's dominant product (G.Q in eig_gq, or
// the H.Z GEMM in the factored solver) that still had an unconverged
// replicate: the algorithmic work the roofline figure is priced on.
thread_local int64_t g_last_rep_iters = 0;
thread_local int64_t g_last_gemm_products = 0;   // replicate-products of the last run: H . Z (factored, both Chebyshev GEMMs) or G S (fused direct solver)

// Sum of the unconverged-replicate counts seen by the products of iterations
// 0..last (shift = 1: the product of iteration it runs before that
// iteration's convergence check, so it sees active[it-1]; active[-1] = nb).
// Device-side form of count_rep_iters for the factored run: adds the
// replicate-iterations (GEMM launches 0..last_gemm, shift 1) and the GEMM
// replicate-products (those plus the Chebyshev GEMMs 0..last_cheb, shift 0)
// to cnt[0], cnt[1] — no host synchronisation after the eigen loop.
DFM_DEV void count_iters_body(const int *__restrict__ active, int last_gemm, int last_cheb, int nb, long long *cnt,
                              int cp0, int cp1) {
  long long a = 0, b = 0;
  for (int it = 0; it <= last_gemm; ++it) a += it - 1 < 0 ? nb : active[it - 1];
  // Chebyshev products: cp0 after the first Rayleigh-Ritz step, cp1 after the others
  for (int it = 0; it <= last_cheb; ++it) b += (long long)active[it] * (it == 0 ? cp0 : cp1);
  // device-scope atomics: a model's two bootstrap lanes count into one context
  atomicAdd(reinterpret_cast<unsigned long long *>(cnt), (unsigned long long)a);
  atomicAdd(reinterpret_cast<unsigned long long *>(cnt + 1), (unsigned long long)(a + b));
}
__global__ void count_iters_kernel(const int *__restrict__ active, int last_gemm, int last_cheb, int nb,
                                   long long *cnt, int cp0, int cp1) {
  if (threadIdx.x == 0) count_iters_body(active, last_gemm, last_cheb, nb, cnt, cp0, cp1);
}
static int64_t count_rep_iters(const int *active_dev, int last, int shift, int nb, hipStream_t st) {
  if (last < 0) return 0;
  std::vector<int> a((size_t)last + 2, 0);
  hipMemcpyAsync(a.data(), active_dev, a.size() * 4, hipMemcpyDeviceToHost, st);
  hipStreamSynchronize(st);
  int64_t s = 0;
  for (int it = 0; it <= last; ++it) s += (it - shift < 0) ? nb : a[it - shift];
  return s;
}

constexpr int kChebDMax = 8, kChebDirectStrict = 4;
static void shifted_cheb(int d, double *a);

// ---------------------------------------------------------------- fused
// The whole direct solve of ONE replicate in ONE workgroup (4 waves), P = 16
// and m <= 16 NGW: the basis Q and the product Y stay in LDS for the whole
// solve (2 x m x 16 doubles: 37 KB at m = 130, three workgroups per CU), G
// streams from L2 / MALL once per product.  Each iteration runs the same
// algebra as the kernel sequence gq -> small -> apply -> cheb:
//   check    wave 0: iteration it-1's residuals (check_converged), retire / count
//   Y = G Q  v_mfma_f64_4x4x4_4b; 4-row groups dealt round-robin to the waves
//   Q'Y, Y'Y, Q'Q   waves 0..2, one product each over all m rows
//   small_rr wave 0 (the other waves wait at the barrier)
//   apply    U = Q A -> global (eig_final reads it), residual sums, V0 = Q Bm
//            and the filter's first Horner term S = (a_d/b) Y Bm + a_{d-1} V0
//   cheb     dg - 1 times S <- G S / b + a_i V0; S_0 (into Q) is the next basis
// The multi-kernel path's launch chain, its host polls and its per-row-block
// partial records are gone: a replicate leaves the loop the moment it
// converges, the others keep iterating.  Sums run in a fixed order.
struct ChebCo { double c2[kChebDMax + 1], c4[kChebDMax + 1]; };

// LDS image of an m x 16 block, row r, column c: the 4-column block is
// XOR-swizzled by (r >> 1) & 3, so the MFMA operand reads (rows 4 (lane >> 4)
// + ((lane >> 2) & 3), columns 4 fb + (lane & 3)) hit 8 distinct 8-bank
// groups per half-wave.
// x, opaque to the optimiser: lane-derived offsets recomputed per phase
// instead of hoisted out of the iteration loop (every phase's hoisted
// offsets live at once otherwise — hundreds of VGPRs, spilled)
DFM_DEV int fz_opaque(int x) { asm volatile("" : "+v"(x)); return x; }

DFM_DEV int fz_ix(int r, int c) { return (r << 4) | ((((c >> 2) ^ ((r >> 1) & 3)) << 2) | (c & 3)); }

// Transpose-reduce of the four v_mfma_f64_4x4x4_4b blocks of accumulators
// a[fb] (column block fb): the lane gets the 4 x 16 result's element
// (row lane >> 4, column lane & 15).
DFM_DEV double mm4_fold(const double (&a)[4], int lane) {
  const int b1 = (lane >> 2) & 1, b2 = (lane >> 3) & 1;
  const double k01 = (b1 ? a[1] : a[0]) + __shfl_xor(b1 ? a[0] : a[1], 4);
  const double k23 = (b1 ? a[3] : a[2]) + __shfl_xor(b1 ? a[2] : a[3], 4);
  return (b2 ? k23 : k01) + __shfl_xor(b2 ? k01 : k23, 8);
}

// acc[q] = rows of 4-row group g = wave + NW q (NW waves share the rows) of G S (G: m x m in global, S:
// the LDS image, rows m..mpad-1 zero).  Lane: row 4 g + (lane & 3), k index
// k0 + 4 (lane >> 4) + ((lane >> 2) & 3) — a G row's 16 k values per chunk are
// one 128-byte line.  G comes from L2 / MALL (a batch's Grams outgrow the
// L2): a register ring holds FZ_DEPTH chunks in flight (3; 2 when a wave
// owns more than 9 groups — registers), the loads of chunk c + FZ_DEPTH - 1
// issue before chunk c's MFMAs.
template <int NGW, int NW, int FZ_DEPTH = (NGW > 9 ? 2 : 3)>
DFM_DEV void fz_gemm(const double *__restrict__ Gr, int64_t ldg, int m, int ng, const double *S, int wave, int lane,
                     double (&acc)[NGW][4]) {
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  const int ld = (int)ldg;   // m <= 256: element offsets fit 32 bits (SGPR base + VGPR offset loads)
  const int nch = (m + 15) >> 4;
#pragma unroll
  for (int q = 0; q < NGW; ++q)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[q][b] = 0.0;
  unsigned off[NGW];   // the lane's G row offset + k of chunk 0
#pragma unroll
  for (int q = 0; q < NGW; ++q) off[q] = (unsigned)((4 * (wave + NW * q) + fi) * ld + fkc);
  double ring[FZ_DEPTH][NGW];
  auto load = [&](int c, double (&dst)[NGW]) {
    const int kg = 16 * c + fkc;
#pragma unroll
    for (int q = 0; q < NGW; ++q) {
      const int g = wave + NW * q, row = 4 * g + fi;
      dst[q] = (g < ng && row < m && kg < m) ? Gr[off[q] + 16 * c] : 0.0;
    }
  };
#pragma unroll
  for (int s = 0; s < FZ_DEPTH - 1; ++s) load(s, ring[s]);
#pragma unroll 1
  for (int c0 = 0; c0 < nch; c0 += FZ_DEPTH) {
#pragma unroll
    for (int s = 0; s < FZ_DEPTH; ++s) {
      const int c = c0 + s;
      load(c + FZ_DEPTH - 1, ring[(s + FZ_DEPTH - 1) % FZ_DEPTH]);
      if (c < nch) {   // wave-uniform
        double bf[4];
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) bf[fb] = S[fz_ix(16 * c + fkc, 4 * fb + fi)];
#pragma unroll
        for (int q = 0; q < NGW; ++q) {
          if (wave + NW * q >= ng) continue;   // wave-uniform
#pragma unroll
          for (int fb = 0; fb < 4; ++fb) acc[q][fb] = mfma4(ring[s][q], bf[fb], acc[q][fb]);
        }
      }
    }
  }
}

// Out (P x P, stride P + 1) = X1' X2 over the mpad rows of two LDS images,
// on ONE wave: output 4-row groups g = 0..3 of v_mfma_f64_4x4x4_4b.
DFM_DEV void fz_xtx(const double *X1, const double *X2, double *Out, int mpad, int lane) {
  constexpr int S = 17;
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3);
  double a4[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int b = 0; b < 4; ++b) a4[g][b] = 0.0;
#pragma unroll 1
  for (int k0 = 0; k0 < mpad; k0 += 16) {
    const int kr = k0 + fkc;
    double af[4], bf[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) af[g] = X1[fz_ix(kr, 4 * g + fi)];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) bf[fb] = X2[fz_ix(kr, 4 * fb + fi)];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int fb = 0; fb < 4; ++fb) a4[g][fb] = mfma4(af[g], bf[fb], a4[g][fb]);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const double v = mm4_fold(a4[g], lane);
    Out[(4 * g + (lane >> 4)) * S + (lane & 15)] = v;
  }
}

// OVL: Y = G Q on waves 0..2 (NG3 groups each) while wave 3 forms Q'Q and
// its inverse Cholesky factor — the Rayleigh-Ritz step's first factorisation
// leaves the critical path.
template <int NGW, int NG3, bool OVL>
__global__ __launch_bounds__(256, NGW <= 9 ? 2 : 1) void eig_fused_kernel(
    const double *__restrict__ G, int64_t ldg, int64_t strideG, EigWork w, int m, int k, int p, double tol,
    int maxit, const double *__restrict__ warm, int kw, uint64_t seed, int warm_strict, int jsweeps, ChebCo cc,
    double *__restrict__ lam, double *__restrict__ Uk, int *__restrict__ status, long long *__restrict__ prof) {
  constexpr int P = 16, S = P + 1;
  __shared__ SmallLds<P> sm;
  __shared__ double s_tail[4 * P];   // the small record's tail: theta[P], dead[P], residual history 2 x P
  __shared__ double s_rw[4][P];      // per-wave residual sums of one apply
  __shared__ double s_res[P];        // their fixed-order total (check_converged's one "row block")
  __shared__ int s_done;
  __shared__ double s_ca[2][kChebDMax + 1];   // filter coefficients, degree 2 | 4 (indexed at run time: LDS, not the kernarg struct)
  extern __shared__ double s_dyn[];  // Q | Y, mpad x 16 each (fz_ix images)
  const int rep = blockIdx.x;
  const int mpad = (m + 15) & ~15, ng = (m + 3) >> 2;
  double *const sQ = s_dyn, *const sY = s_dyn + mpad * P;
  const double *Gr = G + (int64_t)rep * strideG;
  double *Ur = w.U + (int64_t)rep * m * P;
  // Every phase derives its thread coordinates from an opaque copy of
  // threadIdx.x: the lane's MFMA operand coordinates (fi, fkc), its element of
  // a folded 4 x 16 group result (orow, oc).  Coordinates derived once would
  // be hoisted out of the iteration loop with everything computed from them,
  // and all phases' offsets would stay live at once (hundreds of VGPRs).
#define FZ_THREAD                                                    \
  const int tid = fz_opaque(threadIdx.x), lane = tid & 63;          \
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);         \
  const int fi = lane & 3, fkc = 4 * (lane >> 4) + ((lane >> 2) & 3); \
  const int orow = lane >> 4, oc = lane & 15;                        \
  (void)wave; (void)fi; (void)fkc; (void)orow; (void)oc

  double tr = 0.0;   // trace (eig_trace_kernel's order); wave 0 keeps it for the checks
  {
    FZ_THREAD;
    // start basis (eig_init_kernel's)
    for (int e = tid; e < mpad * P; e += 256) {
      const int row = e >> 4, c = e & 15;
      double v = 0.0;
      if (row < m) {
        if (c < kw) v = warm[(int64_t)row * kw + c];
        else if (c < p) v = hash_unit(seed, row, c);
      }
      sQ[fz_ix(row, c)] = v;
      sY[fz_ix(row, c)] = 0.0;
    }
    if (tid < 4 * P) s_tail[tid] = 0.0;
    if (tid < P) s_res[tid] = 0.0;
    if (tid <= kChebDMax) { s_ca[0][tid] = cc.c2[tid]; s_ca[1][tid] = cc.c4[tid]; }
    if (wave == 0) {
      for (int i = lane; i < m; i += 64) tr += Gr[(int64_t)i * ldg + i];
      tr = wave_sum(tr);
      if (lane == 0) { w.trace[rep] = tr; w.done[rep] = 0; }
    }
  }
  __syncthreads();
  // phase profile of replicate 0 (DFM_EIG_PROF): thread 0's wall clock at the
  // phase-ending barriers, summed per phase over the iterations
  const bool pf = prof && rep == 0;   // workgroup-uniform: the sums stay in SGPRs
  long long pt = pf ? wall_clock64() : 0, pacc[6] = {0, 0, 0, 0, 0, 0};
#define FZ_MARK(i)                                           \
  do {                                                       \
    if (pf) { const long long t_ = wall_clock64(); pacc[i] += t_ - pt; pt = t_; } \
  } while (0)

  int it = 0;
  for (;; ++it) {
    {
      FZ_THREAD;
      if (wave == 0) {
        const int d = check_converged<P>(w, s_tail, s_res, tr, 0, rep, 0, 1, k, p, tol, it, 0);
        if (lane == 0) s_done = d;
      }
    }
    __syncthreads();
    FZ_MARK(0);
    if (s_done || it == maxit) break;   // converged, or the check-only pass after maxit steps

    {   // Y = G Q
      FZ_THREAD;
      constexpr int NG = OVL ? NG3 : NGW, NW = OVL ? 3 : 4;
      if (!OVL || wave < 3) {
        double acc[NG][4];
        fz_gemm<NG, NW>(Gr, ldg, m, ng, sQ, wave, lane, acc);
#pragma unroll
        for (int q = 0; q < NG; ++q) {
          const int g = wave + NW * q;
          if (g >= ng) continue;
          const double v = mm4_fold(acc[q], lane);
          const int row = 4 * g + orow;
          if (row < m) sY[fz_ix(row, oc)] = v;
        }
      } else {
        fz_xtx(sQ, sQ, sm.R2, mpad, lane);   // Q'Q
        wave_lds_sync();
        wave_chol_inv<P>(sm.R2, sm.R4, sm.dead, p);
      }
    }
    __syncthreads();
    FZ_MARK(1);

    {   // Q'Y -> R1, Y'Y -> R3 (and Q'Q -> R2 unless OVL formed it), stride P + 1, over all mpad rows
      FZ_THREAD;
      if (wave < (OVL ? 2 : 3)) {
        const double *X1 = wave == 1 ? sY : sQ, *X2 = wave == 2 ? sQ : sY;
        fz_xtx(X1, X2, wave == 0 ? sm.R1 : (wave == 1 ? sm.R3 : sm.R2), mpad, lane);
      }
    }
    __syncthreads();
    FZ_MARK(2);

    {
      FZ_THREAD;
      if (wave == 0) {
        if (pf) {   // stamps of the Rayleigh-Ritz stages (the last step's) after the phase sums
          EigWork wd = w;
          wd.dbg = prof + 8;
          small_rr<P>(sm, wd, rep, p, jsweeps | (OVL ? SMALL_CHOL1_DONE : 0) | SMALL_STAGE_A, nullptr, s_tail);
        } else {
          small_rr<P>(sm, w, rep, p, jsweeps | (OVL ? SMALL_CHOL1_DONE : 0) | SMALL_STAGE_A, nullptr, s_tail);
        }
      }
    }
    __syncthreads();
    FZ_MARK(3);

    // U pass (waves 1..3; A = R2, theta): U = Q A -> global, residual sums
    // of W = Y A - U diag(theta) — beside wave 0's chol(Z'Z) and Bm = R1
    {
      FZ_THREAD;
      if (wave == 0) {
        if (pf) {
          EigWork wd = w;
          wd.dbg = prof + 8;
          small_rr<P>(sm, wd, rep, p, jsweeps | SMALL_STAGE_B, nullptr, s_tail);
        } else {
          small_rr<P>(sm, w, rep, p, jsweeps | SMALL_STAGE_B, nullptr, s_tail);
        }
        if (lane < P) s_rw[0][lane] = 0.0;
      } else {
        double bA[4];
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) bA[fb] = sm.R2[fkc * S + 4 * fb + fi];
        const double th_c = s_tail[oc];
        double rs = 0.0;
#pragma unroll 1
        for (int g = wave - 1; g < ng; g += 3) {
          const int ra = 4 * g + fi;
          const double aq = sQ[fz_ix(ra, fkc)], ay = sY[fz_ix(ra, fkc)];
          double u4[4], ya4[4];
#pragma unroll
          for (int fb = 0; fb < 4; ++fb) {
            u4[fb] = mfma4(aq, bA[fb], 0.0);
            ya4[fb] = mfma4(ay, bA[fb], 0.0);
          }
          const double u = mm4_fold(u4, lane), ya = mm4_fold(ya4, lane);
          const int row = 4 * g + orow;
          if (row < m) {
            if (oc < k) { const double wv = ya - th_c * u; rs += wv * wv; }
            Ur[(int64_t)row * P + oc] = u;
          }
        }
        rs += __shfl_xor(rs, 16);
        rs += __shfl_xor(rs, 32);
        if (lane < P) s_rw[wave][lane] = rs;
      }
    }
    __syncthreads();
    FZ_MARK(4);

    // next basis: V = Y Bm, V0 = Q Bm -> the filter's first Horner term S =
    // (a_d / b) V + a_{d-1} V0 into Y, V0 into Q (dead columns re-randomised)
    const int dg = (warm_strict && it < 4) ? kChebDirectStrict : 2;
    const double *ca = s_ca[dg == 2 ? 0 : 1];
    const double bch = s_tail[p - 1];
    {
      FZ_THREAD;
      if (tid < P) s_res[tid] = ((s_rw[0][tid] + s_rw[1][tid]) + s_rw[2][tid]) + s_rw[3][tid];
      const bool dead_c = oc < p && s_tail[P + oc] != 0.0;
      double bB[4];
#pragma unroll
      for (int fb = 0; fb < 4; ++fb) bB[fb] = sm.R1[fkc * S + 4 * fb + fi];
      const double fa1 = ca[dg], fa0 = ca[dg - 1];
#pragma unroll 1
      for (int g = wave; g < ng; g += 4) {
        const int ra = 4 * g + fi;
        const double aq = sQ[fz_ix(ra, fkc)], ay = sY[fz_ix(ra, fkc)];
        double qn4[4], qb4[4];
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
          qn4[fb] = mfma4(ay, bB[fb], 0.0);
          qb4[fb] = mfma4(aq, bB[fb], 0.0);
        }
        double qn = mm4_fold(qn4, lane), qb = mm4_fold(qb4, lane);
        const int row = 4 * g + orow;
        if (dead_c) qn = hash_unit(seed, row, 1000003ull * (it + 1) + oc);
        if (oc >= p) { qn = 0.0; qb = 0.0; }
        if (row < m) {
          const double sv = dead_c ? qn : (bch > 0.0 ? fma(fa1 / bch, qn, fa0 * qb) : qn);
          sY[fz_ix(row, oc)] = oc >= p ? 0.0 : sv;
          sQ[fz_ix(row, oc)] = oc >= p ? 0.0 : (dead_c ? qn : qb);
        }
      }
    }
    __syncthreads();

    // Chebyshev filter: S_{dg-1} in Y; S_i = G S_{i+1} / b + a_i V0; S_0 into Q
    const double cb = bch > 0.0 ? 1.0 / bch : 1.0;
    for (int j = 1; j < dg; ++j) {
      const double cv0 = bch > 0.0 ? ca[dg - 1 - j] : 0.0;
      const bool last = j == dg - 1;
      double *So = last ? sQ : sY;
      FZ_THREAD;
      double acc[NGW][4];
      fz_gemm<NGW, 4>(Gr, ldg, m, ng, sY, wave, lane, acc);
      if (!last) __syncthreads();   // every wave has read S_{i+1} before S_i overwrites it
      const bool dead_c = oc < p && s_tail[P + oc] != 0.0;
#pragma unroll
      for (int q = 0; q < NGW; ++q) {
        const int g = wave + 4 * q;
        if (g >= ng) continue;
        const double gv = mm4_fold(acc[q], lane);
        const int row = 4 * g + orow;
        if (row < m) {
          const int ix = fz_ix(row, oc);
          const double v0 = sQ[ix];
          double sn = dead_c ? v0 : fma(cb, gv, cv0 * v0);
          if (oc >= p) sn = 0.0;
          So[ix] = sn;
        }
      }
      __syncthreads();
    }
    FZ_MARK(5);
  }
  // the last apply's Ritz vectors (this workgroup's own global writes: the
  // barrier that ended the iteration makes them visible) -> signs, outputs
  eig_final_body<P>(Ur, s_tail, s_done, rep, m, k, lam, Uk, status);
  if (pf && threadIdx.x == 0) {
    for (int i = 0; i < 6; ++i) prof[i] = pacc[i];
    prof[6] = it;
    prof[7] = wall_clock64() - pt;   // the final step
  }
#undef FZ_MARK
#undef FZ_THREAD
}

static int fused_ngw(int m) { return m <= 64 ? 4 : (m <= 144 ? 9 : (m <= 256 ? 16 : 0)); }
static bool fused_enabled() {
  static const bool on = [] { const char *e = getenv("DFM_EIG_FUSED"); return !(e && atoi(e) == 0); }();
  return on;
}

// Solve nb problems.  Returns 0 ok, 1 not converged (status per replicate),
// negative on bad args, or a hipError_t (>1000).
template <int P>
static int eig_run_t(const double *G, int64_t ldg, int64_t strideG, int m, int nb, int k, int p,
                     const double *warm, int kw, double tol, int maxit, int poll, char *ws,
                     double *lam, double *Uk, double *trace_out, int *status, int *iters_host,
                     hipStream_t st, timer_fn tf, void *tctx, int64_t rep0, int subspace) {
  const int nrb = (m + EROWS - 1) / EROWS;
  EigWork w = carve(ws, m, nb, P, maxit);
  w.subspace = subspace;
  hipMemsetAsync(w.active, 0, (size_t)(maxit + 2) * 4, st);
  hipMemsetAsync(w.iters, 0, (size_t)nb * 4, st);
  const uint64_t seed = 0x5eed0000ull + (uint64_t)m * 131 + k;
  // degree: 4 for the first four filters of a warm-started batch or a single
  // fit under the strict eigenvector rule (C2's Chow statistics: 8-9
  // Rayleigh-Ritz steps with degree 2, 5 with degree 4 in tools/eig_proto.py),
  // 2 for the polishing steps after them and for eigenvalue-only solves
  // (single fits, nb = 1, too: cold-started, polished to 1e-14 by run_eig)
  const bool warm_strict = tol >= 0.0 && ((warm && kw >= k) || nb == 1);
  if constexpr (P == 16) {
    const int ngw = fused_enabled() ? fused_ngw(m) : 0;
    if (ngw) {
      ChebCo cc;
      shifted_cheb(kChebDirectStrict, cc.c4);
      shifted_cheb(2, cc.c2);
      size_t lds = (size_t)2 * ((m + 15) & ~15) * P * sizeof(double);
#ifdef DFM_FUSED_PAD   // (A/B builds: extra dynamic LDS -> fewer resident workgroups per CU)
      lds += DFM_FUSED_PAD;
#endif
      // DFM_EIG_PROF=1: phase profile of replicate 0 of every fused solve -> stderr
      static const bool want_prof = [] { const char *e = getenv("DFM_EIG_PROF"); return e && atoi(e) != 0; }();
      long long *prof = nullptr;
      if (want_prof) {
        static thread_local long long *buf = nullptr;
        if (!buf && hipMalloc((void **)&buf, 24 * sizeof(long long)) != hipSuccess) buf = nullptr;
        prof = buf;
      }
      if (tf) tf(tctx, DFM_KC_EIG_GQ, 1);
#define DFM_FUSED(...)                                                                                          \
  hipFuncSetAttribute((const void *)eig_fused_kernel<__VA_ARGS__>, hipFuncAttributeMaxDynamicSharedMemorySize,    \
                      (int)lds);                                                                                  \
  hipLaunchKernelGGL((eig_fused_kernel<__VA_ARGS__>), dim3(nb), dim3(256), lds, st, G, ldg, strideG, w, m, k, p, tol, \
                     maxit, warm, kw, seed, (int)warm_strict, fused_sweeps(), cc, lam, Uk, status, prof)
      if (ngw == 4) { DFM_FUSED(4, 6, true); }
      else if (ngw == 9) { DFM_FUSED(9, 12, true); }
      else { DFM_FUSED(16, 22, false); }
#undef DFM_FUSED
      if (tf) tf(tctx, DFM_KC_EIG_GQ, 0);
      // iteration statistics from the per-iteration unconverged counts
      std::vector<int> a((size_t)maxit + 2, 0);
      hipMemcpyAsync(a.data(), w.active, a.size() * 4, hipMemcpyDeviceToHost, st);
      hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return 1000 + (int)e;
      int last = maxit;
      for (int i = 0; i <= maxit; ++i)
        if (a[i] == 0) { last = i; break; }
      g_last_iters = last;
      // a[i] replicates took Rayleigh-Ritz step i, each with dg(i) products
      // G S (Y = G Q and the filter's dg - 1 Horner steps)
      int64_t s = 0, prods = 0;
      for (int i = 0; i <= std::min(last, maxit - 1); ++i) {
        s += a[i];
        prods += (int64_t)a[i] * ((warm_strict && i < 4) ? kChebDirectStrict : 2);
      }
      g_last_rep_iters = s;
      g_last_gemm_products = prods;
      if (prof) {
        long long h[24];
        hipMemcpy(h, prof, sizeof(h), hipMemcpyDeviceToHost);
        const long long *d = h + 8;   // small_rr stamps 1..10, sweeps at 15
        fprintf(stderr, "eig_fused small stages us: chol1=%.2f mm=%.2f jacobi(%lld sweeps)=%.2f sort=%.2f mm3=%.2f "
                "chol2=%.2f mm=%.2f\n", (d[2] - d[1]) / 100.0, (d[4] - d[3]) / 100.0, d[15], (d[5] - d[4]) / 100.0,
                (d[6] - d[5]) / 100.0, (d[7] - d[6]) / 100.0, (d[8] - d[7]) / 100.0, (d[10] - d[9]) / 100.0);
        fprintf(stderr, "eig_fused m=%d nb=%d rep0: iters=%lld us check=%.1f gq=%.1f part=%.1f small=%.1f apply=%.1f "
                "cheb=%.1f final=%.1f\n", m, nb, h[6], h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0,
                h[4] / 100.0, h[5] / 100.0, h[7] / 100.0);
      }
      if (trace_out) hipMemcpyAsync(trace_out, w.trace, (size_t)nb * 8, hipMemcpyDeviceToDevice, st);
      if (iters_host) hipMemcpyAsync(iters_host, w.iters, (size_t)nb * 4, hipMemcpyDeviceToHost, st);
      e = hipGetLastError();
      if (e != hipSuccess) return 1000 + (int)e;
      return 0;
    }
  }
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 1);
  {
    const int64_t n = (int64_t)m * P;
    dim3 grid((unsigned)((n + 255) / 256), nb);
    hipLaunchKernelGGL(eig_init_kernel<P>, grid, dim3(256), 0, st, w.Q, m, p, warm, kw, w.done, seed, rep0);
    hipLaunchKernelGGL(eig_trace_kernel, dim3(nb), dim3(64), 0, st, G, ldg, strideG, m, w.trace);
  }
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 0);
  int it = 0;
  bool finished = false;
  std::vector<int> act;
  const int cheb = 1;   // Chebyshev filter between Rayleigh-Ritz steps
  double ca4[kChebDMax + 1], ca2[kChebDMax + 1];
  shifted_cheb(kChebDirectStrict, ca4);
  shifted_cheb(2, ca2);
  int next_poll = poll;
  for (; it <= maxit; ++it) {
    const int dg = warm_strict && it < 4 ? kChebDirectStrict : 2;
    const double *ca = dg == 2 ? ca2 : ca4;
    const int check_only = (it == maxit);
    if (tf) tf(tctx, DFM_KC_EIG_GQ, 1);
    hipLaunchKernelGGL(eig_gq_kernel<P>, dim3(nrb, nb), dim3(256), 0, st, G, ldg, strideG, w, m, k,
                       p, tol, it, check_only);
    if (tf) tf(tctx, DFM_KC_EIG_GQ, 0);
    if (check_only) break;
    if (tf) tf(tctx, DFM_KC_EIG_SMALL, 1);
    hipLaunchKernelGGL(eig_small_kernel<P>, dim3(nb), dim3(64), 0, st, w, p, nrb, kJacobiSweeps);
    if (tf) tf(tctx, DFM_KC_EIG_SMALL, 0);
    if (tf) tf(tctx, DFM_KC_EIG_APPLY, 1);
    hipLaunchKernelGGL(eig_apply_kernel<P>, dim3(nrb, nb), dim3(256), 0, st, w, m, p, k, it, seed, rep0, cheb,
                       ca[dg], ca[dg - 1]);
    for (int j = 1; cheb && j < dg; ++j) {   // S_{dg-1-j}: in w.Y / w.S alternately, S_0 into w.Q
      const double *sin = (j & 1) ? w.Y : w.S;
      double *sout = j == dg - 1 ? w.Q : ((j & 1) ? w.S : w.Y);
      hipLaunchKernelGGL(eig_cheb_kernel<P>, dim3(nrb, nb), dim3(256), 0, st, G, ldg, strideG, w, m, p, sin, sout,
                         ca[dg - 1 - j]);
    }
    if (tf) tf(tctx, DFM_KC_EIG_APPLY, 0);
    if (it == next_poll) {
      int a = -1;
      hipMemcpyAsync(&a, w.active + it, 4, hipMemcpyDeviceToHost, st);
      hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) return 1000 + (int)e;
      if (a == 0) { finished = true; break; }
      // a straggler tail (< 1/8 of the batch active): poll every step, so the
      // empty iterations after its last replicate retires are not launched
      next_poll = it + ((int64_t)a * 8 < nb ? 1 : poll);
    }
  }
  (void)finished;
  g_last_iters = it;
  g_last_rep_iters = count_rep_iters(w.active, std::min(it, maxit - 1), 0, nb, st);
  g_last_gemm_products = g_last_rep_iters;
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 1);
  hipLaunchKernelGGL(eig_final_kernel<P>, dim3(nb), dim3(256), 0, st, w, m, k, lam, Uk, status, trace_out);
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 0);
  if (iters_host) {
    hipMemcpyAsync(iters_host, w.iters, (size_t)nb * 4, hipMemcpyDeviceToHost, st);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return 1000 + (int)e;
  return 0;
}

int eig_block_P(int m, int k) {
  const int p = std::min(m, std::max(k + 8, 16));
  return p <= 16 ? 16 : (p <= 32 ? 32 : -1);
}
// A requested block below k + 1 is raised to k + 1: the Chebyshev filter's
// interval [0, theta_p] must lie below every wanted eigenvalue, so the block
// needs at least one guard vector (p == k: theta_p is the k-th WANTED value
// and the filter stops amplifying it — the k-th vector then never converges)
int eig_block_p(int m, int k, int req) {
  int p = req > 0 ? std::max(req, k + 1) : std::max(k + 8, 16);
  p = std::min(p, m);
  return p;
}

// Block of the factored bootstrap solver (N > T, eig_run_fact2_t): k + 4
// columns, at least 8 (C3: 12 instead of the explicit-Gram solvers' 16).  The
// H.Z GEMM's work and the Z / HZ traffic scale with the block (Z, HZ hold it
// compactly, rounded up to even), and the Chebyshev filter does the damping
// that extra guard vectors would otherwise buy: tools/eig_proto.py at C3
// (warm start + the degree-6 first filter) retires 94 % of replicates at the
// 2nd Rayleigh-Ritz step with 12 columns (7.12 products) as with 16 (7.00).
// A requested block (dfm_ctx_set_eig_params) is taken as for the other
// solvers; DFM_FACT_GUARD (A/B) overrides the 4.
int fact_block_p(int m, int k, int req) {
  if (req > 0) return eig_block_p(m, k, req);
  static const int guard = [] { const char *e = getenv("DFM_FACT_GUARD"); return e ? atoi(e) : 4; }();
  if (guard <= 0) return eig_block_p(m, k, 0);
  return std::min(m, std::max(k + guard, 8));
}

int eig_run(const double *G, int64_t ldg, int64_t strideG, int m, int nb, int k, int p,
            const double *warm, int kw, double tol, int maxit, int poll, char *ws, double *lam,
            double *Uk, double *trace_out, int *status, int *iters_host, hipStream_t st,
            timer_fn tf, void *tctx, int64_t rep0, int subspace) {
  if (p < k || p > 32 || p > m) return -1;
  if (p <= 16)
    return eig_run_t<16>(G, ldg, strideG, m, nb, k, p, warm, kw, tol, maxit, poll, ws, lam, Uk,
                         trace_out, status, iters_host, st, tf, tctx, rep0, subspace);
  return eig_run_t<32>(G, ldg, strideG, m, nb, k, p, warm, kw, tol, maxit, poll, ws, lam, Uk,
                       trace_out, status, iters_host, st, tf, tctx, rep0, subspace);
}


// ===================================================================== factored
// Factored bootstrap (N > T).  With X* = F L' + D P E  (F = F_r, L = L_r of the
// base fit, D = diag(eta), P the row selection of idx; src/bootstrap.jl:45):
//   G* Q = X* X*' Q = F [S a + (EL)' Z] + D P [(EL) a + H Z]
//   a = F'Q (r x p), Z = P' D Q (T x p, scatter through a CSR of idx),
//   S = L'L, EL = E L (T x r), H = E E' (T x T)  — S, EL, H shared by all
// replicates.  H Z for a whole batch is ONE MFMA GEMM (dfm_gemm.hip) with H
// resident in L2; everything else is O(T r p) per replicate.
// waves per replicate workgroup of the factored passes (prep, y2, ap2, Chebyshev)
#ifndef DFM_BW
#define DFM_BW 4
#endif
constexpr int BW = DFM_BW;   // dynamic LDS of ap2: 16 T + 4 bytes

struct FactBase {
  int T, r;
  int64_t ldH;
  const double *F, *EL, *S, *H, *cF, *hd;   // T x r, T x r, r x r, T x ldH, T, T
  const double *FtF = nullptr;   // F'F (16 x 16) when the model holds it (else computed per solve)
};

// Z, the H.Z GEMM's B operand, replicate-major in 16-row chunks (round 6,
// gemmh_zrm_kernel): replicate rep's element (s, c) at
// rep zrs + (s >> 4) 16 pz + 16 c + (s & 15), zrs = round_up(T, 16) pz; the
// chunk rows s >= T are zero (boot_prep_kernel writes them each call)
DFM_DEV int64_t zrm_stride(int T, int pz) { return (int64_t)((T + 15) & ~15) * pz; }
DFM_DEV int64_t zrm_ix(int rep, int s, int c, int pz, int64_t zrs) {
  return (int64_t)rep * zrs + (int64_t)(s >> 4) * (16 * pz) + 16 * c + (s & 15);
}

// Per replicate: CSR of idx (bucket s lists t ascending — fixed summation
// order, bit-reproducible), and trace(G*) = sum_t ||x*_t||^2 =
// sum_t [F_t S F_t' + 2 eta_t F_t.(EL)_idx_t + eta_t^2 H_idx_t,idx_t].
//
// Round 6: the same kernel then forms the first H.Z product's operand
// Z0 = P'D Q0 and the first step's ab = [a; cc] (a = F'Q0, cc = EL'Z0) —
// the init pass of boot_ap2_kernel before, the same arithmetic in the same
// order (its tile loop and zscatter_tail), without that pass's launch and
// its reload of the CSR this kernel already holds in LDS.
template <int P, bool STG>
DFM_DEV void zscatter_tail(const FactBase &fb, int T, int r, int ntile, int tid, int wave, int lane,
                           const double *set, const int *so, const int *sl, const double *Qn,
                           double *__restrict__ Zc, int pz, int rep, double *__restrict__ ab,
                           const dv4 *aacc, double *sred, int ps, double *zst, const double *apre = nullptr);
// a = F'Q0 of the first product for the whole batch: F and the warm start Q0
// are shared by every replicate, so boot_prep_kernel's per-workgroup tile
// loop and fixed-order wave sums are run ONCE, in the same order (one
// workgroup of the same shape: bit-identical), into apre in ab's layout
// (round 6; before, every replicate's workgroup formed the same 16 x P block).
template <int P>
__global__ __launch_bounds__(256) void prep_a_kernel(FactBase fb, const double *__restrict__ Q0, int ps,
                                                     double *__restrict__ apre) {
  constexpr int NT = P / 16;
  __shared__ double sred[NT * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4, T = fb.T, r = fb.r;
  const int ntile = (T + 15) >> 4;
  dv4 aacc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) aacc[ct] = dv4{0.0, 0.0, 0.0, 0.0};
  for (int tile = wave; tile < ntile; tile += BW) {
    const int t0 = tile * 16;
    double fa[4], qv[NT][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int t = t0 + 4 * g + lk;
      const int tc = min(t, T - 1);
      fa[g] = (t < T && li < r) ? fb.F[(int64_t)tc * r + li] : 0.0;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
        qv[ct][g] = (t < T && 16 * ct + li < ps) ? Q0[(int64_t)tc * ps + 16 * ct + li] : 0.0;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) aacc[ct] = mfma16(fa[g], qv[ct][g], aacc[ct]);
  }
  for (int wv = 0; wv < BW; ++wv) {
    if (wave == wv)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int e = (ct * 4 + g) * 64 + lane;
          sred[e] = (wv ? sred[e] : 0.0) + aacc[ct][g];
        }
    __syncthreads();
  }
  for (int e = tid; e < NT * 256; e += 64 * BW) {
    const int l = e & 63, g = (e >> 6) & 3, ct = e >> 8;
    apre[(4 * g + (l >> 4)) * P + 16 * ct + (l & 15)] = sred[e];
  }
}

template <int P>
__global__ __launch_bounds__(256) void boot_prep_kernel(FactBase fb, const int32_t *__restrict__ idx,
                                                        const double *__restrict__ eta, int *__restrict__ off,
                                                        int *__restrict__ lst, double *__restrict__ trace,
                                                        double *__restrict__ PF, double *__restrict__ E2,
                                                        const double *__restrict__ Q0, int ps,
                                                        double *__restrict__ Zc, int64_t ldz, int pz,
                                                        double *__restrict__ ab, const double *__restrict__ apre) {
  static_assert(BW * 64 == 256, "prep runs the factored passes' wave layout");
  constexpr int NT = P / 16;
  __shared__ double sred[NT * 256];
  __shared__ double zst[BW][16 * P];   // per-wave Z chunk staging (zscatter_tail)
  extern __shared__ int sh[];   // cnt[T+1], six[T], sorted list L[T] (+ so[T+1], eta[T]: Zc)
  __shared__ double red[256];
  __shared__ int scan[256];
  const int tid = threadIdx.x, rep = blockIdx.x, T = fb.T, r = fb.r;
  const int32_t *ix = idx + (int64_t)rep * T;
  const double *et = eta ? eta + (int64_t)rep * T : nullptr;
  int *cnt = sh, *six = sh + T + 1;
  for (int s = tid; s <= T; s += 256) cnt[s] = 0;
  for (int t = tid; t < T; t += 256) six[t] = ix[t];
  __syncthreads();
  for (int t = tid; t < T; t += 256) atomicAdd(&cnt[six[t] + 1], 1);
  __syncthreads();
  // inclusive scan of cnt[0..T]: per-thread chunks, a 256-wide scan of the chunk sums
  const int per = (T + 1 + 255) / 256, c0 = min(T + 1, tid * per), c1 = min(T + 1, c0 + per);
  int run = 0;
  for (int s = c0; s < c1; ++s) run += cnt[s];
  scan[tid] = run;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int v = tid >= o ? scan[tid - o] : 0;
    __syncthreads();
    scan[tid] += v;
    __syncthreads();
  }
  run = scan[tid] - run;
  for (int s = c0; s < c1; ++s) { run += cnt[s]; cnt[s] = run; }   // cnt[s] = start of bucket s
  __syncthreads();
  for (int s = tid; s <= T; s += 256) off[(int64_t)rep * (T + 1) + s] = cnt[s];
  __syncthreads();
  // placement: LDS atomics hand out slots inside each bucket (any order),
  // then each bucket is insertion-sorted by t — ascending t per bucket, the
  // serial counting sort's order, in O(T) work (buckets are short)
  // (in LDS, then one coalesced copy out: the shifts of a sort in global
  // memory were chains of dependent global round trips)
  int *L = sh + 2 * T + 1;
  for (int t = tid; t < T; t += 256) L[atomicAdd(&cnt[six[t]], 1)] = t;
  __syncthreads();   // cnt[s] is now the END of bucket s; L visible workgroup-wide
  for (int s = tid; s < T; s += 256) {
    const int b0 = s ? cnt[s - 1] : 0, b1 = cnt[s];
    for (int i = b0 + 1; i < b1; ++i) {
      const int v = L[i];
      int j = i - 1;
      while (j >= b0 && L[j] > v) { L[j + 1] = L[j]; --j; }
      L[j + 1] = v;
    }
  }
  __syncthreads();
  for (int t = tid; t < T; t += 256) lst[(int64_t)rep * T + t] = L[t];
  // LDS after the sorted list: bucket starts so[0..T] and eta_t (PF below, zscatter_tail)
  int *so = sh + 3 * T + 1;
  double *set = reinterpret_cast<double *>(sh + ((4 * T + 2 + 1) & ~1));
  for (int q = tid; q <= T; q += 256) so[q] = q ? cnt[q - 1] : 0;
  for (int t = tid; t < T; t += 256) set[t] = et ? et[t] : 1.0;
  __syncthreads();
  if (PF)   // P'D F (row stride r) and P'D^2 1 of the middle Horner steps (boot_cheb_mid_kernel):
    for (int s = tid; s < T; s += 256) {   // this thread's own sorted buckets, t ascending
      const int b0 = s ? cnt[s - 1] : 0, b1 = cnt[s];
      double a[16], a2 = 0.0;
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] = 0.0;
      for (int q = b0; q < b1; ++q) {
        const int t = L[q];
        const double h = set[t];
        a2 = fma(h, h, a2);
        if ((r & 1) == 0) {   // 16-B loads of the F row (F rows start 16-B aligned)
          const double2 *f2 = reinterpret_cast<const double2 *>(fb.F + (int64_t)t * r);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (2 * j < r) {
              const double2 f = f2[j];
              a[2 * j] = fma(h, f.x, a[2 * j]);
              a[2 * j + 1] = fma(h, f.y, a[2 * j + 1]);
            }
        } else {
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (j < r) a[j] = fma(h, fb.F[(int64_t)t * r + j], a[j]);
        }
      }
      double *pf = PF + ((int64_t)rep * T + s) * r;
      if ((r & 1) == 0) {   // 16-B stores (rows start 16-B aligned for even r)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (2 * j < r) reinterpret_cast<double2 *>(pf)[j] = double2{a[2 * j], a[2 * j + 1]};
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j < r) pf[j] = a[j];
      }
      E2[(int64_t)rep * T + s] = a2;
    }
  if (Zc) {
    // a = F'Q0 in boot_ap2_kernel's init order (its tiles, its accumulator layout)
    const int lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
    const int ntile = (T + 15) >> 4;
    dv4 aacc[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) aacc[ct] = dv4{0.0, 0.0, 0.0, 0.0};
    for (int tile = wave; tile < (apre ? 0 : ntile); tile += BW) {   // (apre: a = F'Q0 formed once per batch)
      const int t0 = tile * 16;
      double fa[4], qv[NT][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int t = t0 + 4 * g + lk;
        const int tc = min(t, T - 1);
        fa[g] = (t < T && li < r) ? fb.F[(int64_t)tc * r + li] : 0.0;
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
          qv[ct][g] = (t < T && 16 * ct + li < ps) ? Q0[(int64_t)tc * ps + 16 * ct + li] : 0.0;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) aacc[ct] = mfma16(fa[g], qv[ct][g], aacc[ct]);
    }
    // the last chunk's rows past T (the H.Z GEMM's zero k-padding of B)
    {
      const int64_t zrs = zrm_stride(T, pz);
      const int npad = ((T + 15) & ~15) - T;
      for (int e = tid; e < npad * pz; e += 256) Zc[zrm_ix(rep, T + e / pz, e % pz, pz, zrs)] = 0.0;
    }
    __syncthreads();   // so / set visible
    zscatter_tail<P, true>(fb, T, r, ntile, tid, wave, lane, set, so, L, Q0, Zc, pz, rep, ab, aacc, sred, ps, zst[wave],
                           apre);
  }
  double acc = 0.0;
  for (int t = tid; t < T; t += 256) {
    const int i = ix[t];
    const double e = et ? et[t] : 1.0;
    double fe = 0.0;
    if ((r & 1) == 0) {   // F and EL rows as 16-B pieces (half the load instructions; same fma order)
      const double2 *f2 = reinterpret_cast<const double2 *>(fb.F + (int64_t)t * r);
      const double2 *e2 = reinterpret_cast<const double2 *>(fb.EL + (int64_t)i * r);
      double2 fv[8], ev[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (2 * j < r) { fv[j] = f2[j]; ev[j] = e2[j]; }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (2 * j < r) { fe = fma(fv[j].x, ev[j].x, fe); fe = fma(fv[j].y, ev[j].y, fe); }
    } else {
      for (int j = 0; j < r; ++j) fe = fma(fb.F[(int64_t)t * r + j], fb.EL[(int64_t)i * r + j], fe);
    }
    acc += fb.cF[t] + 2.0 * e * fe + e * e * fb.hd[i];
  }
  red[tid] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) { if (tid < o) red[tid] += red[tid + o]; __syncthreads(); }
  if (tid == 0) trace[rep] = red[0];
}

hipError_t launch_gemm_loadings(const double *Eaug, int64_t lda, const double *ZF, int Kp, int rp, int N, int nrep,
                                int K, int r, double invT, double *Lout, hipStream_t st);
hipError_t launch_gemm(bool a_trans, const double *A, int64_t lda, const double *B, int64_t ldb,
                       double *C, int64_t ldc, int M, int Nc, int K, hipStream_t st,
                       const int *col_done = nullptr, int col_group = 1, bool b_padded = false,
                       const int *clist = nullptr, const int *ccount = nullptr);
hipError_t launch_gemm_zrm(const double *A, int64_t lda, const double *Z, int pz, int64_t zrs, double *C,
                           int64_t ldc, int M, int Nc, int K, hipStream_t st, const int *col_done, const int *clist,
                           const int *ccount);

// Z (the GEMM's B operand) has round_up(T, 16) rows, the pad rows zero, so
// the H.Z GEMM streams it with running DMA pointers and no k-tail clamp
static int64_t z_rows(int T) { return ((int64_t)T + 15) / 16 * 16; }
// the middle Horner steps' per-replicate operands (boot_cheb_mid_kernel):
// PF = P'D F (T x r, allocated T x 16), e2 = P'D^2 1 (T), FV = F'V0 (16 x P),
// and F'F (16 x 16, shared)
static size_t fact_mid_doubles(int T, int nb, int P) {
  return (size_t)nb * T * 17 + (size_t)nb * 16 * P + 256;
}
size_t fact_workspace_bytes(int T, int nb, int P) {
  const int64_t ldz = (int64_t)nb * P;
  const int nrb = (T + EROWS - 1) / EROWS;
  return (size_t)(z_rows(T) + T) * ldz * 8 + (size_t)nb * nrb * 2 * 32 * P * 8 + 4096 +
         fact_mid_doubles(T, nb, P) * 8 + 4096;
}

// ================================================= fused factored iteration
// For T <= F2_T_MAX and r <= 16 (C3: T = 500, r = 8) one iteration of
// the factored solver is four launches instead of five, with no per-row-block
// partial arrays and no separate convergence pass:
//   GEMM  HZ = H Z                          (shared H, all unconverged replicates)
//   y2    Y = F (S a + cc) + D (EL[idx] a + HZ[idx]),  Q'Y, Y'Y, Q'Q   (one WG / replicate)
//   small Rayleigh-Ritz on p x p            (eig_small_kernel, nrb = 1)
//   ap2   U = Q A, Qn = Y Bm, residuals ||Y A - U diag(theta)|| -> converged?
//         else Z = P' D Qn (CSR gather from an LDS image), a = F'Qn, cc = EL'Z
// Every T x P product is a v_mfma_f64_16x16x4 chain whose operands are the
// rows a lane already holds: A[i][k] at lane i + 16k, B[k][j] at lane j + 16k,
// C[row][col] at lane col + 16 (row % 4), register row / 4
// (tools/mfma16_layout.hip).  An accumulator register g holds rows
// 4g .. 4g+3 in exactly the B-operand layout, so Q'Y etc. need no lane movement.
// Reductions over waves run in a fixed order: bit-reproducible, batch-invariant.
constexpr int F2_T_MAX = 4096;

// Convergence verdict from per-column squared residuals res2[j] (j < k), on
// one whole wave (same rules as check_converged: strict eigenvector-residual
// test, or for tol < 0 the Kato-Temple eigenvalue bound).
DFM_DEV bool decide_converged(const double *res2, const double *th, const double *prev, double *next,
                              int k, int p, double tol, double trace, int itc, int subspace) {
  const int lane = threadIdx.x & 63;
  const double th0 = fabs(th[0]);
  bool okall = true, floor_ok = true;
  double bsum = 0.0, tsum = 0.0;
  for (int j = lane; j < k; j += 64) {
    const double rs = res2[j], res = sqrt(rs);
    double gap = INFINITY;
    if (subspace && tol >= 0.0 && k < p) {   // strict rule, subspace form (EigWork::subspace; k == p: neighbours)
      gap = fabs(th[j] - th[k]);
    } else {
      if (j > 0) gap = fmin(gap, fabs(th[j] - th[j - 1]));
      if (j + 1 < p) gap = fmin(gap, fabs(th[j] - th[j + 1]));
    }
    bool okj;
    if (tol < 0.0) {
      const double bnd = rs / (0.5 * gap);
      bsum += bnd;
      tsum += th[j];
      okj = bnd <= -tol * fabs(th[j]) || res <= 2e-14 * th0;
    } else {
      const bool stagn = itc > 2 && res <= 1e-11 * th0 && res > 0.5 * prev[j];
      okj = res <= tol * gap || res <= 2e-14 * th0 || stagn;
    }
    floor_ok = floor_ok && res <= 2e-14 * th0;
    okall = okall && okj;
    next[j] = res;
  }
  bool ok = !__any(!okall);
  if (tol < 0.0) {
    bsum = wave_sum(bsum);
    tsum = wave_sum(tsum);
    const double vnum = fmax(fabs(trace - tsum), 1e-6 * fabs(trace));
    ok = ok && (bsum <= -tol * vnum || !__any(!floor_ok));
  }
  return ok;
}

#ifdef DFM_DIAG_X
// diagnostic build only (tools/c3_excess.py): how far each replicate's
// eigenvalue-bound test is from passing at Rayleigh-Ritz step it + 1
__device__ double g_diag_x[4][16384];
DFM_DEV void diag_excess(const double *res2, const double *th, int k, int p, double tol, double trace, int rep,
                         int it) {
  const int lane = threadIdx.x & 63;
  double r1 = 0.0, bsum = 0.0, tsum = 0.0;
  for (int j = lane; j < k; j += 64) {
    const double gap = fmin(j > 0 ? fabs(th[j] - th[j - 1]) : INFINITY, j + 1 < p ? fabs(th[j] - th[j + 1]) : INFINITY);
    const double bnd = res2[j] / (0.5 * gap);
    bsum += bnd; tsum += th[j];
    r1 = fmax(r1, bnd / (-tol * fabs(th[j])));
  }
  bsum = wave_sum(bsum); tsum = wave_sum(tsum);
  for (int o = 32; o >= 1; o >>= 1) r1 = fmax(r1, __shfl_xor(r1, o));
  const double vnum = fmax(fabs(trace - tsum), 1e-6 * fabs(trace));
  const double x = fmax(r1, bsum / (-tol * vnum));
  if (lane == 0 && it >= 0 && it < 4 && rep < 16384) g_diag_x[it][rep] = x;
}
extern "C" int dfm_diag_read_x(double *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag_x), sizeof(g_diag_x)) == hipSuccess ? 0 : -1;
}
#endif

// One 16-row tile's operands for y2: F / EL[idx] rows in A-operand layout
// (row t0 + (lane & 15), factor 4kk + (lane >> 4)), HZ[idx] and Q in the
// accumulator layout (row t0 + 4g + (lane >> 4), column 16ct + (lane & 15)).
// Rows >= T load row T-1 and are masked by the consumer.
template <int P>
struct Y2Tile {
  double fA[4], eA[4], hz[P / 16][4], q[P / 16][4];
};
// STG (P = 16, even r <= 8, pz <= 16; y2 and the last Horner step — y2
// reads its MFMA B operands from LDS per tile when staged, else the staged
// form spills: 128 VGPRs + 52 B of scratch, y2 60 % slower, profiles/
// r06_c3_ab.txt items 19 and 23): every
// operand of the tile arrives as 16-B pieces through this wave's LDS stage
// (stg, Y2_STG doubles) — the F rows as one contiguous range, each EL[idx]
// and HZ[idx] row as r / 2 and pz / 2 pieces, the Q rows as one contiguous
// range — and is transposed to its register layout there: half the load
// requests of one-double-per-lane loads, for passes bound by the texture-
// address unit (round 6).  Stage layout: F rows [0, 144) (kept for the
// caller's accumulator-layout read of F, fa), EL rows [144, 288), then HZ
// and Q rows over [144, 688) once the EL reads are done.
constexpr int Y2_STG = 16 * 9 + 2 * 16 * 17;
template <int P, bool STG = false>
DFM_DEV void y2_load(Y2Tile<P> &L, int tile, int T, int r, int KR, int lane, const int *six, const FactBase &fb,
                     const double *__restrict__ HZ, int64_t ldz, int pz, int rep, const double *__restrict__ Qr,
                     int ps, double *stg = nullptr) {
  constexpr int NT = P / 16;
  const int li = lane & 15, lk = lane >> 4, t0 = tile * 16;
  const int ta = min(t0 + li, T - 1);
  if constexpr (STG) {
    static_assert(P == 16, "the staged loader covers one 16-column block");
    const int nrow = min(16, T - t0), hr = r >> 1, hp = pz >> 1, hq = ps >> 1;
    // issue every piece first (F, EL: 8 r <= 64 pieces; HZ, Q: 8 pz, 8 ps <= 128)
    double2 fv, ev, hv[2], qv[2];
    {
      const int row = hr ? lane / hr : 0, jp = lane - row * hr;
      const bool ok = lane < nrow * hr;
      fv = ok ? reinterpret_cast<const double2 *>(fb.F + (int64_t)t0 * r)[lane] : double2{0.0, 0.0};
      ev = ok ? reinterpret_cast<const double2 *>(fb.EL + (int64_t)six[t0 + row] * r)[jp] : double2{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = u * 64 + lane;
      const int row = e / hp, jp = e - row * hp;
      const bool okh = e < nrow * hp;
      hv[u] = okh ? reinterpret_cast<const double2 *>(HZ + (int64_t)six[t0 + row] * ldz + (int64_t)rep * pz)[jp]
                  : double2{0.0, 0.0};
      const bool okq = e < nrow * hq;
      qv[u] = okq ? reinterpret_cast<const double2 *>(Qr + (int64_t)t0 * ps)[e] : double2{0.0, 0.0};
    }
    const int RF = r + 1, RH = pz + 1, RQ = ps + 1;
    double *sF = stg, *sE = stg + 16 * 9;         // (RF <= 9)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous tile's staged reads are done
    if (lane < 16 * hr) {
      const int row = lane / hr, j = 2 * (lane - row * hr);
      sF[row * RF + j] = fv.x; sF[row * RF + j + 1] = fv.y;
      sE[row * RF + j] = ev.x; sE[row * RF + j + 1] = ev.y;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bool ok = kk < KR && 4 * kk + lk < r && t0 + li < T;
      L.fA[kk] = ok ? sF[li * RF + 4 * kk + lk] : 0.0;
      L.eA[kk] = ok ? sE[li * RF + 4 * kk + lk] : 0.0;
    }
    double *sH = stg + 16 * 9, *sQ = sH + 16 * 17;   // over EL (read above), after F (kept for fa)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = u * 64 + lane;
      if (e < 16 * hp) {
        const int row = e / hp, j = 2 * (e - row * hp);
        sH[row * RH + j] = hv[u].x; sH[row * RH + j + 1] = hv[u].y;
      }
      if (e < 16 * hq) {
        const int row = e / hq, j = 2 * (e - row * hq);
        sQ[row * RQ + j] = qv[u].x; sQ[row * RQ + j + 1] = qv[u].y;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      L.hz[0][g] = li < pz ? sH[(4 * g + lk) * RH + li] : 0.0;
      L.q[0][g] = li < ps ? sQ[(4 * g + lk) * RQ + li] : 0.0;
    }
    return;
  } else {
    const int ia = six[ta];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int j = max(0, min(4 * kk + lk, r - 1));   // never index -1 (r = 0: expanding windows)
      L.fA[kk] = (kk < KR && 4 * kk + lk < r && t0 + li < T) ? fb.F[(int64_t)ta * r + j] : 0.0;
      L.eA[kk] = (kk < KR && 4 * kk + lk < r && t0 + li < T) ? fb.EL[(int64_t)ia * r + j] : 0.0;
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int t = min(t0 + 4 * g + lk, T - 1);
    const int i = six[t];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      const int c = 16 * ct + li;
      L.hz[ct][g] = c < pz ? HZ[(int64_t)i * ldz + (int64_t)rep * pz + c] : 0.0;   // compact Z / HZ: pz columns
      L.q[ct][g] = c < ps ? Qr[(int64_t)t * ps + c] : 0.0;   // compact rows: ps columns
    }
  }
}

// y2: one workgroup (4 waves) per replicate; wave w takes 16-row tiles w, w+4, ...
template <int P, bool STG>
// 4 workgroups per CU (~113 VGPRs, no spills; a tile is loaded at the top of
// its own iteration, no register prefetch of the next): these per-replicate
// passes are HBM-latency-bound, and resident waves buy more bandwidth than
// per-wave prefetch did (2 -> 4 WGs/CU: y2 -24 %, ap2 -13 %)
__global__ __launch_bounds__(64 * BW, 4) void boot_y2_kernel(FactBase fb, EigWork w, int T, const int32_t *__restrict__ idx,
                                                      const double *__restrict__ eta,
                                                      const double *__restrict__ HZ, int64_t ldz, int pz,
                                                      const double *__restrict__ ab,
                                                      const double *__restrict__ Qc, int64_t qs,
                                                      double *__restrict__ Yo, int ps) {
  constexpr int NT = P / 16;
  const int rep = blockIdx.x;
  if (w.done[rep]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = fb.r;
  const int li = lane & 15, lk = lane >> 4;
  __shared__ double sa[16 * P], sb[16 * P];          // a = F'Q, S a + cc  (rows >= r zero)
  __shared__ double red[3 * NT * NT * 256];
  extern __shared__ double sdyn[];                   // eta (T doubles), idx (T ints)
  __shared__ double stgy[STG ? BW : 1][STG ? Y2_STG : 1];   // per-wave operand staging (y2_load)
  double *set = sdyn;
  int *six = (int *)(sdyn + T);
  {
    const int32_t *ixg = idx + (int64_t)rep * T;
    const double *etg = eta ? eta + (int64_t)rep * T : nullptr;
    for (int e = tid; e < T; e += 64 * BW) { six[e] = ixg[e]; set[e] = etg ? etg[e] : 1.0; }
  }
  const double *abr = ab + (int64_t)rep * 32 * P;
  for (int e = tid; e < 16 * P; e += 64 * BW) sa[e] = abr[e];
  __syncthreads();
  for (int e = tid; e < 16 * P; e += 64 * BW) {
    const int j = e / P, c = e % P;
    double v = abr[16 * P + e];
    if (j < r)
      for (int i = 0; i < r; ++i) v = fma(fb.S[j * r + i], sa[i * P + c], v);
    sb[e] = v;
  }
  __syncthreads();
  const int KR = (r + 3) >> 2;
  double bA[4][NT], bB[4][NT];   // (STG: read from LDS per tile instead, to make room for the staged loader)
  if constexpr (!STG) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        bA[kk][ct] = sa[(4 * kk + lk) * P + 16 * ct + li];
        bB[kk][ct] = sb[(4 * kk + lk) * P + 16 * ct + li];
      }
  }
  dv4 acc[3][NT][NT];
#pragma unroll
  for (int m3 = 0; m3 < 3; ++m3)
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[m3][a][b] = dv4{0.0, 0.0, 0.0, 0.0};
  const double *Qr = Qc + (int64_t)rep * qs;   // qs = 0: the shared warm start (first step)
  double *Yr = Yo + (int64_t)rep * T * P;
  const int ntile = (T + 15) >> 4;
  // each tile's operands load at the top of its iteration (occupancy hides the latency)
  Y2Tile<P> cur;
  for (int tile = wave; tile < ntile; tile += BW) {
    y2_load<P, STG>(cur, tile, T, r, KR, lane, six, fb, HZ, ldz, pz, rep, Qr, ps, stgy[STG ? wave : 0]);
    const int t0 = tile * 16;
    dv4 yF[NT], yE[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) { yF[ct] = dv4{0.0, 0.0, 0.0, 0.0}; yE[ct] = yF[ct]; }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < KR) {
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          if constexpr (STG) {
            yF[ct] = mfma16(cur.fA[kk], sb[(4 * kk + lk) * P + 16 * ct + li], yF[ct]);
            yE[ct] = mfma16(cur.eA[kk], sa[(4 * kk + lk) * P + 16 * ct + li], yE[ct]);
          } else {
            yF[ct] = mfma16(cur.fA[kk], bB[kk][ct], yF[ct]);
            yE[ct] = mfma16(cur.eA[kk], bA[kk][ct], yE[ct]);
          }
        }
      }
    }
    double Yv[NT][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int t = t0 + 4 * g + lk;
      const bool v = t < T;
      const double e = v ? set[t] : 0.0;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        const int c = 16 * ct + li;
        const double y = v ? fma(e, yE[ct][g] + cur.hz[ct][g], yF[ct][g]) : 0.0;
        if (v && c < ps) Yr[(int64_t)t * ps + c] = y;
        Yv[ct][g] = y;
        if (!v) cur.q[ct][g] = 0.0;   // clamped row: no contribution to Q'Y, Q'Q
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          acc[0][a][b] = mfma16(cur.q[a][g], Yv[b][g], acc[0][a][b]);
          acc[1][a][b] = mfma16(Yv[a][g], Yv[b][g], acc[1][a][b]);
          acc[2][a][b] = mfma16(cur.q[a][g], cur.q[b][g], acc[2][a][b]);
        }
  }
  // fixed-order sum over the four waves
  for (int wv = 0; wv < BW; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int m3 = 0; m3 < 3; ++m3)
#pragma unroll
        for (int a = 0; a < NT; ++a)
#pragma unroll
          for (int b = 0; b < NT; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int e = ((m3 * NT + a) * NT + b) * 256 + g * 64 + lane;
              red[e] = (wv ? red[e] : 0.0) + acc[m3][a][b][g];
            }
    }
    __syncthreads();
  }
  double *pp = w.part + (int64_t)rep * 3 * P * P;
  for (int e = tid; e < 3 * NT * NT * 256; e += 64 * BW) {
    const int l = e & 63, g = (e >> 6) & 3, blk = e >> 8;
    const int b = blk % NT, a = (blk / NT) % NT, m3 = blk / (NT * NT);
    pp[m3 * P * P + (16 * a + 4 * g + (l >> 4)) * P + 16 * b + (l & 15)] = red[e];
  }
}

// End b of the Chebyshev filter's damping interval [0, b]: theta_p, the
// block's smallest Ritz value (above every unwanted eigenvalue once the block
// has converged a little), or after the first Rayleigh-Ritz step of a warm
// start at least bbeta * theta_k: there the guard columns' Ritz values are
// still far below lambda_p (C3: theta_16 ~ 0.8e3 vs lambda_17 ~ 8e3) and
// [0, theta_p] would leave most of the unwanted spectrum undamped, while the
// wanted theta_k is already accurate (b < theta_k keeps every wanted
// eigenvalue amplified; a b short of lambda_{p+1} only slows the filter).
template <int P>
DFM_DEV double filter_end(const double *small, int k, int p, double bbeta) {
  const double tp = small[2 * P * P + p - 1];
  return bbeta > 0.0 ? fmax(tp, bbeta * small[2 * P * P + k - 1]) : tp;
}

// One 16-row tile's operands for ap2 (ap2_load_lds): Q and Y rows in A-operand layout
// (row t0 + (lane & 15), column 4kk + (lane >> 4)), F rows for a = F'Qn in
// A-operand layout per row group g (row t0 + 4g + (lane >> 4), factor lane & 15),
// and (init) Q in the accumulator layout.  Rows >= T read row T-1 (masked later).
template <int P>
struct Ap2Tile {
  double qa[P / 4], yo[P / 4], fa[4], q[P / 16][4];
};

// ap2_load through a wave-private LDS transpose: the tile's Q and Y rows
// (16 x P each) are read with coalesced 16-B loads (4 lanes per 128-B row)
// and re-read from LDS in the MFMA A-operand layout (row lane & 15, column
// 4 kk + (lane >> 4)), instead of 2 P/4 loads that each touch 16 rows.
// Row stride P + 1: conflict-free A-layout reads.  F rows and the init
// layout as ap2_load.
template <int P>
DFM_DEV void ap2_load_lds(Ap2Tile<P> &L, int tile, int T, int r, int lane, int init, const double *__restrict__ Qr,
                          const double *Yr, const FactBase &fb, double *tq, double *ty, int ps) {
  constexpr int NT = P / 16, KP = P / 4, PER = P / 4;   // doubles per lane per matrix
  const int li = lane & 15, lk = lane >> 4, t0 = tile * 16;
  if (!init) {
    const int rr = lane >> 2, c0 = (lane & 3) * PER, t = t0 + rr;
    const bool ok = t < T;
    const int tc = ok ? t : T - 1;
    double2 qv[PER / 2], yv[PER / 2];
#pragma unroll
    for (int j = 0; j < PER / 2; ++j) {
#ifdef DFM_AP2_DIAG_NOLOAD   // (timing diagnostic, WRONG results: no Q / Y tile loads)
      qv[j] = double2{1e-3 * (tc + j), 1e-3 * c0}; yv[j] = double2{1e-3 * c0, 1e-3 * (tc - j)};
#else
      // compact rows (ps columns, ps even): pairs past ps are the zero columns
      const bool in = c0 + 2 * j < ps;
      qv[j] = in ? *reinterpret_cast<const double2 *>(Qr + (int64_t)tc * ps + c0 + 2 * j) : double2{0.0, 0.0};
      yv[j] = in ? *reinterpret_cast<const double2 *>(Yr + (int64_t)tc * ps + c0 + 2 * j) : double2{0.0, 0.0};
#endif
    }
#pragma unroll
    for (int j = 0; j < PER / 2; ++j) {
      tq[rr * (P + 1) + c0 + 2 * j] = ok ? qv[j].x : 0.0;
      tq[rr * (P + 1) + c0 + 2 * j + 1] = ok ? qv[j].y : 0.0;
      ty[rr * (P + 1) + c0 + 2 * j] = ok ? yv[j].x : 0.0;
      ty[rr * (P + 1) + c0 + 2 * j + 1] = ok ? yv[j].y : 0.0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's writes land before its reads
#pragma unroll
    for (int kk = 0; kk < KP; ++kk) {
      L.qa[kk] = tq[li * (P + 1) + 4 * kk + lk];
      L.yo[kk] = ty[li * (P + 1) + 4 * kk + lk];
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < KP; ++kk) { L.qa[kk] = 0.0; L.yo[kk] = 0.0; }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int t = t0 + 4 * g + lk;
    const int tc = min(t, T - 1);
    // only lanes holding a factor column of a row < T load (r = 0, the
    // expanding windows' case without base factors, loads nothing)
    L.fa[g] = (t < T && li < r) ? fb.F[(int64_t)tc * r + li] : 0.0;
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) L.q[ct][g] = (init && 16 * ct + li < ps) ? Qr[(int64_t)tc * ps + 16 * ct + li] : 0.0;
  }
}

// Shared tail of ap2 and the Chebyshev step: Z = P' D Qn by CSR gather
// (bucket s lists t ascending), cc = EL' Z, and the fixed-order wave sums of
// a = F' Qn (aacc, accumulated by the caller) and cc into ab[rep].  STG (the
// prep pass): zst is this wave's LDS staging (16 pz doubles) and a tile's Z
// chunk (16 rows x pz, contiguous in the replicate-major layout) leaves as
// 16-B pieces instead of one 128-B-strided element per lane — prep -3 %; in
// ap2 / the last Horner step the same staging measured +0.3 % (round 6, item
// 13 of profiles/r06_c3_ab.txt), so they store directly.
template <int P, bool STG>
DFM_DEV void zscatter_tail(const FactBase &fb, int T, int r, int ntile, int tid, int wave, int lane,
                           const double *set, const int *so, const int *sl, const double *Qn,
                           double *__restrict__ Zc, int pz, int rep, double *__restrict__ ab,
                           const dv4 *aacc, double *sred, int ps, double *zst, const double *apre) {
  const int64_t zrs = zrm_stride(T, pz);
  constexpr int NT = P / 16;
  const int li = lane & 15, lk = lane >> 4;
  dv4 cacc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) cacc[ct] = dv4{0.0, 0.0, 0.0, 0.0};
  for (int tile = wave; tile < ntile; tile += BW) {
    const int s0 = tile * 16;
    // all four row groups' first GU bucket entries are fetched together
    // (independent loads in flight); longer buckets finish serially
    constexpr int GU = 3;
    double z[4][NT];
    int qn0[4], qn1[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = s0 + 4 * g + lk;
      qn0[g] = s < T ? so[s] : 0;
      qn1[g] = s < T ? so[s + 1] : 0;
    }
    double val[4][GU][NT], ev[4][GU];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int q = qn0[g] + u;
        const bool ok = q < qn1[g];
        const int t = sl[ok ? q : 0];
        ev[g][u] = ok ? set[t] : 0.0;
        // (lanes past their bucket issue no load: most second / third entries
        // are empty, and these passes are bound by the texture-address unit)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
          val[g][u][ct] = (ok && 16 * ct + li < ps) ? Qn[(int64_t)t * ps + 16 * ct + li] : 0.0;
      }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < GU; ++u) acc = fma(ev[g][u], val[g][u][ct], acc);
        z[g][ct] = acc;
      }
      for (int q = qn0[g] + GU; q < qn1[g]; ++q) {
        const int t = sl[q];
        const double e = set[t];
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
          z[g][ct] = fma(e, 16 * ct + li < ps ? Qn[(int64_t)t * ps + 16 * ct + li] : 0.0, z[g][ct]);
      }
    }
    if constexpr (STG) {
      // (rows past T: 0, the chunk's pad-row value the H.Z GEMM's k-padding needs)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous tile's staged reads are done
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
          if (16 * ct + li < pz) zst[16 * (16 * ct + li) + 4 * g + lk] = s0 + 4 * g + lk < T ? z[g][ct] : 0.0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      double2 *zc2 = reinterpret_cast<double2 *>(Zc + (int64_t)rep * zrs + (int64_t)tile * 16 * pz);
      for (int e = lane; e < 8 * pz; e += 64) zc2[e] = double2{zst[2 * e], zst[2 * e + 1]};
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = s0 + 4 * g + lk;
      const bool v = s < T;
      const double ea = (v && li < r) ? fb.EL[(int64_t)s * r + li] : 0.0;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        if (!STG && v && 16 * ct + li < pz) Zc[zrm_ix(rep, s, 16 * ct + li, pz, zrs)] = z[g][ct];
        cacc[ct] = mfma16(ea, z[g][ct], cacc[ct]);
      }
    }
  }
  // a and cc: fixed-order sums over the waves -> ab[rep] = [a (16 x P); cc (16 x P)]
  // (apre: a was formed once for the whole batch, prep_a_kernel — the same sums)
  double *abr = ab + (int64_t)rep * 32 * P;
  if (apre)
    for (int e = tid; e < 16 * P; e += 64 * BW) abr[e] = apre[e];
  for (int pass = apre ? 1 : 0; pass < 2; ++pass) {
    for (int wv = 0; wv < BW; ++wv) {
      if (wave == wv)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int e = (ct * 4 + g) * 64 + lane;
            const double v = pass ? cacc[ct][g] : aacc[ct][g];
            sred[e] = (wv ? sred[e] : 0.0) + v;
          }
      __syncthreads();
    }
    for (int e = tid; e < NT * 256; e += 64 * BW) {
      const int l = e & 63, g = (e >> 6) & 3, ct = e >> 8;
      abr[pass * 16 * P + (4 * g + (l >> 4)) * P + 16 * ct + (l & 15)] = sred[e];
    }
    __syncthreads();
  }
}

// ap2: one workgroup per replicate.  init = 1: Qn := Q (the warm start), no
// Ritz step.  Qn goes to global memory (over the Y rows this wave just read)
// and is gathered back through the CSR after the barrier: same-CU L1, so the
// workgroup-scope fence of __syncthreads makes it visible.  Dynamic LDS:
// eta (T doubles), off (T+1 ints), lst (T ints) of this replicate.
template <int P>
// 4 workgroups per CU (see boot_y2_kernel)
__global__ __launch_bounds__(64 * BW, 4) void boot_ap2_kernel(FactBase fb, EigWork w, int T, int k, int p, double tol,
                                                       int it, int init, int last, int cheb, double fa1,
                                                       double fa0, double bbeta, const double *__restrict__ eta,
                                                       const int *__restrict__ off, const int *__restrict__ lst,
                                                       const double *__restrict__ Qc, int64_t qs,
                                                       double *__restrict__ Yq, double *__restrict__ Zc, int64_t ldz,
                                                       int pz, double *__restrict__ ab, uint64_t seed, int ps) {
  constexpr int NT = P / 16, KP = P / 4;
  const int rep = blockIdx.x;
  if (!init && w.done[rep]) return;
  extern __shared__ double sdyn[];
  double *set = sdyn;                          // eta_t
  int *so = (int *)(sdyn + T), *sl = so + T + 1;
  __shared__ double sred[NT * 256];
  __shared__ double sres[BW][P];
  __shared__ double stile[BW][2][16 * (P + 1)];   // per-wave Q / Y tile transposes (ap2_load_lds)
  __shared__ int s_conv;
  __shared__ double sAm[P * P], sBm[P * P];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = fb.r;
  const int li = lane & 15, lk = lane >> 4;
  {
    const double *et = eta ? eta + (int64_t)rep * T : nullptr;
    const int *o = off + (int64_t)rep * (T + 1);
    const int *L = lst + (int64_t)rep * T;
    for (int e = tid; e < T; e += 64 * BW) { set[e] = et ? et[e] : 1.0; so[e] = o[e]; sl[e] = L[e]; }
    if (tid == 0) so[T] = o[T];
  }
  double *small = w.small + (int64_t)rep * small_stride<P>();
  // the Rayleigh-Ritz step's A and Bm (P x P each) in LDS: the MFMA B
  // operands are read per tile instead of held in 2 KP NT registers (round 6:
  // the kernel sat at 128 VGPRs with 32 B of scratch)
  for (int e = tid; e < P * P; e += 64 * BW) {
    sAm[e] = init ? 0.0 : small[e];
    sBm[e] = init ? 0.0 : small[P * P + e];
  }
  double th[NT];
  bool dd[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) {
    const int c = 16 * ct + li;
    th[ct] = init ? 0.0 : small[2 * P * P + c];
    dd[ct] = init ? false : (small[2 * P * P + P + c] != 0.0);
  }
  __syncthreads();
  const double *Qr = Qc + (int64_t)rep * qs;   // qs = 0: the shared warm start (init / first step)
  double *Yr = Yq + (int64_t)rep * T * P;
  // the filter's first Horner term (boot_cheb_kernel): S = (fa1 / b) Y Bm + fa0 Q Bm,
  // fa1 / fa0 = T*_d's y^d / y^(d-1) coefficients, b = filter_end
  const double bch = init ? 0.0 : filter_end<P>(small, k, p, bbeta);
  const double cf1 = bch > 0.0 ? fa1 / bch : 1.0, cf0 = bch > 0.0 ? fa0 : 0.0;
  double res2[NT];
  dv4 aacc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) { res2[ct] = 0.0; aacc[ct] = dv4{0.0, 0.0, 0.0, 0.0}; }
  const int ntile = (T + 15) >> 4;
  // each tile's operands load at the top of its iteration (occupancy hides the latency)
  Ap2Tile<P> cur;
  for (int tile = wave; tile < ntile; tile += BW) {
    ap2_load_lds<P>(cur, tile, T, r, lane, init, Qr, Yr, fb, stile[wave][0], stile[wave][1], ps);
    const int t0 = tile * 16;
    double qv[NT][4];
    if (init) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) qv[ct][g] = (t0 + 4 * g + lk < T) ? cur.q[ct][g] : 0.0;
    } else {
      dv4 u[NT], ya[NT], qn[NT], qb[NT];
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) { u[ct] = dv4{0.0, 0.0, 0.0, 0.0}; ya[ct] = u[ct]; qn[ct] = u[ct]; qb[ct] = u[ct]; }
#pragma unroll
      for (int kk = 0; kk < KP; ++kk)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          const double am = sAm[(4 * kk + lk) * P + 16 * ct + li], bm = sBm[(4 * kk + lk) * P + 16 * ct + li];
          u[ct] = mfma16(cur.qa[kk], am, u[ct]);
          ya[ct] = mfma16(cur.yo[kk], am, ya[ct]);
          qn[ct] = mfma16(cur.yo[kk], bm, qn[ct]);
          if (cheb) qb[ct] = mfma16(cur.qa[kk], bm, qb[ct]);
        }
      if (cheb) {   // V0 = Q Bm for the filter's later steps (boot_cheb_kernel), kept in w.U
        double *Xr = w.U + (int64_t)rep * T * P;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int t = t0 + 4 * g + lk;
          if (t < T)
#pragma unroll
            for (int ct = 0; ct < NT; ++ct) {
              const int c = 16 * ct + li;
              double x = qb[ct][g];
              if (c < p && dd[ct]) x = hash_unit(seed, t, 1000003ull * (it + 1) + c);   // = S
              if (c >= p) x = 0.0;
              if (c < ps) Xr[(int64_t)t * ps + c] = x;
            }
        }
      }
      // every wave reads only its own tiles' Y rows, loaded (above) before
      // these stores: Qn may overwrite this tile's Y rows
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int t = t0 + 4 * g + lk;
        const bool v = t < T;
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          const int c = 16 * ct + li;
          const double wr = ya[ct][g] - th[ct] * u[ct][g];
          if (v && c < k) res2[ct] = fma(wr, wr, res2[ct]);
          // the filter's first Horner term S_{d-1} = (a_d / b) K_1 + a_{d-1} V0
          // (K_1 = Y Bm = G* V0), or the plain power step Y Bm
          double q = cheb ? fma(cf1, qn[ct][g], cf0 * qb[ct][g]) : qn[ct][g];
          if (c < p && dd[ct]) q = hash_unit(seed, t, 1000003ull * (it + 1) + c);
          if (c >= p || !v) q = 0.0;
          qv[ct][g] = q;
          if (v && c < ps) Yr[(int64_t)t * ps + c] = q;
        }
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) aacc[ct] = mfma16(cur.fa[g], qv[ct][g], aacc[ct]);
  }
  // residuals: sum over the 4 row-lanes of a column, then over waves (fixed order)
  if (!init) {
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      double v = res2[ct];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lk == 0) sres[wave][16 * ct + li] = v;
    }
  }
  __syncthreads();
  if (wave == 0) {
    int conv = 0;
    if (!init) {
      if (lane < P) {
        double v = sres[0][lane];
#pragma unroll
        for (int wv = 1; wv < BW; ++wv) v += sres[wv][lane];
        sres[0][lane] = v;
      }
      __builtin_amdgcn_wave_barrier();
      const int itc = it + 1;
      const double *prev = small + 2 * P * P + 2 * P + ((itc - 1) & 1) * P;
      double *next = small + 2 * P * P + 2 * P + (itc & 1) * P;
      conv = decide_converged(sres[0], small + 2 * P * P, prev, next, k, p, tol, w.trace[rep], itc, w.subspace) ? 1 : 0;
#ifdef DFM_DIAG_X
      diag_excess(sres[0], small + 2 * P * P, k, p, tol, w.trace[rep], rep, it);
#endif
    }
    if (lane == 0) {
      s_conv = conv;
      if (conv) { w.done[rep] = 1; w.iters[rep] = it + 1; }
      else if (!init) atomicAdd(&w.active[it], 1);
    }
  }
  __syncthreads();
  if (!init && (s_conv || last)) {
    if (w.no_vectors) return;   // eigenvalue-only statistics: eig_final reads theta only
    // Ritz vectors U = Q A for the final output (eig_final_kernel)
    double *Ur = w.U + (int64_t)rep * T * P;
    for (int tile = wave; tile < ntile; tile += BW) {
      const int t0 = tile * 16, ta = t0 + li;
      dv4 u[NT];
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) u[ct] = dv4{0.0, 0.0, 0.0, 0.0};
      double qa[KP];
#pragma unroll
      for (int kk = 0; kk < KP; ++kk) qa[kk] = (ta < T && 4 * kk + lk < ps) ? Qr[(int64_t)ta * ps + 4 * kk + lk] : 0.0;
#pragma unroll
      for (int kk = 0; kk < KP; ++kk)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) u[ct] = mfma16(qa[kk], sAm[(4 * kk + lk) * P + 16 * ct + li], u[ct]);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int t = t0 + 4 * g + lk;
        if (t < T)
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) Ur[(int64_t)t * P + 16 * ct + li] = u[ct][g];
      }
    }
    return;
  }
  // Z = P' D Qn by CSR gather (bucket s lists t ascending), cc = EL' Z
  const double *Qn = init ? Qr : Yr;
  zscatter_tail<P, false>(fb, T, r, ntile, tid, wave, lane, set, so, sl, Qn, Zc, pz, rep, ab, aacc, sred, ps, nullptr);
}

// One Horner step of the degree-d Chebyshev filter of the factored solver.
// With V0 = Q Bm and y = G*/b (b = filter_end), the filter is the shifted
// Chebyshev polynomial T*_d(y) = T_d(2y - 1) = sum_i a_i y^i, evaluated as
// S_d = a_d V0, S_i = G* S_{i+1} / b + a_i V0, T*_d(y) V0 = S_0: ap2 leaves
// S_{d-1} = (a_d / b) K_1 + a_{d-1} V0 (K_1 = Y Bm = G* V0, no product) with
// its Z, a, cc, and V0 in w.U; each step gets W = G* S_{i+1} from the GEMM
// H . Z(S_{i+1}) (formed exactly as y2 forms Y) and writes S_i = W / b + a_i V0
// with the Z, a, cc of S_i for the next GEMM (or, S_0, the next Rayleigh-Ritz
// step).  The same step serves the middle and the end of the filter, with
// one running vector (the monomial form also rewrote a running sum per
// step).  Degree 2: T2(2G/b - 1)(Q Bm) = (8/b^2) G*^2 V0 - (8/b) G* V0 + V0.
// The filter damps the unwanted spectrum ~T_d(2 lambda_k/b - 1) times
// relative to the wanted one; the basis is orthonormalised by the next
// Rayleigh-Ritz step (CholQR folded into eig_small).
template <int P, bool STG>
__global__ __launch_bounds__(64 * BW, 4) void boot_cheb_kernel(FactBase fb, EigWork w, int T, int p,
                                                        const int32_t *__restrict__ idx,
                                                        const double *__restrict__ eta,
                                                        const int *__restrict__ off, const int *__restrict__ lst,
                                                        const double *__restrict__ HZ, int64_t ldz, int pz,
                                                        double *__restrict__ ab, double fai, double bbeta, int k,
                                                        double *__restrict__ Qo,
                                                        double *__restrict__ Zc, int ps) {
  constexpr int NT = P / 16;
  const int rep = blockIdx.x;
  if (w.done[rep]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = fb.r;
  const int li = lane & 15, lk = lane >> 4;
  __shared__ double sa[16 * P], sb[16 * P];
  __shared__ double sred[NT * 256];
  __shared__ double stg[STG ? BW : 1][STG ? Y2_STG : 1];   // per-wave operand staging (y2_load)
  extern __shared__ double sdyn[];
  double *set = sdyn;                          // eta_t
  int *six = (int *)(sdyn + T);                // idx_t
  int *so = six + T, *sl = so + T + 1;         // CSR of idx
  {
    const int32_t *ixg = idx + (int64_t)rep * T;
    const double *etg = eta ? eta + (int64_t)rep * T : nullptr;
    const int *o = off + (int64_t)rep * (T + 1);
    const int *L = lst + (int64_t)rep * T;
    for (int e = tid; e < T; e += 64 * BW) { six[e] = ixg[e]; set[e] = etg ? etg[e] : 1.0; so[e] = o[e]; sl[e] = L[e]; }
    if (tid == 0) so[T] = o[T];
  }
  double *abr = ab + (int64_t)rep * 32 * P;
  for (int e = tid; e < 16 * P; e += 64 * BW) sa[e] = abr[e];
  __syncthreads();
  for (int e = tid; e < 16 * P; e += 64 * BW) {
    const int j = e / P, c = e % P;
    double v = abr[16 * P + e];
    if (j < r)
      for (int i = 0; i < r; ++i) v = fma(fb.S[j * r + i], sa[i * P + c], v);
    sb[e] = v;
  }
  __syncthreads();
  const double *small = w.small + (int64_t)rep * small_stride<P>();
  const double b = filter_end<P>(small, k, p, bbeta);
  // b <= 0 (a degenerate block): plain power steps
  const double cb = b > 0.0 ? 1.0 / b : 1.0, cv0 = b > 0.0 ? fai : 0.0;
  bool dd[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) dd[ct] = small[2 * P * P + P + 16 * ct + li] != 0.0;
  const int KR = (r + 3) >> 2;
  double bA[4][NT], bB[4][NT];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      bA[kk][ct] = sa[(4 * kk + lk) * P + 16 * ct + li];
      bB[kk][ct] = sb[(4 * kk + lk) * P + 16 * ct + li];
    }
  const double *Xr = w.U + (int64_t)rep * T * P;   // V0 = Q Bm (ap2)
  double *Qr = Qo + (int64_t)rep * T * P;
  dv4 aacc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) aacc[ct] = dv4{0.0, 0.0, 0.0, 0.0};
  const int ntile = (T + 15) >> 4;
  Y2Tile<P> cur;
  for (int tile = wave; tile < ntile; tile += BW) {
    y2_load<P, STG>(cur, tile, T, r, KR, lane, six, fb, HZ, ldz, pz, rep, Xr, ps, stg[STG ? wave : 0]);   // cur.q = V0 rows
    const int t0 = tile * 16;
    dv4 yF[NT], yE[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) { yF[ct] = dv4{0.0, 0.0, 0.0, 0.0}; yE[ct] = yF[ct]; }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < KR) {
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          yF[ct] = mfma16(cur.fA[kk], bB[kk][ct], yF[ct]);
          yE[ct] = mfma16(cur.eA[kk], bA[kk][ct], yE[ct]);
        }
      }
    }
    double qv[NT][4], fa[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int t = t0 + 4 * g + lk;
      const bool v = t < T;
      const int tc = min(t, T - 1);
      if constexpr (STG)
        fa[g] = (v && li < r) ? stg[wave][(4 * g + lk) * (r + 1) + li] : 0.0;
      else
        fa[g] = (v && li < r) ? fb.F[(int64_t)tc * r + min(li, max(r - 1, 0))] : 0.0;   // never F[-1] (r = 0)
      const double e = v ? set[t] : 0.0;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        const int c = 16 * ct + li;
        const double wv = fma(e, yE[ct][g] + cur.hz[ct][g], yF[ct][g]);
        double q = dd[ct] ? cur.q[ct][g] : fma(cb, wv, cv0 * cur.q[ct][g]);
        if (c >= p || !v) q = 0.0;
        qv[ct][g] = q;
        if (v && c < ps) Qr[(int64_t)t * ps + c] = q;
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) aacc[ct] = mfma16(fa[g], qv[ct][g], aacc[ct]);
  }
  __syncthreads();   // every wave's Qn rows visible to the CSR gather
  zscatter_tail<P, false>(fb, T, r, ntile, tid, wave, lane, set, so, sl, Qr, Zc, pz, rep, ab, aacc, sred, ps, nullptr);
}

// The middle Horner steps in row-local form.  With W = G* S_{i+1} = F bB +
// D P u (bB = S a + cc, u = EL a + HZ, a / cc of S_{i+1}) and S_i = W / b +
// a_i V0, the next GEMM operand and the step's reductions need no S_i rows:
//   Z_i = P'D S_i = (PF bB + e2 . u) / b + a_i PV,
//   a_i = F'S_i   = (F'F bB + PF'u) / b + a_i FV,     cc_i = EL'Z_i,
// with PF = P'D F, e2 = P'D^2 1 (boot_prep_kernel, once per solve), PV = P'D V0
// and FV = F'V0 (ap2, once per filter).  Every row s reads HZ[s], PV[s],
// PF[s], e2[s], EL[s] and writes Z[s]: no CSR gather, no S_i write and
// re-read, no barrier between the two (the last step, which must hand S_0 to
// the next Rayleigh-Ritz step, stays boot_cheb_kernel).  Columns that
// deflated (dd) carry V0: Z = PV, a = FV; columns >= p are zero.
// F'F (16 x 16, rows / columns >= r zero), one workgroup: four row quarters
// per entry (t ascending in each), summed in a fixed order
__global__ __launch_bounds__(1024) void ftf_kernel(FactBase fb, double *__restrict__ FtF) {
  __shared__ double part[4][256];
  const int e = threadIdx.x & 255, q = threadIdx.x >> 8, j = e >> 4, i = e & 15, r = fb.r;
  const int t0 = q * ((fb.T + 3) / 4), t1 = min(fb.T, t0 + (fb.T + 3) / 4);
  double acc = 0.0;
  if (j < r && i < r) {
    // 8 rows' loads in flight before their (in-order) products: the one-row
    // loop was ~125 dependent L2 round trips (30-40 us on every lane's stream)
    int t = t0;
    for (; t + 8 <= t1; t += 8) {
      double a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) { a[u] = fb.F[(int64_t)(t + u) * r + j]; b[u] = fb.F[(int64_t)(t + u) * r + i]; }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fma(a[u], b[u], acc);
    }
    for (; t < t1; ++t) acc = fma(fb.F[(int64_t)t * r + j], fb.F[(int64_t)t * r + i], acc);
  }
  part[q][e] = acc;
  __syncthreads();
  if (q == 0) FtF[e] = (part[0][e] + part[1][e]) + (part[2][e] + part[3][e]);
}

// fixed-order sum over the waves of a 16 x P accumulator block -> dst (row-major, stride P)
template <int P>
DFM_DEV void wave_block_store(const dv4 *acc, double *sred, int wave, int lane, int tid, double *__restrict__ dst) {
  constexpr int NT = P / 16;
  for (int wv = 0; wv < BW; ++wv) {
    if (wave == wv)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int e = (ct * 4 + g) * 64 + lane;
          sred[e] = (wv ? sred[e] : 0.0) + acc[ct][g];
        }
    __syncthreads();
  }
  if (dst)
    for (int e = tid; e < NT * 256; e += 64 * BW) {
      const int l = e & 63, g = (e >> 6) & 3, ct = e >> 8;
      dst[(4 * g + (l >> 4)) * P + 16 * ct + (l & 15)] = sred[e];
    }
}

// PV = P'D V0 and FV = F'V0 for a filter with middle steps, launched between
// the Rayleigh-Ritz step's eig_small and ap2: V0 = Q Bm is linear in Q, so
// PV = Z(Q) Bm and FV = a(Q) Bm from the Z = P'D Q and a = F'Q that the
// previous step left in Zc / ab (ap2 overwrites both) — row-local, no CSR
// gather of V0.  Columns that ap2 refills (dead pivots: V0 = hash_unit) take
// the explicit sums over their buckets / rows.
template <int P>
__global__ __launch_bounds__(64 * BW, 4) void boot_pv_kernel(FactBase fb, EigWork w, int T, int p, int it,
                                                      const double *__restrict__ eta, const int *__restrict__ off,
                                                      const int *__restrict__ lst, const double *__restrict__ Zc,
                                                      int64_t ldz, int pz, const double *__restrict__ ab, uint64_t seed,
                                                      double *__restrict__ PV, double *__restrict__ FV, int ps) {
  constexpr int NT = P / 16, KP = P / 4;
  const int rep = blockIdx.x;
  if (w.done[rep]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = fb.r;
  const int li = lane & 15, lk = lane >> 4;
  const double *small = w.small + (int64_t)rep * small_stride<P>();
  const uint64_t hc = 1000003ull * (it + 1);
  double bBm[KP][NT];
  bool dd[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) {
    const int c = 16 * ct + li;
    dd[ct] = small[2 * P * P + P + c] != 0.0;
#pragma unroll
    for (int kk = 0; kk < KP; ++kk) bBm[kk][ct] = small[P * P + (4 * kk + lk) * P + c];
  }
  const double *et = eta ? eta + (int64_t)rep * T : nullptr;
  const int *o = off + (int64_t)rep * (T + 1);
  const int *L = lst + (int64_t)rep * T;
  double *pvr = PV + (int64_t)rep * T * P;
  const int ntile = (T + 15) >> 4;
  for (int tile = wave; tile < ntile; tile += BW) {
    const int t0 = tile * 16, ta = min(t0 + li, T - 1);
    double za[KP];
#pragma unroll
    for (int kk = 0; kk < KP; ++kk)
      za[kk] = (t0 + li < T && 4 * kk + lk < pz) ? Zc[zrm_ix(rep, ta, 4 * kk + lk, pz, zrm_stride(T, pz))] : 0.0;
    dv4 v[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) v[ct] = dv4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < KP; ++kk)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) v[ct] = mfma16(za[kk], bBm[kk][ct], v[ct]);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = t0 + 4 * g + lk;
      if (s < T)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          const int c = 16 * ct + li;
          double x = v[ct][g];
          if (c < p && dd[ct]) {   // refilled column: sum over bucket s (t ascending)
            x = 0.0;
            for (int q = o[s]; q < o[s + 1]; ++q) {
              const int t = L[q];
              x = fma(et ? et[t] : 1.0, hash_unit(seed, t, hc + c), x);
            }
          }
          if (c >= p) x = 0.0;
          if (c < ps) pvr[(int64_t)s * ps + c] = x;
        }
    }
  }
  const double *aq = ab + (int64_t)rep * 32 * P;
  double *fvr = FV + (int64_t)rep * 16 * P;
  for (int e = tid; e < 16 * P; e += 64 * BW) {
    const int j = e / P, c = e % P;
    double x = 0.0;
    if (j < r && c < p) {
      if (small[2 * P * P + P + c] != 0.0) {
        for (int t = 0; t < T; ++t) x = fma(fb.F[(int64_t)t * r + j], hash_unit(seed, t, hc + c), x);
      } else {
        for (int i = 0; i < P; ++i) x = fma(aq[j * P + i], small[P * P + i * P + c], x);
      }
    }
    fvr[e] = x;
  }
}

template <int P, bool FAST>
__global__ __launch_bounds__(64 * BW, 4) void boot_cheb_mid_kernel(FactBase fb, EigWork w, int T, int p,
                                                            const double *__restrict__ HZ, int64_t ldz, int pz,
                                                            double *__restrict__ ab, double fai, double bbeta, int k,
                                                            const double *__restrict__ PF,
                                                            const double *__restrict__ E2,
                                                            const double *__restrict__ PV,
                                                            const double *__restrict__ FV,
                                                            const double *__restrict__ FtF,
                                                            double *__restrict__ Zc, int ps) {
  constexpr int NT = P / 16;
  const int rep = blockIdx.x;
  if (w.done[rep]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = fb.r;
  const int li = lane & 15, lk = lane >> 4;
  __shared__ double sa[16 * P], sb[16 * P];
  __shared__ double sred[NT * 256];
  // per-wave staging (round 6: this pass is bound by the texture-address unit,
  // TA_TA_BUSY 0.95 of its cycles): the tile's PF and EL rows arrive as ONE
  // contiguous 16-row range each (16 r doubles) instead of two differently
  // shaped gathers of the same rows, and the tile's Z chunk (16 rows x pz,
  // contiguous in the replicate-major layout) leaves as whole 16-B pieces
  // instead of one 128-B-strided element per lane
  __shared__ double stg[BW][2][16 * 17];
  double *abr = ab + (int64_t)rep * 32 * P;
  for (int e = tid; e < 16 * P; e += 64 * BW) sa[e] = abr[e];
  __syncthreads();
  for (int e = tid; e < 16 * P; e += 64 * BW) {
    const int j = e / P, c = e % P;
    double v = abr[16 * P + e];
    if (j < r)
      for (int i = 0; i < r; ++i) v = fma(fb.S[j * r + i], sa[i * P + c], v);
    sb[e] = v;
  }
  __syncthreads();
  const double *small = w.small + (int64_t)rep * small_stride<P>();
  const double b = filter_end<P>(small, k, p, bbeta);
  const double cb = b > 0.0 ? 1.0 / b : 1.0, cv0 = b > 0.0 ? fai : 0.0;
  bool dd[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) dd[ct] = small[2 * P * P + P + 16 * ct + li] != 0.0;
  const int KR = (r + 3) >> 2;
  const double *pfr = PF + (int64_t)rep * T * r, *e2r = E2 + (int64_t)rep * T, *pvr = PV + (int64_t)rep * T * P;
  dv4 aacc[NT], cacc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct) { aacc[ct] = dv4{0.0, 0.0, 0.0, 0.0}; cacc[ct] = aacc[ct]; }
  const int ntile = (T + 15) >> 4;
  const int RS = r | 1;   // staged row stride (odd: the 16-row reads spread over the banks)
  double *sP = stg[wave][0], *sE = stg[wave][1];
  const int64_t zrs = zrm_stride(T, pz);
  for (int tile = wave; tile < ntile; tile += BW) {
    const int t0 = tile * 16;
    const int nr = min(16, T - t0) * r;   // valid doubles of the tile's contiguous PF / EL range
    double hz[NT][4], pv[NT][4], e2v[4];
    double pst[4], est[4];
    double2 pst2 = double2{0.0, 0.0}, est2 = double2{0.0, 0.0};
    if constexpr (FAST) {   // even r <= 8: the 8 r <= 64 pieces of 16 B, one round
      const bool ok = 2 * lane < nr;
      pst2 = ok ? reinterpret_cast<const double2 *>(pfr + (int64_t)t0 * r)[lane] : double2{0.0, 0.0};
      est2 = ok ? reinterpret_cast<const double2 *>(fb.EL + (int64_t)t0 * r)[lane] : double2{0.0, 0.0};
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {   // 16 r <= 256 doubles: four rounds of 64 lanes
        const int e = u * 64 + lane;
        pst[u] = e < nr ? pfr[(int64_t)t0 * r + e] : 0.0;
        est[u] = e < nr ? fb.EL[(int64_t)t0 * r + e] : 0.0;
      }
    }
    const double e2l = t0 + li < T ? e2r[t0 + li] : 0.0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = t0 + 4 * g + lk;
      const int sc = min(s, T - 1);
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        const int c = 16 * ct + li;
        hz[ct][g] = c < pz ? HZ[(int64_t)sc * ldz + (int64_t)rep * pz + c] : 0.0;
        pv[ct][g] = c < ps ? pvr[(int64_t)sc * ps + c] : 0.0;
      }
    }
    if constexpr (FAST) {
      if (2 * lane < 16 * r) {
        const int e = 2 * lane, row = e / r, j = e - row * r;
        sP[row * RS + j] = pst2.x; sP[row * RS + j + 1] = pst2.y;
        sE[row * RS + j] = est2.x; sE[row * RS + j + 1] = est2.y;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = u * 64 + lane;
        if (e < 16 * r) {
          const int row = e / r, j = e - row * r;
          sP[row * RS + j] = pst[u];
          sE[row * RS + j] = est[u];
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's writes land before its reads
    double pA[4], eA[4], pfa[4], ea[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int j = 4 * kk + lk;
      const bool ok = kk < KR && j < r && t0 + li < T;
      pA[kk] = ok ? sP[li * RS + j] : 0.0;
      eA[kk] = ok ? sE[li * RS + j] : 0.0;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = t0 + 4 * g + lk;
      const bool v = s < T;
      e2v[g] = v ? __shfl(e2l, 4 * g + lk, 16) : 0.0;
      pfa[g] = (v && li < r) ? sP[(4 * g + lk) * RS + li] : 0.0;
      ea[g] = (v && li < r) ? sE[(4 * g + lk) * RS + li] : 0.0;
    }
    dv4 yP[NT], yE[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) { yP[ct] = dv4{0.0, 0.0, 0.0, 0.0}; yE[ct] = yP[ct]; }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < KR) {   // B operands a / bB from LDS (registers are this kernel's limit)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {
          yP[ct] = mfma16(pA[kk], sb[(4 * kk + lk) * P + 16 * ct + li], yP[ct]);
          yE[ct] = mfma16(eA[kk], sa[(4 * kk + lk) * P + 16 * ct + li], yE[ct]);
        }
      }
    }
    double uv[NT][4], zv[NT][4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int s = t0 + 4 * g + lk;
      const bool v = s < T;
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        const int c = 16 * ct + li;
        const double u = yE[ct][g] + hz[ct][g];
        double z = dd[ct] ? pv[ct][g] : fma(cb, fma(e2v[g], u, yP[ct][g]), cv0 * pv[ct][g]);
        if (c >= p || !v) z = 0.0;
        uv[ct][g] = v ? u : 0.0;
        zv[ct][g] = z;
      }
    }
    // the Z chunk through the PF staging (its reads above are complete in
    // this wave's LDS order): chunk element 16 c + (s & 15); rows past T hold
    // z = 0, the value boot_prep_kernel left in the chunk's pad rows
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        const int c = 16 * ct + li;
        if (c < pz) sP[16 * c + 4 * g + lk] = zv[ct][g];
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    {
      double2 *zc2 = reinterpret_cast<double2 *>(Zc + (int64_t)rep * zrs + (int64_t)tile * 16 * pz);
      for (int e = lane; e < 8 * pz; e += 64) zc2[e] = double2{sP[2 * e], sP[2 * e + 1]};
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        aacc[ct] = mfma16(pfa[g], uv[ct][g], aacc[ct]);
        cacc[ct] = mfma16(ea[g], zv[ct][g], cacc[ct]);
      }
  }
  // a_i = (F'F bB + PF'u) / b + a_i FV  (dd columns: FV; columns >= p: 0)
  wave_block_store<P>(aacc, sred, wave, lane, tid, nullptr);
  const double *fvr = FV + (int64_t)rep * 16 * P;
  for (int e = tid; e < 16 * P; e += 64 * BW) {
    const int j = e / P, c = e % P;
    const int ct = c >> 4, l = ((j & 3) << 4) | (c & 15), g = j >> 2;
    double a = 0.0;
    if (j < r && c < p) {
      if (small[2 * P * P + P + c] != 0.0) a = fvr[e];
      else {
        double f = 0.0;
        for (int i = 0; i < r; ++i) f = fma(FtF[j * 16 + i], sb[i * P + c], f);
        a = fma(cb, f + sred[(ct * 4 + g) * 64 + l], cv0 * fvr[e]);
      }
    }
    abr[e] = a;
  }
  __syncthreads();
  wave_block_store<P>(cacc, sred, wave, lane, tid, abr + 16 * P);
}

// Ascending list of the still-active replicates (done == 0) and their count,
// one 1024-thread workgroup: per-thread chunk counts, an LDS scan, in-order
// writes.  Feeds the compacted H.Z GEMM of the straggler phase.
__global__ __launch_bounds__(256) void zero_spans_kernel(ZeroSpans z) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
#pragma unroll
  for (int s = 0; s < 4; ++s)
    for (int64_t i = i0; i < z.n[s]; i += stride) z.p[s][i] = 0;
}
hipError_t launch_zero_spans(const ZeroSpans &z, hipStream_t st) {
  int64_t mx = 0;
  for (int s = 0; s < 4; ++s) mx = std::max<int64_t>(mx, z.p[s] ? z.n[s] : 0);
  if (mx == 0) return hipSuccess;
  ZeroSpans c = z;
  for (int s = 0; s < 4; ++s)
    if (!c.p[s]) c.n[s] = 0;
  hipLaunchKernelGGL(zero_spans_kernel, dim3((unsigned)std::min<int64_t>(512, (mx + 255) / 256)), dim3(256), 0, st, c);
  return hipGetLastError();
}

__global__ __launch_bounds__(1024) void active_list_kernel(const int *__restrict__ done, int nb,
                                                           int *__restrict__ list, int *__restrict__ count) {
  __shared__ int part[1024];
  const int tid = threadIdx.x, per = (nb + 1023) / 1024;
  const int b0 = min(nb, tid * per), b1 = min(nb, b0 + per);
  int c = 0;
  for (int i = b0; i < b1; ++i) c += done[i] ? 0 : 1;
  part[tid] = c;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int pos = part[tid] - c;
  for (int i = b0; i < b1; ++i)
    if (!done[i]) list[pos++] = i;
  if (tid == 1023) *count = part[1023];
}

// Shifted Chebyshev coefficients T*_d(y) = T_d(2y - 1) = sum_i a_i y^i
// (T*_0 = 1, T*_1 = 2y - 1, T*_{n+1} = 2 (2y - 1) T*_n - T*_{n-1}).
static void shifted_cheb(int d, double *a) {   // a[0..kChebDMax]
  double t0[kChebDMax + 1] = {1.0}, t1[kChebDMax + 1] = {-1.0, 2.0};
  if (d == 0) { for (int i = 0; i <= kChebDMax; ++i) a[i] = t0[i]; return; }
  for (int n = 1; n < d; ++n) {
    double t2[kChebDMax + 1];
    for (int i = 0; i <= kChebDMax; ++i) t2[i] = -2.0 * t1[i] - t0[i] + (i > 0 ? 4.0 * t1[i - 1] : 0.0);
    for (int i = 0; i <= kChebDMax; ++i) { t0[i] = t1[i]; t1[i] = t2[i]; }
  }
  for (int i = 0; i <= kChebDMax; ++i) a[i] = t1[i];
}
// Filter schedule of the factored solver.  From a warm start (the base fit's
// eigenvectors): a degree-6 filter on [0, max(theta_p, 0.2 theta_k)] after
// the first Rayleigh-Ritz step, degree 2 on [0, theta_p] after the later ones.
// C3 (tools/eig_proto.py, the CPU model of this loop; tools/c3_excess.py, the
// convergence excess measured on the GPU): with degree 2 throughout the first
// filter gains only ~3e3 in the eigenvalue bound (theta_16 ~ 0.8e3 far below
// lambda_17 ~ 8e3) against ~5e4 for the later ones, and replicates retire at
// the 4th (96 %) or 5th Rayleigh-Ritz step after 7.09 products; with this
// schedule every replicate of the CPU model retires at the 2nd step after 7
// products — two Rayleigh-Ritz passes and the straggler tail fewer, two more
// Chebyshev passes.  Cold starts (no warm vectors: expanding windows) keep
// degree 2 on [0, theta_p].
constexpr int kChebWarmD0 = 6, kChebD = 2;
constexpr double kChebWarmBeta = 0.2;
// The filter amplifies wanted eigenvalue lambda_1 over lambda_k by about
// T_d(x_1) / T_d(x_k) ~ (x_1 / x_k)^d, x = 2 lambda / b - 1 (x_k = 9 at
// b = 0.2 lambda_k): the filtered block's condition number.  Its degree is
// capped so that stays below ~1e6 (CholQR2 keeps every wanted direction in
// fp64): C3's lambda_1 / lambda_8 = 1.6 allows 6 (the cap); a panel with one
// dominant factor (C2's base fit: lambda_1 / lambda_4 = 50) gets 3.
// DFM_FACT_D0 / DFM_FACT_BETA (A/B only) override the first filter's degree
// cap and interval factor.
static int warm_d0_cap() {
  static const int v = [] { const char *e = getenv("DFM_FACT_D0"); return e ? std::max(kChebD, std::min(kChebDMax, atoi(e))) : kChebWarmD0; }();
  return v;
}
static double warm_beta() {
  static const double v = [] { const char *e = getenv("DFM_FACT_BETA"); return e ? atof(e) : kChebWarmBeta; }();
  return v;
}
static int first_filter_degree(double spread) {
  const double ratio = std::max(1.0001, 1.1 * spread);
  const int d = (int)std::floor(std::log(1e6) / std::log(ratio));
  return std::max(kChebD, std::min(warm_d0_cap(), d));
}

template <int P>
static int eig_run_fact2_t(const FactBase &fb, const int32_t *idx, const double *eta, int nb, int k, int p,
                           const double *warm, int kw, double tol, int maxit, int poll, char *ws,
                           char *fws, double *lam, double *Uk, double *trace_out, int *status,
                           hipStream_t st, timer_fn tf, void *tctx, int *off, int *lst, long long *cnt,
                           int subspace, double spread, const PollBuf *pb) {
  const int m = fb.T;
  EigWork w = carve(ws, m, nb, P, maxit);
  w.subspace = subspace;
  w.no_vectors = Uk == nullptr;
  // Z / HZ hold pz = p rounded up to even columns per replicate (the GEMM's
  // 16-byte DMA pairs): the H.Z GEMM's work scales with the block p, not P
  const int pz = (p + 1) & ~1;
  // (round 6, measured and rejected: Z / HZ rows padded to 128-B lines cut the
  // H.Z GEMM's FETCH_SIZE 0.40 -> 0.32 GB per launch — unpadded, a 512-B tile
  // row straddles five lines, one shared with another XCD's column block — but
  // left the GEMM's time unchanged and slowed the gathering passes 2-4 % with
  // an even or an odd number of lines per row: C3 15.09 -> 15.27-15.38 ms)
  const int ncz = nb * pz;
  const int64_t ldz = ncz;           // HZ: T x nb pz, column-interleaved (rows gathered by idx)
  const int64_t zrs = z_rows(m) * pz;   // Z: replicate-major 16-row chunks (zrm_ix), nb zrs <= z_rows ldz
  // the per-replicate T-row buffers (Q, Y, V0 in U, PV in S, the warm start
  // Q0) hold compact rows of ps = pz columns (columns >= p are zero, so the
  // register layouts' columns ps..P-1 load as zero and are never stored):
  // ~20 % fewer bytes in the per-replicate passes at C3 (P = 16, pz = 12).
  // Replicate slots keep the P-column stride (T P doubles), so a retired
  // replicate's final Ritz vectors (U, row stride P, eig_final_kernel) never
  // overlap another replicate's compact rows.
  const int ps = pz;
  double *Zc = (double *)fws;
  double *HZ = Zc + (size_t)z_rows(m) * ldz;
  double *ab = HZ + (size_t)m * ldz;
  // middle Horner steps' operands (fact_mid_doubles), after ab's region
  double *PFb = ab + (size_t)nb * ((m + EROWS - 1) / EROWS) * 2 * 32 * P + 512;
  double *E2b = PFb + (size_t)nb * m * 16, *FVb = E2b + (size_t)nb * m, *FtF = FVb + (size_t)nb * 16 * P;
  const size_t lds = (size_t)m * 8 + (size_t)(2 * m + 1) * 4;
  {   // counters, flags and Z's zero k-padding rows: one launch
    ZeroSpans zs{};
    zs.p[0] = w.active; zs.n[0] = maxit + 2;
    zs.p[1] = w.iters; zs.n[1] = nb;
    zs.p[2] = w.done; zs.n[2] = nb;
    if (launch_zero_spans(zs, st) != hipSuccess) return 1001;
  }
  const uint64_t seed = 0x5eed0000ull + (uint64_t)m * 131 + k;
  double *cur = w.Q, *alt = w.Y;
  const int cheb = 1;   // degree-2 Chebyshev filter between Rayleigh-Ritz steps
  // the warm start is the same for every replicate: ONE m x P block (Q0),
  // read with replicate stride 0 by the init pass and the first step's y2 /
  // ap2 (L2-resident) instead of nb materialised copies
  double *Q0 = nullptr;
  if (stream_malloc((void **)&Q0, (size_t)m * P * 8 + (size_t)16 * P * 8 + (size_t)(nb + 4) * 4, st) != hipSuccess)
    return 1002;
  double *apre = Q0 + (size_t)m * P;   // a = F'Q0, the same for every replicate (prep_a_kernel)
  // straggler phase (< 1/8 of the batch active at a poll): the GEMMs tile only
  // the listed replicates' column groups (list built once, a superset of the
  // later active sets; replicates retired since are computed and ignored)
  int *alist = (int *)(apre + 16 * P), *acount = alist + nb;
  bool cl_on = false;
  struct Q0Free { double *q; hipStream_t s; ~Q0Free() { hipFreeAsync(q, s); } } q0free{Q0, st};
  const double *qin = Q0;
  int64_t qs = 0;
  const bool warm_started = warm && kw >= k && spread >= 1.0;
  const int d0 = warm_started ? first_filter_degree(spread) : kChebD;
  // a first filter of degree >= 3 has middle Horner steps (boot_cheb_mid_kernel)
  const bool mid = d0 >= 3;
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 1);
  {
    const int64_t n = (int64_t)m * P;
    dim3 grid((unsigned)((n + 255) / 256), 1);
    hipLaunchKernelGGL(eig_init_kernel<P>, grid, dim3(256), 0, st, Q0, m, p, warm, kw, w.done, seed, (int64_t)0, ps);
    // the CSR, trace, PF / e2 and the first product's Z0 and ab (the init
    // pass boot_ap2_kernel<init = 1> ran separately before round 6)
    const size_t prep_lds = (size_t)((4 * m + 3) & ~1) * 4 + (size_t)m * 8;
    if (prep_lds > 65536)   // T > 2730 (up to F2_T_MAX: 96 KB): above the default dynamic-LDS cap
      hipFuncSetAttribute((const void *)boot_prep_kernel<P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)prep_lds);
    hipLaunchKernelGGL(prep_a_kernel<P>, dim3(1), dim3(256), 0, st, fb, Q0, ps, apre);
    hipLaunchKernelGGL(boot_prep_kernel<P>, dim3(nb), dim3(256), prep_lds, st,
                       fb, idx, eta, off, lst, w.trace, mid ? PFb : nullptr, E2b, Q0, ps, Zc, ldz, pz, ab, apre);
  }
  if (mid && !fb.FtF) hipLaunchKernelGGL(ftf_kernel, dim3(1), dim3(1024), 0, st, fb, FtF);
  const double *ftf = fb.FtF ? fb.FtF : FtF;
  // the last Horner step stages F / EL[idx] rows through LDS for r <= 8 (round 6)
  const bool stg_ok = P == 16 && fb.r <= 8 && (fb.r & 1) == 0 && pz <= 16;
  auto chk = stg_ok ? boot_cheb_kernel<P, P == 16> : boot_cheb_kernel<P, false>;
  auto y2k = stg_ok ? boot_y2_kernel<P, P == 16> : boot_y2_kernel<P, false>;
  auto cmk = stg_ok ? boot_cheb_mid_kernel<P, true> : boot_cheb_mid_kernel<P, false>;

  {   // the last Horner step's dynamic LDS (eta, idx, CSR: 20 T bytes) past 64 KB for T > 3276
    const size_t cheb_lds = (size_t)m * 8 + (size_t)(3 * m + 1) * 4;
    if (cheb_lds > 65536)
      hipFuncSetAttribute((const void *)chk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)cheb_lds);
  }
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 0);
  const double beta0 = warm_started ? warm_beta() : 0.0;
  double ca0[kChebDMax + 1], ca1[kChebDMax + 1];
  shifted_cheb(d0, ca0);
  shifted_cheb(kChebD, ca1);
  // Convergence polls from the step most replicates retire at (first_poll)
  // on.  After each such step the device rebuilds the list of active
  // replicates (the GEMMs compact to it once it holds < 1/8 of the batch,
  // decided on the device, so no host round trip sits in front of the
  // straggler phase) and, with a pinned read-back buffer, the active count is
  // copied to host[it] behind an event.  Outside the tail the host does not
  // wait for it: it queues the next step first and reads the previous step's
  // count then (one step of look-ahead — the GPU always has a step queued
  // while the host decides; a step queued after the last replicate retired
  // runs as a no-op and counts for nothing, its active count being 0).  In the
  // straggler tail each step is short and most likely the last, so the count
  // is awaited before the step's Chebyshev products, as a blocking poll
  // (queued no-op steps cost more than the wait: 2.50 -> 2.58 ms per
  // 1 250-replicate shard with look-ahead throughout).  Without the buffer: a
  // blocking poll every `poll` steps, every step in the tail.
  const int first_poll = warm_started ? 1 : poll - 1;
  const bool ahead = pb && pb->host && pb->cap >= maxit + 2;
  int it = 0, last_gemm = -1, last_cheb = -1, next_poll = first_poll, pend = -1, steps = -1;
  bool tail = false;
  for (; it < maxit; ++it) {
    const int dg = it == 0 ? d0 : kChebD;
    const double *ca = it == 0 ? ca0 : ca1;
    const double bb = it == 0 ? beta0 : 0.0;
    if (tf) tf(tctx, DFM_KC_GEMM, 1);
    hipError_t e = launch_gemm_zrm(fb.H, fb.ldH, Zc, pz, zrs, HZ, ldz, m, ncz, m, st, w.done,
                                   cl_on ? alist : nullptr, cl_on ? acount : nullptr);
    if (tf) tf(tctx, DFM_KC_GEMM, 0);
    if (e != hipSuccess) return 1000 + (int)e;
    last_gemm = it;
    if (tf) tf(tctx, DFM_KC_EIG_GQ, 1);
    hipLaunchKernelGGL(y2k, dim3(nb), dim3(64 * BW), (size_t)m * 12, st, fb, w, m, idx, eta, HZ, ldz, pz,
                       ab, qin, qs, alt, ps);
    if (tf) tf(tctx, DFM_KC_EIG_GQ, 0);
    if (tf) tf(tctx, DFM_KC_EIG_SMALL, 1);
    hipLaunchKernelGGL(eig_small_kernel<P>, dim3(nb), dim3(64), 0, st, w, p, 1, kJacobiSweeps);
    if (tf) tf(tctx, DFM_KC_EIG_SMALL, 0);
    if (tf) tf(tctx, DFM_KC_EIG_APPLY, 1);
    if (mid && it == 0 && it < maxit - 1)   // before ap2 overwrites Z(Q) and a(Q)
      hipLaunchKernelGGL(boot_pv_kernel<P>, dim3(nb), dim3(64 * BW), 0, st, fb, w, m, p, it, eta, off, lst, Zc, ldz,
                         pz, ab, seed, w.S, FVb, ps);
    hipLaunchKernelGGL(boot_ap2_kernel<P>, dim3(nb), dim3(64 * BW), lds, st, fb, w, m, k, p, tol, it, 0,
                       it == maxit - 1 ? 1 : 0, cheb, ca[dg], ca[dg - 1], bb, eta, off, lst, qin, qs, alt, Zc, ldz,
                       pz, ab, seed, ps);
    if (tf) tf(tctx, DFM_KC_EIG_APPLY, 0);
    if (it >= first_poll) {
      if (ahead) {
        if ((e = hipMemcpyAsync(pb->host + it, w.active + it, 4, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipEventRecord(pb->ev[it & 1], st)) != hipSuccess)
          return 1000 + (int)e;
      }
      hipLaunchKernelGGL(active_list_kernel, dim3(1), dim3(1024), 0, st, w.done, nb, alist, acount);
      cl_on = true;
      if (ahead) {
        if (pend >= 0) {   // the previous step's count: this step is already queued behind it
          if ((e = hipEventSynchronize(pb->ev[pend & 1])) != hipSuccess) return 1000 + (int)e;
          const int a = pb->host[pend];
          if (a == 0) { steps = pend + 1; ++it; break; }   // (this step ran as a no-op)
          tail = (int64_t)a * 8 < nb;
          pend = -1;
        }
        if (tail) {   // in the straggler tail: this step's count now, before its Chebyshev products
          if ((e = hipEventSynchronize(pb->ev[it & 1])) != hipSuccess) return 1000 + (int)e;
          const int a = pb->host[it];
          if (a == 0) { ++it; break; }
        } else {
          pend = it;
        }
      } else if (it == next_poll) {
        int a = -1;
        hipMemcpyAsync(&a, w.active + it, 4, hipMemcpyDeviceToHost, st);
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return 1000 + (int)e;
        if (a == 0) { ++it; break; }
        next_poll = it + ((int64_t)a * 8 < nb ? 1 : poll);
      }
    }
    if (cheb && it < maxit - 1) {
      // d - 1 products G* S_{i+1} and Horner steps S_i, i = d-2 .. 0: the new
      // basis S_0 goes back into cur (Q), Y stays in alt
      for (int sp = 2; sp <= dg; ++sp) {
        if (tf) tf(tctx, DFM_KC_GEMM, 1);
        e = launch_gemm_zrm(fb.H, fb.ldH, Zc, pz, zrs, HZ, ldz, m, ncz, m, st, w.done,
                            cl_on ? alist : nullptr, cl_on ? acount : nullptr);
        if (tf) tf(tctx, DFM_KC_GEMM, 0);
        if (e != hipSuccess) return 1000 + (int)e;
        if (tf) tf(tctx, DFM_KC_EIG_APPLY, 1);
        if (mid && it == 0 && sp < dg)
          hipLaunchKernelGGL(cmk, dim3(nb), dim3(64 * BW), 0, st, fb, w, m, p, HZ, ldz, pz, ab,
                             ca[dg - sp], bb, k, PFb, E2b, w.S, FVb, ftf, Zc, ps);
        else
          hipLaunchKernelGGL(chk, dim3(nb), dim3(64 * BW), (size_t)m * 8 + (size_t)(3 * m + 1) * 4,
                             st, fb, w, m, p, idx, eta, off, lst, HZ, ldz, pz, ab, ca[dg - sp], bb, k, cur, Zc, ps);
        if (tf) tf(tctx, DFM_KC_EIG_APPLY, 0);
      }
      last_cheb = it;
    } else {
      std::swap(cur, alt);
    }
    qin = cur;
    qs = (int64_t)m * P;
  }
  if (steps < 0) steps = it;
  g_last_iters = steps;
  // the Chebyshev GEMM of iteration it runs after that iteration's check
  if (cnt) {   // (counted by eig_final_kernel below)
    g_last_rep_iters = g_last_gemm_products = 0;
  } else {
    g_last_rep_iters = count_rep_iters(w.active, last_gemm, 1, nb, st);
    const int64_t c0 = count_rep_iters(w.active, std::min(last_cheb, 0), 0, nb, st);
    const int64_t call = count_rep_iters(w.active, last_cheb, 0, nb, st);
    g_last_gemm_products = g_last_rep_iters + c0 * (d0 - 1) + (call - c0) * (kChebD - 1);
  }
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 1);
  hipLaunchKernelGGL(eig_final_kernel<P>, dim3(nb), dim3(256), 0, st, w, m, k, lam, Uk, status, trace_out, cnt,
                     last_gemm, last_cheb, d0 - 1, kChebD - 1);
  if (tf) tf(tctx, DFM_KC_EIG_OTHER, 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return 1000 + (int)e;
  return 0;
}

int eig_run_factored(const FactBase &fb, const int32_t *idx, const double *eta, int nb, int k, int p,
                     const double *warm, int kw, double tol, int maxit, int poll, char *ws, char *fws,
                     double *lam, double *Uk, double *trace_out, int *status, hipStream_t st,
                     timer_fn tf, void *tctx, int *off, int *lst, long long *cnt, int subspace, double spread,
                     const PollBuf *pb) {
  if (p < k || p > 32 || p > fb.T || fb.r > 32) return -1;
  if (fb.r > 16 || fb.T > F2_T_MAX) return -1;   // callers take the direct path
  if (p <= 16)
    return eig_run_fact2_t<16>(fb, idx, eta, nb, k, p, warm, kw, tol, maxit, poll, ws, fws, lam, Uk,
                               trace_out, status, st, tf, tctx, off, lst, cnt, subspace, spread, pb);
  return eig_run_fact2_t<32>(fb, idx, eta, nb, k, p, warm, kw, tol, maxit, poll, ws, fws, lam, Uk,
                             trace_out, status, st, tf, tctx, off, lst, cnt, subspace, spread, pb);
}
int fact_t_max() { return F2_T_MAX; }

// ---- factored loadings pass: L* = X*' F* / T = (L (F'F*) + E' P' D F*) / T
// boot_zf: replicate rep's block ZB = ZF + rep Kp rp (Kp x rp, row-major):
//          ZB[s][j] = sum_{t in bucket s} eta_t F*[t][j]   (s < T)
//          ZB[T + i][j] = M1[rep][i][j] = (F' F*)[i][j]    (i < r)
//          zero rows T + r .. Kp - 1 and zero column r when rp > r;
//          F* = sqrt(T) U* written to Fout.
// The block is contiguous, so every row segment lands in whole lines.
__global__ __launch_bounds__(256) void boot_zf_kernel(FactBase fb, const double *__restrict__ Uk,
                                                      const double *__restrict__ eta,
                                                      const int *__restrict__ off, const int *__restrict__ lst,
                                                      double *__restrict__ Fout, double *__restrict__ ZF, int Kp,
                                                      int rp, double *__restrict__ M1) {
  const int tid = threadIdx.x, rep = blockIdx.x, T = fb.T, r = fb.r;
  const double sT = sqrt((double)T);
  const double *U = Uk + (int64_t)rep * T * r;
  double *Fr = Fout + (int64_t)rep * T * r;
  double *ZB = ZF + (int64_t)rep * Kp * rp;
  const double *et = eta ? eta + (int64_t)rep * T : nullptr;
  const int *o = off + (int64_t)rep * (T + 1);
  const int *L = lst + (int64_t)rep * T;
  for (int e = tid; e < T * r; e += 256) Fr[e] = sT * U[e];
  for (int e = tid; e < T * rp; e += 256) {
    const int sI = e / rp, j = e - sI * rp;
    double z = 0.0;
    if (j < r)
      for (int q = o[sI]; q < o[sI + 1]; ++q) {
        const int t = L[q];
        z = fma(et ? et[t] : 1.0, sT * U[(int64_t)t * r + j], z);
      }
    ZB[e] = z;
  }
  for (int e = (T + r) * rp + tid; e < Kp * rp; e += 256) ZB[e] = 0.0;
  if (rp > r)
    for (int i = tid; i < r; i += 256) ZB[(int64_t)(T + i) * rp + r] = 0.0;
  // M1 = F' F*: 4 row-interleaved partial sums per entry (four independent
  // chains of T/4 instead of one of T), combined in a fixed order
  __shared__ double m1p[4][256];
  const int part = tid >> 6;
  for (int e0 = 0; e0 < r * r; e0 += 64) {
    const int e = e0 + (tid & 63);
    double acc = 0.0;
    if (e < r * r) {
      const int i = e / r, j = e % r;
      for (int t = part; t < T; t += 4) acc = fma(fb.F[(int64_t)t * r + i], sT * U[(int64_t)t * r + j], acc);
    }
    m1p[part][tid & 63] = acc;
    __syncthreads();
    if (tid < 64 && e < r * r) {
      const double v = (m1p[0][tid] + m1p[1][tid]) + (m1p[2][tid] + m1p[3][tid]);
      M1[(int64_t)rep * r * r + e] = v;
      // the same block as k-rows T..T+r-1 of the loadings GEMM's B operand
      ZB[(int64_t)(T + e / r) * rp + e % r] = v;
    }
    __syncthreads();
  }
}

// rows T.. of [E; L'; 0]: row T+i = column i of L (i < r), then zero rows
__global__ void eaug_tail_kernel(const double *__restrict__ Lb, int N, int r, int64_t ld, double *__restrict__ tail) {
  const int i = blockIdx.y;
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= ld) return;
  tail[(int64_t)i * ld + n] = (i < r && n < N) ? Lb[n * r + i] : 0.0;
}

static int zf_rp(int r) { return (r + 1) / 2 * 2; }
static int zf_kp(int T, int r) { return (T + r + 15) / 16 * 16; }
int fact_loadings(const FactBase &fb, const double *Ep, int64_t ld, int N, const double *Lb,
                  const double *Uk, const double *eta, const int *off, const int *lst, int nb,
                  double *Fout, double *Lout, char *ws, hipStream_t st) {
  const int T = fb.T, r = fb.r, rp = zf_rp(r), Kp = zf_kp(T, r);
  double *ZF = (double *)ws;                       // nb blocks of Kp x rp
  double *M1 = ZF + (size_t)nb * Kp * rp;
  double *Eaug = M1 + (size_t)nb * r * r;          // [E; L'; 0]: Kp x ld
  // (staging U*, eta and the CSR in LDS first measured slower: 0.62 -> 0.76 ms at C3)
  hipLaunchKernelGGL(boot_zf_kernel, dim3(nb), dim3(256), 0, st, fb, Uk, eta, off, lst, Fout, ZF, Kp, rp, M1);
  // one GEMM of depth T + r does the whole finish (see gemm_loadings_kernel),
  // for every batch size: the same arithmetic for every replicate whatever
  // the batch composition (batch- and shard-invariant loadings)
  hipMemcpy2DAsync(Eaug, (size_t)ld * 8, Ep, (size_t)ld * 8, (size_t)ld * 8, T, hipMemcpyDeviceToDevice, st);
  hipLaunchKernelGGL(eaug_tail_kernel, dim3((unsigned)((ld + 255) / 256), Kp - T), dim3(256), 0, st, Lb, N, r, ld,
                     Eaug + (size_t)T * ld);
  const hipError_t e = launch_gemm_loadings(Eaug, ld, ZF, Kp, rp, N, nb, T + r, r, 1.0 / T, Lout, st);
  return e == hipSuccess ? 0 : 1000 + (int)e;
}
size_t fact_loadings_bytes(int T, int N, int r, int nb) {
  const int64_t ld = ((int64_t)N + 15) / 16 * 16;
  const int Kp = zf_kp(T, r);
  return ((size_t)nb * Kp * zf_rp(r) + (size_t)nb * r * r + (size_t)Kp * ld) * 8 + 1024;
}

// ---- model-level precompute: EL = E L (T x r), S = L'L, cF, hd
__global__ void fact_pre_kernel(const double *__restrict__ Ep, int64_t ld, int T, int N, int r,
                                const double *__restrict__ Lb, const double *__restrict__ Fb,
                                const double *__restrict__ H, int64_t ldH, double *__restrict__ EL,
                                double *__restrict__ S, double *__restrict__ cF, double *__restrict__ hd) {
  const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x < r * r) {
    const int i = threadIdx.x / r, j = threadIdx.x % r;
    double acc = 0.0;
    for (int n = 0; n < N; ++n) acc = fma(Lb[(int64_t)n * r + i], Lb[(int64_t)n * r + j], acc);
    S[threadIdx.x] = acc;
  }
  if (t >= T) return;
  for (int j = 0; j < r; ++j) {
    double acc = 0.0;
    for (int n = lane; n < N; n += 64) acc = fma(Ep[(int64_t)t * ld + n], Lb[(int64_t)n * r + j], acc);
    acc = wave_sum(acc);
    if (lane == 0) EL[(int64_t)t * r + j] = acc;
  }
  if (lane == 0) hd[t] = H[(int64_t)t * ldH + t];
}
__global__ void fact_cf_kernel(int T, int r, const double *__restrict__ Fb, const double *__restrict__ S,
                               double *__restrict__ cF) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  double acc = 0.0;
  for (int i = 0; i < r; ++i) {
    double u = 0.0;
    for (int j = 0; j < r; ++j) u = fma(S[i * r + j], Fb[(int64_t)t * r + j], u);
    acc = fma(Fb[(int64_t)t * r + i], u, acc);
  }
  cF[t] = acc;
}
// FSF = F S F' (T x T, ldH), the common-component Gram C C' of the base fit
// (C = F L', S = L'L): entry (s, t >= s) computed once and mirrored, so the
// matrix is exactly symmetric.
__global__ void fact_fsf_kernel(int T, int r, const double *__restrict__ Fb, const double *__restrict__ S,
                                double *__restrict__ FSF, int64_t ldH) {
  const int t = blockIdx.x * 256 + threadIdx.x, s = blockIdx.y;
  if (t >= T || t < s) return;
  double acc = 0.0;
  for (int i = 0; i < r; ++i) {
    double u = 0.0;
    for (int j = 0; j < r; ++j) u = fma(S[i * r + j], Fb[(int64_t)t * r + j], u);
    acc = fma(Fb[(int64_t)s * r + i], u, acc);
  }
  FSF[(int64_t)s * ldH + t] = acc;
  FSF[(int64_t)t * ldH + s] = acc;
}
hipError_t launch_fact_fsf(int T, int r, const double *Fb, const double *S, double *FSF, int64_t ldH, hipStream_t st) {
  hipLaunchKernelGGL(fact_fsf_kernel, dim3((T + 255) / 256, T), dim3(256), 0, st, T, r, Fb, S, FSF, ldH);
  return hipGetLastError();
}

// Replicate Grams of the direct (Gram-forming) path for N > T without
// breaks, by the factored identity instead of the T x T x N SYRK:
//   X* = F L' + D P E  =>  G* = X* X*' = F S F' + F c' + c F' + D P H P' D,
//   c_t = eta_t EL[idx_t]  (EL = E L, H = E E', S = L'L: model precompute),
// i.e. G*[s][t] = FSF[s][t] + sum_j (F_sj c_tj + c_sj F_tj)
//                 + (eta_s eta_t) H[idx_s][idx_t]          (2 T^2 r flop, not T^2 N).
// Each term is symmetric in (s, t) operation by operation (separately rounded
// products and sums — no contraction — in a fixed order), so G* is exactly
// symmetric.
// One workgroup per (replicate, GF_R rows): the rows' H rows H[idx_s][:]
// staged in LDS (gathered by idx_t from there), one thread per column t
// holding F_t and c_t in registers.
constexpr int GF_R = 8;
template <int RM>
__global__ __launch_bounds__(256) void gram_fact_kernel(FactBase fb, const double *__restrict__ FSF,
                                                        const int32_t *__restrict__ idx,
                                                        const double *__restrict__ eta, int R,
                                                        double *__restrict__ G, int64_t ldg, int64_t strideG) {
  extern __shared__ double gdyn[];
  const int T = fb.T, r = fb.r, tid = threadIdx.x, rep = blockIdx.y, s0 = blockIdx.x * R;
  const int ns = min(R, T - s0);
  double *sH = gdyn;                       // R x T: H[idx_s][:]
  double *sFc = sH + (size_t)R * T;        // R x 2 RM: F_s, c_s
  const int32_t *ix = idx + (int64_t)rep * T;
  const double *et = eta ? eta + (int64_t)rep * T : nullptr;
  for (int e = tid; e < ns * T; e += 256) {
    const int i = e / T, t = e - i * T;
    sH[e] = fb.H[(int64_t)ix[s0 + i] * fb.ldH + t];
  }
  for (int e = tid; e < ns * RM; e += 256) {
    const int i = e / RM, j = e - i * RM, sI = s0 + i;
    const double es = et ? et[sI] : 1.0;
    sFc[i * 2 * RM + j] = j < r ? fb.F[(int64_t)sI * r + j] : 0.0;
    sFc[i * 2 * RM + RM + j] = j < r ? es * fb.EL[(int64_t)ix[sI] * r + j] : 0.0;
  }
  __syncthreads();
  double *Gr = G + (int64_t)rep * strideG;
  for (int t = tid; t < T; t += 256) {
    const int it = ix[t];
    const double eT = et ? et[t] : 1.0;
    double Ft[RM], ct[RM];
#pragma unroll
    for (int j = 0; j < RM; ++j) {
      Ft[j] = j < r ? fb.F[(int64_t)t * r + j] : 0.0;
      ct[j] = j < r ? eT * fb.EL[(int64_t)it * r + j] : 0.0;
    }
    // GF_R rows at a time: every row's FSF entry and H gather issued before the sums
    for (int i0 = 0; i0 < ns; i0 += GF_R) {
      double fsf[GF_R], hv[GF_R], es[GF_R];
#pragma unroll
      for (int u = 0; u < GF_R; ++u) {
        const int i = min(i0 + u, ns - 1), sI = s0 + i;
        fsf[u] = FSF[(int64_t)sI * fb.ldH + t];
        hv[u] = sH[i * T + it];
        es[u] = et ? et[sI] : 1.0;
      }
#pragma unroll
      for (int u = 0; u < GF_R; ++u) {
        const int i = i0 + u;
        if (i >= ns) break;
        const double *fc = sFc + i * 2 * RM;
        double x = 0.0;
#pragma unroll
        for (int j = 0; j < RM; ++j)
          if (j < r) x = __dadd_rn(x, __dadd_rn(__dmul_rn(fc[j], ct[j]), __dmul_rn(fc[RM + j], Ft[j])));
        Gr[(int64_t)(s0 + i) * ldg + t] = __dadd_rn(__dadd_rn(fsf[u], x), __dmul_rn(__dmul_rn(es[u], eT), hv[u]));
      }
    }
  }
}
int gram_fact_rows(int T) { return std::max(1, std::min(GF_R, 4096 / std::max(T, 1))); }
size_t gram_fact_lds(int T, int r) {
  const int R = gram_fact_rows(T), RM = r <= 8 ? 8 : 16;
  return (size_t)R * T * 8 + (size_t)R * 2 * RM * 8;
}
hipError_t launch_gram_fact(const FactBase &fb, const double *FSF, const int32_t *idx, const double *eta, int nb,
                            double *G, int64_t ldg, int64_t strideG, hipStream_t st) {
  const int R = gram_fact_rows(fb.T);
  const size_t lds = gram_fact_lds(fb.T, fb.r);
  dim3 grid((fb.T + R - 1) / R, nb);
  if (fb.r <= 8)
    hipLaunchKernelGGL(gram_fact_kernel<8>, grid, dim3(256), lds, st, fb, FSF, idx, eta, R, G, ldg, strideG);
  else
    hipLaunchKernelGGL(gram_fact_kernel<16>, grid, dim3(256), lds, st, fb, FSF, idx, eta, R, G, ldg, strideG);
  return hipGetLastError();
}

hipError_t launch_fact_ftf(const FactBase &fb, double *FtF, hipStream_t st) {
  hipLaunchKernelGGL(ftf_kernel, dim3(1), dim3(1024), 0, st, fb, FtF);
  return hipGetLastError();
}

int fact_precompute(const double *Ep, int64_t ld, int T, int N, int r, const double *Lb, const double *Fb,
                    const double *H, int64_t ldH, double *EL, double *S, double *cF, double *hd, hipStream_t st) {
  hipLaunchKernelGGL(fact_pre_kernel, dim3((T + 3) / 4), dim3(256), 0, st, Ep, ld, T, N, r, Lb, Fb, H, ldH,
                     EL, S, cF, hd);
  hipLaunchKernelGGL(fact_cf_kernel, dim3((T + 255) / 256), dim3(256), 0, st, T, r, Fb, S, cF);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : 1000 + (int)e;
}

// ------------------------------------------------------------ full spectrum
// All eigenvalues (descending) of one m x m symmetric matrix, m <= SPEC_MAX,
// by parallel cyclic Jacobi with the whole matrix resident in LDS.  Used for
// the PCp criteria's unrestricted sigma^2 = V(ceil(m/2)) (src/criteria.jl:18)
// and for full IC sweeps (k up to ceil(m/2), src/DynamicFactorModel.jl:54).
constexpr int SPEC_MAX = 140;
// Matrix rep has size m0 + dm * rep (expanding windows share one prefix Gram);
// ev rows have stride mst.
__global__ __launch_bounds__(256) void spectrum_kernel(const double *__restrict__ G, int64_t ldg,
                                                       int64_t strideG, int mst, int m0, int dm,
                                                       double *__restrict__ ev) {
  constexpr int S = SPEC_MAX + 1;
  __shared__ double H[SPEC_MAX * S];
  __shared__ double rc[SPEC_MAX / 2], rs[SPEC_MAX / 2];
  __shared__ int ra[SPEC_MAX / 2], rbb[SPEC_MAX / 2];
  __shared__ int sdone;
  const int tid = threadIdx.x, rep = blockIdx.x;
  const double *g = G + (int64_t)rep * strideG;
  const int m = m0 + dm * rep;
  const int n = m + (m & 1);
  for (int e = tid; e < n * n; e += 256) {
    const int a = e / n, c = e % n;
    H[a * S + c] = (a < m && c < m) ? 0.5 * (g[(int64_t)a * ldg + c] + g[(int64_t)c * ldg + a]) : 0.0;
  }
  __syncthreads();
  // classic threshold Jacobi (see eig_small_kernel): rotate while |h_ab| >
  // 4 eps sqrt(|h_aa h_bb|); stop after a sweep that rotates nothing
  for (int sweep = 0; sweep < 80; ++sweep) {
    if (tid == 0) sdone = 1;
    __syncthreads();
    for (int r = 0; r < n - 1; ++r) {
      for (int s = tid; s < n / 2; s += 256) {
        const int pa = s, pb = n - 1 - s;
        int a = pa == 0 ? 0 : 1 + (pa - 1 + r) % (n - 1);
        int b = pb == 0 ? 0 : 1 + (pb - 1 + r) % (n - 1);
        if (a > b) { const int t = a; a = b; b = t; }
        double c = 1.0, sn = 0.0;
        const double hab = H[a * S + b], haa = H[a * S + a], hbb = H[b * S + b];
        if (fabs(hab) > 1e-300 && fabs(hab) > 8.9e-16 * sqrt(fabs(haa) * fabs(hbb))) {
          sdone = 0;
          const double zeta = (hbb - haa) / (2.0 * hab);
          const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          c = 1.0 / sqrt(1.0 + t * t);
          sn = t * c;
        }
        ra[s] = a; rbb[s] = b; rc[s] = c; rs[s] = sn;
      }
      __syncthreads();
      for (int e = tid; e < (n / 2) * n; e += 256) {
        const int s = e / n, kk = e % n;
        const int a = ra[s], b = rbb[s];
        const double c = rc[s], sn = rs[s];
        const double ha = H[kk * S + a], hb = H[kk * S + b];
        H[kk * S + a] = c * ha - sn * hb;
        H[kk * S + b] = sn * ha + c * hb;
      }
      __syncthreads();
      for (int e = tid; e < (n / 2) * n; e += 256) {
        const int s = e / n, kk = e % n;
        const int a = ra[s], b = rbb[s];
        const double c = rc[s], sn = rs[s];
        const double ha = H[a * S + kk], hb = H[b * S + kk];
        H[a * S + kk] = c * ha - sn * hb;
        H[b * S + kk] = sn * ha + c * hb;
      }
      __syncthreads();
    }
    if (sdone) break;
    __syncthreads();
  }
  // sort descending; the padding index (if any) carries an exact 0 that is dropped
  for (int i = tid; i < n; i += 256) {
    const double v = H[i * S + i];
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const double u = H[j * S + j];
      if (u > v || (u == v && j < i)) ++rank;
    }
    if (rank < m) ev[(int64_t)rep * mst + rank] = v;
  }
}

int spectrum_max() { return SPEC_MAX; }
hipError_t launch_spectrum_jacobi(const double *G, int64_t ldg, int64_t strideG, int m, int m0, int dm, int nb,
                                  double *ev, hipStream_t st) {
  if (m > SPEC_MAX || m0 < 1 || m0 + dm * (nb - 1) > m) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spectrum_kernel, dim3(nb), dim3(256), 0, st, G, ldg, strideG, m, m0, dm, ev);
  return hipGetLastError();
}

}  // namespace dfm
