// dfm_common.h — shared device types and helpers for libdfm (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DFM_DEV __device__ __forceinline__

namespace dfm {

// A resampled panel X*, never materialised: for row t of replicate b
//   X*[t, n] = C[t, n] + eta_b[t] * E[idx_b[t], n]
// C == nullptr -> 0, eta == nullptr -> 1, idx == nullptr -> identity.
// C and E are row-major T x N with row stride `ld` (elements); idx/eta are
// B x rs row-major (rs = T except for a break block, whose idx/eta rows are
// the block's columns of the full B x T draws).  This is the wild/residual bootstrap of
// src/bootstrap.jl:44-45 (:24 for the residual form) and, with C = E = X and
// no idx/eta, the plain panel of principal_components (src/DynamicFactorModel.jl:75).
struct PanelSrc {
  const double *C;
  const double *E;
  const int32_t *idx;
  const double *eta;
  int64_t ld;
  int64_t rs;   // elements between consecutive replicates' idx / eta rows
};

// v_mfma_f64_4x4x4_4b_f64: 4 independent 4x4x4 blocks per instruction
// (75 TF/s measured on MI355X vs 49.5 for 16x16x4 — tools/mfma_f64_probe.hip).
// Lane l: k = l>>4, blk = (l>>2)&3, i = l&3.
//   A[blk][i][k] at lane 16k + 4blk + i, B[blk][k][j] at 16k + 4blk + j,
//   C[blk][i][j] at lane 16i + 4blk + j  (tools/mfma4_layout.hip, one-hot probe).
DFM_DEV double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// v_mfma_f64_16x16x4: A[i][k] at lane i + 16k, B[k][j] at lane j + 16k,
// C[row][col] at lane col + 16 (row % 4), register row / 4 (tools/mfma16_layout.hip).
typedef double dv4 __attribute__((ext_vector_type(4)));
DFM_DEV dv4 mfma16(double a, double b, dv4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

DFM_DEV double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Deterministic pseudo-random start vectors for the subspace iteration.
DFM_DEV double hash_unit(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full ^
               (c + 0x165667B19E3779F9ull) * 0x27D4EB2F165667C5ull;
  x ^= x >> 31; x *= 0x7FB5D329728EA185ull; x ^= x >> 27; x *= 0x81DADEF4BC2DD44Dull; x ^= x >> 33;
  return (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
}

// Debug build (csrc Makefile EXTRA=-DDFM_DEBUG_MEM, never the production
// library): every fresh device allocation is filled with 0xFF bytes — NaN
// doubles, -1 ints — so a read of memory no kernel of the call wrote shows up
// as NaN / an out-of-range index deterministically instead of as stale data.
#ifdef DFM_DEBUG_MEM
inline void dbg_poison_sync(void *p, size_t bytes) {   // null stream only: the contexts' (non-blocking) streams run on
  if (p && bytes) { (void)hipMemset(p, 0xFF, bytes); (void)hipStreamSynchronize(nullptr); }
}
inline void dbg_poison_async(void *p, size_t bytes, hipStream_t st) {
  if (p && bytes) (void)hipMemsetAsync(p, 0xFF, bytes, st);
}
#define DFM_POISON_SYNC(p, b) ::dfm::dbg_poison_sync((void *)(p), (size_t)(b))
#define DFM_POISON_ASYNC(p, b, st) ::dfm::dbg_poison_async((void *)(p), (size_t)(b), (st))
#else
#define DFM_POISON_SYNC(p, b) ((void)0)
#define DFM_POISON_ASYNC(p, b, st) ((void)0)
#endif

// Stream-ordered scratch from the pool of the context that owns `st` (each
// dfm_ctx has its own hipMemPool: a block freed on one context's stream is
// never handed to another context's stream — the two bootstrap lanes of a
// model, dfm_bootstrap_multi's shards); streams no context owns fall back to
// the device's default pool.  Debug builds poison the block.
hipError_t stream_malloc(void **p, size_t bytes, hipStream_t st);

// Zero up to four spans of 32-bit words in ONE launch (a call's counters,
// flags and padding rows: each separate memset was a host API round of a few
// microseconds in the lanes' prologues, with the GPU idle behind it).
struct ZeroSpans {
  int *p[4];
  int64_t n[4];   // words; 0 = unused
};
hipError_t launch_zero_spans(const ZeroSpans &z, hipStream_t st);

// A context's pinned read-back slots for the factored solver's convergence
// polls (eig_run_factored): the active count of iteration it is copied into
// host[it] behind event ev[it & 1] while the next iteration is already
// queued, so the GPU never waits on the host's decision.
struct PollBuf {
  int *host = nullptr;   // hipHostMalloc'd, cap ints
  int cap = 0;
  hipEvent_t ev[2] = {};
};

// The device gate.  The lasso path kernel needs every workgroup of a grid
// sized to the whole chip co-resident (leader/helper hand-offs); a kernel of
// another libdfm context on the same device would hold CUs and make its
// hand-offs wait out their timeouts.  Every public call that launches work
// holds a DeviceShare of its device for its duration (nested calls on one
// thread count once); the lasso launch takes a DeviceSolo — it waits until no
// libdfm call is in progress on the device, starts none while it runs, and
// drains the device's queued work (hipDeviceSynchronize) before launching.
// held == false: the calling thread is itself inside a shared call on the
// device (the solo could never drain), and the caller fails.
struct DeviceShare {
  explicit DeviceShare(int device);
  ~DeviceShare();
  DeviceShare(const DeviceShare &) = delete;
  DeviceShare &operator=(const DeviceShare &) = delete;
  int dev;
};
struct DeviceSolo {
  explicit DeviceSolo(int device);
  ~DeviceSolo();
  DeviceSolo(const DeviceSolo &) = delete;
  DeviceSolo &operator=(const DeviceSolo &) = delete;
  int dev;
  bool held = false;
};

}  // namespace dfm

// Kernel classes for per-kernel HIP-event timing (dfm_ctx_read_timing).
enum {
  DFM_KC_GRAM = 0, DFM_KC_EIG_GQ, DFM_KC_EIG_SMALL, DFM_KC_EIG_APPLY, DFM_KC_EIG_OTHER,
  DFM_KC_FACTORS, DFM_KC_OLS, DFM_KC_STATS, DFM_KC_CHOW, DFM_KC_MISC, DFM_KC_GEMM, DFM_KC_COUNT
};
