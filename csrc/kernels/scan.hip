// Device-wide exclusive prefix sum (reduce-then-scan).
//
// Used by every variable-length encoder (record sizes -> byte offsets) and by
// the frame-table compaction (frames per tile -> frame index base).
//   pass 1: per-block reduce
//   pass 2: scan of block sums    (recursive when > E blocks)
//   pass 3: per-block scan + add block base
// Three short launches; at 1M records the whole scan is a few microseconds,
// far below the byte-moving kernels it feeds.
//
// Two pass-3 engines (zk_scan_set_mode):
//   SCAN_SHFL  256 threads x 8 elements, lane-serial then wave shuffle scan.
//   SCAN_MFMA  the "MFMA-packed byte scan": 256 threads x 16 elements.  A
//              wave owns 1024 values as 16 segments x 64.  Each value is
//              split into byte planes; one i8 MFMA (16x16x64) per (plane,
//              quarter) multiplies a strictly-lower-triangular ones matrix
//              by 16 segments' bytes, giving the in-segment exclusive prefix
//              of 16 positions x 16 segments; the planes are recombined with
//              shifts.  Bytes are fed as (b - 128) because the operand is
//              signed; the bias is added back per position.  Only the
//              planes some value in the wave needs are multiplied (record
//              sizes < 64 KiB: 2 planes, 8 MFMAs per 1024 values).  A wave
//              holding any value outside [0, 2^32) takes the shuffle path.
#include "zk_common.h"
#include "zk_mfma_scan.h"

#include <stdlib.h>

namespace zk {

constexpr int SCAN_T = 256;
constexpr int SCAN_V = 8;
constexpr int64_t SCAN_E = SCAN_T * SCAN_V;

template <typename T>
__global__ __launch_bounds__(SCAN_T) void scan_reduce(const T* __restrict__ in,
                                                     int64_t n,
                                                     int64_t* __restrict__ bsum) {
  __shared__ int64_t sm[SCAN_T / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * SCAN_E + threadIdx.x * SCAN_V;
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_V; ++j)
    if (base + j < n) s += (int64_t)in[base + j];
  int64_t tot;
  block_excl_scan(s, sm, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

template <typename T>
__global__ __launch_bounds__(SCAN_T) void scan_apply(const T* __restrict__ in,
                                                    int64_t n,
                                                    const int64_t* __restrict__ bbase,
                                                    int64_t* __restrict__ out,
                                                    int64_t* __restrict__ total) {
  __shared__ int64_t sm[SCAN_T / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * SCAN_E + threadIdx.x * SCAN_V;
  int64_t v[SCAN_V];
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_V; ++j) {
    v[j] = (base + j < n) ? (int64_t)in[base + j] : 0;
    s += v[j];
  }
  int64_t tot;
  int64_t p = block_excl_scan(s, sm, &tot) + (bbase ? bbase[blockIdx.x] : 0);
#pragma unroll
  for (int j = 0; j < SCAN_V; ++j) {
    if (base + j < n) out[base + j] = p;
    p += v[j];
  }
  if (total != nullptr && blockIdx.x == gridDim.x - 1 &&
      threadIdx.x == SCAN_T - 1)
    *total = p;
}

// One workgroup scans any n in one launch: 1024 threads x 8 values per
// chunk, a running carry across chunks.  Used for the short scans (frame
// counts per tile, the encoders' block sums), where the reduce / scan /
// apply chain was three launches of ~5 us each for a few thousand values.
constexpr int SB_T = 1024;
constexpr int SB_V = 8;
constexpr int64_t SCAN_ONE_MAX = 1 << 16;       // use it up to this n

// A one-workgroup scan sits on its stream's critical path, and with two
// connections in flight it waits for a CU with room for the whole
// workgroup behind the other stream's kernel: up to 2048 values (the
// encoders' block sums of a 512K-record batch) a 256-thread workgroup
// scans them in one chunk.
constexpr int SB_T_SMALL = 256;

template <typename T, int NT = SB_T>
__global__ __launch_bounds__(NT) void scan_one_block(
    const T* __restrict__ in, int64_t n, int64_t* __restrict__ out,
    int64_t* __restrict__ total) {
  __shared__ int64_t sm[NT / 64 + 1];
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < n; c0 += (int64_t)NT * SB_V) {   // uniform
    // thread t owns values c0 + t*V .. +V-1 (its own run: the scan order)
    const int64_t b = c0 + (int64_t)threadIdx.x * SB_V;
    int64_t v[SB_V];
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < SB_V; ++j) {
      v[j] = b + j < n ? (int64_t)in[b + j] : 0;
      s += v[j];
    }
    int64_t tot;
    int64_t p = carry + block_excl_scan(s, sm, &tot);
#pragma unroll
    for (int j = 0; j < SB_V; ++j) {
      if (b + j < n) out[b + j] = p;
      p += v[j];
    }
    carry += tot;
  }
  if (total != nullptr && threadIdx.x == 0) *total = carry;
}

template <typename T>
static void launch_one_block(const T* in, int64_t n, int64_t* out,
                             int64_t* total, hipStream_t st) {
  if (n <= (int64_t)SB_T_SMALL * SB_V)
    scan_one_block<T, SB_T_SMALL><<<1, SB_T_SMALL, 0, st>>>(in, n, out, total);
  else
    scan_one_block<T><<<1, SB_T, 0, st>>>(in, n, out, total);
}

// ---------------------------------------------------------------------------
// MFMA byte-plane engine
// ---------------------------------------------------------------------------

// Block sums for the V-per-thread engines.  The sum is order-free, so
// thread t reads t, t + 256, ... (coalesced) rather than its own run.
template <typename T, int V, int NT>
__global__ __launch_bounds__(NT) void scan_reduce_v(const T* __restrict__ in,
                                                   int64_t n,
                                                   int64_t* __restrict__ bsum) {
  __shared__ int64_t sm[NT / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * (NT * V) + threadIdx.x;
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < V; ++j)
    if (base + j * NT < n) s += (int64_t)in[base + j * NT];
  int64_t tot;
  if (NT == 64) {
    tot = __shfl(wave_incl_scan(s), 63, 64);
  } else {
    block_excl_scan(s, sm, &tot);
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

template <typename T, int NT>
__global__ __launch_bounds__(NT) void scan_apply_mfma(
    const T* __restrict__ in, int64_t n, const int64_t* __restrict__ bbase,
    int64_t* __restrict__ out, int64_t* __restrict__ total) {
  constexpr int64_t MS_E = (int64_t)NT * MS_V;
  __shared__ int64_t stage[ms_stage_slots<NT>()];
  __shared__ int64_t wsum[NT / 64 + 1];
  const int64_t bstart = (int64_t)blockIdx.x * MS_E;
  const int64_t b0 = bbase ? bbase[blockIdx.x] : 0;
  const int64_t t = mfma_scan_chunk<T, NT>(in + bstart, min(n - bstart, MS_E),
                                           out + bstart, b0, stage, wsum);
  if (total != nullptr && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    *total = b0 + t;
}

// One workgroup, any n, one launch, on MFMA (the encoders' block sums: 2048
// of them for a 512K-request connection of the GET step).  128 threads:
// 2048 values in one chunk, and a workgroup small enough to find a CU
// quickly beside the other connection's kernels.
constexpr int SB_T_MFMA = 128;

template <int NT = SB_T_MFMA>
__global__ __launch_bounds__(NT) void scan_one_block_mfma(
    const int64_t* __restrict__ in, int64_t n, int64_t* __restrict__ out,
    int64_t* __restrict__ total) {
  __shared__ int64_t wsum[NT / 64 + 1];
  const int64_t t = mfma_scan_block_direct<NT>(in, n, out, wsum);
  if (total != nullptr && threadIdx.x == 0) *total = t;
}

// ZKMI_SMALL_SCAN: the engine of the one-workgroup scans (zk_scan_small_i64:
// K10 / K13's block sums; tree_finish_scan): "shfl" (default) or "mfma".
// The MFMA version costs the GET step 2.6 % (profiles/r6_mfma_ab.md): a
// 2048-value scan is latency, not arithmetic.
static int small_scan_mode() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ZKMI_SMALL_SCAN");
    v = (e != nullptr && e[0] == 'm') ? 1 : 0;
  }
  return v;
}

template <typename T>
static int scan_rec(const T* in, int64_t* out, int64_t n, int64_t* total,
                    int64_t* ws, hipStream_t st);

// NT = threads per block of the MFMA engine (64: one wave, 1024 values per
// block, many small blocks in flight; 256: 4096 per block).  Up to
// SCAN_ONE_MAX values go to the one-workgroup scan (one launch) unless
// `force` (SCAN_MFMA_FORCE: the multi-block MFMA path at any n, for the
// tests).  A level of one block is the recursion's end: round 5 forced the
// engine below SCAN_ONE_MAX without it, and the host recursed on nb = 1
// until its stack overflowed (the "crash in the microbenchmark").
template <typename T, int NT>
static int scan_rec_mfma(const T* in, int64_t* out, int64_t n, int64_t* total,
                         int64_t* ws, hipStream_t st, bool force) {
  constexpr int64_t E = (int64_t)NT * MS_V;
  if (n <= 0 || (n <= SCAN_ONE_MAX && !force))
    return scan_rec<T>(in, out, n, total, ws, st);
  const int64_t nb = (n + E - 1) / E;
  if (nb == 1) {
    scan_apply_mfma<T, NT><<<1, NT, 0, st>>>(in, n, nullptr, out, total);
    ZK_LAUNCH_CHECK();
    return 0;
  }
  int64_t* bsum = ws;
  int64_t* bbase = ws + nb;
  scan_reduce_v<T, MS_V, NT><<<(unsigned)nb, NT, 0, st>>>(in, n, bsum);
  ZK_LAUNCH_CHECK();
  int rc = scan_rec_mfma<int64_t, NT>(bsum, bbase, nb, nullptr, ws + 2 * nb,
                                      st, force);
  if (rc) return rc;
  scan_apply_mfma<T, NT><<<(unsigned)nb, NT, 0, st>>>(in, n, bbase, out, total);
  ZK_LAUNCH_CHECK();
  return 0;
}

enum { SCAN_SHFL = 0, SCAN_MFMA = 1, SCAN_MFMA_W1 = 2, SCAN_MFMA_W4 = 3,
       SCAN_MFMA_FORCE = 4 };
static int g_scan_mode = SCAN_MFMA;

template <typename T>
static int scan_mfma(const T* in, int64_t* out, int64_t n, int64_t* total,
                     int64_t* ws, hipStream_t st, int mode) {
  // measured (profiles/r1_v10_scan_engines.md): one-wave blocks are as fast
  // or faster than four-wave ones at every n, so auto = one wave
  if (mode == SCAN_MFMA_W4)
    return scan_rec_mfma<T, 256>(in, out, n, total, ws, st, false);
  return scan_rec_mfma<T, 64>(in, out, n, total, ws, st,
                              mode == SCAN_MFMA_FORCE);
}

template <typename T>
static int scan_rec(const T* in, int64_t* out, int64_t n, int64_t* total,
                    int64_t* ws, hipStream_t st) {
  if (n <= 0) {
    if (total) hipMemsetAsync(total, 0, sizeof(int64_t), st);
    return 0;
  }
  const int64_t nb = (n + SCAN_E - 1) / SCAN_E;
  if (nb == 1) {
    scan_apply<T><<<1, SCAN_T, 0, st>>>(in, n, nullptr, out, total);
    ZK_LAUNCH_CHECK();
    return 0;
  }
  if (n <= SCAN_ONE_MAX) {
    launch_one_block<T>(in, n, out, total, st);
    ZK_LAUNCH_CHECK();
    return 0;
  }
  int64_t* bsum = ws;
  int64_t* bbase = ws + nb;
  scan_reduce<T><<<(unsigned)nb, SCAN_T, 0, st>>>(in, n, bsum);
  ZK_LAUNCH_CHECK();
  int rc = scan_rec<int64_t>(bsum, bbase, nb, nullptr, ws + 2 * nb, st);
  if (rc) return rc;
  scan_apply<T><<<(unsigned)nb, SCAN_T, 0, st>>>(in, n, bbase, out, total);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // namespace zk

extern "C" {

// Workspace (int64 elements) needed by zk_scan_* for n inputs.
// Sized for the smallest block of any engine (one MFMA wave, 1024 values),
// an upper bound for the others.
// Also covers the encoders' per-256-record block sums and bases
// (2 * ceil(n / 256)).
int64_t zk_scan_workspace(int64_t n) {
  // the encoders: block sums, block bases, per-block flags (+2)
  const int64_t enc = 3 * ((n + 255) / 256) + 2;
  int64_t w = 0;
  while (n > zk::SCAN_E) {
    const int64_t nb = (n + zk::MS_WAVE_E - 1) / zk::MS_WAVE_E;
    w += 2 * nb;
    n = nb;
  }
  return w + 2 > enc ? w + 2 : enc;
}

// Exclusive scan of n values (any n) by one workgroup, one launch: the
// encoders' block sums.
int zk_scan_small_i64_mode(const int64_t* in, int64_t* out, int64_t n,
                           int64_t* total, int mode, hipStream_t st) {
  if (n <= 0) {
    if (total) return hipMemsetAsync(total, 0, sizeof(int64_t), st);
    return 0;
  }
  if (mode == 1)
    zk::scan_one_block_mfma<><<<1, zk::SB_T_MFMA, 0, st>>>(in, n, out, total);
  else
    zk::launch_one_block<int64_t>(in, n, out, total, st);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_scan_small_i64(const int64_t* in, int64_t* out, int64_t n,
                      int64_t* total, hipStream_t st) {
  return zk_scan_small_i64_mode(in, out, n, total, zk::small_scan_mode(), st);
}

// The one-workgroup scan's engine (1 = MFMA, 0 = shuffle), for
// tree_finish_scan (tree.hip) and the tests.
int zk_scan_small_mode(void) { return zk::small_scan_mode(); }

// 0 = shuffle engine, 1 = MFMA byte-plane engine; returns the old mode.
// 2 / 3 force one-wave / four-wave MFMA blocks (auto picks by n); 4 the
// multi-block MFMA path even where one workgroup would do (tests).
int zk_scan_set_mode(int mode) {
  const int old = zk::g_scan_mode;
  zk::g_scan_mode = (mode >= 0 && mode <= 4) ? mode : zk::SCAN_MFMA;
  return old;
}

int zk_scan_excl_i64(const int64_t* in, int64_t* out, int64_t n,
                     int64_t* total, int64_t* ws, hipStream_t st) {
  if (zk::g_scan_mode != zk::SCAN_SHFL)
    return zk::scan_mfma<int64_t>(in, out, n, total, ws, st, zk::g_scan_mode);
  return zk::scan_rec<int64_t>(in, out, n, total, ws, st);
}

int zk_scan_excl_i32(const int32_t* in, int64_t* out, int64_t n,
                     int64_t* total, int64_t* ws, hipStream_t st) {
  if (zk::g_scan_mode != zk::SCAN_SHFL)
    return zk::scan_mfma<int32_t>(in, out, n, total, ws, st, zk::g_scan_mode);
  return zk::scan_rec<int32_t>(in, out, n, total, ws, st);
}

}  // extern "C"
