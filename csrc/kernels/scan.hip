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

constexpr int MS_V = 16;                        // values per lane
constexpr int MS_WAVE_E = 64 * MS_V;            // 1024 per wave
typedef int v4i __attribute__((ext_vector_type(4)));

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

// Strictly lower-triangular ones, as this lane's A fragment for quarter q:
// A[i][k] = (k < 16q + i), lane l holding row i = l & 15 and the 16 k's
// 16 (l >> 4) + e.  B uses the same (lane, e) -> k map, so the sum over k is
// exact whatever order the hardware walks the k's in.
ZK_DEV v4i tri_frag(int q, int lane) {
  const int i = lane & 15, k0 = 16 * (lane >> 4), lim = 16 * q + i;
  v4i a;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    uint32_t x = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      x |= (uint32_t)(k0 + 4 * w + b < lim ? 1 : 0) << (8 * b);
    a[w] = (int)x;
  }
  return a;
}

// LDS staging: 64-value segments padded by 16 bytes, so the 16 lanes of a
// group reading their 16-value runs (ds_read_b128) hit distinct banks.
template <typename T>
ZK_DEV int lds_idx(int x) { return x + (x >> 6) * (int)(16 / sizeof(T)); }

template <typename T, int NT>
__global__ __launch_bounds__(NT) void scan_apply_mfma(
    const T* __restrict__ in, int64_t n, const int64_t* __restrict__ bbase,
    int64_t* __restrict__ out, int64_t* __restrict__ total) {
  constexpr int64_t MS_E = (int64_t)NT * MS_V;
  __shared__ int64_t stage[MS_E + (MS_E / 64) * 2];      // int64 slots
  __shared__ int64_t wsum[NT / 64 + 1];
  T* const tin = reinterpret_cast<T*>(stage);
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int j = lane & 15, g = lane >> 4;        // segment, lane group
  const int64_t bstart = (int64_t)blockIdx.x * MS_E;
  const bool full = bstart + MS_E <= n;

  // 1. coalesced global -> LDS
#pragma unroll
  for (int k = 0; k < MS_V; ++k) {
    const int x = tid + k * NT;
    tin[lds_idx<T>(x)] = (full || bstart + x < n) ? in[bstart + x] : (T)0;
  }
  __syncthreads();

  // 2. my 16-value run: segment j of wave w, values 16 g .. 16 g + 15
  const int r0 = w * 1024 + 64 * j + 16 * g;
  int64_t v[MS_V];
  int64_t s = 0;
  uint64_t orv = 0;
#pragma unroll
  for (int e = 0; e < MS_V; ++e) {
    v[e] = (int64_t)tin[lds_idx<T>(r0 + e)];
    s += v[e];
    orv |= (uint64_t)v[e];
  }

  // segment prefix over the 4 lane groups, then over the 16 segments
  const int64_t s0 = __shfl(s, j, 64), s1 = __shfl(s, j + 16, 64),
                s2 = __shfl(s, j + 32, 64), s3 = __shfl(s, j + 48, 64);
  const int64_t seg_tot = s0 + s1 + s2 + s3;
  const int64_t pre_g = (g > 0 ? s0 : 0) + (g > 1 ? s1 : 0) + (g > 2 ? s2 : 0);
  const int64_t seg_inc = wave_incl_scan(lane < 16 ? seg_tot : 0);
  const int64_t seg_base = __shfl(seg_inc, j, 64) - seg_tot;
  const int64_t wave_tot = __shfl(seg_inc, 15, 64);
  uint64_t wor = orv;                            // wave-uniform OR
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) wor |= __shfl_xor(wor, d, 64);

  // wave totals -> block prefix (this barrier also frees `stage`)
  if (lane == 0) wsum[w] = wave_tot;
  __syncthreads();
  const int64_t b0 = bbase ? bbase[blockIdx.x] : 0;
  int64_t wpre = b0;
  for (int x = 0; x < w; ++x) wpre += wsum[x];
  if (total != nullptr && blockIdx.x == gridDim.x - 1 && tid == NT - 1) {
    int64_t t = b0;
    for (int x = 0; x < NT / 64; ++x) t += wsum[x];
    *total = t;
  }
  const int64_t base = wpre + seg_base;          // segment j's start
  const int sbase = w * 1024 + 64 * j;           // segment j in `stage`

  // 3. prefixes -> LDS (int64 slots)
  if (wor >> 32) {
    // some value needs > 32 bits (or is negative): lane-serial, in the
    // layout this lane loaded
    int64_t p = base + pre_g;
#pragma unroll
    for (int e = 0; e < MS_V; ++e) {
      stage[lds_idx<int64_t>(r0 + e)] = p;
      p += v[e];
    }
  } else {
    const int planes = (wor >> 24) ? 4 : (wor >> 16) ? 3 : (wor >> 8) ? 2 : 1;
    // B fragments: plane p of my 16 values, biased to signed bytes
    v4i bfr[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t byte = (uint32_t)(v[4 * w4 + b] >> (8 * p)) & 255u;
          x |= ((byte - 128u) & 255u) << (8 * b);
        }
        bfr[p][w4] = (int)x;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4i a = tri_frag(q, lane);
      int64_t acc[4] = {0, 0, 0, 0};
      for (int p = 0; p < planes; ++p) {
        const v4i z = {0, 0, 0, 0};
        const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bfr[p], z, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int pos = 16 * q + 4 * g + r;    // row of D = position
          acc[r] += (int64_t)(d[r] + 128 * pos) << (8 * p);
        }
      }
      // D layout (16x16): col = lane & 15 (segment j), row = 4 (lane >> 4) + r
#pragma unroll
      for (int r = 0; r < 4; ++r)
        stage[lds_idx<int64_t>(sbase + 16 * q + 4 * g + r)] = base + acc[r];
    }
  }
  __syncthreads();

  // 4. coalesced LDS -> global
#pragma unroll
  for (int k = 0; k < MS_V; ++k) {
    const int x = tid + k * NT;
    if (full || bstart + x < n) out[bstart + x] = stage[lds_idx<int64_t>(x)];
  }
}

template <typename T>
static int scan_rec(const T* in, int64_t* out, int64_t n, int64_t* total,
                    int64_t* ws, hipStream_t st);

// NT = threads per block of the MFMA engine (64: one wave, 1024 values per
// block, many small blocks in flight; 256: 4096 per block).  A
// level that fits one shuffle block (<= SCAN_E values) is handed to the
// shuffle engine: one short launch beats the MFMA pipeline's latency there.
template <typename T, int NT>
static int scan_rec_mfma(const T* in, int64_t* out, int64_t n, int64_t* total,
                         int64_t* ws, hipStream_t st) {
  constexpr int64_t E = (int64_t)NT * MS_V;
  if (n <= SCAN_ONE_MAX) return scan_rec<T>(in, out, n, total, ws, st);
  const int64_t nb = (n + E - 1) / E;
  int64_t* bsum = ws;
  int64_t* bbase = ws + nb;
  scan_reduce_v<T, MS_V, NT><<<(unsigned)nb, NT, 0, st>>>(in, n, bsum);
  ZK_LAUNCH_CHECK();
  int rc = scan_rec_mfma<int64_t, NT>(bsum, bbase, nb, nullptr, ws + 2 * nb, st);
  if (rc) return rc;
  scan_apply_mfma<T, NT><<<(unsigned)nb, NT, 0, st>>>(in, n, bbase, out, total);
  ZK_LAUNCH_CHECK();
  return 0;
}

enum { SCAN_SHFL = 0, SCAN_MFMA = 1, SCAN_MFMA_W1 = 2, SCAN_MFMA_W4 = 3 };
static int g_scan_mode = SCAN_MFMA;

template <typename T>
static int scan_mfma(const T* in, int64_t* out, int64_t n, int64_t* total,
                     int64_t* ws, hipStream_t st, int mode) {
  // measured (profiles/r1_v10_scan_engines.md): one-wave blocks are as fast
  // or faster than four-wave ones at every n, so auto = one wave
  if (mode == SCAN_MFMA_W4)
    return scan_rec_mfma<T, 256>(in, out, n, total, ws, st);
  return scan_rec_mfma<T, 64>(in, out, n, total, ws, st);
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
int zk_scan_small_i64(const int64_t* in, int64_t* out, int64_t n,
                      int64_t* total, hipStream_t st) {
  if (n <= 0) {
    if (total) return hipMemsetAsync(total, 0, sizeof(int64_t), st);
    return 0;
  }
  zk::launch_one_block<int64_t>(in, n, out, total, st);
  ZK_LAUNCH_CHECK();
  return 0;
}

// 0 = shuffle engine, 1 = MFMA byte-plane engine; returns the old mode.
// 2 / 3 force one-wave / four-wave MFMA blocks (auto picks by n).
int zk_scan_set_mode(int mode) {
  const int old = zk::g_scan_mode;
  zk::g_scan_mode = (mode >= 0 && mode <= 3) ? mode : zk::SCAN_MFMA;
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
