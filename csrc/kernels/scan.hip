// Device-wide exclusive prefix sum (reduce-then-scan).
//
// Used by every variable-length encoder (record sizes -> byte offsets) and by
// the frame-table compaction (frames per tile -> frame index base).
//   pass 1: per-block reduce      (E = 256 threads x 8 elements)
//   pass 2: scan of block sums    (recursive when > E blocks)
//   pass 3: per-block scan + add block base
// Three short launches; at 1M records the whole scan is a few microseconds,
// far below the byte-moving kernels it feeds.
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
int64_t zk_scan_workspace(int64_t n) {
  int64_t w = 0;
  while (n > zk::SCAN_E) {
    const int64_t nb = (n + zk::SCAN_E - 1) / zk::SCAN_E;
    w += 2 * nb;
    n = nb;
  }
  return w + 2;
}

int zk_scan_excl_i64(const int64_t* in, int64_t* out, int64_t n,
                     int64_t* total, int64_t* ws, hipStream_t st) {
  return zk::scan_rec<int64_t>(in, out, n, total, ws, st);
}

int zk_scan_excl_i32(const int32_t* in, int64_t* out, int64_t n,
                     int64_t* total, int64_t* ws, hipStream_t st) {
  return zk::scan_rec<int32_t>(in, out, n, total, ws, st);
}

}  // extern "C"
