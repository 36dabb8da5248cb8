// R2 request router (zkmi/parallel/sharded.py): the owner rank of every
// request is FNV-1a(path) % world, and the request descriptors are split
// stably by owner, so each owner's requests are contiguous and K10 encodes
// one byte segment per destination rank for the all-to-all over xGMI.
//
// The reference pipelines every request of a client over its one
// connection, keyed by xid (lib/connection-fsm.js:384-408); on a node of
// GPU sessions the pipeline is partitioned by the rank that serves a path.
//
// Three passes, no host read:
//   route_owner_k    owner per request + per-block owner histogram in LDS
//   (scan)           exclusive scan of the histogram in owner-major order
//                    (zk_scan_excl_i64): base of every (owner, block) run
//   route_scatter_k  stable scatter: the rank of a request among its
//                    block's requests of the same owner comes from one
//                    wave ballot per owner plus an LDS prefix over waves
#include "zk_common.h"

extern "C" int zk_scan_excl_i64(const int64_t* in, int64_t* out, int64_t n,
                                int64_t* total, int64_t* ws, hipStream_t st);

namespace zk {

constexpr int RT_T = 256;
constexpr int RT_MAXW = 64;            // ranks a router splits over

// FNV-1a 32 over the path bytes, read a dword at a time (unaligned mode).
ZK_DEV uint32_t path_fnv1a(const uint8_t* p, int32_t n) {
  uint32_t h = 2166136261u;
  int32_t k = 0;
  for (; k + 4 <= n; k += 4) {
    uint32_t w;
    __builtin_memcpy(&w, p + k, 4);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      h ^= (w >> (8 * b)) & 0xffu;
      h *= 16777619u;
    }
  }
  for (; k < n; ++k) { h ^= p[k]; h *= 16777619u; }
  return h;
}

__global__ __launch_bounds__(RT_T) void route_owner_k(
    int64_t n, int32_t world, const int64_t* __restrict__ poff,
    const int32_t* __restrict__ plen, const uint8_t* __restrict__ arena,
    int32_t* __restrict__ owner, int64_t* __restrict__ hist) {
  __shared__ int32_t h[RT_MAXW];
  if (threadIdx.x < world) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * RT_T + threadIdx.x;
  if (i < n) {
    const uint32_t o = path_fnv1a(arena + poff[i], plen[i]) % (uint32_t)world;
    owner[i] = (int32_t)o;
    atomicAdd(&h[o], 1);
  }
  __syncthreads();
  if (threadIdx.x < world)
    hist[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(RT_T) void route_scatter_k(
    int64_t n, int32_t world, const int32_t* __restrict__ owner,
    const int64_t* __restrict__ base, const int64_t* __restrict__ idx,
    const int32_t* __restrict__ xid, const int64_t* __restrict__ poff,
    const int32_t* __restrict__ plen, int64_t* __restrict__ idx_s,
    int32_t* __restrict__ xid_s, int64_t* __restrict__ poff_s,
    int32_t* __restrict__ plen_s) {
  __shared__ int32_t cnt[RT_T / WAVE][RT_MAXW];
  const int64_t i = (int64_t)blockIdx.x * RT_T + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t o = i < n ? owner[i] : -1;
  const uint64_t below = (1ull << lane) - 1;
  int32_t r = 0;
  for (int32_t w = 0; w < world; ++w) {
    const uint64_t m = __ballot(o == w);
    if (o == w) r = __popcll(m & below);
    if (lane == 0) cnt[wv][w] = __popcll(m);
  }
  __syncthreads();
  if (i >= n) return;
  for (int k = 0; k < wv; ++k) r += cnt[k][o];
  const int64_t pos = base[(int64_t)o * gridDim.x + blockIdx.x] + r;
  idx_s[pos] = idx[i];
  xid_s[pos] = xid[i];
  poff_s[pos] = poff[i];
  plen_s[pos] = plen[i];
}

// counts[w] = requests owned by rank w (sum of its histogram row).
__global__ __launch_bounds__(RT_T) void route_counts_k(
    int64_t nblk, int32_t world, const int64_t* __restrict__ base,
    const int64_t* __restrict__ total, int64_t* __restrict__ counts) {
  const int w = threadIdx.x;
  if (w >= world) return;
  const int64_t b0 = base[(int64_t)w * nblk];
  const int64_t b1 = w + 1 < world ? base[(int64_t)(w + 1) * nblk] : *total;
  counts[w] = b1 - b0;
}

}  // namespace zk

extern "C" {

// int64 scratch a route of n requests over `world` ranks needs: the
// histogram, its scan, the scan total and the scan workspace.
int64_t zk_route_workspace(int64_t n, int32_t world);

int64_t zk_scan_workspace(int64_t n);

int64_t zk_route_workspace(int64_t n, int32_t world) {
  const int64_t nblk = (n + zk::RT_T - 1) / zk::RT_T;
  const int64_t m = nblk * world;
  return 2 * m + 8 + zk_scan_workspace(m);
}

// Route n request descriptors (idx, xid, path off/len) to `world` owners:
// writes owner[n], the owner-grouped descriptors (*_s) and counts[world].
int zk_route_requests(int64_t n, int32_t world, const int64_t* poff,
                      const int32_t* plen, const uint8_t* arena,
                      const int64_t* idx, const int32_t* xid, int32_t* owner,
                      int64_t* idx_s, int32_t* xid_s, int64_t* poff_s,
                      int32_t* plen_s, int64_t* counts, int64_t* ws,
                      hipStream_t st) {
  if (world < 1 || world > zk::RT_MAXW) return (int)hipErrorInvalidValue;
  if (n <= 0) return hipMemsetAsync(counts, 0, sizeof(int64_t) * world, st);
  const int64_t nblk = (n + zk::RT_T - 1) / zk::RT_T;
  const int64_t m = nblk * world;
  int64_t* hist = ws;
  int64_t* base = ws + m;
  int64_t* total = ws + 2 * m;
  int64_t* sws = ws + 2 * m + 8;
  zk::route_owner_k<<<(unsigned)nblk, zk::RT_T, 0, st>>>(
      n, world, poff, plen, arena, owner, hist);
  ZK_LAUNCH_CHECK();
  int rc = zk_scan_excl_i64(hist, base, m, total, sws, st);
  if (rc) return rc;
  zk::route_counts_k<<<1, zk::RT_T, 0, st>>>(nblk, world, base, total,
                                              counts);
  ZK_LAUNCH_CHECK();
  zk::route_scatter_k<<<(unsigned)nblk, zk::RT_T, 0, st>>>(
      n, world, owner, base, idx, xid, poff, plen, idx_s, xid_s, poff_s,
      plen_s);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
