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
//   route_scatter_k  (its first workgroup: the per-owner counts)
//                    stable scatter: the rank of a request among its
//                    block's requests of the same owner comes from one
//                    wave ballot per owner plus an LDS prefix over waves
#include "zk_common.h"


namespace zk {

constexpr int RT_T = 256;
constexpr int RT_MAXW = 64;            // ranks a router splits over

ZK_DEV uint32_t fnv_word(uint32_t h, uint32_t w, int nb) {
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    if (b < nb) {
      h ^= (w >> (8 * b)) & 0xffu;
      h *= 16777619u;
    }
  }
  return h;
}

// FNV-1a 32 over the path bytes.  A path of up to 48 bytes (the usual) is
// loaded first, its whole 16-byte chunks issued together (unaligned mode)
// and the last partial one in 8 / 4 / 2 / 1-byte pieces, then
// hashed from registers: one memory round trip a request (a dword a step
// was one dependent load per 4 bytes, 49 us per 1M-request route).
ZK_DEV uint32_t path_fnv1a(const uint8_t* p, int32_t n) {
  uint32_t h = 2166136261u;
  if (n <= 48) {
    uint4 q[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int32_t o = 16 * j, left = n - o;
      if (left >= 16) {
        __builtin_memcpy(&q[j], p + o, 16);
      } else if (left > 0) {
        // the path's last partial chunk, read no further than its end (the
        // last path of an arena can end at its allocation's end)
        uint8_t* d = reinterpret_cast<uint8_t*>(&q[j]);
        q[j] = uint4{0, 0, 0, 0};
        int32_t k = 0;
        if (left - k >= 8) { __builtin_memcpy(d + k, p + o + k, 8); k += 8; }
        if (left - k >= 4) { __builtin_memcpy(d + k, p + o + k, 4); k += 4; }
        if (left - k >= 2) { __builtin_memcpy(d + k, p + o + k, 2); k += 2; }
        if (left - k >= 1) d[k] = p[o + k];
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const uint32_t w[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int left = n - 16 * j - 4 * d;
        if (left <= 0) return h;
        h = fnv_word(h, w[d], left < 4 ? left : 4);
      }
    }
    return h;
  }
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

// The groups' order: owner self first, then self + 1, ... (rotation), so
// a rank's own segment heads every stream and stays in place (seg_pack /
// seg_unpack SEG_INPLACE).  self = 0: rank order.
ZK_DEV int32_t rot_of(int32_t o, int32_t self, int32_t world) {
  const int32_t r = o - self;
  return r < 0 ? r + world : r;
}

__global__ __launch_bounds__(RT_T) void route_owner_k(
    int64_t n, int32_t world, int32_t self, const int64_t* __restrict__ poff,
    const int32_t* __restrict__ plen, const uint8_t* __restrict__ arena,
    int32_t* __restrict__ owner, int64_t* __restrict__ hist) {
  __shared__ int32_t h[RT_MAXW];
  if (threadIdx.x < world) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * RT_T + threadIdx.x;
  if (i < n) {
    const uint32_t o = path_fnv1a(arena + poff[i], plen[i]) % (uint32_t)world;
    owner[i] = (int32_t)o;
    atomicAdd(&h[rot_of((int32_t)o, self, world)], 1);
  }
  __syncthreads();
  if (threadIdx.x < world)
    hist[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// counts[w] = requests owned by rank w (sum of its histogram row; rows
// in rotation order): the scatter's first workgroup writes them.
ZK_DEV void route_counts(int64_t nblk, int32_t world, int32_t self,
                         const int64_t* __restrict__ base,
                         const int64_t* __restrict__ total,
                         int64_t* __restrict__ counts) {
  const int k = threadIdx.x;
  if (k >= world) return;
  const int64_t b0 = base[(int64_t)k * nblk];
  const int64_t b1 = k + 1 < world ? base[(int64_t)(k + 1) * nblk] : *total;
  const int w = k + self < world ? k + self : k + self - world;
  counts[w] = b1 - b0;
}

__global__ __launch_bounds__(RT_T) void route_scatter_k(
    int64_t n, int32_t world, int32_t self, const int64_t* __restrict__ total,
    int64_t* __restrict__ counts, const int32_t* __restrict__ owner,
    const int64_t* __restrict__ base, const int64_t* __restrict__ idx,
    const int32_t* __restrict__ xid, const int64_t* __restrict__ poff,
    const int32_t* __restrict__ plen, int64_t* __restrict__ idx_s,
    int32_t* __restrict__ xid_s, int64_t* __restrict__ poff_s,
    int32_t* __restrict__ plen_s) {
  __shared__ int32_t cnt[RT_T / WAVE][RT_MAXW];
  const int64_t i = (int64_t)blockIdx.x * RT_T + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (blockIdx.x == 0) route_counts(gridDim.x, world, self, base, total,
                                    counts);
  const int32_t o = i < n ? rot_of(owner[i], self, world) : -1;
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

// ---------------------------------------------------------------------------
// Fixed-capacity per-peer segments (the sync-free R2 exchange).
//
// all_to_all_single with equal splits needs no host-side split sizes, so a
// step never reads the device back: every rank sends each peer one slot of
// `slot_cap` bytes = a 16-byte header {payload bytes, records} (int64 x2)
// and the payload.  seg_pack_k cuts a framed stream whose records are
// grouped by destination (counts[w] consecutive records each) into the
// slots; seg_unpack_k concatenates the received slots' payloads back into
// one contiguous stream (source rank order) with its device length and the
// per-source record counts.  A segment that does not fit its slot is sent
// empty and counted in stats[0] (the receiving check then fails loudly).

constexpr int SG_T = 256;
constexpr int64_t SEG_HDR = 16;
// mode bit: segments in rotation order (this rank's first, as the router
// groups them with self) and this rank's own segment left where it is —
// seg_pack writes only its header (self slot = a 16-byte header), and
// seg_unpack's output is the packed stream's own buffer, which already
// starts with it: the local segment is never copied (requests and replies
// alike; with one rank the step copies nothing).
constexpr int32_t SEG_INPLACE = 1;

// Position of rank w's segment in a stream, and the records before it.
ZK_DEV int32_t seg_pos(int32_t w, int32_t self, int32_t world, int32_t mode) {
  if (!(mode & SEG_INPLACE)) return w;
  const int32_t r = w - self;
  return r < 0 ? r + world : r;
}
ZK_DEV int32_t seg_rank(int32_t k, int32_t self, int32_t world,
                        int32_t mode) {
  if (!(mode & SEG_INPLACE)) return k;
  return k + self < world ? k + self : k + self - world;
}

// Where the slot for / from rank w sits.  Without a separate self slot:
// w * slot_cap in `base`.  With one (`self_slot`, the all-to-all skips the
// local segment): the collective buffer holds the other ranks' slots in
// rank order with a 16-byte stub for this rank (all_to_all_single needs one
// chunk per rank; 16 bytes, not a slot, cross the collective), and the
// local segment lives in self_slot — no copy of it through the collective.
ZK_DEV uint8_t* slot_at(uint8_t* base, uint8_t* self_slot, int32_t w,
                        int32_t self, int64_t slot_cap) {
  if (self_slot == nullptr) return base + (int64_t)w * slot_cap;
  if (w == self) return self_slot;
  if (w < self) return base + (int64_t)w * slot_cap;
  return base + (int64_t)(w - 1) * slot_cap + SEG_HDR;
}

// Copy n bytes s -> d with the nt threads of a team (this thread is t):
// 16-byte stores aligned on the destination, 16-byte loads at any address
// (gfx950 unaligned mode); the ragged head and tail go byte by byte, so a
// team writes exactly its own bytes and neighbouring spans never race.
ZK_DEV void team_copy(uint8_t* __restrict__ d, const uint8_t* __restrict__ s,
                      int64_t n, int64_t t, int64_t nt) {
  if (n <= 0) return;
  int64_t head = (16 - (int64_t)((uintptr_t)d & 15)) & 15;
  if (head > n) head = n;
  if (t < head) d[t] = s[t];
  const int64_t body = (n - head) >> 4;
  uint8_t* db = d + head;
  const uint8_t* sb = s + head;
  for (int64_t k = t; k < body; k += nt) {
    uint4 v;
    __builtin_memcpy(&v, sb + 16 * k, 16);
    *reinterpret_cast<uint4*>(db + 16 * k) = v;
  }
  const int64_t t0 = head + 16 * body;
  if (t < n - t0) d[t0 + t] = s[t0 + t];
}

__global__ __launch_bounds__(SG_T) void seg_pack_k(
    const uint8_t* __restrict__ src, int64_t src_cap,
    const int64_t* __restrict__ rec_off, const int64_t* __restrict__ nrec_dev,
    int64_t nrec_cap, const int64_t* __restrict__ total,
    const int64_t* __restrict__ counts, int32_t world, int32_t self,
    int64_t slot_cap, uint8_t* __restrict__ out,
    unsigned long long* __restrict__ stats, uint8_t* __restrict__ self_out,
    int32_t mode) {
  const int32_t w = blockIdx.y;
  int64_t f = 0;
  const int32_t pw = seg_pos(w, self, world, mode);
  for (int32_t k = 0; k < pw; ++k) f += counts[seg_rank(k, self, world, mode)];
  const int64_t c = counts[w];
  int64_t nrec = nrec_cap;
  if (nrec_dev != nullptr && *nrec_dev < nrec) nrec = *nrec_dev;
  const int64_t tot = *total;
  const int64_t s0 = f < nrec ? rec_off[f] : tot;
  const int64_t e0 = f + c < nrec ? rec_off[f + c] : tot;
  const int64_t bytes = e0 - s0;
  const bool keep = (mode & SEG_INPLACE) && w == self;   // (s0 == 0)
  const bool ok = c >= 0 && f >= 0 && f + c <= nrec && s0 >= 0 &&
                  bytes >= 0 && e0 <= src_cap && bytes <= slot_cap - SEG_HDR &&
                  (!keep || s0 == 0);
  uint8_t* slot = slot_at(out, self_out, w, self, slot_cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t h[2] = {ok ? bytes : 0, ok ? c : 0};
    __builtin_memcpy(slot, h, 16);
    if (!ok) atomicAdd(&stats[0], 1ull);
    else if (w != self) {
      atomicAdd(&stats[1], (unsigned long long)bytes);
      atomicAdd(&stats[2], (unsigned long long)c);
    }
  }
  if (!ok || keep) return;
  team_copy(slot + SEG_HDR, src + s0, bytes,
            (int64_t)blockIdx.x * SG_T + threadIdx.x,
            (int64_t)gridDim.x * SG_T);
}

ZK_DEV void seg_hdr(const uint8_t* slot, int64_t slot_cap, int64_t* bytes,
                    int64_t* recs) {
  int64_t h[2];
  __builtin_memcpy(h, slot, 16);
  *bytes = h[0] < 0 ? 0 : (h[0] > slot_cap - SEG_HDR ? slot_cap - SEG_HDR
                                                      : h[0]);
  *recs = h[1] < 0 ? 0 : h[1];
}

__global__ __launch_bounds__(SG_T) void seg_unpack_k(
    const uint8_t* __restrict__ in, int32_t world, int32_t self,
    int64_t slot_cap, uint8_t* __restrict__ out,
    int64_t* __restrict__ total_out, int64_t* __restrict__ counts_out,
    unsigned long long* __restrict__ stats,
    const uint8_t* __restrict__ self_in, int32_t mode) {
  const int32_t w = blockIdx.y;
  auto slot = [&](int32_t k) {
    return (const uint8_t*)slot_at((uint8_t*)in, (uint8_t*)self_in, k, self,
                                   slot_cap);
  };
  int64_t pre = 0, mine = 0, all = 0, peers = 0;
  const int32_t pw = seg_pos(w, self, world, mode);
  for (int32_t k = 0; k < world; ++k) {
    int64_t b, r;
    seg_hdr(slot(k), slot_cap, &b, &r);
    if (seg_pos(k, self, world, mode) < pw) pre += b;
    if (k == w) mine = b;
    if (k != self) peers += b;
    all += b;
  }
  if (blockIdx.x == 0 && w == 0) {
    if (threadIdx.x == 0) {
      *total_out = all;
      if (stats != nullptr) atomicAdd(&stats[0], (unsigned long long)peers);
    }
    if (threadIdx.x < world) {
      int64_t b, r;
      seg_hdr(slot(threadIdx.x), slot_cap, &b, &r);
      counts_out[threadIdx.x] = r;
    }
  }
  if ((mode & SEG_INPLACE) && w == self) return;    // already at out[0]
  team_copy(out + pre, slot(w) + SEG_HDR, mine,
            (int64_t)blockIdx.x * SG_T + threadIdx.x,
            (int64_t)gridDim.x * SG_T);
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
// self: the groups in rotation order from owner self (route_owner_k).
int zk_route_requests2(int64_t n, int32_t world, int32_t self,
                       const int64_t* poff, const int32_t* plen,
                       const uint8_t* arena, const int64_t* idx,
                       const int32_t* xid, int32_t* owner, int64_t* idx_s,
                       int32_t* xid_s, int64_t* poff_s, int32_t* plen_s,
                       int64_t* counts, int64_t* ws, hipStream_t st);

int zk_route_requests(int64_t n, int32_t world, const int64_t* poff,
                      const int32_t* plen, const uint8_t* arena,
                      const int64_t* idx, const int32_t* xid, int32_t* owner,
                      int64_t* idx_s, int32_t* xid_s, int64_t* poff_s,
                      int32_t* plen_s, int64_t* counts, int64_t* ws,
                      hipStream_t st) {
  return zk_route_requests2(n, world, 0, poff, plen, arena, idx, xid, owner,
                            idx_s, xid_s, poff_s, plen_s, counts, ws, st);
}

int zk_route_requests2(int64_t n, int32_t world, int32_t self,
                       const int64_t* poff, const int32_t* plen,
                       const uint8_t* arena, const int64_t* idx,
                       const int32_t* xid, int32_t* owner, int64_t* idx_s,
                       int32_t* xid_s, int64_t* poff_s, int32_t* plen_s,
                       int64_t* counts, int64_t* ws, hipStream_t st) {
  if (world < 1 || world > zk::RT_MAXW || self < 0 || self >= world)
    return (int)hipErrorInvalidValue;
  if (n <= 0) return hipMemsetAsync(counts, 0, sizeof(int64_t) * world, st);
  const int64_t nblk = (n + zk::RT_T - 1) / zk::RT_T;
  const int64_t m = nblk * world;
  int64_t* hist = ws;
  int64_t* base = ws + m;
  int64_t* total = ws + 2 * m;
  int64_t* sws = ws + 2 * m + 8;
  zk::route_owner_k<<<(unsigned)nblk, zk::RT_T, 0, st>>>(
      n, world, self, poff, plen, arena, owner, hist);
  ZK_LAUNCH_CHECK();
  int rc = zk_scan_excl_i64(hist, base, m, total, sws, st);
  if (rc) return rc;
  zk::route_scatter_k<<<(unsigned)nblk, zk::RT_T, 0, st>>>(
      n, world, self, total, counts, owner, base, idx, xid, poff, plen, idx_s,
      xid_s, poff_s, plen_s);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Team size per segment: enough blocks to stream a full slot, at most 512.
static unsigned seg_blocks(int64_t slot_cap) {
  int64_t b = (slot_cap + 16 * zk::SG_T - 1) / (16 * zk::SG_T);
  return (unsigned)(b < 1 ? 1 : (b > 512 ? 512 : b));
}

// Pack the framed stream src (records at rec_off, nrec = min(*nrec_dev,
// nrec_cap) of them, *total bytes) into `world` slots of slot_cap bytes:
// slot w gets records [sum(counts[:w]), +counts[w]).  stats (uint64 [3]):
// += segments that did not fit, payload bytes and records for peers.
// self_out (may be null): this rank's own slot, apart from `out` (see
// slot_at; `out` then holds (world - 1) slots + a 16-byte stub).
int zk_seg_pack(const uint8_t* src, int64_t src_cap, const int64_t* rec_off,
                const int64_t* nrec_dev, int64_t nrec_cap,
                const int64_t* total, const int64_t* counts, int32_t world,
                int32_t self, int64_t slot_cap, uint8_t* out,
                unsigned long long* stats, uint8_t* self_out, int32_t mode,
                hipStream_t st) {
  if (world < 1 || world > zk::RT_MAXW || slot_cap < 32 || (slot_cap & 15))
    return (int)hipErrorInvalidValue;
  if ((mode & zk::SEG_INPLACE) && self_out == nullptr)
    return (int)hipErrorInvalidValue;
  dim3 grid(seg_blocks(slot_cap), (unsigned)world);
  zk::seg_pack_k<<<grid, zk::SG_T, 0, st>>>(
      src, src_cap, rec_off, nrec_dev, nrec_cap, total, counts, world, self,
      slot_cap, out, stats, self_out, mode);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Concatenate the payloads of `world` received slots into out (source rank
// order); *total_out = its length, counts_out[w] = records from rank w,
// stats[0] (optional) += payload bytes from the other ranks.  out must hold
// world * (slot_cap - 16) bytes.
// self_in (may be null): this rank's own slot, apart from `in` (slot_at).
int zk_seg_unpack(const uint8_t* in, int32_t world, int32_t self,
                  int64_t slot_cap, uint8_t* out, int64_t* total_out,
                  int64_t* counts_out, unsigned long long* stats,
                  const uint8_t* self_in, int32_t mode, hipStream_t st) {
  if (world < 1 || world > zk::RT_MAXW || slot_cap < 32 || (slot_cap & 15))
    return (int)hipErrorInvalidValue;
  if ((mode & zk::SEG_INPLACE) && self_in == nullptr)
    return (int)hipErrorInvalidValue;
  dim3 grid(seg_blocks(slot_cap), (unsigned)world);
  zk::seg_unpack_k<<<grid, zk::SG_T, 0, st>>>(in, world, self, slot_cap, out,
                                               total_out, counts_out, stats,
                                               self_in, mode);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
