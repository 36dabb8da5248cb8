// Benchmark-side helpers for the synthetic pipelines
// (zkmi/bench/synthetic.py GetPipeline, WatchPipeline): request generation
// and the per-reply validation, each ONE fused kernel instead of ~15 small
// torch element-wise launches per step.  Semantics are those of the torch code
// they replace: uniform random node per request, consecutive xids, and a
// reply counts as OK only if it decoded cleanly, carries err OK, opcode
// GET_DATA, the request's xid, czxid == node + 1 and the node's data length.
#include "zk_common.h"

namespace zk {

constexpr int BG_T = 256;

// splitmix64: counter-based, so step s / request i always draw the same node
ZK_DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}


// With `sizes` / `bsum`, also the K10 encode's sizes pass for these
// GET_DATA requests (zk_encode_requests_presized: one launch less a step):
// each frame's bytes (length word, xid, op, path buffer, watch flag) and
// each 256-request block's sum, as req_sizes writes them.
__global__ __launch_bounds__(BG_T) void bench_gen_get(
    int64_t n, uint64_t seed, int64_t leaf0, int64_t nleaves,
    int32_t xid_base, const int64_t* __restrict__ node_pw,
    int64_t* __restrict__ idx, int32_t* __restrict__ xid,
    int64_t* __restrict__ path_off, int32_t* __restrict__ path_len,
    const int64_t* __restrict__ state, int64_t* __restrict__ sizes,
    int64_t* __restrict__ bsum) {
  static_assert(BG_T == 256, "the encoder's blocks (ENC_T)");
  const int64_t i = (int64_t)blockIdx.x * BG_T + threadIdx.x;
  int64_t sz = 0;
  if (i < n) {
    if (state != nullptr) {
      // device-resident {seed, step} (a captured graph replays new
      // batches): the step's seed and xids derive from the step counter
      const uint64_t st = (uint64_t)state[1];
      seed = (uint64_t)state[0] * 0x9E3779B97F4A7C15ull + st;
      xid_base = (int32_t)((st * (uint64_t)n) & 0x7fffffffu);
    }
    const uint64_t r = splitmix64(seed ^ (uint64_t)i * 0xD1B54A32D192ED03ull);
    // multiply-shift range reduction (bias < 2^-32 for 1M leaves)
    const int64_t v = leaf0 + (int64_t)(((r >> 32) * (uint64_t)nleaves) >> 32);
    idx[i] = v;
    xid[i] = (int32_t)(((uint32_t)xid_base + (uint32_t)i) & 0x7fffffffu);
    const int64_t pw = node_pw[v];         // offset << 24 | length (tree.hip)
    const int32_t pl = (int32_t)(pw & 0xFFFFFF);
    path_off[i] = pw >> 24;
    path_len[i] = pl;
    // the frame: length word, xid, op, path buffer, watch flag
    sz = 4 + 4 + 4 + 4 + pl + 1;
    if (sizes != nullptr) sizes[i] = sz;
  }
  if (sizes != nullptr) {                  // (block-uniform)
    __shared__ int64_t sm[BG_T / 64 + 1];
    int64_t tot;
    block_excl_scan(sz, sm, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
  }
}

// Grid-stride with a bounded grid: one device-scope atomic per block, and a
// single counter word sustains only ~88 returning atomics per microsecond
// (MI355X_MICROARCH.md "dequeue"), so 4096 one-shot blocks would serialise
// ~46 us on it.
constexpr int BG_CHECK_BLOCKS = 512;

__global__ __launch_bounds__(BG_T) void bench_check_get(
    int64_t n, const int32_t* __restrict__ status,
    const int32_t* __restrict__ err, const int32_t* __restrict__ opcode,
    const int32_t* __restrict__ rxid, const int64_t* __restrict__ czxid,
    const int32_t* __restrict__ pay_len, const int64_t* __restrict__ idx,
    const int32_t* __restrict__ xid, const int32_t* __restrict__ data_len,
    unsigned long long* __restrict__ ok) {
  __shared__ int64_t sm[BG_T / 64 + 1];
  int64_t good = 0;
  for (int64_t i = (int64_t)blockIdx.x * BG_T + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * BG_T) {
    const int64_t v = idx[i];
    good += status[i] == 0 && err[i] == 0 && opcode[i] == OP_GET_DATA &&
            rxid[i] == xid[i] && czxid[i] == v + 1 &&
            pay_len[i] == data_len[v];
  }
  int64_t tot;
  block_excl_scan(good, sm, &tot);
  if (threadIdx.x == 0 && tot) atomicAdd(ok, (unsigned long long)tot);
}

// Watch fan-out (zkmi/bench/synthetic.py WatchPipeline): every rank
// receives the notification streams of all ranks (R1 all-gather), decodes
// them (K1 + K8) and checks each record against the node its producer drew:
// record i belongs to producer rank i / n_per, index i % n_per, drawn with
// seeds[rank] exactly as bench_gen_get draws it.  OK = clean decode,
// NOTIFICATION, err OK, type NodeDataChanged, state SyncConnected and the
// path bytes equal to the node's path.  With `want` (int64 [total]) record
// i must name node want[i] instead (the write-triggered workload: the
// nodes a writer set, in write order).
__global__ __launch_bounds__(BG_T) void bench_check_notif(
    int64_t total, int64_t n_per, const uint64_t* __restrict__ seeds,
    const int64_t* __restrict__ want,
    int64_t leaf0, int64_t nleaves, const int64_t* __restrict__ node_path_off,
    const int32_t* __restrict__ node_path_len,
    const uint8_t* __restrict__ path_arena, const uint8_t* __restrict__ rx,
    const int32_t* __restrict__ status, const int32_t* __restrict__ err,
    const int32_t* __restrict__ opcode, const int32_t* __restrict__ aux0,
    const int32_t* __restrict__ aux1, const int64_t* __restrict__ pay_off,
    const int32_t* __restrict__ pay_len, unsigned long long* __restrict__ ok) {
  __shared__ int64_t sm[BG_T / 64 + 1];
  int64_t good = 0;
  for (int64_t i = (int64_t)blockIdx.x * BG_T + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * BG_T) {
    int64_t v;
    if (want != nullptr) {
      v = want[i];
    } else {
      const int64_t r = i / n_per, j = i - r * n_per;
      const uint64_t h =
          splitmix64(seeds[r] ^ (uint64_t)j * 0xD1B54A32D192ED03ull);
      v = leaf0 + (int64_t)(((h >> 32) * (uint64_t)nleaves) >> 32);
    }
    const bool inr = v >= leaf0 && v < leaf0 + nleaves;
    const int32_t pl = inr ? node_path_len[v] : -1;
    bool g = inr && status[i] == 0 && err[i] == 0 && opcode[i] == OP_NOTIFICATION &&
             aux0[i] == 3 && aux1[i] == 3 && pay_len[i] == pl;
    if (g) {
      const uint8_t* a = rx + pay_off[i];
      const uint8_t* b = path_arena + node_path_off[v];
      for (int32_t k = 0; k < pl && g; ++k) g = a[k] == b[k];
    }
    good += g;
  }
  int64_t tot;
  block_excl_scan(good, sm, &tot);
  if (threadIdx.x == 0 && tot) atomicAdd(ok, (unsigned long long)tot);
}

// A write batch's consecutive xids: xid[i] = (*base + i) mod 2^31 (the
// session's next xid on the device; the caller advances it).  One launch
// for what took an add, a mask and a narrowing copy of a 64-bit iota.
__global__ __launch_bounds__(BG_T) void bench_xids(
    int64_t n, const int64_t* __restrict__ base, int32_t* __restrict__ xid) {
  const int64_t i = (int64_t)blockIdx.x * BG_T + threadIdx.x;
  if (i < n) xid[i] = (int32_t)((uint64_t)(*base + i) & 0x7fffffffu);
}

// The write pipelines' per-reply check in one pass (the storm's: clean
// decode, err OK, the request's xid, the expected payload length) counted
// into *ok, and the batch's largest reply zxid folded into *zmax — eight
// element-wise launches and two reductions over the batch before.
// want_len: per request (want_len_c < 0) or the constant want_len_c.
__global__ __launch_bounds__(BG_T) void bench_check_writes(
    int64_t n, const int32_t* __restrict__ status,
    const int32_t* __restrict__ err, const int32_t* __restrict__ rxid,
    const int32_t* __restrict__ xid, const int32_t* __restrict__ pay_len,
    const int32_t* __restrict__ want_len, int32_t want_len_c,
    const int64_t* __restrict__ zxid, unsigned long long* __restrict__ ok,
    unsigned long long* __restrict__ zmax) {
  __shared__ int64_t sm[BG_T / 64 + 1];
  __shared__ unsigned long long zw[BG_T / 64];
  constexpr int U = 4;               // requests a thread, loads issued first
  int64_t good = 0;
  unsigned long long zm = 0;         // (zxids are >= 0)
  const int64_t stride = (int64_t)gridDim.x * BG_T;
  for (int64_t i0 = (int64_t)blockIdx.x * BG_T + threadIdx.x; i0 < n;
       i0 += U * stride) {
    int32_t s[U], e[U], rx[U], x[U], pl[U], wl[U];
    int64_t z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      const bool in = i < n;
      s[u] = in ? status[i] : 1;
      e[u] = in ? err[i] : 0;
      rx[u] = in ? rxid[i] : 0;
      x[u] = in ? xid[i] : 0;
      pl[u] = in ? pay_len[i] : 0;
      wl[u] = in ? (want_len_c >= 0 ? want_len_c : want_len[i]) : 0;
      z[u] = in ? zxid[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      good += s[u] == 0 && e[u] == 0 && rx[u] == x[u] && pl[u] == wl[u];
      zm = max(zm, (unsigned long long)z[u]);
    }
  }
  int64_t tot;
  block_excl_scan(good, sm, &tot);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1)
    zm = max(zm, (unsigned long long)__shfl_xor((long long)zm, d, 64));
  if ((threadIdx.x & 63) == 0) zw[threadIdx.x >> 6] = zm;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
#pragma unroll
    for (int w = 0; w < BG_T / 64; ++w) b = max(b, zw[w]);
    if (b) atomicMax(zmax, b);
    if (tot) atomicAdd(ok, (unsigned long long)tot);
  }
}

// The storm's handshake check and credential update in one single-lane
// launch (about fifteen one-element tensor ops a step before, each a
// kernel): a resume must come back RESUMED with the current session's id,
// password and timeout, and the expired session tried beside it (`prev`)
// refused with id 0; a birth must be NEW with the id the step expects
// (`want`), which with its password becomes the current credentials (the
// old current ones the previous).  hs_ok &= the outcome.
__global__ void bench_storm_hs(int32_t resume, int32_t prev, int32_t timeout,
                               const int32_t* __restrict__ status,
                               const int64_t* __restrict__ sid,
                               const int32_t* __restrict__ tmo,
                               const int32_t* __restrict__ outcome,
                               const int64_t* __restrict__ bound,
                               const uint8_t* __restrict__ resp,
                               const int64_t* __restrict__ want,
                               int64_t* __restrict__ cred_sid,
                               uint8_t* __restrict__ cred_pw,
                               bool* __restrict__ hs_ok) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  bool ok;
  if (resume) {
    ok = status[0] == 0 && sid[0] == cred_sid[0] && outcome[0] == SC_RESUMED &&
         tmo[0] == timeout;
    for (int k = 0; k < 16; ++k) ok = ok && resp[24 + k] == cred_pw[k];
    if (prev) ok = ok && outcome[1] == SC_EXPIRED && sid[1] == 0;
  } else {
    const int64_t w = *want;
    ok = status[0] == 0 && outcome[0] == SC_NEW && sid[0] == w && bound[0] == w;
    cred_sid[1] = cred_sid[0];
    for (int k = 0; k < 16; ++k) cred_pw[16 + k] = cred_pw[k];
    cred_sid[0] = sid[0];
    for (int k = 0; k < 16; ++k) cred_pw[k] = resp[24 + k];
  }
  *hs_ok = *hs_ok && ok;
}

}  // namespace zk

extern "C" {

int zk_bench_storm_hs(int32_t resume, int32_t prev, int32_t timeout,
                      const int32_t* status, const int64_t* sid,
                      const int32_t* tmo, const int32_t* outcome,
                      const int64_t* bound, const uint8_t* resp,
                      const int64_t* want, int64_t* cred_sid,
                      uint8_t* cred_pw, bool* hs_ok, hipStream_t st) {
  zk::bench_storm_hs<<<1, 64, 0, st>>>(resume, prev, timeout, status, sid, tmo,
                                       outcome, bound, resp, want, cred_sid,
                                       cred_pw, hs_ok);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_bench_xids(int64_t n, const int64_t* base, int32_t* xid,
                  hipStream_t st) {
  if (n <= 0) return 0;
  zk::bench_xids<<<(unsigned)((n + zk::BG_T - 1) / zk::BG_T), zk::BG_T, 0,
                   st>>>(n, base, xid);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_bench_check_writes(int64_t n, const int32_t* status, const int32_t* err,
                          const int32_t* rxid, const int32_t* xid,
                          const int32_t* pay_len, const int32_t* want_len,
                          int32_t want_len_c, const int64_t* zxid,
                          unsigned long long* ok, unsigned long long* zmax,
                          hipStream_t st) {
  if (n <= 0) return 0;
  // four requests a thread in one pass (two atomics a block: 2048 for a
  // 1M-request batch)
  const int64_t nb = min((n + 4 * zk::BG_T - 1) / (4 * zk::BG_T),
                         (int64_t)(2 * zk::BG_CHECK_BLOCKS));
  zk::bench_check_writes<<<(unsigned)nb, zk::BG_T, 0, st>>>(
      n, status, err, rxid, xid, pay_len, want_len, want_len_c, zxid, ok,
      zmax);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_bench_check_notif(int64_t total, int64_t n_per, const uint64_t* seeds,
                         const int64_t* want, int64_t leaf0, int64_t nleaves,
                         const int64_t* node_path_off,
                         const int32_t* node_path_len,
                         const uint8_t* path_arena, const uint8_t* rx,
                         const int32_t* status, const int32_t* err,
                         const int32_t* opcode, const int32_t* aux0,
                         const int32_t* aux1, const int64_t* pay_off,
                         const int32_t* pay_len, unsigned long long* ok,
                         hipStream_t st) {
  if (total <= 0 || n_per <= 0) return 0;
  const int64_t nb = min((total + zk::BG_T - 1) / zk::BG_T,
                         (int64_t)zk::BG_CHECK_BLOCKS);
  zk::bench_check_notif<<<(unsigned)nb, zk::BG_T, 0, st>>>(
      total, n_per, seeds, want, leaf0, nleaves, node_path_off, node_path_len,
      path_arena, rx, status, err, opcode, aux0, aux1, pay_off, pay_len, ok);
  ZK_LAUNCH_CHECK();
  return 0;
}

// sizes / bsum (both or neither): the encode's sizes pass too (see the
// kernel; bsum holds one int64 per 256 requests)
int zk_bench_gen_get(int64_t n, uint64_t seed, int64_t leaf0, int64_t nleaves,
                     int32_t xid_base, const int64_t* node_pw, int64_t* idx,
                     int32_t* xid, int64_t* path_off, int32_t* path_len,
                     const int64_t* state, int64_t* sizes, int64_t* bsum,
                     hipStream_t st) {
  if (n <= 0) return 0;
  if ((sizes == nullptr) != (bsum == nullptr)) return (int)hipErrorInvalidValue;
  zk::bench_gen_get<<<(unsigned)((n + zk::BG_T - 1) / zk::BG_T), zk::BG_T, 0,
                      st>>>(n, seed, leaf0, nleaves, xid_base, node_pw, idx,
                            xid, path_off, path_len, state, sizes, bsum);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_bench_check_get(int64_t n, const int32_t* status, const int32_t* err,
                       const int32_t* opcode, const int32_t* rxid,
                       const int64_t* czxid, const int32_t* pay_len,
                       const int64_t* idx, const int32_t* xid,
                       const int32_t* data_len, unsigned long long* ok,
                       hipStream_t st) {
  if (n <= 0) return 0;
  const int64_t nb = min((n + zk::BG_T - 1) / zk::BG_T,
                         (int64_t)zk::BG_CHECK_BLOCKS);
  zk::bench_check_get<<<(unsigned)nb, zk::BG_T, 0, st>>>(
      n, status, err, opcode, rxid, czxid, pay_len, idx, xid, data_len, ok);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
