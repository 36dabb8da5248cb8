// Batched Jute decoders: client replies (K2 header + opcode resolve, K3 Stat,
// K4 GET_DATA, K5 children, K6 ACL, K7 create/exists/set_data, K8
// notifications) and server-mode requests (K12).
// Reference: lib/zk-buffer.js:275-442 (replies), :58-253 (requests).
//
// One thread per frame; inputs come from the frame table produced by
// frame_scan.hip (body offset + length into the RX buffer).  Payloads are
// never copied: data, paths and string vectors are returned as (offset,
// length) into the RX buffer, so a GET_DATA reply costs its 16-byte header,
// 4-byte length and 68-byte Stat in loads regardless of the data size.
// Outputs are SoA so the consumer (Python / the next kernel) reads them
// coalesced.  Ragged vectors (children, ACL entries, SET_WATCHES paths) are
// expanded by a second pass after a scan of the per-frame counts.
#include "zk_common.h"
#include "zk_reqparse.h"

namespace zk {

constexpr int DEC_T = 256;

// A Stat already in registers: the frame's last 68 bytes as 17 dwords in
// memory order (see decode_replies_k).
ZK_DEV void read_stat_regs(const uint32_t* w, const ZkReplyOut& o, int64_t i) {
  const int64_t c = o.cap;
  auto b32 = [&](int k) { return (int32_t)bswap32(w[k]); };
  auto b64 = [&](int k) {
    return (int64_t)(((uint64_t)bswap32(w[k]) << 32) | bswap32(w[k + 1]));
  };
  o.stat64[0 * c + i] = b64(0);
  o.stat64[1 * c + i] = b64(2);
  o.stat64[2 * c + i] = b64(4);
  o.stat64[3 * c + i] = b64(6);
  o.stat32[0 * c + i] = b32(8);
  o.stat32[1 * c + i] = b32(9);
  o.stat32[2 * c + i] = b32(10);
  o.stat64[4 * c + i] = b64(11);
  o.stat32[3 * c + i] = b32(13);
  o.stat32[4 * c + i] = b32(14);
  o.stat64[5 * c + i] = b64(15);
}

ZK_DEV bool read_stat(const uint8_t* p, const ZkReplyOut& o, int64_t i) {
  const int64_t c = o.cap;
  o.stat64[0 * c + i] = ld_be64(p + 0);
  o.stat64[1 * c + i] = ld_be64(p + 8);
  o.stat64[2 * c + i] = ld_be64(p + 16);
  o.stat64[3 * c + i] = ld_be64(p + 24);
  o.stat32[0 * c + i] = ld_be32(p + 32);
  o.stat32[1 * c + i] = ld_be32(p + 36);
  o.stat32[2 * c + i] = ld_be32(p + 40);
  o.stat64[4 * c + i] = ld_be64(p + 44);
  o.stat32[3 * c + i] = ld_be32(p + 52);
  o.stat32[4 * c + i] = ld_be32(p + 56);
  o.stat64[5 * c + i] = ld_be64(p + 60);
  return true;
}


// Optional fused check of GET_DATA replies against the requests that were
// sent (the benchmark's validation, otherwise a separate pass over the SoA
// it just wrote): reply i must be a clean GET_DATA success for request i —
// same xid, the node's czxid (idx + 1) and data length; with `slab` also
// the payload BYTES of one reply in 16 (which ones rotates with the step
// counter), compared against the node's slot in the tree's slab — a
// corrupted copy that keeps the length fails the check.  Counts go to
// acc[block % slots] (one atomic per block, spread over the slots so the
// blocks of a launch do not queue on one word).
struct ZkGetCheck {
  const int64_t* idx;
  const int32_t* xid;
  const int32_t* data_len;
  unsigned long long* acc;
  int32_t slots;
  int64_t* tick;   // optional: tick[1] += 1 once per launch (a captured
                   // graph's step counter, see bench_gen_get's state)
  const uint8_t* slab;        // optional: the payload sample's reference
  const int64_t* slot_off;
};
constexpr int CHK_SAMPLE = 16;

// Wave-cooperative byte comparison: do n bytes at a (any alignment;
// readable up to 19 bytes past a + n — a reply's data is followed by its
// 68-byte Stat) equal n bytes at b (4-byte aligned; a node slot, padded
// past its data capacity)?  Lane l compares bytes [16 l, 16 l + 16) of
// every 1 KiB: aligned dword loads funnel-shifted into place.  All lanes of
// the wave call it with the same arguments.
ZK_DEV bool wave_bytes_equal(const uint8_t* a, const uint8_t* b, int32_t n,
                             int lane) {
  uint32_t diff = 0;
  for (int32_t o = 16 * lane; o < n; o += 1024) {
    const uintptr_t ua = (uintptr_t)(a + o);
    const uint32_t* wa = (const uint32_t*)(ua & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(ua & 3);
    const uint32_t* wb = (const uint32_t*)(b + o);
    uint32_t va[5], vb[4];
#pragma unroll
    for (int q = 0; q < 5; ++q) va[q] = wa[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) vb[q] = wb[q];
    const int32_t rem = n - o;                 // bytes of this chunk in n
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int32_t keep = rem - 4 * q;        // bytes of dword q in n
      const uint32_t mask = keep >= 4 ? 0xFFFFFFFFu
                          : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
      diff |= (__builtin_amdgcn_alignbyte(va[q + 1], va[q], sh) ^ vb[q]) &
              mask;
    }
  }
  return __ballot(diff != 0) == 0;
}

template <bool CHECK>
__global__ __launch_bounds__(DEC_T) void decode_replies_k(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ foff,
    const int32_t* __restrict__ flen, const int64_t* __restrict__ n_dev,
    int64_t ncap, const int64_t* __restrict__ xid_tab, int64_t xid_mask,
    ZkReplyOut o, ZkGetCheck chk) {
  const uint32_t nwg = gridDim.x;
  const int64_t i = (int64_t)xcd_remap(blockIdx.x, nwg) * DEC_T + threadIdx.x;
  const bool live = i < ncap && i < *n_dev;
  if (!CHECK && !live) return;
  int64_t good = 0;
  // the payload sample of this step (read before block 0 advances tick)
  const int64_t salt = CHECK && chk.tick != nullptr ? chk.tick[1] : 0;
  bool samp = false;                 // this reply's payload is compared
  int64_t s_off = 0, s_node = 0;
  int32_t s_len = 0;
  if (live) {
  const uint8_t* p = buf + foff[i];
  const int64_t L = flen[i];
  int32_t status = ST_OK;
  int32_t op = OP_UNKNOWN;
  int64_t poff = -1;
  int32_t plen = 0, a0 = 0, a1 = 0;
  int32_t xid = 0, err = 0;
  int64_t zxid = 0;
  // Every reply that carries a Stat ends with it (data + Stat, Stat,
  // children + Stat, ACL + Stat: zk-buffer.js:333-362), so the frame's last
  // 68 bytes are loaded together with the header instead of after the
  // opcode lookup and the data length; they are used when the body is
  // exactly "prefix + Stat" (else the Stat is read where the prefix ends).
  // (issued after the opcode lookup's load: vmcnt retires loads in order,
  // so the Stat loads then overlap that lookup instead of delaying it)
  uint32_t hw[4] = {0, 0, 0, 0};
  if (L >= 16) __builtin_memcpy(hw, p, 16);
  const bool tail_ok = L >= 16 + STAT_BYTES;
  uint32_t sw[STAT_BYTES / 4];
  if (L < 16) {
    status = ST_BAD_DECODE;
  } else {
    xid = (int32_t)bswap32(hw[0]);
    zxid = (int64_t)(((uint64_t)bswap32(hw[1]) << 32) | bswap32(hw[2]));
    err = (int32_t)bswap32(hw[3]);
    switch (xid) {
      case XID_NOTIFICATION: op = OP_NOTIFICATION; break;
      case XID_PING: op = OP_PING; break;
      case XID_AUTH: op = OP_AUTH; break;
      case XID_SET_WATCHES: op = OP_SET_WATCHES; break;
      default: {
        const int64_t e = xid_tab[xid & xid_mask];
        if (xid >= 0 && (int32_t)(e >> 32) == xid) op = (int32_t)e;
        else status = ST_NO_XID;
      }
    }
  }
  if (tail_ok) __builtin_memcpy(sw, p + L - STAT_BYTES, STAT_BYTES);
  if (status == ST_OK && err == ERR_OK) {
    const uint8_t* b = p + 16;
    const int64_t A = L - 16;
    switch (op) {
      case OP_GET_DATA: {
        if (A < 4) { status = ST_BAD_DECODE; break; }
        int32_t dl = ld_be32(b);
        if (dl < 0) dl = 0;
        if (4 + (int64_t)dl + STAT_BYTES > A) { status = ST_BAD_DECODE; break; }
        poff = foff[i] + 20;
        plen = dl;
        if (tail_ok && 4 + (int64_t)dl + STAT_BYTES == A) read_stat_regs(sw, o, i);
        else read_stat(b + 4 + dl, o, i);
        break;
      }
      case OP_EXISTS: case OP_SET_DATA:
        if (A < STAT_BYTES) { status = ST_BAD_DECODE; break; }
        if (tail_ok && A == STAT_BYTES) read_stat_regs(sw, o, i);
        else read_stat(b, o, i);
        break;
      case OP_CREATE: {
        if (A < 4) { status = ST_BAD_DECODE; break; }
        int32_t l = ld_be32(b);
        if (l < 0) l = 0;
        if (4 + (int64_t)l > A) { status = ST_BAD_DECODE; break; }
        poff = foff[i] + 20;
        plen = l;
        break;
      }
      case OP_GET_CHILDREN: case OP_GET_CHILDREN2: {
        if (A < 4) { status = ST_BAD_DECODE; break; }
        const int32_t cnt = max(ld_be32(b), 0);
        const int64_t k = skip_strings(b + 4, A - 4, cnt);
        if (k < 0) { status = ST_BAD_DECODE; break; }
        poff = foff[i] + 20;
        plen = (int32_t)k;
        a0 = cnt;
        if (op == OP_GET_CHILDREN2) {
          if (4 + k + STAT_BYTES > A) { status = ST_BAD_DECODE; break; }
          if (tail_ok && 4 + k + STAT_BYTES == A) read_stat_regs(sw, o, i);
          else read_stat(b + 4 + k, o, i);
        }
        break;
      }
      case OP_GET_ACL: {
        if (A < 4) { status = ST_BAD_DECODE; break; }
        const int32_t cnt = max(ld_be32(b), 0);
        const int64_t k = skip_acl(b + 4, A - 4, cnt);
        if (k < 0 || 4 + k + STAT_BYTES > A) { status = ST_BAD_DECODE; break; }
        poff = foff[i] + 20;
        plen = (int32_t)k;
        a0 = cnt;
        if (tail_ok && 4 + k + STAT_BYTES == A) read_stat_regs(sw, o, i);
        else read_stat(b + 4 + k, o, i);
        break;
      }
      case OP_NOTIFICATION: {
        if (A < 12) { status = ST_BAD_DECODE; break; }
        a0 = ld_be32(b);
        a1 = ld_be32(b + 4);
        int32_t l = ld_be32(b + 8);
        if (l < 0) l = 0;
        if (12 + (int64_t)l > A) { status = ST_BAD_DECODE; break; }
        poff = foff[i] + 28;
        plen = l;
        break;
      }
      case OP_PING: case OP_SYNC: case OP_DELETE: case OP_SET_WATCHES:
      case OP_CLOSE_SESSION: case OP_AUTH:
        break;
      default:
        status = ST_BAD_OPCODE;
    }
  }
  o.xid[i] = xid;
  o.err[i] = err;
  o.opcode[i] = op;
  o.zxid[i] = zxid;
  o.status[i] = status;
  o.pay_off[i] = poff;
  o.pay_len[i] = plen;
  o.aux0[i] = a0;
  o.aux1[i] = a1;
  if (CHECK && status == ST_OK && err == ERR_OK && op == OP_GET_DATA) {
    const int64_t v = chk.idx[i];
    good = xid == chk.xid[i] && o.stat64[i] == v + 1 &&
           plen == chk.data_len[v];
    samp = good && chk.slab != nullptr && plen > 0 &&
           ((i + salt) & (CHK_SAMPLE - 1)) == 0;
    s_off = poff;
    s_node = v;
    s_len = plen;
  }
  }  // live
  if (CHECK) {
    // the sampled payloads, one at a time by the whole wave
    uint64_t pend = __ballot(samp);
    const int lane = threadIdx.x & 63;
    while (pend) {
      const int l = (int)__builtin_ctzll(pend);
      pend &= pend - 1;
      const int64_t po = __shfl(s_off, l, 64);
      const int64_t vn = __shfl(s_node, l, 64);
      const int32_t pl = __shfl(s_len, l, 64);
      const bool eq = wave_bytes_equal(
          buf + po, chk.slab + chk.slot_off[vn] + ZK_SLOT_DATA, pl, lane);
      if (lane == l && !eq) good = 0;
    }
    if (chk.tick != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
      chk.tick[1] += 1;
    __shared__ int64_t sm[DEC_T / 64 + 1];
    int64_t tot;
    block_excl_scan(good, sm, &tot);
    if (threadIdx.x == 0 && tot)
      atomicAdd(&chk.acc[blockIdx.x % (uint32_t)chk.slots],
                (unsigned long long)tot);
  }
}

// Expand string vectors: region (offset of first string) + count per row ->
// (off,len) of every string, rows laid out by the scanned `base`.
__global__ __launch_bounds__(DEC_T) void expand_strings_k(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ region,
    const int32_t* __restrict__ count, const int64_t* __restrict__ base,
    int64_t n, int64_t* __restrict__ soff, int32_t* __restrict__ slen) {
  const int64_t i = (int64_t)blockIdx.x * DEC_T + threadIdx.x;
  if (i >= n) return;
  const int32_t c = count[i];
  if (c <= 0 || region[i] < 0) return;
  int64_t k = region[i];
  int64_t w = base[i];
  for (int32_t j = 0; j < c; ++j) {
    int32_t l = ld_be32(buf + k);
    if (l < 0) l = 0;
    soff[w + j] = k + 4;
    slen[w + j] = l;
    k += 4 + l;
  }
}

// Expand ACL vectors: perms, scheme (off,len), id (off,len) per entry.
__global__ __launch_bounds__(DEC_T) void expand_acl_k(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ region,
    const int32_t* __restrict__ count, const int64_t* __restrict__ base,
    int64_t n, int32_t* __restrict__ perms, int64_t* __restrict__ s_off,
    int32_t* __restrict__ s_len, int64_t* __restrict__ i_off,
    int32_t* __restrict__ i_len) {
  const int64_t i = (int64_t)blockIdx.x * DEC_T + threadIdx.x;
  if (i >= n) return;
  const int32_t c = count[i];
  if (c <= 0 || region[i] < 0) return;
  int64_t k = region[i];
  int64_t w = base[i];
  for (int32_t j = 0; j < c; ++j) {
    perms[w + j] = ld_be32(buf + k);
    k += 4;
    int32_t l = max(ld_be32(buf + k), 0);
    s_off[w + j] = k + 4;
    s_len[w + j] = l;
    k += 4 + l;
    l = max(ld_be32(buf + k), 0);
    i_off[w + j] = k + 4;
    i_len[w + j] = l;
    k += 4 + l;
  }
}

// ---------------------------------------------------------------- K12
__global__ __launch_bounds__(DEC_T) void decode_requests_k(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ foff,
    const int32_t* __restrict__ flen, const int64_t* __restrict__ n_dev,
    int64_t ncap, ZkReqOut o) {
  const uint32_t nwg = gridDim.x;
  const int64_t i = (int64_t)xcd_remap(blockIdx.x, nwg) * DEC_T + threadIdx.x;
  if (i >= ncap || i >= *n_dev) return;
  const ReqFields f = parse_request(buf, foff[i], flen[i]);
  o.xid[i] = f.xid;
  o.opcode[i] = f.op;
  o.status[i] = f.status;
  o.path_off[i] = f.poff;
  o.path_len[i] = f.pl;
  o.data_off[i] = f.doff;
  o.data_len[i] = f.dl;
  o.arg[i] = f.arg;
  o.vec_off[i] = f.voff;
  o.vec_count[i] = f.vc;
  o.rel_zxid[i] = f.rel;
}

// ---------------------------------------------------------------- K9
// ConnectResponse batch decode (zk-buffer.js:41-48): protocolVersion,
// timeOut, sessionId, passwd (offset/len into buf).  One row per session
// handshake — control plane, batched across a node's sessions.
__global__ __launch_bounds__(DEC_T) void decode_connect_k(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ foff,
    const int32_t* __restrict__ flen, int64_t n, int32_t* __restrict__ proto,
    int32_t* __restrict__ tmo, int64_t* __restrict__ sid,
    int64_t* __restrict__ pw_off, int32_t* __restrict__ pw_len,
    int32_t* __restrict__ status) {
  const int64_t i = (int64_t)blockIdx.x * DEC_T + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = buf + foff[i];
  const int64_t L = flen[i];
  int32_t st = ST_OK, pv = 0, to = 0, pl = 0;
  int64_t s = 0, po = -1;
  if (L < 20) {
    st = ST_BAD_DECODE;
  } else {
    pv = ld_be32(p);
    to = ld_be32(p + 4);
    s = ld_be64(p + 8);
    int32_t l = ld_be32(p + 16);
    if (l < 0) l = 0;
    if (20 + (int64_t)l > L) st = ST_BAD_DECODE;   // a trailing readOnly
    else { po = foff[i] + 20; pl = l; }            // byte is tolerated
  }
  proto[i] = pv; tmo[i] = to; sid[i] = s; pw_off[i] = po; pw_len[i] = pl;
  status[i] = st;
}

static inline unsigned nblk(int64_t n) {
  return (unsigned)((n + DEC_T - 1) / DEC_T);
}

}  // namespace zk

extern "C" {

int zk_decode_replies(const uint8_t* buf, const int64_t* foff,
                      const int32_t* flen, const int64_t* n_dev, int64_t ncap,
                      const int64_t* xid_tab, int64_t xid_mask,
                      const ZkReplyOut* o, hipStream_t st) {
  if (ncap <= 0) return 0;
  zk::decode_replies_k<false><<<zk::nblk(ncap), zk::DEC_T, 0, st>>>(
      buf, foff, flen, n_dev, ncap, xid_tab, xid_mask, *o,
      zk::ZkGetCheck{nullptr, nullptr, nullptr, nullptr, 1, nullptr, nullptr,
                     nullptr});
  ZK_LAUNCH_CHECK();
  return 0;
}

// zk_decode_replies + the fused GET_DATA check (ZkGetCheck): idx / xid are
// the requests sent (ncap of them), data_len the tree's per-node lengths,
// acc `slots` (1..64) int64 counters the caller sums; slab / slot_off
// (optional, both or neither): the tree's node slots, for the sampled
// payload comparison.
int zk_decode_replies_check2(const uint8_t* buf, const int64_t* foff,
                             const int32_t* flen, const int64_t* n_dev,
                             int64_t ncap, const int64_t* xid_tab,
                             int64_t xid_mask, const ZkReplyOut* o,
                             const int64_t* idx, const int32_t* xid,
                             const int32_t* data_len, unsigned long long* acc,
                             int32_t slots, int64_t* tick,
                             const uint8_t* slab, const int64_t* slot_off,
                             hipStream_t st) {
  if (ncap <= 0) return 0;
  if (slots < 1 || slots > 64) return (int)hipErrorInvalidValue;
  if ((slab == nullptr) != (slot_off == nullptr))
    return (int)hipErrorInvalidValue;
  zk::decode_replies_k<true><<<zk::nblk(ncap), zk::DEC_T, 0, st>>>(
      buf, foff, flen, n_dev, ncap, xid_tab, xid_mask, *o,
      zk::ZkGetCheck{idx, xid, data_len, acc, slots, tick, slab, slot_off});
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_expand_strings(const uint8_t* buf, const int64_t* region,
                      const int32_t* count, const int64_t* base, int64_t n,
                      int64_t* soff, int32_t* slen, hipStream_t st) {
  if (n <= 0) return 0;
  zk::expand_strings_k<<<zk::nblk(n), zk::DEC_T, 0, st>>>(buf, region, count,
                                                          base, n, soff, slen);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_expand_acl(const uint8_t* buf, const int64_t* region,
                  const int32_t* count, const int64_t* base, int64_t n,
                  int32_t* perms, int64_t* s_off, int32_t* s_len,
                  int64_t* i_off, int32_t* i_len, hipStream_t st) {
  if (n <= 0) return 0;
  zk::expand_acl_k<<<zk::nblk(n), zk::DEC_T, 0, st>>>(
      buf, region, count, base, n, perms, s_off, s_len, i_off, i_len);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_decode_connect_responses(const uint8_t* buf, const int64_t* foff,
                                const int32_t* flen, int64_t n,
                                int32_t* proto, int32_t* tmo, int64_t* sid,
                                int64_t* pw_off, int32_t* pw_len,
                                int32_t* status, hipStream_t st) {
  if (n <= 0) return 0;
  zk::decode_connect_k<<<zk::nblk(n), zk::DEC_T, 0, st>>>(
      buf, foff, flen, n, proto, tmo, sid, pw_off, pw_len, status);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_decode_requests(const uint8_t* buf, const int64_t* foff,
                       const int32_t* flen, const int64_t* n_dev,
                       int64_t ncap, const ZkReqOut* o, hipStream_t st) {
  if (ncap <= 0) return 0;
  zk::decode_requests_k<<<zk::nblk(ncap), zk::DEC_T, 0, st>>>(
      buf, foff, flen, n_dev, ncap, *o);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
