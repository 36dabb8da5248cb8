// Batched Jute encoders (client requests K10, SET_WATCHES K11, server replies
// K13).  Reference: lib/zk-buffer.js:97-273 (requests), jute-buffer.js:107-189
// (primitives, length prefix), zk-streams.js:121-148 (framing + xid map).
//
// Shape: one thread per record in three phases — framed size, device-wide
// exclusive scan (scan.hip), then write at the scanned offset.  Consecutive
// records are adjacent in the output, so a wave's stores cover a contiguous
// span that the L2 merges into full lines.  The write pass also records
// xid -> opcode in the connection's HBM table (the reply decoder needs it:
// replies are not self-describing, zk-buffer.js:288-291).
#include "zk_common.h"

#include <stdlib.h>


namespace zk {

constexpr int ENC_T = 256;

ZK_DEV int64_t req_body_size(const ZkReqBatch& b, int64_t i, bool* ok) {
  const int32_t op = b.opcode[i];
  const int64_t pl = b.path_len ? max(b.path_len[i], 0) : 0;
  *ok = true;
  switch (op) {
    case OP_GET_DATA: case OP_EXISTS: case OP_GET_CHILDREN:
    case OP_GET_CHILDREN2:
      return 8 + 4 + pl + 1;
    case OP_CREATE: {
      const int64_t dl = max(b.data_len[i], 0);
      const int64_t al = b.acl_len[b.acl_id[i]];
      return 8 + 4 + pl + 4 + dl + al + 4;
    }
    case OP_DELETE:
      return 8 + 4 + pl + 4;
    case OP_SET_DATA: {
      const int64_t dl = max(b.data_len[i], 0);
      return 8 + 4 + pl + 4 + dl + 4;
    }
    case OP_GET_ACL: case OP_SYNC:
      return 8 + 4 + pl;
    case OP_PING: case OP_CLOSE_SESSION:
      return 8;
    default:
      *ok = false;
      return 0;
  }
}

// Offsets are reduce-then-scan fused into the producer and the consumer:
// the sizes kernel also writes its block's sum and the write kernel sums
// the block sums before its own (sum_blocks) and adds a block scan of the
// sizes.  Two launches where a separate device-wide scan made five (and a
// one-workgroup scan of the block sums between them made three, until
// round 5; it is still used past FUSED_SCAN_BLOCKS).
// A malformed request is flagged per block (bbad, a plain store every
// launch) and req_write's block 0 folds the flags into err, so err needs no
// zeroing launch before the encode.
__global__ __launch_bounds__(ENC_T) void req_sizes(ZkReqBatch b, int64_t n,
                                                  int64_t* __restrict__ sizes,
                                                  int64_t* __restrict__ bbad,
                                                  int64_t* __restrict__ bsum) {
  __shared__ int64_t sm[ENC_T / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * ENC_T + threadIdx.x;
  int64_t sz = 0;
  bool bad = false;
  if (i < n) {
    bool ok;
    const int64_t s = req_body_size(b, i, &ok);
    sz = ok ? 4 + s : 0;
    sizes[i] = sz;
    bad = !ok;
  }
  int64_t tot;
  block_excl_scan(sz, sm, &tot);
  const int any = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    bsum[blockIdx.x] = tot;
    bbad[blockIdx.x] = any ? 1 : 0;
  }
}

// ---------------------------------------------------------------- K11
// SET_WATCHES: relZxid + three string vectors (data, exist, child), one
// frame.  Paths are given as (off,len) lists; kind[i] in {0,1,2}; the host
// passes them grouped by kind (counts c0,c1,c2) so the vector order is
// implicit.  Each thread writes one path at its scanned offset.
__global__ __launch_bounds__(ENC_T) void sw_sizes(const int32_t* __restrict__ plen,
                                                 int64_t n,
                                                 int64_t* __restrict__ sizes) {
  const int64_t i = (int64_t)blockIdx.x * ENC_T + threadIdx.x;
  if (i < n) sizes[i] = 4 + max(plen[i], 0);
}

__global__ __launch_bounds__(ENC_T) void sw_write(
    const int64_t* __restrict__ poff, const int32_t* __restrict__ plen,
    const uint8_t* __restrict__ arena, int64_t n, int64_t c0, int64_t c1,
    const int64_t* __restrict__ off, const int64_t* __restrict__ total,
    int64_t rel_zxid, uint8_t* __restrict__ out, int64_t cap,
    int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * ENC_T + threadIdx.x;
  const int64_t strings = *total;
  // layout: len | xid | op | relZxid | c0 | v0.. | c1 | v1.. | c2 | v2..
  const int64_t frame = 4 + 8 + 8 + 12 + strings;
  if (frame > cap) {
    if (i == 0) atomicOr(err, 2);
    return;
  }
  if (i == 0) {
    st_be32(out, (int32_t)(frame - 4));
    st_be32(out + 4, XID_SET_WATCHES);
    st_be32(out + 8, OP_SET_WATCHES);
    st_be64(out + 12, rel_zxid);
  }
  const int64_t c2 = n - c0 - c1;
  // vector-count words sit before each group
  if (i == 0) {
    int64_t s1 = (c0 > 0) ? off[c0 - 1] + 4 + max(plen[c0 - 1], 0) : 0;
    int64_t s2 = (c1 > 0) ? off[c0 + c1 - 1] + 4 + max(plen[c0 + c1 - 1], 0)
                          : s1;
    st_be32(out + 20, (int32_t)c0);
    st_be32(out + 24 + s1, (int32_t)c1);
    st_be32(out + 28 + s2, (int32_t)c2);
  }
  if (i >= n) return;
  const int64_t g = (i < c0) ? 0 : (i < c0 + c1 ? 1 : 2);
  uint8_t* o = out + 24 + 4 * g + off[i];
  put_buffer(o, arena + poff[i], plen[i]);
}

// ---------------------------------------------------------------- K13
// Server-mode reply encode (absent from the reference, zk-streams.js:140).
ZK_DEV int64_t resp_body_size(const ZkRespBatch& r, const ZkNodeStore& s,
                              int64_t i) {
  int64_t sz = 16;                              // xid, zxid, err
  if (r.err[i] != ERR_OK) return sz;
  switch (r.opcode[i]) {
    case OP_GET_DATA: {
      const int64_t nd = r.node[i];
      return sz + 4 + max(s.data_len[nd], 0) + STAT_BYTES;
    }
    case OP_EXISTS: case OP_SET_DATA:
      return sz + STAT_BYTES;
    case OP_CREATE:
      return sz + 4 + max(r.path_len[i], 0);
    case OP_NOTIFICATION:
      return sz + 8 + 4 + max(r.path_len[i], 0);
    default:
      return sz;                                // header-only replies
  }
}

__global__ __launch_bounds__(ENC_T) void resp_sizes(ZkRespBatch r,
                                                   ZkNodeStore s,
                                                   const int64_t* __restrict__ n_dev,
                                                   int64_t ncap,
                                                   int64_t* __restrict__ sizes,
                                                   int64_t* __restrict__ bsum) {
  __shared__ int64_t sm[ENC_T / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * ENC_T + threadIdx.x;
  int64_t sz = 0;
  if (i < ncap) {
    sz = (i < *n_dev) ? 4 + resp_body_size(r, s, i) : 0;
    sizes[i] = sz;
  }
  int64_t tot;
  block_excl_scan(sz, sm, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// ---- record sinks ----------------------------------------------------------
// The same record-emission code writes either straight to global memory
// (GSink: one thread's stores are scattered across the wave -> poorly
// coalesced) or into an LDS image of the block's contiguous output span
// (LSink) that the block then streams out with 16-byte coalesced stores.
// LSink packs bytes into aligned dwords; only a record's first and last
// dword can be shared with a neighbour, and those are OR-ed into the
// zero-initialised image (ds_or_b32), everything else is a plain ds_write.
//
// The image is bank-swizzled: dword w lives at swz(w) = w ^ ((w >> 4) & 31),
// a permutation inside each aligned 32-dword group.  Lanes emit their
// records in lockstep, so their k-th dwords sit one record apart; ds_write_b32
// banks are (dword mod 32) over 32-lane groups, and at 192-byte records (48
// dwords) an unswizzled image put 16 lanes on a bank.  Any swizzle that
// keeps aligned 4-dword groups together (rounds 1-4: bits 2-5 XORed with the
// 64-dword row, 2.49 M conflict cycles a 512K-reply dispatch) leaves lanes
// writing dword k of 4-aligned records on 8 banks, 4-way; this one moves
// bits 0-1 too (conflict-free at 48 dwords; 2-3 way for odd record sizes),
// so the read-out assembles each 16-byte vector from four dword reads
// (~2.4-way on those reads, against 4-way on every record write before).
// SW = 1: the rounds 1-4 swizzle (bits 2-5 XOR the 64-dword row: 4-dword
// groups stay whole, the read-out moves 16-byte vectors; 4-way on the
// record writes), kept for A/B (ZKMI_ENC_SWZ=1).
template <int SW>
ZK_DEV int64_t swz(int64_t w) {
  if (SW == 1) return w ^ (((w >> 6) & 15) << 2);
  return w ^ ((w >> 4) & 31);
}
struct GSink {
  uint8_t* o;
  ZK_DEV void be32(int32_t v) { st_be32(o, v); o += 4; }
  ZK_DEV void be64(int64_t v) { st_be64(o, v); o += 8; }
  ZK_DEV void u8(uint32_t b) { *o++ = (uint8_t)b; }
  ZK_DEV void bytes(const uint8_t* s, int64_t n) { copy_bytes(o, s, n); o += n; }
  ZK_DEV void put4(uint32_t x) { __builtin_memcpy(o, &x, 4); o += 4; }
  ZK_DEV void finish() {}
};

template <int SW>
struct LSink {
  uint32_t* w;
  int64_t widx;
  uint64_t acc;
  int nb;
  bool first;
  ZK_DEV LSink(uint32_t* lds, int64_t rel) : w(lds), widx(rel >> 2), acc(0),
                                             nb((int)(rel & 3)), first(true) {}
  ZK_DEV void flush() {
    const uint32_t v = (uint32_t)acc;
    if (first) { atomicOr(&w[swz<SW>(widx)], v); first = false; }
    else w[swz<SW>(widx)] = v;
    ++widx;
    acc >>= 32;
    nb -= 4;
  }
  ZK_DEV void put4(uint32_t x) {          // 4 bytes in memory order
    acc |= (uint64_t)x << (8 * nb);
    nb += 4;
    flush();
  }
  ZK_DEV void u8(uint32_t b) {
    acc |= (uint64_t)(b & 0xffu) << (8 * nb);
    if (++nb == 4) flush();
  }
  ZK_DEV void be32(int32_t v) { put4(bswap32((uint32_t)v)); }
  ZK_DEV void be64(int64_t v) {
    put4(bswap32((uint32_t)((uint64_t)v >> 32)));
    put4(bswap32((uint32_t)v));
  }
  ZK_DEV void bytes(const uint8_t* s, int64_t n) {
    int64_t i = 0;
    // 128-byte batches: eight 16-byte loads in flight before the first
    // LDS write (one round trip per 128 bytes instead of per 16 — large
    // payloads, e.g. KiB GET_DATA replies, were latency-bound here)
    for (; i + 128 <= n; i += 128) {
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) __builtin_memcpy(&v[j], s + i + 16 * j, 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        put4(v[j].x); put4(v[j].y); put4(v[j].z); put4(v[j].w);
      }
    }
    for (; i + 16 <= n; i += 16) {
      uint4 v; __builtin_memcpy(&v, s + i, 16);
      put4(v.x); put4(v.y); put4(v.z); put4(v.w);
    }
    for (; i + 4 <= n; i += 4) {
      uint32_t v; __builtin_memcpy(&v, s + i, 4);
      put4(v);
    }
    for (; i < n; ++i) u8(s[i]);
  }
  ZK_DEV void finish() {
    if (nb > 0) atomicOr(&w[swz<SW>(widx)], (uint32_t)acc);
  }
};

template <class K>
ZK_DEV void k_buffer(K& k, const uint8_t* src, int32_t len) {
  if (len <= 0) { k.be32(-1); return; }
  k.be32(len);
  k.bytes(src, len);
}

// dword k of a register array of 16-byte vectors (k constant after
// unrolling, so the array stays in VGPRs)
ZK_DEV uint32_t vword(const uint4* v, int k) {
  const uint4& q = v[k >> 2];
  switch (k & 3) {
    case 0: return q.x;
    case 1: return q.y;
    case 2: return q.z;
    default: return q.w;
  }
}

// GET_DATA replies with up to this much data are emitted from registers.
constexpr int GET_REG_DATA = 128;

// hole > 0 (a large GET_DATA reply, see staged_emit_holes): the [len | data]
// bytes [pre, pre + hole) are left out; the waves copy them slot -> out.
template <class K>
ZK_DEV void emit_response(K& k, const ZkRespBatch& r, const ZkNodeStore& s,
                          int64_t i, int64_t body, int64_t pre = 0,
                          int64_t hole = 0) {
  const int32_t xid = r.xid[i], err = r.err[i], op = r.opcode[i];
  const int64_t zxid = r.zxid[i];
  const int64_t nd = body - 16 - STAT_BYTES;          // GET: 4 + data length
  if (hole > 0) {
    const uint8_t* slot = s.slab + (r.slot ? r.slot[i]
                                           : s.slot_off[r.node[i]]);
    k.be32((int32_t)body);
    k.be32(xid);
    k.be64(zxid);
    k.be32(err);
    k.bytes(slot + ZK_SLOT_LEN, pre);
    k.bytes(slot + ZK_SLOT_LEN + pre + hole, nd - pre - hole);
    k.bytes(slot + ZK_SLOT_STAT, STAT_BYTES);
    k.finish();
    return;
  }
  if (err == ERR_OK && op == OP_GET_DATA && nd <= 4 + GET_REG_DATA) {
    // Fast path: every load of the record is issued before the first
    // sink write (the generic copy below waits on each 16-byte load in
    // turn, ~11 dependent round trips per reply).  Whole 16-byte vectors
    // from the slot start to the end of the data stay inside the slot:
    // slot_bytes rounds the data capacity up to 16 and adds 4.
    constexpr int NV = (ZK_SLOT_DATA + GET_REG_DATA + 15) / 16;
    constexpr int W0 = ZK_SLOT_LEN / 4;               // [len | data] dword
    const uint8_t* slot = s.slab + (r.slot ? r.slot[i]
                                           : s.slot_off[r.node[i]]);
    const int nv = (int)((ZK_SLOT_LEN + nd + 15) >> 4);
    uint4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j)
      v[j] = j < nv ? *(const uint4*)(slot + 16 * j) : make_uint4(0, 0, 0, 0);
    k.be32((int32_t)body);
    k.be32(xid);
    k.be64(zxid);
    k.be32(err);
    const int wfull = (int)(nd >> 2), tb = (int)(nd & 3);
#pragma unroll
    for (int w = 0; w < NV * 4 - W0; ++w) {
      if (w < wfull) {
        k.put4(vword(v, W0 + w));
      } else if (w == wfull && tb) {
        const uint32_t x = vword(v, W0 + w);
        for (int b = 0; b < tb; ++b) k.u8(x >> (8 * b));
      }
    }
#pragma unroll
    for (int w = 0; w < STAT_BYTES / 4; ++w) k.put4(vword(v, w));
    k.finish();
    return;
  }
  k.be32((int32_t)body);
  k.be32(xid);
  k.be64(zxid);
  k.be32(err);
  if (err == ERR_OK) {
    switch (op) {
      case OP_GET_DATA: {
        // wire-format slot: [len | data] then Stat — two contiguous copies.
        // The data length is implied by the frame size (header 16, length
        // word 4, Stat 68), so only the slot itself is read.
        const uint8_t* slot = s.slab + (r.slot ? r.slot[i]
                                               : s.slot_off[r.node[i]]);
        k.bytes(slot + ZK_SLOT_LEN, nd);
        k.bytes(slot + ZK_SLOT_STAT, STAT_BYTES);
        break;
      }
      case OP_EXISTS: case OP_SET_DATA:
        k.bytes(s.slab + (r.slot ? r.slot[i] : s.slot_off[r.node[i]]) +
                    ZK_SLOT_STAT, STAT_BYTES);
        break;
      case OP_CREATE:
        k_buffer(k, r.path_arena + r.path_off[i], r.path_len[i]);
        break;
      case OP_NOTIFICATION:
        k.be32(r.aux[i]);
        k.be32(3 /* SYNC_CONNECTED */);
        k_buffer(k, r.path_arena + r.path_off[i], r.path_len[i]);
        break;
      default:
        break;
    }
  }
  k.finish();
}

// LDS image per block; with the block's offset table (EncLocal, 4 KiB) a
// block holds 32 KiB, 5 blocks per CU.
constexpr int64_t STAGE_BYTES = 28 * 1024;

// The block's record offsets and sizes (index k = record r0 + k).
struct EncLocal {
  int64_t off[ENC_T];
  int64_t sz[ENC_T];
  int64_t sm[ENC_T / 64 + 1];
};

// off = base + block scan of sizes; also written to rec_off.
ZK_DEV void block_offsets(int64_t r0, int64_t r1,
                          const int64_t* __restrict__ sizes, int64_t base,
                          int64_t* __restrict__ rec_off, EncLocal& E) {
  const int64_t i = r0 + threadIdx.x;
  const int64_t sz = i < r1 ? sizes[i] : 0;
  int64_t tot;
  const int64_t o = base + block_excl_scan(sz, E.sm, &tot);
  E.off[threadIdx.x] = o;
  E.sz[threadIdx.x] = sz;
  if (i < r1 && rec_off != nullptr) rec_off[i] = o;
  __syncthreads();
}

// The write pass's block base without a scan launch: the sizes pass wrote
// every block's sum (bsum, complete: an earlier launch), so block b sums
// bsum[0, b) itself — four independent L2 loads a thread per 1024 blocks,
// one round trip at the usual batch sizes.  Past FUSED_SCAN_BLOCKS the sum
// grows with the grid (quadratic traffic) and the host scans bsum first
// (zk_scan_small_i64 -> bbase).  Also the grand total, for the block that
// needs it (the last one: it writes *total, err and the terminator).
constexpr int64_t FUSED_SCAN_BLOCKS = 4096;

ZK_DEV int64_t sum_blocks(const int64_t* __restrict__ bsum, int64_t b,
                          int64_t* sm) {
  int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  int64_t k = threadIdx.x;
  for (; k + 3 * ENC_T < b; k += 4 * ENC_T) {
    a0 += bsum[k];
    a1 += bsum[k + ENC_T];
    a2 += bsum[k + 2 * ENC_T];
    a3 += bsum[k + 3 * ENC_T];
  }
  for (; k < b; k += ENC_T) a0 += bsum[k];
  int64_t tot;
  block_excl_scan(a0 + a1 + a2 + a3, sm, &tot);
  return tot;
}

// This block's base (bbase, or fused: sum_blocks) and, in the last block,
// the stream total (fused: computed and stored; else read).
ZK_DEV int64_t block_base(const int64_t* __restrict__ bbase,
                          const int64_t* __restrict__ bsum,
                          int64_t* __restrict__ total, int64_t* sm,
                          int64_t* T) {
  const int64_t b = blockIdx.x;
  if (bsum == nullptr) {
    *T = *total;
    return bbase[b];
  }
  const int64_t base = sum_blocks(bsum, b, sm);
  *T = -1;                              // (known in the last block only)
  if (b == (int64_t)gridDim.x - 1) {
    *T = base + bsum[b];
    if (threadIdx.x == 0) *total = *T;
  }
  return base;
}

template <int SW>
ZK_DEV uint8_t lds_byte(const uint32_t* lw, int64_t b) {
  return ((const uint8_t*)(lw + swz<SW>(b >> 2)))[b & 3];
}

// 16 image bytes at image byte y (16-aligned): four dword reads (the
// swizzle scatters a 4-dword group over banks), one 16-byte vector.
template <int SW>
ZK_DEV uint4 lds_vec(const uint32_t* lw, int64_t y) {
  const int64_t w = y >> 2;
  if (SW == 1) return *(const uint4*)(lw + swz<SW>(w));
  return make_uint4(lw[swz<SW>(w)], lw[swz<SW>(w + 1)], lw[swz<SW>(w + 2)],
                    lw[swz<SW>(w + 3)]);
}

// Stream the block's LDS image [B0, B1) (image base a0 = B0 & ~15) out to
// global memory: the 16-byte aligned interior with dwordx4 stores (a dword
// a lane — four times the store instructions — cost the GET step 4 %), the
// <= 15 head / tail bytes with byte stores (they abut other blocks' spans).
template <int SW>
ZK_DEV void stage_out(const uint32_t* lw, int64_t a0, int64_t B0, int64_t B1,
                      uint8_t* __restrict__ out) {
  const int64_t c0 = (B0 + 15) & ~(int64_t)15;
  const int64_t c1 = B1 & ~(int64_t)15;
  if (c0 < c1) {
    for (int64_t x = c0 + (int64_t)threadIdx.x * 16; x < c1;
         x += (int64_t)blockDim.x * 16)
      *(uint4*)(out + x) = lds_vec<SW>(lw, x - a0);
    const int64_t hb = c0 - B0, tb = B1 - c1;
    if ((int64_t)threadIdx.x < hb) {
      const int64_t x = B0 + threadIdx.x;
      out[x] = lds_byte<SW>(lw, x - a0);
    } else if ((int64_t)threadIdx.x >= 16 && (int64_t)threadIdx.x < 16 + tb) {
      const int64_t x = c1 + threadIdx.x - 16;
      out[x] = lds_byte<SW>(lw, x - a0);
    }
  } else {
    for (int64_t x = B0 + threadIdx.x; x < B1; x += blockDim.x)
      out[x] = lds_byte<SW>(lw, x - a0);
  }
}

// Emit records [r0, r1) (one per thread, <= blockDim) through the block's
// LDS image.  Records are staged in runs that fit the image (record i ends
// at off[i] + sizes[i]; ends grow with i, so "fits" is a prefix of the
// run, counted with one barrier); a single record larger than the image is
// written straight to global memory.  off / sizes are the block's EncLocal
// tables (index i - r0).
template <int SW, class F>
ZK_DEV void staged_emit(int64_t r0, int64_t r1, const int64_t* off,
                        const int64_t* sizes, uint8_t* __restrict__ out,
                        uint32_t* lw, F emit, int64_t stage = STAGE_BYTES) {
  int64_t rs = r0;
  while (rs < r1) {                              // block-uniform
    const int64_t B0 = off[rs - r0];
    const int64_t a0 = B0 & ~(int64_t)15;
    const int64_t i = rs + threadIdx.x;
    const bool fits = i < r1 &&
                      off[i - r0] + sizes[i - r0] - a0 + 16 <= stage;
    const int k = __syncthreads_count(fits);
    if (k == 0) {
      if (threadIdx.x == 0) {
        GSink g{out + B0};
        emit(g, rs);
      }
      rs += 1;
      continue;
    }
    const int64_t re = rs + k;
    const int64_t B1 = off[re - 1 - r0] + sizes[re - 1 - r0];
    const int64_t nrow = ((B1 - a0 + 3) >> 8) + 1;     // 64-dword rows
    for (int64_t x = threadIdx.x; x < nrow * 16; x += blockDim.x)
      ((uint4*)lw)[x] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (i < re) {
      LSink<SW> l(lw, off[i - r0] - a0);
      emit(l, i);
    }
    __syncthreads();
    stage_out<SW>(lw, a0, B0, B1, out);
    __syncthreads();                             // image reused next run
    rs = re;
  }
}

// Terminated streams: four 0xFF bytes (frame length -1, BAD_LENGTH) right
// after the stream when they fit.  A frame scan run over a host-known upper
// bound of the stream length then stops exactly at the stream end, so the
// pipeline needs no device-to-host read of the length before scanning.
ZK_DEV void put_terminator(bool term, int64_t T, uint8_t* out, int64_t cap) {
  if (!term || T < 0 || threadIdx.x != 0) return;
  if (T + 4 <= cap) st_be32(out + T, -1);
}

// ---- K13: large GET_DATA replies --------------------------------------------
// A reply's [len | data] bytes sit at out [q0, q0 + nd), q0 = off + 20.  When
// their 16-byte aligned interior [h0, h1) holds at least BIG_HOLE bytes it
// is a HOLE: left out of the block's LDS image and copied slot -> out by the
// waves, one reply per wave-iteration (64 lanes x 16 bytes, stores
// coalesced), instead of by the reply's own lane one dword at a time (one
// lane per record left a wave as slow as its longest record and a 28 KiB
// image held ~46 replies of ~600 B, so most of a block's lanes idled).  The
// image keeps the rest of every record — headers, the data's unaligned head
// and tail, Stats — in COMPACTED coordinates (out offset minus the holes
// before it; holes are multiples of 16, so 16-byte vectors stay aligned),
// and a run is streamed out segment by segment between its holes.
constexpr int64_t BIG_HOLE = 256;

struct EncHoles {
  int64_t hb[ENC_T];        // (holes before record k, block-exclusive) << 9
                            // | big records before it
  int32_t hole[ENC_T];      // record k's hole bytes (0: none)
  int16_t bl[ENC_T];        // the block's big records in order (-1: written
                            // whole, not a hole)
};

ZK_DEV int64_t hole_h0(int64_t off) { return (off + 20 + 15) & ~(int64_t)15; }

// Stream a run's compacted image out: segment k (0..K) runs between the
// holes of the run's big records k-1 and k (j0: the run's first big record
// in the block's list); image position y of segment k is out position
// y + a0c + (hole bytes before it).  One thread per segment; the run's first
// and last 16-byte chunks are shared with other runs / blocks (byte stores).
template <int SW>
ZK_DEV void stage_out_segs(const uint32_t* lw, int64_t a0c, int64_t B0,
                           int64_t B1, int64_t yend, int64_t hb0, int64_t K,
                           int64_t j0, const int64_t* off, const EncHoles& H,
                           uint8_t* __restrict__ out) {
  for (int64_t k = threadIdx.x; k <= K; k += blockDim.x) {
    int64_t y0, y1, d;
    if (k == 0) {
      y0 = B0 - (a0c + hb0);
      d = hb0;
    } else {
      const int li = H.bl[j0 + k - 1];
      const int64_t hc = H.hb[li] >> 9;
      y0 = hole_h0(off[li]) - hc - a0c;
      d = hc + H.hole[li];
    }
    if (k == K) {
      y1 = yend;
    } else {
      const int li = H.bl[j0 + k];
      y1 = hole_h0(off[li]) - (H.hb[li] >> 9) - a0c;
    }
    for (int64_t y = y0 & ~(int64_t)15; y < y1; y += 16) {
      const int64_t x = y + a0c + d;
      const uint4 v = lds_vec<SW>(lw, y);
      if (x >= B0 && x + 16 <= B1) {
        *(uint4*)(out + x) = v;
      } else {
        const uint8_t* b = (const uint8_t*)&v;
        for (int q = 0; q < 16; ++q)
          if (x + q >= B0 && x + q < B1) out[x + q] = b[q];
      }
    }
  }
}

// One hole, slot -> out, by a 16-lane quarter of a wave: 16 bytes a lane per
// chunk, four chunks (1 KiB a quarter) loaded before any is stored (one
// dependent round trip per hole, not per chunk).  The source is read as
// dwords and realigned (alignbyte) to the 16-byte aligned destination; its
// last dword may reach 3 bytes past the data: inside the slot (its data
// capacity is rounded up to 16, plus 4).
ZK_DEV void copy_hole_q(const uint8_t* __restrict__ src, uint8_t* dst,
                        int64_t n, int ql) {
  constexpr int U = 4;
  const int sh = (int)((uintptr_t)src & 3);
  const uint32_t* sa = (const uint32_t*)((uintptr_t)src & ~(uintptr_t)3);
  for (int64_t x0 = (int64_t)ql * 16; x0 < n; x0 += 16 * 16 * U) {
    uint32_t w[U][5];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t x = x0 + 16 * 16 * u;
      if (x < n) {
        const uint32_t* p = sa + (x >> 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) w[u][k] = p[k];
        w[u][4] = sh ? p[4] : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t x = x0 + 16 * 16 * u;
      if (x < n) {
        uint4 v;
        v.x = __builtin_amdgcn_alignbyte(w[u][1], w[u][0], sh);
        v.y = __builtin_amdgcn_alignbyte(w[u][2], w[u][1], sh);
        v.z = __builtin_amdgcn_alignbyte(w[u][3], w[u][2], sh);
        v.w = __builtin_amdgcn_alignbyte(w[u][4], w[u][3], sh);
        *(uint4*)(dst + x) = v;
      }
    }
  }
}

// staged_emit for replies with holes.  off / sizes: the block's EncLocal
// tables; H: the holes (set up by resp_write).
template <int SW, class F>
ZK_DEV void staged_emit_holes(int64_t r0, int64_t r1, const int64_t* off,
                              const int64_t* sizes, EncHoles& H,
                              uint8_t* __restrict__ out, uint32_t* lw, F emit,
                              int64_t stage) {
  int64_t rs = r0;
  while (rs < r1) {                              // block-uniform
    const int64_t ls = rs - r0;
    const int64_t B0 = off[ls];
    const int64_t hb0 = H.hb[ls] >> 9;
    const int64_t a0c = (B0 & ~(int64_t)15) - hb0;   // compacted image base
    const int64_t i = rs + threadIdx.x;
    const int64_t li = i - r0;
    const bool fits = i < r1 && off[li] - (H.hb[li] >> 9) + sizes[li] -
                                        H.hole[li] - a0c + 16 <= stage;
    const int k = __syncthreads_count(fits);
    if (k == 0) {
      // one record larger than the image, compacted: written whole
      if (threadIdx.x == 0) {
        GSink g{out + B0};
        emit(g, rs, 0, 0);
        if (H.hole[ls]) H.bl[H.hb[ls] & 511] = -1;
      }
      rs += 1;
      continue;
    }
    const int64_t re = rs + k;
    const int64_t le = re - 1 - r0;
    const int64_t B1 = off[le] + sizes[le];
    const int64_t hbe = (H.hb[le] >> 9) + H.hole[le];    // holes to run end
    const int64_t yend = B1 - hbe - a0c;
    const int64_t nrow = ((yend + 3) >> 8) + 1;         // 64-dword rows
    for (int64_t x = threadIdx.x; x < nrow * 16; x += blockDim.x)
      ((uint4*)lw)[x] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (i < re) {
      LSink<SW> l(lw, off[li] - (H.hb[li] >> 9) - a0c);
      const int64_t hl = H.hole[li];
      emit(l, i, hl ? hole_h0(off[li]) - (off[li] + 20) : 0, hl);
    }
    __syncthreads();
    const int64_t j0 = H.hb[ls] & 511;
    const int64_t K = ((H.hb[le] & 511) + (H.hole[le] ? 1 : 0)) - j0;
    if (K == 0) {
      stage_out<SW>(lw, B0 & ~(int64_t)15, B0, B1, out);
    } else {
      stage_out_segs<SW>(lw, a0c, B0, B1, yend, hb0, K, j0, off, H, out);
    }
    __syncthreads();                             // image reused next run
    rs = re;
  }
}

// Uniform GET_DATA replies (every record of the block a successful
// GET_DATA of the same size S, S a multiple of 16, the block's span
// 16-byte aligned — a read batch of equal-sized znodes): the block's span
// is written straight from the slots, 16 bytes a lane per piece, every
// store of a wave 1 KiB contiguous, no LDS image.  A record is
//   [0,4) S - 4 | [4,8) xid | [8,16) zxid | [16,20) err |
//   [20, S - 68) the slot's [len | data] | [S - 68, S) the slot's Stat,
// and S % 16 == 0 makes the data length a multiple of 4, so every dword of
// a 16-byte piece is one aligned dword of the slot (or of the header).
// The records' header words and slot offsets are staged in LDS once per
// block (coalesced loads); a piece's record is c / P by a float reciprocal
// (P = S / 16 pieces a record) — the first version divided 64-bit integers
// and loaded the header fields per piece, and ran the GET step at 0.96 ms
// against the LDS image's 0.65.
ZK_DEV void emit_uniform(const ZkRespBatch& r, const ZkNodeStore& s,
                         int64_t r0, int64_t nrec, int64_t S, int64_t B0,
                         uint8_t* __restrict__ out, uint32_t* lw) {
  uint32_t* hx = lw;                                // [nrec][5] header words
  int64_t* hs = (int64_t*)(lw + 5 * ENC_T);         // [nrec] slot offsets
  if ((int64_t)threadIdx.x < nrec) {
    const int64_t i = r0 + threadIdx.x;
    const uint64_t z = (uint64_t)r.zxid[i];
    uint32_t* h = hx + 5 * threadIdx.x;
    h[0] = bswap32((uint32_t)(S - 4));
    h[1] = bswap32((uint32_t)r.xid[i]);
    h[2] = bswap32((uint32_t)(z >> 32));
    h[3] = bswap32((uint32_t)z);
    h[4] = bswap32((uint32_t)r.err[i]);
    hs[threadIdx.x] = r.slot ? r.slot[i] : s.slot_off[r.node[i]];
  }
  __syncthreads();
  const uint32_t P = (uint32_t)(S >> 4);
  const uint32_t split = (uint32_t)(S - STAT_BYTES);   // 24 + data length
  const uint32_t pieces = (uint32_t)nrec * P;
  const float invP = 1.0f / (float)P;
  constexpr int U = 4;                   // pieces in flight per lane
  for (uint32_t c0 = threadIdx.x; c0 < pieces; c0 += U * ENC_T) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = c0 + (uint32_t)u * ENC_T;
      if (c >= pieces) continue;
      uint32_t k = (uint32_t)((float)c * invP);
      if (k * P > c) --k;
      else if ((k + 1) * P <= c) ++k;
      const uint32_t p0 = (c - k * P) << 4;          // the piece's record byte
      const uint8_t* slot = s.slab + hs[k];
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t p = p0 + 4 * q;
        w[q] = p < 20 ? hx[5 * k + (p >> 2)]
                      : *(const uint32_t*)(slot + (p < split
                                                       ? p + (ZK_SLOT_LEN - 20)
                                                       : p - split));
      }
      v[u] = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = c0 + (uint32_t)u * ENC_T;
      if (c < pieces) *(uint4*)(out + B0 + ((int64_t)c << 4)) = v[u];
    }
  }
}

// bsum != null: fused (block_base); every block checks its own span
// against cap, the last one writes *total and err (2: over capacity, the
// stream is then incomplete).
template <int SW>
__global__ __launch_bounds__(ENC_T) void resp_write(
    ZkRespBatch r, ZkNodeStore s, const int64_t* __restrict__ n_dev,
    int64_t ncap, const int64_t* __restrict__ sizes,
    const int64_t* __restrict__ bbase, const int64_t* __restrict__ bsum,
    int64_t* __restrict__ rec_off, int64_t* __restrict__ total,
    uint8_t* __restrict__ out, int64_t cap, int32_t* __restrict__ err,
    int32_t term, int64_t stage, int32_t uniform) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lw[];
  __shared__ EncLocal E;
  const int64_t n = min(*n_dev, ncap);
  const int64_t r0 = (int64_t)blockIdx.x * ENC_T;
  int64_t T;
  const int64_t base = block_base(bbase, bsum, total, E.sm, &T);
  const bool last = blockIdx.x == gridDim.x - 1;
  if (bsum != nullptr ? last : blockIdx.x == 0) {
    put_terminator(term, T, out, cap);
    // err written whole by one thread (no zeroing launch before the encode)
    if (threadIdx.x == 0) *err = T > cap ? 2 : 0;
  }
  if (r0 >= n) return;
  if (T > cap) return;
  const int64_t r1 = min(r0 + ENC_T, n);
  if (bsum != nullptr && base + bsum[blockIdx.x] > cap) return;
  block_offsets(r0, r1, sizes, base, rec_off, E);
  // uniform GET_DATA replies: straight from the slots (emit_uniform)
  if (uniform) {                                  // (a kernel argument)
    const int64_t i = r0 + threadIdx.x;
    const int64_t S = E.sz[0];
    const bool u = i >= r1 ||
                   (r.opcode[i] == OP_GET_DATA && r.err[i] == ERR_OK &&
                    E.sz[threadIdx.x] == S);
    if (__syncthreads_and(u) && (S & 15) == 0 && (E.off[0] & 15) == 0 &&
        S >= 96 && stage >= 5 * 4 * ENC_T + 8 * ENC_T) {
      emit_uniform(r, s, r0, r1 - r0, S, E.off[0], out, lw);
      return;
    }
  }
  // the holes (large GET_DATA replies), their block scan and list
  __shared__ EncHoles H;
  {
    const int64_t i = r0 + threadIdx.x;
    int64_t hole = 0;
    if (i < r1 && r.opcode[i] == OP_GET_DATA && r.err[i] == ERR_OK) {
      const int64_t o = E.off[threadIdx.x];
      const int64_t nd = E.sz[threadIdx.x] - 4 - 16 - STAT_BYTES;
      const int64_t h0 = hole_h0(o);
      const int64_t h1 = (o + 20 + nd) & ~(int64_t)15;
      if (h1 - h0 >= BIG_HOLE) hole = h1 - h0;
    }
    int64_t tot;
    const int64_t hb = block_excl_scan(hole * 512 + (hole ? 1 : 0), E.sm,
                                       &tot);
    H.hb[threadIdx.x] = hb;
    H.hole[threadIdx.x] = (int32_t)hole;
    if (hole) H.bl[hb & 511] = (int16_t)threadIdx.x;
    __syncthreads();
  }
  staged_emit_holes<SW>(r0, r1, E.off, E.sz, H, out, lw,
                    [&](auto& k, int64_t i, int64_t pre, int64_t hole) {
    emit_response(k, r, s, i, E.sz[i - r0] - 4, pre, hole);
  }, stage);
  __syncthreads();                 // (bl: records written whole)
  // the holes: four replies per wave-iteration, one per 16-lane quarter,
  // each quarter's loads all issued before its stores
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t lt = r1 - 1 - r0;
  const int64_t nb = (H.hb[lt] & 511) + (H.hole[lt] ? 1 : 0);
  for (int64_t j0 = 4 * wv; j0 < nb; j0 += 4 * (ENC_T / 64)) {
    const int64_t j = j0 + (lane >> 4);
    const int li = j < nb ? H.bl[j] : -1;          // -1: written whole
    const uint8_t* src = nullptr;
    uint8_t* dst = nullptr;
    int64_t hn = 0;
    if (li >= 0) {
      const int64_t i = r0 + li;
      const uint8_t* slot = s.slab + (r.slot ? r.slot[i]
                                             : s.slot_off[r.node[i]]);
      const int64_t o = E.off[li];
      const int64_t h0 = hole_h0(o);
      src = slot + ZK_SLOT_LEN + (h0 - (o + 20));
      dst = out + h0;
      hn = H.hole[li];
    }
    copy_hole_q(src, dst, hn, lane & 15);
  }
}

// ---------------------------------------------------------------- K10 write
constexpr int REQ_REG_PATH = 64;   // read-request paths emitted from registers

template <class K>
ZK_DEV void emit_request(K& k, const ZkReqBatch& b, int64_t i, int64_t body) {
  const int32_t op = b.opcode[i];
  const int32_t xid = b.xid[i];
  if ((op == OP_GET_DATA || op == OP_EXISTS || op == OP_GET_CHILDREN ||
       op == OP_GET_CHILDREN2) && b.path_len[i] > 0 &&
      b.path_len[i] <= REQ_REG_PATH) {
    // Fast path for the read requests: the path (<= 64 bytes) is loaded as
    // unaligned dwords inside its own bytes, all before the first sink
    // write, instead of one dependent round trip per 16-byte piece.
    const int32_t pl = b.path_len[i];
    const uint8_t* src = b.path_arena + b.path_off[i];
    const int32_t watch = b.arg[i];
    uint32_t w[REQ_REG_PATH / 4];
#pragma unroll
    for (int j = 0; j < REQ_REG_PATH / 4; ++j) {
      w[j] = 0;
      if (4 * j + 4 <= pl) __builtin_memcpy(&w[j], src + 4 * j, 4);
    }
    uint32_t tail = 0;
    const int32_t nw = pl >> 2, tb = pl & 3;
    for (int q = 0; q < tb; ++q) tail |= (uint32_t)src[4 * nw + q] << (8 * q);
    k.be32((int32_t)body);
    k.be32(xid);
    k.be32(op);
    k.be32(pl);
#pragma unroll
    for (int j = 0; j < REQ_REG_PATH / 4; ++j)
      if (j < nw) k.put4(w[j]);
    for (int q = 0; q < tb; ++q) k.u8(tail >> (8 * q));
    k.u8(watch ? 1 : 0);
    k.finish();
    return;
  }
  k.be32((int32_t)body);
  k.be32(xid);
  k.be32(op);
  if (op == OP_PING || op == OP_CLOSE_SESSION) {
    k.finish();
    return;
  }
  k_buffer(k, b.path_arena + b.path_off[i], b.path_len[i]);
  switch (op) {
    case OP_GET_DATA: case OP_EXISTS: case OP_GET_CHILDREN:
    case OP_GET_CHILDREN2:
      k.u8(b.arg[i] ? 1 : 0);
      break;
    case OP_CREATE: {
      k_buffer(k, b.data_arena + b.data_off[i], b.data_len[i]);
      const int32_t a = b.acl_id[i];
      k.bytes(b.acl_arena + b.acl_off[a], b.acl_len[a]);
      k.be32(b.arg[i]);
      break;
    }
    case OP_DELETE:
      k.be32(b.arg[i]);
      break;
    case OP_SET_DATA:
      k_buffer(k, b.data_arena + b.data_off[i], b.data_len[i]);
      k.be32(b.arg[i]);
      break;
    default:
      break;
  }
  k.finish();
}

// Records are staged through the block's LDS image and streamed out with
// 16-byte stores (a thread's own scattered 4-byte / byte stores wrote ~7x
// the frame bytes as partial-line writes: WRITE_SIZE 254 MB for a 36 MB
// GET_DATA stream).  Unknown opcodes were flagged by req_sizes and get
// size 0 (nothing written).
template <int SW>
__global__ __launch_bounds__(ENC_T) void req_write(
    ZkReqBatch b, int64_t n, const int64_t* __restrict__ sizes,
    const int64_t* __restrict__ bbase, const int64_t* __restrict__ bsum,
    int64_t* __restrict__ rec_off, int64_t* __restrict__ total,
    uint8_t* __restrict__ out, int64_t cap, int64_t* __restrict__ xid_tab,
    int64_t xid_mask, int32_t* __restrict__ err, int32_t term,
    const int64_t* __restrict__ bbad, int64_t nb) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lw[];
  __shared__ EncLocal E;
  const int64_t r0 = (int64_t)blockIdx.x * ENC_T;
  int64_t T;
  const int64_t base = block_base(bbase, bsum, total, E.sm, &T);
  if (bsum != nullptr ? blockIdx.x == gridDim.x - 1 : blockIdx.x == 0) {
    put_terminator(term, T, out, cap);
    // err, written whole (1: a malformed request, 2: over capacity)
    int64_t e = 0;
    for (int64_t k = threadIdx.x; k < nb; k += ENC_T) e |= bbad[k];
    const int any = __syncthreads_or(e != 0);
    if (threadIdx.x == 0) *err = (any ? 1 : 0) | (T > cap ? 2 : 0);
  }
  if (r0 >= n) return;
  if (T > cap) return;                      // capacity guard (whole batch)
  const int64_t r1 = min(r0 + ENC_T, n);
  // fused: each block's own span (the last block flags the batch)
  if (bsum != nullptr && base + bsum[blockIdx.x] > cap) return;
  block_offsets(r0, r1, sizes, base, rec_off, E);
  staged_emit<SW>(r0, r1, E.off, E.sz, out, lw, [&](auto& k, int64_t i) {
    const int64_t sz = E.sz[i - r0];
    if (sz > 0) emit_request(k, b, i, sz - 4);
  });
  const int64_t i = r0 + threadIdx.x;
  if (i < r1 && xid_tab != nullptr && sizes[i] > 0) {
    const int32_t xid = b.xid[i];
    if (xid >= 0)
      xid_tab[xid & xid_mask] = ((int64_t)xid << 32) | (uint32_t)b.opcode[i];
  }
}

// ---------------------------------------------------------------- K9
// ConnectRequest batch encode (zk-buffer.js:32-39): one handshake record
// per session (node-wide session (re)attach after a failover, R3).
__global__ __launch_bounds__(ENC_T) void cr_sizes(const int32_t* __restrict__ pwl,
                                                 int64_t n,
                                                 int64_t* __restrict__ sizes) {
  const int64_t i = (int64_t)blockIdx.x * ENC_T + threadIdx.x;
  if (i < n) sizes[i] = 4 + 28 + max(pwl[i], 0);   // frame + body
}

__global__ __launch_bounds__(ENC_T) void cr_write(
    const int32_t* __restrict__ proto, const int64_t* __restrict__ zxid,
    const int32_t* __restrict__ tmo, const int64_t* __restrict__ sid,
    const int64_t* __restrict__ pwo, const int32_t* __restrict__ pwl,
    const uint8_t* __restrict__ arena, int64_t n,
    const int64_t* __restrict__ off, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * ENC_T + threadIdx.x;
  if (i >= n) return;
  GSink g{out + off[i]};
  g.be32(28 + max(pwl[i], 0));   // 4+8+4+8 fixed + 4-byte passwd length
  g.be32(proto[i]);
  g.be64(zxid[i]);
  g.be32(tmo[i]);
  g.be64(sid[i]);
  k_buffer(g, arena + pwo[i], pwl[i]);
}

static inline unsigned nblk(int64_t n) {
  return (unsigned)((n + ENC_T - 1) / ENC_T);
}

// A/B switches, read once (profiles/r5_encoder_ab.md, GET step, 2 x 50
// steps each): the image swizzle — 1 (default) keeps 4-dword groups whole
// (4-way conflicts on the record writes, 16-byte read-out), 0 scatters
// them (conflict-free writes, four dword reads per 16-byte vector): 0
// removes the conflict cycles and costs the step 0.5 %, the dword reads
// cost more LDS issue than the conflicts did; the block sums — a one-
// workgroup scan launch (default) or every write block summing the sums
// before its own (ZKMI_ENC_FUSED=1: one launch less, but 1.3 % slower: each
// block's sum is a round trip before its first store).
static int enc_swz() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("ZKMI_ENC_SWZ"); v = e ? atoi(e) : 1; }
  return v;
}
// Uniform GET_DATA reply blocks written straight from the slots
// (emit_uniform; ZKMI_ENC_UNIFORM=0 sends them through the LDS image).
// Its first version ran the GET step at 0.958 ms against the image's 0.651
// (a 64-bit division and per-record loads per 16-byte piece); reworked,
// 0.575 against 0.615 (profiles/r5_uniform_writer_ab.md).
static int enc_uniform() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("ZKMI_ENC_UNIFORM"); v = e ? atoi(e) : 1; }
  return v;
}
static bool enc_fused() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("ZKMI_ENC_FUSED"); v = e ? atoi(e) : 0; }
  return v != 0;
}

}  // namespace zk

extern "C" {

// terminate != 0: four 0xFF bytes follow the stream (put_terminator).
int zk_encode_requests2(const ZkReqBatch* b, int64_t n, int64_t* sizes,
                        int64_t* rec_off, int64_t* total, int64_t* scan_ws,
                        uint8_t* out, int64_t out_cap, int64_t* xid_tab,
                        int64_t xid_mask, int32_t* err, int32_t terminate,
                        hipStream_t st) {
  if (n <= 0) {
    int rc = hipMemsetAsync(total, 0, 8, st);
    if (!rc) rc = hipMemsetAsync(err, 0, 4, st);
    if (!rc && terminate && out_cap >= 4) rc = hipMemsetAsync(out, 0xFF, 4, st);
    return rc;
  }
  const unsigned nb = zk::nblk(n);
  int64_t* bsum = scan_ws;                 // zk_scan_workspace(n) >= 3 nb
  int64_t* bbase = scan_ws + nb;
  int64_t* bbad = scan_ws + 2 * nb;
  zk::req_sizes<<<nb, zk::ENC_T, 0, st>>>(*b, n, sizes, bbad, bsum);
  ZK_LAUNCH_CHECK();
  const bool fused = nb <= zk::FUSED_SCAN_BLOCKS && zk::enc_fused();
  if (!fused) {
    int rc = zk_scan_small_i64(bsum, bbase, nb, total, st);
    if (rc) return rc;
  }
  if (zk::enc_swz() == 1)
    zk::req_write<1><<<nb, zk::ENC_T, zk::STAGE_BYTES, st>>>(
        *b, n, sizes, bbase, fused ? bsum : nullptr, rec_off, total, out,
        out_cap, xid_tab, xid_mask, err, terminate, bbad, (int64_t)nb);
  else
    zk::req_write<0><<<nb, zk::ENC_T, zk::STAGE_BYTES, st>>>(
        *b, n, sizes, bbase, fused ? bsum : nullptr, rec_off, total, out,
        out_cap, xid_tab, xid_mask, err, terminate, bbad, (int64_t)nb);
  ZK_LAUNCH_CHECK();
  return 0;
}

// zk_encode_requests2 with the sizes pass done by the producer of the batch
// (bench_gen_get): `sizes` (frame bytes per request) and `bsum` (their sum
// per 256-request block) are given, every request well-formed.  Two
// launches: the block sums' scan, the write.
int zk_encode_requests_presized(const ZkReqBatch* b, int64_t n,
                                const int64_t* sizes, const int64_t* bsum,
                                int64_t* rec_off, int64_t* total,
                                int64_t* scan_ws, uint8_t* out,
                                int64_t out_cap, int64_t* xid_tab,
                                int64_t xid_mask, int32_t* err,
                                int32_t terminate, hipStream_t st) {
  if (n <= 0)
    return zk_encode_requests2(b, n, nullptr, rec_off, total, scan_ws, out,
                               out_cap, xid_tab, xid_mask, err, terminate,
                               st);
  const unsigned nb = zk::nblk(n);
  int64_t* bbase = scan_ws + nb;
  int rc = zk_scan_small_i64(bsum, bbase, nb, total, st);
  if (rc) return rc;
  if (zk::enc_swz() == 1)
    zk::req_write<1><<<nb, zk::ENC_T, zk::STAGE_BYTES, st>>>(
        *b, n, sizes, bbase, nullptr, rec_off, total, out, out_cap, xid_tab,
        xid_mask, err, terminate, nullptr, 0);
  else
    zk::req_write<0><<<nb, zk::ENC_T, zk::STAGE_BYTES, st>>>(
        *b, n, sizes, bbase, nullptr, rec_off, total, out, out_cap, xid_tab,
        xid_mask, err, terminate, nullptr, 0);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_encode_requests(const ZkReqBatch* b, int64_t n, int64_t* sizes,
                       int64_t* rec_off, int64_t* total, int64_t* scan_ws,
                       uint8_t* out, int64_t out_cap, int64_t* xid_tab,
                       int64_t xid_mask, int32_t* err, hipStream_t st) {
  return zk_encode_requests2(b, n, sizes, rec_off, total, scan_ws, out,
                             out_cap, xid_tab, xid_mask, err, 0, st);
}

// Returns the frame length through *frame_len (device int64): 4 + body.
int zk_encode_set_watches(const int64_t* poff, const int32_t* plen,
                          const uint8_t* arena, int64_t n, int64_t c0,
                          int64_t c1, int64_t rel_zxid, int64_t* sizes,
                          int64_t* off, int64_t* total, int64_t* scan_ws,
                          uint8_t* out, int64_t out_cap, int32_t* err,
                          hipStream_t st) {
  if (n > 0) {
    zk::sw_sizes<<<zk::nblk(n), zk::ENC_T, 0, st>>>(plen, n, sizes);
    ZK_LAUNCH_CHECK();
    int rc = zk_scan_excl_i64(sizes, off, n, total, scan_ws, st);
    if (rc) return rc;
  } else {
    hipMemsetAsync(total, 0, 8, st);
  }
  zk::sw_write<<<zk::nblk(n > 0 ? n : 1), zk::ENC_T, 0, st>>>(
      poff, plen, arena, n, c0, c1, off, total, rel_zxid, out, out_cap, err);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_encode_connect_requests(const int32_t* proto, const int64_t* zxid,
                               const int32_t* tmo, const int64_t* sid,
                               const int64_t* pwo, const int32_t* pwl,
                               const uint8_t* arena, int64_t n, int64_t* sizes,
                               int64_t* off, int64_t* total, int64_t* scan_ws,
                               uint8_t* out, hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(total, 0, 8, st);
  zk::cr_sizes<<<zk::nblk(n), zk::ENC_T, 0, st>>>(pwl, n, sizes);
  ZK_LAUNCH_CHECK();
  int rc = zk_scan_excl_i64(sizes, off, n, total, scan_ws, st);
  if (rc) return rc;
  zk::cr_write<<<zk::nblk(n), zk::ENC_T, 0, st>>>(proto, zxid, tmo, sid, pwo,
                                                  pwl, arena, n, off, out);
  ZK_LAUNCH_CHECK();
  return 0;
}

// presized != 0: `sizes` (frame size per reply, 0 past *n_dev) and the
// per-256-reply block sums in scan_ws[0, nblk(ncap)) were already written
// by the producer (zk_tree_serve), so the sizes pass is skipped.
// stage (bytes, 0: STAGE_BYTES): the LDS each workgroup gets — the image of
// its replies, or the uniform writer's header table (7 KiB).  A caller whose
// replies are uniform GET_DATA blocks (the GET pipeline) asks for little, so
// more workgroups (and another stream's kernels) fit a CU.
int zk_encode_responses3(const ZkRespBatch* r, const ZkNodeStore* s,
                         const int64_t* n_dev, int64_t ncap, int64_t* sizes,
                         int64_t* rec_off, int64_t* total, int64_t* scan_ws,
                         uint8_t* out, int64_t out_cap, int32_t* err,
                         int32_t presized, int32_t terminate, int64_t stage,
                         hipStream_t st);

int zk_encode_responses2(const ZkRespBatch* r, const ZkNodeStore* s,
                         const int64_t* n_dev, int64_t ncap, int64_t* sizes,
                         int64_t* rec_off, int64_t* total, int64_t* scan_ws,
                         uint8_t* out, int64_t out_cap, int32_t* err,
                         int32_t presized, int32_t terminate, hipStream_t st) {
  return zk_encode_responses3(r, s, n_dev, ncap, sizes, rec_off, total,
                              scan_ws, out, out_cap, err, presized, terminate,
                              0, st);
}

int zk_encode_responses3(const ZkRespBatch* r, const ZkNodeStore* s,
                         const int64_t* n_dev, int64_t ncap, int64_t* sizes,
                         int64_t* rec_off, int64_t* total, int64_t* scan_ws,
                         uint8_t* out, int64_t out_cap, int32_t* err,
                         int32_t presized, int32_t terminate, int64_t stage_req,
                         hipStream_t st) {
  if (ncap <= 0) {
    int rc = hipMemsetAsync(total, 0, 8, st);
    if (!rc) rc = hipMemsetAsync(err, 0, 4, st);
    if (!rc && terminate && out_cap >= 4) rc = hipMemsetAsync(out, 0xFF, 4, st);
    return rc;
  }
  const unsigned nb = zk::nblk(ncap);
  int64_t* bsum = scan_ws;
  int64_t* bbase = scan_ws + nb;
  if (!presized) {
    zk::resp_sizes<<<nb, zk::ENC_T, 0, st>>>(*r, *s, n_dev, ncap, sizes,
                                             bsum);
    ZK_LAUNCH_CHECK();
  }
  // presized == 2: the block bases and *total are already in place
  // (zk_tree_finish_scan scanned the serve's block sums)
  const bool fused = presized != 2 && nb <= zk::FUSED_SCAN_BLOCKS &&
                     zk::enc_fused();
  if (!fused && presized != 2) {
    int rc = zk_scan_small_i64(bsum, bbase, nb, total, st);
    if (rc) return rc;
  }
  // reply image per workgroup (a 56 KiB image gained 0.5 % on 0-1024 B
  // payloads and cost GET 2 %)
  // (at least the uniform writer's header table and a few records' image)
  const int64_t stage = stage_req <= 0 ? zk::STAGE_BYTES
                        : stage_req < 8192 ? 8192
                        : stage_req > zk::STAGE_BYTES ? zk::STAGE_BYTES
                                                      : (stage_req + 15) & ~15;
  if (zk::enc_swz() == 1)
    zk::resp_write<1><<<nb, zk::ENC_T, (size_t)stage, st>>>(
        *r, *s, n_dev, ncap, sizes, bbase, fused ? bsum : nullptr, rec_off,
        total, out, out_cap, err, terminate, stage, zk::enc_uniform());
  else
    zk::resp_write<0><<<nb, zk::ENC_T, (size_t)stage, st>>>(
        *r, *s, n_dev, ncap, sizes, bbase, fused ? bsum : nullptr, rec_off,
        total, out, out_cap, err, terminate, stage, zk::enc_uniform());
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_encode_responses(const ZkRespBatch* r, const ZkNodeStore* s,
                        const int64_t* n_dev, int64_t ncap, int64_t* sizes,
                        int64_t* rec_off, int64_t* total, int64_t* scan_ws,
                        uint8_t* out, int64_t out_cap, int32_t* err,
                        hipStream_t st) {
  return zk_encode_responses2(r, s, n_dev, ncap, sizes, rec_off, total,
                              scan_ws, out, out_cap, err, 0, 0, st);
}

}  // extern "C"
