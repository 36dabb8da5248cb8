// GPU-resident synthetic ZooKeeper tree (the server side of the 1M-znode
// benchmark, the create/set/delete mix and the ephemeral create storm).  Not
// part of the reference — it stands in for the JVM server the reference's
// tests talk to, so that the whole request -> reply path runs at HBM speed.
//
// Layout (HBM, sized by the caller for 288 GB parts):
//   * open-addressing hash table of 64-byte entries {key, val, path head,
//     data length} (one line per probe): key = word-wise multiply-xorshift
//     hash of the path | 1, val = node and slot + 1 (-2 = tombstone, 0 =
//     empty or being published), linear probing, pow2 capacity;
//   * node slots in wire format (zk_batch.h ZkNodeStore), so replies are
//     contiguous copies;
//   * a path arena holding each node's path for exact-match verification;
//   * counters (TC_*): node high-water mark, zxid, path-arena top, slab top,
//     the free-node ring (head / tail / published tail) and the dirty count;
//   * a free-node ring: DELETE (and session expiry) push the node index,
//     CREATE pops one published by an EARLIER launch (tree_publish_k runs
//     between batches), reusing its slot and path storage when they fit;
//   * host-endian shadows of each node's cversion / numChildren (one packed
//     word, cn_*) and pzxid.
//     Children come and go with plain atomicAdd / atomicMax on these (a
//     big-endian Stat word would need a CAS retry loop, and ~1000 parents
//     shared by a million writes contend); every parent touched in a launch
//     is put on a dirty list once, and tree_fixup_k rewrites the wire-format
//     Stat words of exactly those parents before replies are encoded.
//
// Single-address counters (free ring, node bump, dirty list) are claimed
// once per BLOCK (ballot/mbcnt ranks + an LDS prefix, one atomic), the rare
// byte claims of the arena bump allocators once per wave (64-lane shuffle
// scan); zxids need no atomic at all (base + request index).  For that the
// serve and expire kernels keep every thread alive to the end (out-of-range
// threads carry a no-op).
//
// Requests are applied concurrently within a batch, except that requests
// on ONE path are applied in batch (xid) order when any of them writes:
// tree_order_* rank every request by the number of earlier same-path
// requests of the batch and the serve kernel runs in passes of equal rank
// (ZooKeeper applies a session's requests in order; requests on different
// paths commute).  Version CAS is an atomicCAS on the slot's big-endian
// version word, so exactly one of several same-version SET_DATAs wins (the
// others get BAD_VERSION), matching ZooKeeper's conditional set.  Every
// write request is assigned a zxid, failed ones included (ZooKeeper logs an
// error txn for them).
#include "zk_common.h"
#include "zk_mfma_scan.h"
#include "zk_reqparse.h"

namespace zk {

constexpr int TR_T = 256;
enum : int {
  TC_NODES = 0, TC_ZXID = 1, TC_PATH_TOP = 2, TC_SLAB_TOP = 3,
  TC_FREE_HEAD = 4, TC_FREE_TAIL = 5, TC_FREE_PUB = 6, TC_DIRTY = 7,
  TC_SESS = 8, TC_N = 9
};
// `session` argument value meaning "the session in counters[TC_SESS]": a
// captured step whose session changes from replay to replay (the storm's
// born / resumed / expired sessions) keeps it on the device
constexpr int64_t SESS_DEV = -2;
ZK_DEV int64_t sess_of(const ZkTree& t, int64_t session) {
  return session == SESS_DEV ? t.counters[TC_SESS] : session;
}
constexpr int64_t NODE_FREE = -2;

// ordered serve: rank byte = min(rank, ORD_RANK) | ORD_SNAP
constexpr int32_t ORD_RANK = 0x7f, ORD_SNAP = 0x80;

ZK_DEV int64_t slot_bytes(int32_t data_cap) {
  return ZK_SLOT_DATA + (((int64_t)data_cap + 15) & ~(int64_t)15) + 4;
}

// ---- aggregated claims (all threads of the block must be active) ---------
ZK_DEV int lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0));
}

// One ticket per thread with `want`: returns base + rank, or -1.  Ranks come
// from ballot/mbcnt within a wave and an LDS prefix over the block's waves;
// ONE atomic per block of NT threads (a single word sustains only ~88
// returning atomics/us, MI355X_MICROARCH.md "dequeue").  Every thread of the
// block must call it.
template <int NT = TR_T>
ZK_DEV int64_t block_ticket(int64_t* ctr, bool want,
                            unsigned long long* also = nullptr) {
  constexpr int TR_T = NT;
  __shared__ int64_t part[TR_T / 64 + 1];
  const int w = threadIdx.x >> 6;
  const uint64_t m = __ballot(want);
  const int rank = __builtin_amdgcn_mbcnt_hi(
      (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  if (lane_id() == 0) part[w] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t tot = 0;
    for (int k = 0; k < TR_T / 64; ++k) {
      const int64_t c = part[k];
      part[k] = tot;
      tot += c;
    }
    part[TR_T / 64] = tot ? (int64_t)atomicAdd((unsigned long long*)ctr,
                                               (unsigned long long)tot)
                          : 0;
    // (a second count of the same threads: its result unused, no wait)
    if (also != nullptr && tot) atomicAdd(also, (unsigned long long)tot);
  }
  __syncthreads();
  const int64_t r = want ? part[TR_T / 64] + part[w] + rank : -1;
  __syncthreads();                                 // part[] reusable
  return r;
}

// Claim `amount` (>= 0) bytes per lane; returns this lane's offset or -1.
ZK_DEV int64_t wave_bytes(int64_t* ctr, int64_t amount) {
  const int lane = lane_id();
  int64_t incl = amount;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  const int64_t tot = __shfl(incl, 63, 64);
  if (tot == 0) return -1;
  int64_t base = 0;
  if (lane == 63)
    base = (int64_t)atomicAdd((unsigned long long*)ctr,
                              (unsigned long long)tot);
  base = __shfl(base, 63, 64);
  return amount > 0 ? base + incl - amount : -1;
}

// ---- hash index -----------------------------------------------------------
// Path hash: 8 bytes per step (unaligned loads), a multiply-xorshift per
// word and a final avalanche — 4 multiplies for a 25-byte path where a
// byte-serial FNV-1a needs 25.
ZK_DEV uint64_t path_hash(const uint8_t* p, int32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  int32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w; __builtin_memcpy(&w, p + i, 8);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  if (i < n) {
    uint64_t w = 0;
    for (int32_t k = 0; i + k < n; ++k) w |= (uint64_t)p[i + k] << (8 * k);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return h;
}

ZK_DEV bool bytes_eq(const uint8_t* a, const uint8_t* b, int32_t n) {
  int32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x, y; __builtin_memcpy(&x, a + i, 8); __builtin_memcpy(&y, b + i, 8);
    if (x != y) return false;
  }
  for (; i < n; ++i) if (a[i] != b[i]) return false;
  return true;
}

// One 64-byte entry per slot (a cache line; open addressing, linear
// probing): int64 words [0] key = path hash | 1 (0 empty), [1] val (node |
// slot offset, below; -2 tombstone, 0 empty or being published), [2] path
// length | data length << 32, [3, 8) the path's first EN_PATH bytes.  A
// lookup loads the entry in one burst and verifies the path and gets a GET
// reply's data length from it: ONE random line per lookup (rounds 2-4 read
// the 16-byte {key, val} entry and then the node's 64-byte lookup line, a
// second dependent random read).  Longer paths compare their tail in the
// arena.  (The per-node 64-byte lookup lines of round 4 are gone.)
constexpr int HT_W = 8;                    // int64 words per entry
constexpr int EN_PATH = 40;                // path bytes held in the entry

ZK_DEV int64_t* ht_ent(const ZkTree& t, int64_t s) { return &t.ht[HT_W * s]; }
ZK_DEV int64_t* ht_key(const ZkTree& t, int64_t s) { return &t.ht[HT_W * s]; }
ZK_DEV int64_t* ht_val(const ZkTree& t, int64_t s) { return &t.ht[HT_W * s + 1]; }

// Node v's path as one word (offset << 24 | length; paths < 16 MiB like
// the frames that carry them): the arena tail of a long path.
ZK_DEV int64_t pw_pack(int64_t off, int32_t len) {
  return (off << 24) | (int64_t)(uint32_t)len;
}

// The entry's path / data length words (everything but key and val); plain
// stores before the val is published.
ZK_DEV void ent_fill(const ZkTree& t, int64_t s, const uint8_t* p, int32_t n,
                     int32_t dl) {
  int64_t* e = ht_ent(t, s);
  e[2] = (int64_t)(uint32_t)n | ((int64_t)dl << 32);
  uint8_t* pb = (uint8_t*)&e[3];
  const int32_t h = n < EN_PATH ? n : EN_PATH;
  copy_bytes(pb, p, h);
}

ZK_DEV void ent_set_dlen(const ZkTree& t, int64_t s, int32_t dl) {
  __builtin_memcpy((uint8_t*)ht_ent(t, s) + 20, &dl, 4);
}

// 8 bytes of p at o (up to n: a shorter tail is zero-filled)
ZK_DEV uint64_t path_word(const uint8_t* p, int32_t o, int32_t n) {
  uint64_t w = 0;
  if (o + 8 <= n) {
    __builtin_memcpy(&w, p + o, 8);
  } else {
    for (int32_t k = 0; o + k < n; ++k) w |= (uint64_t)p[o + k] << (8 * k);
  }
  return w;
}

// Does entry e (its words loaded) name path p[0, n) of node v?
ZK_DEV bool ent_is(const ZkTree& t, const int64_t (&e)[HT_W], int64_t v,
                   const uint8_t* p, int32_t n) {
  if ((int32_t)(uint32_t)e[2] != n) return false;
  const int32_t h = n < EN_PATH ? n : EN_PATH;
#pragma unroll
  for (int w = 0; w < EN_PATH / 8; ++w) {
    if (8 * w >= h) break;
    uint64_t x = (uint64_t)e[3 + w];
    const int32_t left = h - 8 * w;
    if (left < 8) x &= (1ull << (8 * left)) - 1;   // (copy_bytes left the
                                                   // rest of the word as is)
    if (x != path_word(p, 8 * w, h)) return false;
  }
  if (n <= EN_PATH) return true;
  const int64_t pw = t.node_pw[v];
  return bytes_eq(t.path_arena + (pw >> 24) + EN_PATH, p + EN_PATH,
                  n - EN_PATH);
}

ZK_DEV void ent_load(const ZkTree& t, int64_t s, int64_t (&e)[HT_W]) {
  const uint4* q = (const uint4*)ht_ent(t, s);
#pragma unroll
  for (int k = 0; k < HT_W / 2; ++k) {
    const uint4 v = q[k];
    e[2 * k] = (int64_t)((uint64_t)v.x | (uint64_t)v.y << 32);
    e[2 * k + 1] = (int64_t)((uint64_t)v.z | (uint64_t)v.w << 32);
  }
}

// A hash val holds the node index (low 32 bits) and its slot offset / 16
// (high 32; slots are 16-byte aligned), plus one, so a hit needs no
// slot_off[v] read.  Live vals are > 0, the tombstone is -2, and 0 is an
// empty or being-published entry: an empty table is all zero bytes (a
// plain memset resets it; the -3 "empty" of before took a strided second
// pass).
ZK_DEV int64_t val_pack(int64_t v, int64_t slot) {
  return ((int64_t)(((uint64_t)slot >> 4) << 32) | v) + 1;
}
ZK_DEV int64_t val_node(int64_t x) { return (x - 1) & 0xFFFFFFFFll; }
// Order this thread's earlier global accesses before its later ones
// without a cache writeback or invalidate: a workgroup-scope fence is a
// wait for the outstanding accesses (the agent-scope atomics around it are
// served at L2, where the order then holds for other CUs too).  An
// agent-scope release / acquire writes back / invalidates caches, ~us each
// (MI355X_MICROARCH.md): in round 6's first expiry with them, 3.9 ms.
ZK_DEV void order_wait() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
}

// Tombstones: any val <= -2.  -2 is the plain one (DELETE, an insert's
// claim); a session expiry tags its own with its txn's zxid (ht_shift
// tells the holes of the launch it runs in from older tombstones).
// -1: an entry being moved (ht_shift).
constexpr int64_t VAL_TOMB = -2;
constexpr int64_t VAL_MOVING = -1;
ZK_DEV bool val_tomb(int64_t x) { return x <= VAL_TOMB; }
ZK_DEV int64_t tomb_tag(int64_t zx) {
  return VAL_TOMB - 1 - (zx & 0x3FFFFFFFFFFFll);
}
ZK_DEV int64_t val_slot(int64_t x) {
  return (int64_t)((uint64_t)(x - 1) >> 32) << 4;
}

// Node of path p (node -1 if absent), its slot offset and data length, and
// the hash entry (for a SET_DATA's data length update).
struct Found {
  int64_t node, slot;
  int32_t dlen;
  int64_t ent;
};

template <bool DLEN = false>
ZK_DEV Found tree_lookup(const ZkTree& t, const uint8_t* p, int32_t n) {
  (void)DLEN;
  const int64_t key = (int64_t)(path_hash(p, n) | 1ull);
  int64_t s = key & t.mask;
  for (int64_t probe = 0; probe <= t.mask; ++probe) {
    // one 64-byte entry per probe, loaded in one burst; entries being
    // written concurrently in this launch may read torn (val 0): not
    // found, as the batch contract allows for same-batch conflicts on one
    // path
    int64_t e[HT_W];
    ent_load(t, s, e);
    if (e[0] == 0) break;
    if (e[0] == key && e[1] > 0) {
      const int64_t node = val_node(e[1]);
      if (ent_is(t, e, node, p, n))
        return Found{node, val_slot(e[1]), (int32_t)(e[2] >> 32), s};
    }
    s = (s + 1) & t.mask;
  }
  return Found{-1, -1, 0, -1};
}

ZK_DEV int64_t tree_find(const ZkTree& t, const uint8_t* p, int32_t n) {
  return tree_lookup(t, p, n).node;
}

// Insert node `v` (path already in the arena).  Returns the existing node if
// the path is present (NODE_EXISTS), else v; TREE_INSERT_TIMEOUT when a
// concurrent claimer of the same key never published its value (the caller
// answers SYSTEMERROR rather than probing on and indexing the path twice).
constexpr int64_t TREE_INSERT_TIMEOUT = -4;
// REUSE: the caller knows no other request of the launch inserts this path
// (a SEQUENTIAL name numbered by zk_tree_seq_order: unique in its batch and
// above every number its parent gave before).  The probe still walks to the
// first empty slot (an existing node of that name answers NODE_EXISTS), but
// then the first tombstone passed on the way — of any key — is taken
// instead: entries of dead names are recycled by the next batch's names.
template <bool REUSE = false>
ZK_DEV int64_t tree_insert(const ZkTree& t, int64_t v, const uint8_t* p,
                           int32_t n, int32_t dl, int64_t so = -1) {
  const int64_t key = (int64_t)(path_hash(p, n) | 1ull);
  const int64_t pv = val_pack(v, so >= 0 ? so : t.store.slot_off[v]);
  int64_t s = key & t.mask;
  int64_t tomb = -1, tv = 0;
  for (int64_t probe = 0; probe <= t.mask; ++probe) {
    int64_t k0 = -1;                   // REUSE: the key loaded below
    if (REUSE) {
      // key and val in one round trip (the val only matters as a
      // tombstone to take, and the CAS on it decides)
      int64_t k = __hip_atomic_load(ht_key(t, s), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
      const int64_t vv = __hip_atomic_load(ht_val(t, s), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (k != 0 && k != key) {
        if (tomb < 0 && val_tomb(vv)) {
          tomb = s;
          tv = vv;
        }
        s = (s + 1) & t.mask;
        continue;
      }
      k0 = k;
      if (k == 0 && tomb >= 0) {
        // the name is absent: take the tombstone (val -2 -> 0 claims it;
        // a lookup in between sees a key with val 0 and probes on)
        if (atomicCAS((unsigned long long*)ht_val(t, tomb),
                      (unsigned long long)tv, 0ull) ==
            (unsigned long long)tv) {
          ent_fill(t, tomb, p, n, dl);
          __hip_atomic_store(ht_key(t, tomb), key, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(ht_val(t, tomb), pv, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          return v;
        }
        tomb = -1;                     // taken by another name: the empty
      }
    }
    // a plain load first: an occupied slot of another key (the usual probe
    // past a tombstone or a collision) costs a load, not an L2 atomic on
    // another line each (keys only ever go 0 -> key within a launch, so a
    // stale 0 just means the CAS below answers); REUSE has just loaded it
    int64_t k = REUSE ? k0 : *ht_key(t, s);
    if (k == 0)
      k = atomicCAS((unsigned long long*)ht_key(t, s), 0ull,
                    (unsigned long long)key);
    if (k == 0) {                         // claimed an empty slot
      ent_fill(t, s, p, n, dl);
      __hip_atomic_store(ht_val(t, s), pv, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      return v;
    }
    if (k == key) {
      int64_t w = 0;
      // The claimer may not have published the val yet: bounded wait.
      for (int spin = 0; spin < 1000000 && w == 0; ++spin)
        w = __hip_atomic_load(ht_val(t, s), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0) return TREE_INSERT_TIMEOUT;
      if (w > 0) {
        int64_t e[HT_W];
        ent_load(t, s, e);
        if (ent_is(t, e, val_node(w), p, n)) return val_node(w);
      }
      // a tombstone of the same key: claim it (0 while its words are
      // rewritten), then publish
      if (val_tomb(w) &&
          atomicCAS((unsigned long long*)ht_val(t, s), (unsigned long long)w,
                    0ull) == (unsigned long long)w) {
        ent_fill(t, s, p, n, dl);
        __hip_atomic_store(ht_val(t, s), pv, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        return v;
      }
    }
    s = (s + 1) & t.mask;
  }
  return -1;
}

// Tombstone node `v`'s hash entry.  Returns its slot for exactly one caller
// when several erase the same node concurrently (the CAS winner owns the
// free), else -1.
ZK_DEV int64_t tree_erase_slot(const ZkTree& t, int64_t v, const uint8_t* p,
                               int32_t n, int64_t tag = VAL_TOMB) {
  const int64_t key = (int64_t)(path_hash(p, n) | 1ull);
  int64_t s = key & t.mask;
  for (int64_t probe = 0; probe <= t.mask; ++probe) {
    // key and val in one round trip: a live val names its node alone (one
    // slot holds it at a time: a move parks the old slot at VAL_MOVING
    // first), and the CAS decides; the key only ends the probe
    const int64_t k = __hip_atomic_load(ht_key(t, s), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    const int64_t cur = __hip_atomic_load(ht_val(t, s), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    if (k == 0) return -1;
    if (k == key && cur > 0 && val_node(cur) == v &&
        atomicCAS((unsigned long long*)ht_val(t, s), (unsigned long long)cur,
                  (unsigned long long)tag) == (unsigned long long)cur)
      return s;
    s = (s + 1) & t.mask;
  }
  return -1;
}

ZK_DEV bool tree_erase(const ZkTree& t, int64_t v, const uint8_t* p,
                       int32_t n) {
  return tree_erase_slot(t, v, p, n) >= 0;
}

// Tombstone reclaim, in a launch where nothing INSERTS (session expiry): a
// tombstone whose next slot is empty lies on no probe chain that reaches a
// live entry (linear probing: an entry's chain from its home slot is
// contiguous non-empty slots), so it can be emptied, and then so can the
// tombstones before it.  Concurrent erasers stay correct: a slot before a
// live entry of its chain never has an empty successor, and the only
// writer of a live entry's val is its own eraser.  Emptiness only grows in
// such a launch, so racing reclaims agree; a missed one is just a tombstone
// left for later.  Without it the storm's never-reused SEQUENTIAL names
// left 1M tombstones a step and the index was rebuilt every few hundred
// steps (round 5: 1.29 ms timed, 1.40 ms sustained).
ZK_DEV int64_t ht_reclaim(const ZkTree& t, int64_t s, bool succ_empty = false);

// Backward shift from the hole s (a tombstone this thread just made), in a
// launch where nothing inserts and the only erasers are those of `session`
// (session expiry): the first live entry after s whose probe chain covers s
// moves into it, its old slot becomes the hole, and so on; the last hole is
// then reclaimed.  Without it, a tombstone right before a live entry (a
// static node, another session's) could only go when an insert passed it,
// and at ~2/3 of the expired names the index filled up anyway (40 create /
// expire rounds: 0 -> 21 % of a 32K-entry table, still growing).  Entries
// of `session` are never moved (their erasers may be probing for them);
// every other live entry has no eraser in the launch, and its val is
// claimed (-3: no lookup matches it) while it moves, so one thread moves it
// and it is found at one slot or the other by any later launch.
ZK_DEV void ht_shift(const ZkTree& t, int64_t s, int64_t session,
                     int64_t tag) {
  for (int moves = 0; moves < 16; ++moves) {
    // the first entry after the hole whose chain covers it: movable (any
    // live entry but `session`'s), or blocking (`session`'s, one moving or
    // being written); none before the run's end: no chain passes the hole
    int64_t j = (s + 1) & t.mask, cand = -1, cv = 0;
    bool blocked = true, tombs = false;
    for (int k = 0; k < 64; ++k, j = (j + 1) & t.mask) {
      // an empty key ends the run whatever the val: the usual first slot
      // (a sparse index) costs one round trip
      if (__hip_atomic_load(ht_key(t, j), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT) == 0) {
        blocked = tombs;
        break;
      }
      // val, key, val: a hole another thread fills between the loads
      // would pair its old key with the new val (the key decides whether
      // the entry covers s), so a val that changed blocks
      const int64_t v1 = __hip_atomic_load(ht_val(t, j), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      order_wait();
      const int64_t key = __hip_atomic_load(ht_key(t, j), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      if (key == 0) {
        // (a tombstone on the way may be another thread's hole that an
        // entry covering s is moving into right now — seen here as the
        // tombstone before, and at its old slot as the tombstone after:
        // then s is not emptied)
        blocked = tombs;
        break;
      }
      order_wait();
      const int64_t val = __hip_atomic_load(ht_val(t, j), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      if (val != v1) break;                         // (blocking)
      if (val_tomb(val)) {                          // tombstone
        if (val == tag) tombs = true;               // (of this launch)
        continue;
      }
      if (val > 0 &&
          ((j - (key & t.mask)) & t.mask) < ((j - s) & t.mask))
        continue;                                   // home after the hole
      if (val > 0 && t.eph[val_node(val)] != session) {
        cand = j;
        cv = val;
      }
      break;                                        // (else: blocking)
    }
    if (cand < 0) {
      if (!blocked) {
        // nothing reaches past the hole: empty it, then the tombstones
        // before it (their successor is now empty)
        __hip_atomic_store(ht_val(t, s), (int64_t)0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        order_wait();
        __hip_atomic_store(ht_key(t, s), (int64_t)0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        // (s's key is this thread's 0 — an empty slot stays empty in the
        // launch — so the reclaim's first step reads only the val before;
        // it is read after the run's end was seen empty, as it must be)
        ht_reclaim(t, (s - 1) & t.mask, true);
      }
      return;
    }
    if (atomicCAS((unsigned long long*)ht_val(t, cand), (unsigned long long)cv,
                  (unsigned long long)VAL_MOVING) != (unsigned long long)cv)
      return;
    if (atomicCAS((unsigned long long*)ht_val(t, s), (unsigned long long)tag,
                  0ull) != (unsigned long long)tag) {
      __hip_atomic_store(ht_val(t, cand), cv, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    int64_t e[HT_W];
    ent_load(t, cand, e);
    int64_t* d = ht_ent(t, s);
#pragma unroll
    for (int w = 2; w < HT_W; ++w) d[w] = e[w];
    __hip_atomic_store(ht_key(t, s), e[0], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    order_wait();                       // the key before the val ...
    __hip_atomic_store(ht_val(t, s), cv, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    order_wait();                       // ... and the copy before the vacate
    __hip_atomic_store(ht_val(t, cand), tag, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    s = cand;                                       // the new hole
  }
  ht_reclaim(t, s);
}

ZK_DEV int64_t ht_reclaim(const ZkTree& t, int64_t s, bool succ_empty) {
  int64_t n = 0;
  for (int k = 0; k < 64; ++k) {
    const int64_t nx = (s + 1) & t.mask;
    if (succ_empty && k == 0) {
      if (!val_tomb(__hip_atomic_load(ht_val(t, s), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT)))
        break;
      __hip_atomic_store(ht_val(t, s), (int64_t)0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      order_wait();
      __hip_atomic_store(ht_key(t, s), (int64_t)0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      ++n;
      s = (s - 1) & t.mask;
      continue;
    }
    // the successor's key first, the val after it: a val read before an
    // entry moved into s (from past nx, which was emptied after) paired
    // with the emptied key would drop the live entry — both loads in one
    // round trip lost a storm node in a 400-step run
    if (__hip_atomic_load(ht_key(t, nx), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT) != 0)
      break;
    if (!val_tomb(__hip_atomic_load(ht_val(t, s), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT)))
      break;
    // val first: a reader between the two stores sees a key with val 0
    // (no match, probe on), then the empty key (end of chain)
    __hip_atomic_store(ht_val(t, s), (int64_t)0, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    order_wait();
    __hip_atomic_store(ht_key(t, s), (int64_t)0, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    ++n;
    s = (s - 1) & t.mask;
  }
  return n;
}

// tree_erase at the entry a lookup just found (slot s): no second probe.
// The CAS against the live val the lookup saw keeps one winner among
// concurrent erasers of the node; a lost race answers like tree_erase.
ZK_DEV bool tree_erase_at(const ZkTree& t, int64_t s, int64_t v) {
  if (s < 0) return false;
  const int64_t cur = __hip_atomic_load(ht_val(t, s), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
  return cur > 0 && val_node(cur) == v &&
         atomicCAS((unsigned long long*)ht_val(t, s), (unsigned long long)cur,
                   (unsigned long long)VAL_TOMB) == (unsigned long long)cur;
}

// ---- watches (one-shot, per watcher slot) ---------------------------------
// A path-keyed table beside the tree (lib/zk-session.js:482-526 describes
// the server semantics the client relies on): key = path
// hash | 1 (0 = empty, linear probing, entries are never removed), two
// 64-bit masks per entry — the data watches (GET_DATA / EXISTS with
// watch=1; an EXISTS on a missing path is ZooKeeper's "exist" watch, kept
// in the same set like the server's dataWatches) and the child watches —
// one bit per watcher slot (<= 64 sessions of the server).  Firing is an
// atomic exchange with 0: one-shot, and each watcher of a path is notified
// exactly once even when several writes of a batch hit the path (the first
// takes the mask).  Paths are keyed, not nodes, so a watch on a missing
// path waits for its creation.
enum : int { WK_DATA = 0, WK_CHILD = 1 };
// notification types (lib/zk-consts.js NOTIFICATION_TYPE)
enum : int32_t { NT_CREATED = 1, NT_DELETED = 2, NT_DATA_CHANGED = 3,
                 NT_CHILDREN_CHANGED = 4 };
constexpr int WT_REC = 5;    // per request: m_path, m_path_child, m_parent,
                             // path word of the node, of its parent

ZK_DEV int64_t wt_slot(const ZkTree& t, uint64_t key, bool insert) {
  int64_t s = (int64_t)key & t.wt_hmask;
  for (int64_t probe = 0; probe <= t.wt_hmask; ++probe) {
    int64_t k = __hip_atomic_load(&t.wt_key[s], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    if (k == (int64_t)key) return s;
    if (k == 0) {
      if (!insert) return -1;
      k = (int64_t)atomicCAS((unsigned long long*)&t.wt_key[s], 0ull,
                             (unsigned long long)key);
      if (k == 0 || k == (int64_t)key) return s;
    }
    s = (s + 1) & t.wt_hmask;
  }
  return -1;                                      // table full
}

ZK_DEV void wt_arm(const ZkTree& t, const uint8_t* p, int32_t n, int kind,
                   int32_t wslot) {
  if (t.wt_key == nullptr || wslot < 0 || wslot > 63) return;
  const int64_t s = wt_slot(t, path_hash(p, n) | 1ull, true);
  if (s >= 0) atomicOr(&t.wt_mask[2 * s + kind], 1ull << wslot);
}

ZK_DEV uint64_t wt_fire(const ZkTree& t, const uint8_t* p, int32_t n,
                        int kind) {
  if (t.wt_key == nullptr) return 0;
  const int64_t s = wt_slot(t, path_hash(p, n) | 1ull, false);
  if (s < 0) return 0;
  unsigned long long* m = &t.wt_mask[2 * s + kind];
  if (__hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    return 0;
  return atomicExch(m, 0ull);
}

// Node v's path from its path word.
ZK_DEV const uint8_t* node_path(const ZkTree& t, int64_t pw) {
  return t.path_arena + (pw >> 24);
}
ZK_DEV int32_t pw_len(int64_t pw) { return (int32_t)(pw & 0xFFFFFF); }

ZK_DEV void fill_stat(uint8_t* st, int64_t cz, int64_t mz, int64_t ct,
                      int64_t mt, int32_t ver, int32_t cver, int32_t aver,
                      int64_t owner, int32_t dlen, int32_t nkids, int64_t pz) {
  st_be64(st + 0, cz); st_be64(st + 8, mz); st_be64(st + 16, ct);
  st_be64(st + 24, mt); st_be32(st + 32, ver); st_be32(st + 36, cver);
  st_be32(st + 40, aver); st_be64(st + 44, owner); st_be32(st + 52, dlen);
  st_be32(st + 56, nkids); st_be64(st + 60, pz);
}

// The parent counters (cversion << 32 | numChildren in one word, so a
// child's create or delete moves both with one device-scope atomic: on the
// multi-XCD part each is a trip to the coherence point).  numChildren never
// goes negative, so a signed add of (dc << 32) + dk never borrows across.
ZK_DEV int64_t cn_pack(int32_t cver, int32_t nchild) {
  return (int64_t)((uint64_t)(uint32_t)cver << 32 | (uint32_t)nchild);
}
ZK_DEV int32_t cn_cver(int64_t x) { return (int32_t)((uint64_t)x >> 32); }
ZK_DEV int32_t cn_nchild(int64_t x) { return (int32_t)(uint32_t)x; }
ZK_DEV int64_t cn_add(const ZkTree& t, int64_t v, int32_t dc, int32_t dk) {
  return (int64_t)atomicAdd((unsigned long long*)&t.cn[v],
                            (unsigned long long)(((int64_t)dc << 32) + dk));
}

// ---- parent bookkeeping ----------------------------------------------------
// Child added (dkids = 1) / removed (-1) under `par` by the txn `zx`;
// `bump_cver` is false when a SEQUENTIAL create already took the cversion.
ZK_DEV void parent_touch(const ZkTree& t, int64_t par, int32_t dkids,
                         bool bump_cver, int64_t zx) {
  cn_add(t, par, bump_cver ? 1 : 0, dkids);
  atomicMax((unsigned long long*)&t.pzxid[par], (unsigned long long)zx);
}

// Put every distinct parent this block touched on the dirty list once
// (block-uniform call).
ZK_DEV void wave_mark_dirty(const ZkTree& t, int64_t par) {
  bool first = false;
  if (par >= 0 && __hip_atomic_load(&t.dirty[par], __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) == 0)
    first = atomicExch(&t.dirty[par], 1) == 0;
  const int64_t k = block_ticket(&t.counters[TC_DIRTY], first);
  if (first) t.dirty_list[k] = par;
}

// Free `v` (block-uniform call; `v < 0` = nothing to free).
ZK_DEV void wave_free(const ZkTree& t, int64_t v,
                      unsigned long long* count = nullptr) {
  if (v >= 0) t.node_parent[v] = NODE_FREE;
  const int64_t k = block_ticket(&t.counters[TC_FREE_TAIL], v >= 0, count);
  if (v >= 0) t.free_list[k % t.free_cap] = v;
}

// wave_mark_dirty with the parent's flag already loaded (flag: its value;
// nonzero: on the list, or no parent)
ZK_DEV void wave_mark_dirty_at(const ZkTree& t, int64_t par, int32_t flag) {
  const bool first = par >= 0 && flag == 0 && atomicExch(&t.dirty[par], 1) == 0;
  const int64_t k = block_ticket(&t.counters[TC_DIRTY], first);
  if (first) t.dirty_list[k] = par;
}

__global__ __launch_bounds__(TR_T) void tree_fill_k(ZkTree t, int64_t n0,
                                                   int64_t n,
                                                   const int32_t* __restrict__ nkids,
                                                   int64_t now_ms) {
  const int64_t v = n0 + (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (v >= n) return;
  const ZkNodeStore& s = t.store;
  uint8_t* slot = s.slab + s.slot_off[v];
  const int32_t dl = s.data_len[v];
  fill_stat(slot, v + 1, v + 1, now_ms, now_ms, 0, nkids[v], 0, 0, dl,
            nkids[v], v + 1);
  st_be32(slot + 68, 0);
  st_be32(slot + ZK_SLOT_LEN, dl > 0 ? dl : -1);
  t.cn[v] = cn_pack(nkids[v], nkids[v]);
  t.pzxid[v] = v + 1;
  t.eph[v] = 0;
  t.dirty[v] = 0;
}

// Free-ring compaction between batches: the ring's pending entries rebuilt
// as every free node in ascending order.  Frees go to the ring in the
// order the workgroups of a batch happened to take their tickets, and
// creates take the ring in ticket order too, so over a few hundred batches
// of create / delete the nodes one workgroup creates scatter over the whole
// node table (each per-node field a random line instead of a shared one):
// the mix step drifted 1.42 -> 1.65 ms and the nest step 6.26 -> 7.78 ms
// over 600 / 200 steps (profiles/r5_free_ring_locality.md).  Sorted, a
// workgroup's creates take nodes from one dense run again.  Two passes and
// a scan over the node high-water mark; at a batch boundary the pending
// entries are exactly the free nodes (the finish published every free).
__global__ __launch_bounds__(TR_T) void free_count_k(ZkTree t,
                                                    int64_t* __restrict__ bsum) {
  __shared__ int32_t c[TR_T / 64];
  const int64_t nn = min(t.counters[TC_NODES], t.store.cap);
  const int64_t v = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  const bool f = v < nn && t.node_parent[v] == NODE_FREE;
  const uint64_t m = __ballot(f);
  if ((threadIdx.x & 63) == 0) c[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t s = 0;
    for (int k = 0; k < TR_T / 64; ++k) s += c[k];
    bsum[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(TR_T) void free_scatter_k(
    ZkTree t, const int64_t* __restrict__ bbase,
    const int64_t* __restrict__ total) {
  __shared__ int32_t c[TR_T / 64];
  const int64_t head = t.counters[TC_FREE_HEAD];
  const int64_t nn = min(t.counters[TC_NODES], t.store.cap);
  const int64_t v = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  const bool f = v < nn && t.node_parent[v] == NODE_FREE;
  const uint64_t m = __ballot(f);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) c[w] = __popcll(m);
  __syncthreads();
  int64_t r = bbase[blockIdx.x] +
              __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  for (int k = 0; k < w; ++k) r += c[k];
  if (f) t.free_list[(head + r) % t.free_cap] = v;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t.counters[TC_FREE_TAIL] = head + *total;
    t.counters[TC_FREE_PUB] = head + *total;
  }
}

__global__ __launch_bounds__(TR_T) void tree_build_k(ZkTree t, int64_t n0,
                                                    int64_t n) {
  const int64_t v = n0 + (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (v >= n || t.node_parent[v] == NODE_FREE) return;
  tree_insert(t, v, t.path_arena + t.node_path_off[v], t.node_path_len[v],
              t.store.data_len[v]);
}

// Write "%010d" of a non-negative sequence number (ZooKeeper's sequential
// suffix; the counter is the parent's cversion).
ZK_DEV void put_seq10(uint8_t* d, int32_t x) {
  uint32_t u = (uint32_t)x;
#pragma unroll
  for (int k = 9; k >= 0; --k) { d[k] = (uint8_t)('0' + u % 10); u /= 10; }
}

// Per-lane state of one request through the three phases of tree_serve_k.
struct Lane {
  int32_t op, err, pl, dl, flags, dlen;
  int64_t node, zx, par, slot;
  const uint8_t* path;
};

// Reply frame size (length word included) of a served request, as
// encode.hip's resp_body_size computes it from the reply descriptors.
ZK_DEV int64_t served_reply_size(int32_t op, int32_t err, int32_t dl,
                                 int32_t rpl) {
  const int64_t sz = 4 + 16;                    // length, xid, zxid, err
  if (err != ERR_OK) return sz;
  switch (op) {
    case OP_GET_DATA: return sz + 4 + max(dl, 0) + STAT_BYTES;
    case OP_EXISTS: case OP_SET_DATA: return sz + STAT_BYTES;
    case OP_CREATE: return sz + 4 + max(rpl, 0);
    default: return sz;
  }
}

// The ordering pass's word for request i (zk_tree_seq_order): parent node
// << 32 | its SEQUENTIAL number, -1 when it has none.
ZK_DEV int32_t seq_num(const ZkTree& t, int64_t i) {
  if (t.seqno == nullptr) return -1;
  const int64_t x = t.seqno[i];
  return x < 0 ? -1 : (int32_t)(uint32_t)x;
}
ZK_DEV int64_t seq_par(const ZkTree& t, int64_t i) {
  return t.seqno == nullptr || t.seqno[i] < 0 ? -1 : t.seqno[i] >> 32;
}

// CREATE (lib/zk-buffer.js:97-136 request shape; semantics of the server the
// reference talks to): parent must exist and not be ephemeral, ACL must be
// non-empty, SEQUENTIAL appends the parent's cversion, EPHEMERAL records the
// owning session in the Stat.  `v` (with storage `po` / `so`) was claimed
// for this lane in phase A; on failure the caller frees it.
ZK_DEV int32_t do_create(const ZkTree& t, Lane& L, const uint8_t* data,
                         int32_t nacl, int64_t session, int64_t now_ms,
                         int64_t v, int64_t i) {
  const ZkNodeStore& s = t.store;
  const bool eph = L.flags & CF_EPHEMERAL, seq = L.flags & CF_SEQUENTIAL;
  // a create the ordering pass numbered: the pass also counted it as its
  // parent's child (one atomic per parent a batch, not one per create); if
  // it fails, tree_serve_k takes the count back (seq_par)
  const int32_t pre = seq ? seq_num(t, i) : -1;
  if (nacl <= 0) return ERR_INVALID_ACL;
  if (v < 0) return ERR_SYSTEM;                       // tree full
  // node v's path and slot offsets, loaded before the parent lookup: their
  // round trip rides under it (a create is a chain of dependent trips)
  const int64_t vpo = t.node_path_off[v];
  const int64_t vso = s.slot_off[v];
  const uint8_t* path = L.path;
  const int32_t pl = L.pl;
  int32_t cut = pl - 1;
  while (cut > 0 && path[cut] != '/') --cut;
  const int64_t par = cut > 0 ? tree_find(t, path, cut) : -1;
  if (cut > 0 && par < 0) return ERR_NO_NODE;
  if (par >= 0 && t.eph[par] != 0)
    return ERR_NO_CHILDREN_FOR_EPHEMERALS;
  // (an existing path is found by tree_insert itself — it probes the same
  // chain and answers NODE_EXISTS before publishing anything — so the
  // usual, successful create walks the chain once, not twice; what this
  // lane wrote to its own node v before is freed by the caller)
  const int32_t npl = pl + (seq ? 10 : 0);
  // a SEQUENTIAL name: the number zk_tree_seq_order assigned it in stream
  // order (the parent's cversion at the batch's start + the request's rank
  // among the batch's sequential creates under that parent; the parent was
  // bumped once for all of them, and a failed create leaves a gap, never a
  // number handed back).  Without one (no ordering pass, or a parent the
  // pass did not find) the parent's cversion is taken here, bumped in the
  // same atomic as its child count — unique, but in arrival order.
  const bool taken = seq && par >= 0 && pre < 0;
  const int32_t seqno = !seq || par < 0 ? 0
                        : pre >= 0      ? pre
                                        : cn_cver(cn_add(t, par, 1, 1));
  uint8_t* pd = t.path_arena + vpo;
  copy_bytes(pd, path, pl);
  if (seq) put_seq10(pd + pl, seqno);
  const int32_t dl = L.dl;
  uint8_t* slot = s.slab + vso;
  fill_stat(slot, L.zx, L.zx, now_ms, now_ms, 0, 0, 0, eph ? session : 0, dl,
            0, L.zx);
  st_be32(slot + ZK_SLOT_LEN, dl > 0 ? dl : -1);
  copy_bytes(slot + ZK_SLOT_DATA, data, dl);
  t.node_path_len[v] = npl;
  s.data_len[v] = dl;
  t.cn[v] = 0;
  t.pzxid[v] = L.zx;
  t.node_parent[v] = par;
  t.node_pw[v] = pw_pack(pd - t.path_arena, npl);
  // No fence before publishing v in the hash: only a same-batch reader of
  // this very path could observe the half-written node (unordered by the
  // batch contract; every field it could read is in bounds), and the next
  // launch sees everything.  A __threadfence here is an XCD-L2 writeback
  // per wave (MI355X_MICROARCH.md: ~3.5 us each) and cost milliseconds.
  const int64_t ins = pre >= 0 ? tree_insert<true>(t, v, pd, npl, dl, vso)
                               : tree_insert(t, v, pd, npl, dl, vso);
  if (ins != v) {
    // the child was not made (the cversion it took stays: a gap)
    if (taken) cn_add(t, par, 0, -1);
    return ins == TREE_INSERT_TIMEOUT ? ERR_SYSTEM : ERR_NODE_EXISTS;
  }
  t.eph[v] = eph ? session : 0;
  if (par >= 0) {
    if (seq) {
      // (cversion and child count: taken above, or by the ordering pass)
      atomicMax((unsigned long long*)&t.pzxid[par], (unsigned long long)L.zx);
    } else {
      parent_touch(t, par, 1, true, L.zx);
    }
  }
  L.par = par;
  L.node = v;
  L.slot = s.slot_off[v];
  return ERR_OK;
}

// Apply one batch of decoded requests; produce reply descriptors for K13.
// r_path_off/len (may be null) receive the created node's path in the tree's
// path arena (SEQUENTIAL names differ from the requested one).  r_slot,
// r_sizes and r_bsum (may be null) receive each reply's slot offset, its
// frame size and the block's size sum, so the reply encoder needs neither
// its sizes pass nor a lookup of the node's slot (zk_encode_responses2
// presized).
// PARSE: the requests come as K1 frames (foff / flen) and each lane parses
// its own in registers (zk_reqparse.h) instead of reading K12's SoA back —
// one launch and a 30 MB write + read less per 512K-request batch.
ZK_DEV void finish_body(const ZkTree& t, const int64_t* n_dev,
                        int64_t bump_zxid, int32_t publish);
ZK_DEV bool serve_last(unsigned* tickets);

// RO: a batch of reads only (GET_DATA / EXISTS; the GET pipeline's): no
// node / storage claims, frees or dirty parents, so none of their five
// block-wide ticket barriers per workgroup; any other op is answered
// UNIMPLEMENTED.  (A run-time vote of the block for the same skip cost the
// create storm 10 %; a template costs the write batches nothing.)
template <bool PARSE, bool RO = false>
__global__ __launch_bounds__(TR_T) void tree_serve_k(
    ZkTree t, const uint8_t* __restrict__ rx, ZkReqOut q,
    const int64_t* __restrict__ foff, const int32_t* __restrict__ flen,
    const int64_t* __restrict__ n_dev, int64_t ncap, int32_t* __restrict__ r_op,
    int32_t* __restrict__ r_xid, int32_t* __restrict__ r_err,
    int64_t* __restrict__ r_node, int64_t* __restrict__ r_zxid,
    int64_t* __restrict__ r_path_off, int32_t* __restrict__ r_path_len,
    int64_t* __restrict__ r_slot, int64_t* __restrict__ r_sizes,
    int64_t* __restrict__ r_bsum, int64_t session, int64_t now_ms,
    const uint8_t* __restrict__ rank, int32_t pass, int32_t last_pass,
    int64_t snap_base, int64_t snap_cap, int64_t* __restrict__ snap_top,
    int32_t wslot, int64_t* __restrict__ fired, unsigned* tickets) {
  session = sess_of(t, session);
  const uint32_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t i = (int64_t)blk * TR_T + threadIdx.x;
  const bool in_batch = i < ncap && i < *n_dev;
  // ordered passes: this launch serves the requests of rank `pass`; the
  // last pass also answers any of a higher rank, refused (SYSTEMERROR: more
  // same-path requests than passes).  rank bit 7: a later request of the
  // batch writes this path, so the reply's slot is snapshotted.
  const int32_t rb = rank != nullptr && in_batch ? (int32_t)rank[i] : 0;
  const int32_t rk = rb & ORD_RANK;
  const bool live = in_batch && (rk == pass || (last_pass && rk > pass));
  const bool refused = live && rk > pass;
  ReqFields rq{ST_BAD_DECODE, 0, OP_PING, 0, 0, 0, 0, -1, -1, -1, 0};
  if (live) {
    if (PARSE) {
      rq = parse_request(rx, foff[i], flen[i]);
    } else {
      rq.status = q.status[i];
      rq.xid = q.xid[i];
      rq.op = q.opcode[i];
      rq.arg = q.arg[i];
      rq.pl = q.path_len[i];
      rq.dl = q.data_len[i];
      rq.vc = q.vec_count[i];
      rq.poff = q.path_off[i];
      rq.doff = q.data_off[i];
    }
  }
  const bool ok_req = live && !refused && rq.status == ST_OK;
  const ZkNodeStore& s = t.store;
  Lane L;
  L.op = live ? rq.op : OP_PING;
  L.err = refused ? ERR_SYSTEM : (live && !ok_req ? ERR_BAD_ARGUMENTS : ERR_OK);
  L.node = -1;
  L.slot = -1;
  L.dlen = 0;
  L.par = -1;
  L.flags = 0;
  L.path = nullptr;
  L.pl = L.dl = 0;
  if (ok_req) {
    L.path = rx + rq.poff;
    L.pl = rq.pl;
    L.dl = max(rq.dl, 0);
    L.flags = rq.arg;
  }
  // ---- phase A: wave-aggregated claims -----------------------------------
  // zxids without atomics: write i of the batch is txn base + i + 1, reads
  // see base; tree_publish_k advances the counter by the batch size.
  const bool write = ok_req && (L.op == OP_CREATE || L.op == OP_SET_DATA ||
                                L.op == OP_DELETE);
  const int64_t zbase = t.counters[TC_ZXID];
  L.zx = write ? zbase + i + 1 : zbase;
  const bool create = !RO && ok_req && L.op == OP_CREATE;
  int64_t v = -1;
  int32_t npl = 0, cap = 0;
  if (create) {
    npl = L.pl + ((L.flags & CF_SEQUENTIAL) ? 10 : 0);
    cap = max(L.dl, 128);
  }
  if (RO && ok_req && L.op != OP_GET_DATA && L.op != OP_EXISTS)
    L.err = ERR_UNIMPLEMENTED;
  if (!RO) {
    const int64_t pub = t.counters[TC_FREE_PUB];
    const int64_t h = block_ticket(&t.counters[TC_FREE_HEAD], create);
    if (create && h < pub) v = t.free_list[h % t.free_cap];
    const bool fresh = create && v < 0;
    const int64_t nv = block_ticket(&t.counters[TC_NODES], fresh);
    if (fresh && nv < s.cap) v = nv;
    // storage: reuse the recycled node's when it fits (path storage comes
    // in 16-byte multiples and keeps its capacity, so nodes recycled across
    // paths of a few lengths stop allocating: the arena is bounded by the
    // node count, not by the number of creates)
    const bool new_path = v >= 0 && (fresh || npl > t.node_path_cap[v]);
    const bool new_slot = v >= 0 && (fresh || cap > s.slot_cap[v]);
    const int32_t pcap = (npl + 15) & ~15;
    const int64_t po = wave_bytes(&t.counters[TC_PATH_TOP],
                                  new_path ? pcap : 0);
    const int64_t sb = new_slot ? slot_bytes(cap) : 0;
    const int64_t so = wave_bytes(&t.counters[TC_SLAB_TOP], sb);
    if (new_path) {
      if (po + pcap <= t.path_cap) {
        t.node_path_off[v] = po;
        t.node_path_len[v] = npl;
        t.node_path_cap[v] = pcap;
      } else {
        t.node_path_len[v] = 0;                     // storage-less free node
        t.node_path_cap[v] = 0;
      }
    }
    if (new_slot) {
      if (so + sb <= t.slab_cap) {
        s.slot_off[v] = so;
        s.slot_cap[v] = cap;
      } else {
        s.slot_cap[v] = -1;
      }
    }
    if (v >= 0 && ((new_path && po + pcap > t.path_cap) ||
                   (new_slot && so + sb > t.slab_cap))) {
      L.err = ERR_SYSTEM;                           // arena full
    }
  }
  // ---- phase B: the operation -------------------------------------------
  int64_t freed = -1;
  // a SEQUENTIAL create the ordering pass numbered (and counted as its
  // parent's child) that never reaches do_create — refused by the ordered
  // passes, or out of arena — takes that child back below
  // (the pass reads a frame's op, path and flags only: a frame it numbered
  // that the full parse refuses is taken back here too)
  bool numbered = !RO && live && seq_num(t, i) >= 0;
  if (ok_req && L.err == ERR_OK) {
    switch (L.op) {
      case OP_GET_DATA: case OP_EXISTS:
        {
          const Found f = tree_lookup<true>(t, L.path, L.pl);
          L.node = f.node;
          L.slot = f.slot;
          L.dlen = f.dlen;
        }
        if (L.node < 0) L.err = ERR_NO_NODE;
        break;
      case OP_SET_DATA: {
        const Found f = tree_lookup(t, L.path, L.pl);
        const int64_t node = f.node;
        if (node < 0) { L.err = ERR_NO_NODE; break; }
        L.slot = f.slot;
        if (L.dl > s.slot_cap[node]) { L.err = ERR_BAD_ARGUMENTS; break; }
        uint8_t* slot = s.slab + L.slot;
        unsigned int* ver = (unsigned int*)(slot + 32);
        const int32_t want = L.flags;
        unsigned int old = *ver, cmp;
        do {                                          // version CAS
          cmp = old;
          if (want != -1 && cmp != bswap32((uint32_t)want)) break;
          old = atomicCAS(ver, cmp, bswap32(bswap32(cmp) + 1));
        } while (old != cmp);
        if (old != cmp || (want != -1 && cmp != bswap32((uint32_t)want))) {
          L.err = ERR_BAD_VERSION;
          break;
        }
        copy_bytes(slot + ZK_SLOT_DATA, rx + rq.doff, L.dl);
        st_be32(slot + ZK_SLOT_LEN, L.dl > 0 ? L.dl : -1);
        s.data_len[node] = L.dl;
        ent_set_dlen(t, f.ent, L.dl);
        st_be64(slot + 8, L.zx);                      // mzxid
        st_be64(slot + 24, now_ms);                   // mtime
        st_be32(slot + 52, L.dl);                     // dataLength
        L.node = node;
        break;
      }
      case OP_CREATE:
        L.err = do_create(t, L, rx + rq.doff, rq.vc, session,
                          now_ms, v, i);
        if (L.err == ERR_OK) numbered = false;      // the child is made
        if (L.err == ERR_OK && r_path_off != nullptr) {
          r_path_off[i] = t.node_path_off[v];
          r_path_len[i] = t.node_path_len[v];
        }
        break;
      case OP_DELETE: {
        const Found f = tree_lookup(t, L.path, L.pl);
        const int64_t node = f.node, so = f.slot;
        if (node < 0) { L.err = ERR_NO_NODE; break; }
        if (cn_nchild(__hip_atomic_load(&t.cn[node], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT)) > 0) {
          L.err = ERR_NOT_EMPTY;
          break;
        }
        const int32_t want = L.flags;
        if (want != -1 && ld_be32(s.slab + so + 32) != want) {
          L.err = ERR_BAD_VERSION;
          break;
        }
        if (!tree_erase_at(t, f.ent, node)) { L.err = ERR_NO_NODE; break; }
        L.par = t.node_parent[node];
        if (L.par >= 0) parent_touch(t, L.par, -1, true, L.zx);
        t.eph[node] = 0;
        freed = node;
        break;
      }
      case OP_SYNC: case OP_PING:
        break;
      case OP_SET_WATCHES:
        // header-only reply; the catch-up (notifications for what changed
        // after relZxid, re-registration of the rest) is zk_watch_resume
        break;
      default:
        L.err = ERR_UNIMPLEMENTED;
    }
  }
  if (numbered) cn_add(t, seq_par(t, i), 0, -1);
  // ---- watches: reads with watch=1 arm (this session's slot), successful
  // writes fire (lib/zk-session.js:558-574 is the client side of the
  // trigger table; the server rules are SURVEY Appendix D)
  if (t.wt_key != nullptr && ok_req) {
    const bool wflag = rq.arg == 1;
    if (L.op == OP_GET_DATA && wflag && L.err == ERR_OK) {
      wt_arm(t, L.path, L.pl, WK_DATA, wslot);
    } else if (L.op == OP_EXISTS && wflag &&
               (L.err == ERR_OK || L.err == ERR_NO_NODE)) {
      wt_arm(t, L.path, L.pl, WK_DATA, wslot);
    } else if (L.err == ERR_OK && (L.op == OP_SET_DATA ||
                                   L.op == OP_CREATE ||
                                   L.op == OP_DELETE)) {
      const int64_t node = L.op == OP_DELETE ? freed : L.node;
      const int64_t pw = t.node_pw[node];
      const int64_t ppw = L.par >= 0 ? t.node_pw[L.par] : 0;
      const uint8_t* np = node_path(t, pw);
      const int32_t nl = pw_len(pw);
      uint64_t m0 = wt_fire(t, np, nl, WK_DATA), m1 = 0, m2 = 0;
      if (L.op == OP_DELETE) m1 = wt_fire(t, np, nl, WK_CHILD) & ~m0;
      if (L.op != OP_SET_DATA && L.par >= 0)
        m2 = wt_fire(t, node_path(t, ppw), pw_len(ppw), WK_CHILD);
      if (fired != nullptr) {
        int64_t* f = fired + (int64_t)WT_REC * i;
        f[0] = (int64_t)m0;
        f[1] = (int64_t)m1;
        f[2] = (int64_t)m2;
        f[3] = pw;
        f[4] = ppw;
      }
    }
  }
  // ---- ordered snapshot: a reply that reads the node's slot (stat, data)
  // while a later pass of this batch writes the node reads a private copy
  // in the slab's scratch tail, taken now (wave-aggregated claim)
  if (rank != nullptr) {
    const bool snap = (rb & ORD_SNAP) && live && L.err == ERR_OK &&
                      (L.op == OP_GET_DATA || L.op == OP_EXISTS ||
                       L.op == OP_SET_DATA);
    const int64_t dl = snap && L.op == OP_GET_DATA ? L.dlen : 0;
    const int64_t sb = snap ? slot_bytes((int32_t)dl) : 0;
    const int64_t so = wave_bytes(snap_top, sb);
    if (snap) {
      if (so + sb <= snap_cap) {
        copy_bytes(s.slab + snap_base + so, s.slab + L.slot,
                   (int32_t)(ZK_SLOT_DATA + dl));
        L.slot = snap_base + so;
      } else {
        L.err = ERR_SYSTEM;              // scratch full (counted by caller)
      }
    }
  }
  // ---- phase C: wave-aggregated frees and dirty parents -----------------
  if (create && L.err != ERR_OK && v >= 0) freed = v;  // return the claim
  // (A read-only block could skip these claims, but guarding them with a
  // block vote cost the create storm 10% in measurement; they stay, except
  // in the RO instance.)
  if (!RO) {
    wave_free(t, freed);
    wave_mark_dirty(t, L.err == ERR_OK ? L.par : -1);
  }
  if (r_sizes != nullptr) {                       // block-uniform
    __shared__ int64_t sm[TR_T / 64 + 1];
    int64_t sz = 0;
    if (live) {
      const bool get = L.err == ERR_OK && L.op == OP_GET_DATA;
      const bool mk = L.err == ERR_OK && L.op == OP_CREATE;
      sz = served_reply_size(L.op, L.err, get ? L.dlen : 0,
                             mk ? t.node_path_len[L.node] : 0);
      r_sizes[i] = sz;
    } else if (in_batch && rk < pass) {
      sz = r_sizes[i];                  // served by an earlier pass
    } else if (!in_batch && i < ncap) {
      r_sizes[i] = 0;
    }
    int64_t tot;
    block_excl_scan(sz, sm, &tot);
    if (threadIdx.x == 0) r_bsum[blk] = tot;
  }
  // the finish in the launch's last workgroup (no tree_finish_k launch)
  if (tickets != nullptr && serve_last(tickets))
    finish_body(t, n_dev, 0, 1);
  if (!live) return;
  r_op[i] = L.op;
  r_xid[i] = rq.xid;
  r_err[i] = L.err;
  r_node[i] = L.op == OP_DELETE ? -1 : L.node;
  r_zxid[i] = L.zx;
  if (r_slot != nullptr) r_slot[i] = L.op == OP_DELETE ? -1 : L.slot;
}

// ---- in-batch ordering (tree_order_*) ---------------------------------------
// ZooKeeper applies a session's pipelined requests in order.  Two requests
// of a batch conflict when they touch the same path and one writes it, or
// when one creates / deletes a CHILD of the path the other operates on (the
// child write changes the parent's cversion / numChildren / pzxid and needs
// the parent to exist; a parent delete needs it gone):
//   * every request with a path joins its own path's group as an A member;
//   * a CREATE / DELETE also joins its parent's group as a C member (a
//     SEQUENTIAL create only that one: its own name is fresh).
// Edges inside a group (the later request runs in a later pass): A-A when
// the group has an A writer, A-C and C-A always, C-C never (children of one
// parent commute).  rank[i] = the longest chain of edges ending at i,
// computed by relaxation (`passes` + 1 rounds; a rank >= passes is refused
// with SYSTEMERROR, as before).  A scratch hash table groups the batch by
// path hash (a 64-bit collision merges two groups: extra ordering, never
// less); only ordered groups get member lists (offsets from a block scan of
// the group sizes: no shared counter).  No kernel here puts more than one
// atomic per block on a shared word, except the per-group counters (a
// single word sustains ~88 returning atomics per us, MI355X_MICROARCH.md).
constexpr int64_t ORD_MAX_GROUP = 1 << 16;   // larger ordered groups: refused
constexpr int ORD_F = 21;                     // bits per packed group count
constexpr int64_t ORD_FM = (1ll << ORD_F) - 1;

struct OrderWs {
  int64_t* ctr;      // [4] -, max rank, scratch top, -
  int64_t* key;      // [h] path hash | 1
  int64_t* cnt;      // [h] A | A writers << 21 | C << 42
  int32_t* fill;     // [h] member-list fill
  int32_t* lastw;    // [h] 1 + index of the group's last writer (A or C)
  int32_t* base;     // [h] member-list offset within its block of entries
  int64_t* bsum;     // [h / TR_T] block totals, then exclusive offsets
  int64_t* eidx;     // [2 ncap] request -> own (A) entry, parent (C) entry
  int32_t* members;  // [2 ncap] request << 1 | (1 = C member)
  int32_t* rnk;      // [ncap] relaxed ranks
  int64_t mask;      // h - 1
};

ZK_DEV bool ord_has_path(int32_t op) {
  return op == OP_CREATE || op == OP_DELETE || op == OP_SET_DATA ||
         op == OP_GET_DATA || op == OP_EXISTS || op == OP_GET_CHILDREN ||
         op == OP_GET_CHILDREN2 || op == OP_GET_ACL || op == OP_SYNC;
}

ZK_DEV bool ord_writes(int32_t op) {
  return op == OP_CREATE || op == OP_DELETE || op == OP_SET_DATA;
}

ZK_DEV int64_t ord_na(int64_t c) { return c & ORD_FM; }
ZK_DEV int64_t ord_naw(int64_t c) { return (c >> ORD_F) & ORD_FM; }
ZK_DEV int64_t ord_nc(int64_t c) { return (c >> (2 * ORD_F)) & ORD_FM; }
ZK_DEV int64_t ord_size(int64_t c) { return ord_na(c) + ord_nc(c); }

// a group with at least one edge
ZK_DEV bool ord_grouped(int64_t c) {
  return (ord_naw(c) >= 1 && ord_na(c) >= 2) ||
         (ord_na(c) >= 1 && ord_nc(c) >= 1);
}

ZK_DEV int64_t ord_entry(const OrderWs& w, int64_t key) {
  int64_t sl = key & w.mask;
  for (int64_t probe = 0; probe <= w.mask; ++probe) {
    const int64_t k = (int64_t)atomicCAS((unsigned long long*)&w.key[sl],
                                         0ull, (unsigned long long)key);
    if (k == 0 || k == key) return sl;
    sl = (sl + 1) & w.mask;
  }
  return -1;
}

__global__ __launch_bounds__(TR_T) void ord_insert_k(
    const uint8_t* __restrict__ rx, ZkReqOut q,
    const int64_t* __restrict__ n_dev, int64_t ncap, OrderWs w) {
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (i >= ncap) return;
  int64_t ea = -1, ec = -1;
  if (i < *n_dev && q.status[i] == ST_OK && ord_has_path(q.opcode[i])) {
    const int32_t op = q.opcode[i];
    const uint8_t* p = rx + q.path_off[i];
    const int32_t pl = q.path_len[i];
    const bool wr = ord_writes(op);
    const bool seq = op == OP_CREATE && (q.arg[i] & CF_SEQUENTIAL);
    if (!seq) {
      ea = ord_entry(w, (int64_t)(path_hash(p, pl) | 1ull));
      if (ea >= 0) {
        atomicAdd((unsigned long long*)&w.cnt[ea],
                  1ull + (wr ? 1ull << ORD_F : 0ull));
        if (wr) atomicMax(&w.lastw[ea], (int32_t)i + 1);
      }
    }
    if (op == OP_CREATE || op == OP_DELETE) {
      int32_t cut = pl - 1;
      while (cut > 0 && p[cut] != '/') --cut;
      if (cut > 0) {                   // the root's children: no group
        ec = ord_entry(w, (int64_t)(path_hash(p, cut) | 1ull));
        if (ec >= 0) {
          atomicAdd((unsigned long long*)&w.cnt[ec], 1ull << (2 * ORD_F));
          atomicMax(&w.lastw[ec], (int32_t)i + 1);
        }
      }
    }
  }
  w.eidx[2 * i] = ea;
  w.eidx[2 * i + 1] = ec;
}

// member-list offsets: a block scan of the ordered groups' sizes per TR_T
// entries
__global__ __launch_bounds__(TR_T) void ord_base_k(OrderWs w) {
  __shared__ int64_t sm[TR_T / 64 + 1];
  const int64_t e = (int64_t)blockIdx.x * TR_T + threadIdx.x;  // h % TR_T == 0
  const int64_t cw = w.cnt[e];
  const int64_t c = ord_grouped(cw) ? ord_size(cw) : 0;
  int64_t tot;
  const int64_t x = block_excl_scan(c, sm, &tot);
  if (c) w.base[e] = (int32_t)x;
  if (threadIdx.x == 0) w.bsum[blockIdx.x] = tot;
}

// exclusive scan of the block totals in place (one block)
constexpr int ORD_SCAN_T = 1024;
__global__ __launch_bounds__(ORD_SCAN_T) void ord_bscan_k(int64_t* bsum,
                                                          int64_t nbh) {
  __shared__ int64_t sm[ORD_SCAN_T / 64 + 1];
  const int64_t per = (nbh + ORD_SCAN_T - 1) / ORD_SCAN_T;
  const int64_t b0 = (int64_t)threadIdx.x * per;
  const int64_t b1 = min(b0 + per, nbh);
  int64_t sum = 0;
  for (int64_t k = b0; k < b1; ++k) sum += bsum[k];
  int64_t tot;
  int64_t x = block_excl_scan(sum, sm, &tot);
  for (int64_t k = b0; k < b1; ++k) {
    const int64_t v = bsum[k];
    bsum[k] = x;
    x += v;
  }
}

ZK_DEV int32_t* ord_list(const OrderWs& w, int64_t e) {
  return w.members + w.bsum[e / TR_T] + w.base[e];
}

__global__ __launch_bounds__(TR_T) void ord_fill_k(int64_t ncap, OrderWs w) {
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (i >= ncap) return;
  w.rnk[i] = 0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int64_t e = w.eidx[2 * i + c];
    if (e < 0 || !ord_grouped(w.cnt[e])) continue;
    const int32_t pos = atomicAdd(&w.fill[e], 1);
    ord_list(w, e)[pos] = ((int32_t)i << 1) | c;
  }
}

// One relaxation round: rank[i] = 1 + the largest rank of an earlier
// request it has an edge to (in place: a rank never exceeds its chain).
__global__ __launch_bounds__(TR_T) void ord_relax_k(int64_t ncap, OrderWs w) {
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (i >= ncap) return;
  int32_t r = 0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int64_t e = w.eidx[2 * i + c];
    if (e < 0) continue;
    const int64_t cw = w.cnt[e];
    if (!ord_grouped(cw)) continue;
    const int64_t sz = ord_size(cw);
    if (sz > ORD_MAX_GROUP) { r = ORD_RANK; break; }   // refused wholesale
    const bool aw = ord_naw(cw) >= 1;
    const int32_t* m = ord_list(w, e);
    // earlier A members with an edge to i form a chain among themselves
    // (A-A edges need an A writer, and then every A pair has one), earlier
    // C members do not: their count + 1 is a lower bound of the rank that
    // makes a one-path group exact in the first round
    int32_t na = 0, anyc = 0;
    for (int64_t k = 0; k < sz; ++k) {
      const int32_t x = m[k];
      const int32_t j = x >> 1;
      if (j >= (int32_t)i) continue;
      const bool jc = x & 1;
      const bool edge = c == 0 ? (jc || aw) : !jc;
      if (!edge) continue;
      r = max(r, w.rnk[j] + 1);
      if (jc) anyc = 1;
      else ++na;
    }
    r = max(r, (c == 0 && aw ? na : min(na, 1)) + anyc);
  }
  w.rnk[i] = min(r, (int32_t)ORD_RANK);
}

__global__ __launch_bounds__(TR_T) void ord_rank_k(int64_t ncap, OrderWs w,
                                                   uint8_t* __restrict__ rank) {
  __shared__ int32_t smx[TR_T / 64];
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  int32_t r = 0;
  bool later_write = false;
  if (i < ncap) {
    r = w.rnk[i];
    // a read of the path whose own group is written later in the batch (by
    // a writer of the path or a child create / delete) snapshots its reply
    const int64_t e = w.eidx[2 * i];
    later_write = e >= 0 && ord_grouped(w.cnt[e]) &&
                  w.lastw[e] > (int32_t)i + 1;
    rank[i] = (uint8_t)(r | (later_write ? ORD_SNAP : 0));
  }
  // the batch's largest rank: one atomic per block
  int32_t mx = r;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
  if ((threadIdx.x & 63) == 0) smx[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < TR_T / 64; ++k) mx = max(mx, smx[k]);
    if (mx > 0) atomicMax((unsigned long long*)&w.ctr[1],
                          (unsigned long long)mx);
  }
}

// ---- SEQUENTIAL numbers in stream order (seq_*) ----------------------------
// A ZooKeeper leader names a SEQUENTIAL create once, from the parent's
// cversion when it prepares the txn, in zxid order; followers apply the
// name.  The serve applies a batch's creates concurrently, so a number
// taken from an atomic at create time follows wave scheduling: one
// session's pipelined creates came out in any order, and the members of a
// replicated tree, each re-executing the same batch, named them
// differently.  Here every SEQUENTIAL create of a batch is numbered
//     base(parent) + its rank among the batch's SEQUENTIAL creates under
//     that parent, in stream order,
// base being the parent's cversion before the batch, which then moves once
// by the group's size (a create that fails leaves a gap).  The numbers are
// a function of the batch and the tree before it: the same on every
// member and every run (reference: test/basic.test.js:550-611 names;
// test/multi-node.test.js:107-165 one tree behind every member).
//
// Five launches, no host read, O(n) work apart from a 1024-element LDS
// sort per chunk; a group is named by its slot e in a scratch hash of the
// parent paths (no dense ids: nothing waits for another workgroup):
//  1. seq_group_k, one 1024-request chunk per workgroup: parse, the parent
//     path's slot, the chunk's (slot, lane) pairs sorted in LDS (bitonic):
//     each request's rank in its chunk and group, each (group, chunk)
//     count, the group's chunk bit; a new group goes on the group list;
//  2. seq_alloc_k: per group, one count slot per chunk it appears in, and
//     the bitmap's per-word popcount prefix;
//  3. seq_index_k: per request, its chunk's index among its group's chunks
//     (chunk order = stream order); chunk leaders store their counts there;
//  4. seq_scan_k, a wave per group: exclusive scan of its chunk counts;
//     the parent looked up and bumped once; scratch left zero;
//  5. seq_out_k: number = base + chunk prefix + rank in the chunk.
// A group is keyed by the 64-bit hash of the parent path (a collision merges
// two parents' numbering: 2^-64 a pair).  A parent the pass does not find
// (created in the same batch) leaves its creates to the serve's atomic.
// (A first version gave groups dense ids, published by the claiming
// workgroup while the others spun on them: 134 us of the storm's 1M-create
// step in seq_group_k alone.)
constexpr int SQ_C = 1024;                 // requests per chunk (workgroup)
constexpr int64_t SQ_MAX = 1 << 24;        // requests a batch

struct SeqWs {
  int64_t* ctr;       // [8] groups, count slots used
  int64_t* key;       // [h] parent path hash | 1 (0 empty)
  uint64_t* mask;     // [h * mw] chunk bitmap per group slot
  uint16_t* pp;       // [h * mw] popcount of the bitmap words before
  int64_t* goff;      // [h] group -> its first count slot
  int32_t* gbase;     // [h] group -> parent cversion before the batch (-1)
  int32_t* gpar;      // [h] group -> its parent node
  int32_t* rep;       // [h] group -> one of its requests
  int32_t* glist;     // [ncap] the batch's group slots
  int32_t* cnts;      // [ncap] chunk counts, then their group prefixes
  int32_t* gid;       // [ncap] request -> group slot (-1)
  int32_t* rin;       // [ncap] request -> rank within its chunk and group
  int32_t* lcnt;      // [ncap] chunk leader -> its group's count there
  int32_t* kk;        // [ncap] request -> its chunk among its group's chunks
  int64_t hmask;
  int32_t mw;         // bitmap words per group (<= SQ_MW)
  int64_t* dbg;       // optional: 4 phase clocks per chunk (zk_tree_seq_debug)
};

// The parent path of a SEQUENTIAL create frame ([p, p + cut)); cut 0 for
// anything else (a root child has no parent node either).  Only what the
// numbering needs is read — the op, the path and the flags, the frame's
// last word — in three dependent loads, not the full parse's walk of the
// data and ACL (whose many dependent loads, a million frames in flight,
// re-fetched the stream's lines ~3x: 300 MB for an 83 MB batch).  A frame
// the serve's full parse then refuses is un-numbered there (tree_serve_k).
ZK_DEV int32_t seq_parent(const uint8_t* rx, int64_t off, int32_t len,
                          const uint8_t** p) {
  if (len < 28) return 0;            // xid op path(4) data(4) acl(4) flags
  const uint8_t* b = rx + off;
  uint32_t h[3];
  __builtin_memcpy(h, b, 12);
  const int32_t pl = (int32_t)bswap32(h[2]);
  if ((int32_t)bswap32(h[1]) != OP_CREATE || pl < 2 || 12 + pl + 12 > len)
    return 0;
  if (!(ld_be32(b + len - 4) & CF_SEQUENTIAL)) return 0;
  *p = b + 12;
  int32_t cut = pl - 1;
  while (cut > 0 && (*p)[cut] != '/') --cut;
  return cut;
}

// The group key (path_hash of the parent path | 1; 0: not a SEQUENTIAL
// create) of the create frame [b, b + len): the frame's first 64 bytes and
// its last word are loaded at once — one round trip after the frame table,
// not seq_parent's chain of a header load, the flags load, a byte load per
// step of the '/' search and the hash's own loads (the probe's clocks: 32
// us a chunk for those, tools/microbench/seq_probe.py) — and the op, the
// flags, the last '/' and the hash come from registers.  A path past the
// 64 bytes (pl > 52) or a frame under them takes seq_parent.
ZK_DEV uint64_t seq_key(const uint8_t* rx, int64_t off, int32_t len) {
  if (len < 64) {
    const uint8_t* p = nullptr;
    const int32_t cut = seq_parent(rx, off, len, &p);
    return cut > 0 ? path_hash(p, cut) | 1ull : 0;
  }
  const uint8_t* b = rx + off;
  uint32_t W[16], fl;
  __builtin_memcpy(W, b, 64);
  __builtin_memcpy(&fl, b + len - 4, 4);
  // (every load issued before the first test: the compiler otherwise sinks
  // the path words and the flags below the op test, one wait each)
  asm volatile("" ::"v"(W[0]), "v"(W[1]), "v"(W[2]), "v"(W[3]), "v"(W[4]),
               "v"(W[5]), "v"(W[6]), "v"(W[7]), "v"(W[8]), "v"(W[9]),
               "v"(W[10]), "v"(W[11]), "v"(W[12]), "v"(W[13]), "v"(W[14]),
               "v"(W[15]), "v"(fl));
  const int32_t pl = (int32_t)bswap32(W[2]);
  if ((int32_t)bswap32(W[1]) != OP_CREATE || pl < 2 || 12 + pl + 12 > len ||
      !(bswap32(fl) & CF_SEQUENTIAL))
    return 0;
  if (pl > 52) {
    const uint8_t* p = nullptr;
    const int32_t cut = seq_parent(rx, off, len, &p);
    return cut > 0 ? path_hash(p, cut) | 1ull : 0;
  }
  // '/' bytes of path positions 1 .. pl - 1 (path byte q: word 3 + q / 4)
  uint64_t slash = 0;
#pragma unroll
  for (int k = 3; k < 16; ++k) {
    const uint32_t x = W[k] ^ 0x2F2F2F2Fu;
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    const uint64_t nib = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) |
                         ((z >> 28) & 8u);
    slash |= nib << (4 * (k - 3));
  }
  slash &= ((1ull << pl) - 1) & ~1ull;
  if (!slash) return 0;
  const int32_t cut = 63 - __builtin_clzll(slash);
  // path_hash(path, cut) from the words: 8-byte pieces, the last masked
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)cut;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    if (8 * j < cut) {
      uint64_t x = (uint64_t)W[3 + 2 * j] | (uint64_t)W[4 + 2 * j] << 32;
      const int32_t left = cut - 8 * j;
      if (left < 8) x &= (1ull << (8 * left)) - 1;
      h = (h ^ x) * 0xFF51AFD7ED558CCDull;
      h ^= h >> 32;
    }
  }
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return h | 1ull;
}

// Within the chunk, each request's rank among the chunk's requests of its
// group (in lane = stream order) and each group's count, without a sort:
// the group slots get chunk-local dense ids through an LDS hash, a wave
// finds each lane's peers (same id) with one ballot per distinct id, and
// per-wave counts cnt[wave][id] in LDS give the count of the waves before.
// Four barriers; a bitonic sort of the chunk's 1024 (slot, lane) pairs
// took 75 barrier stages: 44 us a launch with nothing to sort, 145 us for
// the storm's 1M creates.
constexpr int SQ_W = SQ_C / 64;              // waves a chunk
constexpr int SQ_LH = 2 * SQ_C;              // LDS hash slots
__global__ __launch_bounds__(SQ_C) void seq_group_k(
    const uint8_t* __restrict__ rx, const int64_t* __restrict__ foff,
    const int32_t* __restrict__ flen, const int64_t* __restrict__ n_dev,
    int64_t ncap, SeqWs w) {
  __shared__ int32_t lkey[SQ_LH];            // group slot e (-1 empty)
  __shared__ int32_t lid[SQ_LH];             // its chunk-local dense id
  __shared__ uint16_t cnt[SQ_W][SQ_C];       // [wave][dense id] counts
  __shared__ int32_t ndense;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t c = blockIdx.x;
  const int64_t i = c * SQ_C + tid;
  int64_t* const dbg = w.dbg ? w.dbg + 5 * c : nullptr;
  if (dbg && tid == 0) dbg[0] = wall_clock64();
  // (the frame table and the count loaded together)
  const int64_t fo = i < ncap ? foff[i] : 0;
  const int32_t fn = i < ncap ? flen[i] : 0;
  const bool in = i < ncap && i < *n_dev;
  int64_t e = -1;
  bool first = false;
  const int64_t key = in ? (int64_t)seq_key(rx, fo, fn) : 0;
  if (dbg) {
    __syncthreads();
    if (tid == 0) dbg[4] = wall_clock64();
  }
  {
    if (key != 0) {
      int64_t s = key & w.hmask;
      for (int64_t probe = 0; probe <= w.hmask; ++probe) {
        // a plain load first (a stale 0 only means the CAS answers)
        int64_t k = w.key[s];
        if (k == 0)
          k = (int64_t)atomicCAS((unsigned long long*)&w.key[s], 0ull,
                                 (unsigned long long)key);
        if (k == 0) { first = true; e = s; break; }
        if (k == key) { e = s; break; }
        s = (s + 1) & w.hmask;
      }
    }
  }
  if (i < ncap) {
    w.lcnt[i] = 0;
    w.gid[i] = (int32_t)e;
  }
  // the group list: one ticket per new group, one atomic per workgroup
  const int64_t k = block_ticket<SQ_C>(&w.ctr[0], first);
  if (first) {
    w.glist[k] = (int32_t)e;
    w.rep[e] = (int32_t)i;
  }
  if (dbg && tid == 0) dbg[1] = wall_clock64();   // (after the ticket's barriers)
  if (!__syncthreads_or(e >= 0)) return;     // (block-uniform)
  // 1. chunk-local dense ids
  for (int x = tid; x < SQ_LH; x += SQ_C) lkey[x] = -1;
  for (int x = tid; x < SQ_C * SQ_W / 2; x += SQ_C)
    reinterpret_cast<uint32_t*>(&cnt[0][0])[x] = 0;   // (uint16 pairs)
  if (tid == 0) ndense = 0;
  __syncthreads();
  int ls = -1;
  if (e >= 0) {
    const int32_t ek = (int32_t)e;
    ls = (int)(((uint32_t)ek * 2654435761u) >> 21) & (SQ_LH - 1);
    for (;;) {
      const int32_t o = atomicCAS(&lkey[ls], -1, ek);
      if (o == -1) {
        lid[ls] = atomicAdd(&ndense, 1);
        break;
      }
      if (o == ek) break;
      ls = (ls + 1) & (SQ_LH - 1);
    }
  }
  __syncthreads();
  if (dbg && tid == 0) dbg[2] = wall_clock64();
  const int d = e >= 0 ? lid[ls] : -1;
  // 2. peers in the wave: one ballot per distinct id
  uint64_t peers = 0;
  uint64_t todo = __ballot(d >= 0);
  while (todo) {
    const int src = __ffsll((unsigned long long)todo) - 1;
    const int dk = __shfl(d, src, 64);
    const uint64_t m = __ballot(d == dk);
    if (d == dk) peers = m;
    todo &= ~m;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int rw = __popcll(peers & below);
  if (d >= 0 && rw == 0) cnt[wv][d] = (uint16_t)__popcll(peers);
  __syncthreads();
  // 3. the waves before, the chunk's count (its first request leads)
  if (d >= 0) {
    int pre = 0, tot = 0;
#pragma unroll
    for (int x = 0; x < SQ_W; ++x) {
      const int v = cnt[x][d];
      pre += x < wv ? v : 0;
      tot += v;
    }
    w.rin[i] = pre + rw;
    if (pre + rw == 0) {
      w.lcnt[i] = tot;
      atomicOr((unsigned long long*)&w.mask[e * w.mw + (c >> 6)],
               1ull << (c & 63));
    }
  }
  if (dbg) {
    __syncthreads();
    if (tid == 0) dbg[3] = wall_clock64();
  }
}

__global__ __launch_bounds__(TR_T) void seq_alloc_k(SeqWs w) {
  const int64_t ng = w.ctr[0];
  const int64_t stride = (int64_t)gridDim.x * TR_T;
  // (g0 is wave-uniform: wave_bytes needs the whole wave)
  for (int64_t g0 = (int64_t)blockIdx.x * TR_T + (threadIdx.x & ~63);
       g0 < ng; g0 += stride) {
    const int64_t g = g0 + (threadIdx.x & 63);
    const int64_t e = g < ng ? w.glist[g] : -1;
    int64_t n = 0;
    if (e >= 0) {
      const uint64_t* m = w.mask + e * w.mw;
      uint16_t* pp = w.pp + e * w.mw;
      for (int k = 0; k < w.mw; ++k) {
        pp[k] = (uint16_t)n;
        n += __popcll(m[k]);
      }
    }
    const int64_t o = wave_bytes(&w.ctr[1], n);
    if (e >= 0) w.goff[e] = o;
  }
}

__global__ __launch_bounds__(TR_T) void seq_index_k(int64_t ncap, SeqWs w) {
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (i >= ncap) return;
  const int64_t e = w.gid[i];
  if (e < 0) return;
  const int64_t c = i / SQ_C;
  const int64_t wd = e * w.mw + (c >> 6);
  const int32_t x = (int32_t)w.pp[wd] +
                    __popcll(w.mask[wd] & ((1ull << (c & 63)) - 1));
  w.kk[i] = x;
  const int32_t lc = w.lcnt[i];
  if (lc > 0) w.cnts[w.goff[e] + x] = lc;
}

__global__ __launch_bounds__(TR_T) void seq_scan_k(
    ZkTree t, const uint8_t* __restrict__ rx, const int64_t* __restrict__ foff,
    const int32_t* __restrict__ flen, SeqWs w) {
  const int lane = threadIdx.x & 63;
  const int64_t ng = w.ctr[0];
  const int64_t nwv = ((int64_t)gridDim.x * TR_T) >> 6;
  for (int64_t g = ((int64_t)blockIdx.x * TR_T + threadIdx.x) >> 6; g < ng;
       g += nwv) {
    const int64_t e = w.glist[g];
    uint64_t* m = w.mask + e * w.mw;
    int64_t n = 0;
    for (int k = lane; k < w.mw; k += 64) n += __popcll(m[k]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d, 64);
    const int64_t o = w.goff[e];
    int64_t run = 0;
    for (int64_t b = 0; b < n; b += 64) {
      const int64_t j = b + lane;
      const int64_t x = j < n ? w.cnts[o + j] : 0;
      const int64_t inc = wave_incl_scan(x);
      if (j < n) w.cnts[o + j] = (int32_t)(run + inc - x);
      run += __shfl(inc, 63, 64);
    }
    // the parent, found and bumped once for the whole group
    if (lane == 0) {
      int32_t base = -1;
      const int32_t r = w.rep[e];
      const uint8_t* p = nullptr;
      const int32_t cut = seq_parent(rx, foff[r], flen[r], &p);
      const int64_t par = cut > 0 ? tree_find(t, p, cut) : -1;
      // cversion and numChildren move by the group's size in one atomic
      // (the serve takes a failed create's child back)
      if (par >= 0 && t.eph[par] == 0)
        base = cn_cver(cn_add(t, par, (int32_t)run, (int32_t)run));
      w.gbase[e] = base;
      w.gpar[e] = (int32_t)par;
      w.key[e] = 0;
    }
    for (int k = lane; k < w.mw; k += 64) m[k] = 0;
  }
}

__global__ __launch_bounds__(TR_T) void seq_out_k(int64_t ncap, SeqWs w,
                                                  int64_t* __restrict__ seqno) {
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (i >= ncap) return;
  const int64_t e = w.gid[i];
  int64_t s = -1;
  if (e >= 0) {
    const int32_t b = w.gbase[e];
    const int32_t x = b >= 0 ? b + w.cnts[w.goff[e] + w.kk[i]] + w.rin[i] : -1;
    if (x >= 0) s = ((int64_t)w.gpar[e] << 32) | (uint32_t)x;
  }
  seqno[i] = s;
}

// ---- tree digest (tests / replica checks) ----------------------------------
// Sum over live nodes of a hash of (path, czxid, mzxid, version, cversion |
// numChildren, pzxid, ephemeralOwner, data): equal on two trees that hold
// the same znodes with the same Stat (times aside) and data, whatever node
// slots and hash entries they sit in.
ZK_DEV uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}

__global__ __launch_bounds__(TR_T) void tree_digest_k(
    ZkTree t, unsigned long long* __restrict__ out) {
  const int64_t v = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  const int64_t nn = min(t.counters[TC_NODES], t.store.cap);
  uint64_t h = 0, live = 0;
  if (v < nn && t.node_parent[v] != NODE_FREE) {
    const int64_t pw = t.node_pw[v];
    const uint8_t* slot = t.store.slab + t.store.slot_off[v];
    const int32_t dl = t.store.data_len[v];
    h = path_hash(node_path(t, pw), pw_len(pw));
    auto mix = [&](uint64_t x) {
      h = (h ^ x) * 0x9E3779B97F4A7C15ull;
      h ^= h >> 29;
    };
    mix((uint64_t)ld_be64(slot));                  // czxid
    mix((uint64_t)ld_be64(slot + 8));              // mzxid
    mix((uint32_t)ld_be32(slot + 32));             // version
    mix((uint64_t)t.cn[v]);
    mix((uint64_t)t.pzxid[v]);
    mix((uint64_t)t.eph[v]);
    mix((uint64_t)(uint32_t)dl);
    mix(path_hash(slot + ZK_SLOT_DATA, max(dl, 0)));
    live = 1;
  }
  h = wave_sum_u64(h);
  live = wave_sum_u64(live);
  if ((threadIdx.x & 63) == 0 && live) {
    atomicAdd(&out[0], (unsigned long long)h);
    atomicAdd(&out[1], (unsigned long long)live);
  }
}

__global__ __launch_bounds__(TR_T) void ht_census_k(
    ZkTree t, unsigned long long* __restrict__ out) {
  uint64_t used = 0, tomb = 0;
  for (int64_t s = (int64_t)blockIdx.x * TR_T + threadIdx.x; s <= t.mask;
       s += (int64_t)gridDim.x * TR_T) {
    if (*ht_key(t, s) != 0) {
      ++used;
      if (val_tomb(*ht_val(t, s))) ++tomb;
    }
  }
  used = wave_sum_u64(used);
  tomb = wave_sum_u64(tomb);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&out[2], (unsigned long long)used);
    atomicAdd(&out[3], (unsigned long long)tomb);
  }
}

// After a serve / expire launch, one kernel:
//  1. rewrite the wire-format Stat words of every dirty parent from the
//     shadows;
//  2. then (thread 0, after a barrier) publish: make the nodes freed by the
//     launch poppable, clamp a head that overshot the previously published
//     tail, reset the dirty list and consume the launch's zxids (`*n_dev`
//     for a batch of requests, 1 for a session expiry, which is one
//     closeSession txn).
constexpr int FIN_T = 1024;

// One workgroup: the dirty list holds the distinct parents a batch touched
// (a few thousand at most in practice), and a single block needs no
// cross-block sign-off — the grid version's atomic sign-off counter took
// 15-60 us per launch on a read-only GET batch, and two streams finishing
// at once could interleave on it.
// The finish (see above) by the calling workgroup (blockDim.x threads):
// tree_finish_k's launch, or the serve launch's last workgroup (serve_last).
// The counters and parent shadows other workgroups updated are read with
// agent-scope loads (this workgroup's L1 may hold older lines).
ZK_DEV void finish_body(const ZkTree& t, const int64_t* n_dev,
                        int64_t bump_zxid, int32_t publish) {
  int64_t* c = t.counters;
  const int64_t nd = __hip_atomic_load(&c[TC_DIRTY], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  for (int64_t k = threadIdx.x; k < nd; k += blockDim.x) {
    const int64_t p = __hip_atomic_load(&t.dirty_list[k], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    uint8_t* slot = t.store.slab + t.store.slot_off[p];
    const int64_t cn = __hip_atomic_load(&t.cn[p], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    st_be32(slot + 36, cn_cver(cn));
    st_be32(slot + 56, cn_nchild(cn));
    st_be64(slot + 60, __hip_atomic_load(&t.pzxid[p], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT));
    t.dirty[p] = 0;
  }
  __syncthreads();                 // every thread has read TC_DIRTY
  if (threadIdx.x != 0) return;
  auto ld = [&](int k) {
    return __hip_atomic_load(&c[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (publish) {
    if (ld(TC_FREE_HEAD) > ld(TC_FREE_PUB)) c[TC_FREE_HEAD] = ld(TC_FREE_PUB);
    c[TC_FREE_PUB] = ld(TC_FREE_TAIL);
  }
  c[TC_DIRTY] = 0;
  c[TC_ZXID] = ld(TC_ZXID) + (n_dev != nullptr ? *n_dev : bump_zxid);
}

template <int NT = FIN_T>
__global__ __launch_bounds__(NT) void tree_finish_k(ZkTree t,
                                                   const int64_t* n_dev,
                                                   int64_t bump_zxid,
                                                   int32_t publish) {
  finish_body(t, n_dev, bump_zxid, publish);
}

// The between-batch finish and the reply encoder's block-sum scan in ONE
// launch of two workgroups: they are independent one-workgroup jobs that
// ran back to back on the connection's stream (tree_finish_k, then K13's
// scan_one_block), each waiting for a CU behind the other connection's
// kernels.  Workgroup 1 scans the serve's per-256-reply size sums (bsum,
// nb of them) into the encoder's block bases and writes the stream total
// (zk_encode_responses3 `prescanned`).
// MFMA: workgroup 1 scans on the matrix cores (zk_mfma_scan.h: 2048 block
// sums of a 512K-reply connection are one 4096-value chunk of four waves).
template <int NT, bool MFMA>
__global__ __launch_bounds__(NT) void tree_finish_scan_k(
    ZkTree t, const int64_t* n_dev, int64_t bump_zxid, int32_t publish,
    const int64_t* __restrict__ bsum, int64_t nb, int64_t* __restrict__ bbase,
    int64_t* __restrict__ total) {
  if (blockIdx.x == 0) {
    finish_body(t, n_dev, bump_zxid, publish);
    return;
  }
  if (MFMA) {
    __shared__ int64_t wsum[NT / 64 + 1];
    const int64_t tot = mfma_scan_block_direct<NT>(bsum, nb, bbase, wsum);
    if (threadIdx.x == 0) *total = tot;
    return;
  }
  // a thread owns FS_V consecutive sums, so a 512K-reply connection's 2048
  // are one block scan (one value a thread per chunk took eight: 9.9 us
  // against scan_one_block's 4.2, profiles/r6_get_pmc.md)
  constexpr int FS_V = 8;
  __shared__ int64_t sm[NT / 64 + 1];
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < nb; c0 += (int64_t)NT * FS_V) {   // (uniform)
    const int64_t b = c0 + (int64_t)threadIdx.x * FS_V;
    int64_t v[FS_V];
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < FS_V; ++j) {
      v[j] = b + j < nb ? bsum[b + j] : 0;
      s += v[j];
    }
    int64_t tot;
    int64_t p = carry + block_excl_scan(s, sm, &tot);
#pragma unroll
    for (int j = 0; j < FS_V; ++j) {
      if (b + j < nb) bbase[b + j] = p;
      p += v[j];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

// Is this the serve launch's last workgroup to finish?  Tickets in groups
// of 64 workgroups (tickets[1 + g]; the last of a group takes one of
// tickets[0]), so no counter takes more than 64 atomics — one counter
// for a whole grid (thousands of same-address atomics) took 15-60 us a
// launch.  The counters are the caller's (one set per server: two
// connections serving one tree at once keep apart) and are left zero.
ZK_DEV bool serve_last(unsigned* tickets) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned ng = (gridDim.x + 63) / 64;
    const unsigned g = blockIdx.x / 64;
    const unsigned gs = min(64u, gridDim.x - g * 64);
    int last = 0;
    if (atomicAdd(&tickets[1 + g], 1u) + 1 == gs) {
      __hip_atomic_store(&tickets[1 + g], 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
      if (atomicAdd(&tickets[0], 1u) + 1 == ng) {
        __hip_atomic_store(&tickets[0], 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
    __threadfence();
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

// Session expiry: remove every ephemeral node owned by `session`
// (lib/zk-session.js expiry; the server side deletes the session's
// ephemerals as ONE closeSession txn: all removals share zxid + 1).  One
// pass over the node table; `removed` counts deletions.
// DBG: phase clocks into dbg (zk_tree_expire_debug), 100 MHz ticks — an
// instance of its own: the clock reads in the plain kernel, even behind a
// null test, took the expiry from ~0.45 to ~1 ms.
template <bool DBG>
__global__ __launch_bounds__(TR_T) void tree_expire_k(
    ZkTree t, int64_t session, int64_t ncap,
    unsigned long long* __restrict__ removed, int32_t* __restrict__ dbg) {
  session = sess_of(t, session);
  const int64_t v = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  const int64_t c0 = DBG ? (int64_t)wall_clock64() : 0;
  int64_t c1 = 0, c2 = 0;
  // the owner from the contiguous shadow (a node's slab line per node was
  // 256 MB of random reads over a 4M-node tree, 335 us an expiry); a
  // freed node's shadow is 0.  The slab's ephemeralOwner of a freed node is
  // left as it was: nothing reads a freed slot, and the create that reuses
  // it writes the whole Stat (fill_stat) — zeroing it was one random slab
  // line written back per removal (256 MB an expiry of 2M nodes)
  bool hit = v < ncap && v < t.counters[TC_NODES] && t.eph[v] == session;
  const int64_t zx = t.counters[TC_ZXID] + 1;
  int64_t par = -1;
  int32_t dflag = 1;
  if (hit) {
    // what the removal reads of node v, at once: its path, its parent and
    // the parent's dirty flag (their round trips ride under the probe's:
    // the thread is a chain of dependent trips to memory; pairing the
    // probe's loads took the storm step 1.298 -> 1.262 ms, these measured
    // within noise)
    const int64_t poff = t.node_path_off[v];
    const int32_t plen = t.node_path_len[v];
    const int64_t p0 = t.node_parent[v];
    if (p0 >= 0)
      dflag = __hip_atomic_load(&t.dirty[p0], __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    const int64_t tag = tomb_tag(zx);
    const int64_t es = tree_erase_slot(t, v, t.path_arena + poff, plen, tag);
    hit = es >= 0;
    if (DBG) c1 = (int64_t)wall_clock64();
    if (hit) {
      ht_shift(t, es, session, tag);
      if (DBG) c2 = (int64_t)wall_clock64();
      par = p0;
      if (par >= 0) parent_touch(t, par, -1, true, zx);
      t.eph[v] = 0;
    }
  }
  // the frees' ticket also counts `removed` (no second block round)
  wave_free(t, hit ? v : -1, removed);
  wave_mark_dirty_at(t, par, dflag);
  if (DBG && hit) {
    // start (low word), lookup + tombstone, backward shift, whole thread
    const int64_t c3 = (int64_t)wall_clock64();
    dbg[4 * v] = (int32_t)c0;
    dbg[4 * v + 1] = (int32_t)(c1 - c0);
    dbg[4 * v + 2] = (int32_t)(c2 - c1);
    dbg[4 * v + 3] = (int32_t)(c3 - c0);
  }
}

// ---- watch event expansion ------------------------------------------------
// Notifications of a served batch, in request order (ZooKeeper delivers a
// session's notifications in zxid order; write i of a batch has zxid base +
// i + 1): request i contributes one event per watcher bit of the masks it
// fired — m_path (type by op), m_path_child (NodeDeleted, a watcher holding
// both a data and a child watch on a deleted path is told once), m_parent
// (NodeChildrenChanged on the parent).  Three launches: counts + block
// sums, one-block scan of the sums, write.
ZK_DEV bool wt_live(const int32_t* r_op, const int32_t* r_err, int64_t i) {
  const int32_t op = r_op[i];
  return r_err[i] == ERR_OK &&
         (op == OP_SET_DATA || op == OP_CREATE || op == OP_DELETE);
}

ZK_DEV int64_t wt_count(const int32_t* r_op, const int32_t* r_err,
                        const int64_t* fired, int64_t i, bool in) {
  if (!in || !wt_live(r_op, r_err, i)) return 0;
  const int64_t* f = fired + (int64_t)WT_REC * i;
  return __popcll((uint64_t)f[0]) + __popcll((uint64_t)f[1]) +
         __popcll((uint64_t)f[2]);
}

__global__ __launch_bounds__(TR_T) void wt_count_k(
    const int32_t* __restrict__ r_op, const int32_t* __restrict__ r_err,
    const int64_t* __restrict__ n_dev, int64_t ncap,
    const int64_t* __restrict__ fired, int64_t* __restrict__ bsum) {
  __shared__ int64_t sm[TR_T / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  const bool in = i < ncap && i < *n_dev;
  int64_t tot;
  block_excl_scan(wt_count(r_op, r_err, fired, i, in), sm, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

ZK_DEV void wt_emit(uint64_t m, int32_t type, int64_t pw, int64_t& o,
                    int64_t cap, int32_t* ev_slot, int32_t* ev_type,
                    int64_t* ev_poff, int32_t* ev_plen) {
  while (m) {
    const int b = __builtin_ctzll(m);
    m &= m - 1;
    if (o < cap) {
      ev_slot[o] = b;
      ev_type[o] = type;
      ev_poff[o] = pw >> 24;
      ev_plen[o] = pw_len(pw);
    }
    ++o;
  }
}

__global__ __launch_bounds__(TR_T) void wt_expand_k(
    const int32_t* __restrict__ r_op, const int32_t* __restrict__ r_err,
    const int64_t* __restrict__ n_dev, int64_t ncap,
    const int64_t* __restrict__ fired, const int64_t* __restrict__ bsum,
    int64_t nb, int64_t cap, int32_t* __restrict__ ev_slot,
    int32_t* __restrict__ ev_type, int64_t* __restrict__ ev_poff,
    int32_t* __restrict__ ev_plen, int64_t* __restrict__ ev_total) {
  __shared__ int64_t sm[TR_T / 64 + 1];
  const int64_t i = (int64_t)blockIdx.x * TR_T + threadIdx.x;
  const bool in = i < ncap && i < *n_dev;
  const int64_t c = wt_count(r_op, r_err, fired, i, in);
  int64_t tot;
  int64_t o = bsum[blockIdx.x] + block_excl_scan(c, sm, &tot);
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) {
    const int64_t all = bsum[blockIdx.x] + tot;
    ev_total[0] = min(all, cap);     // events written (the encoder's count)
    ev_total[1] = all;               // events fired (> [0]: overflow)
  }
  if (c == 0) return;
  const int64_t* f = fired + (int64_t)WT_REC * i;
  const int32_t op = r_op[i];
  const int32_t t0 = op == OP_SET_DATA ? NT_DATA_CHANGED
                   : op == OP_CREATE ? NT_CREATED : NT_DELETED;
  wt_emit((uint64_t)f[0], t0, f[3], o, cap, ev_slot, ev_type, ev_poff,
          ev_plen);
  wt_emit((uint64_t)f[1], NT_DELETED, f[3], o, cap, ev_slot, ev_type,
          ev_poff, ev_plen);
  wt_emit((uint64_t)f[2], NT_CHILDREN_CHANGED, f[4], o, cap, ev_slot,
          ev_type, ev_poff, ev_plen);
}

// ---- SET_WATCHES catch-up (one workgroup) ---------------------------------
// A resumed session re-sends its watches with relZxid = the last zxid it saw
// (lib/zk-session.js:421-471, lib/zk-buffer.js:255-273).  For every path
// (SURVEY Appendix D): data watch — node gone: NodeDeleted, mzxid > rel:
// NodeDataChanged, else re-armed; exist watch — node there: NodeCreated,
// else re-armed; child watch — node gone: NodeDeleted, pzxid > rel:
// NodeChildrenChanged, else re-armed.  Events name the request's path
// bytes (offsets into rx), in request order (data, exist, child lists).
constexpr int WR_T = 1024;

__global__ __launch_bounds__(WR_T) void wt_resume_k(
    ZkTree t, const uint8_t* __restrict__ rx,
    const int64_t* __restrict__ foff, const int32_t* __restrict__ flen,
    const int64_t* __restrict__ n_dev, int64_t ncap, int32_t wslot,
    int64_t* __restrict__ ent, int64_t ent_cap, int64_t cap,
    int32_t* __restrict__ ev_type, int64_t* __restrict__ ev_poff,
    int32_t* __restrict__ ev_plen, int64_t* __restrict__ out) {
  __shared__ int64_t sm[WR_T / 64 + 1];
  __shared__ int64_t s_n, s_rel;
  int64_t o = 0, rearmed = 0;
  const int64_t nfr = min(*n_dev, ncap);
  for (int64_t fr = 0; fr < nfr; ++fr) {
    // thread 0 lists the frame's paths (kind << 62 | off << 24 | len);
    // a frame that is not a well-formed SET_WATCHES lists none
    if (threadIdx.x == 0) {
      const ReqFields rq = parse_request(rx, foff[fr], flen[fr]);
      int64_t m = 0;
      if (rq.status == ST_OK && rq.op == OP_SET_WATCHES) {
        int64_t k = rq.voff;
        for (int g = 0; g < 3; ++g) {
          const int32_t c = max(ld_be32(rx + k), 0);
          k += 4;
          for (int32_t j = 0; j < c; ++j) {
            const int32_t l = max(ld_be32(rx + k), 0);
            if (m < ent_cap)
              ent[m] = ((int64_t)g << 62) | ((k + 4) << 24) | l;
            ++m;
            k += 4 + l;
          }
        }
      }
      s_n = min(m, ent_cap);
      s_rel = rq.rel;
    }
    __syncthreads();
    const int64_t n = s_n, rel = s_rel;
    for (int64_t b = 0; b < n; b += WR_T) {
      const int64_t j = b + threadIdx.x;
      int32_t type = 0;
      int64_t po = 0;
      int32_t pl = 0;
      if (j < n) {
        const int64_t e = ent[j];
        const int g = (int)((uint64_t)e >> 62);
        po = (e >> 24) & ((1ll << 38) - 1);
        pl = (int32_t)(e & 0xFFFFFF);
        const uint8_t* p = rx + po;
        const Found f = tree_lookup(t, p, pl);
        if (g == 0) {                              // data watch
          if (f.node < 0) type = NT_DELETED;
          else if (ld_be64(t.store.slab + f.slot + 8) > rel)
            type = NT_DATA_CHANGED;
        } else if (g == 1) {                       // exist watch
          if (f.node >= 0) type = NT_CREATED;
        } else {                                   // child watch
          if (f.node < 0) type = NT_DELETED;
          else if (t.pzxid[f.node] > rel) type = NT_CHILDREN_CHANGED;
        }
        if (type == 0) {
          wt_arm(t, p, pl, g == 2 ? WK_CHILD : WK_DATA, wslot);
          ++rearmed;
        }
      }
      int64_t tot;
      const int64_t x = o + block_excl_scan(type != 0 ? 1 : 0, sm, &tot);
      if (type != 0 && x < cap) {
        ev_type[x] = type;
        ev_poff[x] = po;
        ev_plen[x] = pl;
      }
      o += tot;
    }
    __syncthreads();
  }
  int64_t tot;
  block_excl_scan(rearmed, sm, &tot);
  if (threadIdx.x == 0) {
    out[0] = min(o, cap);        // events written
    out[1] = tot;                // watches re-armed
    out[2] = o;                  // events (> out[0]: overflow)
  }
}

}  // namespace zk

extern "C" {

int zk_tree_fill(const ZkTree* t, int64_t n0, int64_t n, const int32_t* nkids,
                 int64_t now_ms, hipStream_t st) {
  if (n <= n0) return 0;
  const int64_t m = n - n0;
  zk::tree_fill_k<<<(unsigned)((m + zk::TR_T - 1) / zk::TR_T), zk::TR_T, 0,
                    st>>>(*t, n0, n, nkids, now_ms);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Workspace (int64) of zk_tree_free_compact for a node capacity.
int64_t zk_tree_free_workspace(int64_t cap) {
  const int64_t nb = (cap + zk::TR_T - 1) / zk::TR_T;
  return 2 * nb + 8 + zk_scan_workspace(nb);
}

// The free ring's pending entries rebuilt in node order (free_count_k).
int zk_tree_free_compact(const ZkTree* t, int64_t* ws, hipStream_t st) {
  const int64_t nb = (t->store.cap + zk::TR_T - 1) / zk::TR_T;
  if (nb <= 0) return 0;
  int64_t* bsum = ws;
  int64_t* bbase = ws + nb;
  int64_t* total = ws + 2 * nb;
  zk::free_count_k<<<(unsigned)nb, zk::TR_T, 0, st>>>(*t, bsum);
  ZK_LAUNCH_CHECK();
  int rc = zk_scan_excl_i64(bsum, bbase, nb, total, ws + 2 * nb + 8, st);
  if (rc) return rc;
  zk::free_scatter_k<<<(unsigned)nb, zk::TR_T, 0, st>>>(*t, bbase, total);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Every hash entry back to empty: all zero bytes (val_pack), one memset.
// (Round 5's first reset wrote {0, -3, 0...} entries from a kernel: 2.2 ms
// for the storm's 4 GB table.)
int zk_tree_ht_reset(const ZkTree* t, hipStream_t st) {
  return hipMemsetAsync(t->ht, 0, (size_t)(t->mask + 1) * zk::HT_W * 8, st);
}

int zk_tree_build(const ZkTree* t, int64_t n0, int64_t n, hipStream_t st) {
  if (n <= n0) return 0;
  const int64_t m = n - n0;
  zk::tree_build_k<<<(unsigned)((m + zk::TR_T - 1) / zk::TR_T), zk::TR_T, 0,
                     st>>>(*t, n0, n);
  ZK_LAUNCH_CHECK();
  return 0;
}

static int finish_launch(const ZkTree* t, int64_t ncap, const int64_t* n_dev,
                         int64_t bump_zxid, hipStream_t st,
                         int32_t publish = 1) {
  (void)ncap;
  // (256 threads: the workgroup finds a CU sooner behind another stream's
  // kernel than 1024 did, and the dirty list is a few thousand entries)
  zk::tree_finish_k<256><<<1, 256, 0, st>>>(*t, n_dev, bump_zxid, publish);
  ZK_LAUNCH_CHECK();
  return 0;
}

// r_slot / r_sizes / r_bsum may be null (see tree_serve_k); r_bsum needs
// ceil(ncap / 256) entries.
int zk_tree_serve(const ZkTree* t, const uint8_t* rx, const ZkReqOut* q,
                  const int64_t* n_dev, int64_t ncap, int32_t* r_op,
                  int32_t* r_xid, int32_t* r_err, int64_t* r_node,
                  int64_t* r_zxid, int64_t* r_path_off, int32_t* r_path_len,
                  int64_t* r_slot, int64_t* r_sizes, int64_t* r_bsum,
                  int64_t session, int64_t now_ms, hipStream_t st) {
  if (ncap <= 0) return 0;
  if ((r_sizes == nullptr) != (r_bsum == nullptr)) return -1;
  zk::tree_serve_k<false><<<(unsigned)((ncap + zk::TR_T - 1) / zk::TR_T),
                            zk::TR_T, 0, st>>>(
      *t, rx, *q, nullptr, nullptr, n_dev, ncap, r_op, r_xid, r_err, r_node,
      r_zxid, r_path_off, r_path_len, r_slot, r_sizes, r_bsum, session,
      now_ms, nullptr, 0, 1, 0, 0, nullptr, -1, nullptr, nullptr);
  ZK_LAUNCH_CHECK();
  // at most one dirty parent per request
  return finish_launch(t, ncap, n_dev, 0, st);
}

// zk_tree_serve straight from K1's frame table (foff / flen, *n_dev
// frames): every lane parses its request in registers (no K12 pass).
// tickets (may be null; zk_serve_tickets(ncap) zeroed uint32, kept per
// server): the launch's last workgroup does the finish (serve_last), no
// tree_finish_k launch.
// wslot: this session's watcher slot (-1: its reads arm no watch); fired
// (may be null; [ncap * 5]): per successful write, the watcher masks it
// fired and the paths (zk_watch_events expands them).
int64_t zk_serve_tickets(int64_t ncap) {
  const int64_t nb = (ncap + zk::TR_T - 1) / zk::TR_T;
  return 1 + (nb + 63) / 64;
}

// finish: ZK_SERVE_FINISH (else no finish at all: the caller launches
// zk_tree_finish or zk_tree_finish_scan) | ZK_SERVE_RO (a batch of GET_DATA
// / EXISTS only: tree_serve_k's RO instance)
int zk_tree_serve_frames2(const ZkTree* t, const uint8_t* rx,
                          const int64_t* foff, const int32_t* flen,
                          const int64_t* n_dev, int64_t ncap, int32_t* r_op,
                          int32_t* r_xid, int32_t* r_err, int64_t* r_node,
                          int64_t* r_zxid, int64_t* r_path_off,
                          int32_t* r_path_len, int64_t* r_slot,
                          int64_t* r_sizes, int64_t* r_bsum, int64_t session,
                          int64_t now_ms, int32_t wslot, int64_t* fired,
                          unsigned* tickets, int32_t finish, hipStream_t st) {
  if (ncap <= 0) return 0;
  if ((r_sizes == nullptr) != (r_bsum == nullptr)) return -1;
  ZkReqOut none{};
  const unsigned nb = (unsigned)((ncap + zk::TR_T - 1) / zk::TR_T);
  if (finish & ZK_SERVE_RO)
    zk::tree_serve_k<true, true><<<nb, zk::TR_T, 0, st>>>(
        *t, rx, none, foff, flen, n_dev, ncap, r_op, r_xid, r_err, r_node,
        r_zxid, r_path_off, r_path_len, r_slot, r_sizes, r_bsum, session,
        now_ms, nullptr, 0, 1, 0, 0, nullptr, wslot, fired, tickets);
  else
    zk::tree_serve_k<true><<<nb, zk::TR_T, 0, st>>>(
        *t, rx, none, foff, flen, n_dev, ncap, r_op, r_xid, r_err, r_node,
        r_zxid, r_path_off, r_path_len, r_slot, r_sizes, r_bsum, session,
        now_ms, nullptr, 0, 1, 0, 0, nullptr, wslot, fired, tickets);
  ZK_LAUNCH_CHECK();
  // tickets: the serve launch's last workgroup did the finish
  return tickets != nullptr || !(finish & ZK_SERVE_FINISH)
             ? 0
             : finish_launch(t, ncap, n_dev, 0, st);
}

int zk_tree_serve_frames(const ZkTree* t, const uint8_t* rx,
                         const int64_t* foff, const int32_t* flen,
                         const int64_t* n_dev, int64_t ncap, int32_t* r_op,
                         int32_t* r_xid, int32_t* r_err, int64_t* r_node,
                         int64_t* r_zxid, int64_t* r_path_off,
                         int32_t* r_path_len, int64_t* r_slot,
                         int64_t* r_sizes, int64_t* r_bsum, int64_t session,
                         int64_t now_ms, int32_t wslot, int64_t* fired,
                         unsigned* tickets, hipStream_t st) {
  return zk_tree_serve_frames2(t, rx, foff, flen, n_dev, ncap, r_op, r_xid,
                               r_err, r_node, r_zxid, r_path_off, r_path_len,
                               r_slot, r_sizes, r_bsum, session, now_ms, wslot,
                               fired, tickets, ZK_SERVE_FINISH, st);
}

// The between-batch finish of a serve (parent Stat fix-up, free-ring
// publish, zxid += *n_dev or bump) on its own: the partner of
// zk_tree_serve_frames2(..., finish = 0).
int zk_tree_finish(const ZkTree* t, const int64_t* n_dev, int64_t bump,
                   int32_t publish, hipStream_t st) {
  return finish_launch(t, 0, n_dev, bump, st, publish);
}

// zk_tree_finish + the presized reply encode's block-sum scan (the serve's
// r_bsum for ncap replies, in scan_ws[0, nb)) -> scan_ws[nb, 2 nb) and
// *total, in one launch (tree_finish_scan_k).
int zk_tree_finish_scan(const ZkTree* t, const int64_t* n_dev, int64_t bump,
                        int32_t publish, int64_t ncap, int64_t* scan_ws,
                        int64_t* total, hipStream_t st) {
  const int64_t nb = ncap > 0 ? (ncap + 255) / 256 : 0;
  if (zk_scan_small_mode() == 1)
    zk::tree_finish_scan_k<256, true><<<2, 256, 0, st>>>(
        *t, n_dev, bump, publish, scan_ws, nb, scan_ws + nb, total);
  else
    zk::tree_finish_scan_k<256, false><<<2, 256, 0, st>>>(
        *t, n_dev, bump, publish, scan_ws, nb, scan_ws + nb, total);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Ordering workspace layout for up to ncap requests: the zeroed prefix
// (counters, key, cw, fill, lastw), then base, bsum, eidx, members, rank.
static int64_t order_hcap(int64_t ncap) {
  int64_t h = 1024;
  while (h < 2 * ncap) h <<= 1;
  return h;
}

static int64_t order_layout(int64_t ncap, uint8_t* ws, zk::OrderWs* w,
                            uint8_t** rank, int64_t* zeroed) {
  const int64_t h = order_hcap(ncap);
  int64_t o = 32;
  if (w != nullptr) {
    w->ctr = (int64_t*)ws;
    w->key = (int64_t*)(ws + o);
  }
  o += h * 8;
  if (w != nullptr) w->cnt = (int64_t*)(ws + o);
  o += h * 8;
  if (w != nullptr) w->fill = (int32_t*)(ws + o);
  o += h * 4;
  if (w != nullptr) w->lastw = (int32_t*)(ws + o);
  o += h * 4;
  if (zeroed != nullptr) *zeroed = o;
  if (w != nullptr) w->base = (int32_t*)(ws + o);
  o += h * 4;
  if (w != nullptr) w->bsum = (int64_t*)(ws + o);
  o += (h / zk::TR_T) * 8;
  if (w != nullptr) w->eidx = (int64_t*)(ws + o);
  o += 2 * ncap * 8;
  if (w != nullptr) w->members = (int32_t*)(ws + o);
  o += 2 * ncap * 4;
  if (w != nullptr) w->rnk = (int32_t*)(ws + o);
  o += ncap * 4;
  if (rank != nullptr) *rank = ws + o;
  o += ncap;
  if (w != nullptr) w->mask = h - 1;
  return o;
}

// Bytes of the ordering workspace for up to ncap requests.
int64_t zk_tree_order_workspace(int64_t ncap) {
  return order_layout(ncap, nullptr, nullptr, nullptr, nullptr);
}

// zk_tree_serve with the batch applied in path order: rank every request
// (tree_order_*), then `passes` serve launches of increasing rank (each
// followed by the parent fix-up; the free nodes are published and the
// batch's zxids consumed by the last).  A request of rank >= passes is
// answered SYSTEMERROR and shows in the max rank (zk_tree_order_stats_offset;
// the caller can read it and use more passes).  The launches do not depend
// on the ranks: no host read.
int zk_tree_serve_ordered(const ZkTree* t, const uint8_t* rx, const ZkReqOut* q,
                          const int64_t* n_dev, int64_t ncap, int32_t* r_op,
                          int32_t* r_xid, int32_t* r_err, int64_t* r_node,
                          int64_t* r_zxid, int64_t* r_path_off,
                          int32_t* r_path_len, int64_t* r_slot,
                          int64_t* r_sizes, int64_t* r_bsum, int64_t session,
                          int64_t now_ms, uint8_t* ws, int64_t ws_bytes,
                          int32_t passes, int64_t snap_base, int64_t snap_cap,
                          int32_t wslot, int64_t* fired, hipStream_t st) {
  if (ncap <= 0) return 0;
  if (ncap > zk::ORD_FM) return -1;          // packed group counts
  if ((r_sizes == nullptr) != (r_bsum == nullptr)) return -1;
  if (passes < 1 || passes > zk::ORD_RANK) return -1;
  if (snap_base < 0 || snap_cap < 0 || (snap_base & 15)) return -1;
  if (ws_bytes < zk_tree_order_workspace(ncap)) return -1;
  if (((uintptr_t)ws & 15) != 0) return -1;
  zk::OrderWs w;
  uint8_t* rank = nullptr;
  int64_t zeroed = 0;
  order_layout(ncap, ws, &w, &rank, &zeroed);
  const int64_t h = w.mask + 1;
  if (hipMemsetAsync(ws, 0, (size_t)zeroed, st) != hipSuccess) return -4;
  const unsigned nb = (unsigned)((ncap + zk::TR_T - 1) / zk::TR_T);
  zk::ord_insert_k<<<nb, zk::TR_T, 0, st>>>(rx, *q, n_dev, ncap, w);
  ZK_LAUNCH_CHECK();
  zk::ord_base_k<<<(unsigned)(h / zk::TR_T), zk::TR_T, 0, st>>>(w);
  ZK_LAUNCH_CHECK();
  zk::ord_bscan_k<<<1, zk::ORD_SCAN_T, 0, st>>>(w.bsum, h / zk::TR_T);
  ZK_LAUNCH_CHECK();
  zk::ord_fill_k<<<nb, zk::TR_T, 0, st>>>(ncap, w);
  ZK_LAUNCH_CHECK();
  // ranks of chains up to `passes` long are exact after passes + 1 rounds
  // (a longer chain ends at rank >= passes: refused either way)
  for (int32_t r = 0; r <= passes; ++r) {
    zk::ord_relax_k<<<nb, zk::TR_T, 0, st>>>(ncap, w);
    ZK_LAUNCH_CHECK();
  }
  zk::ord_rank_k<<<nb, zk::TR_T, 0, st>>>(ncap, w, rank);
  ZK_LAUNCH_CHECK();
  for (int32_t pass = 0; pass < passes; ++pass) {
    const int32_t last = pass == passes - 1;
    zk::tree_serve_k<false><<<nb, zk::TR_T, 0, st>>>(
        *t, rx, *q, nullptr, nullptr, n_dev, ncap, r_op, r_xid, r_err, r_node, r_zxid,
        r_path_off, r_path_len, r_slot, r_sizes, r_bsum, session, now_ms,
        rank, pass, last, snap_base, snap_cap, &w.ctr[2], wslot, fired,
        nullptr);
    ZK_LAUNCH_CHECK();
    // nodes freed by a pass are recycled from the next batch on: a reply of
    // this batch may still name them
    const int rc = finish_launch(t, ncap, last ? n_dev : nullptr, 0, st,
                                 last);
    if (rc) return rc;
  }
  return 0;
}

// Byte offset in the ordering workspace of {max rank, scratch bytes used}
// of the last ordered serve (int64 each; read them after the stream).
int64_t zk_tree_order_stats_offset(int64_t ncap) {
  (void)ncap;
  return 8;
}

// Workspace of zk_tree_seq_order: the prefix that must start zeroed (and is
// left zeroed: hash keys, published ids, chunk bitmaps), then the counters
// (reset every call) and the per-group / per-request arrays.
static int64_t seq_layout(int64_t ncap, uint8_t* ws, zk::SeqWs* w,
                          int64_t* zeroed) {
  int64_t h = 1024;
  while (h < 2 * ncap) h <<= 1;
  const int64_t nch = (ncap + zk::SQ_C - 1) / zk::SQ_C;
  const int32_t mw = (int32_t)((nch + 63) / 64 > 0 ? (nch + 63) / 64 : 1);
  auto at = [&](int64_t o) { return ws != nullptr ? ws + o : nullptr; };
  auto a16 = [](int64_t x) { return (x + 15) & ~(int64_t)15; };
  int64_t o = 0;
  if (w != nullptr) {
    w->hmask = h - 1;
    w->mw = mw;
    w->key = (int64_t*)at(o);
  }
  o += h * 8;
  if (w != nullptr) w->mask = (uint64_t*)at(o);
  o += h * mw * 8;
  if (zeroed != nullptr) *zeroed = o;
  if (w != nullptr) w->ctr = (int64_t*)at(o);
  o += 64;
  if (w != nullptr) w->pp = (uint16_t*)at(o);
  o += a16(h * mw * 2);
  if (w != nullptr) w->goff = (int64_t*)at(o);
  o += h * 8;
  if (w != nullptr) w->gbase = (int32_t*)at(o);
  o += h * 4;
  if (w != nullptr) w->rep = (int32_t*)at(o);
  o += h * 4;
  if (w != nullptr) w->gpar = (int32_t*)at(o);
  o += h * 4;
  int32_t** arr[] = {w ? &w->glist : nullptr, w ? &w->cnts : nullptr,
                     w ? &w->gid : nullptr,   w ? &w->rin : nullptr,
                     w ? &w->lcnt : nullptr,  w ? &w->kk : nullptr};
  for (int32_t** p : arr) {
    if (p != nullptr) *p = (int32_t*)at(o);
    o += a16(ncap * 4);
  }
  return o;
}

// Phase clocks of seq_group_k (tools/microbench/seq_probe.py): buf holds
// 5 int64 per 1024-request chunk — start, the key table probe and group
// ticket done, chunk-local ids done, end, and (an extra barrier) the parse
// done (wall_clock64 ticks, 100 MHz); nullptr turns them off.
static int64_t* g_seq_dbg = nullptr;
void zk_tree_seq_debug(int64_t* buf) { g_seq_dbg = buf; }

int64_t zk_tree_seq_workspace(int64_t ncap) {
  return ncap > 0 ? seq_layout(ncap, nullptr, nullptr, nullptr) : 0;
}

int64_t zk_tree_seq_zeroed(int64_t ncap) {
  int64_t z = 0;
  if (ncap > 0) seq_layout(ncap, nullptr, nullptr, &z);
  return z;
}

// SEQUENTIAL numbers of the batch's create frames (foff / flen, *n_dev of
// them) in stream order -> seqno[ncap] (parent node << 32 | number; -1:
// none); see seq_* above.  Run
// it before the serve of the same frames, with t->seqno = seqno there.
int zk_tree_seq_order(const ZkTree* t, const uint8_t* rx, const int64_t* foff,
                      const int32_t* flen, const int64_t* n_dev, int64_t ncap,
                      uint8_t* ws, int64_t ws_bytes, int64_t* seqno,
                      hipStream_t st) {
  if (ncap <= 0) return 0;
  if (ncap > zk::SQ_MAX) return -1;
  if (ws_bytes < zk_tree_seq_workspace(ncap) || ((uintptr_t)ws & 15))
    return -1;
  zk::SeqWs w;
  int64_t zeroed = 0;
  seq_layout(ncap, ws, &w, &zeroed);
  w.dbg = g_seq_dbg;
  if (hipMemsetAsync(w.ctr, 0, 64, st) != hipSuccess) return -4;
  const unsigned nchunk = (unsigned)((ncap + zk::SQ_C - 1) / zk::SQ_C);
  const unsigned nb = (unsigned)((ncap + zk::TR_T - 1) / zk::TR_T);
  const unsigned ng = nb < 1024 ? nb : 1024;   // grid-stride over groups
  zk::seq_group_k<<<nchunk, zk::SQ_C, 0, st>>>(rx, foff, flen, n_dev, ncap, w);
  ZK_LAUNCH_CHECK();
  zk::seq_alloc_k<<<ng, zk::TR_T, 0, st>>>(w);
  ZK_LAUNCH_CHECK();
  zk::seq_index_k<<<nb, zk::TR_T, 0, st>>>(ncap, w);
  ZK_LAUNCH_CHECK();
  zk::seq_scan_k<<<ng, zk::TR_T, 0, st>>>(*t, rx, foff, flen, w);
  ZK_LAUNCH_CHECK();
  zk::seq_out_k<<<nb, zk::TR_T, 0, st>>>(ncap, w, seqno);
  ZK_LAUNCH_CHECK();
  return 0;
}

// out[4] (zeroed here): node digest sum, live nodes, hash entries in use,
// tombstones (zk_abi.h).
int zk_tree_digest(const ZkTree* t, unsigned long long* out, hipStream_t st) {
  if (hipMemsetAsync(out, 0, 32, st) != hipSuccess) return -4;
  const int64_t nb = (t->store.cap + zk::TR_T - 1) / zk::TR_T;
  if (nb > 0) {
    zk::tree_digest_k<<<(unsigned)nb, zk::TR_T, 0, st>>>(*t, out);
    ZK_LAUNCH_CHECK();
  }
  zk::ht_census_k<<<2048, zk::TR_T, 0, st>>>(*t, out);
  ZK_LAUNCH_CHECK();
  return 0;
}

static int32_t* g_exp_dbg = nullptr;
void zk_tree_expire_debug(int32_t* buf) { g_exp_dbg = buf; }

int zk_tree_expire(const ZkTree* t, int64_t session, int64_t ncap,
                   unsigned long long* removed, hipStream_t st) {
  if (ncap <= 0) return 0;
  const unsigned nb = (unsigned)((ncap + zk::TR_T - 1) / zk::TR_T);
  if (g_exp_dbg != nullptr)
    zk::tree_expire_k<true><<<nb, zk::TR_T, 0, st>>>(*t, session, ncap, removed,
                                                     g_exp_dbg);
  else
    zk::tree_expire_k<false><<<nb, zk::TR_T, 0, st>>>(*t, session, ncap,
                                                      removed, nullptr);
  ZK_LAUNCH_CHECK();
  return finish_launch(t, ncap, nullptr, 1, st);
}

// Expand the watch masks a served batch fired (tree_serve's `fired`) into
// notification events in request order: ev_slot (watcher slot), ev_type,
// ev_poff / ev_plen (path in the tree's path arena); ev_total[0] = events
// written (at most `cap`), ev_total[1] = events fired.  bsum: ceil(ncap /
// 256) int64.
int zk_watch_events(const int32_t* r_op, const int32_t* r_err,
                    const int64_t* n_dev, int64_t ncap, const int64_t* fired,
                    int64_t* bsum, int64_t cap, int32_t* ev_slot,
                    int32_t* ev_type, int64_t* ev_poff, int32_t* ev_plen,
                    int64_t* ev_total, hipStream_t st) {
  if (ncap <= 0) return hipMemsetAsync(ev_total, 0, 16, st);
  const int64_t nb = (ncap + zk::TR_T - 1) / zk::TR_T;
  zk::wt_count_k<<<(unsigned)nb, zk::TR_T, 0, st>>>(r_op, r_err, n_dev, ncap,
                                                    fired, bsum);
  ZK_LAUNCH_CHECK();
  zk::ord_bscan_k<<<1, zk::ORD_SCAN_T, 0, st>>>(bsum, nb);
  ZK_LAUNCH_CHECK();
  zk::wt_expand_k<<<(unsigned)nb, zk::TR_T, 0, st>>>(
      r_op, r_err, n_dev, ncap, fired, bsum, nb, cap, ev_slot, ev_type,
      ev_poff, ev_plen, ev_total);
  ZK_LAUNCH_CHECK();
  return 0;
}

// SET_WATCHES catch-up for the frames (foff / flen, *n_dev of them) of a
// resumed session with watcher slot wslot: events (ev_type, ev_poff /
// ev_plen into rx) for what changed after each frame's relZxid, the other
// watches re-armed.  out[0] = events written (<= cap), out[1] = re-armed
// watches, out[2] = events.  ent: scratch for ent_cap paths.
int zk_watch_resume(const ZkTree* t, const uint8_t* rx, const int64_t* foff,
                    const int32_t* flen, const int64_t* n_dev, int64_t ncap,
                    int32_t wslot, int64_t* ent, int64_t ent_cap, int64_t cap,
                    int32_t* ev_type, int64_t* ev_poff, int32_t* ev_plen,
                    int64_t* out, hipStream_t st) {
  if (t->wt_key == nullptr) return -1;
  zk::wt_resume_k<<<1, zk::WR_T, 0, st>>>(*t, rx, foff, flen, n_dev, ncap,
                                           wslot, ent, ent_cap, cap, ev_type,
                                           ev_poff, ev_plen, out);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
