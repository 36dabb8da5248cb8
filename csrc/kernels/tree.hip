// GPU-resident synthetic ZooKeeper tree (the server side of the 1M-znode
// benchmark and of the create/set/delete mix).  Not part of the reference —
// it stands in for the JVM server the reference tests talk to, so that the
// whole request -> reply path can be driven at HBM speed.
//
// Layout (HBM, sized by the caller for 288 GB parts):
//   * open-addressing hash table: keys = FNV-1a(path) | 1, vals = node index
//     (-2 = tombstone, -3 = being published), linear probing, pow2 capacity;
//   * node slots in wire format (zk_batch.h ZkNodeStore), so replies are
//     contiguous copies;
//   * a path arena holding each node's path for exact-match verification;
//   * counters: [0] node count, [1] zxid, [2] path-arena top, [3] slab top.
// Requests are applied concurrently within a batch; conflicting operations
// on the same path inside ONE batch are unordered (the benchmark generator
// never emits them).  Version CAS is an atomicCAS on the slot's big-endian
// version word, so exactly one of several same-version SET_DATAs wins (the
// others get BAD_VERSION), matching ZooKeeper's conditional set.
#include "zk_common.h"
#include "zk_batch.h"

extern "C" {
struct ZkTree {
  int64_t* keys;
  int64_t* vals;
  int64_t mask;
  int64_t* node_path_off;
  int32_t* node_path_len;
  int64_t* node_parent;        // parent node index (-1 for roots)
  uint8_t* path_arena;
  int64_t path_cap;
  int64_t slab_cap;
  int64_t* counters;
  ZkNodeStore store;
};
}

namespace zk {

constexpr int TR_T = 256;

ZK_DEV int64_t slot_bytes(int32_t data_cap) {
  return ZK_SLOT_DATA + (((int64_t)data_cap + 15) & ~(int64_t)15) + 4;
}

ZK_DEV uint64_t fnv1a(const uint8_t* p, int32_t n) {
  uint64_t h = 1469598103934665603ull;
  int32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    uint32_t w; __builtin_memcpy(&w, p + i, 4);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      h ^= (w >> (8 * b)) & 0xff;
      h *= 1099511628211ull;
    }
  }
  for (; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

ZK_DEV bool bytes_eq(const uint8_t* a, const uint8_t* b, int32_t n) {
  int32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    uint32_t x, y; __builtin_memcpy(&x, a + i, 4); __builtin_memcpy(&y, b + i, 4);
    if (x != y) return false;
  }
  for (; i < n; ++i) if (a[i] != b[i]) return false;
  return true;
}

ZK_DEV int64_t tree_find(const ZkTree& t, const uint8_t* p, int32_t n) {
  const int64_t key = (int64_t)(fnv1a(p, n) | 1ull);
  int64_t s = key & t.mask;
  for (int64_t probe = 0; probe <= t.mask; ++probe) {
    const int64_t k = __hip_atomic_load(&t.keys[s], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    if (k == 0) return -1;
    if (k == key) {
      const int64_t v = __hip_atomic_load(&t.vals[s], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      if (v >= 0 && t.node_path_len[v] == n &&
          bytes_eq(t.path_arena + t.node_path_off[v], p, n))
        return v;
    }
    s = (s + 1) & t.mask;
  }
  return -1;
}

// Insert node `v` (path already in the arena).  Returns the existing node if
// the path is present (NODE_EXISTS), else v.
ZK_DEV int64_t tree_insert(const ZkTree& t, int64_t v, const uint8_t* p,
                           int32_t n) {
  const int64_t key = (int64_t)(fnv1a(p, n) | 1ull);
  int64_t s = key & t.mask;
  for (int64_t probe = 0; probe <= t.mask; ++probe) {
    const int64_t k = atomicCAS((unsigned long long*)&t.keys[s], 0ull,
                                (unsigned long long)key);
    if (k == 0) {                         // claimed an empty slot
      __hip_atomic_store(&t.vals[s], v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      return v;
    }
    if (k == key) {
      int64_t w = -3;
      // The claimer may not have published vals yet: bounded wait.
      for (int spin = 0; spin < 1000000 && w == -3; ++spin)
        w = __hip_atomic_load(&t.vals[s], __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
      if (w >= 0 && t.node_path_len[w] == n &&
          bytes_eq(t.path_arena + t.node_path_off[w], p, n))
        return w;
      if (w == -2 &&                      // tombstone of the same key: reuse
          atomicCAS((unsigned long long*)&t.vals[s], (unsigned long long)-2,
                    (unsigned long long)v) == (unsigned long long)-2)
        return v;
    }
    s = (s + 1) & t.mask;
  }
  return -1;
}

ZK_DEV void tree_erase(const ZkTree& t, int64_t v, const uint8_t* p,
                       int32_t n) {
  const int64_t key = (int64_t)(fnv1a(p, n) | 1ull);
  int64_t s = key & t.mask;
  for (int64_t probe = 0; probe <= t.mask; ++probe) {
    const int64_t k = t.keys[s];
    if (k == 0) return;
    if (k == key && t.vals[s] == v) {
      atomicExch((unsigned long long*)&t.vals[s], (unsigned long long)-2);
      return;
    }
    s = (s + 1) & t.mask;
  }
}

// Atomic add on a big-endian 32-bit field (cversion / numChildren).
ZK_DEV void be32_atomic_add(uint8_t* p, int32_t d) {
  unsigned int* w = (unsigned int*)p;
  unsigned int old = *w, assumed;
  do {
    assumed = old;
    const unsigned int nv = bswap32((uint32_t)((int32_t)bswap32(assumed) + d));
    old = atomicCAS(w, assumed, nv);
  } while (old != assumed);
}

ZK_DEV void fill_stat(uint8_t* st, int64_t cz, int64_t mz, int64_t ct,
                      int64_t mt, int32_t ver, int32_t cver, int32_t aver,
                      int64_t owner, int32_t dlen, int32_t nkids, int64_t pz) {
  st_be64(st + 0, cz); st_be64(st + 8, mz); st_be64(st + 16, ct);
  st_be64(st + 24, mt); st_be32(st + 32, ver); st_be32(st + 36, cver);
  st_be32(st + 40, aver); st_be64(st + 44, owner); st_be32(st + 52, dlen);
  st_be32(st + 56, nkids); st_be64(st + 60, pz);
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
}

__global__ __launch_bounds__(TR_T) void tree_build_k(ZkTree t, int64_t n0,
                                                    int64_t n) {
  const int64_t v = n0 + (int64_t)blockIdx.x * TR_T + threadIdx.x;
  if (v >= n) return;
  tree_insert(t, v, t.path_arena + t.node_path_off[v], t.node_path_len[v]);
}

// Apply one batch of decoded requests; produce reply descriptors for K13.
__global__ __launch_bounds__(TR_T) void tree_serve_k(
    ZkTree t, const uint8_t* __restrict__ rx, ZkReqOut q,
    const int64_t* __restrict__ n_dev, int64_t ncap, int32_t* __restrict__ r_op,
    int32_t* __restrict__ r_xid, int32_t* __restrict__ r_err,
    int64_t* __restrict__ r_node, int64_t* __restrict__ r_zxid,
    int64_t now_ms) {
  const int64_t i = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * TR_T +
                    threadIdx.x;
  if (i >= ncap || i >= *n_dev) return;
  const int32_t op = q.opcode[i];
  int32_t err = ERR_OK;
  int64_t node = -1;
  int64_t zx = __hip_atomic_load(&t.counters[1], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
  const ZkNodeStore& s = t.store;
  if (q.status[i] != ST_OK) {
    err = -8;                                       // BAD_ARGUMENTS
  } else {
    const uint8_t* path = rx + q.path_off[i];
    const int32_t pl = q.path_len[i];
    switch (op) {
      case OP_GET_DATA: case OP_EXISTS:
        node = tree_find(t, path, pl);
        if (node < 0) err = ERR_NO_NODE;
        break;
      case OP_SET_DATA: {
        node = tree_find(t, path, pl);
        if (node < 0) { err = ERR_NO_NODE; break; }
        const int32_t dl = max(q.data_len[i], 0);
        if (dl > s.slot_cap[node]) { err = -8; break; }
        uint8_t* slot = s.slab + s.slot_off[node];
        unsigned int* ver = (unsigned int*)(slot + 32);
        const int32_t want = q.arg[i];
        if (want == -1) {
          be32_atomic_add(slot + 32, 1);
        } else if (atomicCAS(ver, bswap32((uint32_t)want),
                             bswap32((uint32_t)(want + 1))) !=
                   bswap32((uint32_t)want)) {
          err = ERR_BAD_VERSION;
          break;
        }
        zx = atomicAdd((unsigned long long*)&t.counters[1], 1ull) + 1;
        copy_bytes(slot + ZK_SLOT_DATA, rx + q.data_off[i], dl);
        st_be32(slot + ZK_SLOT_LEN, dl > 0 ? dl : -1);
        s.data_len[node] = dl;
        st_be64(slot + 8, zx);                      // mzxid
        st_be64(slot + 24, now_ms);                 // mtime
        st_be32(slot + 52, dl);                     // dataLength
        break;
      }
      case OP_CREATE: {
        int32_t cut = pl - 1;                       // parent must exist
        while (cut > 0 && path[cut] != '/') --cut;
        const int64_t par = cut > 0 ? tree_find(t, path, cut) : -1;
        if (cut > 0 && par < 0) { err = ERR_NO_NODE; break; }
        if (tree_find(t, path, pl) >= 0) { err = ERR_NODE_EXISTS; break; }
        const int32_t dl = max(q.data_len[i], 0);
        const int32_t cap = max(dl, 128);
        const int64_t v = atomicAdd((unsigned long long*)&t.counters[0], 1ull);
        const int64_t po = atomicAdd((unsigned long long*)&t.counters[2],
                                     (unsigned long long)pl);
        const int64_t so = atomicAdd((unsigned long long*)&t.counters[3],
                                     (unsigned long long)slot_bytes(cap));
        if (v >= s.cap || po + pl > t.path_cap ||
            so + slot_bytes(cap) > t.slab_cap) {
          err = -1;                                 // SYSTEM_ERROR: full
          break;
        }
        copy_bytes(t.path_arena + po, path, pl);
        uint8_t* slot = s.slab + so;
        zx = atomicAdd((unsigned long long*)&t.counters[1], 1ull) + 1;
        fill_stat(slot, zx, zx, now_ms, now_ms, 0, 0, 0, 0, dl, 0, zx);
        st_be32(slot + ZK_SLOT_LEN, dl > 0 ? dl : -1);
        copy_bytes(slot + ZK_SLOT_DATA, rx + q.data_off[i], dl);
        t.node_path_off[v] = po;
        t.node_path_len[v] = pl;
        t.node_parent[v] = par;
        s.slot_off[v] = so;
        s.slot_cap[v] = cap;
        s.data_len[v] = dl;
        __threadfence();
        const int64_t got = tree_insert(t, v, t.path_arena + po, pl);
        if (got != v) { err = ERR_NODE_EXISTS; break; }
        if (par >= 0) {
          uint8_t* ps = s.slab + s.slot_off[par];
          be32_atomic_add(ps + 36, 1);              // cversion
          be32_atomic_add(ps + 56, 1);              // numChildren
          st_be64(ps + 60, zx);                     // pzxid (last writer)
        }
        node = v;
        break;
      }
      case OP_DELETE: {
        node = tree_find(t, path, pl);
        if (node < 0) { err = ERR_NO_NODE; break; }
        uint8_t* slot = s.slab + s.slot_off[node];
        if (ld_be32(slot + 56) > 0) { err = ERR_NOT_EMPTY; node = -1; break; }
        const int32_t want = q.arg[i];
        if (want != -1 && ld_be32(slot + 32) != want) {
          err = ERR_BAD_VERSION; node = -1; break;
        }
        tree_erase(t, node, path, pl);
        zx = atomicAdd((unsigned long long*)&t.counters[1], 1ull) + 1;
        const int64_t par = t.node_parent[node];
        if (par >= 0) {
          uint8_t* ps = s.slab + s.slot_off[par];
          be32_atomic_add(ps + 36, 1);
          be32_atomic_add(ps + 56, -1);
          st_be64(ps + 60, zx);
        }
        node = -1;
        break;
      }
      case OP_SYNC: case OP_PING:
        break;
      default:
        err = -6;                                   // UNIMPLEMENTED
    }
  }
  r_op[i] = op;
  r_xid[i] = q.xid[i];
  r_err[i] = err;
  r_node[i] = node;
  r_zxid[i] = zx;
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

int zk_tree_build(const ZkTree* t, int64_t n0, int64_t n, hipStream_t st) {
  if (n <= n0) return 0;
  const int64_t m = n - n0;
  zk::tree_build_k<<<(unsigned)((m + zk::TR_T - 1) / zk::TR_T), zk::TR_T, 0,
                     st>>>(*t, n0, n);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_tree_serve(const ZkTree* t, const uint8_t* rx, const ZkReqOut* q,
                  const int64_t* n_dev, int64_t ncap, int32_t* r_op,
                  int32_t* r_xid, int32_t* r_err, int64_t* r_node,
                  int64_t* r_zxid, int64_t now_ms, hipStream_t st) {
  if (ncap <= 0) return 0;
  zk::tree_serve_k<<<(unsigned)((ncap + zk::TR_T - 1) / zk::TR_T), zk::TR_T,
                     0, st>>>(*t, rx, *q, n_dev, ncap, r_op, r_xid, r_err,
                              r_node, r_zxid, now_ms);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
