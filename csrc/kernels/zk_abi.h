// The host/device ABI of libzkmi_hip.so, in ONE place: every descriptor
// struct a launcher takes and every extern "C" launcher prototype.  The
// kernel sources (through zk_common.h) and the torch operator library
// (csrc/torch/zkmi_ops.cpp) both include it, so a launcher whose definition
// drifts from its prototype does not compile (C linkage cannot overload),
// and the static_asserts below pin each struct's layout on both compilers
// (hipcc for the kernels, g++ for the op library).  The build stamps of both
// libraries hash this file (tools/build_native.py).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

extern "C" {


// K10 — request descriptors (SoA).  `arg` is watch (GET_DATA / EXISTS /
// GET_CHILDREN*), flags (CREATE) or version (DELETE / SET_DATA).  Lengths < 0
// mean "empty" and go on the wire as -1.
struct ZkReqBatch {
  const int32_t* opcode;
  const int32_t* xid;
  const int32_t* arg;
  const int64_t* path_off;
  const int32_t* path_len;
  const int64_t* data_off;
  const int32_t* data_len;
  const int32_t* acl_id;
  const uint8_t* path_arena;
  const uint8_t* data_arena;
  const int64_t* acl_off;   // pre-encoded ACL vectors (count + entries)
  const int32_t* acl_len;
  const uint8_t* acl_arena;
};

// Node store of the GPU-resident synthetic server (HBM).  Each node owns a
// 16-byte aligned slot in `slab` laid out in WIRE format, so a reply is two
// contiguous copies, not 13 field gathers from SoA arrays (a random node is
// then 2-3 cache lines instead of ~13):
//   [0,68)   Stat, big-endian (version at +32, 4-byte aligned for CAS)
//   [72,76)  data length, big-endian (-1 when empty, as Jute writes it)
//   [76,..)  data bytes (capacity slot_cap)
struct ZkNodeStore {
  uint8_t* slab;
  int64_t* slot_off;  // [cap] byte offset of the node's slot in slab
  int32_t* data_len;  // [cap] host-endian copy of the data length
  int32_t* slot_cap;  // [cap] data capacity of the slot
  int64_t cap;
};
#define ZK_SLOT_STAT 0
#define ZK_SLOT_LEN 72
#define ZK_SLOT_DATA 76

// K13 — reply descriptors for server-mode encode.
struct ZkRespBatch {
  const int32_t* opcode;
  const int32_t* xid;
  const int32_t* err;
  const int64_t* node;      // node index (stat / data source), -1 if none
  const int64_t* zxid;
  const int64_t* path_off;  // CREATE reply path / NOTIFICATION path
  const int32_t* path_len;
  const uint8_t* path_arena;
  const int32_t* aux;       // NOTIFICATION type
  const int64_t* slot;      // node's slot offset in the slab (null: look
                            // it up through node -> slot_off)
};

// K2-K8 — decoded replies (SoA, `cap` rows).
struct ZkReplyOut {
  int32_t* xid;
  int32_t* err;
  int32_t* opcode;
  int32_t* status;
  int64_t* zxid;
  int64_t* stat64;   // [6][cap]
  int32_t* stat32;   // [5][cap]
  int64_t* pay_off;  // data / created path / notification path / vector region
  int32_t* pay_len;
  int32_t* aux0;     // notification type | child / acl count
  int32_t* aux1;     // notification state
  int64_t cap;
};

// K12 — decoded requests (server mode).
struct ZkReqOut {
  int32_t* xid;
  int32_t* opcode;
  int32_t* status;
  int64_t* path_off;
  int32_t* path_len;
  int64_t* data_off;
  int32_t* data_len;
  int32_t* arg;       // watch / version / flags
  int64_t* vec_off;   // CREATE: ACL region; SET_WATCHES: first vector
  int32_t* vec_count; // CREATE: ACL entries; SET_WATCHES: total paths
  int64_t* rel_zxid;  // SET_WATCHES
  int64_t cap;
};

// The GPU-resident synthetic server's tree (tree.hip).
struct ZkTree {
  int64_t* ht;                 // [2 * (mask + 1)] interleaved {key, val}
  int64_t mask;
  int64_t* node_path_off;
  int32_t* node_path_len;
  int64_t* node_parent;        // parent node index, -1 = root, -2 = free
  uint8_t* path_arena;
  int64_t path_cap;
  int64_t slab_cap;
  int64_t* counters;           // see TC_* below
  ZkNodeStore store;
  int64_t* free_list;          // ring of deleted node indices
  int64_t free_cap;
  // [cap] cversion << 32 | numChildren, host-endian: a child's create or
  // delete updates both with one atomic
  int64_t* cn;
  int64_t* pzxid;              // [cap] host-endian pzxid
  int32_t* dirty;              // [cap] parent-on-dirty-list flag
  int64_t* dirty_list;         // [cap]
  int64_t* node_pw;            // [cap] path word: offset << 24 | length
  int32_t* node_path_cap;      // [cap] bytes of the node's path storage
  int64_t* eph;                // [cap] host-endian ephemeralOwner shadow
  // watch table (null wt_key: the tree keeps no watches), see wt_* below
  int64_t* wt_key;             // [wt_hmask + 1] path hash | 1, 0 = empty
  unsigned long long* wt_mask; // [2 * (wt_hmask + 1)] data / child masks
  int64_t wt_hmask;
  // [ncap] per request of the batch being served: its parent node << 32 |
  // its SEQUENTIAL number, assigned in stream order by zk_tree_seq_order
  // (-1: none; the serve then takes the parent's cversion atomically).
  // Null: no request has one.
  const int64_t* seqno;
};

// Server-side session table (session.hip, K9 server mode).
struct ZkSessionTable {
  int64_t* sid;       // [cap]
  uint8_t* passwd;    // [cap * 16]
  int32_t* timeout;   // [cap]
  int32_t* state;     // [cap] SS_*
  int64_t* next;      // [1] allocation counter
  int64_t cap;
  // 0: one server's table (slot = the id's index).  > 0: an ensemble's
  // replicated table, `span` slots per member: the session with id
  // (member << 56 | index + 1) lives at slot (member - 1) * span + index
  int64_t span;
};

// ---- launchers (stream-ordered; return 0 or a hipError_t) ----------------
int64_t zk_scan_workspace(int64_t n);
int zk_scan_set_mode(int mode);
// engine of the one-workgroup scans (ZKMI_SMALL_SCAN): 1 MFMA, 0 shuffle
int zk_scan_small_mode(void);
// the one-workgroup exclusive scan with an explicit engine (1 MFMA, 0 shfl)
int zk_scan_small_i64_mode(const int64_t*, int64_t*, int64_t, int64_t*, int,
                           hipStream_t);
int zk_scan_excl_i64(const int64_t*, int64_t*, int64_t, int64_t*, int64_t*,
                     hipStream_t);
int zk_scan_excl_i32(const int32_t*, int64_t*, int64_t, int64_t*, int64_t*,
                     hipStream_t);
int zk_encode_requests2(const ZkReqBatch*, int64_t, int64_t*, int64_t*,
                        int64_t*, int64_t*, uint8_t*, int64_t, int64_t*,
                        int64_t, int32_t*, int32_t, hipStream_t);
int zk_encode_requests_presized(const ZkReqBatch*, int64_t, const int64_t*,
                                const int64_t*, int64_t*, int64_t*, int64_t*,
                                uint8_t*, int64_t, int64_t*, int64_t,
                                int32_t*, int32_t, hipStream_t);
int zk_encode_set_watches(const int64_t*, const int32_t*, const uint8_t*,
                          int64_t, int64_t, int64_t, int64_t, int64_t*,
                          int64_t*, int64_t*, int64_t*, uint8_t*, int64_t,
                          int32_t*, hipStream_t);
int zk_encode_connect_requests(const int32_t*, const int64_t*, const int32_t*,
                               const int64_t*, const int64_t*, const int32_t*,
                               const uint8_t*, int64_t, int64_t*, int64_t*,
                               int64_t*, int64_t*, uint8_t*, hipStream_t);
int zk_encode_responses2(const ZkRespBatch*, const ZkNodeStore*,
                         const int64_t*, int64_t, int64_t*, int64_t*,
                         int64_t*, int64_t*, uint8_t*, int64_t, int32_t*,
                         int32_t, int32_t, hipStream_t);
int zk_encode_responses3(const ZkRespBatch*, const ZkNodeStore*,
                         const int64_t*, int64_t, int64_t*, int64_t*, int64_t*,
                         int64_t*, uint8_t*, int64_t, int32_t*, int32_t,
                         int32_t, int64_t, hipStream_t);
int64_t zk_frame_scan_workspace(int64_t n);
int zk_frame_scan5(const uint8_t*, const int64_t*, int64_t, int64_t,
                   uint8_t*, int64_t, int64_t*, int32_t*, int64_t, int64_t*,
                   int32_t, int32_t, int32_t, hipStream_t);
int zk_frame_scan_stats(const uint8_t*, int64_t, int32_t, uint32_t*,
                        hipStream_t);
int zk_frame_scan_dbg(int64_t* host, int64_t tiles);
int zk_decode_replies(const uint8_t*, const int64_t*, const int32_t*,
                      const int64_t*, int64_t, const int64_t*, int64_t,
                      const ZkReplyOut*, hipStream_t);
int zk_decode_replies_check2(const uint8_t*, const int64_t*, const int32_t*,
                             const int64_t*, int64_t, const int64_t*, int64_t,
                             const ZkReplyOut*, const int64_t*, const int32_t*,
                             const int32_t*, unsigned long long*, int32_t,
                             int64_t*, const uint8_t*, const int64_t*,
                             hipStream_t);
int zk_expand_strings(const uint8_t*, const int64_t*, const int32_t*,
                      const int64_t*, int64_t, int64_t*, int32_t*,
                      hipStream_t);
int zk_expand_acl(const uint8_t*, const int64_t*, const int32_t*,
                  const int64_t*, int64_t, int32_t*, int64_t*, int32_t*,
                  int64_t*, int32_t*, hipStream_t);
int zk_decode_requests(const uint8_t*, const int64_t*, const int32_t*,
                       const int64_t*, int64_t, const ZkReqOut*, hipStream_t);
int zk_decode_connect_responses(const uint8_t*, const int64_t*,
                                const int32_t*, int64_t, int32_t*, int32_t*,
                                int64_t*, int64_t*, int32_t*, int32_t*,
                                hipStream_t);
int zk_tree_fill(const ZkTree*, int64_t, int64_t, const int32_t*, int64_t,
                 hipStream_t);
int zk_tree_build(const ZkTree*, int64_t, int64_t, hipStream_t);
// every hash entry back to empty (before a rebuild)
int zk_tree_ht_reset(const ZkTree*, hipStream_t);
// the free ring's pending entries rebuilt in node order (between batches)
int64_t zk_tree_free_workspace(int64_t cap);
int zk_tree_free_compact(const ZkTree*, int64_t*, hipStream_t);
int zk_tree_serve(const ZkTree*, const uint8_t*, const ZkReqOut*,
                  const int64_t*, int64_t, int32_t*, int32_t*, int32_t*,
                  int64_t*, int64_t*, int64_t*, int32_t*, int64_t*, int64_t*,
                  int64_t*, int64_t, int64_t, hipStream_t);
int64_t zk_serve_tickets(int64_t);
int zk_tree_serve_frames(const ZkTree*, const uint8_t*, const int64_t*,
                         const int32_t*, const int64_t*, int64_t, int32_t*,
                         int32_t*, int32_t*, int64_t*, int64_t*, int64_t*,
                         int32_t*, int64_t*, int64_t*, int64_t*, int64_t,
                         int64_t, int32_t, int64_t*, unsigned*,
                         hipStream_t);
int zk_tree_serve_frames2(const ZkTree*, const uint8_t*, const int64_t*,
                          const int32_t*, const int64_t*, int64_t, int32_t*,
                          int32_t*, int32_t*, int64_t*, int64_t*, int64_t*,
                          int32_t*, int64_t*, int64_t*, int64_t*, int64_t,
                          int64_t, int32_t, int64_t*, unsigned*, int32_t,
                          hipStream_t);
// zk_tree_serve_frames2's last flag word
#define ZK_SERVE_FINISH 1
#define ZK_SERVE_RO 2
int zk_tree_finish(const ZkTree*, const int64_t*, int64_t, int32_t,
                   hipStream_t);
int zk_tree_finish_scan(const ZkTree*, const int64_t*, int64_t, int32_t,
                        int64_t, int64_t*, int64_t*, hipStream_t);
int zk_tree_serve_ordered(const ZkTree*, const uint8_t*, const ZkReqOut*,
                          const int64_t*, int64_t, int32_t*, int32_t*,
                          int32_t*, int64_t*, int64_t*, int64_t*, int32_t*,
                          int64_t*, int64_t*, int64_t*, int64_t, int64_t,
                          uint8_t*, int64_t, int32_t, int64_t, int64_t,
                          int32_t, int64_t*, hipStream_t);
int zk_watch_events(const int32_t*, const int32_t*, const int64_t*, int64_t,
                    const int64_t*, int64_t*, int64_t, int32_t*, int32_t*,
                    int64_t*, int32_t*, int64_t*, hipStream_t);
int zk_watch_resume(const ZkTree*, const uint8_t*, const int64_t*,
                    const int32_t*, const int64_t*, int64_t, int32_t,
                    int64_t*, int64_t, int64_t, int32_t*, int64_t*, int32_t*,
                    int64_t*, hipStream_t);
int64_t zk_tree_order_workspace(int64_t);
int64_t zk_tree_order_stats_offset(int64_t);
int zk_tree_expire(const ZkTree*, int64_t, int64_t, unsigned long long*,
                   hipStream_t);
// SEQUENTIAL numbers of a batch in stream order (tree.hip seq_*): bytes of
// the workspace for ncap requests, the prefix of it that must be zero when
// it is first used (the kernels leave it zero), and the ordering itself
// (writes seqno[ncap]; bumps each parent's cversion once per batch).
int64_t zk_tree_seq_workspace(int64_t ncap);
int64_t zk_tree_seq_zeroed(int64_t ncap);
void zk_tree_seq_debug(int64_t* buf);
// tree_expire_k's phase clocks: 4 int32 per node of the expiries that follow
// (the buffer covers the tree's node capacity; nullptr turns them off)
void zk_tree_expire_debug(int32_t* buf);
int zk_tree_seq_order(const ZkTree*, const uint8_t*, const int64_t*,
                      const int32_t*, const int64_t*, int64_t, uint8_t*,
                      int64_t, int64_t*, hipStream_t);
// order-independent digest of the live nodes: out[0] = sum of per-node
// hashes (path, czxid, mzxid, version, cversion, numChildren, owner, pzxid,
// data), out[1] = live nodes, out[2] = hash entries in use (live +
// tombstones), out[3] = tombstones
int zk_tree_digest(const ZkTree*, unsigned long long*, hipStream_t);
int zk_bench_gen_get(int64_t, uint64_t, int64_t, int64_t, int32_t,
                     const int64_t*, int64_t*, int32_t*, int64_t*, int32_t*,
                     const int64_t*, int64_t*, int64_t*, hipStream_t);
int zk_bench_xids(int64_t, const int64_t*, int32_t*, hipStream_t);
int zk_bench_storm_hs(int32_t, int32_t, int32_t, const int32_t*,
                      const int64_t*, const int32_t*, const int32_t*,
                      const int64_t*, const uint8_t*, const int64_t*,
                      int64_t*, uint8_t*, bool*, hipStream_t);
int zk_bench_check_writes(int64_t, const int32_t*, const int32_t*,
                          const int32_t*, const int32_t*, const int32_t*,
                          const int32_t*, int32_t, const int64_t*,
                          unsigned long long*, unsigned long long*,
                          hipStream_t);
int zk_bench_check_get(int64_t, const int32_t*, const int32_t*,
                       const int32_t*, const int32_t*, const int64_t*,
                       const int32_t*, const int64_t*, const int32_t*,
                       const int32_t*, unsigned long long*, hipStream_t);
int zk_bench_check_notif(int64_t, int64_t, const uint64_t*, const int64_t*,
                         int64_t, int64_t,
                         const int64_t*, const int32_t*, const uint8_t*,
                         const uint8_t*, const int32_t*, const int32_t*,
                         const int32_t*, const int32_t*, const int32_t*,
                         const int64_t*, const int32_t*, unsigned long long*,
                         hipStream_t);
int64_t zk_route_workspace(int64_t n, int32_t world);
int zk_route_requests(int64_t, int32_t, const int64_t*, const int32_t*,
                      const uint8_t*, const int64_t*, const int32_t*,
                      int32_t*, int64_t*, int32_t*, int64_t*, int32_t*,
                      int64_t*, int64_t*, hipStream_t);
int zk_route_requests2(int64_t, int32_t, int32_t, const int64_t*,
                       const int32_t*, const uint8_t*, const int64_t*,
                       const int32_t*, int32_t*, int64_t*, int32_t*, int64_t*,
                       int32_t*, int64_t*, int64_t*, hipStream_t);
int zk_seg_pack(const uint8_t*, int64_t, const int64_t*, const int64_t*,
                int64_t, const int64_t*, const int64_t*, int32_t, int32_t,
                int64_t, uint8_t*, unsigned long long*, uint8_t*, int32_t,
                hipStream_t);
int zk_seg_unpack(const uint8_t*, int32_t, int32_t, int64_t, uint8_t*,
                  int64_t*, int64_t*, unsigned long long*, const uint8_t*,
                  int32_t, hipStream_t);
int zk_session_connect(const uint8_t*, const int64_t*, const int32_t*,
                       const int64_t*, int64_t, const ZkSessionTable*,
                       int64_t, uint64_t, int32_t, int32_t, const int64_t*,
                       uint8_t*, int64_t*, int32_t*, hipStream_t);
int zk_session_close(const ZkSessionTable*, const int64_t*, int64_t,
                     int64_t, hipStream_t);
int zk_session_install(const ZkSessionTable*, const int64_t*, int64_t,
                       int64_t, hipStream_t);
int zk_scan_small_i64(const int64_t*, int64_t*, int64_t, int64_t*,
                      hipStream_t);
}  // extern "C"

// Layout pins (LP64 on both sides: pointers and int64_t are 8 bytes).
static_assert(sizeof(void*) == 8, "LP64 only");
static_assert(sizeof(ZkReqBatch) == 13 * 8, "ZkReqBatch layout");
static_assert(sizeof(ZkNodeStore) == 5 * 8, "ZkNodeStore layout");
static_assert(sizeof(ZkRespBatch) == 10 * 8, "ZkRespBatch layout");
static_assert(sizeof(ZkReplyOut) == 12 * 8, "ZkReplyOut layout");
static_assert(sizeof(ZkReqOut) == 12 * 8, "ZkReqOut layout");
static_assert(sizeof(ZkSessionTable) == 7 * 8, "ZkSessionTable layout");
static_assert(sizeof(ZkTree) == 27 * 8, "ZkTree layout");
static_assert(offsetof(ZkTree, store) == 9 * 8, "ZkTree.store");
static_assert(offsetof(ZkTree, free_list) == 14 * 8, "ZkTree.free_list");
static_assert(offsetof(ZkTree, wt_hmask) == 25 * 8, "ZkTree.wt_hmask");
static_assert(offsetof(ZkRespBatch, slot) == 9 * 8, "ZkRespBatch.slot");
static_assert(offsetof(ZkReplyOut, cap) == 11 * 8, "ZkReplyOut.cap");
static_assert(offsetof(ZkReqOut, rel_zxid) == 10 * 8, "ZkReqOut.rel_zxid");
