// Host/device batch descriptors shared by the HIP launchers and the Python
// ctypes bindings (zkmi/ops/_lib.py mirrors these layouts field for field).
#pragma once
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

}  // extern "C"
