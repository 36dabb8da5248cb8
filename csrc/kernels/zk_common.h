// zkmi HIP kernels — shared device helpers (gfx950 / CDNA4 only).
//
// Byte-level Jute access: every multi-byte field on the ZooKeeper wire is
// big-endian and unaligned (records are packed back to back).  gfx950 runs
// global memory in unaligned-access mode, so a 4/8-byte __builtin_memcpy
// from any byte address compiles to one global_load_dword(x2); we byte-swap
// in registers.  (Checked in the .s: no ubyte loads for these.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zk_abi.h"

#define ZK_DEV __device__ __forceinline__

namespace zk {

// Handshake outcome per ConnectRequest (session.hip; zkmi/ops/_lib.py SC_*)
enum : int32_t { SC_NEW = 0, SC_RESUMED = 1, SC_EXPIRED = 2, SC_REFUSED = 3,
                 SC_BAD = 4, SC_FULL = 5 };

constexpr int WAVE = 64;

// opcodes (lib/zk-consts.js:84-105; csrc/proto mirror, tests check parity)
enum : int32_t {
  OP_NOTIFICATION = 0, OP_CREATE = 1, OP_DELETE = 2, OP_EXISTS = 3,
  OP_GET_DATA = 4, OP_SET_DATA = 5, OP_GET_ACL = 6, OP_SET_ACL = 7,
  OP_GET_CHILDREN = 8, OP_SYNC = 9, OP_PING = 11, OP_GET_CHILDREN2 = 12,
  OP_CHECK = 13, OP_MULTI = 14, OP_AUTH = 100, OP_SET_WATCHES = 101,
  OP_SASL = 102, OP_CREATE_SESSION = -10, OP_CLOSE_SESSION = -11,
  OP_ERROR = -1, OP_UNKNOWN = -1000
};
enum : int32_t {
  XID_NOTIFICATION = -1, XID_PING = -2, XID_AUTH = -4, XID_SET_WATCHES = -8
};
enum : int32_t { ERR_OK = 0, ERR_SYSTEM = -1, ERR_UNIMPLEMENTED = -6,
                 ERR_BAD_ARGUMENTS = -8, ERR_NO_NODE = -101,
                 ERR_BAD_VERSION = -103, ERR_NO_CHILDREN_FOR_EPHEMERALS = -108,
                 ERR_NODE_EXISTS = -110, ERR_NOT_EMPTY = -111,
                 ERR_INVALID_ACL = -114 };
// CREATE flags (lib/zk-buffer.js createFlags mapping)
enum : int32_t { CF_EPHEMERAL = 1, CF_SEQUENTIAL = 2 };
// per-record decode status
enum : int32_t { ST_OK = 0, ST_BAD_DECODE = 1, ST_NO_XID = 2,
                 ST_BAD_OPCODE = 3 };
constexpr int32_t STAT_BYTES = 68;
constexpr int64_t MAX_PACKET = 16 * 1024 * 1024;

ZK_DEV uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
ZK_DEV uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }

ZK_DEV int32_t ld_be32(const uint8_t* p) {
  uint32_t v; __builtin_memcpy(&v, p, 4); return (int32_t)bswap32(v);
}
ZK_DEV int64_t ld_be64(const uint8_t* p) {
  uint64_t v; __builtin_memcpy(&v, p, 8); return (int64_t)bswap64(v);
}
ZK_DEV void st_be32(uint8_t* p, int32_t x) {
  uint32_t v = bswap32((uint32_t)x); __builtin_memcpy(p, &v, 4);
}
ZK_DEV void st_be64(uint8_t* p, int64_t x) {
  uint64_t v = bswap64((uint64_t)x); __builtin_memcpy(p, &v, 8);
}

// Copy n bytes global->global; 16-byte body with a byte tail.  Source and
// destination are arbitrary byte addresses (unaligned mode).
ZK_DEV void copy_bytes(uint8_t* __restrict__ d, const uint8_t* __restrict__ s,
                       int64_t n) {
  int64_t i = 0;
  for (; i + 16 <= n; i += 16) {
    uint4 v; __builtin_memcpy(&v, s + i, 16); __builtin_memcpy(d + i, &v, 16);
  }
  for (; i + 4 <= n; i += 4) {
    uint32_t v; __builtin_memcpy(&v, s + i, 4); __builtin_memcpy(d + i, &v, 4);
  }
  for (; i < n; ++i) d[i] = s[i];
}

// Jute buffer/ustring: i32 length then bytes; an EMPTY buffer is written as
// length -1 (lib/jute-buffer.js:127-130).
ZK_DEV uint8_t* put_buffer(uint8_t* o, const uint8_t* src, int32_t len) {
  if (len <= 0) { st_be32(o, -1); return o + 4; }
  st_be32(o, len); copy_bytes(o + 4, src, len); return o + 4 + len;
}

// XCD-aware block remap (guide §5.5 T1, bijective form): consecutive logical
// tiles land on the same XCD so neighbouring frames share an L2.
ZK_DEV uint32_t xcd_remap(uint32_t orig, uint32_t nwg) {
  const uint32_t xcd = orig & 7u, q = nwg >> 3, r = nwg & 7u;
  const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

// Wave-level inclusive scan of int64 over 64 lanes (DPP-free shuffle form).
ZK_DEV int64_t wave_incl_scan(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Block-wide exclusive scan (blockDim.x multiple of 64, <= 1024).  `sm` must
// hold blockDim.x/64 int64s.  Returns the exclusive prefix; *total gets the
// block sum (valid in every thread).
ZK_DEV int64_t block_excl_scan(int64_t v, int64_t* sm, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  int64_t inc = wave_incl_scan(v);
  if (lane == 63) sm[w] = inc;
  __syncthreads();
  if (w == 0) {
    int64_t x = lane < nw ? sm[lane] : 0;
    int64_t xi = wave_incl_scan(x);
    if (lane < nw) sm[lane] = xi - x;
    if (lane == nw - 1) sm[nw] = xi;
  }
  __syncthreads();
  int64_t r = sm[w] + inc - v;
  *total = sm[nw];
  __syncthreads();
  return r;
}

}  // namespace zk

#define ZK_LAUNCH_CHECK() \
  do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)
