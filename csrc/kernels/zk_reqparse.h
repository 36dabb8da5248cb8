// Server-mode request parse (K12), shared by decode_requests_k (SoA output)
// and the GPU server's fused serve (csrc/kernels/tree.hip), which parses
// each frame in registers instead of reading the SoA back.
// Reference: lib/zk-buffer.js:58-253 (request layouts).
#pragma once
#include "zk_common.h"

namespace zk {

// Walk `count` ustrings starting at p; returns bytes consumed or -1.
ZK_DEV int64_t skip_strings(const uint8_t* p, int64_t avail, int32_t count) {
  int64_t k = 0;
  for (int32_t j = 0; j < count; ++j) {
    if (k + 4 > avail) return -1;
    int32_t l = ld_be32(p + k);
    if (l < 0) l = 0;
    k += 4 + l;
    if (k > avail) return -1;
  }
  return k;
}

// ACL vector entries: perms i32, scheme ustring, id ustring.
ZK_DEV int64_t skip_acl(const uint8_t* p, int64_t avail, int32_t count) {
  int64_t k = 0;
  for (int32_t j = 0; j < count; ++j) {
    if (k + 4 > avail) return -1;
    k += 4;
    int64_t s = skip_strings(p + k, avail - k, 2);
    if (s < 0) return -1;
    k += s;
  }
  return k;
}

struct ReqFields {
  int32_t status, xid, op, arg, pl, dl, vc;
  int64_t poff, doff, voff, rel;
};

// Frame body [base, base + L) of buf -> the request's fields (offsets are
// absolute in buf).
ZK_DEV ReqFields parse_request(const uint8_t* __restrict__ buf, int64_t base,
                               int64_t L) {
  const uint8_t* p = buf + base;
  int32_t status = ST_OK, xid = 0, op = OP_UNKNOWN, arg = 0;
  int64_t poff = -1, doff = -1, voff = -1, rel = 0;
  int32_t pl = 0, dl = 0, vc = 0;
  if (L < 8) {
    status = ST_BAD_DECODE;
  } else {
    xid = ld_be32(p);
    op = ld_be32(p + 4);
    int64_t k = 8;
    auto get_str = [&](int64_t& off, int32_t& len) -> bool {
      if (k + 4 > L) return false;
      int32_t l = ld_be32(p + k);
      if (l < 0) l = 0;
      if (k + 4 + l > L) return false;
      off = base + k + 4;
      len = l;
      k += 4 + l;
      return true;
    };
    auto get_i32 = [&](int32_t& v) -> bool {
      if (k + 4 > L) return false;
      v = ld_be32(p + k);
      k += 4;
      return true;
    };
    bool ok = true;
    switch (op) {
      case OP_GET_DATA: case OP_EXISTS: case OP_GET_CHILDREN:
      case OP_GET_CHILDREN2:
        ok = get_str(poff, pl) && k + 1 <= L;
        if (ok) { arg = p[k]; ok = (arg == 0 || arg == 1); ++k; }
        break;
      case OP_CREATE: {
        ok = get_str(poff, pl) && get_str(doff, dl) && get_i32(vc);
        if (!ok) break;
        if (vc < 0) vc = 0;
        voff = base + k;
        const int64_t s = skip_acl(p + k, L - k, vc);
        ok = s >= 0;
        if (ok) { k += s; ok = get_i32(arg); }
        break;
      }
      case OP_DELETE:
        ok = get_str(poff, pl) && get_i32(arg);
        break;
      case OP_SET_DATA:
        ok = get_str(poff, pl) && get_str(doff, dl) && get_i32(arg);
        break;
      case OP_GET_ACL: case OP_SYNC:
        ok = get_str(poff, pl);
        break;
      case OP_SET_WATCHES: {
        if (k + 8 > L) { ok = false; break; }
        rel = ld_be64(p + k);
        k += 8;
        voff = base + k;
        for (int g = 0; g < 3 && ok; ++g) {
          int32_t c;
          ok = get_i32(c);
          if (!ok) break;
          c = max(c, 0);
          const int64_t s = skip_strings(p + k, L - k, c);
          ok = s >= 0;
          k += s;
          vc += c;
        }
        break;
      }
      case OP_PING: case OP_CLOSE_SESSION:
        break;
      default:
        status = ST_BAD_OPCODE;
    }
    if (!ok) status = ST_BAD_DECODE;
  }
  return ReqFields{status, xid, op, arg, pl, dl, vc, poff, doff, voff, rel};
}

}  // namespace zk
