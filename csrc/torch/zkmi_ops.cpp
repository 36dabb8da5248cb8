// torch.ops.zkmi — the HIP batch codec (csrc/kernels, libzkmi_hip.so) as a
// PyTorch-ROCm operator library.
//
// Every op takes tensors, checks dtype / device / contiguity / length
// before a pointer reaches a kernel (a wrong tensor raises; it never
// corrupts memory), runs on the caller's current HIP stream and raises
// on a launch error.  The kernels' launchers are the extern "C" functions
// of libzkmi_hip.so; the batch descriptors they take (ZkReqBatch, ZkTree,
// ...) are assembled here from tensor lists in the field order of
// csrc/kernels/zk_batch.h and tree.hip.  Mutated arguments are marked
// (a!) in the schemas.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../kernels/zk_abi.h"


namespace {

using at::Tensor;
using c10::ScalarType;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void hip_ok(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "zkmi: ", what, " failed (hip error ", rc, ")");
}

const char* dtname(ScalarType t) { return c10::toString(t); }

// A device tensor of `dt`, contiguous, with at least `min_numel` elements,
// on the same device as `ref` (when given).
template <typename T>
T* P(const Tensor& t, ScalarType dt, int64_t min_numel, const char* name,
     const Tensor* ref = nullptr) {
  TORCH_CHECK(t.defined(), "zkmi: ", name, " is undefined");
  TORCH_CHECK(t.is_cuda(), "zkmi: ", name, " must be a GPU tensor, got ",
              t.device());
  TORCH_CHECK(t.scalar_type() == dt, "zkmi: ", name, " must be ",
              dtname(dt), ", got ", dtname(t.scalar_type()));
  TORCH_CHECK(t.is_contiguous(), "zkmi: ", name, " must be contiguous");
  TORCH_CHECK(t.numel() >= min_numel, "zkmi: ", name, " has ", t.numel(),
              " elements, needs ", min_numel);
  if (ref != nullptr)
    TORCH_CHECK(t.device() == ref->device(), "zkmi: ", name, " is on ",
                t.device(), ", expected ", ref->device());
  return reinterpret_cast<T*>(t.data_ptr());
}

template <typename T>
T* Popt(const c10::optional<Tensor>& t, ScalarType dt, int64_t min_numel,
        const char* name, const Tensor* ref = nullptr) {
  if (!t.has_value() || !t->defined()) return nullptr;
  return P<T>(*t, dt, min_numel, name, ref);
}

#define U8 ScalarType::Byte
#define I32 ScalarType::Int
#define I64 ScalarType::Long

void need(const std::vector<Tensor>& v, size_t k, const char* what) {
  TORCH_CHECK(v.size() == k, "zkmi: ", what, " needs ", k, " tensors, got ",
              v.size());
}

// -- descriptor assembly ---------------------------------------------------

// [opcode, xid, arg, path_off, path_len, data_off, data_len, acl_id,
//  path_arena, data_arena, acl_off, acl_len, acl_arena], n records
ZkReqBatch req_batch(const std::vector<Tensor>& b, int64_t n) {
  need(b, 13, "request batch");
  const Tensor* r = &b[0];
  ZkReqBatch s;
  s.opcode = P<int32_t>(b[0], I32, n, "batch.opcode", r);
  s.xid = P<int32_t>(b[1], I32, n, "batch.xid", r);
  s.arg = P<int32_t>(b[2], I32, n, "batch.arg", r);
  s.path_off = P<int64_t>(b[3], I64, n, "batch.path_off", r);
  s.path_len = P<int32_t>(b[4], I32, n, "batch.path_len", r);
  s.data_off = P<int64_t>(b[5], I64, n, "batch.data_off", r);
  s.data_len = P<int32_t>(b[6], I32, n, "batch.data_len", r);
  s.acl_id = P<int32_t>(b[7], I32, n, "batch.acl_id", r);
  s.path_arena = P<uint8_t>(b[8], U8, 1, "batch.path_arena", r);
  s.data_arena = P<uint8_t>(b[9], U8, 1, "batch.data_arena", r);
  s.acl_off = P<int64_t>(b[10], I64, 1, "batch.acl_off", r);
  s.acl_len = P<int32_t>(b[11], I32, 1, "batch.acl_len", r);
  s.acl_arena = P<uint8_t>(b[12], U8, 1, "batch.acl_arena", r);
  return s;
}

// [slab, slot_off, data_len, slot_cap]
ZkNodeStore node_store(const std::vector<Tensor>& v, size_t at,
                       const Tensor* r) {
  ZkNodeStore s;
  const int64_t cap = v[at + 1].numel();
  s.slab = P<uint8_t>(v[at], U8, 1, "store.slab", r);
  s.slot_off = P<int64_t>(v[at + 1], I64, 1, "store.slot_off", r);
  s.data_len = P<int32_t>(v[at + 2], I32, cap, "store.data_len", r);
  s.slot_cap = P<int32_t>(v[at + 3], I32, cap, "store.slot_cap", r);
  s.cap = cap;
  return s;
}

// [ht, node_path_off, node_path_len, node_parent, path_arena, counters,
//  slab, slot_off, data_len, slot_cap, free_list, cn, pzxid, dirty,
//  dirty_list, node_pw, node_path_cap, eph] + optionally [wt_key, wt_mask]
//  (watches); sizes give mask, caps
ZkTree tree(const std::vector<Tensor>& v) {
  TORCH_CHECK(v.size() == 18 || v.size() == 20,
              "zkmi: tree needs 18 tensors (20 with a watch table), got ",
              v.size());
  const Tensor* r = &v[0];
  ZkTree t;
  // 64-byte entries: key, val, lengths, the path's head (tree.hip HT_W)
  const int64_t hw = v[0].numel() / 8;
  TORCH_CHECK(hw > 0 && (hw & (hw - 1)) == 0 && v[0].numel() % 8 == 0,
              "zkmi: tree.ht must hold a power of two of 8-word entries");
  const int64_t cap = v[7].numel();
  t.ht = P<int64_t>(v[0], I64, 8, "tree.ht", r);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.ht) % 64 == 0,
              "zkmi: tree.ht must be 64-byte aligned");
  t.mask = hw - 1;
  t.node_path_off = P<int64_t>(v[1], I64, cap, "tree.node_path_off", r);
  t.node_path_len = P<int32_t>(v[2], I32, cap, "tree.node_path_len", r);
  t.node_parent = P<int64_t>(v[3], I64, cap, "tree.node_parent", r);
  t.path_arena = P<uint8_t>(v[4], U8, 1, "tree.path_arena", r);
  t.path_cap = v[4].numel();
  t.counters = P<int64_t>(v[5], I64, 9, "tree.counters", r);
  t.store = node_store(v, 6, r);
  t.slab_cap = v[6].numel();
  t.free_list = P<int64_t>(v[10], I64, 1, "tree.free_list", r);
  t.free_cap = v[10].numel();
  t.cn = P<int64_t>(v[11], I64, cap, "tree.cn", r);
  t.pzxid = P<int64_t>(v[12], I64, cap, "tree.pzxid", r);
  t.dirty = P<int32_t>(v[13], I32, cap, "tree.dirty", r);
  t.dirty_list = P<int64_t>(v[14], I64, cap, "tree.dirty_list", r);
  t.node_pw = P<int64_t>(v[15], I64, cap, "tree.node_pw", r);
  t.node_path_cap = P<int32_t>(v[16], I32, cap, "tree.node_path_cap", r);
  t.eph = P<int64_t>(v[17], I64, cap, "tree.eph", r);
  t.wt_key = nullptr;
  t.wt_mask = nullptr;
  t.wt_hmask = 0;
  if (v.size() == 20) {
    const int64_t h = v[18].numel();
    TORCH_CHECK(h > 0 && (h & (h - 1)) == 0,
                "zkmi: tree.wt_key must hold a power of two of entries");
    t.wt_key = P<int64_t>(v[18], I64, h, "tree.wt_key", r);
    t.wt_mask = reinterpret_cast<unsigned long long*>(
        P<int64_t>(v[19], I64, 2 * h, "tree.wt_mask", r));
    t.wt_hmask = h - 1;
  }
  t.seqno = nullptr;
  return t;
}

// [xid, err, opcode, status, zxid, stat64 [6, cap], stat32 [5, cap],
//  pay_off, pay_len, aux0, aux1]
ZkReplyOut reply_out(const std::vector<Tensor>& v, int64_t cap,
                     const Tensor* r) {
  need(v, 11, "reply table");
  ZkReplyOut o;
  o.xid = P<int32_t>(v[0], I32, cap, "reply.xid", r);
  o.err = P<int32_t>(v[1], I32, cap, "reply.err", r);
  o.opcode = P<int32_t>(v[2], I32, cap, "reply.opcode", r);
  o.status = P<int32_t>(v[3], I32, cap, "reply.status", r);
  o.zxid = P<int64_t>(v[4], I64, cap, "reply.zxid", r);
  TORCH_CHECK(v[5].dim() == 2 && v[5].size(0) == 6 && v[5].size(1) == cap,
              "zkmi: reply.stat64 must be [6, ", cap, "]");
  TORCH_CHECK(v[6].dim() == 2 && v[6].size(0) == 5 && v[6].size(1) == cap,
              "zkmi: reply.stat32 must be [5, ", cap, "]");
  o.stat64 = P<int64_t>(v[5], I64, 6 * cap, "reply.stat64", r);
  o.stat32 = P<int32_t>(v[6], I32, 5 * cap, "reply.stat32", r);
  o.pay_off = P<int64_t>(v[7], I64, cap, "reply.pay_off", r);
  o.pay_len = P<int32_t>(v[8], I32, cap, "reply.pay_len", r);
  o.aux0 = P<int32_t>(v[9], I32, cap, "reply.aux0", r);
  o.aux1 = P<int32_t>(v[10], I32, cap, "reply.aux1", r);
  o.cap = cap;
  return o;
}

// [xid, opcode, status, path_off, path_len, data_off, data_len, arg,
//  vec_off, vec_count, rel_zxid]
ZkReqOut req_out(const std::vector<Tensor>& v, int64_t cap, const Tensor* r) {
  need(v, 11, "request table");
  ZkReqOut o;
  o.xid = P<int32_t>(v[0], I32, cap, "req.xid", r);
  o.opcode = P<int32_t>(v[1], I32, cap, "req.opcode", r);
  o.status = P<int32_t>(v[2], I32, cap, "req.status", r);
  o.path_off = P<int64_t>(v[3], I64, cap, "req.path_off", r);
  o.path_len = P<int32_t>(v[4], I32, cap, "req.path_len", r);
  o.data_off = P<int64_t>(v[5], I64, cap, "req.data_off", r);
  o.data_len = P<int32_t>(v[6], I32, cap, "req.data_len", r);
  o.arg = P<int32_t>(v[7], I32, cap, "req.arg", r);
  o.vec_off = P<int64_t>(v[8], I64, cap, "req.vec_off", r);
  o.vec_count = P<int32_t>(v[9], I32, cap, "req.vec_count", r);
  o.rel_zxid = P<int64_t>(v[10], I64, cap, "req.rel_zxid", r);
  o.cap = cap;
  return o;
}

// [opcode, xid, err, node, zxid, path_off, path_len, path_arena, aux]
ZkRespBatch resp_batch(const std::vector<Tensor>& v,
                       const c10::optional<Tensor>& slot, int64_t cap,
                       const Tensor* r) {
  need(v, 9, "response batch");
  ZkRespBatch b;
  b.opcode = P<int32_t>(v[0], I32, cap, "resp.opcode", r);
  b.xid = P<int32_t>(v[1], I32, cap, "resp.xid", r);
  b.err = P<int32_t>(v[2], I32, cap, "resp.err", r);
  b.node = P<int64_t>(v[3], I64, cap, "resp.node", r);
  b.zxid = P<int64_t>(v[4], I64, cap, "resp.zxid", r);
  b.path_off = P<int64_t>(v[5], I64, cap, "resp.path_off", r);
  b.path_len = P<int32_t>(v[6], I32, cap, "resp.path_len", r);
  b.path_arena = P<uint8_t>(v[7], U8, 1, "resp.path_arena", r);
  b.aux = P<int32_t>(v[8], I32, cap, "resp.aux", r);
  b.slot = Popt<int64_t>(slot, I64, cap, "resp.slot", r);
  return b;
}

// [sid, passwd, timeout, state, next]
ZkSessionTable session_table(const std::vector<Tensor>& v, int64_t span) {
  need(v, 5, "session table");
  const Tensor* r = &v[0];
  const int64_t cap = v[0].numel();
  ZkSessionTable s;
  s.sid = P<int64_t>(v[0], I64, cap, "sessions.sid", r);
  s.passwd = P<uint8_t>(v[1], U8, 16 * cap, "sessions.passwd", r);
  s.timeout = P<int32_t>(v[2], I32, cap, "sessions.timeout", r);
  s.state = P<int32_t>(v[3], I32, cap, "sessions.state", r);
  s.next = P<int64_t>(v[4], I64, 1, "sessions.next", r);
  s.cap = cap;
  TORCH_CHECK(span >= 0 && span <= cap, "zkmi: sessions.span out of range");
  s.span = span;
  return s;
}

// -- ops ---------------------------------------------------------------------

int64_t scan_workspace(int64_t n) { return zk_scan_workspace(n); }
int64_t serve_tickets(int64_t ncap) { return zk_serve_tickets(ncap); }
int64_t scan_set_mode(int64_t m) { return zk_scan_set_mode((int)m); }
int64_t scan_small_mode() { return zk_scan_small_mode(); }

// the one-workgroup scan (K10 / K13 block sums) on a chosen engine
void scan_small(const Tensor& x, const Tensor& base, const Tensor& total,
                bool mfma) {
  const int64_t n = x.numel();
  hip_ok(zk_scan_small_i64_mode(P<int64_t>(x, I64, n, "x"),
                                P<int64_t>(base, I64, n, "base", &x), n,
                                P<int64_t>(total, I64, 1, "total", &x),
                                mfma ? 1 : 0, cur_stream()),
         "scan_small");
}

void scan_excl(const Tensor& x, const Tensor& base, const Tensor& total,
               const Tensor& ws) {
  const int64_t n = x.numel();
  auto b = P<int64_t>(base, I64, std::max<int64_t>(n, 1), "base", &x);
  auto t = P<int64_t>(total, I64, 1, "total", &x);
  auto w = P<int64_t>(ws, I64, zk_scan_workspace(std::max<int64_t>(n, 1)),
                      "ws", &x);
  if (x.scalar_type() == I32)
    hip_ok(zk_scan_excl_i32(P<int32_t>(x, I32, n, "x"), b, n, t, w,
                            cur_stream()), "scan_excl");
  else
    hip_ok(zk_scan_excl_i64(P<int64_t>(x, I64, n, "x"), b, n, t, w,
                            cur_stream()), "scan_excl");
}

void encode_requests(const std::vector<Tensor>& batch, int64_t n,
                     const Tensor& sizes, const Tensor& rec_off,
                     const Tensor& total, const Tensor& ws, const Tensor& out,
                     const c10::optional<Tensor>& xid_tab, int64_t xid_mask,
                     const Tensor& err, bool terminate) {
  ZkReqBatch b = req_batch(batch, n);
  const Tensor* r = &batch[0];
  const int64_t m = std::max<int64_t>(n, 1);
  int64_t* tab = Popt<int64_t>(xid_tab, I64, xid_mask + 1, "xid_tab", r);
  hip_ok(zk_encode_requests2(
             &b, n, P<int64_t>(sizes, I64, m, "sizes", r),
             P<int64_t>(rec_off, I64, m, "rec_off", r),
             P<int64_t>(total, I64, 1, "total", r),
             P<int64_t>(ws, I64, zk_scan_workspace(m), "ws", r),
             P<uint8_t>(out, U8, 1, "out", r), out.numel(), tab, xid_mask,
             P<int32_t>(err, I32, 1, "err", r), terminate ? 1 : 0,
             cur_stream()),
         "encode_requests");
}

// encode_requests with the sizes and block sums given (bench_gen_get wrote
// them): the encode's scan and write only
void encode_requests_presized(const std::vector<Tensor>& batch, int64_t n,
                              const Tensor& sizes, const Tensor& bsum,
                              const Tensor& rec_off, const Tensor& total,
                              const Tensor& ws, const Tensor& out,
                              const c10::optional<Tensor>& xid_tab,
                              int64_t xid_mask, const Tensor& err,
                              bool terminate) {
  ZkReqBatch b = req_batch(batch, n);
  const Tensor* r = &batch[0];
  const int64_t m = std::max<int64_t>(n, 1);
  int64_t* tab = Popt<int64_t>(xid_tab, I64, xid_mask + 1, "xid_tab", r);
  hip_ok(zk_encode_requests_presized(
             &b, n, P<int64_t>(sizes, I64, m, "sizes", r),
             P<int64_t>(bsum, I64, (m + 255) / 256, "bsum", r),
             P<int64_t>(rec_off, I64, m, "rec_off", r),
             P<int64_t>(total, I64, 1, "total", r),
             P<int64_t>(ws, I64, zk_scan_workspace(m), "ws", r),
             P<uint8_t>(out, U8, 1, "out", r), out.numel(), tab, xid_mask,
             P<int32_t>(err, I32, 1, "err", r), terminate ? 1 : 0,
             cur_stream()),
         "encode_requests_presized");
}

void encode_set_watches(const Tensor& poff, const Tensor& plen,
                        const Tensor& arena, int64_t n, int64_t c0,
                        int64_t c1, int64_t rel_zxid, const Tensor& sizes,
                        const Tensor& off, const Tensor& total,
                        const Tensor& ws, const Tensor& out,
                        const Tensor& err) {
  const int64_t m = std::max<int64_t>(n, 1);
  TORCH_CHECK(c0 >= 0 && c1 >= 0 && c0 + c1 <= n, "zkmi: bad vector split");
  hip_ok(zk_encode_set_watches(
             P<int64_t>(poff, I64, m, "poff"),
             P<int32_t>(plen, I32, m, "plen", &poff),
             P<uint8_t>(arena, U8, 1, "arena", &poff), n, c0, c1, rel_zxid,
             P<int64_t>(sizes, I64, m, "sizes", &poff),
             P<int64_t>(off, I64, m, "off", &poff),
             P<int64_t>(total, I64, 1, "total", &poff),
             P<int64_t>(ws, I64, zk_scan_workspace(m), "ws", &poff),
             P<uint8_t>(out, U8, 1, "out", &poff), out.numel(),
             P<int32_t>(err, I32, 1, "err", &poff), cur_stream()),
         "encode_set_watches");
}

void encode_connect_requests(const Tensor& proto, const Tensor& zxid,
                             const Tensor& tmo, const Tensor& sid,
                             const Tensor& pwo, const Tensor& pwl,
                             const Tensor& arena, int64_t n,
                             const Tensor& sizes, const Tensor& off,
                             const Tensor& total, const Tensor& ws,
                             const Tensor& out) {
  const int64_t m = std::max<int64_t>(n, 1);
  const Tensor* r = &proto;
  // frame + 28 fixed bytes + password per record
  TORCH_CHECK(out.numel() >= n * 32 + arena.numel() || n == 0,
              "zkmi: connect request out buffer too small");
  hip_ok(zk_encode_connect_requests(
             P<int32_t>(proto, I32, m, "proto"),
             P<int64_t>(zxid, I64, m, "zxid", r),
             P<int32_t>(tmo, I32, m, "timeout", r),
             P<int64_t>(sid, I64, m, "sid", r),
             P<int64_t>(pwo, I64, m, "passwd_off", r),
             P<int32_t>(pwl, I32, m, "passwd_len", r),
             P<uint8_t>(arena, U8, 1, "arena", r), n,
             P<int64_t>(sizes, I64, m, "sizes", r),
             P<int64_t>(off, I64, m, "off", r),
             P<int64_t>(total, I64, 1, "total", r),
             P<int64_t>(ws, I64, zk_scan_workspace(m), "ws", r),
             P<uint8_t>(out, U8, 1, "out", r), cur_stream()),
         "encode_connect_requests");
}

void encode_responses(const std::vector<Tensor>& resp,
                      const c10::optional<Tensor>& slot,
                      const std::vector<Tensor>& store, const Tensor& n_dev,
                      int64_t ncap, const Tensor& sizes, const Tensor& rec_off,
                      const Tensor& total, const Tensor& ws, const Tensor& out,
                      const Tensor& err, bool presized, bool terminate,
                      int64_t stage, bool prescanned) {
  TORCH_CHECK(!prescanned || presized,
              "zkmi: encode_responses prescanned needs presized");
  need(store, 4, "node store");
  const Tensor* r = &resp[0];
  ZkRespBatch b = resp_batch(resp, slot, ncap, r);
  ZkNodeStore s = node_store(store, 0, r);
  const int64_t m = std::max<int64_t>(ncap, 1);
  hip_ok(zk_encode_responses3(
             &b, &s, P<int64_t>(n_dev, I64, 1, "count", r), ncap,
             P<int64_t>(sizes, I64, m, "sizes", r),
             P<int64_t>(rec_off, I64, m, "rec_off", r),
             P<int64_t>(total, I64, 1, "total", r),
             P<int64_t>(ws, I64, zk_scan_workspace(m), "ws", r),
             P<uint8_t>(out, U8, 1, "out", r), out.numel(),
             P<int32_t>(err, I32, 1, "err", r),
             presized ? (prescanned ? 2 : 1) : 0,
             terminate ? 1 : 0, stage, cur_stream()),
         "encode_responses");
}

int64_t frame_scan_workspace(int64_t n) { return zk_frame_scan_workspace(n); }

void frame_scan(const Tensor& buf, const c10::optional<Tensor>& n_dev,
                int64_t n_cap, int64_t max_packet, const Tensor& ws,
                const Tensor& foff, const Tensor& flen, const Tensor& result,
                int64_t window, bool clean, int64_t flags) {
  TORCH_CHECK(n_cap >= 0 && n_cap <= buf.numel(),
              "zkmi: frame_scan length ", n_cap, " past the buffer (",
              buf.numel(), " bytes)");
  TORCH_CHECK(ws.numel() >= zk_frame_scan_workspace(n_cap),
              "zkmi: frame_scan workspace too small");
  const int64_t cap = foff.numel();
  hip_ok(zk_frame_scan5(
             P<uint8_t>(buf, U8, 1, "buf"),
             Popt<int64_t>(n_dev, I64, 1, "n", &buf), n_cap, max_packet,
             P<uint8_t>(ws, U8, 1, "ws", &buf), ws.numel(),
             P<int64_t>(foff, I64, 1, "frame_off", &buf),
             P<int32_t>(flen, I32, cap, "frame_len", &buf), cap,
             P<int64_t>(result, I64, 4, "result", &buf), (int32_t)window,
             clean ? 1 : 0, (int32_t)flags, cur_stream()),
         "frame_scan");
}

std::vector<int64_t> frame_scan_stats(const Tensor& ws, int64_t n_cap,
                                      int64_t window) {
  uint32_t o[4] = {0, 0, 0, 0};
  hip_ok(zk_frame_scan_stats(P<uint8_t>(ws, U8, 1, "ws"), n_cap,
                             (int32_t)window, o, cur_stream()),
         "frame_scan_stats");
  return {o[0], o[1], o[2], o[3]};
}

// Per-tile timing records of the last K1 run built with ZKMI_FS_DBG
// (tools/diag/k1_dbg.py): [tiles, 8] int64 on the host.
Tensor frame_scan_dbg(int64_t tiles) {
  Tensor out = at::zeros({tiles, 8}, at::kLong);
  hip_ok(zk_frame_scan_dbg(out.data_ptr<int64_t>(), tiles), "frame_scan_dbg");
  return out;
}

void decode_replies(const Tensor& buf, const Tensor& foff, const Tensor& flen,
                    const Tensor& n_dev, const Tensor& xid_tab,
                    int64_t xid_mask, const std::vector<Tensor>& out) {
  const int64_t cap = foff.numel();
  ZkReplyOut o = reply_out(out, cap, &buf);
  hip_ok(zk_decode_replies(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(foff, I64, cap, "frame_off", &buf),
             P<int32_t>(flen, I32, cap, "frame_len", &buf),
             P<int64_t>(n_dev, I64, 1, "count", &buf), cap,
             P<int64_t>(xid_tab, I64, xid_mask + 1, "xid_tab", &buf),
             xid_mask, &o, cur_stream()),
         "decode_replies");
}

// decode_replies + the fused GET_DATA check (bench validation): request i
// was (idx[i], xid[i]); counts of good replies go to acc (1..64 slots,
// summed by the caller).  slab + slot_off (the tree's node slots): one
// reply in 16 also has its payload bytes compared with its node's.
void decode_replies_check(const Tensor& buf, const Tensor& foff,
                          const Tensor& flen, const Tensor& n_dev,
                          const Tensor& xid_tab, int64_t xid_mask,
                          const std::vector<Tensor>& out, const Tensor& idx,
                          const Tensor& xid, const Tensor& data_len,
                          const Tensor& acc,
                          const c10::optional<Tensor>& tick,
                          const c10::optional<Tensor>& slab,
                          const c10::optional<Tensor>& slot_off) {
  const int64_t cap = foff.numel();
  ZkReplyOut o = reply_out(out, cap, &buf);
  const int32_t slots = (int32_t)std::min<int64_t>(acc.numel(), 64);
  TORCH_CHECK(slots >= 1, "zkmi: decode_replies_check needs an acc slot");
  TORCH_CHECK(slab.has_value() == slot_off.has_value(),
              "zkmi: decode_replies_check: slab and slot_off go together");
  // every slot_off entry the sampled idx can reach lies in data_len's range
  if (slot_off.has_value())
    TORCH_CHECK(slot_off->numel() >= data_len.numel(),
                "zkmi: decode_replies_check: slot_off shorter than data_len");
  hip_ok(zk_decode_replies_check2(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(foff, I64, cap, "frame_off", &buf),
             P<int32_t>(flen, I32, cap, "frame_len", &buf),
             P<int64_t>(n_dev, I64, 1, "count", &buf), cap,
             P<int64_t>(xid_tab, I64, xid_mask + 1, "xid_tab", &buf),
             xid_mask, &o, P<int64_t>(idx, I64, cap, "idx", &buf),
             P<int32_t>(xid, I32, cap, "xid", &buf),
             P<int32_t>(data_len, I32, 1, "data_len", &buf),
             reinterpret_cast<unsigned long long*>(
                 P<int64_t>(acc, I64, slots, "acc", &buf)),
             slots, Popt<int64_t>(tick, I64, 2, "tick", &buf),
             Popt<uint8_t>(slab, U8, 1, "slab", &buf),
             Popt<int64_t>(slot_off, I64, 1, "slot_off", &buf), cur_stream()),
         "decode_replies_check");
}

void expand_strings(const Tensor& buf, const Tensor& region,
                    const Tensor& count, const Tensor& base,
                    const Tensor& soff, const Tensor& slen) {
  const int64_t n = region.numel();
  hip_ok(zk_expand_strings(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(region, I64, n, "region", &buf),
             P<int32_t>(count, I32, n, "count", &buf),
             P<int64_t>(base, I64, n, "base", &buf), n,
             P<int64_t>(soff, I64, 1, "str_off", &buf),
             P<int32_t>(slen, I32, soff.numel(), "str_len", &buf),
             cur_stream()),
         "expand_strings");
}

void expand_acl(const Tensor& buf, const Tensor& region, const Tensor& count,
                const Tensor& base, const Tensor& perms, const Tensor& so,
                const Tensor& sl, const Tensor& io, const Tensor& il) {
  const int64_t n = region.numel();
  const int64_t m = perms.numel();
  hip_ok(zk_expand_acl(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(region, I64, n, "region", &buf),
             P<int32_t>(count, I32, n, "count", &buf),
             P<int64_t>(base, I64, n, "base", &buf), n,
             P<int32_t>(perms, I32, 1, "perms", &buf),
             P<int64_t>(so, I64, m, "scheme_off", &buf),
             P<int32_t>(sl, I32, m, "scheme_len", &buf),
             P<int64_t>(io, I64, m, "id_off", &buf),
             P<int32_t>(il, I32, m, "id_len", &buf), cur_stream()),
         "expand_acl");
}

void decode_requests(const Tensor& buf, const Tensor& foff,
                     const Tensor& flen, const Tensor& n_dev,
                     const std::vector<Tensor>& out) {
  const int64_t cap = foff.numel();
  ZkReqOut o = req_out(out, cap, &buf);
  hip_ok(zk_decode_requests(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(foff, I64, cap, "frame_off", &buf),
             P<int32_t>(flen, I32, cap, "frame_len", &buf),
             P<int64_t>(n_dev, I64, 1, "count", &buf), cap, &o,
             cur_stream()),
         "decode_requests");
}

void decode_connect_responses(const Tensor& buf, const Tensor& foff,
                              const Tensor& flen, int64_t n,
                              const Tensor& proto, const Tensor& tmo,
                              const Tensor& sid, const Tensor& pw_off,
                              const Tensor& pw_len, const Tensor& status) {
  const int64_t m = std::max<int64_t>(n, 1);
  hip_ok(zk_decode_connect_responses(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(foff, I64, n, "frame_off", &buf),
             P<int32_t>(flen, I32, n, "frame_len", &buf), n,
             P<int32_t>(proto, I32, m, "proto", &buf),
             P<int32_t>(tmo, I32, m, "timeout", &buf),
             P<int64_t>(sid, I64, m, "sid", &buf),
             P<int64_t>(pw_off, I64, m, "passwd_off", &buf),
             P<int32_t>(pw_len, I32, m, "passwd_len", &buf),
             P<int32_t>(status, I32, m, "status", &buf), cur_stream()),
         "decode_connect_responses");
}

void tree_fill(const std::vector<Tensor>& t, int64_t n0, int64_t n,
               const Tensor& nkids, int64_t now_ms) {
  ZkTree s = tree(t);
  TORCH_CHECK(n0 >= 0 && n <= s.store.cap, "zkmi: tree_fill range");
  hip_ok(zk_tree_fill(&s, n0, n, P<int32_t>(nkids, I32, n, "nkids", &t[0]),
                      now_ms, cur_stream()),
         "tree_fill");
}

int64_t tree_free_workspace(int64_t cap) {
  return zk_tree_free_workspace(cap);
}

void tree_free_compact(const std::vector<Tensor>& t, const Tensor& ws) {
  ZkTree s = tree(t);
  hip_ok(zk_tree_free_compact(
             &s, P<int64_t>(ws, I64, zk_tree_free_workspace(s.store.cap),
                            "ws", &t[0]),
             cur_stream()),
         "tree_free_compact");
}

// tree_finish + the presized reply encode's block-sum scan in one launch
// (ws: the response workspace the serve wrote its block sums into; total:
// the encode's total, then encode_responses(prescanned=True)).
void tree_finish_scan(const std::vector<Tensor>& t,
                      const c10::optional<Tensor>& n_dev, int64_t bump,
                      bool publish, int64_t ncap, const Tensor& ws,
                      const Tensor& total) {
  ZkTree s = tree(t);
  const int64_t nb = (ncap + 255) / 256;
  hip_ok(zk_tree_finish_scan(&s, Popt<int64_t>(n_dev, I64, 1, "count", &t[0]),
                             bump, publish ? 1 : 0, ncap,
                             P<int64_t>(ws, I64, 2 * nb, "ws", &t[0]),
                             P<int64_t>(total, I64, 1, "total", &t[0]),
                             cur_stream()),
         "tree_finish_scan");
}

void tree_ht_reset(const std::vector<Tensor>& t) {
  ZkTree s = tree(t);
  hip_ok(zk_tree_ht_reset(&s, cur_stream()), "tree_ht_reset");
}

void tree_build(const std::vector<Tensor>& t, int64_t n0, int64_t n) {
  ZkTree s = tree(t);
  TORCH_CHECK(n0 >= 0 && n <= s.store.cap, "zkmi: tree_build range");
  hip_ok(zk_tree_build(&s, n0, n, cur_stream()), "tree_build");
}

// r = [op, xid, err, node, zxid, path_off, path_len, slot, sizes, bsum]
void tree_serve(const std::vector<Tensor>& t, const Tensor& rx,
                const std::vector<Tensor>& q, const Tensor& n_dev,
                int64_t ncap, const std::vector<Tensor>& r, int64_t session,
                int64_t now_ms) {
  ZkTree s = tree(t);
  const Tensor* d = &t[0];
  ZkReqOut qo = req_out(q, ncap, d);
  need(r, 10, "serve outputs");
  const int64_t nb = (ncap + 255) / 256;
  hip_ok(zk_tree_serve(
             &s, P<uint8_t>(rx, U8, 1, "rx", d), &qo,
             P<int64_t>(n_dev, I64, 1, "count", d), ncap,
             P<int32_t>(r[0], I32, ncap, "r.opcode", d),
             P<int32_t>(r[1], I32, ncap, "r.xid", d),
             P<int32_t>(r[2], I32, ncap, "r.err", d),
             P<int64_t>(r[3], I64, ncap, "r.node", d),
             P<int64_t>(r[4], I64, ncap, "r.zxid", d),
             P<int64_t>(r[5], I64, ncap, "r.path_off", d),
             P<int32_t>(r[6], I32, ncap, "r.path_len", d),
             P<int64_t>(r[7], I64, ncap, "r.slot", d),
             P<int64_t>(r[8], I64, ncap, "r.sizes", d),
             P<int64_t>(r[9], I64, nb, "r.block_sums", d), session, now_ms,
             cur_stream()),
         "tree_serve");
}

// tree_serve from K1's frame table: each lane parses its request frame in
// registers (no K12 decode pass).
void tree_serve_frames(const std::vector<Tensor>& t, const Tensor& rx,
                       const Tensor& foff, const Tensor& flen,
                       const Tensor& n_dev, int64_t ncap,
                       const std::vector<Tensor>& r, int64_t session,
                       int64_t now_ms, int64_t wslot,
                       const c10::optional<Tensor>& fired,
                       const c10::optional<Tensor>& tickets, bool finish,
                       const c10::optional<Tensor>& seqno, bool read_only) {
  ZkTree s = tree(t);
  const Tensor* d = &t[0];
  need(r, 10, "serve outputs");
  s.seqno = Popt<int64_t>(seqno, I64, ncap, "seqno", d);
  TORCH_CHECK(wslot >= -1 && wslot < 64, "zkmi: watcher slot -1..63");
  const int64_t nb = (ncap + 255) / 256;
  hip_ok(zk_tree_serve_frames2(
             &s, P<uint8_t>(rx, U8, 1, "rx", d),
             P<int64_t>(foff, I64, ncap, "frame_off", d),
             P<int32_t>(flen, I32, ncap, "frame_len", d),
             P<int64_t>(n_dev, I64, 1, "count", d), ncap,
             P<int32_t>(r[0], I32, ncap, "r.opcode", d),
             P<int32_t>(r[1], I32, ncap, "r.xid", d),
             P<int32_t>(r[2], I32, ncap, "r.err", d),
             P<int64_t>(r[3], I64, ncap, "r.node", d),
             P<int64_t>(r[4], I64, ncap, "r.zxid", d),
             P<int64_t>(r[5], I64, ncap, "r.path_off", d),
             P<int32_t>(r[6], I32, ncap, "r.path_len", d),
             P<int64_t>(r[7], I64, ncap, "r.slot", d),
             P<int64_t>(r[8], I64, ncap, "r.sizes", d),
             P<int64_t>(r[9], I64, nb, "r.block_sums", d), session, now_ms,
             (int32_t)wslot, Popt<int64_t>(fired, I64, 5 * ncap, "fired", d),
             reinterpret_cast<unsigned*>(Popt<int32_t>(
                 tickets, I32, zk_serve_tickets(ncap), "tickets", d)),
             (finish ? ZK_SERVE_FINISH : 0) | (read_only ? ZK_SERVE_RO : 0),
             cur_stream()),
         "tree_serve_frames");
}

// The serve's finish on its own (after tree_serve_frames(..., finish=False)):
// zxid += *n_dev (or bump when n_dev is None).
void tree_finish(const std::vector<Tensor>& t, const c10::optional<Tensor>& n_dev,
                 int64_t bump, bool publish) {
  ZkTree s = tree(t);
  hip_ok(zk_tree_finish(&s, Popt<int64_t>(n_dev, I64, 1, "count", &t[0]), bump,
                        publish ? 1 : 0, cur_stream()),
         "tree_finish");
}

int64_t tree_order_workspace(int64_t n) {
  TORCH_CHECK(n >= 0, "zkmi: tree_order_workspace n");
  return zk_tree_order_workspace(n);
}

int64_t tree_order_stats_offset(int64_t n) {
  TORCH_CHECK(n >= 0, "zkmi: tree_order_stats_offset n");
  return zk_tree_order_stats_offset(n);
}

// tree_serve with same-path requests applied in batch order over `passes`
// launches.  `scratch` (optional) is the slab's tail past the tree's view of
// it (t[6] = slab[:cap]); snapshot replies are written there and named by
// their offset from the slab start, so the encoder must be given the whole
// slab.
void tree_serve_ordered(const std::vector<Tensor>& t, const Tensor& rx,
                        const std::vector<Tensor>& q, const Tensor& n_dev,
                        int64_t ncap, const std::vector<Tensor>& r,
                        int64_t session, int64_t now_ms, const Tensor& ws,
                        int64_t passes, const c10::optional<Tensor>& scratch,
                        int64_t wslot, const c10::optional<Tensor>& fired,
                        const c10::optional<Tensor>& seqno) {
  TORCH_CHECK(wslot >= -1 && wslot < 64, "zkmi: watcher slot -1..63");
  ZkTree s = tree(t);
  const Tensor* d = &t[0];
  s.seqno = Popt<int64_t>(seqno, I64, ncap, "seqno", d);
  ZkReqOut qo = req_out(q, ncap, d);
  need(r, 10, "serve outputs");
  TORCH_CHECK(passes >= 1 && passes <= 127, "zkmi: passes in 1..127");
  const int64_t need_ws = zk_tree_order_workspace(ncap);
  uint8_t* w = P<uint8_t>(ws, U8, need_ws, "order workspace", d);
  int64_t snap_base = 0, snap_cap = 0;
  if (scratch.has_value() && scratch->defined()) {
    const Tensor& sc = *scratch;
    P<uint8_t>(sc, U8, 0, "scratch", d);
    TORCH_CHECK(sc.storage().is_alias_of(t[6].storage()),
                "zkmi: scratch must be a view of the tree's slab");
    snap_base = (int64_t)((const uint8_t*)sc.data_ptr() -
                          (const uint8_t*)t[6].data_ptr());
    TORCH_CHECK(snap_base >= s.slab_cap && snap_base % 16 == 0,
                "zkmi: scratch must start 16-aligned past the tree's slab");
    snap_cap = sc.numel();
  }
  const int64_t nb = (ncap + 255) / 256;
  hip_ok(zk_tree_serve_ordered(
             &s, P<uint8_t>(rx, U8, 1, "rx", d), &qo,
             P<int64_t>(n_dev, I64, 1, "count", d), ncap,
             P<int32_t>(r[0], I32, ncap, "r.opcode", d),
             P<int32_t>(r[1], I32, ncap, "r.xid", d),
             P<int32_t>(r[2], I32, ncap, "r.err", d),
             P<int64_t>(r[3], I64, ncap, "r.node", d),
             P<int64_t>(r[4], I64, ncap, "r.zxid", d),
             P<int64_t>(r[5], I64, ncap, "r.path_off", d),
             P<int32_t>(r[6], I32, ncap, "r.path_len", d),
             P<int64_t>(r[7], I64, ncap, "r.slot", d),
             P<int64_t>(r[8], I64, ncap, "r.sizes", d),
             P<int64_t>(r[9], I64, nb, "r.block_sums", d), session, now_ms,
             w, ws.numel(), (int32_t)passes, snap_base, snap_cap,
             (int32_t)wslot, Popt<int64_t>(fired, I64, 5 * ncap, "fired", d),
             cur_stream()),
         "tree_serve_ordered");
}

void watch_events(const Tensor& r_op, const Tensor& r_err, const Tensor& n_dev,
                  int64_t ncap, const Tensor& fired, const Tensor& bsum,
                  const Tensor& ev_slot, const Tensor& ev_type,
                  const Tensor& ev_poff, const Tensor& ev_plen,
                  const Tensor& ev_total) {
  const Tensor* d = &r_op;
  const int64_t cap = ev_slot.numel();
  hip_ok(zk_watch_events(
             P<int32_t>(r_op, I32, ncap, "r.opcode"),
             P<int32_t>(r_err, I32, ncap, "r.err", d),
             P<int64_t>(n_dev, I64, 1, "count", d), ncap,
             P<int64_t>(fired, I64, 5 * ncap, "fired", d),
             P<int64_t>(bsum, I64, (ncap + 255) / 256, "bsum", d), cap,
             P<int32_t>(ev_slot, I32, cap, "ev_slot", d),
             P<int32_t>(ev_type, I32, cap, "ev_type", d),
             P<int64_t>(ev_poff, I64, cap, "ev_path_off", d),
             P<int32_t>(ev_plen, I32, cap, "ev_path_len", d),
             P<int64_t>(ev_total, I64, 2, "ev_total", d), cur_stream()),
         "watch_events");
}

void watch_resume(const std::vector<Tensor>& t, const Tensor& rx,
                  const Tensor& foff, const Tensor& flen, const Tensor& n_dev,
                  int64_t ncap, int64_t wslot, const Tensor& ent,
                  const Tensor& ev_type, const Tensor& ev_poff,
                  const Tensor& ev_plen, const Tensor& out) {
  ZkTree s = tree(t);
  TORCH_CHECK(s.wt_key != nullptr, "zkmi: watch_resume needs a watch table");
  TORCH_CHECK(wslot >= 0 && wslot < 64, "zkmi: watcher slot 0..63");
  const Tensor* d = &t[0];
  const int64_t cap = ev_type.numel();
  hip_ok(zk_watch_resume(
             &s, P<uint8_t>(rx, U8, 1, "rx", d),
             P<int64_t>(foff, I64, ncap, "frame_off", d),
             P<int32_t>(flen, I32, ncap, "frame_len", d),
             P<int64_t>(n_dev, I64, 1, "count", d), ncap, (int32_t)wslot,
             P<int64_t>(ent, I64, 1, "ent", d), ent.numel(), cap,
             P<int32_t>(ev_type, I32, cap, "ev_type", d),
             P<int64_t>(ev_poff, I64, cap, "ev_path_off", d),
             P<int32_t>(ev_plen, I32, cap, "ev_path_len", d),
             P<int64_t>(out, I64, 3, "out", d), cur_stream()),
         "watch_resume");
}

// SEQUENTIAL numbers in stream order (tree.hip seq_*): workspace bytes for
// ncap requests (zero the first tree_seq_zeroed(ncap) once), then per batch
// the ordering of the request frames -> seqno (int64 [ncap]) for the serve.
int64_t tree_seq_workspace(int64_t n) {
  TORCH_CHECK(n >= 0, "zkmi: tree_seq_workspace n");
  return zk_tree_seq_workspace(n);
}

int64_t tree_seq_zeroed(int64_t n) {
  TORCH_CHECK(n >= 0, "zkmi: tree_seq_zeroed n");
  return zk_tree_seq_zeroed(n);
}

void tree_seq_order(const std::vector<Tensor>& t, const Tensor& rx,
                    const Tensor& foff, const Tensor& flen, const Tensor& n_dev,
                    int64_t ncap, const Tensor& ws, const Tensor& seqno) {
  ZkTree s = tree(t);
  const Tensor* d = &t[0];
  TORCH_CHECK(ncap <= (1 << 24), "zkmi: tree_seq_order: ncap <= 16M");
  hip_ok(zk_tree_seq_order(
             &s, P<uint8_t>(rx, U8, 1, "rx", d),
             P<int64_t>(foff, I64, ncap, "frame_off", d),
             P<int32_t>(flen, I32, ncap, "frame_len", d),
             P<int64_t>(n_dev, I64, 1, "count", d), ncap,
             P<uint8_t>(ws, U8, zk_tree_seq_workspace(ncap), "seq workspace",
                        d),
             ws.numel(), P<int64_t>(seqno, I64, ncap, "seqno", d),
             cur_stream()),
         "tree_seq_order");
}

// seq_group_k's phase clocks into buf (int64, 5 per 1024-request chunk of
// the batches that follow; an empty tensor turns them off)
void tree_seq_debug(const Tensor& buf) {
  if (buf.numel() == 0) {
    zk_tree_seq_debug(nullptr);
    return;
  }
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kLong &&
                  buf.is_contiguous(),
              "zkmi: tree_seq_debug wants a contiguous device int64 tensor");
  zk_tree_seq_debug(buf.data_ptr<int64_t>());
}

// tree_expire_k's phase clocks into buf (int32, 4 per node slot: start,
// lookup + tombstone, backward shift, whole thread; an empty tensor turns
// them off).  buf must cover 4 x the tree's node capacity.
void tree_expire_debug(const Tensor& buf) {
  if (buf.numel() == 0) {
    zk_tree_expire_debug(nullptr);
    return;
  }
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kInt &&
                  buf.is_contiguous(),
              "zkmi: tree_expire_debug wants a contiguous device int32 tensor");
  zk_tree_expire_debug(buf.data_ptr<int32_t>());
}

// out (int64 [4]): node digest, live nodes, hash entries used, tombstones
void tree_digest(const std::vector<Tensor>& t, const Tensor& out) {
  ZkTree s = tree(t);
  hip_ok(zk_tree_digest(&s,
                        reinterpret_cast<unsigned long long*>(
                            P<int64_t>(out, I64, 4, "digest", &t[0])),
                        cur_stream()),
         "tree_digest");
}

void tree_expire(const std::vector<Tensor>& t, int64_t session, int64_t ncap,
                 const Tensor& removed) {
  ZkTree s = tree(t);
  TORCH_CHECK(ncap <= s.store.cap, "zkmi: tree_expire range");
  hip_ok(zk_tree_expire(&s, session, ncap,
                        reinterpret_cast<unsigned long long*>(P<int64_t>(
                            removed, I64, 1, "removed", &t[0])),
                        cur_stream()),
         "tree_expire");
}

void bench_gen_get(int64_t n, int64_t seed, int64_t leaf0, int64_t nleaves,
                   int64_t xid_base, const Tensor& node_pw, const Tensor& idx,
                   const Tensor& xid, const Tensor& poff, const Tensor& plen,
                   const c10::optional<Tensor>& state,
                   const c10::optional<Tensor>& sizes,
                   const c10::optional<Tensor>& bsum) {
  TORCH_CHECK(sizes.has_value() == bsum.has_value(),
              "zkmi: bench_gen_get: sizes and bsum together");
  TORCH_CHECK(leaf0 >= 0 && leaf0 + nleaves <= node_pw.numel(),
              "zkmi: bench_gen_get leaf range");
  TORCH_CHECK(nleaves > 0, "zkmi: bench_gen_get needs leaves");
  hip_ok(zk_bench_gen_get(n, (uint64_t)seed, leaf0, nleaves,
                          (int32_t)xid_base,
                          P<int64_t>(node_pw, I64, 1, "node_pw"),
                          P<int64_t>(idx, I64, n, "idx", &node_pw),
                          P<int32_t>(xid, I32, n, "xid", &node_pw),
                          P<int64_t>(poff, I64, n, "path_off", &node_pw),
                          P<int32_t>(plen, I32, n, "path_len", &node_pw),
                          Popt<int64_t>(state, I64, 2, "state", &node_pw),
                          Popt<int64_t>(sizes, I64, n, "sizes", &node_pw),
                          Popt<int64_t>(bsum, I64, (n + 255) / 256, "bsum",
                                        &node_pw),
                          cur_stream()),
         "bench_gen_get");
}

// the storm's handshake check + credential update (bench.hip)
void bench_storm_hs(bool resume, bool prev, int64_t timeout,
                    const Tensor& status, const Tensor& sid, const Tensor& tmo,
                    const Tensor& outcome, const Tensor& bound,
                    const Tensor& resp, const Tensor& want,
                    const Tensor& cred_sid, const Tensor& cred_pw,
                    const Tensor& hs_ok) {
  const Tensor* d = &status;
  const int64_t m = resume && prev ? 2 : 1;
  TORCH_CHECK(hs_ok.scalar_type() == at::kBool && hs_ok.is_cuda(),
              "zkmi: bench_storm_hs hs_ok");
  hip_ok(zk_bench_storm_hs(
             resume ? 1 : 0, prev ? 1 : 0, (int32_t)timeout,
             P<int32_t>(status, I32, m, "status", d),
             P<int64_t>(sid, I64, m, "sessionId", d),
             P<int32_t>(tmo, I32, m, "timeOut", d),
             P<int32_t>(outcome, I32, m, "outcome", d),
             P<int64_t>(bound, I64, 1, "bound", d),
             P<uint8_t>(resp, U8, 40, "resp", d),
             P<int64_t>(want, I64, 1, "want", d),
             P<int64_t>(cred_sid, I64, 2, "cred_sid", d),
             P<uint8_t>(cred_pw, U8, 32, "cred_pw", d),
             hs_ok.data_ptr<bool>(), cur_stream()),
         "bench_storm_hs");
}

void bench_xids(int64_t n, const Tensor& base, const Tensor& xid) {
  hip_ok(zk_bench_xids(n, P<int64_t>(base, I64, 1, "xid base"),
                       P<int32_t>(xid, I32, n, "xid", &base), cur_stream()),
         "bench_xids");
}

// reply: the decode's SoA (status, err, xid, pay_len, zxid used); want_len
// per request, or want_len_c >= 0 for all
void bench_check_writes(int64_t n, const Tensor& status, const Tensor& err,
                        const Tensor& rxid, const Tensor& xid,
                        const Tensor& pay_len,
                        const c10::optional<Tensor>& want_len,
                        int64_t want_len_c, const Tensor& zxid,
                        const Tensor& ok, const Tensor& zmax) {
  TORCH_CHECK(want_len.has_value() || want_len_c >= 0,
              "zkmi: bench_check_writes needs a want_len");
  const Tensor* d = &status;
  hip_ok(zk_bench_check_writes(
             n, P<int32_t>(status, I32, n, "status", d),
             P<int32_t>(err, I32, n, "err", d),
             P<int32_t>(rxid, I32, n, "reply xid", d),
             P<int32_t>(xid, I32, n, "xid", d),
             P<int32_t>(pay_len, I32, n, "pay_len", d),
             Popt<int32_t>(want_len, I32, n, "want_len", d),
             (int32_t)want_len_c, P<int64_t>(zxid, I64, n, "zxid", d),
             reinterpret_cast<unsigned long long*>(
                 P<int64_t>(ok, I64, 1, "ok", d)),
             reinterpret_cast<unsigned long long*>(
                 P<int64_t>(zmax, I64, 1, "zmax", d)),
             cur_stream()),
         "bench_check_writes");
}

void bench_check_get(int64_t n, const std::vector<Tensor>& reply,
                     const Tensor& idx, const Tensor& xid,
                     const Tensor& data_len, const Tensor& acc) {
  const int64_t cap = reply[0].numel();
  TORCH_CHECK(n <= cap, "zkmi: bench_check_get n past the reply table");
  ZkReplyOut o = reply_out(reply, cap, &idx);
  hip_ok(zk_bench_check_get(
             n, o.status, o.err, o.opcode, o.xid, o.stat64, o.pay_len,
             P<int64_t>(idx, I64, n, "idx"),
             P<int32_t>(xid, I32, n, "xid", &idx),
             P<int32_t>(data_len, I32, 1, "data_len", &idx),
             reinterpret_cast<unsigned long long*>(
                 P<int64_t>(acc, I64, 1, "acc", &idx)),
             cur_stream()),
         "bench_check_get");
}

void bench_check_notif(int64_t total, int64_t n_per, const Tensor& seeds,
                       int64_t leaf0, int64_t nleaves,
                       const Tensor& node_path_off,
                       const Tensor& node_path_len, const Tensor& path_arena,
                       const Tensor& rx, const std::vector<Tensor>& reply,
                       const Tensor& acc, const c10::optional<Tensor>& want) {
  const int64_t cap = reply[0].numel();
  TORCH_CHECK(total <= cap, "zkmi: bench_check_notif past the reply table");
  const bool have_want = want.has_value() && want->defined();
  TORCH_CHECK(have_want || (n_per > 0 && seeds.numel() * n_per >= total),
              "zkmi: bench_check_notif seeds");
  ZkReplyOut o = reply_out(reply, cap, &rx);
  hip_ok(zk_bench_check_notif(
             total, n_per,
             reinterpret_cast<const uint64_t*>(
                 P<int64_t>(seeds, I64, 1, "seeds", &rx)),
             Popt<int64_t>(want, I64, total, "want", &rx), leaf0, nleaves,
             P<int64_t>(node_path_off, I64, leaf0 + nleaves,
                        "node_path_off", &rx),
             P<int32_t>(node_path_len, I32, leaf0 + nleaves,
                        "node_path_len", &rx),
             P<uint8_t>(path_arena, U8, 1, "path_arena", &rx),
             P<uint8_t>(rx, U8, 1, "rx"), o.status, o.err, o.opcode, o.aux0,
             o.aux1, o.pay_off, o.pay_len,
             reinterpret_cast<unsigned long long*>(
                 P<int64_t>(acc, I64, 1, "acc", &rx)),
             cur_stream()),
         "bench_check_notif");
}

int64_t route_workspace(int64_t n, int64_t world) {
  return zk_route_workspace(n, (int32_t)world);
}

void route_requests(int64_t n, int64_t world, const Tensor& poff,
                    const Tensor& plen, const Tensor& arena,
                    const Tensor& idx, const Tensor& xid, const Tensor& owner,
                    const Tensor& idx_s, const Tensor& xid_s,
                    const Tensor& poff_s, const Tensor& plen_s,
                    const Tensor& counts, const Tensor& ws, int64_t self) {
  TORCH_CHECK(world >= 1 && world <= 64, "zkmi: route world 1..64");
  TORCH_CHECK(self >= 0 && self < world, "zkmi: route self rank");
  const Tensor* r = &poff;
  hip_ok(zk_route_requests2(
             n, (int32_t)world, (int32_t)self,
             P<int64_t>(poff, I64, n, "path_off"),
             P<int32_t>(plen, I32, n, "path_len", r),
             P<uint8_t>(arena, U8, 1, "arena", r),
             P<int64_t>(idx, I64, n, "idx", r),
             P<int32_t>(xid, I32, n, "xid", r),
             P<int32_t>(owner, I32, n, "owner", r),
             P<int64_t>(idx_s, I64, n, "idx_s", r),
             P<int32_t>(xid_s, I32, n, "xid_s", r),
             P<int64_t>(poff_s, I64, n, "path_off_s", r),
             P<int32_t>(plen_s, I32, n, "path_len_s", r),
             P<int64_t>(counts, I64, world, "counts", r),
             P<int64_t>(ws, I64, zk_route_workspace(n, (int32_t)world),
                        "ws", r),
             cur_stream()),
         "route_requests");
}

void seg_pack(const Tensor& src, const Tensor& rec_off,
              const c10::optional<Tensor>& nrec, int64_t nrec_cap,
              const Tensor& total, const Tensor& counts, int64_t world,
              int64_t self, int64_t slot_cap, const Tensor& out,
              const Tensor& stats, const c10::optional<Tensor>& self_out,
              bool inplace) {
  TORCH_CHECK(!inplace || self_out.has_value(),
              "zkmi: seg_pack inplace needs the self header (self_out)");
  TORCH_CHECK(world >= 1 && world <= 64, "zkmi: seg_pack world 1..64");
  TORCH_CHECK(self >= 0 && self < world, "zkmi: seg_pack self rank");
  TORCH_CHECK(slot_cap >= 32 && slot_cap % 16 == 0,
              "zkmi: seg_pack slot_cap must be a multiple of 16, >= 32");
  TORCH_CHECK(nrec_cap >= 0, "zkmi: seg_pack nrec_cap");
  const Tensor* r = &src;
  hip_ok(zk_seg_pack(P<uint8_t>(src, U8, 1, "src"), src.numel(),
                     P<int64_t>(rec_off, I64, std::max<int64_t>(nrec_cap, 1),
                                "rec_off", r),
                     Popt<int64_t>(nrec, I64, 1, "nrec", r), nrec_cap,
                     P<int64_t>(total, I64, 1, "total", r),
                     P<int64_t>(counts, I64, world, "counts", r),
                     (int32_t)world, (int32_t)self, slot_cap,
                     P<uint8_t>(out, U8,
                                self_out ? (world - 1) * slot_cap + 16
                                         : world * slot_cap, "out", r),
                     reinterpret_cast<unsigned long long*>(
                         P<int64_t>(stats, I64, 3, "stats", r)),
                     Popt<uint8_t>(self_out, U8, inplace ? 16 : slot_cap,
                                   "self_out", r),
                     inplace ? 1 : 0, cur_stream()),
         "seg_pack");
}

void seg_unpack(const Tensor& inp, int64_t world, int64_t self,
                int64_t slot_cap, const Tensor& out, const Tensor& total,
                const Tensor& counts, const c10::optional<Tensor>& stats,
                const c10::optional<Tensor>& self_in, bool inplace) {
  TORCH_CHECK(!inplace || self_in.has_value(),
              "zkmi: seg_unpack inplace needs the self header (self_in)");
  TORCH_CHECK(world >= 1 && world <= 64, "zkmi: seg_unpack world 1..64");
  TORCH_CHECK(self >= 0 && self < world, "zkmi: seg_unpack self rank");
  TORCH_CHECK(slot_cap >= 32 && slot_cap % 16 == 0,
              "zkmi: seg_unpack slot_cap must be a multiple of 16, >= 32");
  const Tensor* r = &inp;
  hip_ok(zk_seg_unpack(P<uint8_t>(inp, U8,
                                 self_in ? (world - 1) * slot_cap + 16
                                         : world * slot_cap, "in"),
                       (int32_t)world, (int32_t)self, slot_cap,
                       P<uint8_t>(out, U8, world * (slot_cap - 16), "out", r),
                       P<int64_t>(total, I64, 1, "total", r),
                       P<int64_t>(counts, I64, world, "counts", r),
                       reinterpret_cast<unsigned long long*>(
                           Popt<int64_t>(stats, I64, 1, "stats", r)),
                       Popt<uint8_t>(self_in, U8, inplace ? 16 : slot_cap,
                                     "self_in", r),
                       inplace ? 1 : 0, cur_stream()),
         "seg_unpack");
}

void session_connect(const Tensor& buf, const Tensor& foff,
                     const Tensor& flen, const Tensor& n_dev, int64_t ncap,
                     const std::vector<Tensor>& tab, int64_t server_id,
                     int64_t secret, int64_t min_to, int64_t max_to,
                     const Tensor& zxid_now, const Tensor& out,
                     const Tensor& resp_sid, const Tensor& outcome,
                     int64_t span) {
  ZkSessionTable s = session_table(tab, span);
  // a member's slots are [(server_id - 1) * span, server_id * span)
  TORCH_CHECK(server_id >= 1 && server_id < 128 &&
                  (span == 0 || server_id * span <= s.cap),
              "zkmi: session_connect server_id out of range for the span");
  const Tensor* r = &buf;
  hip_ok(zk_session_connect(
             P<uint8_t>(buf, U8, 1, "buf"),
             P<int64_t>(foff, I64, ncap, "frame_off", r),
             P<int32_t>(flen, I32, ncap, "frame_len", r),
             P<int64_t>(n_dev, I64, 1, "count", r), ncap, &s, server_id,
             (uint64_t)secret, (int32_t)min_to, (int32_t)max_to,
             P<int64_t>(zxid_now, I64, 1, "zxid_now", r),
             P<uint8_t>(out, U8, 41 * ncap, "out", r),
             P<int64_t>(resp_sid, I64, ncap, "resp_sid", r),
             P<int32_t>(outcome, I32, ncap, "outcome", r), cur_stream()),
         "session_connect");
}

void session_close(const std::vector<Tensor>& tab, const Tensor& sids,
                   int64_t server_id, int64_t span) {
  ZkSessionTable s = session_table(tab, span);
  hip_ok(zk_session_close(&s, P<int64_t>(sids, I64, 0, "sids", &tab[0]),
                          sids.numel(), server_id, cur_stream()),
         "session_close");
}

void session_install(const std::vector<Tensor>& tab, const Tensor& rec,
                     int64_t server_id, int64_t span) {
  ZkSessionTable s = session_table(tab, span);
  TORCH_CHECK(rec.numel() % 4 == 0, "zkmi: session records are 4 x int64");
  hip_ok(zk_session_install(&s, P<int64_t>(rec, I64, 0, "records", &tab[0]),
                            rec.numel() / 4, server_id, cur_stream()),
         "session_install");
}

}  // namespace

TORCH_LIBRARY(zkmi, m) {
  m.def("scan_workspace(int n) -> int", &scan_workspace);
  m.def("scan_set_mode(int mode) -> int", &scan_set_mode);
  m.def("scan_small_mode() -> int", &scan_small_mode);
  m.def("scan_small(Tensor x, Tensor(a!) base, Tensor(b!) total, "
        "bool mfma) -> ()", &scan_small);
  m.def("scan_excl(Tensor x, Tensor(a!) base, Tensor(b!) total, "
        "Tensor(c!) ws) -> ()", &scan_excl);
  m.def("encode_requests(Tensor[] batch, int n, Tensor(a!) sizes, "
        "Tensor(b!) rec_off, Tensor(c!) total, Tensor(d!) ws, "
        "Tensor(e!) out, Tensor(f!)? xid_tab, int xid_mask, Tensor(g!) err, "
        "bool terminate) -> ()", &encode_requests);
  m.def("encode_requests_presized(Tensor[] batch, int n, Tensor sizes, "
        "Tensor bsum, Tensor(b!) rec_off, Tensor(c!) total, Tensor(d!) ws, "
        "Tensor(e!) out, Tensor(f!)? xid_tab, int xid_mask, Tensor(g!) err, "
        "bool terminate) -> ()", &encode_requests_presized);
  m.def("encode_set_watches(Tensor poff, Tensor plen, Tensor arena, int n, "
        "int c0, int c1, int rel_zxid, Tensor(a!) sizes, Tensor(b!) off, "
        "Tensor(c!) total, Tensor(d!) ws, Tensor(e!) out, Tensor(f!) err) "
        "-> ()", &encode_set_watches);
  m.def("encode_connect_requests(Tensor proto, Tensor zxid, Tensor timeout, "
        "Tensor sid, Tensor passwd_off, Tensor passwd_len, Tensor arena, "
        "int n, Tensor(a!) sizes, Tensor(b!) off, Tensor(c!) total, "
        "Tensor(d!) ws, Tensor(e!) out) -> ()", &encode_connect_requests);
  m.def("encode_responses(Tensor[] resp, Tensor? slot, Tensor[] store, "
        "Tensor count, int ncap, Tensor(a!) sizes, Tensor(b!) rec_off, "
        "Tensor(c!) total, Tensor(d!) ws, Tensor(e!) out, Tensor(f!) err, "
        "bool presized, bool terminate, int stage=0, "
        "bool prescanned=False) -> ()",
        &encode_responses);
  m.def("frame_scan_workspace(int n) -> int", &frame_scan_workspace);
  m.def("frame_scan(Tensor buf, Tensor? n, int n_cap, int max_packet, "
        "Tensor(a!) ws, Tensor(b!) frame_off, Tensor(c!) frame_len, "
        "Tensor(d!) result, int window, bool clean=False, int flags=0) "
        "-> ()",
        &frame_scan);
  m.def("frame_scan_stats(Tensor ws, int n_cap, int window) -> int[]",
        &frame_scan_stats);
  m.def("frame_scan_dbg(int tiles) -> Tensor", &frame_scan_dbg);
  m.def("decode_replies(Tensor buf, Tensor frame_off, Tensor frame_len, "
        "Tensor count, Tensor xid_tab, int xid_mask, Tensor(a!)[] out) -> ()",
        &decode_replies);
  m.def("decode_replies_check(Tensor buf, Tensor frame_off, Tensor frame_len, "
        "Tensor count, Tensor xid_tab, int xid_mask, Tensor(a!)[] out, "
        "Tensor idx, Tensor xid, Tensor data_len, Tensor(b!) acc, "
        "Tensor(c!)? tick=None, Tensor? slab=None, Tensor? slot_off=None) "
        "-> ()",
        &decode_replies_check);
  m.def("expand_strings(Tensor buf, Tensor region, Tensor count, "
        "Tensor base, Tensor(a!) str_off, Tensor(b!) str_len) -> ()",
        &expand_strings);
  m.def("expand_acl(Tensor buf, Tensor region, Tensor count, Tensor base, "
        "Tensor(a!) perms, Tensor(b!) scheme_off, Tensor(c!) scheme_len, "
        "Tensor(d!) id_off, Tensor(e!) id_len) -> ()", &expand_acl);
  m.def("decode_requests(Tensor buf, Tensor frame_off, Tensor frame_len, "
        "Tensor count, Tensor(a!)[] out) -> ()", &decode_requests);
  m.def("decode_connect_responses(Tensor buf, Tensor frame_off, "
        "Tensor frame_len, int n, Tensor(a!) proto, Tensor(b!) timeout, "
        "Tensor(c!) sid, Tensor(d!) passwd_off, Tensor(e!) passwd_len, "
        "Tensor(f!) status) -> ()", &decode_connect_responses);
  m.def("tree_fill(Tensor(a!)[] tree, int n0, int n, Tensor nkids, "
        "int now_ms) -> ()", &tree_fill);
  m.def("tree_build(Tensor(a!)[] tree, int n0, int n) -> ()", &tree_build);
  m.def("tree_ht_reset(Tensor(a!)[] tree) -> ()", &tree_ht_reset);
  m.def("tree_finish_scan(Tensor(a!)[] tree, Tensor? count, int bump, "
        "bool publish, int ncap, Tensor(b!) ws, Tensor(c!) total) -> ()",
        &tree_finish_scan);
  m.def("tree_free_workspace(int cap) -> int", &tree_free_workspace);
  m.def("tree_free_compact(Tensor(a!)[] tree, Tensor(b!) ws) -> ()",
        &tree_free_compact);
  m.def("tree_serve(Tensor(a!)[] tree, Tensor rx, Tensor[] requests, "
        "Tensor count, int ncap, Tensor(b!)[] out, int session, int now_ms) "
        "-> ()", &tree_serve);
  m.def("tree_serve_frames(Tensor(a!)[] tree, Tensor rx, Tensor frame_off, "
        "Tensor frame_len, Tensor count, int ncap, Tensor(b!)[] out, "
        "int session, int now_ms, int wslot=-1, Tensor(c!)? fired=None, "
        "Tensor(d!)? tickets=None, bool finish=True, Tensor? seqno=None, "
        "bool read_only=False) -> ()", &tree_serve_frames);
  m.def("tree_finish(Tensor(a!)[] tree, Tensor? count, int bump=0, "
        "bool publish=True) -> ()", &tree_finish);
  m.def("tree_order_workspace(int n) -> int", &tree_order_workspace);
  m.def("tree_order_stats_offset(int n) -> int", &tree_order_stats_offset);
  m.def("tree_serve_ordered(Tensor(a!)[] tree, Tensor rx, Tensor[] requests, "
        "Tensor count, int ncap, Tensor(b!)[] out, int session, int now_ms, "
        "Tensor(c!) ws, int passes, Tensor? scratch, int wslot=-1, "
        "Tensor(d!)? fired=None, Tensor? seqno=None) -> ()",
        &tree_serve_ordered);
  m.def("tree_seq_workspace(int n) -> int", &tree_seq_workspace);
  m.def("tree_seq_zeroed(int n) -> int", &tree_seq_zeroed);
  m.def("tree_seq_debug(Tensor buf) -> ()", &tree_seq_debug);
  m.def("tree_expire_debug(Tensor buf) -> ()", &tree_expire_debug);
  m.def("tree_seq_order(Tensor(a!)[] tree, Tensor rx, Tensor frame_off, "
        "Tensor frame_len, Tensor count, int ncap, Tensor(b!) ws, "
        "Tensor(c!) seqno) -> ()", &tree_seq_order);
  m.def("tree_digest(Tensor[] tree, Tensor(a!) out) -> ()", &tree_digest);
  m.def("watch_events(Tensor r_op, Tensor r_err, Tensor count, int ncap, "
        "Tensor fired, Tensor(a!) bsum, Tensor(b!) ev_slot, "
        "Tensor(c!) ev_type, Tensor(d!) ev_path_off, Tensor(e!) ev_path_len, "
        "Tensor(f!) ev_total) -> ()", &watch_events);
  m.def("watch_resume(Tensor(a!)[] tree, Tensor rx, Tensor frame_off, "
        "Tensor frame_len, Tensor count, int ncap, int wslot, "
        "Tensor(b!) ent, Tensor(c!) ev_type, Tensor(d!) ev_path_off, "
        "Tensor(e!) ev_path_len, Tensor(f!) out) -> ()", &watch_resume);
  m.def("tree_expire(Tensor(a!)[] tree, int session, int ncap, "
        "Tensor(b!) removed) -> ()", &tree_expire);
  m.def("bench_gen_get(int n, int seed, int leaf0, int nleaves, "
        "int xid_base, Tensor node_pw, Tensor(a!) idx, Tensor(b!) xid, "
        "Tensor(c!) path_off, Tensor(d!) path_len, Tensor? state=None, "
        "Tensor(e!)? sizes=None, Tensor(f!)? bsum=None) -> ()",
        &bench_gen_get);
  m.def("bench_xids(int n, Tensor base, Tensor(a!) xid) -> ()", &bench_xids);
  m.def("bench_storm_hs(bool resume, bool prev, int timeout, Tensor status, "
        "Tensor sid, Tensor tmo, Tensor outcome, Tensor bound, Tensor resp, "
        "Tensor want, Tensor(a!) cred_sid, Tensor(b!) cred_pw, "
        "Tensor(c!) hs_ok) -> ()", &bench_storm_hs);
  m.def("bench_check_writes(int n, Tensor status, Tensor err, Tensor rxid, "
        "Tensor xid, Tensor pay_len, Tensor? want_len, int want_len_c, "
        "Tensor zxid, Tensor(a!) ok, Tensor(b!) zmax) -> ()",
        &bench_check_writes);
  m.def("bench_check_get(int n, Tensor[] reply, Tensor idx, Tensor xid, "
        "Tensor data_len, Tensor(a!) acc) -> ()", &bench_check_get);
  m.def("bench_check_notif(int total, int n_per, Tensor seeds, int leaf0, "
        "int nleaves, Tensor node_path_off, Tensor node_path_len, "
        "Tensor path_arena, Tensor rx, Tensor[] reply, Tensor(a!) acc, "
        "Tensor? want=None) -> ()", &bench_check_notif);
  m.def("route_workspace(int n, int world) -> int", &route_workspace);
  m.def("serve_tickets(int ncap) -> int", &serve_tickets);
  m.def("route_requests(int n, int world, Tensor path_off, Tensor path_len, "
        "Tensor arena, Tensor idx, Tensor xid, Tensor(a!) owner, "
        "Tensor(b!) idx_s, Tensor(c!) xid_s, Tensor(d!) path_off_s, "
        "Tensor(e!) path_len_s, Tensor(f!) counts, Tensor(g!) ws, "
        "int self=0) -> ()",
        &route_requests);
  m.def("seg_pack(Tensor src, Tensor rec_off, Tensor? nrec, int nrec_cap, "
        "Tensor total, Tensor counts, int world, int self, int slot_cap, "
        "Tensor(a!) out, Tensor(b!) stats, Tensor(c!)? self_out=None, "
        "bool inplace=False) -> ()",
        &seg_pack);
  m.def("seg_unpack(Tensor inp, int world, int self, int slot_cap, "
        "Tensor(a!) out, Tensor(b!) total, Tensor(c!) counts, "
        "Tensor(d!)? stats=None, Tensor? self_in=None, "
        "bool inplace=False) -> ()", &seg_unpack);
  m.def("session_connect(Tensor buf, Tensor frame_off, Tensor frame_len, "
        "Tensor count, int ncap, Tensor(a!)[] table, int server_id, "
        "int secret, int min_to, int max_to, Tensor zxid_now, Tensor(b!) out, "
        "Tensor(c!) resp_sid, Tensor(d!) outcome, int span=0) -> ()",
        &session_connect);
  m.def("session_close(Tensor(a!)[] table, Tensor sids, int server_id=0, "
        "int span=0) -> ()", &session_close);
  m.def("session_install(Tensor(a!)[] table, Tensor records, int server_id, "
        "int span) -> ()", &session_install);
}
