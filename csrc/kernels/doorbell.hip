// Persistent doorbell codec (SURVEY §7.1 "low latency without launch-per-op",
// §7.4.3): one resident wave polls a ring of request slots in host-coherent
// memory and encodes / decodes single records as soon as the host rings, so
// an interactive op pays a PCIe round trip instead of a kernel launch.
//
// Record shapes (reference lib/zk-buffer.js):
//   encode  header {xid, opcode} + path [+ watch bool | version i32]
//           (GET_DATA / EXISTS / GET_CHILDREN(2) / GET_ACL / SYNC / DELETE,
//           zk-buffer.js:138-231) and header-only PING / CLOSE_SESSION
//           (:129-132), framed with the i32 length (jute-buffer.js:181-189);
//   decode  reply header {xid, zxid, err} (zk-buffer.js:281-291) and, when
//           err == OK, the GET_DATA (data + Stat, :359-362) or EXISTS /
//           SET_DATA (Stat, :346-352) body; other bodies are left to the
//           host (status ST_BAD_OPCODE).
//
// Safety on a shared machine: the wave exits when the host sets ctl->stop,
// and unconditionally once `max_ticks` of s_memrealtime (100 MHz) have passed
// since it started, so it always drains even if its process died.  It polls
// with relaxed system-scope loads and s_sleep, acquiring once per record.
#include "zk_common.h"

#include <stddef.h>
#include <string.h>
#include <time.h>

extern "C" {

constexpr int ZK_DB_IN = 1024;      // path bytes (encode) / reply body (decode)
constexpr int ZK_DB_OUT = 1056;     // framed request bytes

struct ZkDbSlot {
  int64_t seq;        // host: ticket when the slot is ready (release)
  int64_t done;       // device: ticket when the result is written (release)
  int32_t kind;       // 1 encode, 2 decode
  int32_t xid;
  int32_t opcode;     // encode: request opcode; decode: opcode of the xid
  int32_t arg;        // encode: watch flag or version
  int32_t in_len;
  int32_t out_len;    // encode: framed length; decode: status
  int64_t zxid;       // decode results from here on
  int32_t err;
  int32_t rxid;
  int64_t stat64[6];  // czxid mzxid ctime mtime ephemeralOwner pzxid
  int32_t stat32[5];  // version cversion aversion dataLength numChildren
  int32_t pay_off;    // data offset in `in` (GET_DATA)
  int32_t pay_len;
  int32_t pad[3];
  uint8_t in[ZK_DB_IN];
  uint8_t out[ZK_DB_OUT];
};

struct ZkDbCtl {
  int64_t stop;
  int64_t served;     // device: records served
  int64_t alive;      // device: 1 while the wave runs, 0 once it left
  int64_t pad;
};

}  // extern "C"

namespace zk {

ZK_DEV int64_t ld_sys_relaxed(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

ZK_DEV void st_sys_release(int64_t* p, int64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The slot lives in uncached host memory, where every dependent load is a
// PCIe round trip; the wave therefore pulls the slot head and the whole
// input area in ONE burst (all loads in flight together) into `c`, an LDS
// copy, and works from there.  Results go back with posted stores.
ZK_DEV void db_encode(ZkDbSlot* s, const ZkDbSlot* c, int lane) {
  const int32_t op = c->opcode;
  const int32_t pl = c->in_len;
  int32_t body;
  switch (op) {
    case OP_PING: case OP_CLOSE_SESSION: body = 8; break;
    case OP_GET_DATA: case OP_EXISTS: case OP_GET_CHILDREN:
    case OP_GET_CHILDREN2: body = 8 + 4 + pl + 1; break;
    case OP_DELETE: body = 8 + 4 + pl + 4; break;
    case OP_GET_ACL: case OP_SYNC: body = 8 + 4 + pl; break;
    default: body = -1; break;
  }
  if (body < 0 || pl < 0 || pl > ZK_DB_IN || body + 4 > ZK_DB_OUT) {
    if (lane == 0) s->out_len = -1;
    return;
  }
  uint8_t* o = s->out;
  if (op != OP_PING && op != OP_CLOSE_SESSION) {
    // path bytes, one lane per byte
    for (int k = lane; k < pl; k += WAVE) o[16 + k] = c->in[k];
  }
  if (lane == 0) {
    st_be32(o, body);
    st_be32(o + 4, c->xid);
    st_be32(o + 8, op);
    if (op != OP_PING && op != OP_CLOSE_SESSION) {
      st_be32(o + 12, pl > 0 ? pl : -1);       // empty -> -1 (jute :127-130)
      uint8_t* t = o + 16 + pl;
      if (op == OP_DELETE) st_be32(t, c->arg);
      else if (op != OP_GET_ACL && op != OP_SYNC) *t = c->arg ? 1 : 0;
    }
    s->out_len = body + 4;
  }
}

ZK_DEV void db_stat(ZkDbSlot* s, const uint8_t* p) {
  s->stat64[0] = ld_be64(p);        // czxid
  s->stat64[1] = ld_be64(p + 8);    // mzxid
  s->stat64[2] = ld_be64(p + 16);   // ctime
  s->stat64[3] = ld_be64(p + 24);   // mtime
  s->stat32[0] = ld_be32(p + 32);   // version
  s->stat32[1] = ld_be32(p + 36);   // cversion
  s->stat32[2] = ld_be32(p + 40);   // aversion
  s->stat64[4] = ld_be64(p + 44);   // ephemeralOwner
  s->stat32[3] = ld_be32(p + 52);   // dataLength
  s->stat32[4] = ld_be32(p + 56);   // numChildren
  s->stat64[5] = ld_be64(p + 60);   // pzxid
}

// Decode is scalar work (a header and a fixed Stat): lane 0 does it.
ZK_DEV void db_decode(ZkDbSlot* s, const ZkDbSlot* c) {
  const int32_t n = c->in_len;
  const uint8_t* b = c->in;
  int32_t st = ST_OK;
  if (n < 16 || n > ZK_DB_IN) {
    s->out_len = ST_BAD_DECODE;
    return;
  }
  s->rxid = ld_be32(b);
  s->zxid = ld_be64(b + 4);
  s->err = ld_be32(b + 12);
  s->pay_off = 0;
  s->pay_len = 0;
  if (s->err == ERR_OK) {
    switch (c->opcode) {
      case OP_GET_DATA: {
        if (n < 20) { st = ST_BAD_DECODE; break; }
        int32_t dl = ld_be32(b + 16);
        if (dl < 0) dl = 0;                    // negative reads as empty
        if (20 + dl + STAT_BYTES > n) { st = ST_BAD_DECODE; break; }
        s->pay_off = 20;
        s->pay_len = dl;
        db_stat(s, b + 20 + dl);
        break;
      }
      case OP_EXISTS: case OP_SET_DATA:
        if (16 + STAT_BYTES > n) { st = ST_BAD_DECODE; break; }
        db_stat(s, b + 16);
        break;
      case OP_PING: case OP_SYNC: case OP_DELETE: case OP_CLOSE_SESSION:
        break;                                 // header-only (:316-325)
      default:
        st = ST_BAD_OPCODE;
    }
  }
  s->out_len = st;
}

__global__ __launch_bounds__(64) void db_serve(ZkDbSlot* __restrict__ slots,
                                               int32_t nslots,
                                               ZkDbCtl* __restrict__ ctl,
                                               int64_t first_ticket,
                                               uint64_t max_ticks) {
  constexpr int HEAD = (int)offsetof(ZkDbSlot, in);          // 96 bytes
  static_assert(HEAD % 16 == 0 && ZK_DB_IN % 16 == 0, "16-byte pulls");
  __shared__ __attribute__((aligned(16))) uint8_t lds[HEAD + ZK_DB_IN];
  const ZkDbSlot* c = reinterpret_cast<const ZkDbSlot*>(lds);
  const int lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  int64_t ticket = first_ticket;
  if (lane == 0) st_sys_release(&ctl->alive, 1);
  for (;;) {
    ZkDbSlot* s = slots + (ticket % nslots);
    // lane 0 polls; the decision is broadcast so the wave stays uniform
    int go = 0;
    if (lane == 0) {
      if (ld_sys_relaxed(&ctl->stop) != 0) go = -1;
      else if (ld_sys_relaxed(&s->seq) == ticket) go = 1;
      else if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) go = -1;
    }
    go = __shfl(go, 0, WAVE);
    if (go < 0) break;
    if (go == 0) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // slot fields after seq
    {
      constexpr int NV = (HEAD + ZK_DB_IN) / 16;               // 70 vectors
      const uint4* src = reinterpret_cast<const uint4*>(s);
      const uint4 a = src[lane];
      const uint4 b = lane + WAVE < NV ? src[lane + WAVE] : make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(lds)[lane] = a;
      if (lane + WAVE < NV) reinterpret_cast<uint4*>(lds)[lane + WAVE] = b;
      __builtin_amdgcn_s_waitcnt(0xC07F);                      // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
    }
    if (c->kind == 1) db_encode(s, c, lane);
    else if (lane == 0) db_decode(s, c);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      __threadfence_system();
      st_sys_release(&s->done, ticket);
      __hip_atomic_fetch_add(&ctl->served, (int64_t)1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ++ticket;
  }
  if (lane == 0) {
    __threadfence_system();
    st_sys_release(&ctl->alive, 0);
  }
}

}  // namespace zk

extern "C" {

// One service: `nslots` slots + a control block in host-coherent, mapped
// memory, and a non-blocking stream for the resident wave.
struct ZkDb {
  ZkDbSlot* slots;
  ZkDbCtl* ctl;
  int32_t nslots;
  int64_t next;        // host: next ticket to hand out
  hipStream_t stream;
};

int64_t zk_db_slot_bytes() { return (int64_t)sizeof(ZkDbSlot); }

void* zk_db_create(int32_t nslots) {
  if (nslots <= 0) return nullptr;
  ZkDb* d = new ZkDb();
  d->nslots = nslots;
  d->next = 1;
  const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
  if (hipHostMalloc((void**)&d->slots, sizeof(ZkDbSlot) * nslots, fl) !=
          hipSuccess ||
      hipHostMalloc((void**)&d->ctl, sizeof(ZkDbCtl), fl) != hipSuccess ||
      hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) !=
          hipSuccess) {
    delete d;
    return nullptr;
  }
  memset(d->slots, 0, sizeof(ZkDbSlot) * nslots);
  memset(d->ctl, 0, sizeof(ZkDbCtl));
  return d;
}

// Launch the resident wave; it serves tickets from d->next on and leaves
// after max_ms at the latest.
int zk_db_start(void* h, int64_t max_ms) {
  ZkDb* d = (ZkDb*)h;
  __atomic_store_n(&d->ctl->stop, 0, __ATOMIC_RELEASE);
  __atomic_store_n(&d->ctl->alive, 1, __ATOMIC_RELEASE);
  ZkDbSlot* ds = nullptr;
  ZkDbCtl* dc = nullptr;
  if (hipHostGetDevicePointer((void**)&ds, d->slots, 0) != hipSuccess ||
      hipHostGetDevicePointer((void**)&dc, d->ctl, 0) != hipSuccess)
    return -1;
  const uint64_t ticks = (uint64_t)(max_ms > 0 ? max_ms : 1) * 100000ull;
  zk::db_serve<<<1, 64, 0, d->stream>>>(ds, d->nslots, dc, d->next, ticks);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Stop the wave and wait for it (bounded by its own deadline).
int zk_db_stop(void* h) {
  ZkDb* d = (ZkDb*)h;
  __atomic_store_n(&d->ctl->stop, 1, __ATOMIC_RELEASE);
  return (int)hipStreamSynchronize(d->stream);
}

void zk_db_destroy(void* h) {
  ZkDb* d = (ZkDb*)h;
  if (d == nullptr) return;
  zk_db_stop(d);
  hipStreamDestroy(d->stream);
  hipHostFree(d->slots);
  hipHostFree(d->ctl);
  delete d;
}

static ZkDbSlot* db_fill(ZkDb* d, int32_t kind, int32_t xid, int32_t opcode,
                         int32_t arg, const uint8_t* in, int32_t in_len,
                         int64_t* ticket) {
  if (in_len < 0 || in_len > ZK_DB_IN) return nullptr;
  const int64_t t = d->next++;
  ZkDbSlot* s = d->slots + (t % d->nslots);
  s->kind = kind;
  s->xid = xid;
  s->opcode = opcode;
  s->arg = arg;
  s->in_len = in_len;
  if (in_len > 0) memcpy(s->in, in, (size_t)in_len);
  __atomic_store_n(&s->seq, t, __ATOMIC_RELEASE);     // ring
  *ticket = t;
  return s;
}

// Wait (spinning) for the slot's result; -2 on timeout, -3 if the wave left.
static int db_wait(ZkDb* d, ZkDbSlot* s, int64_t t, int64_t timeout_us) {
  struct timespec a, b;
  clock_gettime(CLOCK_MONOTONIC, &a);
  for (uint64_t k = 0;; ++k) {
    if (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) == t) return 0;
    __builtin_ia32_pause();
    if ((k & 1023) == 1023) {
      if (__atomic_load_n(&d->ctl->alive, __ATOMIC_ACQUIRE) == 0) return -3;
      clock_gettime(CLOCK_MONOTONIC, &b);
      const int64_t us = (b.tv_sec - a.tv_sec) * 1000000 +
                         (b.tv_nsec - a.tv_nsec) / 1000;
      if (us > timeout_us) return -2;
    }
  }
}

// Encode one request; copies the framed bytes to `out` (cap bytes) and
// returns their length, or < 0.
int32_t zk_db_encode(void* h, int32_t xid, int32_t opcode, int32_t arg,
                     const uint8_t* path, int32_t path_len, uint8_t* out,
                     int32_t cap, int64_t timeout_us) {
  ZkDb* d = (ZkDb*)h;
  int64_t t;
  ZkDbSlot* s = db_fill(d, 1, xid, opcode, arg, path, path_len, &t);
  if (s == nullptr) return -1;
  const int rc = db_wait(d, s, t, timeout_us);
  if (rc) return rc;
  const int32_t n = s->out_len;
  if (n < 0 || n > cap) return -1;
  memcpy(out, s->out, (size_t)n);
  return n;
}

// Decode one reply body; fills res (int64[16]: status, xid, zxid, err,
// pay_off, pay_len, czxid, mzxid, ctime, mtime, ephemeralOwner, pzxid,
// version, cversion, aversion, dataLength | numChildren << 32).
int32_t zk_db_decode(void* h, int32_t opcode, const uint8_t* body,
                     int32_t len, int64_t* res, int64_t timeout_us) {
  ZkDb* d = (ZkDb*)h;
  int64_t t;
  ZkDbSlot* s = db_fill(d, 2, 0, opcode, 0, body, len, &t);
  if (s == nullptr) return -1;
  const int rc = db_wait(d, s, t, timeout_us);
  if (rc) return rc;
  res[0] = s->out_len;
  res[1] = s->rxid;
  res[2] = s->zxid;
  res[3] = s->err;
  res[4] = s->pay_off;
  res[5] = s->pay_len;
  for (int k = 0; k < 6; ++k) res[6 + k] = s->stat64[k];
  res[12] = s->stat32[0];
  res[13] = s->stat32[1];
  res[14] = s->stat32[2];
  res[15] = (int64_t)(uint32_t)s->stat32[3] |
            ((int64_t)s->stat32[4] << 32);
  return 0;
}

int64_t zk_db_served(void* h) {
  return __atomic_load_n(&((ZkDb*)h)->ctl->served, __ATOMIC_ACQUIRE);
}

}  // extern "C"
