// Server side of the session handshake (K9, server mode) for the GPU-resident
// synthetic server: a batch of ConnectRequest frames is decoded, checked
// against the session table in HBM and answered with ConnectResponse frames.
//
// What a ZooKeeper server does with a ConnectRequest, as the reference relies
// on it (lib/zk-session.js:147-205, :265-339):
//   * sessionId 0 -> a new session: fresh id, 16-byte password, negotiated
//     timeout (clamped to [min_to, max_to], 2 and 20 ticks);
//   * a known, live session with the right password -> resumed: same id and
//     password, timeout renegotiated; its ephemerals are untouched;
//   * anything else (unknown, expired or closed id, wrong password) -> the
//     "expired" answer: sessionId 0, timeOut 0, zero password
//     (lib/zk-session.js:169-173 turns that into 'expired');
//   * a client that has seen a zxid newer than the server's is refused
//     (same answer; a real server drops the connection).
// Responses are fixed-size (41 bytes: frame length, protocolVersion,
// timeOut, sessionId, 16-byte passwd, the readOnly byte real servers append,
// test/streams.test.js:24), so frame i lands at i * 41 with no scan.
#include "zk_common.h"

namespace zk {

constexpr int SS_T = 256;
constexpr int32_t CR_RESP_BYTES = 41;
enum : int32_t { SS_FREE = 0, SS_ALIVE = 1, SS_CLOSED = 2 };
// (per-request outcomes: SC_* in zk_common.h)

// The table slot of session id s (-1: not one this table can hold).
ZK_DEV int64_t sess_slot(const ZkSessionTable& tab, int64_t s,
                         int64_t server_id) {
  const int64_t srv = (s >> 56) & 0x7f;
  const int64_t idx = (s & 0x00ffffffffffffffll) - 1;
  if (idx < 0) return -1;
  if (tab.span == 0) return srv == server_id && idx < tab.cap ? idx : -1;
  if (srv < 1 || idx >= tab.span || srv * tab.span > tab.cap) return -1;
  return (srv - 1) * tab.span + idx;
}

ZK_DEV uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(SS_T) void session_connect_k(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ foff,
    const int32_t* __restrict__ flen, const int64_t* __restrict__ n_dev,
    int64_t ncap, ZkSessionTable tab, int64_t server_id, uint64_t secret,
    int32_t min_to, int32_t max_to, const int64_t* __restrict__ zxid_now,
    uint8_t* __restrict__ out, int64_t* __restrict__ resp_sid,
    int32_t* __restrict__ outcome) {
  const int64_t i = (int64_t)blockIdx.x * SS_T + threadIdx.x;
  const int64_t n = min(*n_dev, ncap);
  if (i >= n) return;
  const uint8_t* p = buf + foff[i];
  const int64_t L = flen[i];
  int32_t oc = SC_BAD, to = 0;
  int64_t sid = 0;
  uint64_t pw0 = 0, pw1 = 0;
  if (L >= 28) {
    const int64_t last = ld_be64(p + 4);
    const int32_t want = ld_be32(p + 12);
    const int64_t csid = ld_be64(p + 16);
    int32_t pwl = ld_be32(p + 24);
    if (pwl < 0) pwl = 0;
    if (28 + (int64_t)pwl > L) {
      oc = SC_BAD;
    } else if (last > *zxid_now) {
      oc = SC_REFUSED;
    } else if (csid == 0) {
      const int64_t own = (int64_t)atomicAdd((unsigned long long*)tab.next,
                                             1ull);
      const int64_t idx = tab.span ? (server_id - 1) * tab.span + own : own;
      if (own < (tab.span ? tab.span : tab.cap) && idx >= 0 && idx < tab.cap) {
        sid = (server_id << 56) | (own + 1);
        to = min(max(want, min_to), max_to);
        pw0 = mix64((uint64_t)sid ^ secret);
        pw1 = mix64(pw0 ^ secret);
        tab.sid[idx] = sid;
        __builtin_memcpy(tab.passwd + idx * 16, &pw0, 8);
        __builtin_memcpy(tab.passwd + idx * 16 + 8, &pw1, 8);
        tab.timeout[idx] = to;
        tab.state[idx] = SS_ALIVE;
        oc = SC_NEW;
      } else {
        oc = SC_FULL;
      }
    } else {
      // (an ensemble member knows every member's sessions: the replicated
      // table; the id equality below rejects a slot never filled)
      const int64_t idx = sess_slot(tab, csid, server_id);
      bool ok = idx >= 0 && pwl == 16;
      if (ok) ok = tab.sid[idx] == csid && tab.state[idx] == SS_ALIVE;
      if (ok) {
        uint64_t a, b, c, d;
        __builtin_memcpy(&a, tab.passwd + idx * 16, 8);
        __builtin_memcpy(&b, tab.passwd + idx * 16 + 8, 8);
        __builtin_memcpy(&c, p + 28, 8);
        __builtin_memcpy(&d, p + 36, 8);
        ok = a == c && b == d;
        pw0 = a;
        pw1 = b;
      }
      if (ok) {
        sid = csid;
        to = min(max(want, min_to), max_to);
        tab.timeout[idx] = to;
        oc = SC_RESUMED;
      } else {
        pw0 = pw1 = 0;
        oc = SC_EXPIRED;
      }
    }
  }
  uint8_t* o = out + i * CR_RESP_BYTES;
  st_be32(o, CR_RESP_BYTES - 4);
  st_be32(o + 4, 0);                    // protocolVersion
  st_be32(o + 8, to);
  st_be64(o + 12, sid);
  st_be32(o + 20, 16);
  __builtin_memcpy(o + 24, &pw0, 8);
  __builtin_memcpy(o + 32, &pw1, 8);
  o[40] = 0;                            // readOnly
  resp_sid[i] = sid;
  outcome[i] = oc;
}

// Close / expire sessions: the table entry dies, so a later resume with its
// id gets the expired answer.  (The ephemerals go with zk_tree_expire.)
__global__ __launch_bounds__(SS_T) void session_close_k(
    ZkSessionTable tab, const int64_t* __restrict__ sids, int64_t n,
    int64_t server_id) {
  const int64_t i = (int64_t)blockIdx.x * SS_T + threadIdx.x;
  if (i >= n) return;
  const int64_t s = sids[i];
  const int64_t idx = sess_slot(tab, s, server_id);
  if (idx >= 0 && tab.sid[idx] == s) tab.state[idx] = SS_CLOSED;
}

// Install replicated session records {sid, timeout, passwd[16]} (an
// ensemble's other members' new sessions, R3): ALIVE at their slots.
__global__ __launch_bounds__(SS_T) void session_install_k(
    ZkSessionTable tab, const int64_t* __restrict__ rec, int64_t n,
    int64_t server_id) {
  const int64_t i = (int64_t)blockIdx.x * SS_T + threadIdx.x;
  if (i >= n) return;
  const int64_t* r = rec + 4 * i;
  const int64_t s = r[0];
  if (s == 0 || ((s >> 56) & 0x7f) == server_id) return;
  const int64_t idx = sess_slot(tab, s, 0);
  if (idx < 0) return;
  tab.sid[idx] = s;
  tab.timeout[idx] = (int32_t)r[1];
  __builtin_memcpy(tab.passwd + idx * 16, &r[2], 16);
  tab.state[idx] = SS_ALIVE;
}

}  // namespace zk

extern "C" {

// ConnectRequest frames (foff/flen from K1, *n_dev of them, at most ncap)
// -> ConnectResponse frames at out[i * 41], the bound session id per
// request (0 = refused / expired) and the outcome code (SC_*).
int zk_session_connect(const uint8_t* buf, const int64_t* foff,
                       const int32_t* flen, const int64_t* n_dev,
                       int64_t ncap, const ZkSessionTable* tab,
                       int64_t server_id, uint64_t secret, int32_t min_to,
                       int32_t max_to, const int64_t* zxid_now, uint8_t* out,
                       int64_t* resp_sid, int32_t* outcome, hipStream_t st) {
  if (ncap <= 0) return 0;
  if (server_id < 0 || server_id > 127) return (int)hipErrorInvalidValue;
  zk::session_connect_k<<<(unsigned)((ncap + zk::SS_T - 1) / zk::SS_T),
                          zk::SS_T, 0, st>>>(
      buf, foff, flen, n_dev, ncap, *tab, server_id, secret, min_to, max_to,
      zxid_now, out, resp_sid, outcome);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_session_close(const ZkSessionTable* tab, const int64_t* sids,
                     int64_t n, int64_t server_id, hipStream_t st) {
  if (n <= 0) return 0;
  zk::session_close_k<<<(unsigned)((n + zk::SS_T - 1) / zk::SS_T), zk::SS_T,
                        0, st>>>(*tab, sids, n, server_id);
  ZK_LAUNCH_CHECK();
  return 0;
}

// rec: n records of 4 int64 {sid, timeout, passwd bytes 0-7, 8-15}
int zk_session_install(const ZkSessionTable* tab, const int64_t* rec,
                       int64_t n, int64_t server_id, hipStream_t st) {
  if (n <= 0) return 0;
  if (tab->span <= 0) return (int)hipErrorInvalidValue;
  zk::session_install_k<<<(unsigned)((n + zk::SS_T - 1) / zk::SS_T),
                          zk::SS_T, 0, st>>>(*tab, rec, n, server_id);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
