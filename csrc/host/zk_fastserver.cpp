// zk_fastserver — a native ZooKeeper wire server for client benchmarks.
//
// The in-process fake server (zkmi/server/fakezk.py) implements the whole
// Appendix-D contract in Python; at tens of thousands of requests per second
// it, not the client, would be what a pipelined client benchmark measures.
// This server speaks the same wire protocol from a pool of epoll threads:
// handshake (new and resumed sessions), PING, GET_DATA, EXISTS, SET_DATA
// (version CAS), CREATE (persistent, EPHEMERAL, SEQUENTIAL), DELETE, SYNC,
// GET_CHILDREN(2), CLOSE_SESSION, and watches: GET_DATA / EXISTS /
// GET_CHILDREN(2) with watch=1 arm one-shot watches, writes fire
// NODE_CREATED / NODE_DELETED / NODE_DATA_CHANGED / NODE_CHILDREN_CHANGED
// notifications (xid -1) with fakezk.py's trigger table, SET_WATCHES
// re-arms them and catches up on changes after relZxid (SURVEY Appendix D;
// reference client side: lib/zk-session.js:558-574, :421-471).  A
// session's watches live with its connection (as on a real ZooKeeper
// server: a client that moves re-arms them with SET_WATCHES).  No ACL
// checks, no expiry.
//
// --members M: M listening ports sharing one tree and session table (the
// 3-server ensemble of test/multi-node.test.js, BASELINE config 4); stdin
// then carries fakezk's ensemble fault commands, one per line, each
// answered by one line:
//   outage <i> [<path>=<hexdata> ...]  close member i's connections and its
//                                      port, then apply the sets (firing
//                                      watches); answers "OK <zxid>"
//   start <i>                          listen on member i's port again
//   timing [reset]                     the wire clock below (any M)
//
// The wire clock (CLOCK_MONOTONIC ns, the clock of Python's perf_counter
// on Linux, so a client can line its own stamps up with it): first / last
// recv that returned bytes, first / last send that moved bytes, and the
// sums of time in recv(), in serving frames (tree lock + replies), in
// send() and with replies waiting for the socket to drain (EAGAIN until the
// next send that moves bytes); bytes in / out, bursts served, send() and
// recv() calls, bursts served in parallel and the time in them.  "timing"
// answers "OK" and those 15 numbers, "timing reset" zeroes them.
// Notifications to a connection served by another worker go through that
// connection's note buffer (its own mutex) and the worker's eventfd; every
// burst drains the notes before serving, so a notification always precedes
// the reply to any request served after the write that fired it.
//
// Every readable burst is answered with one send(): all complete frames of
// the burst are served in order (ZooKeeper answers a session's requests in
// order) and their replies appended to one output buffer.
//
// Threads: the main thread accepts and hands each connection to one of
// --threads workers (round robin; each worker runs its own epoll set), so
// k client connections are served by up to k cores.  The tree is shared
// under a reader/writer lock taken once per burst: a burst of reads (GET,
// EXISTS, children, SYNC, PING) shares it, a burst holding any write or
// the handshake takes it alone.  (Round 2's single epoll thread served
// ~1.4 M GETs/s — the bound of the bulk TCP benchmark.)
//
// Usage: zk_fastserver [--port P] [--preload N] [--data-bytes B]
//                      [--fanout F] [--threads T] [--members M]
// --preload creates /bench, /bench/dDDDDDD and N leaves
// /bench/dDDDDDD/nNNNNNNNNN with B bytes of data each (the layout of
// zkmi/bench/synthetic.py GpuTree).  Prints "PORT <n>" (M = 1) or
// "PORTS <p1> ... <pM>" once listening and exits when stdin reaches EOF.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/eventfd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

enum : int32_t {
  OP_CREATE = 1, OP_DELETE = 2, OP_EXISTS = 3, OP_GET_DATA = 4,
  OP_SET_DATA = 5, OP_GET_ACL = 6, OP_GET_CHILDREN = 8, OP_SYNC = 9,
  OP_PING = 11, OP_GET_CHILDREN2 = 12, OP_SET_WATCHES = 101,
  OP_CLOSE_SESSION = -11
};
enum : int32_t {           // notification types, state SyncConnected
  EV_CREATED = 1, EV_DELETED = 2, EV_DATA_CHANGED = 3,
  EV_CHILDREN_CHANGED = 4, ST_SYNC_CONNECTED = 3
};
enum : int32_t {
  E_OK = 0, E_MARSHALLING = -5, E_UNIMPLEMENTED = -6, E_BAD_ARGUMENTS = -8,
  E_NO_NODE = -101, E_BAD_VERSION = -103, E_NO_CHILDREN_FOR_EPHEMERALS = -108,
  E_NODE_EXISTS = -110, E_NOT_EMPTY = -111
};
constexpr int32_t MAX_PACKET = 16 * 1024 * 1024;

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

// The wire clock (header comment): all fields atomics, workers add to them
struct WireClock {
  enum { FIRST_RX, LAST_RX, FIRST_TX, LAST_TX, RECV, SERVE, SEND, BLOCKED,
         RX_BYTES, TX_BYTES, BURSTS, SENDS, RECVS, PAR_BURSTS, PAR_NS, N };
  std::atomic<int64_t> v[N];
  WireClock() { reset(); }
  void reset() { for (auto& x : v) x.store(0, std::memory_order_relaxed); }
  void add(int k, int64_t d) { v[k].fetch_add(d, std::memory_order_relaxed); }
  void first(int k, int64_t t) {
    int64_t z = 0;
    v[k].compare_exchange_strong(z, t, std::memory_order_relaxed);
  }
  void last(int k, int64_t t) {
    int64_t o = v[k].load(std::memory_order_relaxed);
    while (o < t && !v[k].compare_exchange_weak(o, t,
                                                std::memory_order_relaxed)) {}
  }
  std::string report() {
    std::string r = "OK";
    for (auto& x : v) r += " " + std::to_string((long long)x.load());
    return r;
  }
};
WireClock wclock;

int64_t now_ms() {
  timeval tv;
  gettimeofday(&tv, nullptr);
  return (int64_t)tv.tv_sec * 1000 + tv.tv_usec / 1000;
}

struct Stat {
  int64_t czxid = 0, mzxid = 0, ctime = 0, mtime = 0;
  int32_t version = 0, cversion = 0, aversion = 0;
  int64_t eph = 0;
  int32_t dlen = 0, nkids = 0;
  int64_t pzxid = 0;
};

// Watching sessions (one-shot): usually none or one, so a short vector.
// SET_WATCHES lists at least this long look their paths up on SW_THREADS
// threads
constexpr size_t SW_PAR_MIN = 8192;
constexpr size_t SW_THREADS = 8;

struct Watchers {
  std::vector<int64_t> s;
  bool add(int64_t sid) {
    for (int64_t x : s) if (x == sid) return false;
    s.push_back(sid);
    return true;
  }
  bool drop(int64_t sid) {
    for (size_t i = 0; i < s.size(); ++i)
      if (s[i] == sid) { s[i] = s.back(); s.pop_back(); return true; }
    return false;
  }
};

struct Node {
  std::string data;
  Stat st;
  std::string path;       // its own path (the index's key check)
  std::set<std::string> kids;
  // the node's own watchers: arming and firing cost no lookup (round 3's
  // path-keyed tables made a watched SET 4 us and a re-arming GET 2.6 us)
  Watchers dw, cw;        // data (GET_DATA / EXISTS), child (GET_CHILDREN)
};

// A set of node pointers (a session's watched nodes): open addressing,
// linear probing, backward-shift erase, at most half full — no allocation
// per element (std::unordered_set's node malloc was most of arming a
// 65536-path SET_WATCHES).
struct PtrSet {
  std::vector<Node*> t = std::vector<Node*>(16, nullptr);
  size_t n = 0;
  static size_t hp(const Node* p) {
    uint64_t x = (uint64_t)(uintptr_t)p;
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 29;
    return (size_t)x;
  }
  size_t size() const { return n; }
  void reserve(size_t k) {
    if (2 * k <= t.size()) return;
    size_t cap = t.size();
    while (cap < 2 * k) cap *= 2;
    std::vector<Node*> old(cap, nullptr);
    old.swap(t);
    n = 0;
    for (Node* p : old)
      if (p != nullptr) insert(p);
  }
  bool insert(Node* p) {
    if (2 * (n + 1) > t.size()) reserve(n + 1);
    const size_t m = t.size() - 1;
    for (size_t s = hp(p) & m;; s = (s + 1) & m) {
      if (t[s] == p) return false;
      if (t[s] == nullptr) { t[s] = p; ++n; return true; }
    }
  }
  bool erase(Node* p) {
    const size_t m = t.size() - 1;
    size_t s = hp(p) & m;
    for (;; s = (s + 1) & m) {
      if (t[s] == nullptr) return false;
      if (t[s] == p) break;
    }
    for (size_t j = (s + 1) & m;; j = (j + 1) & m) {
      if (t[j] == nullptr) break;
      const size_t home = hp(t[j]) & m;
      if (((j - home) & m) >= ((j - s) & m)) {
        t[s] = t[j];
        s = j;
      }
    }
    t[s] = nullptr;
    --n;
    return true;
  }
  template <class F>
  void each(F f) const {
    for (Node* p : t)
      if (p != nullptr) f(p);
  }
};

// -- big-endian reader / writer ---------------------------------------------

struct Rd {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  int32_t i32() {
    if (e - p < 4) { ok = false; return 0; }
    uint32_t v; memcpy(&v, p, 4); p += 4; return (int32_t)ntohl(v);
  }
  int64_t i64() {
    uint64_t hi = (uint32_t)i32(), lo = (uint32_t)i32();
    return (int64_t)(hi << 32 | lo);
  }
  bool boolean() {
    if (e - p < 1) { ok = false; return false; }
    return *p++ != 0;
  }
  // buffer / ustring: i32 length (negative = empty), bytes
  bool buf(const uint8_t** s, int32_t* n) {
    int32_t l = i32();
    if (!ok) return false;
    if (l < 0) l = 0;
    if (e - p < l) { ok = false; return false; }
    *s = p; *n = l; p += l;
    return true;
  }
};

struct Wr {
  std::string* o;
  void i32(int32_t v) { uint32_t x = htonl((uint32_t)v); o->append((char*)&x, 4); }
  void i64(int64_t v) { i32((int32_t)(v >> 32)); i32((int32_t)v); }
  void buf(const char* s, size_t n) {
    if (n == 0) { i32(-1); return; }
    i32((int32_t)n); o->append(s, n);
  }
  void stat(const Stat& s) {
    i64(s.czxid); i64(s.mzxid); i64(s.ctime); i64(s.mtime);
    i32(s.version); i32(s.cversion); i32(s.aversion); i64(s.eph);
    i32(s.dlen); i32(s.nkids); i64(s.pzxid);
  }
};

// Big-endian writes at a cursor into space already sized (a reply built in
// place: one resize, no per-field append).
struct Put {
  uint8_t* q;
  void i32(int32_t v) {
    const uint32_t x = htonl((uint32_t)v);
    memcpy(q, &x, 4);
    q += 4;
  }
  void i64(int64_t v) { i32((int32_t)(v >> 32)); i32((int32_t)v); }
  void raw(const void* s, size_t n) {
    if (n) memcpy(q, s, n);
    q += n;
  }
  void stat(const Stat& s) {
    i64(s.czxid); i64(s.mzxid); i64(s.ctime); i64(s.mtime);
    i32(s.version); i32(s.cversion); i32(s.aversion); i64(s.eph);
    i32(s.dlen); i32(s.nkids); i64(s.pzxid);
  }
};
constexpr size_t STAT_LEN = 68;

struct Worker;

// Helper threads that serve one connection's large read burst in parallel
// (ServePool::run).  A single pipelined connection's batch of a million
// GETs was served by its one worker thread, ~0.9 us a request, and nothing
// was sent before all of it was served: the bulk TCP benchmark's bound
// (the server's wire clock, `timing`).  Reads of a burst touch the tree
// under the worker's shared lock only, so chunks of the burst are served
// into separate buffers by several threads and appended in order.
struct ServePool {
  std::vector<std::thread> th;
  std::mutex mu, run_mu;
  std::condition_variable cv, done_cv;
  std::function<void(int)> job;
  int next = 0, total = 0, pending = 0;
  uint64_t gen = 0;
  bool stop = false;

  explicit ServePool(int n) {
    for (int i = 0; i < n; ++i) th.emplace_back([this] { loop(); });
  }
  ~ServePool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  int size() const { return (int)th.size(); }
  // grab and run tasks of the current job until none is left
  void work() {
    for (;;) {
      int k;
      {
        std::lock_guard<std::mutex> g(mu);
        if (next >= total) return;
        k = next++;
      }
      job(k);
      std::lock_guard<std::mutex> g(mu);
      if (--pending == 0) done_cv.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      work();
    }
  }
  // n tasks f(0..n-1), the caller working too; false (nothing ran) when
  // another connection's burst holds the pool
  bool run(int n, const std::function<void(int)>& f) {
    std::unique_lock<std::mutex> r(run_mu, std::try_to_lock);
    if (!r.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> g(mu);
      job = f;
      next = 0;
      total = n;
      pending = n;
      ++gen;
    }
    cv.notify_all();
    work();
    std::unique_lock<std::mutex> g(mu);
    done_cv.wait(g, [&] { return pending == 0; });
    job = nullptr;
    return true;
  }
};

struct Conn {
  int fd;
  int member = 0;
  bool hs = false;
  bool closing = false;
  int64_t sid = 0;
  std::string in, out;
  size_t in_off = 0, out_off = 0;
  int64_t t_block = 0;   // replies waiting for the socket since (wire clock)
  Worker* w = nullptr;
  std::mutex nmu;        // notes: notifications from other workers' writes
  std::string notes;
};

struct Server {
  ServePool* pool = nullptr;     // parallel read bursts (nullptr: serial)
  std::shared_mutex mu;          // the tree and the session table
  std::unordered_map<std::string, std::unique_ptr<Node>> nodes;
  std::unordered_map<int64_t, std::string> sessions;    // sid -> passwd
  int64_t zxid = 1;
  int64_t next_sid = 1;
  uint64_t pw_state = 0x9E3779B97F4A7C15ull;
  // watches (under wmu; readers arm them under the shared tree lock): a
  // node's data and child watchers live in the node; exist watches of
  // missing paths here (fakezk.py keeps both kinds in one path table); the
  // session's connection route
  std::mutex wmu;
  std::unordered_map<std::string, Watchers> ew;
  // what each session armed (the index drop_watches walks instead of the
  // tree): nodes it data-/child-watches, missing paths it exist-watches
  struct SessW {
    PtrSet d, c;
    std::unordered_set<std::string> e;
  };
  std::unordered_map<int64_t, SessW> sw;
  uint64_t sw_epoch = 0;         // bumped (under wmu) when an entry goes
  // a thread's last session index entry (arming reads: one lookup a burst,
  // not one a GET); valid while sw_epoch holds
  struct SwCache {
    const void* srv = nullptr;
    int64_t sid = 0;
    uint64_t epoch = ~0ull;
    SessW* ss = nullptr;
  };
  SessW* sess_w(int64_t sid) {       // (under wmu)
    static thread_local SwCache tl;
    if (tl.srv != this || tl.sid != sid || tl.epoch != sw_epoch) {
      tl.ss = &sw[sid];
      tl.srv = this;
      tl.sid = sid;
      tl.epoch = sw_epoch;
    }
    return tl.ss;
  }
  std::unordered_map<int64_t, Conn*> route;
  std::atomic<uint64_t> n_notes{0};
  // members: connections per member (under mu, exclusive to change)
  std::vector<std::set<Conn*>> mconns;

  // The path index: open addressing over a 64-bit path hash (linear
  // probing, backward-shift deletion, at most half full), one slot per
  // node beside `nodes` (which owns them).  A lookup is one slot line, the
  // node and its path; std::unordered_map's bucket, list node and key
  // buffer made a GET ~1.2 us of cache misses on a 1M-node tree, and the
  // slots are what a read burst prefetches ahead (serve_parallel).
  struct IxEnt {
    uint64_t h;
    Node* nd;
  };
  std::vector<IxEnt> ix = std::vector<IxEnt>(1024, IxEnt{0, nullptr});
  size_t ix_used = 0;
  static uint64_t phash(const char* s, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xFF51AFD7ED558CCDull);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      memcpy(&w, s + i, 8);
      h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
      h ^= h >> 29;
    }
    uint64_t w = 0;
    for (size_t k = 0; i + k < n; ++k) w |= (uint64_t)(uint8_t)s[i + k] << (8 * k);
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 32;
    return h;
  }
  const IxEnt* ix_slot(uint64_t h) const { return &ix[h & (ix.size() - 1)]; }
  Node* ix_find(const char* p, size_t n, uint64_t h) const {
    const size_t m = ix.size() - 1;
    for (size_t s = h & m;; s = (s + 1) & m) {
      const IxEnt& e = ix[s];
      if (e.nd == nullptr) return nullptr;
      if (e.h == h && e.nd->path.size() == n &&
          memcmp(e.nd->path.data(), p, n) == 0)
        return e.nd;
    }
  }
  void ix_put(Node* nd) {
    if (2 * (ix_used + 1) > ix.size()) {
      std::vector<IxEnt> old(ix.size() * 2, IxEnt{0, nullptr});
      old.swap(ix);
      ix_used = 0;
      for (const IxEnt& e : old)
        if (e.nd != nullptr) ix_put(e.nd);
    }
    const uint64_t h = phash(nd->path.data(), nd->path.size());
    const size_t m = ix.size() - 1;
    for (size_t s = h & m;; s = (s + 1) & m) {
      IxEnt& e = ix[s];
      if (e.nd == nullptr) { e = IxEnt{h, nd}; ++ix_used; return; }
      if (e.h == h && e.nd->path == nd->path) { e.nd = nd; return; }
    }
  }
  void ix_del(const std::string& p) {
    const uint64_t h = phash(p.data(), p.size());
    const size_t m = ix.size() - 1;
    size_t s = h & m;
    for (;; s = (s + 1) & m) {
      if (ix[s].nd == nullptr) return;
      if (ix[s].h == h && ix[s].nd->path == p) break;
    }
    // backward shift: an entry after the hole moves into it unless its
    // home lies in (hole, its slot]
    for (size_t j = (s + 1) & m;; j = (j + 1) & m) {
      if (ix[j].nd == nullptr) break;
      const size_t home = ix[j].h & m;
      if (((j - home) & m) >= ((j - s) & m)) {
        ix[s] = ix[j];
        s = j;
      }
    }
    ix[s] = IxEnt{0, nullptr};
    --ix_used;
  }
  Node* find(const std::string& p) {
    return ix_find(p.data(), p.size(), phash(p.data(), p.size()));
  }
  static std::string parent_of(const std::string& p) {
    size_t k = p.rfind('/');
    return k == 0 ? std::string("/") : p.substr(0, k);
  }
  Node* make(const std::string& path, const char* d, size_t n, int64_t eph) {
    auto nd = std::make_unique<Node>();
    nd->data.assign(d, n);
    int64_t z = ++zxid, t = now_ms();
    nd->st.czxid = nd->st.mzxid = nd->st.pzxid = z;
    nd->st.ctime = nd->st.mtime = t;
    nd->st.eph = eph;
    nd->st.dlen = (int32_t)n;
    nd->path = path;
    Node* raw = nd.get();
    nodes[path] = std::move(nd);
    ix_put(raw);
    if (path != "/") {
      Node* par = find(parent_of(path));
      if (par != nullptr) {
        par->kids.insert(path.substr(path.rfind('/') + 1));
        par->st.nkids = (int32_t)par->kids.size();
        par->st.cversion++;
        par->st.pzxid = z;
      }
    }
    return raw;
  }
  std::string passwd() {
    std::string s(16, '\0');
    for (int k = 0; k < 2; ++k) {
      pw_state += 0x9E3779B97F4A7C15ull;
      uint64_t z = pw_state;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      memcpy(&s[8 * k], &z, 8);
    }
    return s;
  }

  // -- watches (callers hold wmu) --------------------------------------------
  // table 0: data watch (of the node, or an exist watch of a missing path);
  // table 1: child watch of the node
  // table 2 (internal): the exist watches of a missing path
  void arm(int table, const std::string& path, Node* nd, int64_t sid,
           SessW* ss = nullptr) {
    if (table == 1) {
      if (nd->cw.add(sid)) (ss ? *ss : sw[sid]).c.insert(nd);
    } else if (nd != nullptr) {
      if (nd->dw.add(sid)) (ss ? *ss : sw[sid]).d.insert(nd);
    } else if (ew[path].add(sid)) {
      (ss ? *ss : sw[sid]).e.insert(path);
    }
  }
  void unlist(int64_t sid, int table, Node* nd, const std::string& path) {
    auto it = sw.find(sid);
    if (it == sw.end()) return;
    if (table == 0) it->second.d.erase(nd);
    else if (table == 1) it->second.c.erase(nd);
    else it->second.e.erase(path);
  }
  // A notification frame for `sid`'s connection: `self` (the connection
  // being served) gets it in its output now, ahead of the reply being
  // built; another connection through its notes and its worker.
  void notify(int64_t sid, int32_t type, const std::string& path, Conn* self);
  // a notification frame (xid -1, SyncConnected) appended to *f
  static void note_frame(std::string* f, int32_t type, const std::string& path);
  // Fire and clear a watcher list (`table`, `nd`: which one, for the
  // sessions' index); returns the sessions notified.
  std::vector<int64_t> fire(Watchers& w, const std::string& path, int32_t type,
                            Conn* self, const std::vector<int64_t>* skip,
                            int table, Node* nd) {
    std::vector<int64_t> sids;
    sids.swap(w.s);
    std::vector<int64_t> fired;
    for (int64_t sid : sids) {
      unlist(sid, table, nd, path);
      if (skip != nullptr &&
          std::find(skip->begin(), skip->end(), sid) != skip->end())
        continue;
      notify(sid, type, path, self);
      fired.push_back(sid);
    }
    return fired;
  }
  // A session's connection is gone: its watches go with it (through the
  // session's index: O(its watches), not a pass over the tree).
  void drop_watches(int64_t sid) {
    auto it = sw.find(sid);
    if (it == sw.end()) return;
    it->second.d.each([&](Node* nd) { nd->dw.drop(sid); });
    it->second.c.each([&](Node* nd) { nd->cw.drop(sid); });
    for (const std::string& p : it->second.e) {
      auto e = ew.find(p);
      if (e == ew.end()) continue;
      e->second.drop(sid);
      if (e->second.s.empty()) ew.erase(e);
    }
    sw.erase(it);
    ++sw_epoch;
  }

  // -- writes (exclusive tree lock; they take wmu to fire) -------------------
  int32_t set_data(const std::string& p, const uint8_t* d, int32_t dl,
                   int32_t ver, Conn* self, Node** out) {
    Node* nd = find(p);
    if (nd == nullptr) return E_NO_NODE;
    if (ver != -1 && ver != nd->st.version) return E_BAD_VERSION;
    nd->data.assign((const char*)d, dl);
    nd->st.version++;
    nd->st.mzxid = ++zxid;
    nd->st.mtime = now_ms();
    nd->st.dlen = dl;
    if (!nd->dw.s.empty()) {
      std::lock_guard<std::mutex> g(wmu);
      fire(nd->dw, p, EV_DATA_CHANGED, self, nullptr, 0, nd);
    }
    *out = nd;
    return E_OK;
  }

  // SET_WATCHES (relZxid, data, exist, child path lists): re-arm, and fire
  // at once what changed after relZxid (fakezk.py set_watches).  A resume
  // carries every watch of the session (tens of thousands for the bulk
  // watches of the node-wide fan-out): the tree lookups — the cost, one
  // hash probe and its cache misses per path — run on several threads
  // (the tree cannot change: the caller holds the shared tree lock), then
  // the watches are armed or fired in list order under wmu.
  void set_watches(Rd& r, int64_t sid, Conn* self) {
    const int64_t rel = r.i64();
    struct Ent { int list; const char* s; int32_t l; };
    std::vector<Ent> es;
    for (int list = 0; list < 3 && r.ok; ++list) {
      const int32_t cnt = r.i32();
      if (!r.ok || cnt < 0) break;
      es.reserve(es.size() + (size_t)cnt);
      for (int32_t k = 0; k < cnt; ++k) {
        const uint8_t* s; int32_t l;
        if (!r.buf(&s, &l)) break;
        es.push_back({list, (const char*)s, l});
      }
    }
    const size_t n = es.size();
    std::vector<Node*> nds(n);
    // the lookups' misses overlapped (serve_parallel's lookahead): path
    // i + 12's index slot, i + 8's node, i + 4's path bytes prefetched
    auto look = [&](size_t a, size_t b) {
      uint64_t hs[16];
      auto slot = [&](size_t g) -> const IxEnt* {
        const IxEnt* e = ix_slot(hs[g & 15]);
        return e->nd != nullptr && e->h == hs[g & 15] ? e : nullptr;
      };
      auto stage = [&](size_t g, int st) {
        if (g >= b) return;
        if (st == 0) {
          hs[g & 15] = phash(es[g].s, (size_t)es[g].l);
          __builtin_prefetch(ix_slot(hs[g & 15]));
        } else if (const IxEnt* e = slot(g)) {
          if (st == 1) {
            __builtin_prefetch(e->nd);
            __builtin_prefetch((const char*)e->nd + 64);
            __builtin_prefetch((const char*)e->nd + 128);
          } else {
            __builtin_prefetch(e->nd->path.data());
          }
        }
      };
      for (size_t g = a; g < a + 12; ++g) stage(g, 0);
      for (size_t g = a; g < a + 8; ++g) stage(g, 1);
      for (size_t g = a; g < a + 4; ++g) stage(g, 2);
      for (size_t i = a; i < b; ++i) {
        stage(i + 12, 0);
        stage(i + 8, 1);
        stage(i + 4, 2);
        nds[i] = ix_find(es[i].s, (size_t)es[i].l, hs[i & 15]);
      }
    };
    // on the read-burst helpers when they are free (no thread started per
    // call), else on this thread
    const int K = n >= SW_PAR_MIN && pool != nullptr
                      ? std::min<int>(pool->size() + 1, (int)SW_THREADS)
                      : 1;
    if (K <= 1 || !pool->run(K, [&](int k) {
          look(n * k / K, n * (k + 1) / K);
        }))
      look(0, n);
    std::lock_guard<std::mutex> g(wmu);
    SessW& ss = sw[sid];
    ss.d.reserve(ss.d.size() + n);
    std::string path;
    auto P = [&](size_t i) -> const std::string& {
      path.assign(es[i].s, (size_t)es[i].l);
      return path;
    };
    for (size_t i = 0; i < n; ++i) {
      if (i + 8 < n && nds[i + 8] != nullptr)
        __builtin_prefetch(nds[i + 8]->dw.s.data());
      Node* nd = nds[i];
      if (es[i].list == 0) {
        if (nd == nullptr) notify(sid, EV_DELETED, P(i), self);
        else if (nd->st.mzxid > rel) notify(sid, EV_DATA_CHANGED, P(i), self);
        else if (nd->dw.add(sid)) ss.d.insert(nd);        // (arm 0)
      } else if (es[i].list == 1) {
        if (nd != nullptr) notify(sid, EV_CREATED, P(i), self);
        else arm(0, P(i), nullptr, sid, &ss);
      } else {
        if (nd == nullptr) notify(sid, EV_DELETED, P(i), self);
        else if (nd->st.pzxid > rel)
          notify(sid, EV_CHILDREN_CHANGED, P(i), self);
        else arm(1, P(i), nd, sid, &ss);
      }
    }
  }

  // One request frame body -> one reply appended to c->out.  Returns false
  // when the connection must close after this reply (CLOSE_SESSION).
  bool serve(const uint8_t* b, int32_t n, Conn* c, std::string* key,
             std::string* out = nullptr) {
    const int64_t sid = c->sid;
    std::string* o = out != nullptr ? out : &c->out;
    Rd r{b, b + n};
    const int32_t xid = r.i32(), op = r.i32();
    if ((op == OP_GET_DATA || op == OP_EXISTS) && r.ok &&
        serve_read(r, xid, op, sid, key, o))
      return true;
    // a SET_WATCHES catch-up notifies this connection before its reply
    if (op == OP_SET_WATCHES && r.ok) set_watches(r, sid, c);
    Wr w{o};
    const size_t at = o->size();
    w.i32(0);                      // frame length, patched below
    w.i32(xid);
    const size_t zat = o->size();
    w.i64(zxid);
    const size_t eat = o->size();
    w.i32(E_OK);
    int32_t err = E_OK;
    bool keep = true;
    auto path = [&]() -> bool {
      const uint8_t* s; int32_t l;
      if (!r.buf(&s, &l)) return false;
      key->assign((const char*)s, l);
      return true;
    };
    if (!r.ok) {
      err = E_MARSHALLING;
    } else {
      switch (op) {
        case OP_PING: case OP_SET_WATCHES: break;
        case OP_CLOSE_SESSION: keep = false; break;
        case OP_GET_DATA: case OP_EXISTS: {
          if (!path()) { err = E_MARSHALLING; break; }
          const bool watch = r.boolean();
          Node* nd = find(*key);
          // EXISTS arms on a missing node too (an exist watch); GET_DATA
          // only on a node it returns
          if (watch && (nd != nullptr || op == OP_EXISTS)) {
            std::lock_guard<std::mutex> g(wmu);
            arm(0, *key, nd, sid);
          }
          if (nd == nullptr) { err = E_NO_NODE; break; }
          if (op == OP_GET_DATA) w.buf(nd->data.data(), nd->data.size());
          w.stat(nd->st);
          break;
        }
        case OP_GET_CHILDREN: case OP_GET_CHILDREN2: {
          if (!path()) { err = E_MARSHALLING; break; }
          const bool watch = r.boolean();
          Node* nd = find(*key);
          if (nd == nullptr) { err = E_NO_NODE; break; }
          if (watch) {
            std::lock_guard<std::mutex> g(wmu);
            arm(1, *key, nd, sid);
          }
          w.i32((int32_t)nd->kids.size());
          for (const auto& k : nd->kids) {
            w.i32((int32_t)k.size());
            o->append(k);
          }
          if (op == OP_GET_CHILDREN2) w.stat(nd->st);
          break;
        }
        case OP_SYNC: {
          if (!path()) { err = E_MARSHALLING; break; }
          w.i32((int32_t)key->size());
          o->append(*key);
          break;
        }
        case OP_SET_DATA: {
          const uint8_t* d; int32_t dl;
          if (!path() || !r.buf(&d, &dl)) { err = E_MARSHALLING; break; }
          const int32_t ver = r.i32();
          Node* nd = nullptr;
          // (a notification to this connection lands before the reply:
          // the reply frame is moved after it)
          const size_t mark = o->size();
          err = set_data(*key, d, dl, ver, c, &nd);
          if (err == E_OK) {
            if (o->size() != mark) {
              std::string note = o->substr(mark);
              o->resize(mark);
              o->insert(at, note);
              return finish(o, at + note.size(), zat + note.size(),
                            eat + note.size(), E_OK, &nd->st, keep);
            }
            w.stat(nd->st);
          }
          break;
        }
        case OP_CREATE: {
          const uint8_t* d; int32_t dl;
          if (!path() || !r.buf(&d, &dl)) { err = E_MARSHALLING; break; }
          const int32_t nacl = r.i32();
          for (int32_t k = 0; k < nacl && r.ok; ++k) {
            const uint8_t* s; int32_t l;
            r.i32(); r.buf(&s, &l); r.buf(&s, &l);
          }
          const int32_t flags = r.i32();
          if (!r.ok) { err = E_MARSHALLING; break; }
          if (key->empty() || (*key)[0] != '/' ||
              (key->size() > 1 && key->back() == '/' && !(flags & 2))) {
            err = E_BAD_ARGUMENTS; break;
          }
          const std::string ppath = parent_of(*key);
          Node* par = find(ppath);
          if (par == nullptr) { err = E_NO_NODE; break; }
          if (par->st.eph != 0) { err = E_NO_CHILDREN_FOR_EPHEMERALS; break; }
          if (flags & 2) {
            char seq[16];
            snprintf(seq, sizeof seq, "%010d", par->st.cversion);
            key->append(seq);
          }
          if (find(*key) != nullptr) { err = E_NODE_EXISTS; break; }
          make(*key, (const char*)d, dl, (flags & 1) ? sid : 0);
          std::string note;
          if (!par->cw.s.empty() || !ew.empty()) {
            std::lock_guard<std::mutex> g(wmu);
            const size_t mark = o->size();
            auto it = ew.find(*key);
            if (it != ew.end()) {
              fire(it->second, *key, EV_CREATED, c, nullptr, 2, nullptr);
              ew.erase(it);
            }
            fire(par->cw, ppath, EV_CHILDREN_CHANGED, c, nullptr, 1, par);
            note = o->substr(mark);
            o->resize(mark);
          }
          w.i32((int32_t)key->size());
          o->append(*key);
          if (!note.empty()) {
            o->insert(at, note);
            return finish(o, at + note.size(), zat + note.size(),
                          eat + note.size(), E_OK, nullptr, keep);
          }
          break;
        }
        case OP_DELETE: {
          if (!path()) { err = E_MARSHALLING; break; }
          const int32_t ver = r.i32();
          Node* nd = find(*key);
          if (nd == nullptr) { err = E_NO_NODE; break; }
          if (ver != -1 && ver != nd->st.version) { err = E_BAD_VERSION; break; }
          if (!nd->kids.empty()) { err = E_NOT_EMPTY; break; }
          const int64_t z = ++zxid;
          const std::string ppath = parent_of(*key);
          Node* par = find(ppath);
          if (par != nullptr) {
            par->kids.erase(key->substr(key->rfind('/') + 1));
            par->st.nkids = (int32_t)par->kids.size();
            par->st.cversion++;
            par->st.pzxid = z;
          }
          std::string note;
          {
            std::lock_guard<std::mutex> g(wmu);
            const size_t mark = o->size();
            const std::vector<int64_t> done =
                fire(nd->dw, *key, EV_DELETED, c, nullptr, 0, nd);
            fire(nd->cw, *key, EV_DELETED, c, &done, 1, nd);
            if (par != nullptr)
              fire(par->cw, ppath, EV_CHILDREN_CHANGED, c, nullptr, 1, par);
            note = o->substr(mark);
            o->resize(mark);
          }
          ix_del(*key);
          nodes.erase(*key);
          if (!note.empty()) {
            o->insert(at, note);
            return finish(o, at + note.size(), zat + note.size(),
                          eat + note.size(), E_OK, nullptr, keep);
          }
          break;
        }
        default: err = E_UNIMPLEMENTED;
      }
    }
    return finish(o, at, zat, eat, err, nullptr, keep);
  }

  // GET_DATA / EXISTS: the reply sized first and written in place (the
  // general path's ~25 string appends a reply were ~230 ns of a GET's
  // ~1 us on a 1M-node tree).  False: a malformed request, for the general
  // path to answer.
  bool serve_read(Rd r, int32_t xid, int32_t op, int64_t sid,
                  std::string* key, std::string* o) {
    const uint8_t* ps;
    int32_t pl;
    if (!r.buf(&ps, &pl)) return false;
    const bool watch = r.boolean();
    if (!r.ok) return false;
    Node* nd = ix_find((const char*)ps, (size_t)pl,
                       phash((const char*)ps, (size_t)pl));
    // EXISTS arms on a missing node too (an exist watch); GET_DATA only on
    // a node it returns
    if (watch && (nd != nullptr || op == OP_EXISTS)) {
      std::lock_guard<std::mutex> g(wmu);
      SessW* ss = sess_w(sid);
      if (nd != nullptr) {
        if (nd->dw.add(sid)) ss->d.insert(nd);          // (arm 0)
      } else {
        key->assign((const char*)ps, pl);
        arm(0, *key, nullptr, sid, ss);
      }
    }
    const size_t dl = nd != nullptr && op == OP_GET_DATA ? nd->data.size() : 0;
    const size_t body = 16 + (nd == nullptr ? 0
                              : (op == OP_GET_DATA ? 4 + dl : 0) + STAT_LEN);
    const size_t at = o->size();
    o->resize(at + 4 + body);
    Put w{(uint8_t*)&(*o)[at]};
    w.i32((int32_t)body);
    w.i32(xid);
    w.i64(zxid);
    w.i32(nd == nullptr ? E_NO_NODE : E_OK);
    if (nd == nullptr) return true;
    if (op == OP_GET_DATA) {
      w.i32(dl == 0 ? -1 : (int32_t)dl);          // (an empty buffer: -1)
      w.raw(nd->data.data(), dl);
    }
    w.stat(nd->st);
    return true;
  }

  // Patch a reply frame's header (the zxid after the request, err, length);
  // `st` (SET_DATA behind a notification): the Stat still to append.
  bool finish(std::string* o, size_t at, size_t zat, size_t eat, int32_t err,
              const Stat* st, bool keep) {
    if (err != E_OK) o->resize(eat + 4);          // header only
    else if (st != nullptr) Wr{o}.stat(*st);
    const int64_t z = zxid;
    uint32_t hi = htonl((uint32_t)(z >> 32)), lo = htonl((uint32_t)z);
    memcpy(&(*o)[zat], &hi, 4);
    memcpy(&(*o)[zat + 4], &lo, 4);
    uint32_t e = htonl((uint32_t)err);
    memcpy(&(*o)[eat], &e, 4);
    uint32_t len = htonl((uint32_t)(o->size() - at - 4));
    memcpy(&(*o)[at], &len, 4);
    return keep;
  }

  // ConnectRequest body -> ConnectResponse frame; the bound session (0 =
  // expired answer).  Exclusive tree lock.
  int64_t handshake(const uint8_t* b, int32_t n, Conn* c) {
    std::string* o = &c->out;
    Rd r{b, b + n};
    r.i32();
    r.i64();
    int32_t to = r.i32();
    int64_t sid = r.i64();
    const uint8_t* pw; int32_t pl = 0;
    r.buf(&pw, &pl);
    std::string pass;
    if (!r.ok) {
      sid = 0; to = 0; pass.assign(16, '\0');
    } else if (sid == 0) {
      sid = (int64_t)0x0100000000000000ll | next_sid++;
      pass = passwd();
      sessions[sid] = pass;
    } else {
      auto it = sessions.find(sid);
      if (it != sessions.end() && pl == 16 &&
          memcmp(pw, it->second.data(), 16) == 0) {
        pass = it->second;
      } else {
        sid = 0; to = 0; pass.assign(16, '\0');
      }
    }
    if (sid != 0) {
      to = to < 4000 ? 4000 : (to > 40000 ? 40000 : to);
      std::lock_guard<std::mutex> g(wmu);
      auto it = route.find(sid);
      // a session moving here from a live connection leaves its watches
      // there (the client re-arms them with SET_WATCHES)
      if (it != route.end() && it->second != c) drop_watches(sid);
      route[sid] = c;
    }
    Wr w{o};
    w.i32(4 + 4 + 8 + 4 + 16 + 1);
    w.i32(0);
    w.i32(to);
    w.i64(sid);
    w.i32(16);
    o->append(pass);
    o->push_back('\0');
    return sid;
  }

  // Connection c is closing (its worker, or an outage): unroute its session
  // and drop the watches that lived on it.  Caller holds mu exclusively.
  void detach(Conn* c) {
    if (c->member >= 0 && c->member < (int)mconns.size())
      mconns[c->member].erase(c);
    if (c->sid == 0) return;
    std::lock_guard<std::mutex> g(wmu);
    auto it = route.find(c->sid);
    if (it != route.end() && it->second == c) {
      route.erase(it);
      drop_watches(c->sid);
    }
  }
};

void preload(Server& S, int64_t n, int32_t dbytes, int32_t fanout) {
  S.make("/", "", 0, 0);
  S.make("/zookeeper", "", 0, 0);
  S.make("/bench", "", 0, 0);
  const int64_t ndirs = (n + fanout - 1) / fanout;
  char p[64];
  for (int64_t d = 0; d < ndirs; ++d) {
    snprintf(p, sizeof p, "/bench/d%06lld", (long long)d);
    S.make(p, "", 0, 0);
  }
  std::string data(dbytes, '\0');
  uint64_t x = 12345;
  for (int64_t i = 0; i < n; ++i) {
    for (int32_t k = 0; k < dbytes; ++k) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      data[k] = (char)(x >> 56);
    }
    snprintf(p, sizeof p, "/bench/d%06lld/n%09lld", (long long)(i / fanout),
             (long long)i);
    S.make(p, data.data(), data.size(), 0);
  }
}

bool flush_out(Conn& c) {
  if (c.out_off >= c.out.size()) return true;
  int64_t t = mono_ns();
  if (c.t_block) { wclock.add(WireClock::BLOCKED, t - c.t_block); c.t_block = 0; }
  bool ok = true;
  while (c.out_off < c.out.size()) {
    ssize_t k = send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off,
                     MSG_NOSIGNAL | MSG_DONTWAIT);
    const int64_t t1 = mono_ns();
    wclock.add(WireClock::SEND, t1 - t);
    wclock.add(WireClock::SENDS, 1);
    if (k > 0) {
      c.out_off += (size_t)k;
      wclock.add(WireClock::TX_BYTES, k);
      wclock.first(WireClock::FIRST_TX, t1);
      wclock.last(WireClock::LAST_TX, t1);
      t = t1;
      continue;
    }
    if (k < 0 && errno == EINTR) { t = t1; continue; }
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      c.t_block = t1;
      return true;
    }
    ok = false;
    break;
  }
  if (!ok) return false;
  c.out.clear();
  c.out_off = 0;
  return true;
}

// Requests that take the tree lock exclusively.  Reads with watch=1 and
// SET_WATCHES only touch the watch tables (their own mutex).
bool is_write(int32_t op) {
  return op == OP_CREATE || op == OP_DELETE || op == OP_SET_DATA ||
         op == OP_CLOSE_SESSION;
}

// One worker: its own epoll set over the connections the acceptor handed
// it (through `pending` + the eventfd), and the connections other workers'
// notifications woke (`woken`).
struct Worker {
  Server* S = nullptr;
  int ep = -1, efd = -1;
  std::mutex mu;
  std::vector<std::pair<int, int>> pending;     // (fd, member)
  std::vector<int> woken;
  std::map<int, std::unique_ptr<Conn>> conns;
  std::string key;
  std::vector<char> rbuf = std::vector<char>(1 << 20);

  void add(int fd, int member) {
    {
      std::lock_guard<std::mutex> g(mu);
      pending.emplace_back(fd, member);
    }
    uint64_t one = 1;
    (void)!write(efd, &one, 8);
  }

  void wake(int fd) {
    {
      std::lock_guard<std::mutex> g(mu);
      woken.push_back(fd);
    }
    uint64_t one = 1;
    (void)!write(efd, &one, 8);
  }

  void drop(int fd) {
    auto it = conns.find(fd);
    if (it != conns.end()) {
      std::unique_lock<std::shared_mutex> ex(S->mu);
      S->detach(it->second.get());
    }
    epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
    conns.erase(fd);
  }

  static void drain_notes(Conn& c) {
    std::lock_guard<std::mutex> g(c.nmu);
    if (!c.notes.empty()) {
      c.out.append(c.notes);
      c.notes.clear();
    }
  }

  // Serve every complete frame of the connection's input (one lock per
  // burst: shared for reads only, exclusive otherwise).
  bool serve_burst(Conn& c) {
    bool writes = !c.hs;
    for (size_t o = c.in_off; !writes && c.in.size() - o >= 8;) {
      uint32_t l, opw;
      memcpy(&l, c.in.data() + o, 4);
      const int32_t len = (int32_t)ntohl(l);
      if (len < 0 || len > MAX_PACKET) break;
      if (c.in.size() - o < 4 + (size_t)len) break;
      if (len >= 8) {
        memcpy(&opw, c.in.data() + o + 8, 4);
        writes = is_write((int32_t)ntohl(opw));
      }
      o += 4 + (size_t)len;
    }
    std::unique_lock<std::shared_mutex> ex(S->mu, std::defer_lock);
    std::shared_lock<std::shared_mutex> sh(S->mu, std::defer_lock);
    if (writes) ex.lock(); else sh.lock();
    // notifications of writes before this burst go out ahead of its replies
    drain_notes(c);
    if (S->pool != nullptr && c.hs &&
        (writes ? serve_parallel_writes(c) : serve_parallel(c)))
      return true;
    // the burst's leading run of reads, for the lookahead
    size_t nread = 0;
    if (c.hs) {
      fr.clear();
      for (size_t o = c.in_off; c.in.size() - o >= 12;) {
        uint32_t l, opw;
        memcpy(&l, c.in.data() + o, 4);
        const int32_t len = (int32_t)ntohl(l);
        if (len < 8 || len > MAX_PACKET || c.in.size() - o < 4 + (size_t)len)
          break;
        memcpy(&opw, c.in.data() + o + 8, 4);
        const int32_t op = (int32_t)ntohl(opw);
        if (op != OP_GET_DATA && op != OP_EXISTS) break;
        fr.emplace_back((uint32_t)(o + 4 - c.in_off), (uint32_t)len);
        o += 4 + (size_t)len;
      }
      nread = fr.size();
    }
    Ahead ah{S, (const uint8_t*)c.in.data() + c.in_off, &fr, nread};
    if (nread > 1) ah.start(0);
    size_t fi = 0;
    bool dead = false;
    while (!c.closing && c.in.size() - c.in_off >= 4) {
      if (fi < nread) ah.step(fi);
      ++fi;
      uint32_t l;
      memcpy(&l, c.in.data() + c.in_off, 4);
      const int32_t len = (int32_t)ntohl(l);
      if (len < 0 || len > MAX_PACKET) { dead = true; break; }
      if (c.in.size() - c.in_off < 4 + (size_t)len) break;
      const uint8_t* b = (const uint8_t*)c.in.data() + c.in_off + 4;
      if (!c.hs) {
        if (!writes) break;            // (cannot happen: !hs => exclusive)
        c.sid = S->handshake(b, len, &c);
        c.hs = true;
        if (c.sid == 0) c.closing = true;
      } else if (!writes && len >= 8) {
        uint32_t opw;
        memcpy(&opw, b + 4, 4);
        if (is_write((int32_t)ntohl(opw))) break;   // next burst, exclusive
        if (!S->serve(b, len, &c, &key)) c.closing = true;
      } else if (!S->serve(b, len, &c, &key)) {
        c.closing = true;
      }
      c.in_off += 4 + (size_t)len;
    }
    return !dead;
  }

  // A read burst of plain reads (GET_DATA, EXISTS, children, SYNC, PING:
  // nothing that notifies this connection) of at least PAR_MIN frames,
  // served in chunks on the pool; the replies appended in request order.
  // False: not such a burst (or the pool is busy): the serial path.
  static constexpr size_t PAR_MIN = 8192;

  // Read lookups' cache misses overlapped (a 1M-node tree is ~0.5 GB of
  // nodes, paths and data: each GET's index slot, node, path and data are
  // DRAM and TLB misses, ~1 us a GET served one after another): while
  // frame f is served, frame f + 12's index slot, f + 8's node and f + 4's
  // path and data are prefetched.  Frames (body offset, length) from
  // `base`; frames without a leading path prefetch nothing.
  struct Ahead {
    Server* S;
    const uint8_t* base;
    const std::vector<std::pair<uint32_t, uint32_t>>* fr;
    size_t end;
    uint64_t hs[16];
    void stage(size_t g, int st) {
      if (g >= end) return;
      if (st == 0) {
        const uint8_t* b = base + (*fr)[g].first;
        const uint32_t n = (*fr)[g].second;
        hs[g & 15] = 0;
        if (n < 12) return;
        uint32_t pl;
        memcpy(&pl, b + 8, 4);
        pl = ntohl(pl);
        if (pl > n - 12) return;
        const uint64_t h = Server::phash((const char*)b + 12, pl);
        hs[g & 15] = h ? h : 1;
        __builtin_prefetch(S->ix_slot(h));
        return;
      }
      const uint64_t h = hs[g & 15];
      if (h == 0) return;
      const Server::IxEnt* e = S->ix_slot(h);
      if (e->nd == nullptr || e->h != h) return;
      const char* nd = (const char*)e->nd;
      if (st == 1) {
        __builtin_prefetch(nd);
        __builtin_prefetch(nd + 64);
        __builtin_prefetch(nd + 128);
      } else {
        __builtin_prefetch(e->nd->path.data());
        __builtin_prefetch(e->nd->data.data());
        __builtin_prefetch(e->nd->data.data() + 64);
      }
    }
    void start(size_t f0) {
      for (size_t g = f0; g < f0 + 12; ++g) stage(g, 0);
      for (size_t g = f0; g < f0 + 8; ++g) stage(g, 1);
      for (size_t g = f0; g < f0 + 4; ++g) stage(g, 2);
    }
    void step(size_t f) {
      stage(f + 12, 0);
      stage(f + 8, 1);
      stage(f + 4, 2);
    }
  };
  std::vector<std::pair<uint32_t, uint32_t>> fr;   // (body offset, length)
  bool serve_parallel(Conn& c) {
    fr.clear();
    size_t o = c.in_off;
    while (c.in.size() - o >= 12) {
      uint32_t l, opw;
      memcpy(&l, c.in.data() + o, 4);
      const int32_t len = (int32_t)ntohl(l);
      if (len < 8 || len > MAX_PACKET) break;
      if (c.in.size() - o < 4 + (size_t)len) break;
      memcpy(&opw, c.in.data() + o + 8, 4);
      const int32_t op = (int32_t)ntohl(opw);
      if (op != OP_GET_DATA && op != OP_EXISTS && op != OP_GET_CHILDREN &&
          op != OP_GET_CHILDREN2 && op != OP_SYNC && op != OP_PING)
        break;
      fr.emplace_back((uint32_t)(o + 4 - c.in_off), (uint32_t)len);
      o += 4 + (size_t)len;
    }
    if (fr.size() < PAR_MIN) return false;
    const int K = std::min<int>(S->pool->size() + 1,
                                (int)(fr.size() / (PAR_MIN / 4)));
    std::vector<std::string> outs(K);
    const uint8_t* base = (const uint8_t*)c.in.data() + c.in_off;
    const size_t nf = fr.size();
    const int64_t tp = mono_ns();
    const bool ran = S->pool->run(K, [&](int k) {
      std::string key;
      const size_t f0 = nf * k / K, f1 = nf * (k + 1) / K;
      outs[k].reserve((f1 - f0) * 200);
      Ahead ah{S, base, &fr, f1};
      ah.start(f0);
      for (size_t f = f0; f < f1; ++f) {
        ah.step(f);
        S->serve(base + fr[f].first, (int32_t)fr[f].second, &c, &key,
                 &outs[k]);
      }
    });
    if (!ran) return false;
    wclock.add(WireClock::PAR_BURSTS, 1);
    wclock.add(WireClock::PAR_NS, mono_ns() - tp);
    for (auto& x : outs) c.out.append(x);
    c.in_off = o;
    return true;
  }

  // A write burst of SET_DATAs (at least WPAR_MIN frames, each path once —
  // the bulk SET of BASELINE config 4: 4096 watched paths a step) on the
  // pool, under the exclusive lock the caller holds.  ZooKeeper's commit
  // order is kept: every outcome depends only on its own node (distinct
  // paths), so the lookups and checks run in parallel, the zxids are then
  // assigned in request order on this thread, the nodes are updated and
  // the replies built in parallel chunks (appended in order), and the
  // watches fire on this thread in request order, each watching
  // connection's notifications appended and its worker woken once (not
  // once per notification).  A watch of the writing session itself (config
  // 4 at one rank: the writer watches every path) is answered as the
  // serial path answers it, its notification right before the write's
  // reply, inside the chunk.  Anything else — another op, a repeated path,
  // a malformed frame, a session routed to another connection — returns
  // false before anything changed: the serial path serves the burst.
  // Round 5's config 4 spent 51 ms of its 70.8 ms write phase (20 steps)
  // here serially.
  static constexpr size_t WPAR_MIN = 512;
  struct WJob {
    Node* nd;
    const uint8_t* d;
    int32_t dl, ver, xid, err;
    bool self;             // the writing session watches the node
    int64_t z;
    std::string path;
  };
  std::vector<WJob> wj;
  bool serve_parallel_writes(Conn& c) {
    fr.clear();
    size_t o = c.in_off;
    while (c.in.size() - o >= 12) {
      uint32_t l, opw;
      memcpy(&l, c.in.data() + o, 4);
      const int32_t len = (int32_t)ntohl(l);
      if (len < 8 || len > MAX_PACKET) break;
      if (c.in.size() - o < 4 + (size_t)len) break;
      memcpy(&opw, c.in.data() + o + 8, 4);
      if ((int32_t)ntohl(opw) != OP_SET_DATA) break;
      fr.emplace_back((uint32_t)(o + 4 - c.in_off), (uint32_t)len);
      o += 4 + (size_t)len;
    }
    const size_t nf = fr.size();
    if (nf < WPAR_MIN) return false;
    const int K = std::min<int>(S->pool->size() + 1, (int)(nf / 128));
    const uint8_t* base = (const uint8_t*)c.in.data() + c.in_off;
    const int64_t sid = c.sid;
    const auto rt = S->route.find(sid);
    const bool routed = rt != S->route.end() && rt->second == &c;
    wj.resize(nf);
    std::atomic<bool> bad{false};
    const int64_t tp = mono_ns();
    // 1. parse, look up, check (the tree is only read)
    if (!S->pool->run(K, [&](int k) {
          const size_t f0 = nf * k / K, f1 = nf * (k + 1) / K;
          Ahead ah{S, base, &fr, f1};
          ah.start(f0);
          for (size_t f = f0; f < f1; ++f) {
            ah.step(f);
            WJob& j = wj[f];
            Rd r{base + fr[f].first, base + fr[f].first + fr[f].second};
            j.xid = r.i32();
            r.i32();
            const uint8_t* s; int32_t sl;
            if (!r.buf(&s, &sl) || !r.buf(&j.d, &j.dl)) { bad = true; return; }
            j.ver = r.i32();
            if (!r.ok) { bad = true; return; }
            j.path.assign((const char*)s, sl);
            j.nd = S->find(j.path);
            j.err = j.nd == nullptr ? E_NO_NODE
                    : (j.ver != -1 && j.ver != j.nd->st.version) ? E_BAD_VERSION
                                                                 : E_OK;
            j.self = false;
            if (j.err == E_OK)
              for (int64_t x : j.nd->dw.s)
                if (x == sid) {
                  if (!routed) { bad = true; return; }
                  j.self = true;
                }
          }
        }))
      return false;
    if (bad) return false;
    {
      std::vector<Node*> ns;
      ns.reserve(nf);
      for (const WJob& j : wj)
        if (j.nd != nullptr) ns.push_back(j.nd);
      std::sort(ns.begin(), ns.end());
      if (std::adjacent_find(ns.begin(), ns.end()) != ns.end()) return false;
    }
    // 2. the commit order: zxids in request order (a failed write leaves
    // the counter, its reply header carries the current one)
    for (WJob& j : wj) j.z = j.err == E_OK ? ++S->zxid : S->zxid;
    // 3. apply and answer, in parallel chunks
    const int64_t t = now_ms();
    std::vector<std::string> outs(K);
    S->pool->run(K, [&](int k) {
      const size_t f0 = nf * k / K, f1 = nf * (k + 1) / K;
      std::string& out = outs[k];
      // sized once: replies (header + Stat, or the header alone) and the
      // session's own notifications
      size_t need = 0;
      for (size_t f = f0; f < f1; ++f) {
        const WJob& j = wj[f];
        need += j.err != E_OK ? 20 : 20 + STAT_LEN;
        if (j.err == E_OK && j.self) need += 32 + j.path.size();
      }
      out.resize(need);
      Put w{(uint8_t*)&out[0]};
      for (size_t f = f0; f < f1; ++f) {
        WJob& j = wj[f];
        if (j.err != E_OK) {
          w.i32(16); w.i32(j.xid); w.i64(j.z); w.i32(j.err);
          continue;
        }
        Node* nd = j.nd;
        nd->data.assign((const char*)j.d, j.dl);
        nd->st.version++;
        nd->st.mzxid = j.z;
        nd->st.mtime = t;
        nd->st.dlen = j.dl;
        // (the session's own watch: its notification, then the reply;
        // note_frame's layout)
        if (j.self) {
          w.i32(28 + (int32_t)j.path.size());
          w.i32(-1); w.i64(-1); w.i32(E_OK);
          w.i32(EV_DATA_CHANGED); w.i32(ST_SYNC_CONNECTED);
          w.i32((int32_t)j.path.size());
          w.raw(j.path.data(), j.path.size());
        }
        w.i32(16 + (int32_t)STAT_LEN); w.i32(j.xid); w.i64(j.z); w.i32(E_OK);
        w.stat(nd->st);
      }
    });
    // 4. the watches, in request order; one append + wake per connection
    std::unordered_map<Conn*, std::string> notes;
    {
      std::lock_guard<std::mutex> g(S->wmu);
      // (a burst's watchers are a few sessions: the last one's index entry,
      // route and note buffer are kept across jobs; each list is cleared in
      // place, its capacity kept for the re-arm)
      int64_t lsid = 0;
      bool known = false;
      Server::SessW* lsw = nullptr;
      Conn* lconn = nullptr;
      std::string* lnotes = nullptr;
      for (WJob& j : wj) {
        if (j.err != E_OK || j.nd->dw.s.empty()) continue;
        for (int64_t x : j.nd->dw.s) {
          if (!known || x != lsid) {
            known = true;
            lsid = x;
            auto a = S->sw.find(x);
            lsw = a == S->sw.end() ? nullptr : &a->second;
            auto b = S->route.find(x);
            lconn = b == S->route.end() ? nullptr : b->second;
            lnotes = lconn != nullptr && x != sid ? &notes[lconn] : nullptr;
          }
          if (lsw != nullptr) lsw->d.erase(j.nd);          // (unlist)
          if (lconn == nullptr) continue;
          S->n_notes.fetch_add(1, std::memory_order_relaxed);
          if (x == sid) continue;              // (in the replies, step 3)
          Server::note_frame(lnotes, EV_DATA_CHANGED, j.path);
        }
        j.nd->dw.s.clear();
      }
    }
    for (auto& kv : notes) {
      bool was_empty;
      {
        std::lock_guard<std::mutex> g(kv.first->nmu);
        was_empty = kv.first->notes.empty();
        kv.first->notes.append(kv.second);
      }
      if (was_empty) kv.first->w->wake(kv.first->fd);
    }
    for (auto& x : outs) c.out.append(x);
    c.in_off = o;
    wclock.add(WireClock::PAR_BURSTS, 1);
    wclock.add(WireClock::PAR_NS, mono_ns() - tp);
    return true;
  }

  void rearm(int fd, Conn& c) {
    epoll_event e{};
    e.events = EPOLLIN | EPOLLRDHUP | (c.out.empty() ? 0u : (uint32_t)EPOLLOUT);
    e.data.fd = fd;
    epoll_ctl(ep, EPOLL_CTL_MOD, fd, &e);
  }

  void run() {
    epoll_event evs[64];
    for (;;) {
      int ne = epoll_wait(ep, evs, 64, -1);
      if (ne < 0 && errno == EINTR) continue;
      for (int k = 0; k < ne; ++k) {
        const int fd = evs[k].data.fd;
        if (fd == efd) {
          uint64_t v;
          (void)!read(efd, &v, 8);
          std::vector<std::pair<int, int>> fds;
          std::vector<int> wk;
          {
            std::lock_guard<std::mutex> g(mu);
            fds.swap(pending);
            wk.swap(woken);
          }
          for (const auto& fm : fds) {
            auto cn = std::make_unique<Conn>();
            cn->fd = fm.first;
            cn->member = fm.second;
            cn->w = this;
            {
              std::unique_lock<std::shared_mutex> ex(S->mu);
              if (fm.second < (int)S->mconns.size())
                S->mconns[fm.second].insert(cn.get());
            }
            conns[fm.first] = std::move(cn);
            epoll_event e{};
            e.events = EPOLLIN | EPOLLRDHUP;
            e.data.fd = fm.first;
            epoll_ctl(ep, EPOLL_CTL_ADD, fm.first, &e);
          }
          for (int f : wk) {
            auto it = conns.find(f);
            if (it == conns.end()) continue;
            Conn& c = *it->second;
            drain_notes(c);
            if (!flush_out(c)) { drop(f); continue; }
            rearm(f, c);
          }
          continue;
        }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        Conn& c = *it->second;
        bool dead = false;
        if (evs[k].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          int64_t t = mono_ns();
          for (;;) {
            ssize_t m = recv(fd, rbuf.data(), rbuf.size(), MSG_DONTWAIT);
            const int64_t t1 = mono_ns();
            wclock.add(WireClock::RECV, t1 - t);
            wclock.add(WireClock::RECVS, 1);
            t = t1;
            if (m > 0) {
              c.in.append(rbuf.data(), (size_t)m);
              wclock.add(WireClock::RX_BYTES, m);
              wclock.first(WireClock::FIRST_RX, t1);
              wclock.last(WireClock::LAST_RX, t1);
              continue;
            }
            if (m == 0) { dead = true; break; }
            if (errno == EINTR) continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK) dead = true;
            break;
          }
          // a read burst may end at a write frame: serve until no frame
          // is left or a partial one
          for (int guard = 0; guard < 1 << 20; ++guard) {
            const size_t before = c.in_off;
            if (!serve_burst(c)) { dead = true; break; }
            if (c.in_off == before || c.closing) break;
          }
          const int64_t t2 = mono_ns();
          wclock.add(WireClock::SERVE, t2 - t);
          wclock.add(WireClock::BURSTS, 1);
          if (c.in_off == c.in.size()) { c.in.clear(); c.in_off = 0; }
          else if (c.in_off > (1u << 20)) { c.in.erase(0, c.in_off); c.in_off = 0; }
        }
        drain_notes(c);
        if (!flush_out(c)) dead = true;
        if (!dead && c.closing && c.out.empty()) dead = true;
        if (dead) { drop(fd); continue; }
        rearm(fd, c);
      }
    }
  }
};

void Server::note_frame(std::string* f, int32_t type, const std::string& path) {
  Wr w{f};
  w.i32(4 + 8 + 4 + 4 + 4 + 4 + (int32_t)path.size());
  w.i32(-1);                       // xid: notification
  w.i64(-1);
  w.i32(E_OK);
  w.i32(type);
  w.i32(ST_SYNC_CONNECTED);
  w.i32((int32_t)path.size());
  f->append(path);
}

void Server::notify(int64_t sid, int32_t type, const std::string& path,
                    Conn* self) {
  auto it = route.find(sid);
  if (it == route.end()) return;
  Conn* c = it->second;
  std::string f;
  note_frame(&f, type, path);
  n_notes.fetch_add(1, std::memory_order_relaxed);
  if (c == self) {
    c->out.append(f);
    return;
  }
  // one wake per batch of notes: a connection whose notes are not empty
  // has a wake pending since they last were (its worker drains them all
  // under nmu) — a write burst firing 4096 watches made 4096 eventfd writes
  bool was_empty;
  {
    std::lock_guard<std::mutex> g(c->nmu);
    was_empty = c->notes.empty();
    c->notes.append(f);
  }
  if (was_empty) c->w->wake(c->fd);
}

// -- members and the fault channel (main thread) ------------------------------

struct Member {
  int port = 0;
  int ls = -1;
};

int listen_on(int port) {
  int ls = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons((uint16_t)port);
  if (bind(ls, (sockaddr*)&a, sizeof a) != 0 || listen(ls, 128) != 0) {
    close(ls);
    return -1;
  }
  return ls;
}

int port_of(int ls) {
  sockaddr_in a{};
  socklen_t al = sizeof a;
  getsockname(ls, (sockaddr*)&a, &al);
  return ntohs(a.sin_port);
}

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}

// One fault command line -> its answer line.
std::string command(Server& S, std::vector<Member>& mem, int ep,
                    const std::string& line) {
  std::vector<std::string> f;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && (line[i] == ' ' || line[i] == '\t')) ++i;
    size_t j = i;
    while (j < line.size() && line[j] != ' ' && line[j] != '\t') ++j;
    if (j > i) f.push_back(line.substr(i, j - i));
    i = j;
  }
  if (f.empty()) return "ERR empty";
  if (f[0] == "timing") {
    if (f.size() > 1 && f[1] == "reset") { wclock.reset(); return "OK"; }
    return wclock.report();
  }
  if (f.size() < 2) return "ERR missing member";
  const int m = atoi(f[1].c_str());
  if (m < 0 || m >= (int)mem.size()) return "ERR no such member";
  if (f[0] == "outage") {
    std::unique_lock<std::shared_mutex> ex(S.mu);
    if (mem[m].ls >= 0) {
      epoll_ctl(ep, EPOLL_CTL_DEL, mem[m].ls, nullptr);
      close(mem[m].ls);
      mem[m].ls = -1;
    }
    // the member's connections end (their workers see the hang-up and
    // free them); their sessions stay, their watches go
    std::vector<Conn*> cs(S.mconns[m].begin(), S.mconns[m].end());
    for (Conn* c : cs) {
      shutdown(c->fd, SHUT_RDWR);
      S.detach(c);
    }
    for (size_t k = 2; k < f.size(); ++k) {
      const size_t eq = f[k].find('=');
      if (eq == std::string::npos) return "ERR bad set";
      const std::string path = f[k].substr(0, eq), hex = f[k].substr(eq + 1);
      std::string d;
      for (size_t h = 0; h + 1 < hex.size(); h += 2)
        d.push_back((char)(hexval(hex[h]) * 16 + hexval(hex[h + 1])));
      Node* nd = nullptr;
      const int32_t err = S.set_data(path, (const uint8_t*)d.data(),
                                     (int32_t)d.size(), -1, nullptr, &nd);
      if (err != E_OK) return "ERR set " + path;
    }
    return "OK " + std::to_string((long long)S.zxid);
  }
  if (f[0] == "start") {
    if (mem[m].ls < 0) {
      mem[m].ls = listen_on(mem[m].port);
      if (mem[m].ls < 0) return "ERR listen";
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = 1000 + (uint64_t)m;
      epoll_ctl(ep, EPOLL_CTL_ADD, mem[m].ls, &ev);
    }
    return "OK " + std::to_string(mem[m].port);
  }
  return "ERR unknown command " + f[0];
}

}  // namespace

int main(int argc, char** argv) {
  int port = 0, members = 1;
  int64_t pre = 0;
  int32_t dbytes = 100, fanout = 1000;
  unsigned hw = std::thread::hardware_concurrency();
  int nthreads = (int)(hw == 0 ? 4 : (hw < 16 ? hw : 16));
  int serve_threads = (int)(hw == 0 ? 0 : (hw < 8 ? hw - 1 : 7));
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--port")) port = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--preload")) pre = atoll(argv[i + 1]);
    else if (!strcmp(argv[i], "--data-bytes")) dbytes = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--fanout")) fanout = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--threads")) nthreads = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--serve-threads"))
      serve_threads = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--members")) members = atoi(argv[i + 1]);
  }
  if (nthreads < 1) nthreads = 1;
  if (members < 1) members = 1;
  Server S;
  // helpers for a connection's large read bursts (--serve-threads; 0: off)
  ServePool pool(serve_threads);
  if (serve_threads > 0) S.pool = &pool;
  S.mconns.resize(members);
  if (pre > 0) preload(S, pre, dbytes, fanout);
  else { S.make("/", "", 0, 0); S.make("/zookeeper", "", 0, 0); }

  int ep = epoll_create1(0);
  std::vector<Member> mem(members);
  for (int m = 0; m < members; ++m) {
    mem[m].ls = listen_on(m == 0 ? port : 0);
    if (mem[m].ls < 0) {
      perror("zk_fastserver: bind/listen");
      return 1;
    }
    mem[m].port = port_of(mem[m].ls);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 1000 + (uint64_t)m;
    epoll_ctl(ep, EPOLL_CTL_ADD, mem[m].ls, &ev);
  }

  std::vector<std::unique_ptr<Worker>> workers;
  for (int t = 0; t < nthreads; ++t) {
    auto w = std::make_unique<Worker>();
    w->S = &S;
    w->ep = epoll_create1(0);
    w->efd = eventfd(0, EFD_NONBLOCK);
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.fd = w->efd;
    epoll_ctl(w->ep, EPOLL_CTL_ADD, w->efd, &e);
    workers.push_back(std::move(w));
  }
  for (auto& w : workers) {
    Worker* wp = w.get();
    std::thread([wp] { wp->run(); }).detach();
  }
  if (members == 1) {
    printf("PORT %d\n", mem[0].port);
  } else {
    printf("PORTS");
    for (const auto& m : mem) printf(" %d", m.port);
    printf("\n");
  }
  fflush(stdout);

  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = 0;                             // stdin: commands; EOF = exit
  epoll_ctl(ep, EPOLL_CTL_ADD, 0, &ev);
  epoll_event evs[8];
  unsigned rr = 0;
  std::string cmd;
  const int one = 1;
  for (;;) {
    int ne = epoll_wait(ep, evs, 8, -1);
    if (ne < 0 && errno == EINTR) continue;
    for (int k = 0; k < ne; ++k) {
      const uint64_t tag = evs[k].data.u64;
      if (tag == 0) {
        char tmp[4096];
        const ssize_t m = read(0, tmp, sizeof tmp);
        if (m <= 0) _exit(0);
        cmd.append(tmp, (size_t)m);
        size_t nl;
        while ((nl = cmd.find('\n')) != std::string::npos) {
          const std::string line = cmd.substr(0, nl);
          cmd.erase(0, nl + 1);
          const std::string ans = command(S, mem, ep, line);
          printf("%s\n", ans.c_str());
          fflush(stdout);
        }
        continue;
      }
      const int m = (int)(tag - 1000);
      if (m < 0 || m >= members || mem[m].ls < 0) continue;
      for (;;) {
        int c = accept4(mem[m].ls, nullptr, nullptr, SOCK_NONBLOCK);
        if (c < 0) break;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        workers[rr++ % workers.size()]->add(c, m);
      }
    }
  }
}
