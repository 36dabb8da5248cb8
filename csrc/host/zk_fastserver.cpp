// zk_fastserver — a native ZooKeeper wire server for client benchmarks.
//
// The in-process fake server (zkmi/server/fakezk.py) implements the whole
// Appendix-D contract (watches, ensembles, fault hooks) in Python; at tens
// of thousands of requests per second it, not the client, would be what a
// pipelined client benchmark measures.  This server speaks the same wire
// protocol from a pool of epoll threads: handshake (new and resumed sessions),
// PING, GET_DATA, EXISTS, SET_DATA (version CAS), CREATE (persistent,
// EPHEMERAL, SEQUENTIAL), DELETE, SYNC, GET_CHILDREN(2), CLOSE_SESSION.  No
// watches (requests with watch=1 are served, the watch is not kept), no
// ACL checks, no expiry: a data-plane server for throughput and RTT runs.
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
//                      [--fanout F] [--threads T]
// --preload creates /bench, /bench/dDDDDDD and N leaves
// /bench/dDDDDDD/nNNNNNNNNN with B bytes of data each (the layout of
// zkmi/bench/synthetic.py GpuTree).  Prints "PORT <n>" once listening and
// exits when stdin reaches EOF.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/eventfd.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

enum : int32_t {
  OP_CREATE = 1, OP_DELETE = 2, OP_EXISTS = 3, OP_GET_DATA = 4,
  OP_SET_DATA = 5, OP_GET_ACL = 6, OP_GET_CHILDREN = 8, OP_SYNC = 9,
  OP_PING = 11, OP_GET_CHILDREN2 = 12, OP_SET_WATCHES = 101,
  OP_CLOSE_SESSION = -11
};
enum : int32_t {
  E_OK = 0, E_MARSHALLING = -5, E_UNIMPLEMENTED = -6, E_BAD_ARGUMENTS = -8,
  E_NO_NODE = -101, E_BAD_VERSION = -103, E_NO_CHILDREN_FOR_EPHEMERALS = -108,
  E_NODE_EXISTS = -110, E_NOT_EMPTY = -111
};
constexpr int32_t MAX_PACKET = 16 * 1024 * 1024;

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

struct Node {
  std::string data;
  Stat st;
  std::set<std::string> kids;
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

struct Server {
  std::shared_mutex mu;          // the tree and the session table
  std::unordered_map<std::string, std::unique_ptr<Node>> nodes;
  std::unordered_map<int64_t, std::string> sessions;    // sid -> passwd
  int64_t zxid = 1;
  int64_t next_sid = 1;
  uint64_t pw_state = 0x9E3779B97F4A7C15ull;

  Node* find(const std::string& p) {
    auto it = nodes.find(p);
    return it == nodes.end() ? nullptr : it->second.get();
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
    Node* raw = nd.get();
    nodes[path] = std::move(nd);
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

  // One request frame body -> one reply appended to `o`.  Returns false
  // when the connection must close after this reply (CLOSE_SESSION).
  bool serve(const uint8_t* b, int32_t n, int64_t sid, std::string* o,
             std::string* key) {
    Rd r{b, b + n};
    const int32_t xid = r.i32(), op = r.i32();
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
          Node* nd = find(*key);
          if (nd == nullptr) { err = E_NO_NODE; break; }
          if (op == OP_GET_DATA) w.buf(nd->data.data(), nd->data.size());
          w.stat(nd->st);
          break;
        }
        case OP_GET_CHILDREN: case OP_GET_CHILDREN2: {
          if (!path()) { err = E_MARSHALLING; break; }
          Node* nd = find(*key);
          if (nd == nullptr) { err = E_NO_NODE; break; }
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
          Node* nd = find(*key);
          if (nd == nullptr) { err = E_NO_NODE; break; }
          if (ver != -1 && ver != nd->st.version) { err = E_BAD_VERSION; break; }
          nd->data.assign((const char*)d, dl);
          nd->st.version++;
          nd->st.mzxid = ++zxid;
          nd->st.mtime = now_ms();
          nd->st.dlen = dl;
          w.stat(nd->st);
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
          Node* par = find(parent_of(*key));
          if (par == nullptr) { err = E_NO_NODE; break; }
          if (par->st.eph != 0) { err = E_NO_CHILDREN_FOR_EPHEMERALS; break; }
          if (flags & 2) {
            char seq[16];
            snprintf(seq, sizeof seq, "%010d", par->st.cversion);
            key->append(seq);
          }
          if (find(*key) != nullptr) { err = E_NODE_EXISTS; break; }
          make(*key, (const char*)d, dl, (flags & 1) ? sid : 0);
          w.i32((int32_t)key->size());
          o->append(*key);
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
          Node* par = find(parent_of(*key));
          if (par != nullptr) {
            par->kids.erase(key->substr(key->rfind('/') + 1));
            par->st.nkids = (int32_t)par->kids.size();
            par->st.cversion++;
            par->st.pzxid = z;
          }
          nodes.erase(*key);
          break;
        }
        default: err = E_UNIMPLEMENTED;
      }
    }
    if (err != E_OK) o->resize(eat + 4);          // header only
    // the header zxid is the one after this request
    int64_t z = zxid;
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
  // expired answer).
  int64_t handshake(const uint8_t* b, int32_t n, std::string* o) {
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
    if (sid != 0) to = to < 4000 ? 4000 : (to > 40000 ? 40000 : to);
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
};

struct Conn {
  int fd;
  bool hs = false;
  bool closing = false;
  int64_t sid = 0;
  std::string in, out;
  size_t in_off = 0, out_off = 0;
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
  while (c.out_off < c.out.size()) {
    ssize_t k = send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off,
                     MSG_NOSIGNAL | MSG_DONTWAIT);
    if (k > 0) { c.out_off += (size_t)k; continue; }
    if (k < 0 && errno == EINTR) continue;
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return true;
    return false;
  }
  c.out.clear();
  c.out_off = 0;
  return true;
}

bool is_write(int32_t op) {
  return op == OP_CREATE || op == OP_DELETE || op == OP_SET_DATA ||
         op == OP_CLOSE_SESSION;
}

// One worker: its own epoll set over the connections the acceptor handed
// it (through `pending` + the eventfd).
struct Worker {
  Server* S = nullptr;
  int ep = -1, efd = -1;
  std::mutex mu;
  std::vector<int> pending;
  std::map<int, std::unique_ptr<Conn>> conns;
  std::string key;
  std::vector<char> rbuf = std::vector<char>(1 << 20);

  void add(int fd) {
    {
      std::lock_guard<std::mutex> g(mu);
      pending.push_back(fd);
    }
    uint64_t one = 1;
    (void)!write(efd, &one, 8);
  }

  void drop(int fd) {
    epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
    conns.erase(fd);
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
    bool dead = false;
    while (!c.closing && c.in.size() - c.in_off >= 4) {
      uint32_t l;
      memcpy(&l, c.in.data() + c.in_off, 4);
      const int32_t len = (int32_t)ntohl(l);
      if (len < 0 || len > MAX_PACKET) { dead = true; break; }
      if (c.in.size() - c.in_off < 4 + (size_t)len) break;
      const uint8_t* b = (const uint8_t*)c.in.data() + c.in_off + 4;
      if (!c.hs) {
        if (!writes) break;            // (cannot happen: !hs => exclusive)
        c.sid = S->handshake(b, len, &c.out);
        c.hs = true;
        if (c.sid == 0) c.closing = true;
      } else if (!writes && len >= 8) {
        uint32_t opw;
        memcpy(&opw, b + 4, 4);
        if (is_write((int32_t)ntohl(opw))) break;   // next burst, exclusive
        if (!S->serve(b, len, c.sid, &c.out, &key)) c.closing = true;
      } else if (!S->serve(b, len, c.sid, &c.out, &key)) {
        c.closing = true;
      }
      c.in_off += 4 + (size_t)len;
    }
    return !dead;
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
          std::vector<int> fds;
          {
            std::lock_guard<std::mutex> g(mu);
            fds.swap(pending);
          }
          for (int c : fds) {
            auto cn = std::make_unique<Conn>();
            cn->fd = c;
            conns[c] = std::move(cn);
            epoll_event e{};
            e.events = EPOLLIN | EPOLLRDHUP;
            e.data.fd = c;
            epoll_ctl(ep, EPOLL_CTL_ADD, c, &e);
          }
          continue;
        }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        Conn& c = *it->second;
        bool dead = false;
        if (evs[k].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
          for (;;) {
            ssize_t m = recv(fd, rbuf.data(), rbuf.size(), MSG_DONTWAIT);
            if (m > 0) { c.in.append(rbuf.data(), (size_t)m); continue; }
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
          if (c.in_off == c.in.size()) { c.in.clear(); c.in_off = 0; }
          else if (c.in_off > (1u << 20)) { c.in.erase(0, c.in_off); c.in_off = 0; }
        }
        if (!flush_out(c)) dead = true;
        if (!dead && c.closing && c.out.empty()) dead = true;
        if (dead) { drop(fd); continue; }
        epoll_event e{};
        e.events = EPOLLIN | EPOLLRDHUP | (c.out.empty() ? 0 : EPOLLOUT);
        e.data.fd = fd;
        epoll_ctl(ep, EPOLL_CTL_MOD, fd, &e);
      }
    }
  }
};

}  // namespace

int main(int argc, char** argv) {
  int port = 0;
  int64_t pre = 0;
  int32_t dbytes = 100, fanout = 1000;
  unsigned hw = std::thread::hardware_concurrency();
  int nthreads = (int)(hw == 0 ? 4 : (hw < 16 ? hw : 16));
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--port")) port = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--preload")) pre = atoll(argv[i + 1]);
    else if (!strcmp(argv[i], "--data-bytes")) dbytes = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--fanout")) fanout = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--threads")) nthreads = atoi(argv[i + 1]);
  }
  if (nthreads < 1) nthreads = 1;
  Server S;
  if (pre > 0) preload(S, pre, dbytes, fanout);
  else { S.make("/", "", 0, 0); S.make("/zookeeper", "", 0, 0); }

  int ls = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons((uint16_t)port);
  if (bind(ls, (sockaddr*)&a, sizeof a) != 0 || listen(ls, 128) != 0) {
    perror("zk_fastserver: bind/listen");
    return 1;
  }
  socklen_t al = sizeof a;
  getsockname(ls, (sockaddr*)&a, &al);

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
  printf("PORT %d\n", ntohs(a.sin_port));
  fflush(stdout);

  int ep = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = ls;
  epoll_ctl(ep, EPOLL_CTL_ADD, ls, &ev);
  ev.data.fd = 0;                              // stdin EOF = shut down
  epoll_ctl(ep, EPOLL_CTL_ADD, 0, &ev);
  epoll_event evs[8];
  unsigned rr = 0;
  for (;;) {
    int ne = epoll_wait(ep, evs, 8, -1);
    if (ne < 0 && errno == EINTR) continue;
    for (int k = 0; k < ne; ++k) {
      const int fd = evs[k].data.fd;
      if (fd == 0) {
        char tmp[256];
        if (read(0, tmp, sizeof tmp) <= 0) _exit(0);
        continue;
      }
      for (;;) {
        int c = accept4(ls, nullptr, nullptr, SOCK_NONBLOCK);
        if (c < 0) break;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        workers[rr++ % workers.size()]->add(c);
      }
    }
  }
}
