// _zkmach — the client's state machines in C++: the ZooKeeper session
// (lib/zk-session.js:38-375), the connection (lib/connection-fsm.js:27-351)
// and the client lifecycle (lib/client.js:123-181).
//
// Not the mooremachine shape.  The reference (and zkmi's Python oracle,
// zkmi/models/*.py under ZKMI_PY_FSM=1) writes each state as a function that
// subscribes its own listeners on every emitter it cares about and tears
// them down on exit — a subscribe / unsubscribe pair per emitter per
// transition.  Here a machine is a table:
//
//   * one dispatch entry per event kind (Relay objects: each is subscribed
//     ONCE to an emitter — a socket, a connection, the expiry timer — and
//     carries its source), so a transition costs no listener churn;
//   * the state x event switch decides, with the source checked against the
//     machine's current peer (an event from a connection the session has
//     moved away from is simply not for any state), and guards computed in
//     C++ (a ConnectResponse's session id, the protocol version, the
//     session's liveness);
//   * entry actions are C++; what they do to the outside world (send a
//     record, destroy a connection, log) goes through the owner's methods —
//     the Python objects keep the API and listener surface only.
//
// Transitions requested while one runs are queued and applied in order;
// `stateChanged` is emitted on the owner after each entry action, then the
// owner's `_fsm_entered(state)` hook runs (the session's watch engine
// ready / unready), as the FSM runtime (zk_fsm.cpp) does.  Once a state has
// requested its transition, further events for it are dropped (the
// runtime's used-handle rule).
#include <Python.h>

#include <cstdint>
#include <ctime>
#include <unordered_map>
#include <vector>

namespace {

// ---- small C-API helpers ----------------------------------------------------

// owner.name(*args) with a borrowed-args format; nullptr on error
PyObject* callm(PyObject* o, const char* name) {
  return PyObject_CallMethod(o, name, nullptr);
}

bool is_none(PyObject* o) { return o == nullptr || o == Py_None; }

// o.attr (new ref), nullptr + error cleared if missing
PyObject* attr(PyObject* o, const char* name) {
  PyObject* v = PyObject_GetAttrString(o, name);
  if (v == nullptr) PyErr_Clear();
  return v;
}

int64_t attr_i64(PyObject* o, const char* name) {
  PyObject* v = attr(o, name);
  if (v == nullptr) return 0;
  const int64_t r = PyLong_Check(v) ? PyLong_AsLongLong(v) : 0;
  if (PyErr_Occurred()) PyErr_Clear();
  Py_DECREF(v);
  return r;
}

int set_attr(PyObject* o, const char* name, PyObject* v) {
  return PyObject_SetAttrString(o, name, v);
}

// pkt[key] (borrowed) from a dict packet
PyObject* field(PyObject* pkt, const char* key) {
  return PyDict_Check(pkt) ? PyDict_GetItemString(pkt, key) : nullptr;
}

int64_t field_i64(PyObject* pkt, const char* key) {
  PyObject* v = field(pkt, key);
  if (v == nullptr || !PyLong_Check(v)) return 0;
  const int64_t r = PyLong_AsLongLong(v);
  if (PyErr_Occurred()) { PyErr_Clear(); return 0; }
  return r;
}

bool field_is(PyObject* pkt, const char* key, const char* want) {
  PyObject* v = field(pkt, key);
  if (v == nullptr || !PyUnicode_Check(v)) return false;
  return PyUnicode_CompareWithASCIIString(v, want) == 0;
}

bool in_state(PyObject* o, const char* st) {
  PyObject* r = PyObject_CallMethod(o, "isInState", "s", st);
  if (r == nullptr) { PyErr_Clear(); return false; }
  const bool b = PyObject_IsTrue(r) == 1;
  Py_DECREF(r);
  return b;
}

// Report an error raised by an owner call without stopping the machine (an
// exception in a loop callback is reported the same way).
void report() {
  if (PyErr_Occurred()) PyErr_WriteUnraisable(nullptr);
}

void call_void(PyObject* o, const char* name) {
  PyObject* r = callm(o, name);
  if (r == nullptr) report();
  Py_XDECREF(r);
}

// o.log.<level>(fmt, *args) — the owner's bunyan-shaped logger
void logv(PyObject* owner, const char* level, PyObject* args) {
  PyObject* log = attr(owner, "log");
  if (log == nullptr) return;
  PyObject* fn = attr(log, level);
  Py_DECREF(log);
  if (fn == nullptr) return;
  PyObject* r = PyObject_CallObject(fn, args);
  Py_DECREF(fn);
  if (r == nullptr) report();
  Py_XDECREF(r);
}

uint64_t u64(int64_t v) { return (uint64_t)v; }

// conn.server[key] (new ref; None when missing) — a connection's backend
PyObject* server_of(PyObject* conn, const char* key) {
  if (conn == nullptr) return Py_NewRef(Py_None);
  PyObject* sv = attr(conn, "server");
  PyObject* v = sv != nullptr && PyDict_Check(sv)
                    ? PyDict_GetItemString(sv, key) : nullptr;
  Py_XINCREF(v);
  Py_XDECREF(sv);
  return v != nullptr ? v : Py_NewRef(Py_None);
}

// ---- machine base -----------------------------------------------------------

struct Machine;

using EnterFn = void (*)(Machine*, int);
using EventFn = void (*)(Machine*, int, PyObject*, PyObject*);

struct Spec {
  const char* const* names;
  int n;
  EnterFn enter;
  EventFn event;
};

// one subscription of a Relay to an emitter
struct Sub {
  PyObject* src;      // the emitter
  PyObject* evt;      // event name (str)
  PyObject* relay;
};

struct Machine {
  PyObject_HEAD
  const Spec* spec;
  PyObject* owner;
  PyObject* loop;
  int state;                    // -1 before the first transition
  std::vector<int>* queue;
  std::vector<Sub>* subs;
  std::vector<int>* history;
  PyObject* entered;            // owner._fsm_entered or nullptr
  bool busy;
  bool pending;                 // the current state asked for a transition
  int64_t transitions;
  // per-kind scratch
  PyObject* peer;               // connection: its socket
  PyObject* ping_iv;            // connection: the ping interval's loop handle
  PyObject* close_xid;          // connection: CLOSE_SESSION xid (closing)
  int close_n;                  // client: teardown parts done
};

PyTypeObject MachineType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject RelayType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// A Relay is subscribed to one emitter event and hands it to its machine as
// (kind, source, args).
struct Relay {
  PyObject_HEAD
  Machine* m;                   // strong ref
  PyObject* src;                // strong ref
  int kind;
};

void request(Machine* m, int st);

PyObject* Relay_call(Relay* r, PyObject* args, PyObject*) {
  Machine* m = r->m;
  if (m == nullptr || m->state < 0) Py_RETURN_NONE;
  if (m->pending) Py_RETURN_NONE;     // the state already chose its exit
  Py_INCREF(m);
  m->spec->event(m, r->kind, r->src, args);
  Py_DECREF(m);
  if (PyErr_Occurred()) return nullptr;
  Py_RETURN_NONE;
}

int Relay_traverse(Relay* r, visitproc visit, void* arg) {
  Py_VISIT((PyObject*)r->m);
  Py_VISIT(r->src);
  return 0;
}

int Relay_clear(Relay* r) {
  Py_CLEAR(r->m);
  Py_CLEAR(r->src);
  return 0;
}

void Relay_dealloc(Relay* r) {
  PyObject_GC_UnTrack(r);
  Relay_clear(r);
  PyObject_GC_Del(r);
}

// Subscribe (src, evt) -> kind unless already subscribed.
int subscribe(Machine* m, PyObject* src, const char* evt, int kind) {
  for (auto& s : *m->subs)
    if (s.src == src && PyUnicode_CompareWithASCIIString(s.evt, evt) == 0)
      return 0;
  Relay* r = PyObject_GC_New(Relay, &RelayType);
  if (r == nullptr) return -1;
  Py_INCREF(m);
  r->m = m;
  Py_INCREF(src);
  r->src = src;
  r->kind = kind;
  PyObject_GC_Track((PyObject*)r);
  PyObject* e = PyUnicode_FromString(evt);
  PyObject* res = e ? PyObject_CallMethod(src, "on", "OO", e, (PyObject*)r)
                    : nullptr;
  if (res == nullptr) {
    Py_XDECREF(e);
    Py_DECREF(r);
    return -1;
  }
  Py_DECREF(res);
  Py_INCREF(src);
  m->subs->push_back(Sub{src, e, (PyObject*)r});
  return 0;
}

// Drop every subscription whose emitter is not in keep[0..nk).
void unsubscribe_others(Machine* m, PyObject* const* keep, int nk) {
  if (keep == nullptr) nk = 0;
  std::vector<Sub> drop;
  std::vector<Sub> stay;
  for (auto& s : *m->subs) {
    bool k = false;
    for (int i = 0; i < nk; ++i) k = k || (keep[i] != nullptr && keep[i] == s.src);
    (k ? stay : drop).push_back(s);
  }
  m->subs->swap(stay);
  for (auto& s : drop) {
    PyObject* r = PyObject_CallMethod(s.src, "removeListener", "OO", s.evt,
                                      s.relay);
    if (r == nullptr) report();
    Py_XDECREF(r);
    Py_DECREF(s.src);
    Py_DECREF(s.evt);
    Py_DECREF(s.relay);
  }
}

// The state names as interned str objects, made once per name: the
// `state` getter (read on every data-API request: the client, session and
// connection states) and stateChanged hand out these instead of a new str.
PyObject* state_name(const Spec* sp, int st) {
  static std::unordered_map<const char*, PyObject*>* cache = nullptr;
  if (cache == nullptr) cache = new std::unordered_map<const char*, PyObject*>;
  const char* k = sp->names[st];
  auto it = cache->find(k);
  if (it != cache->end()) {
    Py_INCREF(it->second);
    return it->second;
  }
  PyObject* o = PyUnicode_InternFromString(k);
  if (o == nullptr) return nullptr;
  Py_INCREF(o);                            // the cache's reference
  cache->emplace(k, o);
  return o;
}

// Enter state `st`: entry action, stateChanged, the owner's hook.
void enter(Machine* m, int st) {
  m->state = st;
  m->pending = false;
  ++m->transitions;
  if (m->history->size() > 64)
    m->history->erase(m->history->begin(), m->history->begin() + 32);
  m->history->push_back(st);
  m->spec->enter(m, st);
  if (PyErr_Occurred()) report();
  PyObject* name = state_name(m->spec, st);
  if (name == nullptr) { report(); return; }
  PyObject* r = PyObject_CallMethod(m->owner, "emit", "sO", "stateChanged",
                                    name);
  if (r == nullptr) report();
  Py_XDECREF(r);
  if (m->entered != nullptr) {
    r = PyObject_CallOneArg(m->entered, name);
    if (r == nullptr) report();
    Py_XDECREF(r);
  }
  Py_DECREF(name);
}

void request(Machine* m, int st) {
  m->queue->push_back(st);
  m->pending = true;
  if (m->busy) return;
  m->busy = true;
  Py_INCREF(m);
  while (!m->queue->empty()) {
    const int nxt = m->queue->front();
    m->queue->erase(m->queue->begin());
    enter(m, nxt);
  }
  m->busy = false;
  Py_DECREF(m);
}

// ---- the session ------------------------------------------------------------
// lib/zk-session.js:38-375.  Peers: owner.conn (and owner.old_conn while a
// move is in flight); the owner keeps them as attributes the rest of the
// client reads.

enum { S_DETACHED, S_ATTACHING, S_ATTACHED, S_REATTACHING, S_CLOSING,
       S_EXPIRED, S_CLOSED, S_N };
const char* const S_NAMES[] = {"detached", "attaching", "attached",
                               "reattaching", "closing", "expired", "closed"};
// event kinds: user / timer inputs, then a connection's
enum { SE_ATTACH, SE_CLOSE, SE_EXPIRY, SE_LOST, SE_PACKET, SE_CSTATE };

// the owner's peers as new references (None -> nullptr)
PyObject* peer(Machine* m, const char* name) {
  PyObject* c = attr(m->owner, name);
  if (c == Py_None) { Py_DECREF(c); return nullptr; }
  return c;
}

void sess_sync_subs(Machine* m) {
  PyObject* c = peer(m, "conn");
  PyObject* o = peer(m, "old_conn");
  PyObject* exp = attr(m->owner, "expiry");
  PyObject* keep[3] = {c, o, exp};
  unsubscribe_others(m, keep, 3);
  for (PyObject* x : {c, o}) {
    if (x == nullptr) continue;
    if (subscribe(m, x, "error", SE_LOST) < 0 ||
        subscribe(m, x, "close", SE_LOST) < 0 ||
        subscribe(m, x, "packet", SE_PACKET) < 0 ||
        subscribe(m, x, "stateChanged", SE_CSTATE) < 0)
      report();
  }
  Py_XDECREF(c);
  Py_XDECREF(o);
  Py_XDECREF(exp);
}

bool sess_alive(Machine* m) {
  PyObject* r = callm(m->owner, "isAlive");
  if (r == nullptr) { report(); return false; }
  const bool b = PyObject_IsTrue(r) == 1;
  Py_DECREF(r);
  return b;
}

// drop the current connection (destroyed) and the expiry
void sess_drop_conn(Machine* m) {
  PyObject* c = peer(m, "conn");
  if (c != nullptr) {
    call_void(c, "destroy");
    Py_DECREF(c);
  }
  set_attr(m->owner, "conn", Py_None);
}

void sess_send_cr(Machine* m, PyObject* conn) {
  PyObject* cr = callm(m->owner, "_connect_request");
  if (cr == nullptr) { report(); return; }
  PyObject* r = PyObject_CallMethod(conn, "send", "O", cr);
  Py_DECREF(cr);
  if (r == nullptr) report();
  Py_XDECREF(r);
}

// A ConnectResponse with a live session id: adopt timeout / id / password.
void sess_adopt(Machine* m, PyObject* pkt) {
  PyObject* to = field(pkt, "timeOut");
  PyObject* sid = field(pkt, "sessionId");
  PyObject* pw = field(pkt, "passwd");
  if (to) set_attr(m->owner, "timeout", to);
  if (sid) set_attr(m->owner, "session_id", sid);
  if (pw) set_attr(m->owner, "passwd", pw);
  call_void(m->owner, "resetExpiryTimer");
}

void sess_enter(Machine* m, int st) {
  PyObject* ow = m->owner;
  switch (st) {
    case S_DETACHED:
      sess_drop_conn(m);
      call_void(ow, "watchersDisconnected");
      break;
    case S_ATTACHING: {
      PyObject* c = peer(m, "conn");
      if (c != nullptr) {
        sess_sync_subs(m);
        sess_send_cr(m, c);
        Py_DECREF(c);
      }
      break;
    }
    case S_ATTACHED: {
      PyObject* t = PyFloat_FromDouble((double)time(nullptr));
      if (t) { set_attr(ow, "last_attach", t); Py_DECREF(t); }
      break;
    }
    case S_REATTACHING: {
      PyObject* o = peer(m, "old_conn");
      PyObject* c = peer(m, "conn");
      if (o == nullptr || c == nullptr) {
        PyErr_SetString(PyExc_AssertionError, "reattaching requires oldConn");
        Py_XDECREF(o);
        Py_XDECREF(c);
        return;
      }
      sess_sync_subs(m);
      PyObject* args = Py_BuildValue(
          "(sKNNNN)",
          "attempting to move zookeeper session %016x from %s:%d to %s:%d",
          (unsigned long long)u64(attr_i64(ow, "session_id")),
          server_of(o, "address"),
          server_of(o, "port"),
          server_of(c, "address"),
          server_of(c, "port"));
      if (args != nullptr) { logv(ow, "debug", args); Py_DECREF(args); }
      else report();
      sess_send_cr(m, c);
      Py_DECREF(o);
      Py_DECREF(c);
      break;
    }
    case S_CLOSING: {
      PyObject* c = peer(m, "conn");
      if (c != nullptr) { call_void(c, "close"); Py_DECREF(c); }
      break;
    }
    case S_EXPIRED:
    case S_CLOSED: {
      sess_drop_conn(m);
      PyObject* ex = attr(ow, "expiry");
      if (ex) { call_void(ex, "cancel"); Py_DECREF(ex); }
      PyObject* wt = attr(ow, "wt");
      if (!is_none(wt)) call_void(wt, "close");
      Py_XDECREF(wt);
      PyObject* args = Py_BuildValue(
          "(s)", st == S_EXPIRED ? "ZK session expired" : "ZK session closed");
      if (args) { logv(ow, st == S_EXPIRED ? "warn" : "info", args); Py_DECREF(args); }
      break;
    }
  }
  sess_sync_subs(m);
}

// The move failed (the new connection refused, lost, or the session's
// deadline passed while moving): back to the old connection if it still
// serves, else detach or expire (lib/zk-session.js:298-320).
void sess_revert(Machine* m) {
  PyObject* ow = m->owner;
  PyObject* o = peer(m, "old_conn");
  PyObject* c = peer(m, "conn");
  const bool alive = sess_alive(m);
  if (alive && o != nullptr && in_state(o, "connected")) {
    PyObject* args = Py_BuildValue(
        "(sKNNNN)",
        "reverted move of session %016x (on %s:%d) to new backend (%s:%d)",
        (unsigned long long)u64(attr_i64(ow, "session_id")),
        server_of(o, "address"),
        server_of(o, "port"),
        server_of(c, "address"),
        server_of(c, "port"));
    if (args) { logv(ow, "warn", args); Py_DECREF(args); } else report();
    set_attr(ow, "conn", o);
    set_attr(ow, "old_conn", Py_None);
    request(m, S_ATTACHED);
  } else if (alive) {
    if (o) call_void(o, "destroy");
    request(m, S_DETACHED);
  } else {
    if (o) call_void(o, "close");
    request(m, S_EXPIRED);
  }
  Py_XDECREF(o);
  Py_XDECREF(c);
}

void sess_event(Machine* m, int kind, PyObject* src, PyObject* args) {
  PyObject* ow = m->owner;
  PyObject* a0 = PyTuple_GET_SIZE(args) > 0 ? PyTuple_GET_ITEM(args, 0) : nullptr;
  PyObject* c = peer(m, "conn");
  // connection events only from the session's current connection
  const bool from_conn = kind >= SE_LOST && c != nullptr && src == c;
  Py_XDECREF(c);
  if (kind >= SE_LOST && !from_conn) return;
  switch (m->state) {
    case S_DETACHED:
      if (kind == SE_ATTACH && a0 != nullptr) {
        set_attr(ow, "conn", a0);
        request(m, S_ATTACHING);
      } else if (kind == SE_CLOSE) {
        request(m, S_CLOSED);
      } else if (kind == SE_EXPIRY) {
        request(m, S_EXPIRED);
      }
      break;
    case S_ATTACHING:
      if (kind == SE_LOST) {
        if (sess_alive(m)) request(m, S_DETACHED);
        else if (attr_i64(ow, "session_id") != 0) request(m, S_EXPIRED);
        else request(m, S_DETACHED);
      } else if (kind == SE_PACKET && a0 != nullptr) {
        const int64_t sid = field_i64(a0, "sessionId");
        if (sid == 0) { request(m, S_EXPIRED); break; }
        const bool resumed = attr_i64(ow, "session_id") != 0;
        PyObject* la = Py_BuildValue(
            "(ssKL)", "%s zookeeper session %016x with timeout %d ms",
            resumed ? "resumed" : "created", (unsigned long long)u64(sid),
            (long long)field_i64(a0, "timeOut"));
        if (la) { logv(ow, "info", la); Py_DECREF(la); } else report();
        // the logger gains the session id (log.child(id=...))
        PyObject* log = attr(ow, "log");
        if (log != nullptr) {
          char buf[20];
          snprintf(buf, sizeof buf, "%016llx", (unsigned long long)u64(sid));
          PyObject* child = attr(log, "child");
          PyObject* kw = Py_BuildValue("{ss}", "id", buf);
          PyObject* empty = PyTuple_New(0);
          PyObject* nl = child && kw && empty ? PyObject_Call(child, empty, kw)
                                              : nullptr;
          if (nl != nullptr) { set_attr(ow, "log", nl); Py_DECREF(nl); }
          else report();
          Py_XDECREF(child); Py_XDECREF(kw); Py_XDECREF(empty);
          Py_DECREF(log);
        }
        sess_adopt(m, a0);
        request(m, S_ATTACHED);
      } else if (kind == SE_EXPIRY) {
        request(m, S_EXPIRED);
      } else if (kind == SE_CLOSE) {
        request(m, S_CLOSING);
      }
      break;
    case S_ATTACHED:
      if (kind == SE_PACKET && a0 != nullptr) {
        // every packet keeps the session alive; replies carry the zxid the
        // next ConnectRequest reports, notifications go to the watchers
        call_void(ow, "resetExpiryTimer");
        if (!field_is(a0, "opcode", "NOTIFICATION")) {
          PyObject* z = field(a0, "zxid");
          if (z != nullptr && PyLong_Check(z) &&
              PyLong_AsLongLong(z) > attr_i64(ow, "_last_zxid"))
            set_attr(ow, "_last_zxid", z);
          if (PyErr_Occurred()) PyErr_Clear();
        } else {
          PyObject* r = PyObject_CallMethod(ow, "processNotification", "O", a0);
          if (r == nullptr) report();
          Py_XDECREF(r);
        }
      } else if (kind == SE_LOST) {
        request(m, sess_alive(m) ? S_DETACHED : S_EXPIRED);
      } else if (kind == SE_EXPIRY) {
        request(m, S_EXPIRED);
      } else if (kind == SE_CLOSE) {
        request(m, S_CLOSING);
      } else if (kind == SE_CSTATE && a0 != nullptr) {
        if (PyUnicode_Check(a0) &&
            PyUnicode_CompareWithASCIIString(a0, "connected") == 0) {
          PyObject* o = peer(m, "old_conn");
          if (o != nullptr) {
            call_void(o, "destroy");
            set_attr(ow, "old_conn", Py_None);
            Py_DECREF(o);
            sess_sync_subs(m);
          }
          call_void(ow, "resumeWatches");
        }
        PyObject* wt = attr(ow, "wt");
        if (!is_none(wt)) call_void(ow, "_wt_sync");   // (after SET_WATCHES)
        Py_XDECREF(wt);
      } else if (kind == SE_ATTACH && a0 != nullptr) {
        PyObject* cur = peer(m, "conn");
        set_attr(ow, "old_conn", cur ? cur : Py_None);
        Py_XDECREF(cur);
        set_attr(ow, "conn", a0);
        request(m, S_REATTACHING);
      }
      break;
    case S_REATTACHING:
      if (kind == SE_PACKET && a0 != nullptr) {
        const int64_t sid = field_i64(a0, "sessionId");
        if (sid == 0) { sess_revert(m); break; }
        // the old connection goes once the new one is 'connected'
        PyObject* c2 = peer(m, "conn");
        PyObject* la = Py_BuildValue(
            "(sKNNL)",
            "moved zookeeper session %016x to more preferred backend (%s:%d) "
            "with timeout %d ms",
            (unsigned long long)u64(sid),
            server_of(c2, "address"),
            server_of(c2, "port"),
            (long long)field_i64(a0, "timeOut"));
        Py_XDECREF(c2);
        if (la) { logv(ow, "info", la); Py_DECREF(la); } else report();
        sess_adopt(m, a0);
        call_void(ow, "watchersDisconnected");
        request(m, S_ATTACHED);
      } else if (kind == SE_LOST || kind == SE_EXPIRY) {
        sess_revert(m);
      } else if (kind == SE_CLOSE) {
        PyObject* o = peer(m, "old_conn");
        if (o) { call_void(o, "close"); Py_DECREF(o); }
        request(m, S_CLOSING);
      }
      break;
    case S_CLOSING:
      if (kind == SE_LOST || kind == SE_EXPIRY) request(m, S_CLOSED);
      break;
    default:
      break;          // expired, closed: final
  }
}

const Spec SESSION{S_NAMES, S_N, sess_enter, sess_event};

// ---- the connection ---------------------------------------------------------
// lib/connection-fsm.js:27-351.  Peers: owner.socket (its TcpSocket) and
// owner.session (the session it handshakes for).  The Python shell keeps
// the byte plumbing that belongs to the transport (the decoder, bulk
// batches, bulk notification capture, the native reply router) behind
// _fx_* / _rx_* effect methods; the states, guards, timers and the close
// handshake are here.

enum { C_INIT, C_CONNECTING, C_HANDSHAKING, C_CONNECTED, C_CLOSING, C_ERROR,
       C_CLOSED, C_N };
const char* const C_NAMES[] = {"init", "connecting", "handshaking",
                               "connected", "closing", "error", "closed"};
enum {
  // the owner's inputs (Machine.fire)
  CE_CONNECT, CE_CLOSE, CE_DESTROY, CE_UNWANTED, CE_RX, CE_RXERR,
  CE_PING_TIMEOUT, CE_BULKDONE,
  // relays: the socket's events, the session's state, timers
  CE_SOCK_CONNECT, CE_SOCK_ERROR, CE_SOCK_END, CE_SOCK_CLOSE, CE_SESS_STATE,
  CE_PING_TICK, CE_IMM
};

// A timer whose callback is a relay of `kind` (src None); new ref to the
// loop's handle.  ms < 0: call_soon.
PyObject* schedule(Machine* m, double ms, int kind) {
  Relay* r = PyObject_GC_New(Relay, &RelayType);
  if (r == nullptr) return nullptr;
  Py_INCREF(m);
  r->m = m;
  r->src = Py_NewRef(Py_None);
  r->kind = kind;
  PyObject_GC_Track((PyObject*)r);
  PyObject* h = ms < 0 ? PyObject_CallMethod(m->loop, "call_soon", "O",
                                             (PyObject*)r)
                       : PyObject_CallMethod(m->loop, "call_later", "dO", ms,
                                             (PyObject*)r);
  Py_DECREF(r);
  return h;
}

void cancel(PyObject*& h) {
  if (h == nullptr) return;
  PyObject* r = callm(h, "cancel");
  if (r == nullptr) report();
  Py_XDECREF(r);
  Py_CLEAR(h);
}

void conn_sync_subs(Machine* m) {
  PyObject* sock = peer(m, "socket");
  // the session's state matters only while handshaking (its 'attached')
  PyObject* sess = m->state == C_HANDSHAKING ? peer(m, "session") : nullptr;
  PyObject* keep[2] = {sock, sess};
  unsubscribe_others(m, keep, 2);
  if (sock != nullptr &&
      (subscribe(m, sock, "connect", CE_SOCK_CONNECT) < 0 ||
       subscribe(m, sock, "error", CE_SOCK_ERROR) < 0 ||
       subscribe(m, sock, "end", CE_SOCK_END) < 0 ||
       subscribe(m, sock, "close", CE_SOCK_CLOSE) < 0))
    report();
  if (sess != nullptr && subscribe(m, sess, "stateChanged", CE_SESS_STATE) < 0)
    report();
  Py_XDECREF(sock);
  Py_XDECREF(sess);
}

// owner.last_error = owner._proto_error(code, msg)
void conn_fail_with(Machine* m, const char* code, const char* msg) {
  PyObject* e = PyObject_CallMethod(m->owner, "_proto_error", "ss", code, msg);
  if (e == nullptr) { report(); return; }
  set_attr(m->owner, "last_error", e);
  Py_DECREF(e);
}

void conn_set_error(Machine* m, PyObject* err) {
  set_attr(m->owner, "last_error", err != nullptr ? err : Py_None);
}

bool conn_drained(Machine* m) {
  PyObject* reqs = attr(m->owner, "reqs");
  PyObject* bulks = attr(m->owner, "bulks");
  const bool d = (reqs == nullptr || PyObject_Length(reqs) < 1) &&
                 (bulks == nullptr || PyObject_Length(bulks) < 1);
  if (PyErr_Occurred()) PyErr_Clear();
  Py_XDECREF(reqs);
  Py_XDECREF(bulks);
  return d;
}

// CLOSE_SESSION once, when nothing is outstanding (lib/connection-fsm.js
// closing state)
void conn_send_close(Machine* m) {
  if (m->close_xid != nullptr) return;
  PyObject* x = callm(m->owner, "nextXid");
  if (x == nullptr) { report(); return; }
  m->close_xid = x;
  PyObject* r = PyObject_CallMethod(m->owner, "_fx_send_close", "O", x);
  if (r == nullptr) report();
  Py_XDECREF(r);
}

double conn_ping_interval(Machine* m) {
  PyObject* sess = peer(m, "session");
  PyObject* cfg = attr(m->owner, "config");
  double T = 0, div = 1, floor_ms = 0;
  if (sess != nullptr) {
    PyObject* t = callm(sess, "getTimeout");
    if (t != nullptr) { T = PyFloat_AsDouble(t); Py_DECREF(t); }
  }
  if (cfg != nullptr) {
    PyObject* a = attr(cfg, "ping_interval_divisor");
    PyObject* b = attr(cfg, "ping_floor_ms");
    if (a) { div = PyFloat_AsDouble(a); Py_DECREF(a); }
    if (b) { floor_ms = PyFloat_AsDouble(b); Py_DECREF(b); }
  }
  if (PyErr_Occurred()) PyErr_Clear();
  Py_XDECREF(sess);
  Py_XDECREF(cfg);
  const double v = div > 0 ? T / div : T;
  return v > floor_ms ? v : floor_ms;
}

void conn_enter(Machine* m, int st) {
  PyObject* ow = m->owner;
  // leaving connected / closing: their timers and the close xid go
  cancel(m->ping_iv);
  Py_CLEAR(m->close_xid);
  switch (st) {
    case C_INIT:
      break;
    case C_CONNECTING: {
      // decoder, encoder, codec, socket (with its data listener) made by
      // the shell; the relays go on the new socket before it dials
      PyObject* r = callm(ow, "_fx_open");
      if (r == nullptr) { report(); break; }
      Py_DECREF(r);
      conn_sync_subs(m);
      r = callm(ow, "_fx_dial");
      if (r == nullptr) report();
      Py_XDECREF(r);
      return;
    }
    case C_HANDSHAKING: {
      PyObject* wanted = attr(ow, "wanted");
      const bool w = wanted != nullptr && PyObject_IsTrue(wanted) == 1;
      Py_XDECREF(wanted);
      if (!w) { request(m, C_CLOSED); break; }
      PyObject* cl = attr(ow, "client");
      PyObject* nc = cl ? attr(cl, "note_capture") : nullptr;
      if (nc != nullptr && PyObject_IsTrue(nc) == 1)
        call_void(ow, "start_note_capture");
      Py_XDECREF(nc);
      PyObject* sess = cl ? callm(cl, "getSession") : nullptr;
      Py_XDECREF(cl);
      if (sess == nullptr) { report(); sess = Py_NewRef(Py_None); }
      set_attr(ow, "session", sess);
      if (sess == Py_None) {
        Py_DECREF(sess);
        request(m, C_CLOSED);
        break;
      }
      conn_sync_subs(m);
      PyObject* att = callm(sess, "isAttaching");
      const bool attaching = att != nullptr && PyObject_IsTrue(att) == 1;
      Py_XDECREF(att);
      if (attaching) {
        PyObject* gs = callm(sess, "getState");
        PyObject* args = Py_BuildValue(
            "(sN)", "found ZKSession in state %s while handshaking",
            gs != nullptr ? gs : Py_NewRef(Py_None));
        if (args) { logv(ow, "debug", args); Py_DECREF(args); }
        PyObject* e = PyObject_CallFunction(PyExc_Exception, "s",
                                            "ZKSession attaching to another "
                                            "connection");
        if (e) { set_attr(ow, "last_error", e); Py_DECREF(e); }
        Py_DECREF(sess);
        request(m, C_ERROR);
        break;
      }
      PyObject* r = PyObject_CallMethod(sess, "attachAndSendCR", "O", ow);
      if (r == nullptr) report();
      Py_XDECREF(r);
      Py_DECREF(sess);
      break;
    }
    case C_CONNECTED: {
      m->ping_iv = schedule(m, conn_ping_interval(m), CE_PING_TICK);
      if (m->ping_iv == nullptr) report();
      call_void(ow, "_fx_connected");      // logger, native reply router on
      // 'connect' on the next tick, unless the state is left before it
      m->close_n = (int)m->transitions;
      PyObject* h = schedule(m, -1, CE_IMM);
      if (h == nullptr) report();
      Py_XDECREF(h);
      break;
    }
    case C_CLOSING:
      call_void(ow, "_fx_route_off");
      if (conn_drained(m)) conn_send_close(m);
      break;
    case C_ERROR:
      // fail the outstanding requests, 'error' emitted even though the
      // state is left at once (lib/connection-fsm.js:318-323)
      call_void(ow, "_fx_error");
      request(m, C_CLOSED);
      break;
    case C_CLOSED: {
      call_void(ow, "_fx_closed");
      m->close_n = (int)m->transitions;
      PyObject* h = schedule(m, -1, CE_IMM);
      if (h == nullptr) report();
      Py_XDECREF(h);
      break;
    }
  }
  conn_sync_subs(m);
}

void conn_event(Machine* m, int kind, PyObject* src, PyObject* args) {
  PyObject* ow = m->owner;
  const Py_ssize_t na = PyTuple_GET_SIZE(args);
  PyObject* a0 = na > 0 ? PyTuple_GET_ITEM(args, 0) : nullptr;
  PyObject* a1 = na > 1 ? PyTuple_GET_ITEM(args, 1) : nullptr;
  // relayed events only from the current socket / session
  if (kind >= CE_SOCK_CONNECT && kind <= CE_SOCK_CLOSE) {
    PyObject* sock = peer(m, "socket");
    const bool cur = sock != nullptr && sock == src;
    Py_XDECREF(sock);
    if (!cur) return;
  } else if (kind == CE_SESS_STATE) {
    PyObject* sess = peer(m, "session");
    const bool cur = sess != nullptr && sess == src;
    Py_XDECREF(sess);
    if (!cur) return;
  }
  const int st = m->state;
  // the closing / error paths every live state shares
  auto lost = [&](int to) {
    conn_fail_with(m, "CONNECTION_LOSS", "Connection closed unexpectedly.");
    request(m, to);
  };
  switch (st) {
    case C_INIT:
      if (kind == CE_CONNECT) request(m, C_CONNECTING);
      break;
    case C_CONNECTING:
      if (kind == CE_SOCK_CONNECT) request(m, C_HANDSHAKING);
      else if (kind == CE_SOCK_ERROR) { conn_set_error(m, a0); request(m, C_ERROR); }
      else if (kind == CE_SOCK_CLOSE || kind == CE_CLOSE || kind == CE_DESTROY)
        request(m, C_CLOSED);
      break;
    case C_HANDSHAKING:
      if (kind == CE_RX && a0 != nullptr) {
        const long more = a1 != nullptr ? PyLong_AsLong(a1) : 0;
        if (more > 0) {
          conn_fail_with(m, "UNEXPECTED_PACKET",
                         "Received unexpected additional packet during "
                         "connect phase");
          request(m, C_ERROR);
          break;
        }
        // the ConnectResponse (host codec or the GPU K9 decoder); a decode
        // failure comes back as the error to fail with
        PyObject* pkt = PyObject_CallMethod(ow, "_decode_cr", "O", a0);
        if (pkt == nullptr) { report(); break; }
        if (!PyDict_Check(pkt)) {
          conn_set_error(m, pkt);
          Py_DECREF(pkt);
          request(m, C_ERROR);
          break;
        }
        if (field_i64(pkt, "protocolVersion") != 0) {
          Py_DECREF(pkt);
          conn_fail_with(m, "VERSION_INCOMPAT",
                         "Server version is not compatible");
          request(m, C_ERROR);
          break;
        }
        PyObject* r = PyObject_CallMethod(ow, "emit", "sO", "packet", pkt);
        Py_DECREF(pkt);
        if (r == nullptr) report();
        Py_XDECREF(r);
      } else if (kind == CE_RXERR || kind == CE_SOCK_ERROR) {
        conn_set_error(m, a0);
        request(m, C_ERROR);
      } else if (kind == CE_SOCK_END || kind == CE_SOCK_CLOSE) {
        lost(C_ERROR);
      } else if (kind == CE_CLOSE || kind == CE_DESTROY || kind == CE_UNWANTED) {
        request(m, C_CLOSED);
      } else if (kind == CE_SESS_STATE && a0 != nullptr) {
        // only when the session attached through THIS connection (after a
        // reattach revert the rejected connection must not turn
        // 'connected'; the reference advances on any 'attached')
        if (PyUnicode_Check(a0) &&
            PyUnicode_CompareWithASCIIString(a0, "attached") == 0) {
          PyObject* sess = peer(m, "session");
          PyObject* sc = sess ? attr(sess, "conn") : nullptr;
          const bool mine = sc == ow;
          Py_XDECREF(sc);
          Py_XDECREF(sess);
          if (mine) request(m, C_CONNECTED);
        }
      }
      break;
    case C_CONNECTED:
      if (kind == CE_RX && a0 != nullptr) {
        // replies, notifications, bulk frames: the shell's plumbing; a
        // decode failure comes back as the error
        PyObject* e = PyObject_CallMethod(ow, "_rx_connected", "O", a0);
        if (e == nullptr) { report(); break; }
        if (e != Py_None) { conn_set_error(m, e); request(m, C_ERROR); }
        Py_DECREF(e);
      } else if (kind == CE_RXERR || kind == CE_SOCK_ERROR) {
        conn_set_error(m, a0);
        request(m, C_ERROR);
      } else if (kind == CE_SOCK_END || kind == CE_SOCK_CLOSE) {
        lost(C_ERROR);
      } else if (kind == CE_CLOSE) {
        request(m, C_CLOSING);
      } else if (kind == CE_DESTROY) {
        request(m, C_CLOSED);
      } else if (kind == CE_PING_TIMEOUT) {
        PyObject* e = callm(ow, "_ping_timeout_error");
        if (e == nullptr) { report(); break; }
        conn_set_error(m, e);
        Py_DECREF(e);
        request(m, C_ERROR);
      } else if (kind == CE_PING_TICK) {
        // re-armed before the ping (a slow ping does not drift the period)
        Py_CLEAR(m->ping_iv);
        m->ping_iv = schedule(m, conn_ping_interval(m), CE_PING_TICK);
        if (m->ping_iv == nullptr) report();
        call_void(ow, "ping");
      } else if (kind == CE_IMM && m->close_n == (int)m->transitions) {
        PyObject* r = PyObject_CallMethod(ow, "emit", "s", "connect");
        if (r == nullptr) report();
        Py_XDECREF(r);
      }
      break;
    case C_CLOSING:
      if (kind == CE_RX && a0 != nullptr) {
        // 0: a reply settled, 1: the CLOSE_SESSION reply (or an undecodable
        // frame: last_error set) — done
        PyObject* r = PyObject_CallMethod(
            ow, "_rx_closing", "OO", a0,
            m->close_xid != nullptr ? m->close_xid : Py_None);
        if (r == nullptr) { report(); break; }
        const long v = PyLong_AsLong(r);
        Py_DECREF(r);
        if (v == 1) { request(m, C_CLOSED); break; }
        if (conn_drained(m)) conn_send_close(m);
      } else if (kind == CE_BULKDONE) {
        if (conn_drained(m)) conn_send_close(m);
      } else if (kind == CE_RXERR || kind == CE_SOCK_ERROR) {
        conn_set_error(m, a0);
        request(m, C_CLOSED);
      } else if (kind == CE_SOCK_END || kind == CE_SOCK_CLOSE) {
        request(m, C_CLOSED);
      }
      // destroy() is ignored while closing, as in the reference: the
      // CLOSE_SESSION exchange completes (or the socket dies)
      break;
    case C_CLOSED:
      if (kind == CE_IMM && m->close_n == (int)m->transitions) {
        call_void(ow, "_fx_closed_later");
      }
      break;
    default:
      break;
  }
}

const Spec CONNECTION{C_NAMES, C_N, conn_enter, conn_event};

// ---- the client lifecycle -----------------------------------------------------
// lib/client.js:123-181: normal -> closing (the session, the connection set
// and the resolver each wind down; all three done) -> closed.

enum { K_NORMAL, K_CLOSING, K_CLOSED, K_N };
const char* const K_NAMES[] = {"normal", "closing", "closed"};
enum { KE_CLOSE, KE_SESS_STATE, KE_SET_STATE, KE_RES_STATE, KE_LOG_TICK };

bool str_is(PyObject* v, const char* s) {
  return v != nullptr && PyUnicode_Check(v) &&
         PyUnicode_CompareWithASCIIString(v, s) == 0;
}

double cfg_ms(Machine* m, const char* name) {
  PyObject* cfg = attr(m->owner, "config");
  PyObject* v = cfg ? attr(cfg, name) : nullptr;
  const double r = v ? PyFloat_AsDouble(v) : 1000.0;
  if (PyErr_Occurred()) PyErr_Clear();
  Py_XDECREF(v);
  Py_XDECREF(cfg);
  return r;
}

void client_bump(Machine* m) {
  if (++m->close_n == 3) request(m, K_CLOSED);
}

void client_enter(Machine* m, int st) {
  PyObject* ow = m->owner;
  switch (st) {
    case K_NORMAL: {
      call_void(ow, "_fx_normal");          // the first session, resolver
      if (subscribe(m, ow, "closeAsserted", KE_CLOSE) < 0) report();
      break;
    }
    case K_CLOSING: {
      PyObject* sess = peer(m, "session");
      PyObject* cset = peer(m, "cset");
      PyObject* res = peer(m, "resolver");
      PyObject* keep[3] = {sess, cset, res};
      unsubscribe_others(m, keep, 3);
      if ((sess && subscribe(m, sess, "stateChanged", KE_SESS_STATE) < 0) ||
          (cset && subscribe(m, cset, "stateChanged", KE_SET_STATE) < 0) ||
          (res && subscribe(m, res, "stateChanged", KE_RES_STATE) < 0))
        report();
      m->close_n = 0;
      if (sess && (in_state(sess, "closed") || in_state(sess, "expired")))
        ++m->close_n;
      if (cset && in_state(cset, "stopped")) ++m->close_n;
      if (res && in_state(res, "stopped")) ++m->close_n;
      if (m->close_n == 3) {
        request(m, K_CLOSED);
      } else {
        if (cset) call_void(cset, "stop");
        if (res) call_void(res, "stop");
        if (sess) call_void(sess, "close");
        m->ping_iv = schedule(m, cfg_ms(m, "close_log_interval_ms"),
                              KE_LOG_TICK);
        if (m->ping_iv == nullptr) report();
      }
      Py_XDECREF(sess);
      Py_XDECREF(cset);
      Py_XDECREF(res);
      break;
    }
    case K_CLOSED: {
      cancel(m->ping_iv);
      unsubscribe_others(m, nullptr, 0);
      PyObject* r = PyObject_CallMethod(ow, "emit", "s", "close");
      if (r == nullptr) report();
      Py_XDECREF(r);
      break;
    }
  }
}

void client_event(Machine* m, int kind, PyObject* src, PyObject* args) {
  (void)src;
  PyObject* a0 = PyTuple_GET_SIZE(args) > 0 ? PyTuple_GET_ITEM(args, 0) : nullptr;
  if (m->state == K_NORMAL) {
    if (kind == KE_CLOSE) request(m, K_CLOSING);
    return;
  }
  if (m->state != K_CLOSING) return;
  switch (kind) {
    case KE_SESS_STATE:
      if (str_is(a0, "closed") || str_is(a0, "expired")) client_bump(m);
      break;
    case KE_SET_STATE:
    case KE_RES_STATE:
      if (str_is(a0, "stopped")) client_bump(m);
      break;
    case KE_LOG_TICK: {
      Py_CLEAR(m->ping_iv);
      m->ping_iv = schedule(m, cfg_ms(m, "close_log_interval_ms"),
                            KE_LOG_TICK);
      PyObject* la = Py_BuildValue(
          "(si)", "still waiting for zk client to shut down, %d/3 done",
          m->close_n);
      if (la) { logv(m->owner, "trace", la); Py_DECREF(la); }
      break;
    }
  }
}

const Spec CLIENT{K_NAMES, K_N, client_enter, client_event};

// ---- Python surface ---------------------------------------------------------

int Machine_traverse(Machine* m, visitproc visit, void* arg) {
  Py_VISIT(m->owner);
  Py_VISIT(m->loop);
  Py_VISIT(m->entered);
  Py_VISIT(m->peer);
  Py_VISIT(m->ping_iv);
  Py_VISIT(m->close_xid);
  if (m->subs != nullptr)
    for (auto& s : *m->subs) {
      Py_VISIT(s.src);
      Py_VISIT(s.evt);
      Py_VISIT(s.relay);
    }
  return 0;
}

int Machine_clear(Machine* m) {
  if (m->subs != nullptr) {
    std::vector<Sub> ss;
    ss.swap(*m->subs);
    for (auto& s : ss) {
      Py_XDECREF(s.src);
      Py_XDECREF(s.evt);
      Py_XDECREF(s.relay);
    }
  }
  Py_CLEAR(m->owner);
  Py_CLEAR(m->loop);
  Py_CLEAR(m->entered);
  Py_CLEAR(m->peer);
  Py_CLEAR(m->ping_iv);
  Py_CLEAR(m->close_xid);
  return 0;
}

void Machine_dealloc(Machine* m) {
  PyObject_GC_UnTrack(m);
  Machine_clear(m);
  delete m->queue;
  delete m->subs;
  delete m->history;
  PyObject_GC_Del(m);
}

const Spec* spec_of(const char* kind) {
  if (strcmp(kind, "session") == 0) return &SESSION;
  if (strcmp(kind, "connection") == 0) return &CONNECTION;
  if (strcmp(kind, "client") == 0) return &CLIENT;
  return nullptr;
}

// Machine(kind, owner, loop): not started (start(initial) enters the first
// state, so the owner can finish its constructor first).
PyObject* Machine_new(PyTypeObject*, PyObject* args, PyObject*) {
  const char* kind;
  PyObject *owner, *loop;
  if (!PyArg_ParseTuple(args, "sOO", &kind, &owner, &loop)) return nullptr;
  const Spec* sp = spec_of(kind);
  if (sp == nullptr) {
    PyErr_Format(PyExc_ValueError, "unknown machine %s", kind);
    return nullptr;
  }
  Machine* m = PyObject_GC_New(Machine, &MachineType);
  if (m == nullptr) return nullptr;
  m->spec = sp;
  Py_INCREF(owner);
  m->owner = owner;
  Py_INCREF(loop);
  m->loop = loop;
  m->state = -1;
  m->queue = new std::vector<int>();
  m->subs = new std::vector<Sub>();
  m->history = new std::vector<int>();
  m->entered = PyObject_GetAttrString(owner, "_fsm_entered");
  if (m->entered == nullptr) PyErr_Clear();
  m->busy = m->pending = false;
  m->transitions = 0;
  m->peer = m->ping_iv = m->close_xid = nullptr;
  m->close_n = 0;
  PyObject_GC_Track((PyObject*)m);
  return (PyObject*)m;
}

int state_index(Machine* m, PyObject* name) {
  if (!PyUnicode_Check(name)) return -1;
  for (int i = 0; i < m->spec->n; ++i)
    if (PyUnicode_CompareWithASCIIString(name, m->spec->names[i]) == 0)
      return i;
  return -1;
}

PyObject* Machine_start(Machine* m, PyObject* name) {
  const int st = state_index(m, name);
  if (st < 0 || m->state >= 0) {
    PyErr_SetString(PyExc_ValueError, "start: unknown state or started");
    return nullptr;
  }
  request(m, st);
  if (PyErr_Occurred()) return nullptr;
  Py_RETURN_NONE;
}

// fire(kind, *args): an input that is not an emitter event (the owner's API
// calls: attach, close; a source of None)
PyObject* Machine_fire(Machine* m, PyObject* args) {
  if (PyTuple_GET_SIZE(args) < 1) {
    PyErr_SetString(PyExc_TypeError, "fire(kind, *args)");
    return nullptr;
  }
  const long kind = PyLong_AsLong(PyTuple_GET_ITEM(args, 0));
  if (kind == -1 && PyErr_Occurred()) return nullptr;
  if (m->state < 0 || m->pending) Py_RETURN_NONE;
  PyObject* rest = PyTuple_GetSlice(args, 1, PyTuple_GET_SIZE(args));
  if (rest == nullptr) return nullptr;
  Py_INCREF(m);
  m->spec->event(m, (int)kind, Py_None, rest);
  Py_DECREF(m);
  Py_DECREF(rest);
  if (PyErr_Occurred()) return nullptr;
  Py_RETURN_NONE;
}

// watch(emitter, evt, kind): subscribe a relay (the owner's fixed inputs,
// e.g. the session's expiry timer)
PyObject* Machine_watch(Machine* m, PyObject* args) {
  PyObject* em;
  const char* evt;
  int kind;
  if (!PyArg_ParseTuple(args, "Osi", &em, &evt, &kind)) return nullptr;
  if (subscribe(m, em, evt, kind) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* Machine_in_state(Machine* m, PyObject* name) {
  if (m->state < 0) Py_RETURN_FALSE;
  return PyBool_FromLong(PyUnicode_Check(name) &&
                         PyUnicode_CompareWithASCIIString(
                             name, m->spec->names[m->state]) == 0);
}

PyObject* Machine_get_state(Machine* m, void*) {
  if (m->state < 0) Py_RETURN_NONE;
  return state_name(m->spec, m->state);
}

PyObject* Machine_get_history(Machine* m, void*) {
  PyObject* l = PyList_New((Py_ssize_t)m->history->size());
  if (l == nullptr) return nullptr;
  for (size_t i = 0; i < m->history->size(); ++i)
    PyList_SET_ITEM(l, (Py_ssize_t)i,
                    PyUnicode_FromString(m->spec->names[(*m->history)[i]]));
  return l;
}

PyObject* Machine_get_subs(Machine* m, void*) {
  return PyLong_FromSize_t(m->subs->size());
}

PyObject* Machine_get_transitions(Machine* m, void*) {
  return PyLong_FromLongLong(m->transitions);
}

PyMethodDef Machine_methods[] = {
    {"start", (PyCFunction)Machine_start, METH_O, "start(state)"},
    {"fire", (PyCFunction)Machine_fire, METH_VARARGS, "fire(kind, *args)"},
    {"watch", (PyCFunction)Machine_watch, METH_VARARGS,
     "watch(emitter, evt, kind)"},
    {"in_state", (PyCFunction)Machine_in_state, METH_O, "in_state(name)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Machine_getset[] = {
    {"state", (getter)Machine_get_state, nullptr, "current state", nullptr},
    {"history", (getter)Machine_get_history, nullptr, "recent states",
     nullptr},
    {"subscriptions", (getter)Machine_get_subs, nullptr,
     "relays subscribed", nullptr},
    {"transitions", (getter)Machine_get_transitions, nullptr,
     "transitions so far", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_zkmach",
                      "the client's state machines (session, connection, "
                      "client) in C++", -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__zkmach() {
  MachineType.tp_name = "zkmi._zkmach.Machine";
  MachineType.tp_basicsize = sizeof(Machine);
  MachineType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  MachineType.tp_traverse = (traverseproc)Machine_traverse;
  MachineType.tp_clear = (inquiry)Machine_clear;
  MachineType.tp_dealloc = (destructor)Machine_dealloc;
  MachineType.tp_methods = Machine_methods;
  MachineType.tp_getset = Machine_getset;
  MachineType.tp_new = Machine_new;
  RelayType.tp_name = "zkmi._zkmach.Relay";
  RelayType.tp_basicsize = sizeof(Relay);
  RelayType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  RelayType.tp_traverse = (traverseproc)Relay_traverse;
  RelayType.tp_clear = (inquiry)Relay_clear;
  RelayType.tp_dealloc = (destructor)Relay_dealloc;
  RelayType.tp_call = (ternaryfunc)Relay_call;
  if (PyType_Ready(&MachineType) < 0 || PyType_Ready(&RelayType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&module);
  if (m == nullptr) return nullptr;
  Py_INCREF(&MachineType);
  if (PyModule_AddObject(m, "Machine", (PyObject*)&MachineType) < 0)
    return nullptr;
  // the session's input kinds (Machine.fire / watch)
  PyModule_AddIntConstant(m, "SE_ATTACH", SE_ATTACH);
  PyModule_AddIntConstant(m, "SE_CLOSE", SE_CLOSE);
  PyModule_AddIntConstant(m, "SE_EXPIRY", SE_EXPIRY);
  // the connection's
  PyModule_AddIntConstant(m, "CE_CONNECT", CE_CONNECT);
  PyModule_AddIntConstant(m, "CE_CLOSE", CE_CLOSE);
  PyModule_AddIntConstant(m, "CE_DESTROY", CE_DESTROY);
  PyModule_AddIntConstant(m, "CE_UNWANTED", CE_UNWANTED);
  PyModule_AddIntConstant(m, "CE_RX", CE_RX);
  PyModule_AddIntConstant(m, "CE_RXERR", CE_RXERR);
  PyModule_AddIntConstant(m, "CE_PING_TIMEOUT", CE_PING_TIMEOUT);
  PyModule_AddIntConstant(m, "CE_BULKDONE", CE_BULKDONE);
  return m;
}
