// _zkwatch — the watch-event engine: every server-side watch of a session
// (ZKWatchEvent, lib/zk-session.js:616-1005) as one entry in a native
// table instead of one Python state machine per (path, event).
//
// An entry is (path, kind), kind = createdOrDeleted (EXISTS watch), data
// (GET_DATA watch) or children (GET_CHILDREN2 watch), in one of the
// reference's states:
//
//   disarmed -> wait -> arming -> armed -> (notify) wait -> arming -> ...
//                         |   \-> wait_node (NO_NODE) -> (created) wait
//                         \-> armed (CD + NO_NODE: 'deleted')
//   armed -> resuming (disconnect) -> armed (SET_WATCHES answered)
//   armed -> doublecheck (4h + U(0, 8h)) -> armed
//
// `wait` is the reference's wait_session / wait_connected pair: the entry
// waits until the session is attached and its connection connected (the
// Python session says so with ready(conn) / unready()).  Arming requests go
// out through the connection's request path with a native request object
// whose (reply, error) pair is this engine (the native router settles it
// straight from the receive buffer), so a notification and its re-arm cost
// no Python frame besides the user-visible emit(path, event, *args) and
// the one request call.  The Python side keeps the listeners (ZKWatcher)
// and the SET_WATCHES resume (resume_lists / resumed).
#include <Python.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

enum Kind : int { K_CD = 0, K_DATA = 1, K_CHILD = 2, K_N = 3 };
enum St : uint8_t {
  S_DISARMED, S_WAIT, S_ARMING, S_ARMED, S_WAIT_NODE, S_RESUMING,
  S_DOUBLECHECK
};
const char* const ST_NAME[] = {"disarmed", "wait_session", "arming", "armed",
                               "wait_node", "resuming", "armed.doublecheck"};
const char* const KIND_EVT[] = {"createdOrDeleted", "dataChanged",
                                "childrenChanged"};
const char* const KIND_OP[] = {"EXISTS", "GET_DATA", "GET_CHILDREN2"};

struct Ev {
  uint8_t st = S_DISARMED;
  bool has_prev = false;
  int64_t prev_zxid = 0;
  uint64_t gen = 0;          // bumped on every transition: stale replies
  uint64_t batch = 0;        // the SET_WATCHES resume it rides in
  double due = 0;            // doublecheck deadline (loop ms), when armed
  std::vector<uint8_t> hist; // recent states (introspection, tests)
};

struct Entry {
  PyObject* path;            // str
  Ev ev[K_N];
};

struct Table {
  PyObject_HEAD
  std::unordered_map<std::string, Entry*>* map;
  PyObject* emit;            // emit(path, event, *args)
  PyObject* loop;            // call_soon / call_later / time_ms
  PyObject* conn;            // the connection while ready, else nullptr
  double dc_ms, dc_rand_ms;  // doublecheck delay
  uint64_t batch;            // last resume batch handed out
  PyObject* timer;           // pending doublecheck timer handle
  double timer_due;
  std::mt19937_64* rng;
  bool kick_pending;         // a deferred (re)arming is queued
};

// ---- the request object the router settles --------------------------------

struct Req {
  PyObject_HEAD
  Table* t;
  PyObject* path;
  int kind;
  uint64_t gen;
  bool dc;                   // a doublecheck read, not an arm
  PyObject* listeners;       // {} (the router's "no listeners" check)
  double t_submit;
};

PyTypeObject ReqType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject TableType = {PyVarObject_HEAD_INIT(nullptr, 0)};

Entry* find(Table* t, PyObject* path) {
  Py_ssize_t n;
  const char* s = PyUnicode_AsUTF8AndSize(path, &n);
  if (s == nullptr) return nullptr;
  auto it = t->map->find(std::string(s, (size_t)n));
  return it == t->map->end() ? nullptr : it->second;
}

double now_ms(Table* t) {
  if (t->loop == nullptr) return 0;
  PyObject* r = PyObject_CallMethod(t->loop, "time_ms", nullptr);
  if (r == nullptr) { PyErr_Clear(); return 0; }
  const double v = PyFloat_AsDouble(r);
  Py_DECREF(r);
  return v;
}

void go(Ev& e, uint8_t st) {
  e.st = st;
  ++e.gen;
  if (e.hist.size() >= 64) e.hist.erase(e.hist.begin(), e.hist.begin() + 32);
  e.hist.push_back(st);
}

void schedule_kick(Table* t);
void schedule_dc(Table* t, double due);

// Send the arming (or doublecheck) request of entry e / kind k.  False when
// it could not leave (the entry then waits for the next ready()).
bool send(Table* t, Entry* en, int k, bool dc) {
  if (t->conn == nullptr) return false;
  Ev& e = en->ev[k];
  PyObject* pkt = Py_BuildValue("{s:s,s:O,s:O}", "opcode",
                                dc ? "EXISTS" : KIND_OP[k], "path", en->path,
                                "watch", dc ? Py_False : Py_True);
  if (pkt == nullptr) return false;
  Req* q = PyObject_GC_New(Req, &ReqType);
  if (q == nullptr) { Py_DECREF(pkt); return false; }
  q->t = nullptr;
  q->path = nullptr;
  q->listeners = nullptr;
  Py_INCREF(t);
  q->t = t;
  Py_INCREF(en->path);
  q->path = en->path;
  q->kind = k;
  q->gen = e.gen;
  q->dc = dc;
  q->listeners = PyDict_New();
  q->t_submit = 0;
  PyObject_GC_Track((PyObject*)q);
  PyObject* r = q->listeners ? PyObject_CallMethod(t->conn, "request", "OO",
                                                   pkt, (PyObject*)q)
                             : nullptr;
  Py_DECREF(pkt);
  Py_DECREF(q);
  if (r == nullptr) {
    PyErr_Clear();          // not connected any more: wait for ready()
    return false;
  }
  Py_DECREF(r);
  return true;
}

// wait -> arming for one entry, when ready
void arm_now(Table* t, Entry* en, int k) {
  Ev& e = en->ev[k];
  if (e.st != S_WAIT || t->conn == nullptr) return;
  go(e, S_ARMING);
  if (!send(t, en, k, false)) go(e, S_WAIT);
}

void to_wait(Table* t, Entry* en, int k) {
  go(en->ev[k], S_WAIT);
  arm_now(t, en, k);
}

void to_armed(Table* t, Ev& e) {
  go(e, S_ARMED);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  e.due = now_ms(t) + t->dc_ms + std::round(u(*t->rng) * t->dc_rand_ms);
  schedule_dc(t, e.due);
}

// ---- Req ------------------------------------------------------------------

// Req and Table are GC types: a request the connection still holds refers
// to its table, the table to the connection (and to the session through
// emit, a bound method), so they form cycles the collector must see.
int Req_traverse(Req* q, visitproc visit, void* arg) {
  Py_VISIT((PyObject*)q->t);
  Py_VISIT(q->listeners);
  return 0;
}

int Req_clear(Req* q) {
  Py_CLEAR(q->t);
  Py_CLEAR(q->listeners);
  return 0;
}

void Req_dealloc(Req* q) {
  PyObject_GC_UnTrack(q);
  Req_clear(q);
  Py_CLEAR(q->path);
  PyObject_GC_Del(q);
}

int64_t stat_zxid(PyObject* stat, int k) {
  static const char* const attr[] = {"czxid", "mzxid", "pzxid"};
  PyObject* v = PyObject_GetAttrString(stat, attr[k]);
  if (v == nullptr) { PyErr_Clear(); return 0; }
  const int64_t z = PyLong_AsLongLong(v);
  Py_DECREF(v);
  if (PyErr_Occurred()) PyErr_Clear();
  return z;
}

PyObject* do_emit(Table* t, PyObject* path, PyObject* args_tail,
                  const char* evt) {
  // emit(path, evt, *args_tail)
  if (t->emit == nullptr) Py_RETURN_NONE;          // closed
  PyObject* ev = PyUnicode_FromString(evt);
  const Py_ssize_t n = args_tail ? PyTuple_GET_SIZE(args_tail) : 0;
  PyObject* args = PyTuple_New(2 + n);
  Py_INCREF(path);
  PyTuple_SET_ITEM(args, 0, path);
  PyTuple_SET_ITEM(args, 1, ev);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* x = PyTuple_GET_ITEM(args_tail, i);
    Py_INCREF(x);
    PyTuple_SET_ITEM(args, 2 + i, x);
  }
  PyObject* r = PyObject_Call(t->emit, args, nullptr);
  Py_DECREF(args);
  return r;
}

// The CD kind of a path emitted 'created': its kinds waiting for the node
// arm again (the reference's wait_node listens for that event).
void wake_wait_node(Table* t, Entry* en) {
  for (int k = 0; k < K_N; ++k)
    if (en->ev[k].st == S_WAIT_NODE) to_wait(t, en, k);
}

PyObject* Req_reply(Req* q, PyObject* pkt) {
  Table* t = q->t;
  Entry* en = find(t, q->path);
  if (en == nullptr) { PyErr_Clear(); Py_RETURN_NONE; }
  Ev& e = en->ev[q->kind];
  if (e.gen != q->gen) Py_RETURN_NONE;              // stale
  PyObject* stat = PyDict_GetItemString(pkt, "stat");  // borrowed
  if (q->dc) {
    if (e.st != S_DOUBLECHECK) Py_RETURN_NONE;
    const int64_t z = stat ? stat_zxid(stat, q->kind) : 0;
    const bool bad = !e.has_prev || z != e.prev_zxid;
    to_armed(t, e);
    if (bad) {
      PyErr_SetString(PyExc_Exception,
                      "ZKWatchEvent double-check failed: zkmi has missed a "
                      "ZK event wakeup, this is a bug");
      return nullptr;
    }
    Py_RETURN_NONE;
  }
  if (e.st != S_ARMING) Py_RETURN_NONE;
  const int64_t z = stat ? stat_zxid(stat, q->kind) : 0;
  if (e.has_prev && z == e.prev_zxid) {
    to_armed(t, e);
    Py_RETURN_NONE;
  }
  PyObject* tail = nullptr;
  const char* evt = nullptr;
  if (q->kind == K_CD) {
    evt = "created";
    tail = PyTuple_Pack(1, stat ? stat : Py_None);
  } else if (q->kind == K_DATA) {
    evt = "dataChanged";
    PyObject* d = PyDict_GetItemString(pkt, "data");
    tail = PyTuple_Pack(2, d ? d : Py_None, stat ? stat : Py_None);
  } else {
    evt = "childrenChanged";
    PyObject* c = PyDict_GetItemString(pkt, "children");
    tail = PyTuple_Pack(2, c ? c : Py_None, stat ? stat : Py_None);
  }
  e.prev_zxid = z;
  e.has_prev = true;
  PyObject* r = do_emit(t, q->path, tail, evt);
  Py_DECREF(tail);
  // a listener that raised: its exception is held while the entry's own
  // transitions (which call into Python) run, then handed on to the
  // caller (the loop's errors, like the Python FSM path)
  PyObject *et = nullptr, *ev = nullptr, *tb = nullptr;
  if (r == nullptr) PyErr_Fetch(&et, &ev, &tb);
  if (e.gen == q->gen) to_armed(t, e);
  if (q->kind == K_CD) wake_wait_node(t, en);
  if (r == nullptr) {
    PyErr_Restore(et, ev, tb);
    return nullptr;
  }
  Py_DECREF(r);
  Py_RETURN_NONE;
}

PyObject* Req_error(Req* q, PyObject* args) {
  Table* t = q->t;
  PyObject* err = PyTuple_GET_SIZE(args) > 0 ? PyTuple_GET_ITEM(args, 0)
                                             : Py_None;
  Entry* en = find(t, q->path);
  if (en == nullptr) { PyErr_Clear(); Py_RETURN_NONE; }
  Ev& e = en->ev[q->kind];
  if (e.gen != q->gen) Py_RETURN_NONE;
  if (q->dc) {
    if (e.st == S_DOUBLECHECK) to_armed(t, e);
    Py_RETURN_NONE;
  }
  if (e.st != S_ARMING) Py_RETURN_NONE;
  std::string code;
  PyObject* c = PyObject_GetAttrString(err, "code");
  if (c == nullptr) PyErr_Clear();
  else if (PyUnicode_Check(c)) code = PyUnicode_AsUTF8(c);
  Py_XDECREF(c);
  if (code == "NO_NODE" && q->kind == K_CD) {
    // existence watches arm on a missing node
    PyObject* r = do_emit(t, q->path, nullptr, "deleted");
    PyObject *et = nullptr, *ev = nullptr, *tb = nullptr;
    if (r == nullptr) PyErr_Fetch(&et, &ev, &tb);
    if (e.gen == q->gen) to_armed(t, e);
    if (r == nullptr) {
      PyErr_Restore(et, ev, tb);
      return nullptr;
    }
    Py_DECREF(r);
    Py_RETURN_NONE;
  }
  if (code == "NO_NODE") {
    // wait for the node: the reference subscribes to the watcher's
    // 'created', which arms its existence watch (zk-session.js:891 ->
    // :595-603); the CD kind's 'created' wakes this one
    go(e, S_WAIT_NODE);
    if (en->ev[K_CD].st == S_DISARMED) to_wait(t, en, K_CD);
    Py_RETURN_NONE;
  }
  // PING_TIMEOUT, a lost connection, anything else: back to waiting for
  // an attached session with a connected connection (retried from the
  // loop, not from inside the settle)
  go(e, S_WAIT);
  schedule_kick(t);
  Py_RETURN_NONE;
}

// settle(evt, *args): the connection's fail paths (a closed connection
// fails every outstanding request) and its Python reply path
PyObject* Req_settle(Req* q, PyObject* args) {
  if (PyTuple_GET_SIZE(args) < 1) Py_RETURN_NONE;
  PyObject* evt = PyTuple_GET_ITEM(args, 0);
  PyObject* rest = PyTuple_GetSlice(args, 1, PyTuple_GET_SIZE(args));
  PyObject* r;
  if (PyUnicode_Check(evt) && PyUnicode_CompareWithASCIIString(evt, "reply") == 0)
    r = PyTuple_GET_SIZE(rest) > 0 ? Req_reply(q, PyTuple_GET_ITEM(rest, 0))
                                   : Py_NewRef(Py_None);
  else
    r = Req_error(q, rest);
  Py_DECREF(rest);
  return r;
}

// fast: the (on_reply, on_error) pair, bound afresh on each read (a pair
// kept on the object would be a reference cycle this type cannot collect)
PyObject* Req_get_fast(Req* q, void*) {
  PyObject* a = PyObject_GetAttrString((PyObject*)q, "_reply");
  PyObject* b = a ? PyObject_GetAttrString((PyObject*)q, "_error") : nullptr;
  PyObject* r = (a && b) ? PyTuple_Pack(2, a, b) : nullptr;
  Py_XDECREF(a);
  Py_XDECREF(b);
  return r;
}
PyObject* Req_get_listeners(Req* q, void*) { return Py_NewRef(q->listeners); }
PyObject* Req_get_t_submit(Req* q, void*) { return PyFloat_FromDouble(q->t_submit); }

PyMethodDef Req_methods[] = {
    {"_reply", (PyCFunction)Req_reply, METH_O, "the reply"},
    {"_error", (PyCFunction)Req_error, METH_VARARGS, "an error"},
    {"settle", (PyCFunction)Req_settle, METH_VARARGS, "settle(evt, *args)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Req_getset[] = {
    {"fast", (getter)Req_get_fast, nullptr, "(on_reply, on_error)", nullptr},
    {"_listeners", (getter)Req_get_listeners, nullptr, "{}", nullptr},
    {"t_submit", (getter)Req_get_t_submit, nullptr, "", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ---- Table ----------------------------------------------------------------

int kind_of(PyObject* o) {
  if (PyLong_Check(o)) {
    const long k = PyLong_AsLong(o);
    return (k >= 0 && k < K_N) ? (int)k : -1;
  }
  if (!PyUnicode_Check(o)) return -1;
  for (int k = 0; k < K_N; ++k)
    if (PyUnicode_CompareWithASCIIString(o, KIND_EVT[k]) == 0) return k;
  return -1;
}

int Table_traverse(Table* t, visitproc visit, void* arg) {
  Py_VISIT(t->emit);
  Py_VISIT(t->loop);
  Py_VISIT(t->conn);
  Py_VISIT(t->timer);
  return 0;
}

void cancel_timer(Table* t) {
  if (t->timer == nullptr) return;
  PyObject* r = PyObject_CallMethod(t->timer, "cancel", nullptr);
  if (r == nullptr) PyErr_Clear();
  Py_XDECREF(r);
  Py_CLEAR(t->timer);
  t->timer_due = 0;
}

int Table_clear(Table* t) {
  Py_CLEAR(t->emit);
  Py_CLEAR(t->loop);
  Py_CLEAR(t->conn);
  Py_CLEAR(t->timer);
  return 0;
}

void Table_dealloc(Table* t) {
  PyObject_GC_UnTrack(t);
  if (t->map != nullptr)
    for (auto& kv : *t->map) {
      Py_XDECREF(kv.second->path);
      delete kv.second;
    }
  delete t->map;
  delete t->rng;
  Table_clear(t);
  Py_TYPE(t)->tp_free((PyObject*)t);
}

// WatchTable(emit, loop, doublecheck_ms, doublecheck_rand_ms)
int Table_init(Table* t, PyObject* args, PyObject*) {
  PyObject *emit, *loop;
  double dc, dcr;
  if (!PyArg_ParseTuple(args, "OOdd", &emit, &loop, &dc, &dcr)) return -1;
  if (t->map == nullptr) t->map = new std::unordered_map<std::string, Entry*>();
  if (t->rng == nullptr) t->rng = new std::mt19937_64(std::random_device{}());
  Py_INCREF(emit);
  Py_XSETREF(t->emit, emit);
  Py_INCREF(loop);
  Py_XSETREF(t->loop, loop);
  Py_CLEAR(t->conn);
  t->dc_ms = dc;
  t->dc_rand_ms = dcr;
  t->batch = 0;
  cancel_timer(t);
  t->kick_pending = false;
  return 0;
}

PyObject* Table_new(PyTypeObject* type, PyObject*, PyObject*) {
  Table* t = (Table*)type->tp_alloc(type, 0);
  if (t != nullptr) {
    t->map = nullptr;
    t->rng = nullptr;
    t->emit = t->loop = t->conn = t->timer = nullptr;
  }
  return (PyObject*)t;
}

void schedule_kick(Table* t) {
  if (t->kick_pending || t->conn == nullptr || t->loop == nullptr) return;
  PyObject* cb = PyObject_GetAttrString((PyObject*)t, "_kick");
  if (cb == nullptr) { PyErr_Clear(); return; }
  PyObject* r = PyObject_CallMethod(t->loop, "call_soon", "O", cb);
  Py_DECREF(cb);
  if (r == nullptr) { PyErr_Clear(); return; }
  Py_DECREF(r);
  t->kick_pending = true;
}

// _kick(): arm every waiting entry (the deferred retry after an error)
PyObject* Table_kick(Table* t, PyObject*) {
  t->kick_pending = false;
  if (t->conn == nullptr) Py_RETURN_NONE;
  std::vector<Entry*> all;
  for (auto& kv : *t->map) all.push_back(kv.second);
  for (Entry* en : all)
    for (int k = 0; k < K_N; ++k) arm_now(t, en, k);
  Py_RETURN_NONE;
}

PyObject* Table_dc_tick(Table* t, PyObject*);

void schedule_dc(Table* t, double due) {
  if (t->loop == nullptr) return;                 // closed
  if (t->timer != nullptr && t->timer_due <= due) return;
  if (t->timer != nullptr) {
    PyObject* r = PyObject_CallMethod(t->timer, "cancel", nullptr);
    if (r == nullptr) PyErr_Clear();
    Py_XDECREF(r);
    Py_CLEAR(t->timer);
  }
  PyObject* cb = PyObject_GetAttrString((PyObject*)t, "_dc_tick");
  if (cb == nullptr) { PyErr_Clear(); return; }
  double wait = due - now_ms(t);
  if (wait < 1) wait = 1;
  PyObject* h = PyObject_CallMethod(t->loop, "call_later", "dO", wait, cb);
  Py_DECREF(cb);
  if (h == nullptr) { PyErr_Clear(); return; }
  t->timer = h;
  t->timer_due = due;
}

// _dc_tick(): armed entries whose doublecheck is due re-read their node
// (armed.doublecheck: zk-session.js:923-970); then the next deadline
PyObject* Table_dc_tick(Table* t, PyObject*) {
  Py_CLEAR(t->timer);
  t->timer_due = 0;
  const double now = now_ms(t);
  double next = -1;
  std::vector<std::pair<Entry*, int>> due;
  for (auto& kv : *t->map)
    for (int k = 0; k < K_N; ++k) {
      Ev& e = kv.second->ev[k];
      if (e.st != S_ARMED) continue;
      if (e.due <= now + 0.5) due.emplace_back(kv.second, k);
      else if (next < 0 || e.due < next) next = e.due;
    }
  for (auto& p : due) {
    Ev& e = p.first->ev[p.second];
    go(e, S_DOUBLECHECK);
    if (!send(t, p.first, p.second, true)) to_armed(t, e);
  }
  if (next >= 0) schedule_dc(t, next);
  Py_RETURN_NONE;
}

// arm(path, kind): the first listener for an event (ZKWatcher._armEvent)
PyObject* Table_arm(Table* t, PyObject* args) {
  PyObject *path, *ko;
  if (!PyArg_ParseTuple(args, "UO", &path, &ko)) return nullptr;
  const int k = kind_of(ko);
  if (k < 0) Py_RETURN_NONE;
  Py_ssize_t n;
  const char* s = PyUnicode_AsUTF8AndSize(path, &n);
  if (s == nullptr) return nullptr;
  std::string key(s, (size_t)n);
  Entry*& en = (*t->map)[key];
  if (en == nullptr) {
    en = new Entry();
    Py_INCREF(path);
    en->path = path;
  }
  if (en->ev[k].st == S_DISARMED) to_wait(t, en, k);
  Py_RETURN_NONE;
}

// notify(path, evt) -> bool: a watch event for `path` (ZKWatcher.notify):
// the kinds it fires go back to arming.  False: no entry for the path.
PyObject* Table_notify(Table* t, PyObject* args) {
  PyObject* path;
  const char* evt;
  if (!PyArg_ParseTuple(args, "Us", &path, &evt)) return nullptr;
  Entry* en = find(t, path);
  if (en == nullptr) {
    if (PyErr_Occurred()) return nullptr;
    Py_RETURN_FALSE;
  }
  int kinds[3], nk = 0;
  const std::string e(evt);
  if (e == "created") { kinds[0] = K_CD; kinds[1] = K_DATA; nk = 2; }
  else if (e == "deleted") {
    kinds[0] = K_CD; kinds[1] = K_DATA; kinds[2] = K_CHILD; nk = 3;
  } else if (e == "dataChanged") { kinds[0] = K_DATA; kinds[1] = K_CD; nk = 2; }
  else if (e == "childrenChanged") { kinds[0] = K_CHILD; nk = 1; }
  else {
    PyErr_Format(PyExc_Exception, "Unknown notification type: %s", evt);
    return nullptr;
  }
  bool notified = false;
  for (int i = 0; i < nk; ++i) {
    Ev& v = en->ev[kinds[i]];
    if (v.st == S_DISARMED) continue;
    notified = true;
    if (v.st == S_ARMED || v.st == S_DOUBLECHECK || v.st == S_RESUMING)
      to_wait(t, en, kinds[i]);
  }
  if (!notified) {
    // our picture of which ZK events hit which watches is wrong
    // (zk-session.js:584-592)
    PyErr_Format(PyExc_Exception,
                 "Got notification for %s but have no matching events on %U",
                 evt, en->path);
    return nullptr;
  }
  Py_RETURN_TRUE;
}

// ready(conn): the session is attached and conn connected: waiting entries
// arm now.  unready(): not any more.
PyObject* Table_ready(Table* t, PyObject* conn) {
  Py_INCREF(conn);
  Py_XSETREF(t->conn, conn);
  return Table_kick(t, nullptr);
}

PyObject* Table_unready(Table* t, PyObject*) {
  Py_CLEAR(t->conn);
  Py_RETURN_NONE;
}

// disconnected(): armed -> resuming (the session lost its connection)
PyObject* Table_disconnected(Table* t, PyObject*) {
  for (auto& kv : *t->map)
    for (int k = 0; k < K_N; ++k) {
      Ev& e = kv.second->ev[k];
      if (e.st == S_ARMED || e.st == S_DOUBLECHECK) go(e, S_RESUMING);
    }
  Py_RETURN_NONE;
}

// resume_lists() -> (batch, data, exist, child): the resuming watches for
// one SET_WATCHES (zk-session.js:421-471)
PyObject* Table_resume_lists(Table* t, PyObject*) {
  const uint64_t b = ++t->batch;
  PyObject* l[3] = {PyList_New(0), PyList_New(0), PyList_New(0)};
  for (auto& kv : *t->map) {
    Entry* en = kv.second;
    for (int k = 0; k < K_N; ++k) {
      Ev& e = en->ev[k];
      if (e.st != S_RESUMING) continue;
      e.batch = b;
      // data -> dataChanged, exist -> createdOrDestroyed, child
      PyList_Append(k == K_DATA ? l[0] : k == K_CD ? l[1] : l[2], en->path);
    }
  }
  return Py_BuildValue("(KNNN)", (unsigned long long)b, l[0], l[1], l[2]);
}

// resumed(batch): SET_WATCHES answered OK: that batch's entries still
// resuming are armed again
PyObject* Table_resumed(Table* t, PyObject* arg) {
  const uint64_t b = PyLong_AsUnsignedLongLong(arg);
  if (PyErr_Occurred()) return nullptr;
  for (auto& kv : *t->map)
    for (int k = 0; k < K_N; ++k) {
      Ev& e = kv.second->ev[k];
      if (e.st == S_RESUMING && e.batch == b) to_armed(t, e);
    }
  Py_RETURN_NONE;
}

// state(path, kind) -> str or None; history(path, kind) -> [str]
PyObject* Table_state(Table* t, PyObject* args) {
  PyObject *path, *ko;
  if (!PyArg_ParseTuple(args, "UO", &path, &ko)) return nullptr;
  const int k = kind_of(ko);
  Entry* en = k >= 0 ? find(t, path) : nullptr;
  if (en == nullptr) {
    if (PyErr_Occurred()) return nullptr;
    Py_RETURN_NONE;
  }
  return PyUnicode_FromString(ST_NAME[en->ev[k].st]);
}

PyObject* Table_history(Table* t, PyObject* args) {
  PyObject *path, *ko;
  if (!PyArg_ParseTuple(args, "UO", &path, &ko)) return nullptr;
  const int k = kind_of(ko);
  Entry* en = k >= 0 ? find(t, path) : nullptr;
  PyObject* l = PyList_New(0);
  if (en == nullptr) { PyErr_Clear(); return l; }
  for (uint8_t s : en->ev[k].hist) {
    PyObject* x = PyUnicode_FromString(ST_NAME[s]);
    PyList_Append(l, x);
    Py_DECREF(x);
  }
  return l;
}

PyObject* Table_contains_path(Table* t, PyObject* path) {
  if (!PyUnicode_Check(path)) Py_RETURN_FALSE;
  Entry* en = find(t, path);
  if (en == nullptr && PyErr_Occurred()) return nullptr;
  return PyBool_FromLong(en != nullptr);
}

// close(): the session is closed or expired: no more timers, requests or
// emits; every entry is dropped (its watchers are dead, README.md:47-51)
PyObject* Table_close(Table* t, PyObject*) {
  cancel_timer(t);
  Py_CLEAR(t->conn);
  if (t->map != nullptr) {
    for (auto& kv : *t->map) {
      Py_XDECREF(kv.second->path);
      delete kv.second;
    }
    t->map->clear();
  }
  t->kick_pending = true;                 // nothing more is scheduled
  Py_CLEAR(t->emit);
  Py_CLEAR(t->loop);
  Py_RETURN_NONE;
}

// counts() -> {state: n}: how many watch events are in each state
PyObject* Table_counts(Table* t, PyObject*) {
  int64_t c[7] = {0};
  for (auto& kv : *t->map)
    for (int k = 0; k < K_N; ++k)
      if (kv.second->ev[k].st != S_DISARMED) ++c[kv.second->ev[k].st];
  PyObject* d = PyDict_New();
  for (int s = 1; s < 7; ++s) {
    PyObject* v = PyLong_FromLongLong(c[s]);
    PyDict_SetItemString(d, ST_NAME[s], v);
    Py_DECREF(v);
  }
  return d;
}

PyMethodDef Table_methods[] = {
    {"arm", (PyCFunction)Table_arm, METH_VARARGS, "arm(path, kind)"},
    {"notify", (PyCFunction)Table_notify, METH_VARARGS, "notify(path, evt)"},
    {"ready", (PyCFunction)Table_ready, METH_O, "ready(conn)"},
    {"unready", (PyCFunction)Table_unready, METH_NOARGS, "unready()"},
    {"disconnected", (PyCFunction)Table_disconnected, METH_NOARGS, ""},
    {"resume_lists", (PyCFunction)Table_resume_lists, METH_NOARGS, ""},
    {"resumed", (PyCFunction)Table_resumed, METH_O, "resumed(batch)"},
    {"state", (PyCFunction)Table_state, METH_VARARGS, "state(path, kind)"},
    {"history", (PyCFunction)Table_history, METH_VARARGS, ""},
    {"has", (PyCFunction)Table_contains_path, METH_O, "has(path)"},
    {"counts", (PyCFunction)Table_counts, METH_NOARGS, ""},
    {"close", (PyCFunction)Table_close, METH_NOARGS, "close()"},
    {"_kick", (PyCFunction)Table_kick, METH_NOARGS, ""},
    {"_dc_tick", (PyCFunction)Table_dc_tick, METH_NOARGS, ""},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_zkwatch",
                      "native watch-event engine", -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__zkwatch() {
  ReqType.tp_name = "zkmi._zkwatch.WatchRequest";
  ReqType.tp_basicsize = sizeof(Req);
  ReqType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  ReqType.tp_traverse = (traverseproc)Req_traverse;
  ReqType.tp_clear = (inquiry)Req_clear;
  ReqType.tp_dealloc = (destructor)Req_dealloc;
  ReqType.tp_methods = Req_methods;
  ReqType.tp_getset = Req_getset;
  TableType.tp_name = "zkmi._zkwatch.WatchTable";
  TableType.tp_basicsize = sizeof(Table);
  TableType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  TableType.tp_traverse = (traverseproc)Table_traverse;
  TableType.tp_clear = (inquiry)Table_clear;
  TableType.tp_new = Table_new;
  TableType.tp_init = (initproc)Table_init;
  TableType.tp_dealloc = (destructor)Table_dealloc;
  TableType.tp_methods = Table_methods;
  if (PyType_Ready(&ReqType) < 0 || PyType_Ready(&TableType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&module);
  if (m == nullptr) return nullptr;
  Py_INCREF(&TableType);
  PyModule_AddObject(m, "WatchTable", (PyObject*)&TableType);
  Py_INCREF(&ReqType);
  PyModule_AddObject(m, "WatchRequest", (PyObject*)&ReqType);
  return m;
}
