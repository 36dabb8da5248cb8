// zkmi native event loop — epoll + eventfd + timer heap + TCP transports.
//
// The reference runs every FSM, timer and socket callback on Node's event
// loop (libuv, native code): net.connect (lib/connection-fsm.js:99-103),
// setTimeout / setImmediate / setInterval (lib/connection-fsm.js:201-207,
// lib/zk-session.js:99-108), socket 'data' / 'end' / 'error' / 'close'.
// This is zkmi's equivalent: one loop thread per Loop, all callbacks on it,
// so the Python FSMs above it need no locks.
//
// Python surface (module _zkloop, wrapped by zkmi/runtime/nloop.py):
//   Loop(on_exception)
//     .run()                          blocks; call on the loop thread
//     .stop()                         any thread
//     .call_soon(fn, args)            -> Handle      any thread
//     .call_later(ms, fn, args)       -> Handle      any thread
//     .time_ms()                      monotonic milliseconds
//     .connect(host, port, protocol, on_fail) -> Transport
//     .listen(host, port, factory)    -> Server
//   Handle .cancel() / .clear() / .unref() / .cancelled
//   Transport (asyncio-Protocol-shaped callbacks on `protocol`:
//     connection_made(tr), data_received(bytes), eof_received(),
//     connection_lost(exc|None))
//     .write(b) -> bool, .write_eof(), .can_write_eof(), .abort(), .close(),
//     .cancel(), .is_closing(), .pause_reading(), .resume_reading(),
//     .get_extra_info(name, default=None)
//   Server .port, .close()
//
// Concurrency: the loop thread holds the GIL except inside epoll_wait; every
// other entry point is a Python call and holds the GIL too, so the GIL
// serialises all access to the queues, the timer heap and the fd table.
// Threads other than the loop thread wake it through the eventfd.
// epoll events carry a registration id, not the fd, so an event for an fd
// that was closed (and its number reused) while the loop slept is dropped.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <arpa/inet.h>
#include <linux/futex.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

double mono_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

// Busy-poll window after activity, ms (ZKMI_LOOP_SPIN_US; 0 = always block
// in epoll_wait).  Default 50 us on hosts with >= 16 online CPUs, off on
// smaller ones: on a GPU box it cut the blocking get() RTT 44 -> 37 us, in
// an 8-CPU container the spinning thread competed with the server and the
// caller and made it slower.
double loop_spin_ms() {
  // a function-local static: initialised once, thread-safely (every loop
  // thread calls this)
  static const double v = [] {
    const char* e = getenv("ZKMI_LOOP_SPIN_US");
    const double dflt = sysconf(_SC_NPROCESSORS_ONLN) >= 16 ? 50.0 : 0.0;
    const double x = (e ? atof(e) : dflt) / 1e3;
    return x < 0 ? 0.0 : x;
  }();
  return v;
}

PyObject* os_error(int err) {
  return PyObject_CallFunction(PyExc_OSError, "is", err, strerror(err));
}

// ---------------------------------------------------------------------------
// Handle
// ---------------------------------------------------------------------------

struct Handle {
  PyObject_HEAD
  PyObject* fn;
  PyObject* args;
  double when;
  uint64_t seq;
  bool cancelled;
};

// Handle, Transport and Server are GC types: a timer's callback, or a
// transport's protocol, usually refers back to the object that holds the
// handle or transport (a connection, a session), and a closed client's
// objects must be collectable.  Objects the loop still holds (queued
// handles, registered transports) are kept alive by those references.
int Handle_traverse(Handle* h, visitproc visit, void* arg) {
  Py_VISIT(h->fn);
  Py_VISIT(h->args);
  return 0;
}

int Handle_clear(Handle* h) {
  Py_CLEAR(h->fn);
  Py_CLEAR(h->args);
  return 0;
}

void Handle_dealloc(Handle* h) {
  PyObject_GC_UnTrack(h);
  Handle_clear(h);
  PyObject_GC_Del(h);
}

PyObject* Handle_cancel(Handle* h, PyObject*) {
  if (!h->cancelled) {
    h->cancelled = true;
    Py_CLEAR(h->fn);
    Py_CLEAR(h->args);
  }
  Py_RETURN_NONE;
}

PyObject* Handle_unref(Handle* h, PyObject*) {
  // loop threads are daemons: a pending timer never keeps the process up
  // (Node's timer.unref(), used at lib/connection-fsm.js:204)
  Py_INCREF(h);
  return (PyObject*)h;
}

PyObject* Handle_get_cancelled(Handle* h, void*) {
  return PyBool_FromLong(h->cancelled);
}

PyMethodDef Handle_methods[] = {
    {"cancel", (PyCFunction)Handle_cancel, METH_NOARGS, "cancel"},
    {"clear", (PyCFunction)Handle_cancel, METH_NOARGS, "cancel"},
    {"unref", (PyCFunction)Handle_unref, METH_NOARGS, "no-op, returns self"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Handle_getset[] = {
    {"cancelled", (getter)Handle_get_cancelled, nullptr, nullptr, nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject HandleType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ---------------------------------------------------------------------------
// Loop / Transport / Server
// ---------------------------------------------------------------------------

struct Loop;

enum Kind { K_TRANSPORT = 1, K_SERVER = 2 };

// Common head of the objects registered with epoll.
struct Watched {
  PyObject_HEAD
  int kind;
  int fd;
  uint64_t reg;          // registration id (0 = not registered)
  uint32_t events;       // epoll mask currently registered
  Loop* loop;            // borrowed (the loop outlives its watched objects)
};

// Bulk reply capture (Transport.capture): while on, the read path frames
// the inbound stream itself and copies every frame whose xid is in
// [x0, x0 + n) — length prefix included — into a caller-owned buffer (the
// pinned host buffer a GPU batch decodes from), so those replies never
// become Python objects; every other frame (notifications, pings, ordinary
// requests) still goes to data_received, in order.  `carry` holds a partial
// frame between reads.  Ends when n frames arrived, the buffer is full (the
// rest flows to Python) or a frame length is bad (Python's framer reports
// it); done(status, nbytes, nframes, last_off) is called on the loop.
struct Capture {
  bool on = false;
  int64_t x0 = 0, n = 0, got = 0, max_packet = 0;
  uint8_t* dst = nullptr;
  size_t size = 0, len = 0, last_off = 0;
  std::string carry;
  PyObject* done = nullptr;
};
enum { CAP_DONE = 0, CAP_FULL = 1, CAP_BAD = 2, CAP_CANCEL = 3 };

// Notification sink (Transport.note_sink): while on, the read path frames
// the inbound stream itself and keeps every NOTIFICATION frame (xid -1),
// length prefix included, in `buf` instead of handing it to Python; the
// node-wide watch fan-out (zkmi/parallel/fanout.py) takes them in bulk
// (take_notes) and forwards the raw bytes.  Other frames go on to Python
// whole.  All access holds the GIL (the loop thread calls into Python).
// With `watchers` (the session's dict path -> ZKWatcher) non-empty, an
// event on a watcher()'s path goes on to Python as well (the session's
// watchers must keep firing) and stays in the sink only when its path is
// also in `bulk` (the session's bulk watch set).
struct NoteSink {
  bool on = false;
  int64_t max_packet = 0;
  std::string buf;
  int64_t frames = 0;
  PyObject* watchers = nullptr;
  PyObject* bulk = nullptr;
};

int32_t be32(const char* p);

// Sink a NOTIFICATION frame (body b, fl bytes): keeps it when it belongs to
// the sink; returns true when Python should also get it (see NoteSink).
bool note_take(NoteSink& ns, const char* frame, int32_t fl) {
  bool keep = true, to_py = false;
  if (ns.watchers != nullptr && PyDict_GET_SIZE(ns.watchers) > 0 &&
      fl >= 16 + 12) {
    // body: xid i32, zxid i64, err i32, type i32, state i32, path ustring
    const char* b = frame + 4;
    const int32_t pl = be32(b + 24);
    if (pl >= 0 && 28 + (int64_t)pl <= fl) {
      PyObject* key = PyUnicode_DecodeUTF8(b + 28, pl, "replace");
      if (key == nullptr) {
        PyErr_Clear();
      } else {
        const int w = PyDict_Contains(ns.watchers, key);
        if (w > 0) {
          to_py = true;
          keep = ns.bulk != nullptr && PySet_Contains(ns.bulk, key) > 0;
        }
        PyErr_Clear();
        Py_DECREF(key);
      }
    }
  }
  if (keep) {
    ns.buf.append(frame, 4 + (size_t)fl);
    ++ns.frames;
  }
  return to_py;
}

// Reply router (Transport.route): the completion path of the interactive
// API.  While on, the read path frames the inbound stream itself and, for
// every reply whose xid is an outstanding request in `reqs` (the
// connection's dict xid -> ZKRequest), decodes it with the host codec
// (zk_host_codec.cpp, straight from the receive buffer), removes the xid
// from `reqs` and `xmap` (the xid -> opcode map) and settles the request:
// an OK reply goes to the request's (on_reply, on_error) pair directly
// (ZKRequest.then), anything else to `on_other(req, pkt)`.  Frames it does
// not own (notifications, pings, SET_WATCHES, bulk replies without a
// capture, unknown xids, undecodable bodies) go to Python in stream order.
// Routed replies update `max_zxid` and `last_rx` here; the session reads
// them when it needs them (lastZxidSeen, expiry) instead of per reply.
typedef PyObject* (*DecodeFn)(const uint8_t*, Py_ssize_t, PyObject*);
typedef bool (*EncodeFn)(PyObject*, std::string*, bool);
struct Router {
  bool on = false;
  bool give_back = false;    // turned off mid-dispatch: carry goes to Python
  int64_t max_packet = 0;
  PyObject* reqs = nullptr;
  PyObject* xmap = nullptr;
  PyObject* on_other = nullptr;
  PyObject* on_note = nullptr;   // NOTIFICATION frames, decoded (optional)
  DecodeFn decode = nullptr;
  EncodeFn encode = nullptr;     // Transport.request (optional)
  int64_t max_zxid = 0;
  double last_rx = 0;
  int64_t routed = 0;
};

// One unit of an inbound read, in stream order: bytes for Python, or a
// routed (request, reply) pair.
struct RxItem {
  PyObject* req;             // nullptr: `bytes` holds frames for Python,
                             // or (with pkt) a decoded notification
  PyObject* pkt;
  int32_t err;
  std::string bytes;
};

struct Transport {
  Watched w;
  PyObject* protocol;
  PyObject* on_fail;
  std::string* wbuf;     // pending output
  size_t woff;
  bool connecting, connected, paused, rd_eof, eof_pending, wr_shut;
  bool closing, closed;
  PyObject* peer;        // (host, port) tuple
  Capture* cap;
  NoteSink* ns;
  Router* rt;
  int dispatching;       // >0 while deliver() hands a read's items out
  bool queued;           // on the loop's dirty list (a coalesced write)
};

struct Server {
  Watched w;
  PyObject* factory;
  int port;
};

struct TimerCmp {
  bool operator()(const Handle* a, const Handle* b) const {
    return a->when != b->when ? a->when > b->when : a->seq > b->seq;
  }
};

struct Loop {
  PyObject_HEAD
  int epfd;
  int evfd;
  bool running;
  bool stopping;
  pthread_t thread;
  uint64_t seq;
  uint64_t next_reg;
  PyObject* on_exception;
  std::deque<Handle*>* ready;
  std::vector<Handle*>* timers;                  // min-heap by (when, seq)
  std::unordered_map<uint64_t, Watched*>* regs;  // strong refs
  double last_active;                            // mono_ms of the last event
  std::vector<Transport*>* dirty;                // writes to flush this turn
  std::vector<PyObject*>* wakes;                 // Waiters set this turn
};

bool on_loop_thread(Loop* L) {
  return L->running && pthread_equal(L->thread, pthread_self());
}

void wake(Loop* L) {
  if (on_loop_thread(L)) return;
  uint64_t one = 1;
  ssize_t r = write(L->evfd, &one, sizeof one);
  (void)r;
}

// ---------------------------------------------------------------------------
// Waiter: a blocking caller's completion flag (Client.call_sync).  The
// caller waits in C with the GIL released: it spins on the flag for a short
// window, then sleeps on it (futex).  Set on the loop thread (the reply's
// callback runs there), the flag flips only once the loop has let go of the
// GIL for its next wait, so the woken caller takes a free GIL: no thread of
// the pair sleeps on the GIL handing the reply over (the bare-lock wake-up
// cost two such sleeps: 11.5 us blocking p50 against 7.0 us for a get()
// chained on the loop, profiles/r5_bench_1gpu_driver_config.log).
// ---------------------------------------------------------------------------

extern PyTypeObject LoopType;

struct Waiter {
  PyObject_HEAD
  Loop* loop;                         // strong ref, may be null
  std::atomic<int> state;             // 0 pending, 1 set
  std::atomic<int> sleeping;          // the caller sleeps on `state`
};

PyTypeObject WaiterType = {PyVarObject_HEAD_INIT(nullptr, 0)};

void waiter_flip(Waiter* w) {
  w->state.store(1, std::memory_order_seq_cst);
  if (w->sleeping.load(std::memory_order_seq_cst))
    syscall(SYS_futex, (int*)&w->state, FUTEX_WAKE_PRIVATE, 1, nullptr,
            nullptr, 0);
}

// The loop's part: after releasing the GIL for its wait, flip every Waiter
// set this turn (no Python); after taking the GIL back, drop their refs.
void flip_wakes(Loop* L) {
  for (PyObject* o : *L->wakes) waiter_flip((Waiter*)o);
}
void drop_wakes(Loop* L) {
  if (L->wakes->empty()) return;
  std::vector<PyObject*> ws;
  ws.swap(*L->wakes);
  for (PyObject* o : ws) Py_DECREF(o);
}

PyObject* Waiter_new(PyTypeObject* type, PyObject* args, PyObject*) {
  PyObject* lp = nullptr;
  if (!PyArg_ParseTuple(args, "|O", &lp)) return nullptr;
  if (lp == Py_None) lp = nullptr;
  if (lp != nullptr && !PyObject_TypeCheck(lp, &LoopType)) {
    PyErr_SetString(PyExc_TypeError, "Waiter(loop): a _zkloop.Loop");
    return nullptr;
  }
  Waiter* w = (Waiter*)type->tp_alloc(type, 0);
  if (w == nullptr) return nullptr;
  w->loop = (Loop*)lp;
  Py_XINCREF(lp);
  new (&w->state) std::atomic<int>(0);
  new (&w->sleeping) std::atomic<int>(0);
  return (PyObject*)w;
}

void Waiter_dealloc(Waiter* w) {
  Py_XDECREF((PyObject*)w->loop);
  Py_TYPE(w)->tp_free((PyObject*)w);
}

// set(): on the loop thread deferred to the loop's next wait; elsewhere now.
PyObject* Waiter_set(Waiter* w, PyObject*) {
  if (w->state.load() != 0) Py_RETURN_NONE;
  Loop* L = w->loop;
  if (L != nullptr && on_loop_thread(L)) {
    Py_INCREF(w);
    L->wakes->push_back((PyObject*)w);
  } else {
    waiter_flip(w);
  }
  Py_RETURN_NONE;
}

// wait(spin_s, timeout_s) -> bool: spin up to spin_s, then sleep until set
// or timeout; the GIL is released throughout.
PyObject* Waiter_wait(Waiter* w, PyObject* args) {
  double spin = 0, timeout = -1;
  if (!PyArg_ParseTuple(args, "|dd", &spin, &timeout)) return nullptr;
  bool ok;
  Py_BEGIN_ALLOW_THREADS
  const double t0 = mono_ms();
  const double spin_end = t0 + spin * 1e3;
  const double end = timeout < 0 ? -1 : t0 + timeout * 1e3;
  while (w->state.load(std::memory_order_acquire) == 0 &&
         mono_ms() < spin_end)
    __builtin_ia32_pause();
  ok = w->state.load(std::memory_order_acquire) != 0;
  if (!ok) {
    w->sleeping.store(1, std::memory_order_seq_cst);
    for (;;) {
      if (w->state.load(std::memory_order_seq_cst) != 0) { ok = true; break; }
      timespec ts, *tp = nullptr;
      if (end >= 0) {
        const double left = end - mono_ms();
        if (left <= 0) break;
        ts.tv_sec = (time_t)(left / 1e3);
        ts.tv_nsec = (long)((left - ts.tv_sec * 1e3) * 1e6);
        tp = &ts;
      }
      syscall(SYS_futex, (int*)&w->state, FUTEX_WAIT_PRIVATE, 0, tp, nullptr,
              0);
    }
  }
  Py_END_ALLOW_THREADS
  return PyBool_FromLong(ok);
}

PyObject* Waiter_is_set(Waiter* w, void*) {
  return PyBool_FromLong(w->state.load() != 0);
}

PyMethodDef Waiter_methods[] = {
    {"set", (PyCFunction)Waiter_set, METH_NOARGS,
     "mark done (from the loop thread: at the loop's next wait)"},
    {"wait", (PyCFunction)Waiter_wait, METH_VARARGS,
     "wait(spin_s=0, timeout_s=-1) -> bool, GIL released"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Waiter_getset[] = {
    {"is_set", (getter)Waiter_is_set, nullptr, nullptr, nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

void report_exception(Loop* L) {
  PyObject *t, *v, *tb;
  PyErr_Fetch(&t, &v, &tb);
  PyErr_NormalizeException(&t, &v, &tb);
  if (tb != nullptr && v != nullptr) PyException_SetTraceback(v, tb);
  if (L->on_exception != nullptr && v != nullptr) {
    PyObject* r = PyObject_CallOneArg(L->on_exception, v);
    if (r == nullptr) PyErr_Print();
    Py_XDECREF(r);
  }
  Py_XDECREF(t);
  Py_XDECREF(v);
  Py_XDECREF(tb);
}

// Call obj.name(*args) on the loop thread; failures go to on_exception.
void invoke(Loop* L, PyObject* obj, const char* name, PyObject* arg) {
  if (obj == nullptr) return;
  PyObject* m = PyObject_GetAttrString(obj, name);
  if (m == nullptr) { report_exception(L); return; }
  PyObject* r = arg ? PyObject_CallOneArg(m, arg) : PyObject_CallNoArgs(m);
  Py_DECREF(m);
  if (r == nullptr) report_exception(L);
  Py_XDECREF(r);
}

Handle* new_handle(PyObject* fn, PyObject* args) {
  Handle* h = PyObject_GC_New(Handle, &HandleType);
  if (h == nullptr) return nullptr;
  Py_INCREF(fn);
  h->fn = fn;
  if (args == nullptr) args = PyTuple_New(0);
  else Py_INCREF(args);
  h->args = args;
  h->when = 0;
  h->seq = 0;
  h->cancelled = false;
  PyObject_GC_Track((PyObject*)h);
  return h;
}

// queue h (a new reference is taken)
void push_ready(Loop* L, Handle* h) {
  Py_INCREF(h);
  L->ready->push_back(h);
  wake(L);
}

void push_timer(Loop* L, Handle* h) {
  Py_INCREF(h);
  h->seq = ++L->seq;
  L->timers->push_back(h);
  std::push_heap(L->timers->begin(), L->timers->end(), TimerCmp());
  wake(L);
}

// Defer fn(*args) to the loop's ready queue (used for callbacks that must
// not run inside the caller's stack, as asyncio defers them).
void defer(Loop* L, PyObject* fn, PyObject* args) {
  Handle* h = new_handle(fn, args);
  if (h == nullptr) { report_exception(L); return; }
  push_ready(L, h);
  Py_DECREF(h);
}

void defer_method(Loop* L, PyObject* obj, const char* name, PyObject* arg) {
  PyObject* m = PyObject_GetAttrString(obj, name);
  if (m == nullptr) { report_exception(L); return; }
  PyObject* args = arg ? PyTuple_Pack(1, arg) : PyTuple_New(0);
  defer(L, m, args);
  Py_DECREF(m);
  Py_XDECREF(args);
}

int set_events(Watched* w, uint32_t ev) {
  if (w->reg == 0 || w->events == ev) return 0;
  epoll_event e;
  e.events = ev;
  e.data.u64 = w->reg;
  if (epoll_ctl(w->loop->epfd, EPOLL_CTL_MOD, w->fd, &e) != 0) return -1;
  w->events = ev;
  return 0;
}

int add_watch(Loop* L, Watched* w, uint32_t ev) {
  w->reg = ++L->next_reg;
  epoll_event e;
  e.events = ev;
  e.data.u64 = w->reg;
  if (epoll_ctl(L->epfd, EPOLL_CTL_ADD, w->fd, &e) != 0) {
    w->reg = 0;
    return -1;
  }
  w->events = ev;
  Py_INCREF(w);
  (*L->regs)[w->reg] = w;
  return 0;
}

// Unregister and close the fd.  Drops the table's reference (the caller
// must hold its own if it still uses w).
void drop_watch(Watched* w) {
  Loop* L = w->loop;
  if (w->fd >= 0) {
    if (w->reg != 0) epoll_ctl(L->epfd, EPOLL_CTL_DEL, w->fd, nullptr);
    close(w->fd);
    w->fd = -1;
  }
  if (w->reg != 0) {
    L->regs->erase(w->reg);
    w->reg = 0;
    Py_DECREF(w);
  }
}

// ---------------------------------------------------------------------------
// Transport
// ---------------------------------------------------------------------------

PyTypeObject TransportType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject ServerType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject LoopType = {PyVarObject_HEAD_INIT(nullptr, 0)};

Transport* new_transport(Loop* L, int fd) {
  Transport* t = PyObject_GC_New(Transport, &TransportType);
  if (t == nullptr) return nullptr;
  t->w.kind = K_TRANSPORT;
  t->w.fd = fd;
  t->w.reg = 0;
  t->w.events = 0;
  t->w.loop = L;
  t->protocol = nullptr;
  t->on_fail = nullptr;
  t->wbuf = new std::string();
  t->woff = 0;
  t->connecting = t->connected = t->paused = t->rd_eof = false;
  t->eof_pending = t->wr_shut = t->closing = t->closed = false;
  t->peer = nullptr;
  t->cap = new Capture();
  t->ns = new NoteSink();
  t->rt = new Router();
  t->dispatching = 0;
  t->queued = false;
  PyObject_GC_Track((PyObject*)t);
  return t;
}

int Transport_traverse(Transport* t, visitproc visit, void* arg) {
  Py_VISIT(t->protocol);
  Py_VISIT(t->on_fail);
  Py_VISIT(t->peer);
  Py_VISIT(t->cap->done);
  Py_VISIT(t->ns->watchers);
  Py_VISIT(t->ns->bulk);
  Py_VISIT(t->rt->reqs);
  Py_VISIT(t->rt->xmap);
  Py_VISIT(t->rt->on_other);
  Py_VISIT(t->rt->on_note);
  return 0;
}

int Transport_clear(Transport* t) {
  Py_CLEAR(t->protocol);
  Py_CLEAR(t->on_fail);
  Py_CLEAR(t->peer);
  Py_CLEAR(t->cap->done);
  Py_CLEAR(t->ns->watchers);
  Py_CLEAR(t->ns->bulk);
  Py_CLEAR(t->rt->reqs);
  Py_CLEAR(t->rt->xmap);
  Py_CLEAR(t->rt->on_other);
  Py_CLEAR(t->rt->on_note);
  return 0;
}

void Transport_dealloc(Transport* t) {
  PyObject_GC_UnTrack(t);
  if (t->w.fd >= 0) close(t->w.fd);
  Transport_clear(t);
  delete t->wbuf;
  delete t->cap;
  delete t->ns;
  delete t->rt;
  PyObject_GC_Del(t);
}

uint32_t wanted(Transport* t) {
  uint32_t ev = 0;
  if (t->connecting) return EPOLLOUT;
  if (!t->paused && !t->rd_eof) ev |= EPOLLIN | EPOLLRDHUP;
  if (t->woff < t->wbuf->size()) ev |= EPOLLOUT;
  return ev;
}

void refresh(Transport* t) {
  if (t->closed) return;
  set_events(&t->w, wanted(t));
}

// Terminal: close the socket and tell the protocol (exc may be nullptr for a
// clean close).  Runs connection_lost now (we are on the loop thread).
void finish(Transport* t, PyObject* exc) {
  if (t->closed) return;
  t->closed = true;
  // a capture dies with the connection (its batch fails with the requests)
  t->cap->on = false;
  t->cap->dst = nullptr;
  t->cap->carry.clear();
  Py_CLEAR(t->cap->done);
  t->rt->on = false;
  Py_INCREF(t);
  drop_watch(&t->w);
  if (t->connected && t->protocol != nullptr)
    invoke(t->w.loop, t->protocol, "connection_lost", exc ? exc : Py_None);
  Py_DECREF(t);
}

void fatal(Transport* t, int err) {
  PyObject* exc = os_error(err);
  if (exc == nullptr) { report_exception(t->w.loop); return; }
  finish(t, exc);
  Py_DECREF(exc);
}

void shut_wr(Transport* t) {
  if (!t->wr_shut && t->w.fd >= 0) {
    shutdown(t->w.fd, SHUT_WR);
    t->wr_shut = true;
  }
}

// Write as much of the buffer as the socket takes; returns errno or 0.
int flush(Transport* t) {
  std::string& b = *t->wbuf;
  while (t->woff < b.size()) {
    ssize_t n = send(t->w.fd, b.data() + t->woff, b.size() - t->woff,
                     MSG_NOSIGNAL | MSG_DONTWAIT);
    if (n > 0) { t->woff += (size_t)n; continue; }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    return n < 0 ? errno : EPIPE;
  }
  if (t->woff == b.size()) {
    b.clear();
    t->woff = 0;
    if (t->eof_pending) shut_wr(t);
  } else if (t->woff > (1u << 20) && t->woff * 2 > b.size()) {
    b.erase(0, t->woff);
    t->woff = 0;
  }
  return 0;
}

void on_connected(Transport* t) {
  t->connecting = false;
  t->connected = true;
  int one = 1;
  setsockopt(t->w.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  Py_CLEAR(t->on_fail);
  Py_INCREF(t);
  invoke(t->w.loop, t->protocol, "connection_made", (PyObject*)t);
  if (!t->closed) {
    int err = t->woff < t->wbuf->size() ? flush(t) : 0;
    if (err) fatal(t, err);
    else refresh(t);
  }
  Py_DECREF(t);
}

void connect_failed(Transport* t, int err) {
  Loop* L = t->w.loop;
  PyObject* cb = t->on_fail;
  t->on_fail = nullptr;
  t->closed = true;
  Py_INCREF(t);
  drop_watch(&t->w);
  if (cb != nullptr) {
    PyObject* exc = os_error(err);
    if (exc != nullptr) {
      PyObject* r = PyObject_CallOneArg(cb, exc);
      if (r == nullptr) report_exception(L);
      Py_XDECREF(r);
      Py_DECREF(exc);
    } else {
      report_exception(L);
    }
    Py_DECREF(cb);
  }
  Py_DECREF(t);
}

void deliver_raw(Transport* t, const char* p, size_t n) {
  if (n == 0 || t->closed) return;
  PyObject* b = PyBytes_FromStringAndSize(p, (Py_ssize_t)n);
  if (b == nullptr) { report_exception(t->w.loop); return; }
  invoke(t->w.loop, t->protocol, "data_received", b);
  Py_DECREF(b);
}

int32_t be32(const char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return (int32_t)ntohl(v);
}

uint64_t be64(const char* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

void deliver(Transport* t, const char* p, size_t n);

// End the capture: done(status, nbytes, nframes, last_off), then the bytes
// after the last parsed frame go on (to a capture done() started, or to
// Python).
void capture_end(Transport* t, int status) {
  Capture& c = *t->cap;
  c.on = false;
  c.dst = nullptr;
  std::string rest;
  rest.swap(c.carry);
  PyObject* cb = c.done;
  c.done = nullptr;
  if (cb != nullptr) {
    PyObject* r = PyObject_CallFunction(cb, "inLn", status, (Py_ssize_t)c.len,
                                        (long long)c.got,
                                        (Py_ssize_t)c.last_off);
    if (r == nullptr) report_exception(t->w.loop);
    Py_XDECREF(r);
    Py_DECREF(cb);
  }
  // The done callback may have started the next capture (a bulk callback
  // chaining the next batch): the leftover bytes then belong to it, so
  // they go through deliver(), which frames them into a capture that is on
  // and passes them to Python raw otherwise.
  if (!t->closed && !rest.empty()) deliver(t, rest.data(), rest.size());
}

// The router's part of a frame (see Router): decode and unlink a reply
// whose xid is outstanding; false leaves the frame to Python.  Calls no
// Python code (dict lookups on int keys, the C decoder).
bool route_frame(Router& rt, const char* f, int32_t fl, int64_t xid,
                 RxItem& it) {
  PyObject* k = PyLong_FromLongLong(xid);
  if (k == nullptr) { PyErr_Clear(); return false; }
  PyObject* req = PyDict_GetItemWithError(rt.reqs, k);     // borrowed
  if (req == nullptr) {
    PyErr_Clear();
    Py_DECREF(k);
    return false;
  }
  PyObject* pkt = rt.decode((const uint8_t*)f + 4, fl, rt.xmap);
  if (pkt == nullptr) {
    // Python's path raises the same decode error on the same bytes
    PyErr_Clear();
    Py_DECREF(k);
    return false;
  }
  Py_INCREF(req);
  if (PyDict_DelItem(rt.reqs, k) != 0) PyErr_Clear();
  if (PyDict_DelItem(rt.xmap, k) != 0) PyErr_Clear();
  Py_DECREF(k);
  const int64_t zxid = (int64_t)be64(f + 8);
  if (zxid > rt.max_zxid) rt.max_zxid = zxid;
  ++rt.routed;
  it.req = req;
  it.pkt = pkt;
  it.err = be32(f + 16);
  return true;
}

// Settle one routed request: (on_reply, on_error) = req.fast, called
// directly for an OK reply when nothing else listens on the request;
// otherwise on_other(req, pkt) (error replies, listener-style requests).
void settle_routed(Transport* t, RxItem& it) {
  Loop* L = t->w.loop;
  PyObject* r = nullptr;
  bool direct = false;
  if (it.err == 0) {
    PyObject* fast = PyObject_GetAttrString(it.req, "fast");
    PyObject* lst = fast ? PyObject_GetAttrString(it.req, "_listeners")
                         : nullptr;
    if (fast && lst && PyTuple_Check(fast) && PyTuple_GET_SIZE(fast) == 2 &&
        PyDict_Check(lst) && PyDict_GET_SIZE(lst) == 0) {
      direct = true;
      r = PyObject_CallOneArg(PyTuple_GET_ITEM(fast, 0), it.pkt);
    }
    if (!fast || !lst) PyErr_Clear();
    Py_XDECREF(fast);
    Py_XDECREF(lst);
  }
  if (!direct) {
    PyObject* cb = t->rt->on_other;
    if (cb != nullptr) r = PyObject_CallFunctionObjArgs(cb, it.req, it.pkt,
                                                       nullptr);
    else r = Py_NewRef(Py_None);
  }
  if (r == nullptr) report_exception(L);
  Py_XDECREF(r);
}

void deliver(Transport* t, const char* p, size_t n) {
  Capture& c = *t->cap;
  NoteSink& ns = *t->ns;
  Router& rt = *t->rt;
  if (!c.on && !ns.on && !rt.on) { deliver_raw(t, p, n); return; }
  std::string buf;
  const char* s = p;
  size_t len = n;
  if (!c.carry.empty()) {
    buf.swap(c.carry);
    buf.append(p, n);
    s = buf.data();
    len = buf.size();
  }
  std::vector<RxItem> items;      // in stream order
  std::string pass;               // frames for Python since the last item
  size_t i = 0;
  int status = -1;
  const int64_t maxp = c.on ? c.max_packet
                            : ns.on ? ns.max_packet : rt.max_packet;
  while (len - i >= 4) {
    if (c.on && c.got >= c.n) break;      // (capture_end re-delivers the rest)
    const int32_t fl = be32(s + i);
    if (fl < 0 || fl > maxp) {
      if (c.on) {
        status = CAP_BAD;
      } else {
        // no capture: Python's framer sees the bad length and reports it
        pass.append(s + i, len - i);
        i = len;
      }
      break;
    }
    if (len - i < 4 + (size_t)fl) break;
    const int64_t xid = fl >= 4 ? be32(s + i + 4) : -2;
    if (c.on && fl >= 16 && xid >= c.x0 && xid < c.x0 + c.n) {
      if (c.len + 4 + (size_t)fl > c.size) { status = CAP_FULL; break; }
      memcpy(c.dst + c.len, s + i, 4 + (size_t)fl);
      c.last_off = c.len;
      c.len += 4 + (size_t)fl;
      ++c.got;
    } else if (ns.on && fl >= 16 && xid == -1 && !note_take(ns, s + i, fl)) {
      // kept by the sink only
    } else if (rt.on && rt.on_note != nullptr && fl >= 16 && xid == -1) {
      // a watch event: decoded here, handed to on_note in stream order
      PyObject* pkt = rt.decode((const uint8_t*)s + i + 4, fl, rt.xmap);
      if (pkt == nullptr) {
        PyErr_Clear();                 // Python's path reports it
        pass.append(s + i, 4 + (size_t)fl);
      } else {
        if (!pass.empty()) {
          RxItem b;
          b.req = b.pkt = nullptr;
          b.err = 0;
          b.bytes.swap(pass);
          items.push_back(std::move(b));
        }
        RxItem nt;
        nt.req = nullptr;
        nt.pkt = pkt;
        nt.err = 0;
        items.push_back(std::move(nt));
      }
    } else if (rt.on && fl >= 16 && xid >= 0) {
      RxItem one;
      one.req = one.pkt = nullptr;
      if (route_frame(rt, s + i, fl, xid, one)) {
        if (!pass.empty()) {
          RxItem b;
          b.req = b.pkt = nullptr;
          b.err = 0;
          b.bytes.swap(pass);
          items.push_back(std::move(b));
        }
        items.push_back(std::move(one));
      } else {
        pass.append(s + i, 4 + (size_t)fl);
      }
    } else {
      pass.append(s + i, 4 + (size_t)fl);
    }
    i += 4 + (size_t)fl;
  }
  if (rt.on && i > 0) rt.last_rx = mono_ms();
  if (status < 0 && c.on && c.got >= c.n) status = CAP_DONE;
  c.carry.assign(s + i, len - i);
  // Hand the read out in order.  Callbacks may close the transport, turn
  // the router off or start a capture: routed replies are settled anyway
  // (they arrived and were unlinked), bytes go to Python while it is open.
  ++t->dispatching;
  for (size_t j = 0; j < items.size(); ++j) {
    RxItem& it = items[j];
    if (it.req == nullptr && it.pkt != nullptr) {
      PyObject* cb = rt.on_note;
      if (cb != nullptr && !t->closed) {
        Py_INCREF(cb);
        PyObject* r = PyObject_CallOneArg(cb, it.pkt);
        if (r == nullptr) report_exception(t->w.loop);
        Py_XDECREF(r);
        Py_DECREF(cb);
      }
      Py_CLEAR(it.pkt);
    } else if (it.req == nullptr) {
      deliver_raw(t, it.bytes.data(), it.bytes.size());
    } else {
      settle_routed(t, it);
      Py_CLEAR(it.req);
      Py_CLEAR(it.pkt);
    }
  }
  deliver_raw(t, pass.data(), pass.size());
  --t->dispatching;
  if (t->dispatching == 0 && rt.give_back) {
    rt.give_back = false;
    if (!c.on && !ns.on && !rt.on && !c.carry.empty() && !t->closed) {
      std::string rest;
      rest.swap(c.carry);
      deliver_raw(t, rest.data(), rest.size());
    }
  }
  if (status >= 0 && c.on && !t->closed) capture_end(t, status);
}

void transport_event(Transport* t, uint32_t ev) {
  Py_INCREF(t);
  if (t->connecting) {
    int err = 0;
    socklen_t len = sizeof err;
    getsockopt(t->w.fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err != 0) connect_failed(t, err);
    else if (ev & (EPOLLOUT | EPOLLERR | EPOLLHUP)) on_connected(t);
    Py_DECREF(t);
    return;
  }
  if ((ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) && !t->paused &&
      !t->rd_eof) {
    char buf[1 << 16];
    for (int rounds = 0; rounds < 64 && !t->closed && !t->paused; ++rounds) {
      ssize_t n = recv(t->w.fd, buf, sizeof buf, MSG_DONTWAIT);
      if (n > 0) {
        deliver(t, buf, (size_t)n);
        if ((size_t)n < sizeof buf) break;
        continue;
      }
      if (n == 0) {
        t->rd_eof = true;
        invoke(t->w.loop, t->protocol, "eof_received", nullptr);
        break;
      }
      if (errno == EINTR) continue;
      if (errno != EAGAIN && errno != EWOULDBLOCK) fatal(t, errno);
      break;
    }
  }
  if (!t->closed && (ev & EPOLLOUT)) {
    int err = flush(t);
    if (err) fatal(t, err);
  }
  if (!t->closed && (ev & EPOLLERR)) {
    int err = 0;
    socklen_t len = sizeof err;
    getsockopt(t->w.fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err) fatal(t, err);
  }
  if (!t->closed && (ev & EPOLLHUP) && t->rd_eof) {
    // both directions are down: nothing more can arrive or leave
    int err = 0;
    socklen_t len = sizeof err;
    getsockopt(t->w.fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err) fatal(t, err);
    else finish(t, nullptr);
  }
  if (!t->closed && t->closing && t->woff == t->wbuf->size())
    finish(t, nullptr);
  refresh(t);
  Py_DECREF(t);
}

// Writes made on the loop thread are coalesced: the bytes wait in wbuf and
// the transport goes on the loop's dirty list, flushed once at the end of
// the loop turn (flush_dirty), so a burst of pipelined requests issued from
// one batch of reply callbacks leaves in one send() instead of one per
// request.  A write from another thread, or one that leaves more than
// kCorkMax unsent, is sent at once.
constexpr size_t kCorkMax = 256 * 1024;

PyObject* queue_write(Transport* t) {
  if (!t->connected) Py_RETURN_TRUE;
  Loop* L = t->w.loop;
  if (on_loop_thread(L) &&
      t->wbuf->size() - t->woff < kCorkMax) {
    if (!t->queued) {
      t->queued = true;
      Py_INCREF(t);
      L->dirty->push_back(t);
    }
    Py_RETURN_TRUE;
  }
  int err = flush(t);
  if (err) {
    // report from the loop, never from inside the caller's stack
    PyObject* e = PyLong_FromLong(err);
    defer_method(L, (PyObject*)t, "_fatal", e);
    Py_XDECREF(e);
    t->closing = true;
    Py_RETURN_FALSE;
  }
  refresh(t);
  Py_RETURN_TRUE;
}

// Send what the loop turn's writes queued (see queue_write).
void flush_dirty(Loop* L) {
  if (L->dirty->empty()) return;
  std::vector<Transport*> ts;
  ts.swap(*L->dirty);
  for (Transport* t : ts) {
    t->queued = false;
    if (!t->closed && t->connected) {
      int err = flush(t);
      if (err) fatal(t, err);
      else if (!t->closed && t->closing && t->woff == t->wbuf->size())
        finish(t, nullptr);
      else refresh(t);
    }
    Py_DECREF(t);
  }
}

PyObject* Transport_write(Transport* t, PyObject* arg) {
  Py_buffer v;
  if (PyObject_GetBuffer(arg, &v, PyBUF_SIMPLE) != 0) return nullptr;
  if (t->closed || t->closing || t->wr_shut || t->eof_pending) {
    PyBuffer_Release(&v);
    Py_RETURN_FALSE;
  }
  t->wbuf->append((const char*)v.buf, (size_t)v.len);
  PyBuffer_Release(&v);
  return queue_write(t);
}

// write_from(addr, n): queue n bytes read from raw memory (a pinned host
// buffer the GPU encoder filled) without a Python bytes object.
PyObject* Transport_write_from(Transport* t, PyObject* args) {
  unsigned long long addr;
  Py_ssize_t n;
  if (!PyArg_ParseTuple(args, "Kn", &addr, &n)) return nullptr;
  if (n < 0 || (addr == 0 && n > 0)) {
    PyErr_SetString(PyExc_ValueError, "write_from: bad buffer");
    return nullptr;
  }
  if (t->closed || t->closing || t->wr_shut || t->eof_pending)
    Py_RETURN_FALSE;
  t->wbuf->append((const char*)(uintptr_t)addr, (size_t)n);
  return queue_write(t);
}

// capture(x0, n, addr, size, max_packet, done, prefix): see Capture.  The
// buffer must stay valid until done() runs or the transport closes.
// `prefix` = bytes the caller's framer already holds (a partial frame),
// parsed first.
PyObject* Transport_capture(Transport* t, PyObject* args) {
  long long x0, n, maxp;
  unsigned long long addr;
  Py_ssize_t size;
  PyObject* done;
  Py_buffer pre;
  if (!PyArg_ParseTuple(args, "LLKnLOy*", &x0, &n, &addr, &size, &maxp, &done,
                        &pre))
    return nullptr;
  Capture& c = *t->cap;
  if (c.on || t->closed || n <= 0 || addr == 0 || size <= 0 ||
      !PyCallable_Check(done)) {
    PyBuffer_Release(&pre);
    PyErr_SetString(PyExc_ValueError, "capture: busy, closed or bad args");
    return nullptr;
  }
  c.on = true;
  c.x0 = x0;
  c.n = n;
  c.got = 0;
  c.max_packet = maxp;
  c.dst = (uint8_t*)(uintptr_t)addr;
  c.size = (size_t)size;
  c.len = c.last_off = 0;
  // with the sink on the native framer already holds the partial frame
  // (Python's holds none); else the caller's framer hands it over below
  if (!t->ns->on && !t->rt->on) c.carry.clear();
  Py_INCREF(done);
  c.done = done;
  std::string head((const char*)pre.buf, (size_t)pre.len);
  PyBuffer_Release(&pre);
  if (!head.empty()) deliver(t, head.data(), head.size());
  Py_RETURN_NONE;
}

// note_sink(on, max_packet, prefix): route NOTIFICATION frames into the
// sink (see NoteSink).  `prefix` = a partial frame the caller's framer
// holds, parsed first.  Turning it off hands a partial frame the native
// framer holds back to Python.
PyObject* Transport_note_sink(Transport* t, PyObject* args) {
  int on;
  long long maxp;
  Py_buffer pre;
  PyObject *watchers = Py_None, *bulk = Py_None;
  if (!PyArg_ParseTuple(args, "pLy*|OO", &on, &maxp, &pre, &watchers, &bulk))
    return nullptr;
  NoteSink& ns = *t->ns;
  if (watchers != Py_None && !PyDict_Check(watchers)) {
    PyBuffer_Release(&pre);
    PyErr_SetString(PyExc_TypeError, "note_sink: watchers must be a dict");
    return nullptr;
  }
  if (bulk != Py_None && !PyAnySet_Check(bulk)) {
    PyBuffer_Release(&pre);
    PyErr_SetString(PyExc_TypeError, "note_sink: bulk must be a set");
    return nullptr;
  }
  Py_XSETREF(ns.watchers, watchers == Py_None ? nullptr : Py_NewRef(watchers));
  Py_XSETREF(ns.bulk, bulk == Py_None ? nullptr : Py_NewRef(bulk));
  std::string head((const char*)pre.buf, (size_t)pre.len);
  PyBuffer_Release(&pre);
  if (on) {
    const bool was = ns.on;
    ns.on = true;
    ns.max_packet = maxp;
    if (!was && !t->cap->on && !t->rt->on) t->cap->carry.clear();
    if (!head.empty() && !t->closed) deliver(t, head.data(), head.size());
  } else if (ns.on) {
    ns.on = false;
    if (t->dispatching > 0) {
      t->rt->give_back = true;
    } else if (!t->cap->on && !t->rt->on && !t->cap->carry.empty()) {
      std::string rest;
      rest.swap(t->cap->carry);
      deliver_raw(t, rest.data(), rest.size());
    }
  }
  Py_RETURN_NONE;
}

// route(on, reqs, xid_map, on_other, decoder, max_packet, prefix
//       [, encoder, on_note]): see Router; on_note(pkt) takes the decoded
// NOTIFICATION frames (without it they go to Python as bytes).  `decoder`
// is the host codec's `_C_decode_reply` capsule (`encoder`: its
// `_C_encode_request`, for Transport.request); `prefix` = a partial frame
// the caller's framer holds, parsed first.
// Turning it off hands a partial frame the native framer holds back to
// Python (after the read being dispatched, when called from a callback).
PyObject* Transport_route(Transport* t, PyObject* args) {
  int on;
  PyObject *reqs, *xmap, *other, *cap;
  PyObject* ecap = Py_None;
  PyObject* note = Py_None;
  long long maxp;
  Py_buffer pre;
  if (!PyArg_ParseTuple(args, "pOOOOLy*|OO", &on, &reqs, &xmap, &other, &cap,
                        &maxp, &pre, &ecap, &note))
    return nullptr;
  std::string head((const char*)pre.buf, (size_t)pre.len);
  PyBuffer_Release(&pre);
  Router& rt = *t->rt;
  if (!on) {
    if (!rt.on) Py_RETURN_NONE;
    rt.on = false;
    if (t->dispatching > 0) {
      rt.give_back = true;
    } else if (!t->cap->on && !t->ns->on && !t->cap->carry.empty()) {
      std::string rest;
      rest.swap(t->cap->carry);
      deliver_raw(t, rest.data(), rest.size());
    }
    Py_RETURN_NONE;
  }
  if (!PyDict_Check(reqs) || !PyDict_Check(xmap) || !PyCallable_Check(other)) {
    PyErr_SetString(PyExc_TypeError, "route: reqs/xid_map dicts, callable");
    return nullptr;
  }
  void* fn = PyCapsule_GetPointer(cap, "zkmi._zkhost.decode_reply_raw");
  if (fn == nullptr) return nullptr;
  void* efn = nullptr;
  if (ecap != Py_None) {
    efn = PyCapsule_GetPointer(ecap, "zkmi._zkhost.encode_request_into");
    if (efn == nullptr) return nullptr;
  }
  if (t->closed) Py_RETURN_NONE;
  const bool was = rt.on;
  Py_INCREF(reqs);
  Py_XSETREF(rt.reqs, reqs);
  Py_INCREF(xmap);
  Py_XSETREF(rt.xmap, xmap);
  Py_INCREF(other);
  Py_XSETREF(rt.on_other, other);
  if (note != Py_None && PyCallable_Check(note)) {
    Py_INCREF(note);
    Py_XSETREF(rt.on_note, note);
  } else {
    Py_CLEAR(rt.on_note);
  }
  rt.decode = (DecodeFn)fn;
  rt.encode = (EncodeFn)efn;
  rt.max_packet = maxp;
  rt.on = true;
  rt.give_back = false;
  if (!was && !t->cap->on && !t->ns->on) t->cap->carry.clear();
  if (!head.empty()) deliver(t, head.data(), head.size());
  Py_RETURN_NONE;
}

// request(pkt, req): the send half of the completion path.  pkt is a
// request dict with its xid set; it is encoded by the host codec straight
// into the write buffer, and req (the ZKRequest its reply settles) and its
// opcode are entered in the router's reqs / xid_map under that xid.  True
// when queued; None when the router is off (or has no encoder; the caller
// sends it its own way); False on a closing transport; raises on a packet
// the codec refuses.
PyObject* Transport_request(Transport* t, PyObject* args) {
  PyObject *pkt, *req;
  if (!PyArg_ParseTuple(args, "O!O", &PyDict_Type, &pkt, &req)) return nullptr;
  Router& rt = *t->rt;
  if (!rt.on || rt.encode == nullptr) Py_RETURN_NONE;   // caller's path
  if (t->closed || t->closing || t->wr_shut || t->eof_pending)
    Py_RETURN_FALSE;
  PyObject* xo = PyDict_GetItemString(pkt, "xid");           // borrowed
  PyObject* op = PyDict_GetItemString(pkt, "opcode");
  if (xo == nullptr || op == nullptr) {
    PyErr_SetString(PyExc_KeyError, "request: xid/opcode");
    return nullptr;
  }
  if (!rt.encode(pkt, t->wbuf, true)) return nullptr;
  if (PyDict_SetItem(rt.reqs, xo, req) != 0 ||
      PyDict_SetItem(rt.xmap, xo, op) != 0)
    return nullptr;
  PyObject* r = queue_write(t);
  if (r == Py_False) {
    // the send failed and the transport is closing: the caller fails this
    // request itself (False), so it must not stay registered — the closed
    // connection would fail it a second time
    if (PyDict_DelItem(rt.reqs, xo) != 0) PyErr_Clear();
    if (PyDict_DelItem(rt.xmap, xo) != 0) PyErr_Clear();
  }
  return r;
}

// route_state() -> (max_zxid, last_rx_ms, routed): what the router saw.
PyObject* Transport_route_state(Transport* t, PyObject*) {
  const Router& rt = *t->rt;
  return Py_BuildValue("(LdL)", (long long)rt.max_zxid, rt.last_rx,
                       (long long)rt.routed);
}

// take_notes() -> (bytes, frames): the notification frames the sink kept
// since the last call.
PyObject* Transport_take_notes(Transport* t, PyObject*) {
  NoteSink& ns = *t->ns;
  PyObject* b = PyBytes_FromStringAndSize(ns.buf.data(),
                                          (Py_ssize_t)ns.buf.size());
  if (b == nullptr) return nullptr;
  const long long nf = ns.frames;
  ns.buf.clear();
  ns.frames = 0;
  return Py_BuildValue("(NL)", b, nf);
}

// capture_cancel(): end an active capture (done gets CAP_CANCEL).
PyObject* Transport_capture_cancel(Transport* t, PyObject*) {
  if (t->cap->on) capture_end(t, CAP_CANCEL);
  Py_RETURN_NONE;
}

PyObject* Transport_fatal(Transport* t, PyObject* arg) {
  int err = (int)PyLong_AsLong(arg);
  if (err == -1 && PyErr_Occurred()) return nullptr;
  fatal(t, err);
  Py_RETURN_NONE;
}

PyObject* Transport_write_eof(Transport* t, PyObject*) {
  if (t->closed || t->wr_shut) Py_RETURN_NONE;
  t->eof_pending = true;
  if (t->connected && t->woff == t->wbuf->size()) shut_wr(t);
  Py_RETURN_NONE;
}

PyObject* Transport_can_write_eof(Transport*, PyObject*) { Py_RETURN_TRUE; }

// Close now, drop unsent output; connection_lost(None) follows from the loop
// (asyncio's abort() contract, which TcpSocket relies on).
PyObject* Transport_abort(Transport* t, PyObject*) {
  if (t->closed) Py_RETURN_NONE;
  const bool was_connected = t->connected;
  t->closed = true;
  Py_CLEAR(t->on_fail);
  Py_INCREF(t);
  drop_watch(&t->w);
  if (was_connected && t->protocol != nullptr)
    defer_method(t->w.loop, t->protocol, "connection_lost", Py_None);
  Py_DECREF(t);
  Py_RETURN_NONE;
}

// Cancel a connect in progress or close: no callbacks at all.
PyObject* Transport_cancel(Transport* t, PyObject*) {
  if (t->closed) Py_RETURN_NONE;
  t->closed = true;
  Py_CLEAR(t->on_fail);
  Py_INCREF(t);
  drop_watch(&t->w);
  Py_DECREF(t);
  Py_RETURN_NONE;
}

PyObject* Transport_close(Transport* t, PyObject*) {
  if (t->closed || t->closing) Py_RETURN_NONE;
  t->closing = true;
  if (!t->connected || t->woff == t->wbuf->size()) {
    Py_INCREF(t);
    const bool was_connected = t->connected;
    t->closed = true;
    drop_watch(&t->w);
    if (was_connected && t->protocol != nullptr)
      defer_method(t->w.loop, t->protocol, "connection_lost", Py_None);
    Py_DECREF(t);
  } else {
    refresh(t);
  }
  Py_RETURN_NONE;
}

PyObject* Transport_is_closing(Transport* t, PyObject*) {
  return PyBool_FromLong(t->closed || t->closing);
}

PyObject* Transport_pause(Transport* t, PyObject*) {
  t->paused = true;
  refresh(t);
  Py_RETURN_NONE;
}

PyObject* Transport_resume(Transport* t, PyObject*) {
  t->paused = false;
  refresh(t);
  Py_RETURN_NONE;
}

PyObject* Transport_extra(Transport* t, PyObject* args) {
  const char* name;
  PyObject* dflt = Py_None;
  if (!PyArg_ParseTuple(args, "s|O", &name, &dflt)) return nullptr;
  if (strcmp(name, "peername") == 0 && t->peer != nullptr) {
    Py_INCREF(t->peer);
    return t->peer;
  }
  if (strcmp(name, "fd") == 0) return PyLong_FromLong(t->w.fd);
  Py_INCREF(dflt);
  return dflt;
}

PyObject* Transport_get_pending(Transport* t, void*) {
  return PyLong_FromSize_t(t->wbuf->size() - t->woff);
}

PyMethodDef Transport_methods[] = {
    {"write", (PyCFunction)Transport_write, METH_O, "queue bytes"},
    {"write_eof", (PyCFunction)Transport_write_eof, METH_NOARGS, "half-close"},
    {"can_write_eof", (PyCFunction)Transport_can_write_eof, METH_NOARGS, ""},
    {"abort", (PyCFunction)Transport_abort, METH_NOARGS, "close now"},
    {"cancel", (PyCFunction)Transport_cancel, METH_NOARGS, "close, no events"},
    {"close", (PyCFunction)Transport_close, METH_NOARGS, "flush then close"},
    {"is_closing", (PyCFunction)Transport_is_closing, METH_NOARGS, ""},
    {"pause_reading", (PyCFunction)Transport_pause, METH_NOARGS, ""},
    {"resume_reading", (PyCFunction)Transport_resume, METH_NOARGS, ""},
    {"get_extra_info", (PyCFunction)Transport_extra, METH_VARARGS, ""},
    {"_fatal", (PyCFunction)Transport_fatal, METH_O, "internal"},
    {"write_from", (PyCFunction)Transport_write_from, METH_VARARGS,
     "queue bytes from raw memory"},
    {"capture", (PyCFunction)Transport_capture, METH_VARARGS,
     "route an xid range of reply frames into a buffer"},
    {"capture_cancel", (PyCFunction)Transport_capture_cancel, METH_NOARGS,
     "end the active capture"},
    {"note_sink", (PyCFunction)Transport_note_sink, METH_VARARGS,
     "keep NOTIFICATION frames natively"},
    {"route", (PyCFunction)Transport_route, METH_VARARGS,
     "settle outstanding requests' replies natively"},
    {"request", (PyCFunction)Transport_request, METH_VARARGS,
     "encode a request into the write buffer and register its reply"},
    {"route_state", (PyCFunction)Transport_route_state, METH_NOARGS,
     "(max_zxid, last_rx_ms, routed) of the reply router"},
    {"take_notes", (PyCFunction)Transport_take_notes, METH_NOARGS,
     "the kept NOTIFICATION frames (bytes, count)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Transport_getset[] = {
    {"pending", (getter)Transport_get_pending, nullptr, "unsent bytes",
     nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ---------------------------------------------------------------------------
// Server
// ---------------------------------------------------------------------------

int Server_traverse(Server* s, visitproc visit, void* arg) {
  Py_VISIT(s->factory);
  return 0;
}

int Server_clear(Server* s) {
  Py_CLEAR(s->factory);
  return 0;
}

void Server_dealloc(Server* s) {
  PyObject_GC_UnTrack(s);
  if (s->w.fd >= 0) close(s->w.fd);
  Server_clear(s);
  PyObject_GC_Del(s);
}

PyObject* peer_tuple(const sockaddr_storage& ss) {
  char host[INET6_ADDRSTRLEN] = {0};
  int port = 0;
  if (ss.ss_family == AF_INET) {
    const sockaddr_in* a = (const sockaddr_in*)&ss;
    inet_ntop(AF_INET, &a->sin_addr, host, sizeof host);
    port = ntohs(a->sin_port);
  } else if (ss.ss_family == AF_INET6) {
    const sockaddr_in6* a = (const sockaddr_in6*)&ss;
    inet_ntop(AF_INET6, &a->sin6_addr, host, sizeof host);
    port = ntohs(a->sin6_port);
  }
  return Py_BuildValue("(si)", host, port);
}

void server_event(Server* s) {
  Loop* L = s->w.loop;
  Py_INCREF(s);
  for (int i = 0; i < 64 && s->w.fd >= 0; ++i) {
    sockaddr_storage ss;
    socklen_t sl = sizeof ss;
    int fd = accept4(s->w.fd, (sockaddr*)&ss, &sl,
                     SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR) continue;
      break;                     // EAGAIN, or a transient accept error
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    Transport* t = new_transport(L, fd);
    if (t == nullptr) { close(fd); report_exception(L); break; }
    t->connected = true;
    t->peer = peer_tuple(ss);
    PyObject* proto = PyObject_CallNoArgs(s->factory);
    if (proto == nullptr) {
      report_exception(L);
      Py_DECREF(t);
      continue;
    }
    t->protocol = proto;
    if (add_watch(L, &t->w, EPOLLIN | EPOLLRDHUP) != 0) {
      Py_DECREF(t);
      continue;
    }
    invoke(L, proto, "connection_made", (PyObject*)t);
    Py_DECREF(t);
  }
  Py_DECREF(s);
}

PyObject* Server_close(Server* s, PyObject*) {
  Py_INCREF(s);
  drop_watch(&s->w);
  Py_DECREF(s);
  Py_RETURN_NONE;
}

PyObject* Server_get_port(Server* s, void*) { return PyLong_FromLong(s->port); }

PyMethodDef Server_methods[] = {
    {"close", (PyCFunction)Server_close, METH_NOARGS, "stop listening"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Server_getset[] = {
    {"port", (getter)Server_get_port, nullptr, "bound port", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ---------------------------------------------------------------------------
// Loop
// ---------------------------------------------------------------------------

PyObject* Loop_new(PyTypeObject* type, PyObject* args, PyObject*) {
  PyObject* on_exc = nullptr;
  if (!PyArg_ParseTuple(args, "|O", &on_exc)) return nullptr;
  Loop* L = (Loop*)type->tp_alloc(type, 0);
  if (L == nullptr) return nullptr;
  L->epfd = epoll_create1(EPOLL_CLOEXEC);
  L->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (L->epfd < 0 || L->evfd < 0) {
    PyErr_SetFromErrno(PyExc_OSError);
    Py_DECREF(L);
    return nullptr;
  }
  epoll_event e;
  e.events = EPOLLIN;
  e.data.u64 = 0;                       // reg 0 = the wake-up eventfd
  epoll_ctl(L->epfd, EPOLL_CTL_ADD, L->evfd, &e);
  L->running = L->stopping = false;
  L->seq = 0;
  L->next_reg = 0;
  L->on_exception = (on_exc && on_exc != Py_None) ? on_exc : nullptr;
  Py_XINCREF(L->on_exception);
  L->ready = new std::deque<Handle*>();
  L->last_active = 0;
  L->timers = new std::vector<Handle*>();
  L->regs = new std::unordered_map<uint64_t, Watched*>();
  L->dirty = new std::vector<Transport*>();
  L->wakes = new std::vector<PyObject*>();
  return (PyObject*)L;
}

void clear_all(Loop* L) {
  for (Transport* t : *L->dirty) {
    t->queued = false;
    Py_DECREF(t);
  }
  L->dirty->clear();
  for (Handle* h : *L->ready) Py_DECREF(h);
  L->ready->clear();
  for (Handle* h : *L->timers) Py_DECREF(h);
  L->timers->clear();
  std::vector<Watched*> ws;
  for (auto& kv : *L->regs) ws.push_back(kv.second);
  for (Watched* w : ws) {
    Py_INCREF(w);
    if (w->kind == K_TRANSPORT) ((Transport*)w)->closed = true;
    drop_watch(w);
    Py_DECREF(w);
  }
}

void Loop_dealloc(Loop* L) {
  if (L->wakes != nullptr) {
    flip_wakes(L);
    drop_wakes(L);
    delete L->wakes;
  }
  if (L->ready != nullptr) clear_all(L);
  delete L->ready;
  delete L->timers;
  delete L->regs;
  delete L->dirty;
  if (L->epfd >= 0) close(L->epfd);
  if (L->evfd >= 0) close(L->evfd);
  Py_XDECREF(L->on_exception);
  Py_TYPE(L)->tp_free((PyObject*)L);
}

void run_handle(Loop* L, Handle* h) {
  if (h->cancelled || h->fn == nullptr) return;
  PyObject* fn = h->fn;
  PyObject* args = h->args;
  Py_INCREF(fn);
  Py_INCREF(args);
  PyObject* r = PyObject_Call(fn, args, nullptr);
  if (r == nullptr) report_exception(L);
  Py_XDECREF(r);
  Py_DECREF(fn);
  Py_DECREF(args);
}

PyObject* Loop_run(Loop* L, PyObject*) {
  if (L->running) {
    PyErr_SetString(PyExc_RuntimeError, "loop already running");
    return nullptr;
  }
  L->thread = pthread_self();
  L->running = true;
  std::vector<epoll_event> evs(256);
  std::vector<Handle*> due;
  while (!L->stopping) {
    flush_dirty(L);
    int timeout = -1;
    if (!L->ready->empty()) {
      timeout = 0;
    } else {
      // drop cancelled timers at the top so they do not shorten the wait
      while (!L->timers->empty() && L->timers->front()->cancelled) {
        std::pop_heap(L->timers->begin(), L->timers->end(), TimerCmp());
        Py_DECREF(L->timers->back());
        L->timers->pop_back();
      }
      if (!L->timers->empty()) {
        const double d = L->timers->front()->when - mono_ms();
        timeout = d <= 0 ? 0 : (int)std::ceil(d);
      }
    }
    int n;
    Py_BEGIN_ALLOW_THREADS
    flip_wakes(L);              // blocked callers wake to a free GIL
    if (timeout != 0 && loop_spin_ms() > 0) {
      // Adaptive busy-poll: for a short window after the last activity the
      // thread polls instead of sleeping, so the reply to a request it just
      // wrote (or the next call_soon) is picked up without a wake-up from
      // an idle core (tens of us per hop on the GPU boxes).  Idle loops
      // still block: the window only follows activity (a timer firing is
      // not activity), and time spent spinning comes off the wait.
      const double t_end = L->last_active + loop_spin_ms();
      const double spin_start = mono_ms();
      for (;;) {
        n = epoll_wait(L->epfd, evs.data(), (int)evs.size(), 0);
        if (n != 0) break;
        const double now = mono_ms();
        if (now >= t_end) {
          int rest = timeout;
          if (rest > 0) {
            const double waited = now - spin_start;
            rest = std::max(0, rest - (int)waited);
          }
          n = epoll_wait(L->epfd, evs.data(), (int)evs.size(), rest);
          break;
        }
      }
    } else {
      n = epoll_wait(L->epfd, evs.data(), (int)evs.size(), timeout);
    }
    Py_END_ALLOW_THREADS
    drop_wakes(L);
    if (n > 0 || !L->ready->empty()) L->last_active = mono_ms();
    if (n < 0 && errno != EINTR) {
      PyErr_SetFromErrno(PyExc_OSError);
      L->running = false;
      flip_wakes(L);
      drop_wakes(L);
      return nullptr;
    }
    for (int i = 0; i < n && !L->stopping; ++i) {
      const uint64_t reg = evs[i].data.u64;
      if (reg == 0) {
        uint64_t v;
        while (read(L->evfd, &v, sizeof v) > 0) {
        }
        continue;
      }
      auto it = L->regs->find(reg);
      if (it == L->regs->end()) continue;        // closed while we slept
      Watched* w = it->second;
      if (w->kind == K_TRANSPORT) transport_event((Transport*)w, evs[i].events);
      else server_event((Server*)w);
    }
    // timers that are due
    const double now = mono_ms();
    while (!L->timers->empty() && L->timers->front()->when <= now) {
      std::pop_heap(L->timers->begin(), L->timers->end(), TimerCmp());
      due.push_back(L->timers->back());
      L->timers->pop_back();
    }
    for (Handle* h : due) {
      if (!L->stopping) run_handle(L, h);
      Py_DECREF(h);
    }
    due.clear();
    // the ready queue as it stands now (new entries wait for the next turn)
    size_t k = L->ready->size();
    while (k-- > 0 && !L->ready->empty() && !L->stopping) {
      Handle* h = L->ready->front();
      L->ready->pop_front();
      run_handle(L, h);
      Py_DECREF(h);
    }
  }
  flush_dirty(L);           // what the last turn wrote still leaves
  clear_all(L);
  L->running = false;
  flip_wakes(L);                // callers set on the last turn
  drop_wakes(L);
  Py_RETURN_NONE;
}

PyObject* Loop_stop(Loop* L, PyObject*) {
  L->stopping = true;
  uint64_t one = 1;
  ssize_t r = write(L->evfd, &one, sizeof one);
  (void)r;
  Py_RETURN_NONE;
}

PyObject* Loop_call_soon(Loop* L, PyObject* args) {
  PyObject *fn, *fargs = nullptr;
  if (!PyArg_ParseTuple(args, "O|O!", &fn, &PyTuple_Type, &fargs))
    return nullptr;
  Handle* h = new_handle(fn, fargs);
  if (h == nullptr) return nullptr;
  push_ready(L, h);
  return (PyObject*)h;
}

PyObject* Loop_call_later(Loop* L, PyObject* args) {
  double ms;
  PyObject *fn, *fargs = nullptr;
  if (!PyArg_ParseTuple(args, "dO|O!", &ms, &fn, &PyTuple_Type, &fargs))
    return nullptr;
  Handle* h = new_handle(fn, fargs);
  if (h == nullptr) return nullptr;
  h->when = mono_ms() + (ms > 0 ? ms : 0);
  push_timer(L, h);
  return (PyObject*)h;
}

PyObject* Loop_time_ms(Loop*, PyObject*) { return PyFloat_FromDouble(mono_ms()); }

PyObject* Loop_in_loop(Loop* L, PyObject*) {
  return PyBool_FromLong(on_loop_thread(L));
}

int resolve(const char* host, int port, sockaddr_storage* ss, socklen_t* sl) {
  addrinfo hints;
  memset(&hints, 0, sizeof hints);
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_NUMERICSERV;
  char ps[16];
  snprintf(ps, sizeof ps, "%d", port);
  addrinfo* res = nullptr;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = getaddrinfo(host, ps, &hints, &res);
  Py_END_ALLOW_THREADS
  if (rc != 0 || res == nullptr) return rc != 0 ? rc : EAI_NONAME;
  memcpy(ss, res->ai_addr, res->ai_addrlen);
  *sl = res->ai_addrlen;
  freeaddrinfo(res);
  return 0;
}

PyObject* Loop_connect(Loop* L, PyObject* args) {
  const char* host;
  int port;
  PyObject *proto, *on_fail;
  if (!PyArg_ParseTuple(args, "siOO", &host, &port, &proto, &on_fail))
    return nullptr;
  Transport* t = new_transport(L, -1);
  if (t == nullptr) return nullptr;
  Py_INCREF(proto);
  t->protocol = proto;
  Py_INCREF(on_fail);
  t->on_fail = on_fail;
  t->peer = Py_BuildValue("(si)", host, port);
  sockaddr_storage ss;
  socklen_t sl;
  int err = 0;
  const int rc = resolve(host, port, &ss, &sl);
  int fd = -1;
  if (rc != 0) {
    err = EHOSTUNREACH;
  } else {
    fd = socket(ss.ss_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (fd < 0) err = errno;
  }
  if (fd >= 0) {
    t->w.fd = fd;
    t->connecting = true;
    if (connect(fd, (sockaddr*)&ss, sl) != 0 && errno != EINPROGRESS)
      err = errno;
    // the outcome (success or failure) is always reported from the loop,
    // like asyncio's create_connection, never inside this call
    if (err == 0 && add_watch(L, &t->w, EPOLLOUT) != 0) err = errno;
  }
  if (err != 0) {
    t->closed = true;
    if (t->w.fd >= 0) { close(t->w.fd); t->w.fd = -1; }
    PyObject* exc = os_error(err);
    PyObject* cb = t->on_fail;
    t->on_fail = nullptr;
    if (exc != nullptr && cb != nullptr) {
      PyObject* a = PyTuple_Pack(1, exc);
      defer(L, cb, a);
      Py_XDECREF(a);
    }
    Py_XDECREF(exc);
    Py_XDECREF(cb);
  }
  return (PyObject*)t;
}

PyObject* Loop_listen(Loop* L, PyObject* args) {
  const char* host;
  int port;
  PyObject* factory;
  if (!PyArg_ParseTuple(args, "siO", &host, &port, &factory)) return nullptr;
  sockaddr_storage ss;
  socklen_t sl;
  if (resolve(host, port, &ss, &sl) != 0) {
    PyErr_Format(PyExc_OSError, "cannot resolve %s", host);
    return nullptr;
  }
  int fd = socket(ss.ss_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return PyErr_SetFromErrno(PyExc_OSError);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (bind(fd, (sockaddr*)&ss, sl) != 0 || listen(fd, 128) != 0) {
    const int e = errno;
    close(fd);
    errno = e;
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  sockaddr_storage bs;
  socklen_t bl = sizeof bs;
  getsockname(fd, (sockaddr*)&bs, &bl);
  Server* s = PyObject_GC_New(Server, &ServerType);
  if (s == nullptr) { close(fd); return nullptr; }
  s->w.kind = K_SERVER;
  s->w.fd = fd;
  s->w.reg = 0;
  s->w.events = 0;
  s->w.loop = L;
  Py_INCREF(factory);
  s->factory = factory;
  s->port = bs.ss_family == AF_INET6 ? ntohs(((sockaddr_in6*)&bs)->sin6_port)
                                     : ntohs(((sockaddr_in*)&bs)->sin_port);
  PyObject_GC_Track((PyObject*)s);
  if (add_watch(L, &s->w, EPOLLIN) != 0) {
    Py_DECREF(s);
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  wake(L);
  return (PyObject*)s;
}

PyObject* Loop_stats(Loop* L, PyObject*) {
  return Py_BuildValue("{s:n,s:n,s:n}", "ready", (Py_ssize_t)L->ready->size(),
                       "timers", (Py_ssize_t)L->timers->size(), "fds",
                       (Py_ssize_t)L->regs->size());
}

PyMethodDef Loop_methods[] = {
    {"run", (PyCFunction)Loop_run, METH_NOARGS, "run until stop()"},
    {"stop", (PyCFunction)Loop_stop, METH_NOARGS, "stop (any thread)"},
    {"call_soon", (PyCFunction)Loop_call_soon, METH_VARARGS,
     "call_soon(fn, args=()) -> Handle"},
    {"call_later", (PyCFunction)Loop_call_later, METH_VARARGS,
     "call_later(ms, fn, args=()) -> Handle"},
    {"time_ms", (PyCFunction)Loop_time_ms, METH_NOARGS, "monotonic ms"},
    {"in_loop", (PyCFunction)Loop_in_loop, METH_NOARGS, "on the loop thread?"},
    {"connect", (PyCFunction)Loop_connect, METH_VARARGS,
     "connect(host, port, protocol, on_fail) -> Transport"},
    {"listen", (PyCFunction)Loop_listen, METH_VARARGS,
     "listen(host, port, factory) -> Server"},
    {"stats", (PyCFunction)Loop_stats, METH_NOARGS, "queue / timer / fd counts"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_zkloop",
                   "zkmi native event loop (epoll)", -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__zkloop(void) {
  HandleType.tp_name = "_zkloop.Handle";
  HandleType.tp_basicsize = sizeof(Handle);
  HandleType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  HandleType.tp_traverse = (traverseproc)Handle_traverse;
  HandleType.tp_clear = (inquiry)Handle_clear;
  HandleType.tp_dealloc = (destructor)Handle_dealloc;
  HandleType.tp_methods = Handle_methods;
  HandleType.tp_getset = Handle_getset;

  TransportType.tp_name = "_zkloop.Transport";
  TransportType.tp_basicsize = sizeof(Transport);
  TransportType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  TransportType.tp_traverse = (traverseproc)Transport_traverse;
  TransportType.tp_clear = (inquiry)Transport_clear;
  TransportType.tp_dealloc = (destructor)Transport_dealloc;
  TransportType.tp_methods = Transport_methods;
  TransportType.tp_getset = Transport_getset;

  ServerType.tp_name = "_zkloop.Server";
  ServerType.tp_basicsize = sizeof(Server);
  ServerType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  ServerType.tp_traverse = (traverseproc)Server_traverse;
  ServerType.tp_clear = (inquiry)Server_clear;
  ServerType.tp_dealloc = (destructor)Server_dealloc;
  ServerType.tp_methods = Server_methods;
  ServerType.tp_getset = Server_getset;

  WaiterType.tp_name = "_zkloop.Waiter";
  WaiterType.tp_basicsize = sizeof(Waiter);
  WaiterType.tp_flags = Py_TPFLAGS_DEFAULT;
  WaiterType.tp_new = Waiter_new;
  WaiterType.tp_dealloc = (destructor)Waiter_dealloc;
  WaiterType.tp_methods = Waiter_methods;
  WaiterType.tp_getset = Waiter_getset;

  LoopType.tp_name = "_zkloop.Loop";
  LoopType.tp_basicsize = sizeof(Loop);
  LoopType.tp_flags = Py_TPFLAGS_DEFAULT;
  LoopType.tp_new = Loop_new;
  LoopType.tp_dealloc = (destructor)Loop_dealloc;
  LoopType.tp_methods = Loop_methods;

  if (PyType_Ready(&HandleType) < 0 || PyType_Ready(&TransportType) < 0 ||
      PyType_Ready(&ServerType) < 0 || PyType_Ready(&LoopType) < 0 ||
      PyType_Ready(&WaiterType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&mod);
  if (m == nullptr) return nullptr;
  Py_INCREF(&LoopType);
  PyModule_AddObject(m, "Loop", (PyObject*)&LoopType);
  Py_INCREF(&HandleType);
  PyModule_AddObject(m, "Handle", (PyObject*)&HandleType);
  Py_INCREF(&TransportType);
  PyModule_AddObject(m, "Transport", (PyObject*)&TransportType);
  Py_INCREF(&ServerType);
  PyModule_AddObject(m, "Server", (PyObject*)&ServerType);
  Py_INCREF(&WaiterType);
  PyModule_AddObject(m, "Waiter", (PyObject*)&WaiterType);
  return m;
}
