// _zkfsm — the FSM runtime every zkmi state machine runs on (the
// `mooremachine` contract the reference builds its ZKClient, ZKConnectionFSM,
// ZKSession and ZKWatchEvent on: SURVEY §2.2; lib/client.js:123,
// lib/connection-fsm.js:27, lib/zk-session.js:38, :675).
//
// A machine is a Python object with `state_<name>(S)` methods; its Core
// (this module) owns everything the runtime does around them:
//
//   * transitions: request(state) queues; the queue drains in order, one
//     state function at a time, and `stateChanged` is emitted on the owner
//     after each state function has run (listeners registered in the entry
//     see the machine's next transitions);
//   * scoped handles: the Handle passed to a state function records every
//     listener, timer, interval and immediate registered through it, and
//     they are all torn down when the state is left (the reference's race
//     fixes, e.g. #39, test/basic.test.js:1173-1174, rely on this);
//   * sub-states 'parent.child' (method state_parent__child): entering a
//     child keeps the parent's handles; isInState('parent') holds in the
//     child; leaving to anything else disposes both;
//   * a stale handle (its state left, or already used for a transition)
//     refuses gotoState.
//
// Timers go through the owner's loop (call_later / call_soon, the native
// epoll loop of zk_loop.cpp); a timer's callback is a Guard that does
// nothing once its handle is disposed, so a cancelled-but-queued timer is
// harmless.  The pure-Python runtime (zkmi/runtime/fsm.py) is kept as the
// test oracle.
#include <Python.h>

#include <string>
#include <vector>

namespace {

struct Core;

// ---- Handle ----------------------------------------------------------------

// One disposer: a listener (emitter, evt, fn) to remove, or a timer handle
// (obj with .cancel()) to cancel.
struct Disp {
  PyObject* a;      // emitter, or the timer handle
  PyObject* evt;    // nullptr: a timer
  PyObject* fn;
};

struct Handle {
  PyObject_HEAD
  Core* core;                   // strong ref
  PyObject* state;              // str
  std::vector<Disp>* disp;
  bool valid;
  bool used;
};

struct Guard {
  PyObject_HEAD
  Handle* h;                    // strong ref
  PyObject* fn;
};

struct Interval {
  PyObject_HEAD
  Handle* h;                    // strong ref
  PyObject* fn;                 // the guarded callback
  PyObject* timer;              // the pending loop handle
  double ms;
  bool cancelled;
};

struct Core {
  PyObject_HEAD
  PyObject* owner;              // the machine (it holds the core too: a
                                // cycle the collector sees, see traverse)
  PyObject* loop;
  PyObject* state;              // str or None
  std::vector<std::pair<PyObject*, Handle*>>* handles;   // outer -> inner
  std::vector<PyObject*>* queue;                          // states (str)
  std::vector<PyObject*>* history;                        // last 64 states
  PyObject* entered;            // owner._fsm_entered (bound) or nullptr
  bool busy;
};

PyTypeObject HandleType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject GuardType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject IntervalType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject CoreType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* Core_request_state(Core* c, PyObject* state);

void dispose(Handle* h) {
  if (!h->valid) return;
  h->valid = false;
  std::vector<Disp> ds;
  ds.swap(*h->disp);
  // in reverse registration order; a failing disposer does not stop the
  // others (its error is reported, like an exception in a loop callback)
  for (auto it = ds.rbegin(); it != ds.rend(); ++it) {
    PyObject* r = it->evt != nullptr
                      ? PyObject_CallMethod(it->a, "removeListener", "OO",
                                            it->evt, it->fn)
                      : PyObject_CallMethod(it->a, "cancel", nullptr);
    if (r == nullptr) PyErr_WriteUnraisable(it->a);
    Py_XDECREF(r);
    Py_XDECREF(it->a);
    Py_XDECREF(it->evt);
    Py_XDECREF(it->fn);
  }
}

int Handle_traverse(Handle* h, visitproc visit, void* arg) {
  Py_VISIT((PyObject*)h->core);
  Py_VISIT(h->state);
  if (h->disp != nullptr)
    for (auto& d : *h->disp) {
      Py_VISIT(d.a);
      Py_VISIT(d.evt);
      Py_VISIT(d.fn);
    }
  return 0;
}

int Handle_clear(Handle* h) {
  if (h->disp != nullptr) {
    std::vector<Disp> ds;
    ds.swap(*h->disp);
    for (auto& d : ds) {
      Py_XDECREF(d.a);
      Py_XDECREF(d.evt);
      Py_XDECREF(d.fn);
    }
  }
  Py_CLEAR(h->core);
  Py_CLEAR(h->state);
  return 0;
}

void Handle_dealloc(Handle* h) {
  PyObject_GC_UnTrack(h);
  Handle_clear(h);
  delete h->disp;
  PyObject_GC_Del(h);
}

Handle* new_handle(Core* c, PyObject* state) {
  Handle* h = PyObject_GC_New(Handle, &HandleType);
  if (h == nullptr) return nullptr;
  Py_INCREF(c);
  h->core = c;
  Py_INCREF(state);
  h->state = state;
  h->disp = new std::vector<Disp>();
  h->valid = true;
  h->used = false;
  PyObject_GC_Track((PyObject*)h);
  return h;
}

PyObject* make_guard(Handle* h, PyObject* fn) {
  Guard* g = PyObject_GC_New(Guard, &GuardType);
  if (g == nullptr) return nullptr;
  Py_INCREF(h);
  g->h = h;
  Py_INCREF(fn);
  g->fn = fn;
  PyObject_GC_Track((PyObject*)g);
  return (PyObject*)g;
}

void add_timer_disp(Handle* h, PyObject* timer) {
  Py_INCREF(timer);
  h->disp->push_back(Disp{timer, nullptr, nullptr});
}

// S.on(emitter, evt, cb): auto-unsubscribed when the state is left
PyObject* Handle_on(Handle* h, PyObject* args) {
  PyObject *em, *evt, *cb;
  if (!PyArg_ParseTuple(args, "OOO", &em, &evt, &cb)) return nullptr;
  if (!h->valid) Py_RETURN_NONE;
  PyObject* r = PyObject_CallMethod(em, "on", "OO", evt, cb);
  if (r == nullptr) return nullptr;
  Py_DECREF(r);
  Py_INCREF(em);
  Py_INCREF(evt);
  Py_INCREF(cb);
  h->disp->push_back(Disp{em, evt, cb});
  Py_RETURN_NONE;
}

// S.timeout(ms, cb) -> the loop's timer handle
PyObject* Handle_timeout(Handle* h, PyObject* args) {
  PyObject *ms, *cb;
  if (!PyArg_ParseTuple(args, "OO", &ms, &cb)) return nullptr;
  PyObject* g = make_guard(h, cb);
  if (g == nullptr) return nullptr;
  PyObject* t = PyObject_CallMethod(h->core->loop, "call_later", "OO", ms, g);
  Py_DECREF(g);
  if (t == nullptr) return nullptr;
  add_timer_disp(h, t);
  return t;
}

// S.immediate(cb)
PyObject* Handle_immediate(Handle* h, PyObject* cb) {
  PyObject* g = make_guard(h, cb);
  if (g == nullptr) return nullptr;
  PyObject* t = PyObject_CallMethod(h->core->loop, "call_soon", "O", g);
  Py_DECREF(g);
  if (t == nullptr) return nullptr;
  add_timer_disp(h, t);
  return t;
}

// S.callback(cb): a wrapper that does nothing once the state is left
PyObject* Handle_callback(Handle* h, PyObject* cb) { return make_guard(h, cb); }

// S.interval(ms, cb) -> Interval (cancel(), unref())
PyObject* Interval_tick(Interval* iv, PyObject*);

PyObject* Handle_interval(Handle* h, PyObject* args) {
  double ms;
  PyObject* cb;
  if (!PyArg_ParseTuple(args, "dO", &ms, &cb)) return nullptr;
  Interval* iv = PyObject_GC_New(Interval, &IntervalType);
  if (iv == nullptr) return nullptr;
  Py_INCREF(h);
  iv->h = h;
  iv->fn = make_guard(h, cb);
  iv->timer = nullptr;
  iv->ms = ms;
  iv->cancelled = false;
  PyObject_GC_Track((PyObject*)iv);
  if (iv->fn == nullptr) { Py_DECREF(iv); return nullptr; }
  PyObject* tick = PyObject_GetAttrString((PyObject*)iv, "_tick");
  PyObject* t = tick ? PyObject_CallMethod(h->core->loop, "call_later", "dO",
                                           ms, tick)
                     : nullptr;
  Py_XDECREF(tick);
  if (t == nullptr) { Py_DECREF(iv); return nullptr; }
  iv->timer = t;
  Py_INCREF(iv);
  h->disp->push_back(Disp{(PyObject*)iv, nullptr, nullptr});
  return (PyObject*)iv;
}

// S.gotoState(name)
PyObject* Handle_goto(Handle* h, PyObject* state) {
  if (!PyUnicode_Check(state)) {
    PyErr_SetString(PyExc_TypeError, "state must be a str");
    return nullptr;
  }
  if (!h->valid || h->used) {
    PyObject* cur = h->core->state;
    PyErr_Format(PyExc_AssertionError,
                 "FSM %s: gotoState(%R) through a handle for state %R that "
                 "was already left or used (now %R)",
                 Py_TYPE(h->core->owner)->tp_name, state, h->state, cur);
    return nullptr;
  }
  h->used = true;
  return Core_request_state(h->core, state);
}

PyObject* Handle_dispose(Handle* h, PyObject*) {
  dispose(h);
  Py_RETURN_NONE;
}

PyObject* Handle_get_valid(Handle* h, void*) { return PyBool_FromLong(h->valid); }
PyObject* Handle_get_state(Handle* h, void*) { return Py_NewRef(h->state); }

PyMethodDef Handle_methods[] = {
    {"on", (PyCFunction)Handle_on, METH_VARARGS, "on(emitter, evt, cb)"},
    {"timeout", (PyCFunction)Handle_timeout, METH_VARARGS, "timeout(ms, cb)"},
    {"interval", (PyCFunction)Handle_interval, METH_VARARGS,
     "interval(ms, cb)"},
    {"immediate", (PyCFunction)Handle_immediate, METH_O, "immediate(cb)"},
    {"callback", (PyCFunction)Handle_callback, METH_O, "callback(cb)"},
    {"gotoState", (PyCFunction)Handle_goto, METH_O, "gotoState(state)"},
    {"_dispose", (PyCFunction)Handle_dispose, METH_NOARGS, ""},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Handle_getset[] = {
    {"_valid", (getter)Handle_get_valid, nullptr, "", nullptr},
    {"_state", (getter)Handle_get_state, nullptr, "", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ---- Guard -----------------------------------------------------------------

PyObject* Guard_call(Guard* g, PyObject* args, PyObject* kw) {
  if (g->h == nullptr || !g->h->valid || g->fn == nullptr) Py_RETURN_NONE;
  return PyObject_Call(g->fn, args, kw);
}

int Guard_traverse(Guard* g, visitproc visit, void* arg) {
  Py_VISIT((PyObject*)g->h);
  Py_VISIT(g->fn);
  return 0;
}

int Guard_clear(Guard* g) {
  Py_CLEAR(g->h);
  Py_CLEAR(g->fn);
  return 0;
}

void Guard_dealloc(Guard* g) {
  PyObject_GC_UnTrack(g);
  Guard_clear(g);
  PyObject_GC_Del(g);
}

// ---- Interval --------------------------------------------------------------

PyObject* Interval_tick(Interval* iv, PyObject*) {
  Py_CLEAR(iv->timer);
  if (iv->cancelled || iv->h == nullptr || !iv->h->valid) Py_RETURN_NONE;
  // re-armed before the callback runs (a slow callback does not drift the
  // period; the callback may leave the state, which cancels the re-arm)
  PyObject* tick = PyObject_GetAttrString((PyObject*)iv, "_tick");
  if (tick == nullptr) return nullptr;
  PyObject* t = PyObject_CallMethod(iv->h->core->loop, "call_later", "dO",
                                    iv->ms, tick);
  Py_DECREF(tick);
  if (t == nullptr) return nullptr;
  iv->timer = t;
  return PyObject_CallNoArgs(iv->fn);
}

PyObject* Interval_cancel(Interval* iv, PyObject*) {
  iv->cancelled = true;
  if (iv->timer != nullptr) {
    PyObject* r = PyObject_CallMethod(iv->timer, "cancel", nullptr);
    Py_XDECREF(r);
    if (r == nullptr) return nullptr;
    Py_CLEAR(iv->timer);
  }
  Py_RETURN_NONE;
}

PyObject* Interval_unref(Interval* iv, PyObject*) {
  // loop threads are daemons (see zk_loop.cpp Handle.unref)
  return Py_NewRef((PyObject*)iv);
}

int Interval_traverse(Interval* iv, visitproc visit, void* arg) {
  Py_VISIT((PyObject*)iv->h);
  Py_VISIT(iv->fn);
  Py_VISIT(iv->timer);
  return 0;
}

int Interval_clear(Interval* iv) {
  Py_CLEAR(iv->h);
  Py_CLEAR(iv->fn);
  Py_CLEAR(iv->timer);
  return 0;
}

void Interval_dealloc(Interval* iv) {
  PyObject_GC_UnTrack(iv);
  Interval_clear(iv);
  PyObject_GC_Del(iv);
}

PyMethodDef Interval_methods[] = {
    {"_tick", (PyCFunction)Interval_tick, METH_NOARGS, ""},
    {"cancel", (PyCFunction)Interval_cancel, METH_NOARGS, "cancel()"},
    {"unref", (PyCFunction)Interval_unref, METH_NOARGS, "unref()"},
    {nullptr, nullptr, 0, nullptr}};

// ---- Core ------------------------------------------------------------------

// "parent.child" starts with "parent."?
bool is_child_of(PyObject* state, PyObject* cur) {
  Py_ssize_t ns, nc;
  const char* s = PyUnicode_AsUTF8AndSize(state, &ns);
  const char* c = PyUnicode_AsUTF8AndSize(cur, &nc);
  if (s == nullptr || c == nullptr) { PyErr_Clear(); return false; }
  return ns > nc && std::char_traits<char>::compare(s, c, (size_t)nc) == 0 &&
         s[nc] == '.';
}

// Enter `state`: dispose the handles of the levels left, run the state
// function with a fresh handle, emit stateChanged.
int enter(Core* c, PyObject* state) {
  // the state function: state_<name> with '.' -> '__'
  std::string name("state_");
  {
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(state, &n);
    if (s == nullptr) return -1;
    for (Py_ssize_t i = 0; i < n; ++i) {
      if (s[i] == '.') name += "__";
      else name += s[i];
    }
  }
  PyObject* fn = PyObject_GetAttrString(c->owner, name.c_str());
  if (fn == nullptr) {
    PyErr_Clear();
    PyErr_Format(PyExc_AssertionError, "%s has no state %R",
                 Py_TYPE(c->owner)->tp_name, state);
    return -1;
  }
  // keep the ancestors' handles only when entering a strict descendant of
  // the current state (parent -> parent.child)
  size_t keep = 0;
  if (c->state != Py_None && is_child_of(state, c->state)) {
    keep = c->handles->size();
    for (auto& p : *c->handles) p.second->used = false;  // may move again
  }
  while (c->handles->size() > keep) {
    auto p = c->handles->back();
    c->handles->pop_back();
    dispose(p.second);
    Py_DECREF(p.first);
    Py_DECREF((PyObject*)p.second);
  }
  Py_INCREF(state);
  Py_SETREF(c->state, state);
  if (c->history->size() > 64) {
    for (size_t i = 0; i < 32; ++i) Py_DECREF((*c->history)[i]);
    c->history->erase(c->history->begin(), c->history->begin() + 32);
  }
  Py_INCREF(state);
  c->history->push_back(state);
  Handle* h = new_handle(c, state);
  if (h == nullptr) { Py_DECREF(fn); return -1; }
  Py_INCREF(state);
  c->handles->emplace_back(state, h);
  PyObject* r = PyObject_CallOneArg(fn, (PyObject*)h);
  Py_DECREF(fn);
  if (r == nullptr) return -1;
  Py_DECREF(r);
  r = PyObject_CallMethod(c->owner, "emit", "sO", "stateChanged", state);
  if (r == nullptr) return -1;
  Py_DECREF(r);
  if (c->entered != nullptr) {
    // the owner's hook after every transition (ZKSession: the watch
    // engine's ready / unready)
    r = PyObject_CallOneArg(c->entered, state);
    if (r == nullptr) return -1;
    Py_DECREF(r);
  }
  return 0;
}

PyObject* Core_request_state(Core* c, PyObject* state) {
  Py_INCREF(state);
  c->queue->push_back(state);
  if (c->busy) Py_RETURN_NONE;
  c->busy = true;
  // a reference to the core for the drain (a state function may drop the
  // owner's last reference to it)
  Py_INCREF(c);
  int rc = 0;
  while (!c->queue->empty()) {
    PyObject* nxt = c->queue->front();
    c->queue->erase(c->queue->begin());
    rc = enter(c, nxt);
    Py_DECREF(nxt);
    // an exception in a state function ends the drain; what it queued
    // stays queued (the next request drains it), as in the Python runtime
    if (rc != 0) break;
  }
  c->busy = false;
  Py_DECREF(c);
  if (rc != 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* Core_request(Core* c, PyObject* state) {
  if (!PyUnicode_Check(state)) {
    PyErr_SetString(PyExc_TypeError, "state must be a str");
    return nullptr;
  }
  return Core_request_state(c, state);
}

// Core(owner, loop)
int Core_init(Core* c, PyObject* args, PyObject*) {
  PyObject *owner, *loop;
  if (!PyArg_ParseTuple(args, "OO", &owner, &loop)) return -1;
  Py_INCREF(owner);
  Py_XSETREF(c->owner, owner);
  Py_INCREF(loop);
  Py_XSETREF(c->loop, loop);
  Py_INCREF(Py_None);
  Py_XSETREF(c->state, Py_None);
  if (c->handles == nullptr) {
    c->handles = new std::vector<std::pair<PyObject*, Handle*>>();
    c->queue = new std::vector<PyObject*>();
    c->history = new std::vector<PyObject*>();
  }
  c->busy = false;
  Py_CLEAR(c->entered);
  if (PyObject_HasAttrString(owner, "_fsm_entered")) {
    c->entered = PyObject_GetAttrString(owner, "_fsm_entered");
    if (c->entered == nullptr) return -1;
  }
  return 0;
}

PyObject* Core_new(PyTypeObject* type, PyObject*, PyObject*) {
  Core* c = (Core*)type->tp_alloc(type, 0);
  if (c != nullptr) {
    c->owner = nullptr;
    c->loop = c->state = c->entered = nullptr;
    c->handles = nullptr;
    c->queue = nullptr;
    c->history = nullptr;
    c->busy = false;
  }
  return (PyObject*)c;
}

int Core_traverse(Core* c, visitproc visit, void* arg) {
  Py_VISIT(c->owner);
  Py_VISIT(c->loop);
  Py_VISIT(c->state);
  Py_VISIT(c->entered);
  if (c->handles != nullptr)
    for (auto& p : *c->handles) {
      Py_VISIT(p.first);
      Py_VISIT((PyObject*)p.second);
    }
  if (c->queue != nullptr)
    for (PyObject* q : *c->queue) Py_VISIT(q);
  return 0;
}

int Core_clear(Core* c) {
  if (c->handles != nullptr) {
    auto hs = std::move(*c->handles);
    c->handles->clear();
    for (auto& p : hs) {
      Py_DECREF(p.first);
      Py_DECREF((PyObject*)p.second);
    }
  }
  if (c->queue != nullptr) {
    for (PyObject* q : *c->queue) Py_DECREF(q);
    c->queue->clear();
  }
  Py_CLEAR(c->loop);
  Py_CLEAR(c->entered);
  Py_CLEAR(c->owner);
  return 0;
}

void Core_dealloc(Core* c) {
  PyObject_GC_UnTrack(c);
  Core_clear(c);
  Py_CLEAR(c->state);
  if (c->history != nullptr)
    for (PyObject* s : *c->history) Py_DECREF(s);
  delete c->handles;
  delete c->queue;
  delete c->history;
  Py_TYPE(c)->tp_free((PyObject*)c);
}

PyObject* Core_get_state(Core* c, void*) { return Py_NewRef(c->state); }

// in_state(name): current == name, or a sub-state of it
PyObject* Core_in_state(Core* c, PyObject* name) {
  if (c->state == Py_None) Py_RETURN_FALSE;
  const int eq = PyUnicode_Compare(c->state, name);
  if (eq == 0) Py_RETURN_TRUE;
  if (PyErr_Occurred()) return nullptr;
  return PyBool_FromLong(is_child_of(c->state, name));
}

PyObject* Core_get_history(Core* c, void*) {
  PyObject* l = PyList_New((Py_ssize_t)c->history->size());
  if (l == nullptr) return nullptr;
  for (size_t i = 0; i < c->history->size(); ++i) {
    Py_INCREF((*c->history)[i]);
    PyList_SET_ITEM(l, (Py_ssize_t)i, (*c->history)[i]);
  }
  return l;
}

// handles() -> [(state, handle)]: the live levels (introspection, tests)
PyObject* Core_handles(Core* c, PyObject*) {
  PyObject* l = PyList_New(0);
  for (auto& p : *c->handles) {
    PyObject* t = PyTuple_Pack(2, p.first, (PyObject*)p.second);
    PyList_Append(l, t);
    Py_DECREF(t);
  }
  return l;
}

PyMethodDef Core_methods[] = {
    {"request", (PyCFunction)Core_request, METH_O, "request(state)"},
    {"in_state", (PyCFunction)Core_in_state, METH_O, "in_state(name)"},
    {"handles", (PyCFunction)Core_handles, METH_NOARGS, ""},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Core_getset[] = {
    {"state", (getter)Core_get_state, nullptr, "current state", nullptr},
    {"history", (getter)Core_get_history, nullptr, "recent states", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_zkfsm",
                      "native FSM runtime (mooremachine contract)", -1,
                      nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__zkfsm() {
  HandleType.tp_name = "zkmi._zkfsm.StateHandle";
  HandleType.tp_basicsize = sizeof(Handle);
  HandleType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  HandleType.tp_traverse = (traverseproc)Handle_traverse;
  HandleType.tp_clear = (inquiry)Handle_clear;
  HandleType.tp_dealloc = (destructor)Handle_dealloc;
  HandleType.tp_methods = Handle_methods;
  HandleType.tp_getset = Handle_getset;
  GuardType.tp_name = "zkmi._zkfsm.Guard";
  GuardType.tp_basicsize = sizeof(Guard);
  GuardType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  GuardType.tp_traverse = (traverseproc)Guard_traverse;
  GuardType.tp_clear = (inquiry)Guard_clear;
  GuardType.tp_dealloc = (destructor)Guard_dealloc;
  GuardType.tp_call = (ternaryfunc)Guard_call;
  IntervalType.tp_name = "zkmi._zkfsm.Interval";
  IntervalType.tp_basicsize = sizeof(Interval);
  IntervalType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  IntervalType.tp_traverse = (traverseproc)Interval_traverse;
  IntervalType.tp_clear = (inquiry)Interval_clear;
  IntervalType.tp_dealloc = (destructor)Interval_dealloc;
  IntervalType.tp_methods = Interval_methods;
  CoreType.tp_name = "zkmi._zkfsm.Core";
  CoreType.tp_basicsize = sizeof(Core);
  CoreType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  CoreType.tp_traverse = (traverseproc)Core_traverse;
  CoreType.tp_clear = (inquiry)Core_clear;
  CoreType.tp_new = Core_new;
  CoreType.tp_init = (initproc)Core_init;
  CoreType.tp_dealloc = (destructor)Core_dealloc;
  CoreType.tp_methods = Core_methods;
  CoreType.tp_getset = Core_getset;
  if (PyType_Ready(&HandleType) < 0 || PyType_Ready(&GuardType) < 0 ||
      PyType_Ready(&IntervalType) < 0 || PyType_Ready(&CoreType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&module);
  if (m == nullptr) return nullptr;
  Py_INCREF(&CoreType);
  PyModule_AddObject(m, "Core", (PyObject*)&CoreType);
  Py_INCREF(&HandleType);
  PyModule_AddObject(m, "StateHandle", (PyObject*)&HandleType);
  return m;
}
