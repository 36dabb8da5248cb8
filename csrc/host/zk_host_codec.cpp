// zkmi host codec — native Jute encode/decode for the interactive path.
//
// CPython extension (no torch headers) used by zkmi/codec.py.  It mirrors the
// pure-Python oracle zkmi/jute.py exactly (same dict keys, same Stat
// objects, same errors) and is checked against it in
// tests/test_host_codec.py.  Reference parity: lib/jute-buffer.js (Jute
// primitives), lib/zk-buffer.js:97-370 (request encode, reply decode),
// lib/zk-streams.js:39-65 (framing; here one pass over a chunk, no
// per-packet memmove).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <cstdint>
#include <cstring>
#include <string>

namespace {

PyObject* g_stat_cls = nullptr;     // zkmi.jute.Stat
// the byte offsets of Stat's 11 __slots__ in field order (init): replies
// build their Stat by filling the slots (g_stat_fast)
Py_ssize_t g_stat_off[11];
bool g_stat_fast = false;
PyObject* g_decode_err = nullptr;   // zkmi.errors.ZKDecodeError

// -- interned names -----------------------------------------------------------
struct Names {
  PyObject *xid, *zxid, *err, *opcode, *path, *data, *stat, *children, *acl,
      *type, *state, *watch, *version, *flags, *perms, *id, *scheme, *relZxid,
      *events, *dataChanged, *createdOrDestroyed, *childrenChanged;
} N;

struct Code { int32_t code; const char* name; PyObject* obj; };

Code g_ops[] = {
    {0, "NOTIFICATION", nullptr}, {1, "CREATE", nullptr},
    {2, "DELETE", nullptr}, {3, "EXISTS", nullptr}, {4, "GET_DATA", nullptr},
    {5, "SET_DATA", nullptr}, {6, "GET_ACL", nullptr}, {7, "SET_ACL", nullptr},
    {8, "GET_CHILDREN", nullptr}, {9, "SYNC", nullptr}, {11, "PING", nullptr},
    {12, "GET_CHILDREN2", nullptr}, {13, "CHECK", nullptr},
    {14, "MULTI", nullptr}, {100, "AUTH", nullptr},
    {101, "SET_WATCHES", nullptr}, {102, "SASL", nullptr},
    {-10, "CREATE_SESSION", nullptr}, {-11, "CLOSE_SESSION", nullptr},
    {-1, "ERROR", nullptr}};

Code g_errs[] = {
    {0, "OK", nullptr}, {-1, "SYSTEM_ERROR", nullptr},
    {-2, "RUNTIME_INCONSISTENCY", nullptr}, {-3, "DATA_INCONSISTENCY", nullptr},
    {-4, "CONNECTION_LOSS", nullptr}, {-5, "MARSHALLING_ERROR", nullptr},
    {-6, "UNIMPLEMENTED", nullptr}, {-7, "OPERATION_TIMEOUT", nullptr},
    {-8, "BAD_ARGUMENTS", nullptr}, {-100, "API_ERROR", nullptr},
    {-101, "NO_NODE", nullptr}, {-102, "NO_AUTH", nullptr},
    {-103, "BAD_VERSION", nullptr}, {-108, "NO_CHILDREN_FOR_EPHEMERALS", nullptr},
    {-110, "NODE_EXISTS", nullptr}, {-111, "NOT_EMPTY", nullptr},
    {-112, "SESSION_EXPIRED", nullptr}, {-113, "INVALID_CALLBACK", nullptr},
    {-114, "INVALID_ACL", nullptr}, {-115, "AUTH_FAILED", nullptr}};

Code g_ntypes[] = {{1, "CREATED", nullptr}, {2, "DELETED", nullptr},
                   {3, "DATA_CHANGED", nullptr},
                   {4, "CHILDREN_CHANGED", nullptr}};

Code g_states[] = {{0, "DISCONNECTED", nullptr}, {3, "SYNC_CONNECTED", nullptr},
                   {4, "AUTH_FAILED", nullptr},
                   {5, "CONNECTED_READ_ONLY", nullptr},
                   {6, "SASL_AUTHENTICATED", nullptr},
                   {-122, "EXPIRED", nullptr}};

Code g_perms[] = {{1, "READ", nullptr}, {2, "WRITE", nullptr},
                  {4, "CREATE", nullptr}, {8, "DELETE", nullptr},
                  {16, "ADMIN", nullptr}};

template <size_t K>
PyObject* name_of(Code (&t)[K], int32_t c) {      // new reference
  for (auto& e : t)
    if (e.code == c) { Py_INCREF(e.obj); return e.obj; }
  return PyLong_FromLong(c);
}

template <size_t K>
bool code_of(Code (&t)[K], const char* s, int32_t* out) {
  for (auto& e : t)
    if (strcmp(e.name, s) == 0) { *out = e.code; return true; }
  return false;
}

// -- reader -------------------------------------------------------------------
struct Reader {
  const uint8_t* p;
  Py_ssize_t off, end;
  bool fail(const char* what) {
    PyErr_Format(g_decode_err, "read of %s at offset %zd overruns record of "
                 "%zd bytes", what, off, end);
    return false;
  }
  bool i32(int32_t* v) {
    if (off + 4 > end) return fail("i32");
    uint32_t x; memcpy(&x, p + off, 4);
    *v = (int32_t)__builtin_bswap32(x);
    off += 4;
    return true;
  }
  bool i64(int64_t* v) {
    if (off + 8 > end) return fail("i64");
    uint64_t x; memcpy(&x, p + off, 8);
    *v = (int64_t)__builtin_bswap64(x);
    off += 8;
    return true;
  }
  bool buf(const uint8_t** s, Py_ssize_t* n) {
    int32_t l;
    if (!i32(&l)) return false;
    if (l < 0) l = 0;
    if (off + l > end) return fail("buffer");
    *s = p + off;
    *n = l;
    off += l;
    return true;
  }
  PyObject* bytes() {
    const uint8_t* s; Py_ssize_t n;
    if (!buf(&s, &n)) return nullptr;
    return PyBytes_FromStringAndSize((const char*)s, n);
  }
  PyObject* ustr() {
    const uint8_t* s; Py_ssize_t n;
    if (!buf(&s, &n)) return nullptr;
    PyObject* r = PyUnicode_DecodeUTF8((const char*)s, n, "strict");
    if (!r) {
      PyErr_Clear();
      PyErr_SetString(g_decode_err, "invalid utf-8 in string");
    }
    return r;
  }
  PyObject* stat() {
    int64_t cz, mz, ct, mt, eo, pz;
    int32_t v, cv, av, dl, nc;
    if (!(i64(&cz) && i64(&mz) && i64(&ct) && i64(&mt) && i32(&v) &&
          i32(&cv) && i32(&av) && i64(&eo) && i32(&dl) && i32(&nc) &&
          i64(&pz)))
      return nullptr;
    if (g_stat_fast) {
      // the Stat's slots filled straight from here: no argument tuple and
      // no Python __init__ frame (one per reply on the interactive path)
      PyTypeObject* tp = (PyTypeObject*)g_stat_cls;
      PyObject* o = tp->tp_alloc(tp, 0);
      if (o == nullptr) return nullptr;
      const long long f[11] = {cz, mz, ct, mt, v, cv, av, eo, dl, nc, pz};
      for (int k = 0; k < 11; ++k) {
        PyObject* x = PyLong_FromLongLong(f[k]);
        if (x == nullptr) { Py_DECREF(o); return nullptr; }
        *(PyObject**)((char*)o + g_stat_off[k]) = x;
      }
      return o;
    }
    return PyObject_CallFunction(g_stat_cls, "LLLLiiiLiiL", (long long)cz,
                                 (long long)mz, (long long)ct, (long long)mt,
                                 v, cv, av, (long long)eo, dl, nc,
                                 (long long)pz);
  }
  PyObject* strvec() {
    int32_t n;
    if (!i32(&n)) return nullptr;
    if (n < 0) n = 0;
    PyObject* l = PyList_New(0);
    for (int32_t k = 0; k < n; ++k) {
      PyObject* s = ustr();
      if (!s) { Py_DECREF(l); return nullptr; }
      PyList_Append(l, s);
      Py_DECREF(s);
    }
    return l;
  }
  PyObject* perms() {
    int32_t v;
    if (!i32(&v)) return nullptr;
    PyObject* l = PyList_New(0);
    for (auto& e : g_perms)
      if (v & e.code) PyList_Append(l, e.obj);
    return l;
  }
  PyObject* acl() {
    int32_t n;
    if (!i32(&n)) return nullptr;
    if (n < 0) n = 0;
    PyObject* l = PyList_New(0);
    for (int32_t k = 0; k < n; ++k) {
      PyObject* pm = perms();
      PyObject* sc = pm ? ustr() : nullptr;
      PyObject* id = sc ? ustr() : nullptr;
      if (!id) { Py_XDECREF(pm); Py_XDECREF(sc); Py_DECREF(l); return nullptr; }
      PyObject* idd = PyDict_New();
      PyDict_SetItem(idd, N.scheme, sc);
      PyDict_SetItem(idd, N.id, id);
      PyObject* ent = PyDict_New();
      PyDict_SetItem(ent, N.perms, pm);
      PyDict_SetItem(ent, N.id, idd);
      PyList_Append(l, ent);
      Py_DECREF(pm); Py_DECREF(sc); Py_DECREF(id); Py_DECREF(idd);
      Py_DECREF(ent);
    }
    return l;
  }
};

bool set_steal(PyObject* d, PyObject* k, PyObject* v) {
  if (!v) return false;
  PyDict_SetItem(d, k, v);
  Py_DECREF(v);
  return true;
}

// One reply body -> dict (new reference), or nullptr with the error set.
// Also reached from the native loop's reply router through the module's
// `_C_decode_reply` capsule, on bytes still in its receive buffer.
PyObject* decode_reply_raw(const uint8_t* body, Py_ssize_t len,
                           PyObject* xmap) {
  Reader r{body, 0, len};
  PyObject* d = nullptr;
  int32_t xid, err;
  int64_t zxid;
  PyObject* op = nullptr;
  if (r.end < 16) {
    PyErr_SetString(g_decode_err, "reply shorter than its 16-byte header");
    goto fail;
  }
  r.i32(&xid); r.i64(&zxid); r.i32(&err);
  switch (xid) {
    case -1: op = g_ops[0].obj; Py_INCREF(op); break;
    case -2: op = name_of(g_ops, 11); break;
    case -4: op = name_of(g_ops, 100); break;
    case -8: op = name_of(g_ops, 101); break;
    default: {
      PyObject* k = PyLong_FromLong(xid);
      op = PyDict_GetItemWithError(xmap, k);   // borrowed
      Py_DECREF(k);
      if (op == nullptr) {
        if (!PyErr_Occurred())
          PyErr_Format(g_decode_err, "reply packet must match a request "
                       "(xid %d)", xid);
        goto fail;
      }
      Py_INCREF(op);
    }
  }
  d = PyDict_New();
  set_steal(d, N.xid, PyLong_FromLong(xid));
  set_steal(d, N.zxid, PyLong_FromLongLong(zxid));
  set_steal(d, N.err, name_of(g_errs, err));
  PyDict_SetItem(d, N.opcode, op);
  if (err == 0) {
    const char* o = PyUnicode_AsUTF8(op);
    if (!o) goto fail;
    bool ok = true;
    if (!strcmp(o, "GET_CHILDREN") || !strcmp(o, "GET_CHILDREN2")) {
      ok = set_steal(d, N.children, r.strvec());
      if (ok && o[12] == '2') ok = set_steal(d, N.stat, r.stat());
    } else if (!strcmp(o, "CREATE")) {
      ok = set_steal(d, N.path, r.ustr());
    } else if (!strcmp(o, "EXISTS") || !strcmp(o, "SET_DATA")) {
      ok = set_steal(d, N.stat, r.stat());
    } else if (!strcmp(o, "GET_ACL")) {
      ok = set_steal(d, N.acl, r.acl()) && set_steal(d, N.stat, r.stat());
    } else if (!strcmp(o, "GET_DATA")) {
      ok = set_steal(d, N.data, r.bytes()) && set_steal(d, N.stat, r.stat());
    } else if (!strcmp(o, "NOTIFICATION")) {
      int32_t t, s;
      ok = r.i32(&t) && r.i32(&s);
      if (ok) {
        set_steal(d, N.type, name_of(g_ntypes, t));
        set_steal(d, N.state, name_of(g_states, s));
        ok = set_steal(d, N.path, r.ustr());
      }
    } else if (!strcmp(o, "SET_WATCHES") || !strcmp(o, "PING") ||
               !strcmp(o, "SYNC") || !strcmp(o, "DELETE") ||
               !strcmp(o, "CLOSE_SESSION") || !strcmp(o, "AUTH")) {
    } else {
      PyErr_Format(g_decode_err, "Unsupported opcode %s", o);
      ok = false;
    }
    if (!ok) goto fail;
  }
  Py_DECREF(op);
  return d;
fail:
  Py_XDECREF(op);
  Py_XDECREF(d);
  return nullptr;
}

PyObject* decode_response(PyObject*, PyObject* args) {
  Py_buffer view;
  PyObject* xmap;
  if (!PyArg_ParseTuple(args, "y*O", &view, &xmap)) return nullptr;
  PyObject* d = decode_reply_raw((const uint8_t*)view.buf, view.len, xmap);
  PyBuffer_Release(&view);
  return d;
}

// -- writer -------------------------------------------------------------------
struct Writer {
  std::string s;
  void i32(int32_t v) {
    uint32_t x = __builtin_bswap32((uint32_t)v);
    s.append((const char*)&x, 4);
  }
  void i64(int64_t v) {
    uint64_t x = __builtin_bswap64((uint64_t)v);
    s.append((const char*)&x, 8);
  }
  void buf(const char* p, Py_ssize_t n) {
    if (n == 0) { i32(-1); return; }          // jute-buffer.js:127-130
    i32((int32_t)n);
    s.append(p, n);
  }
  bool ustr(PyObject* o) {
    Py_ssize_t n;
    const char* p = PyUnicode_AsUTF8AndSize(o, &n);
    if (!p) return false;
    buf(p, n);
    return true;
  }
  bool bytes(PyObject* o) {
    if (o == nullptr || o == Py_None) { buf("", 0); return true; }
    Py_buffer v;
    if (PyObject_GetBuffer(o, &v, PyBUF_SIMPLE) < 0) return false;
    buf((const char*)v.buf, v.len);
    PyBuffer_Release(&v);
    return true;
  }
};

PyObject* get(PyObject* d, PyObject* k) {        // borrowed or nullptr
  return PyDict_GetItemWithError(d, k);
}

bool mask_from(PyObject* o, Code* tbl, size_t n, bool upper, int32_t* out) {
  if (o == nullptr || o == Py_None) { *out = 0; return true; }
  if (PyLong_Check(o)) { *out = (int32_t)PyLong_AsLong(o); return true; }
  int32_t m = 0;
  PyObject* it = PyObject_GetIter(o);
  if (!it) return false;
  PyObject* x;
  while ((x = PyIter_Next(it))) {
    const char* s = PyUnicode_AsUTF8(x);
    if (!s) { Py_DECREF(x); Py_DECREF(it); return false; }
    std::string k(s);
    if (upper) for (auto& c : k) c = (char)toupper(c);
    bool found = false;
    for (size_t i = 0; i < n; ++i)
      if (k == tbl[i].name) { m |= tbl[i].code; found = true; }
    if (!found) {
      PyErr_Format(PyExc_ValueError, "unknown %s %R",
                   upper ? "permission" : "flag", x);
      Py_DECREF(x); Py_DECREF(it);
      return false;
    }
    Py_DECREF(x);
  }
  Py_DECREF(it);
  if (PyErr_Occurred()) return false;
  *out = m;
  return true;
}

Code g_flags[] = {{1, "EPHEMERAL", nullptr}, {2, "SEQUENTIAL", nullptr}};

bool write_acl(Writer& w, PyObject* acl) {
  if (acl == nullptr || acl == Py_None) { w.i32(0); return true; }
  Py_ssize_t n = PySequence_Size(acl);
  if (n < 0) return false;
  w.i32((int32_t)n);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* e = PySequence_GetItem(acl, i);
    if (!e) return false;
    int32_t m;
    PyObject* idd = get(e, N.id);
    bool ok = mask_from(get(e, N.perms), g_perms, 5, true, &m);
    if (ok) {
      w.i32(m);
      ok = idd && w.ustr(get(idd, N.scheme)) && w.ustr(get(idd, N.id));
    }
    Py_DECREF(e);
    if (!ok) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_KeyError, "acl id");
      return false;
    }
  }
  return true;
}

bool write_vec(Writer& w, PyObject* v) {
  if (v == nullptr || v == Py_None) { w.i32(0); return true; }
  Py_ssize_t n = PySequence_Size(v);
  if (n < 0) return false;
  w.i32((int32_t)n);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* s = PySequence_GetItem(v, i);
    bool ok = s && w.ustr(s);
    Py_XDECREF(s);
    if (!ok) return false;
  }
  return true;
}

long as_long(PyObject* o, long dflt) {
  if (o == nullptr || o == Py_None) return dflt;
  return PyLong_AsLong(o);
}

// Encode one request dict, appending it to `out` (with its 4-byte length
// prefix when `framed`).  False with the error set on a bad packet (`out`
// is then left as it was).  Also reached from the native loop's request
// path through the module's `_C_encode_request` capsule.
bool encode_request_into(PyObject* d, std::string* out, bool framed) {
  if (!PyDict_Check(d)) {
    PyErr_SetString(PyExc_TypeError, "packet must be a dict");
    return false;
  }
  PyObject* opo = get(d, N.opcode);
  PyObject* xo = get(d, N.xid);
  if (!opo || !xo) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_KeyError, "opcode/xid");
    return false;
  }
  const char* op = PyUnicode_AsUTF8(opo);
  if (!op) return false;
  int32_t code;
  if (!code_of(g_ops, op, &code)) {
    PyErr_Format(PyExc_ValueError, "Unsupported opcode %s", op);
    return false;
  }
  const size_t base = out->size();
  Writer w;
  w.s.swap(*out);
  if (framed) w.i32(0);                  // length, patched below
  w.i32((int32_t)PyLong_AsLong(xo));
  w.i32(code);
  bool ok = true;
  switch (code) {
    case 8: case 12: case 4: case 3:                 // children, data, exists
      ok = w.ustr(get(d, N.path));
      if (ok) {
        PyObject* wt = get(d, N.watch);
        w.s.push_back((wt && PyObject_IsTrue(wt)) ? 1 : 0);
      }
      break;
    case 1: {                                        // CREATE
      int32_t fl;
      ok = w.ustr(get(d, N.path)) && w.bytes(get(d, N.data)) &&
           write_acl(w, get(d, N.acl)) &&
           mask_from(get(d, N.flags), g_flags, 2, false, &fl);
      if (ok) w.i32(fl);
      break;
    }
    case 2:                                          // DELETE
      ok = w.ustr(get(d, N.path));
      if (ok) w.i32((int32_t)as_long(get(d, N.version), 0));
      break;
    case 6: case 9:                                  // GET_ACL, SYNC
      ok = w.ustr(get(d, N.path));
      break;
    case 5:                                          // SET_DATA
      ok = w.ustr(get(d, N.path)) && w.bytes(get(d, N.data));
      if (ok) w.i32((int32_t)as_long(get(d, N.version), -1));
      break;
    case 101: {                                      // SET_WATCHES
      PyObject* ev = get(d, N.events);
      w.i64((int64_t)PyLong_AsLongLong(get(d, N.relZxid)));
      ok = ev && write_vec(w, get(ev, N.dataChanged)) &&
           write_vec(w, get(ev, N.createdOrDestroyed)) &&
           write_vec(w, get(ev, N.childrenChanged));
      break;
    }
    case 11: case -11:                               // PING, CLOSE_SESSION
      break;
    default:
      PyErr_Format(PyExc_ValueError, "Unsupported opcode %s", op);
      ok = false;
  }
  w.s.swap(*out);
  if (!ok || PyErr_Occurred()) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_KeyError, "packet field");
    out->resize(base);
    return false;
  }
  if (framed) {
    const uint32_t n = __builtin_bswap32((uint32_t)(out->size() - base - 4));
    memcpy(&(*out)[base], &n, 4);
  }
  return true;
}

PyObject* encode_request(PyObject*, PyObject* arg) {
  std::string s;
  s.reserve(64);
  if (!encode_request_into(arg, &s, false)) return nullptr;
  return PyBytes_FromStringAndSize(s.data(), (Py_ssize_t)s.size());
}

PyObject* frame(PyObject*, PyObject* arg) {
  Py_buffer v;
  if (PyObject_GetBuffer(arg, &v, PyBUF_SIMPLE) < 0) return nullptr;
  PyObject* out = PyBytes_FromStringAndSize(nullptr, v.len + 4);
  char* p = PyBytes_AS_STRING(out);
  uint32_t n = __builtin_bswap32((uint32_t)v.len);
  memcpy(p, &n, 4);
  memcpy(p + 4, v.buf, v.len);
  PyBuffer_Release(&v);
  return out;
}

// scan_frames(buf, start=0, end=None, max_packet=16MiB)
//   -> (list[(body_off, body_len)], consumed, bad_at)
PyObject* scan_frames(PyObject*, PyObject* args) {
  Py_buffer v;
  Py_ssize_t start = 0;
  PyObject* endo = Py_None;
  long long maxp = 16 * 1024 * 1024;
  if (!PyArg_ParseTuple(args, "y*|nOL", &v, &start, &endo, &maxp))
    return nullptr;
  Py_ssize_t end = (endo == Py_None) ? v.len : PyLong_AsSsize_t(endo);
  const uint8_t* p = (const uint8_t*)v.buf;
  PyObject* frames = PyList_New(0);
  Py_ssize_t off = start, bad = -1;
  while (end - off >= 4) {
    uint32_t x; memcpy(&x, p + off, 4);
    const int32_t n = (int32_t)__builtin_bswap32(x);
    if (n < 0 || (long long)n > maxp) { bad = off; break; }
    if (end - off - 4 < n) break;
    PyObject* t = Py_BuildValue("(nn)", off + 4, (Py_ssize_t)n);
    PyList_Append(frames, t);
    Py_DECREF(t);
    off += 4 + n;
  }
  PyBuffer_Release(&v);
  return Py_BuildValue("(Nnn)", frames, off, bad);
}

PyObject* init(PyObject*, PyObject* args) {
  PyObject *stat, *derr = nullptr;
  if (!PyArg_ParseTuple(args, "O|O", &stat, &derr)) return nullptr;
  Py_XDECREF(g_stat_cls);
  Py_INCREF(stat);
  g_stat_cls = stat;
  static const char* fields[11] = {
      "czxid", "mzxid", "ctime", "mtime", "version", "cversion", "aversion",
      "ephemeralOwner", "dataLength", "numChildren", "pzxid"};
  g_stat_fast = PyType_Check(stat);
  for (int k = 0; k < 11 && g_stat_fast; ++k) {
    PyObject* d = PyObject_GetAttrString(stat, fields[k]);
    if (d == nullptr) { PyErr_Clear(); g_stat_fast = false; break; }
    if (Py_TYPE(d) == &PyMemberDescr_Type &&
        ((PyMemberDescrObject*)d)->d_member->type == T_OBJECT_EX)
      g_stat_off[k] = ((PyMemberDescrObject*)d)->d_member->offset;
    else
      g_stat_fast = false;
    Py_DECREF(d);
  }
  if (derr) {
    Py_XDECREF(g_decode_err);
    Py_INCREF(derr);
    g_decode_err = derr;
  }
  Py_RETURN_NONE;
}

PyMethodDef methods[] = {
    {"init", init, METH_VARARGS, "init(StatClass, DecodeError)"},
    {"encode_request", encode_request, METH_O, "request dict -> body bytes"},
    {"decode_response", decode_response, METH_VARARGS,
     "decode_response(body, xid_map) -> dict"},
    {"scan_frames", scan_frames, METH_VARARGS,
     "scan_frames(buf, start, end, max_packet) -> (frames, consumed, bad)"},
    {"frame", frame, METH_O, "length-prefix a record"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_zkhost",
                   "zkmi native host codec", -1, methods};

template <size_t K>
void intern(Code (&t)[K]) {
  for (auto& e : t) e.obj = PyUnicode_InternFromString(e.name);
}

}  // namespace

PyMODINIT_FUNC PyInit__zkhost(void) {
#define I(x) N.x = PyUnicode_InternFromString(#x)
  I(xid); I(zxid); I(err); I(opcode); I(path); I(data); I(stat);
  I(children); I(acl); I(type); I(state); I(watch); I(version); I(flags);
  I(perms); I(id); I(scheme); I(relZxid); I(events); I(dataChanged);
  I(createdOrDestroyed); I(childrenChanged);
#undef I
  intern(g_ops); intern(g_errs); intern(g_ntypes); intern(g_states);
  intern(g_perms); intern(g_flags);
  g_decode_err = PyExc_ValueError;
  Py_INCREF(g_decode_err);
  PyObject* m = PyModule_Create(&mod);
  if (m == nullptr) return nullptr;
  // C entry point for the native loop (csrc/host/zk_loop.cpp, Router)
  PyObject* cap = PyCapsule_New((void*)&decode_reply_raw,
                                "zkmi._zkhost.decode_reply_raw", nullptr);
  if (cap == nullptr || PyModule_AddObject(m, "_C_decode_reply", cap) < 0) {
    Py_XDECREF(cap);
    Py_DECREF(m);
    return nullptr;
  }
  PyObject* cap2 = PyCapsule_New((void*)&encode_request_into,
                                 "zkmi._zkhost.encode_request_into", nullptr);
  if (cap2 == nullptr || PyModule_AddObject(m, "_C_encode_request", cap2) < 0) {
    Py_XDECREF(cap2);
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
