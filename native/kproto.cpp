// _kproto: native JSON-dict <-> Kubernetes protobuf transcoder for the apiserver.
//
// The reference serves `application/vnd.kubernetes.protobuf` from gogo-generated marshalers
// (staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:88 Decode,
// :171 Encode). amdkube's objects are Python dicts (the JSON form), so the cost that matters is
// dict -> wire bytes and wire bytes -> dict. This module does both directly over the CPython
// API from a flat schema table that api/protobuf.py derives from the wire table
// (api/proto/k8s_wire.json): no intermediate message objects, one pass per direction.
//
//   init(table, proto_error, enc_cb, dec_cb)   table: [(special, [(num, key|None, kind, stype, ktype, sub)...])]
//   encode(obj, msg, strict) -> (bytes, lossless)
//   decode(buf, msg) -> dict
//   envelope_parts(buf) -> (apiVersion, kind, raw, contentType) | None     (runtime.Unknown after k8s\0)
//   splice_list(apiVersion, listKind, rv, [stored...]) -> bytes | None      (<Kind>List from stored envelopes)
//
// Field kinds and the JSON conventions (Time as RFC 3339, Quantity as string, IntOrString as
// int|string, bytes as base64, inlined Go structs flattened into the parent object) follow
// api/protobuf.py, which keeps a pure-Python path for the rare types handled by callback
// (Duration, RawExtension, JSON Schema props). `strict` reports whether the object would come
// back unchanged from a decode (no unknown keys, no type coercion, canonical times), which is
// what the storage layer needs to decide between protobuf and JSON storage.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

enum Kind : uint8_t { SCALAR = 0, MSG = 1, REP_SCALAR = 2, REP_MSG = 3, MAP_SCALAR = 4, MAP_MSG = 5, INLINE = 6 };
// FieldDescriptorProto.Type
enum SType : uint8_t {
  T_DOUBLE = 1, T_FLOAT = 2, T_INT64 = 3, T_UINT64 = 4, T_INT32 = 5, T_FIXED64 = 6, T_FIXED32 = 7, T_BOOL = 8,
  T_STRING = 9, T_MESSAGE = 11, T_BYTES = 12, T_UINT32 = 13, T_ENUM = 14, T_SFIXED32 = 15, T_SFIXED64 = 16,
  T_SINT32 = 17, T_SINT64 = 18
};
enum Special : int { SP_NONE = 0, SP_TIME = 1, SP_MICROTIME = 2, SP_QUANTITY = 3, SP_INTORSTR = 4, SP_LISTWRAP = 5,
                     SP_CALLBACK = 9 };

struct Field {
  uint32_t num;
  PyObject* key;  // interned str; nullptr for INLINE
  uint8_t kind, stype, ktype;
  int32_t sub;
};

struct Msg {
  int special = 0;
  std::vector<Field> fields;         // ascending field number
  std::vector<int16_t> by_num;       // field number -> index into fields (-1: unknown)
  PyObject* keys = nullptr;          // frozenset of JSON keys this message consumes (incl. inlined)
};

std::vector<Msg> g_msgs;
PyObject* g_err = nullptr;      // api.protobuf.ProtoError
PyObject* g_enc_cb = nullptr;   // (msg, value) -> (bytes, lossless)
PyObject* g_dec_cb = nullptr;   // (msg, bytes) -> object
PyObject* g_b64enc = nullptr;   // binascii.b2a_base64
PyObject* g_b64dec = nullptr;   // binascii.a2b_base64
PyObject* g_s_apiVersion = nullptr;
PyObject* g_s_kind = nullptr;

// ------------------------------------------------------------------------------ writer
struct Out {
  std::string b;
  void byte(uint8_t c) { b.push_back(static_cast<char>(c)); }
  void varint(uint64_t v) {
    char tmp[10];
    int n = 0;
    while (v >= 0x80) { tmp[n++] = static_cast<char>((v & 0x7f) | 0x80); v >>= 7; }
    tmp[n++] = static_cast<char>(v);
    b.append(tmp, n);
  }
  void tag(uint32_t num, int wt) { varint((uint64_t(num) << 3) | wt); }
  void fixed32(uint32_t v) { char t[4]; std::memcpy(t, &v, 4); b.append(t, 4); }
  void fixed64(uint64_t v) { char t[8]; std::memcpy(t, &v, 8); b.append(t, 8); }
  void bytes(uint32_t num, const char* p, size_t n) { tag(num, 2); varint(n); b.append(p, n); }
  // length-delimited child: reserve one length byte, write the child, widen if needed
  size_t open(uint32_t num) { tag(num, 2); b.push_back(0); return b.size(); }
  void close(size_t start) {
    size_t len = b.size() - start;
    if (len < 0x80) { b[start - 1] = static_cast<char>(len); return; }
    char tmp[10];
    int n = 0;
    uint64_t v = len;
    while (v >= 0x80) { tmp[n++] = static_cast<char>((v & 0x7f) | 0x80); v >>= 7; }
    tmp[n++] = static_cast<char>(v);
    b.insert(start, static_cast<size_t>(n - 1), '\0');
    std::memcpy(&b[start - 1], tmp, n);
  }
};

struct Ctx {
  bool strict;
  bool lossless = true;
};

int fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  PyObject* s = PyUnicode_FromFormatV(fmt, ap);
  va_end(ap);
  if (s) { PyErr_SetObject(g_err, s); Py_DECREF(s); }
  return -1;
}

// ------------------------------------------------------------------------------ time
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + static_cast<int64_t>(doe) - 719468;
}

void civil_from_days(int64_t z, int64_t& y, unsigned& m, unsigned& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = static_cast<unsigned>(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = static_cast<int64_t>(yoe) + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp + (mp < 10 ? 3 : -9);
  y += m <= 2;
}

bool digits(const char* s, int n, int& v) {
  v = 0;
  for (int i = 0; i < n; i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
  }
  return true;
}

// YYYY-MM-DDTHH:MM:SS(.frac)?(Z|+HH:MM|-HH:MM)
bool parse_rfc3339(const char* s, Py_ssize_t n, int64_t& secs, int32_t& nanos) {
  if (n < 20 || s[4] != '-' || s[7] != '-' || s[10] != 'T' || s[13] != ':' || s[16] != ':') return false;
  int Y, M, D, h, mi, se;
  if (!digits(s, 4, Y) || !digits(s + 5, 2, M) || !digits(s + 8, 2, D) || !digits(s + 11, 2, h) ||
      !digits(s + 14, 2, mi) || !digits(s + 17, 2, se))
    return false;
  if (M < 1 || M > 12 || D < 1 || D > 31 || h > 23 || mi > 59 || se > 60) return false;
  Py_ssize_t i = 19;
  nanos = 0;
  if (i < n && s[i] == '.') {
    i++;
    int nd = 0;
    int64_t f = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') {
      if (nd < 9) { f = f * 10 + (s[i] - '0'); nd++; }
      i++;
    }
    if (nd == 0) return false;
    while (nd < 9) { f *= 10; nd++; }
    nanos = static_cast<int32_t>(f);
  }
  int64_t off = 0;
  if (i < n && s[i] == 'Z') {
    i++;
  } else if (i + 6 == n && (s[i] == '+' || s[i] == '-') && s[i + 3] == ':') {
    int oh, om;
    if (!digits(s + i + 1, 2, oh) || !digits(s + i + 4, 2, om)) return false;
    off = (s[i] == '+' ? 1 : -1) * (oh * 3600 + om * 60);
    i += 6;
  } else {
    return false;
  }
  if (i != n) return false;
  secs = days_from_civil(Y, M, D) * 86400 + h * 3600 + mi * 60 + se - off;
  return true;
}

PyObject* format_time(int64_t secs, int32_t nanos, bool micro) {
  int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
  int64_t rem = secs - days * 86400;
  int64_t y;
  unsigned m, d;
  civil_from_days(days, y, m, d);
  char buf[64];
  int n;
  if (micro)
    n = snprintf(buf, sizeof buf, "%04lld-%02u-%02uT%02d:%02d:%02d.%06dZ", static_cast<long long>(y), m, d,
                 static_cast<int>(rem / 3600), static_cast<int>(rem / 60 % 60), static_cast<int>(rem % 60),
                 static_cast<int>(nanos / 1000));
  else
    n = snprintf(buf, sizeof buf, "%04lld-%02u-%02uT%02d:%02d:%02dZ", static_cast<long long>(y), m, d,
                 static_cast<int>(rem / 3600), static_cast<int>(rem / 60 % 60), static_cast<int>(rem % 60));
  return PyUnicode_FromStringAndSize(buf, n);
}

// ------------------------------------------------------------------------------ encode
int encode_msg(Out& o, PyObject* d, int mi, Ctx& c, bool top, bool check_keys = true);

// one scalar value (no tag) of type t
int put_scalar(Out& o, uint32_t num, uint8_t t, PyObject* v, Ctx& c) {
  switch (t) {
    case T_STRING: {
      PyObject* s = v;
      PyObject* tmp = nullptr;
      if (!PyUnicode_Check(v)) {
        c.lossless = false;
        tmp = s = PyObject_Str(v);
        if (!s) return -1;
      }
      Py_ssize_t n;
      const char* p = PyUnicode_AsUTF8AndSize(s, &n);
      if (!p) { Py_XDECREF(tmp); return -1; }
      o.bytes(num, p, static_cast<size_t>(n));
      Py_XDECREF(tmp);
      return 0;
    }
    case T_BYTES: {
      if (PyBytes_Check(v)) {
        c.lossless = false;
        o.bytes(num, PyBytes_AS_STRING(v), PyBytes_GET_SIZE(v));
        return 0;
      }
      if (!PyUnicode_Check(v)) return fail("bytes field wants a base64 string, got %s", Py_TYPE(v)->tp_name);
      PyObject* raw = PyObject_CallOneArg(g_b64dec, v);
      if (!raw) { PyErr_Clear(); return fail("invalid base64 in a bytes field"); }
      if (c.strict) {   // canonical base64 only: it must come back identical
        PyObject* back = PyObject_CallFunction(g_b64enc, "O", raw);
        if (!back) { Py_DECREF(raw); return -1; }
        Py_ssize_t bn = PyBytes_GET_SIZE(back);
        const char* bp = PyBytes_AS_STRING(back);
        if (bn > 0 && bp[bn - 1] == '\n') bn--;
        Py_ssize_t sn;
        const char* sp = PyUnicode_AsUTF8AndSize(v, &sn);
        if (!sp || sn != bn || std::memcmp(sp, bp, bn) != 0) c.lossless = false;
        Py_DECREF(back);
      }
      o.bytes(num, PyBytes_AS_STRING(raw), PyBytes_GET_SIZE(raw));
      Py_DECREF(raw);
      return 0;
    }
    case T_BOOL: {
      if (!PyBool_Check(v)) c.lossless = false;
      int b = PyObject_IsTrue(v);
      if (b < 0) return -1;
      o.tag(num, 0);
      o.byte(static_cast<uint8_t>(b));
      return 0;
    }
    case T_DOUBLE:
    case T_FLOAT: {
      if (!PyFloat_Check(v) && !(PyLong_Check(v) && !PyBool_Check(v))) c.lossless = false;
      double x = PyFloat_AsDouble(v);
      if (x == -1.0 && PyErr_Occurred()) {
        PyErr_Clear();
        PyObject* f = PyNumber_Float(v);
        if (!f) { PyErr_Clear(); return fail("cannot convert %R to a number", v); }
        x = PyFloat_AS_DOUBLE(f);
        Py_DECREF(f);
      }
      if (t == T_DOUBLE) { o.tag(num, 1); uint64_t u; std::memcpy(&u, &x, 8); o.fixed64(u); }
      else { o.tag(num, 5); float fl = static_cast<float>(x); uint32_t u; std::memcpy(&u, &fl, 4); o.fixed32(u); }
      return 0;
    }
    default: {  // integers
      int64_t x;
      if (PyLong_Check(v)) {
        if (PyBool_Check(v)) c.lossless = false;
        int overflow = 0;
        long long ll = PyLong_AsLongLongAndOverflow(v, &overflow);
        if (overflow) {
          if (t == T_UINT64 || t == T_FIXED64) {
            unsigned long long u = PyLong_AsUnsignedLongLong(v);
            if (PyErr_Occurred()) return -1;
            ll = static_cast<long long>(u);
          } else {
            return fail("integer %R out of range", v);
          }
        } else if (ll == -1 && PyErr_Occurred()) {
          return -1;
        }
        x = ll;
      } else {
        c.lossless = false;
        PyObject* n = PyNumber_Long(v);
        if (!n) { PyErr_Clear(); return fail("cannot convert %R to an integer", v); }
        x = PyLong_AsLongLong(n);
        Py_DECREF(n);
        if (x == -1 && PyErr_Occurred()) return -1;
      }
      if ((t == T_INT32 || t == T_ENUM || t == T_SINT32 || t == T_SFIXED32) && (x < INT32_MIN || x > INT32_MAX))
        return fail("value %R out of range for a 32-bit field", v);
      if ((t == T_UINT32 || t == T_FIXED32) && (x < 0 || x > static_cast<int64_t>(UINT32_MAX)))
        return fail("value %R out of range for an unsigned 32-bit field", v);
      switch (t) {
        case T_INT32: case T_ENUM: o.tag(num, 0); o.varint(static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(x)))); break;
        case T_UINT32: o.tag(num, 0); o.varint(static_cast<uint32_t>(x)); break;
        case T_SINT32: { int32_t y = static_cast<int32_t>(x); o.tag(num, 0); o.varint(static_cast<uint32_t>((y << 1) ^ (y >> 31))); break; }
        case T_SINT64: o.tag(num, 0); o.varint((static_cast<uint64_t>(x) << 1) ^ static_cast<uint64_t>(x >> 63)); break;
        case T_FIXED32: case T_SFIXED32: o.tag(num, 5); o.fixed32(static_cast<uint32_t>(x)); break;
        case T_FIXED64: case T_SFIXED64: o.tag(num, 1); o.fixed64(static_cast<uint64_t>(x)); break;
        default: o.tag(num, 0); o.varint(static_cast<uint64_t>(x)); break;
      }
      return 0;
    }
  }
}

// a message-typed value under field `num` (handles the special JSON forms)
int put_msg(Out& o, uint32_t num, int sub, PyObject* v, Ctx& c) {
  size_t st = o.open(num);
  if (encode_msg(o, v, sub, c, false) < 0) return -1;
  o.close(st);
  return 0;
}

int encode_special(Out& o, PyObject* v, int mi, Ctx& c) {
  const Msg& m = g_msgs[mi];
  switch (m.special) {
    case SP_TIME:
    case SP_MICROTIME: {
      if (!PyUnicode_Check(v)) return fail("a time wants an RFC 3339 string, got %R", v);
      Py_ssize_t n;
      const char* s = PyUnicode_AsUTF8AndSize(v, &n);
      if (!s) return -1;
      // tolerate surrounding whitespace like the Python path (s.strip())
      while (n > 0 && (s[0] == ' ' || s[0] == '\t' || s[0] == '\n')) { s++; n--; }
      while (n > 0 && (s[n - 1] == ' ' || s[n - 1] == '\t' || s[n - 1] == '\n')) n--;
      int64_t secs;
      int32_t nanos;
      if (!parse_rfc3339(s, n, secs, nanos)) return fail("invalid RFC 3339 time %R", v);
      o.tag(1, 0); o.varint(static_cast<uint64_t>(secs));
      o.tag(2, 0); o.varint(static_cast<uint64_t>(static_cast<int64_t>(nanos)));
      if (c.strict) {
        PyObject* back = format_time(secs, nanos, m.special == SP_MICROTIME);
        if (!back) return -1;
        int eq = PyUnicode_Compare(back, v) == 0;
        Py_DECREF(back);
        if (!eq) c.lossless = false;
      }
      return 0;
    }
    case SP_QUANTITY:
      return put_scalar(o, 1, T_STRING, v, c);
    case SP_INTORSTR: {
      if (PyLong_Check(v) && !PyBool_Check(v)) {
        o.tag(1, 0); o.byte(0);
        return put_scalar(o, 2, T_INT32, v, c);
      }
      if (PyUnicode_Check(v)) {
        o.tag(1, 0); o.byte(1);
        return put_scalar(o, 3, T_STRING, v, c);
      }
      return fail("int-or-string wants an int or a string, got %R", v);
    }
    case SP_LISTWRAP: {   // JSON list <-> message{repeated string items = 1} (authentication ExtraValue)
      if (!PyList_Check(v)) return fail("expected a list, got %s", Py_TYPE(v)->tp_name);
      for (Py_ssize_t i = 0; i < PyList_GET_SIZE(v); i++)
        if (put_scalar(o, 1, T_STRING, PyList_GET_ITEM(v, i), c) < 0) return -1;
      return 0;
    }
    default: {   // SP_CALLBACK: the Python path
      PyObject* r = PyObject_CallFunction(g_enc_cb, "iO", mi, v);
      if (!r) return -1;
      PyObject* b = PyTuple_Check(r) && PyTuple_GET_SIZE(r) == 2 ? PyTuple_GET_ITEM(r, 0) : nullptr;
      if (!b || !PyBytes_Check(b)) { Py_DECREF(r); return fail("special encoder returned a bad value"); }
      o.b.append(PyBytes_AS_STRING(b), PyBytes_GET_SIZE(b));
      if (!PyObject_IsTrue(PyTuple_GET_ITEM(r, 1))) c.lossless = false;
      Py_DECREF(r);
      return 0;
    }
  }
}

bool empty_value(PyObject* v) {
  return v == Py_None || (PyList_Check(v) && PyList_GET_SIZE(v) == 0) || (PyDict_Check(v) && PyDict_GET_SIZE(v) == 0);
}

int encode_msg(Out& o, PyObject* d, int mi, Ctx& c, bool top, bool check_keys) {
  const Msg& m = g_msgs[mi];
  if (m.special) return encode_special(o, d, mi, c);
  if (!PyDict_Check(d)) return fail("expected an object, got %s", Py_TYPE(d)->tp_name);
  if (check_keys && c.strict && c.lossless && m.keys) {   // keys the schema would drop
    PyObject *k, *v;
    Py_ssize_t pos = 0;
    while (PyDict_Next(d, &pos, &k, &v)) {
      if (empty_value(v)) continue;
      int has = PySet_Contains(m.keys, k);
      if (has < 0) return -1;
      if (!has && !(top && (k == g_s_apiVersion || k == g_s_kind ||
                            PyUnicode_Compare(k, g_s_apiVersion) == 0 || PyUnicode_Compare(k, g_s_kind) == 0))) {
        c.lossless = false;
        break;
      }
    }
  }
  for (const Field& f : m.fields) {
    if (f.kind == INLINE) {   // a Go struct the JSON flattens: its keys live in this dict
      size_t st = o.open(f.num);
      size_t before = o.b.size();
      if (encode_msg(o, d, f.sub, c, false, false) < 0) return -1;
      if (o.b.size() == before) {   // nothing of it present: drop the tag and the placeholder
        size_t tl = 1;
        for (uint64_t t = (uint64_t(f.num) << 3) | 2; t >= 0x80; t >>= 7) tl++;
        o.b.resize(st - 1 - tl);
      } else {
        o.close(st);
      }
      continue;
    }
    PyObject* v = PyDict_GetItemWithError(d, f.key);
    if (!v) {
      if (PyErr_Occurred()) return -1;
      continue;
    }
    if (v == Py_None) continue;
    switch (f.kind) {
      case SCALAR:
        if (put_scalar(o, f.num, f.stype, v, c) < 0) return -1;
        break;
      case MSG:
        if (put_msg(o, f.num, f.sub, v, c) < 0) return -1;
        break;
      case REP_SCALAR:
      case REP_MSG: {
        if (!PyList_Check(v) && !PyTuple_Check(v)) return fail("field %U wants a list", f.key);
        PyObject* seq = PySequence_Fast(v, "list");
        Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
        PyObject** items = PySequence_Fast_ITEMS(seq);
        for (Py_ssize_t i = 0; i < n; i++) {
          if (items[i] == Py_None) {
            Py_DECREF(seq);
            return fail("field %U: null list item", f.key);
          }
          int r = f.kind == REP_SCALAR ? put_scalar(o, f.num, f.stype, items[i], c) : put_msg(o, f.num, f.sub, items[i], c);
          if (r < 0) { Py_DECREF(seq); return -1; }
        }
        Py_DECREF(seq);
        break;
      }
      default: {   // maps: repeated entry{key = 1, value = 2}
        if (!PyDict_Check(v)) return fail("field %U wants an object", f.key);
        PyObject *k, *x;
        Py_ssize_t pos = 0;
        while (PyDict_Next(v, &pos, &k, &x)) {
          if (x == Py_None) continue;
          size_t st = o.open(f.num);
          if (put_scalar(o, 1, f.ktype, k, c) < 0) return -1;
          int r = f.kind == MAP_SCALAR ? put_scalar(o, 2, f.stype, x, c) : put_msg(o, 2, f.sub, x, c);
          if (r < 0) return -1;
          o.close(st);
        }
      }
    }
  }
  return 0;
}

// ------------------------------------------------------------------------------ decode
struct In {
  const uint8_t* p;
  const uint8_t* e;
  bool varint(uint64_t& v) {
    v = 0;
    for (int sh = 0; sh < 64 && p < e; sh += 7) {
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << sh;
      if (!(b & 0x80)) return true;
    }
    return false;
  }
};

PyObject* decode_msg(const uint8_t* p, size_t n, int mi);

PyObject* scalar_obj(uint8_t t, uint64_t v) {
  switch (t) {
    case T_BOOL: return PyBool_FromLong(v != 0);
    case T_INT32: case T_ENUM: case T_SFIXED32: return PyLong_FromLong(static_cast<int32_t>(v));
    case T_UINT32: case T_FIXED32: return PyLong_FromUnsignedLong(static_cast<uint32_t>(v));
    case T_UINT64: case T_FIXED64: return PyLong_FromUnsignedLongLong(v);
    case T_SINT32: { uint32_t u = static_cast<uint32_t>(v); return PyLong_FromLong(static_cast<int32_t>((u >> 1) ^ (0u - (u & 1)))); }
    case T_SINT64: return PyLong_FromLongLong(static_cast<int64_t>((v >> 1) ^ (0 - (v & 1))));
    case T_DOUBLE: { double d; std::memcpy(&d, &v, 8); return PyFloat_FromDouble(d); }
    case T_FLOAT: { float f; uint32_t u = static_cast<uint32_t>(v); std::memcpy(&f, &u, 4); return PyFloat_FromDouble(f); }
    default: return PyLong_FromLongLong(static_cast<int64_t>(v));
  }
}

PyObject* ld_obj(uint8_t t, const uint8_t* p, size_t n) {   // string / bytes
  if (t == T_BYTES) {
    PyObject* raw = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(p), n);
    if (!raw) return nullptr;
    PyObject* b = PyObject_CallFunction(g_b64enc, "O", raw);   // b2a_base64 adds a newline
    Py_DECREF(raw);
    if (!b) return nullptr;
    Py_ssize_t bn = PyBytes_GET_SIZE(b);
    const char* bp = PyBytes_AS_STRING(b);
    if (bn > 0 && bp[bn - 1] == '\n') bn--;
    PyObject* s = PyUnicode_DecodeASCII(bp, bn, "strict");
    Py_DECREF(b);
    return s;
  }
  PyObject* s = PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(p), n, "strict");
  if (!s) {
    PyErr_Clear();
    s = PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(p), n, "replace");
  }
  return s;
}

// a scalar of type t at wire type wt from `in` (for a length-delimited string/bytes, p/n given)
PyObject* read_scalar(In& in, uint8_t t, int wt) {
  uint64_t v = 0;
  if (wt == 0) {
    if (!in.varint(v)) return nullptr;
  } else if (wt == 1) {
    if (in.e - in.p < 8) return nullptr;
    std::memcpy(&v, in.p, 8);
    in.p += 8;
  } else if (wt == 5) {
    if (in.e - in.p < 4) return nullptr;
    uint32_t u;
    std::memcpy(&u, in.p, 4);
    in.p += 4;
    v = u;
  } else {
    return nullptr;
  }
  return scalar_obj(t, v);
}

bool skip(In& in, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return in.varint(v);
    case 1: if (in.e - in.p < 8) return false; in.p += 8; return true;
    case 5: if (in.e - in.p < 4) return false; in.p += 4; return true;
    case 2: if (!in.varint(v) || static_cast<uint64_t>(in.e - in.p) < v) return false; in.p += v; return true;
    default: return false;
  }
}

PyObject* truncated() {
  fail("truncated or malformed protobuf message");
  return nullptr;
}

PyObject* decode_special(const uint8_t* p, size_t n, int mi) {
  const Msg& m = g_msgs[mi];
  In in{p, p + n};
  switch (m.special) {
    case SP_TIME:
    case SP_MICROTIME: {
      int64_t secs = 0;
      int32_t nanos = 0;
      while (in.p < in.e) {
        uint64_t tag;
        if (!in.varint(tag)) return truncated();
        uint64_t v;
        if ((tag & 7) == 0 && (tag >> 3) <= 2) {
          if (!in.varint(v)) return truncated();
          if ((tag >> 3) == 1) secs = static_cast<int64_t>(v); else nanos = static_cast<int32_t>(v);
        } else if (!skip(in, tag & 7)) {
          return truncated();
        }
      }
      return format_time(secs, nanos, m.special == SP_MICROTIME);
    }
    case SP_QUANTITY:
    case SP_INTORSTR:
    case SP_LISTWRAP: {
      int64_t type = 0, ival = 0;
      PyObject* str = nullptr;
      PyObject* lst = m.special == SP_LISTWRAP ? PyList_New(0) : nullptr;
      while (in.p < in.e) {
        uint64_t tag;
        if (!in.varint(tag)) { Py_XDECREF(str); Py_XDECREF(lst); return truncated(); }
        uint32_t num = static_cast<uint32_t>(tag >> 3);
        int wt = tag & 7;
        bool strfield = (m.special == SP_QUANTITY && num == 1) || (m.special == SP_INTORSTR && num == 3) ||
                        (m.special == SP_LISTWRAP && num == 1);
        if (wt == 2 && strfield) {
          uint64_t ln;
          if (!in.varint(ln) || static_cast<uint64_t>(in.e - in.p) < ln) { Py_XDECREF(str); Py_XDECREF(lst); return truncated(); }
          PyObject* s = ld_obj(T_STRING, in.p, ln);
          in.p += ln;
          if (!s) { Py_XDECREF(str); Py_XDECREF(lst); return nullptr; }
          if (lst) { PyList_Append(lst, s); Py_DECREF(s); }
          else { Py_XDECREF(str); str = s; }
        } else if (wt == 0 && m.special == SP_INTORSTR && (num == 1 || num == 2)) {
          uint64_t v;
          if (!in.varint(v)) { Py_XDECREF(str); return truncated(); }
          if (num == 1) type = static_cast<int64_t>(v); else ival = static_cast<int32_t>(v);
        } else if (!skip(in, wt)) {
          Py_XDECREF(str); Py_XDECREF(lst);
          return truncated();
        }
      }
      if (lst) return lst;
      if (m.special == SP_INTORSTR) {
        if (type == 1) return str ? str : PyUnicode_FromString("");
        Py_XDECREF(str);
        return PyLong_FromLongLong(ival);
      }
      return str ? str : PyUnicode_FromString("");
    }
    default: {
      PyObject* b = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(p), n);
      if (!b) return nullptr;
      PyObject* r = PyObject_CallFunction(g_dec_cb, "iO", mi, b);
      Py_DECREF(b);
      return r;
    }
  }
}

PyObject* decode_msg(const uint8_t* p, size_t n, int mi) {
  const Msg& m = g_msgs[mi];
  if (m.special) return decode_special(p, n, mi);
  const size_t nf = m.fields.size();
  // per-field slots, filled in wire order, emitted in field order
  PyObject* small[48];
  std::vector<PyObject*> big;
  PyObject** slot = small;
  if (nf > 48) { big.assign(nf, nullptr); slot = big.data(); }
  else std::memset(small, 0, sizeof(PyObject*) * nf);
  auto cleanup = [&]() { for (size_t i = 0; i < nf; i++) Py_XDECREF(slot[i]); };
  In in{p, p + n};
  while (in.p < in.e) {
    uint64_t tag;
    if (!in.varint(tag)) { cleanup(); return truncated(); }
    uint32_t num = static_cast<uint32_t>(tag >> 3);
    int wt = tag & 7;
    int idx = num < m.by_num.size() ? m.by_num[num] : -1;
    if (idx < 0) {
      if (!skip(in, wt)) { cleanup(); return truncated(); }
      continue;
    }
    const Field& f = m.fields[idx];
    const uint8_t* cp = nullptr;
    uint64_t ln = 0;
    if (wt == 2) {
      if (!in.varint(ln) || static_cast<uint64_t>(in.e - in.p) < ln) { cleanup(); return truncated(); }
      cp = in.p;
      in.p += ln;
    }
    PyObject* val = nullptr;
    switch (f.kind) {
      case SCALAR:
        if (wt == 2 && (f.stype == T_STRING || f.stype == T_BYTES)) val = ld_obj(f.stype, cp, ln);
        else if (wt != 2) val = read_scalar(in, f.stype, wt);
        else { cleanup(); return truncated(); }
        if (!val) { cleanup(); return PyErr_Occurred() ? nullptr : truncated(); }
        Py_XSETREF(slot[idx], val);
        break;
      case MSG:
      case INLINE:
        if (wt != 2) { cleanup(); return truncated(); }
        val = decode_msg(cp, ln, f.sub);
        if (!val) { cleanup(); return nullptr; }
        Py_XSETREF(slot[idx], val);
        break;
      case REP_SCALAR:
      case REP_MSG: {
        if (!slot[idx] && !(slot[idx] = PyList_New(0))) { cleanup(); return nullptr; }
        if (f.kind == REP_MSG) {
          if (wt != 2) { cleanup(); return truncated(); }
          val = decode_msg(cp, ln, f.sub);
          if (!val) { cleanup(); return nullptr; }
          PyList_Append(slot[idx], val);
          Py_DECREF(val);
        } else if (wt == 2 && f.stype != T_STRING && f.stype != T_BYTES) {   // packed
          In pk{cp, cp + ln};
          int pwt = (f.stype == T_DOUBLE || f.stype == T_FIXED64 || f.stype == T_SFIXED64) ? 1 :
                    (f.stype == T_FLOAT || f.stype == T_FIXED32 || f.stype == T_SFIXED32) ? 5 : 0;
          while (pk.p < pk.e) {
            val = read_scalar(pk, f.stype, pwt);
            if (!val) { cleanup(); return truncated(); }
            PyList_Append(slot[idx], val);
            Py_DECREF(val);
          }
        } else {
          val = wt == 2 ? ld_obj(f.stype, cp, ln) : read_scalar(in, f.stype, wt);
          if (!val) { cleanup(); return PyErr_Occurred() ? nullptr : truncated(); }
          PyList_Append(slot[idx], val);
          Py_DECREF(val);
        }
        break;
      }
      default: {   // map entry
        if (wt != 2) { cleanup(); return truncated(); }
        if (!slot[idx] && !(slot[idx] = PyDict_New())) { cleanup(); return nullptr; }
        In en{cp, cp + ln};
        PyObject* k = nullptr;
        PyObject* x = nullptr;
        while (en.p < en.e) {
          uint64_t t2;
          if (!en.varint(t2)) break;
          uint32_t n2 = static_cast<uint32_t>(t2 >> 3);
          int w2 = t2 & 7;
          const uint8_t* ep = nullptr;
          uint64_t el = 0;
          if (w2 == 2) {
            if (!en.varint(el) || static_cast<uint64_t>(en.e - en.p) < el) { Py_XDECREF(k); Py_XDECREF(x); cleanup(); return truncated(); }
            ep = en.p;
            en.p += el;
          }
          PyObject* got = nullptr;
          if (n2 == 1) {
            got = w2 == 2 ? ld_obj(f.ktype, ep, el) : read_scalar(en, f.ktype, w2);
            Py_XSETREF(k, got);
          } else if (n2 == 2) {
            if (f.kind == MAP_MSG) got = w2 == 2 ? decode_msg(ep, el, f.sub) : nullptr;
            else got = w2 == 2 ? ld_obj(f.stype, ep, el) : read_scalar(en, f.stype, w2);
            Py_XSETREF(x, got);
          } else {
            if (w2 != 2 && !skip(en, w2)) break;
            continue;
          }
          if (!got) { Py_XDECREF(k); Py_XDECREF(x); cleanup(); return PyErr_Occurred() ? nullptr : truncated(); }
        }
        if (!k) k = f.ktype == T_STRING ? PyUnicode_FromString("") : PyLong_FromLong(0);
        if (!x) {   // an entry without a value holds the type's zero value
          if (f.kind == MAP_MSG) x = decode_msg(nullptr, 0, f.sub);
          else if (f.stype == T_STRING || f.stype == T_BYTES) x = PyUnicode_FromString("");
          else x = scalar_obj(f.stype, 0);
        }
        if (!k || !x || PyDict_SetItem(slot[idx], k, x) < 0) { Py_XDECREF(k); Py_XDECREF(x); cleanup(); return nullptr; }
        Py_DECREF(k);
        Py_DECREF(x);
      }
    }
  }
  PyObject* out = PyDict_New();
  if (!out) { cleanup(); return nullptr; }
  for (size_t i = 0; i < nf; i++) {
    if (!slot[i]) continue;
    const Field& f = m.fields[i];
    int r;
    if (f.kind == INLINE) r = PyDict_Check(slot[i]) ? PyDict_Update(out, slot[i]) : 0;
    else r = PyDict_SetItem(out, f.key, slot[i]);
    if (r < 0) { Py_DECREF(out); cleanup(); return nullptr; }
  }
  cleanup();
  return out;
}

// ------------------------------------------------------------------------------ envelopes
// the top-level length-delimited fields of runtime.Unknown after the magic:
// typeMeta = 1 {apiVersion = 1, kind = 2}, raw = 2, contentEncoding = 3, contentType = 4
struct Env {
  const uint8_t* av = nullptr; size_t avn = 0;
  const uint8_t* kind = nullptr; size_t kn = 0;
  const uint8_t* raw = nullptr; size_t rawn = 0;
  const uint8_t* ct = nullptr; size_t ctn = 0;
  bool has_raw = false;
};

bool parse_env(const uint8_t* p, size_t n, Env& e) {
  if (n < 4 || std::memcmp(p, "k8s\0", 4) != 0) return false;
  In in{p + 4, p + n};
  while (in.p < in.e) {
    uint64_t tag, ln;
    if (!in.varint(tag)) return false;
    if ((tag & 7) != 2) { if (!skip(in, tag & 7)) return false; continue; }
    if (!in.varint(ln) || static_cast<uint64_t>(in.e - in.p) < ln) return false;
    const uint8_t* cp = in.p;
    in.p += ln;
    switch (tag >> 3) {
      case 1: {
        In tm{cp, cp + ln};
        while (tm.p < tm.e) {
          uint64_t t2, l2;
          if (!tm.varint(t2)) return false;
          if ((t2 & 7) != 2) { if (!skip(tm, t2 & 7)) return false; continue; }
          if (!tm.varint(l2) || static_cast<uint64_t>(tm.e - tm.p) < l2) return false;
          if ((t2 >> 3) == 1) { e.av = tm.p; e.avn = l2; }
          else if ((t2 >> 3) == 2) { e.kind = tm.p; e.kn = l2; }
          tm.p += l2;
        }
        break;
      }
      case 2: e.raw = cp; e.rawn = ln; e.has_raw = true; break;
      case 4: e.ct = cp; e.ctn = ln; break;
      default: break;
    }
  }
  return true;
}

bool is_json_ct(const Env& e) {
  for (size_t i = 0; i + 4 <= e.ctn; i++)
    if (std::memcmp(e.ct + i, "json", 4) == 0) return true;
  return false;
}

// ------------------------------------------------------------------------------ module
PyObject* py_init(PyObject*, PyObject* args) {
  PyObject *table, *err, *enc_cb, *dec_cb;
  if (!PyArg_ParseTuple(args, "OOOO", &table, &err, &enc_cb, &dec_cb)) return nullptr;
  PyObject* seq = PySequence_Fast(table, "table must be a sequence");
  if (!seq) return nullptr;
  std::vector<Msg> msgs(PySequence_Fast_GET_SIZE(seq));
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); i++) {
    PyObject* ent = PySequence_Fast_GET_ITEM(seq, i);
    int special;
    PyObject *fields, *keys;
    if (!PyArg_ParseTuple(ent, "iOO", &special, &fields, &keys)) { Py_DECREF(seq); return nullptr; }
    Msg& m = msgs[i];
    m.special = special;
    Py_INCREF(keys);
    m.keys = keys;
    PyObject* fs = PySequence_Fast(fields, "fields must be a sequence");
    if (!fs) { Py_DECREF(seq); return nullptr; }
    uint32_t maxn = 0;
    for (Py_ssize_t j = 0; j < PySequence_Fast_GET_SIZE(fs); j++) {
      unsigned int num, kind, stype, ktype;
      int sub;
      PyObject* key;
      if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(fs, j), "IOIIIi", &num, &key, &kind, &stype, &ktype, &sub)) {
        Py_DECREF(fs); Py_DECREF(seq); return nullptr;
      }
      if (sub >= static_cast<int>(msgs.size()) || ((kind == MSG || kind == REP_MSG || kind == MAP_MSG || kind == INLINE) && sub < 0)) {
        Py_DECREF(fs); Py_DECREF(seq);
        PyErr_SetString(PyExc_ValueError, "bad sub-message index");
        return nullptr;
      }
      Field f{num, nullptr, static_cast<uint8_t>(kind), static_cast<uint8_t>(stype), static_cast<uint8_t>(ktype), sub};
      if (key != Py_None) {
        Py_INCREF(key);
        PyUnicode_InternInPlace(&key);
        f.key = key;
      } else if (kind != INLINE) {
        Py_DECREF(fs); Py_DECREF(seq);
        PyErr_SetString(PyExc_ValueError, "only inline fields may lack a key");
        return nullptr;
      }
      m.fields.push_back(f);
      if (num > maxn) maxn = num;
    }
    Py_DECREF(fs);
    m.by_num.assign(maxn + 1, -1);
    for (size_t j = 0; j < m.fields.size(); j++) m.by_num[m.fields[j].num] = static_cast<int16_t>(j);
  }
  Py_DECREF(seq);
  g_msgs.swap(msgs);   // old tables leak their refs on purpose (a re-init is test-only)
  Py_INCREF(err); Py_XSETREF(g_err, err);
  Py_INCREF(enc_cb); Py_XSETREF(g_enc_cb, enc_cb);
  Py_INCREF(dec_cb); Py_XSETREF(g_dec_cb, dec_cb);
  Py_RETURN_NONE;
}

bool check_idx(int mi) {
  if (mi < 0 || mi >= static_cast<int>(g_msgs.size())) {
    PyErr_SetString(PyExc_IndexError, "message index out of range (init first)");
    return false;
  }
  return true;
}

PyObject* py_encode(PyObject*, PyObject* args) {
  PyObject* obj;
  int mi, strict = 0;
  if (!PyArg_ParseTuple(args, "Oi|p", &obj, &mi, &strict) || !check_idx(mi)) return nullptr;
  Out o;
  o.b.reserve(512);
  Ctx c{strict != 0};
  if (encode_msg(o, obj, mi, c, true) < 0) return nullptr;
  PyObject* b = PyBytes_FromStringAndSize(o.b.data(), o.b.size());
  if (!b) return nullptr;
  return Py_BuildValue("(NO)", b, c.lossless ? Py_True : Py_False);
}

PyObject* py_decode(PyObject*, PyObject* args) {
  Py_buffer buf;
  int mi;
  if (!PyArg_ParseTuple(args, "y*i", &buf, &mi)) return nullptr;
  if (!check_idx(mi)) { PyBuffer_Release(&buf); return nullptr; }
  PyObject* r = decode_msg(static_cast<const uint8_t*>(buf.buf), buf.len, mi);
  PyBuffer_Release(&buf);
  return r;
}

PyObject* py_envelope_parts(PyObject*, PyObject* args) {
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "y*", &buf)) return nullptr;
  Env e;
  PyObject* r;
  if (!parse_env(static_cast<const uint8_t*>(buf.buf), buf.len, e)) {
    r = Py_None;
    Py_INCREF(r);
  } else {
    r = Py_BuildValue("(s#s#y#s#)", e.av ? reinterpret_cast<const char*>(e.av) : "", static_cast<Py_ssize_t>(e.avn),
                      e.kind ? reinterpret_cast<const char*>(e.kind) : "", static_cast<Py_ssize_t>(e.kn),
                      e.raw ? reinterpret_cast<const char*>(e.raw) : "", static_cast<Py_ssize_t>(e.rawn),
                      e.ct ? reinterpret_cast<const char*>(e.ct) : "", static_cast<Py_ssize_t>(e.ctn));
  }
  PyBuffer_Release(&buf);
  return r;
}

PyObject* py_splice_list(PyObject*, PyObject* args) {
  const char *av, *kind, *rv;
  Py_ssize_t avn, kn, rvn;
  PyObject* values;
  if (!PyArg_ParseTuple(args, "s#s#s#O", &av, &avn, &kind, &kn, &rv, &rvn, &values)) return nullptr;
  PyObject* seq = PySequence_Fast(values, "values must be a sequence");
  if (!seq) return nullptr;
  Out body;
  size_t total = 16 + rvn;
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); i++) {
    PyObject* v = PySequence_Fast_GET_ITEM(seq, i);
    if (PyBytes_Check(v)) total += PyBytes_GET_SIZE(v) + 6;
  }
  body.b.reserve(total);
  {   // ListMeta{resourceVersion = 2} = 1
    size_t st = body.open(1);
    body.bytes(2, rv, rvn);
    body.close(st);
  }
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); i++) {
    PyObject* v = PySequence_Fast_GET_ITEM(seq, i);
    if (!PyBytes_Check(v)) { Py_DECREF(seq); Py_RETURN_NONE; }
    Env e;
    if (!parse_env(reinterpret_cast<const uint8_t*>(PyBytes_AS_STRING(v)), PyBytes_GET_SIZE(v), e) || !e.has_raw ||
        is_json_ct(e)) {
      Py_DECREF(seq);
      Py_RETURN_NONE;
    }
    body.bytes(2, reinterpret_cast<const char*>(e.raw), e.rawn);
  }
  Py_DECREF(seq);
  Out o;
  o.b.reserve(body.b.size() + avn + kn + 32);
  o.b.append("k8s\0", 4);
  size_t st = o.open(1);
  o.bytes(1, av, avn);
  o.bytes(2, kind, kn);
  o.close(st);
  o.bytes(2, body.b.data(), body.b.size());
  return PyBytes_FromStringAndSize(o.b.data(), o.b.size());
}

PyMethodDef kMethods[] = {
    {"init", py_init, METH_VARARGS, "init(table, proto_error, enc_cb, dec_cb)"},
    {"encode", py_encode, METH_VARARGS, "encode(obj, msg_index, strict=False) -> (bytes, lossless)"},
    {"decode", py_decode, METH_VARARGS, "decode(buf, msg_index) -> dict"},
    {"envelope_parts", py_envelope_parts, METH_VARARGS, "envelope_parts(buf) -> (apiVersion, kind, raw, contentType) | None"},
    {"splice_list", py_splice_list, METH_VARARGS, "splice_list(apiVersion, listKind, rv, values) -> bytes | None"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_kproto", "Native Kubernetes protobuf transcoder", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__kproto(void) {
  PyObject* binascii = PyImport_ImportModule("binascii");
  if (!binascii) return nullptr;
  g_b64enc = PyObject_GetAttrString(binascii, "b2a_base64");
  g_b64dec = PyObject_GetAttrString(binascii, "a2b_base64");
  Py_DECREF(binascii);
  if (!g_b64enc || !g_b64dec) return nullptr;
  g_s_apiVersion = PyUnicode_InternFromString("apiVersion");
  g_s_kind = PyUnicode_InternFromString("kind");
  g_err = PyExc_ValueError;
  Py_INCREF(g_err);
  return PyModule_Create(&kModule);
}
