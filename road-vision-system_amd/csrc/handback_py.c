/* Detection lists from a handed-back result record, in C (CPython API).
 *
 * The reference ends every frame with a List[Detection] per camera
 * (src/detect/yolo_ultralytics.py:44-52 builds them from .cpu().numpy(),
 * src/track/sort_tracker.py:234-247 fills track_id / distance_m / speed_kmh).
 * rvs_amd.handback.to_detections builds the same objects from the record
 * rv_results_handback writes (csrc/results.hip: int32 n[S] padded to 16 B,
 * then S x dmax rows of 48 B {f32 x1,y1,x2,y2,conf; i32 cls, track_id, pad;
 * f64 dist, speed}); this module does it without the Python interpreter in
 * the per-object loop: each Detection is allocated with its type's tp_alloc
 * and given a fresh attribute dict (a dataclass instance is exactly that),
 * ~4x cheaper than the column-wise Python version, so a host consumer
 * thread keeps up with the device (bench.py's timed region).
 *
 * build(record, S, dmax, names, cls) -> list of S lists
 *   record: a buffer (the pinned host record), names: list of class names,
 *   cls: the Detection class.  -1 track ids and NaN metrics become None,
 *   class ids outside names become str(id) -- as the Python version.
 * shells(cls, n) -> list of n Detection objects whose 10 fields are None
 * build(record, S, dmax, names, cls, pool) -- the same lists, but each
 *   Detection is taken from the end of `pool` (a list of shells, consumed)
 *   and its fields are set in place; a fresh one is made when the pool runs
 *   out.  Object and attribute-dict allocation then happen when the shells
 *   are made -- by a consumer while it waits for the next hand-back --
 *   instead of after the hand-back (a third less work after it).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
  float x1, y1, x2, y2, conf;
  int32_t cls, track_id, pad;
  double dist, speed;
} Row;

static PyObject* k_names[10];
static const char* k_fields[10] = {"x1",     "y1",       "x2",       "y2",         "conf",
                                   "cls_id", "cls_name", "track_id", "distance_m", "speed_kmh"};

/* a Detection whose 10 fields are None (a dataclass instance: its type's
   allocation plus an attribute dict) */
static PyObject* new_shell(PyTypeObject* tp) {
  PyObject* d = _PyDict_NewPresized(10);
  if (!d) return NULL;
  for (int f = 0; f < 10; ++f)
    if (PyDict_SetItem(d, k_names[f], Py_None) < 0) {
      Py_DECREF(d);
      return NULL;
    }
  PyObject* obj = tp->tp_alloc(tp, 0);
  if (!obj || PyObject_GenericSetDict(obj, d, NULL) < 0) {
    Py_XDECREF(obj);
    Py_DECREF(d);
    return NULL;
  }
  Py_DECREF(d);
  return obj;
}

static PyObject* shells(PyObject* self, PyObject* args) {
  PyObject* cls;
  Py_ssize_t n;
  if (!PyArg_ParseTuple(args, "On", &cls, &n)) return NULL;
  if (!PyType_Check(cls)) {
    PyErr_SetString(PyExc_TypeError, "cls must be the Detection class");
    return NULL;
  }
  if (n < 0) n = 0;
  PyObject* out = PyList_New(n);
  if (!out) return NULL;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* o = new_shell((PyTypeObject*)cls);
    if (!o) {
      Py_DECREF(out);
      return NULL;
    }
    PyList_SET_ITEM(out, i, o);
  }
  return out;
}

static PyObject* build(PyObject* self, PyObject* args) {
  PyObject *rec_obj, *names, *cls, *pool = NULL;
  Py_ssize_t S, dmax;
  if (!PyArg_ParseTuple(args, "OnnOO|O", &rec_obj, &S, &dmax, &names, &cls, &pool)) return NULL;
  if (pool == Py_None) pool = NULL;
  if (pool && !PyList_Check(pool)) {
    PyErr_SetString(PyExc_TypeError, "pool must be a list of Detection shells");
    return NULL;
  }
  if (!PyType_Check(cls)) {
    PyErr_SetString(PyExc_TypeError, "cls must be the Detection class");
    return NULL;
  }
  if (!PyList_Check(names)) {
    PyErr_SetString(PyExc_TypeError, "names must be a list");
    return NULL;
  }
  Py_buffer buf;
  if (PyObject_GetBuffer(rec_obj, &buf, PyBUF_SIMPLE) < 0) return NULL;
  const Py_ssize_t hdr = (S * 4 + 15) & ~(Py_ssize_t)15;
  if (S < 0 || dmax < 0 || buf.len < hdr + S * dmax * (Py_ssize_t)sizeof(Row)) {
    PyBuffer_Release(&buf);
    PyErr_SetString(PyExc_ValueError, "record smaller than S x dmax rows");
    return NULL;
  }
  const int32_t* n = (const int32_t*)buf.buf;
  const Row* rows = (const Row*)((const char*)buf.buf + hdr);
  PyTypeObject* tp = (PyTypeObject*)cls;
  const Py_ssize_t nn = PyList_GET_SIZE(names);
  Py_ssize_t np = pool ? PyList_GET_SIZE(pool) : 0;  // shells left (taken from the end)
  const Py_ssize_t np0 = np;
  PyObject* out = PyList_New(S);
  if (!out) goto fail;
  for (Py_ssize_t s = 0; s < S; ++s) {
    Py_ssize_t c = n[s];
    c = c < 0 ? 0 : (c > dmax ? dmax : c);
    PyObject* lst = PyList_New(c);
    if (!lst) goto fail;
    PyList_SET_ITEM(out, s, lst);
    for (Py_ssize_t i = 0; i < c; ++i) {
      const Row* r = rows + s * dmax + i;
      PyObject* v[10];
      v[0] = PyFloat_FromDouble(r->x1);
      v[1] = PyFloat_FromDouble(r->y1);
      v[2] = PyFloat_FromDouble(r->x2);
      v[3] = PyFloat_FromDouble(r->y2);
      v[4] = PyFloat_FromDouble(r->conf);
      v[5] = PyLong_FromLong(r->cls);
      if (r->cls >= 0 && r->cls < nn) {
        v[6] = PyList_GET_ITEM(names, r->cls);
        Py_INCREF(v[6]);
        if (!PyUnicode_Check(v[6])) {
          PyObject* t = PyObject_Str(v[6]);
          Py_DECREF(v[6]);
          v[6] = t;
        }
      } else {
        v[6] = PyUnicode_FromFormat("%d", (int)r->cls);
      }
      if (r->track_id < 0) {
        Py_INCREF(Py_None);
        v[7] = Py_None;
      } else {
        v[7] = PyLong_FromLong(r->track_id);
      }
      if (isnan(r->dist)) {
        Py_INCREF(Py_None);
        v[8] = Py_None;
      } else {
        v[8] = PyFloat_FromDouble(r->dist);
      }
      if (isnan(r->speed)) {
        Py_INCREF(Py_None);
        v[9] = Py_None;
      } else {
        v[9] = PyFloat_FromDouble(r->speed);
      }
      PyObject* obj;
      PyObject* d;
      int bad;
      if (np > 0) {  // a shell: its dict already holds the 10 keys
        obj = PyList_GET_ITEM(pool, np - 1);
        Py_INCREF(obj);
        --np;
        d = PyObject_GenericGetDict(obj, NULL);
        bad = !d;
      } else {
        d = _PyDict_NewPresized(10);
        obj = tp->tp_alloc(tp, 0);
        bad = !d || !obj;
        if (!bad && PyObject_GenericSetDict(obj, d, NULL) < 0) bad = 1;
      }
      for (int f = 0; f < 10; ++f) {
        if (!v[f]) bad = 1;
        if (!bad && PyDict_SetItem(d, k_names[f], v[f]) < 0) bad = 1;
        Py_XDECREF(v[f]);
      }
      Py_XDECREF(d);
      if (bad) {
        Py_XDECREF(obj);
        goto fail;
      }
      PyList_SET_ITEM(lst, i, obj);
    }
  }
  if (pool && np < np0 && PyList_SetSlice(pool, np, np0, NULL) < 0) goto fail;
  PyBuffer_Release(&buf);
  return out;
fail:
  if (pool && np < np0) PyList_SetSlice(pool, np, np0, NULL);
  PyBuffer_Release(&buf);
  Py_XDECREF(out);
  if (!PyErr_Occurred()) PyErr_NoMemory();
  return NULL;
}

static PyMethodDef methods[] = {
    {"build", build, METH_VARARGS,
     "build(record, S, dmax, names, Detection[, pool]) -> S lists of Detection"},
    {"shells", shells, METH_VARARGS, "shells(Detection, n) -> n Detection objects, fields None"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_rvhandback",
                                    "Detection lists from a result record (C)", -1, methods};

PyMODINIT_FUNC PyInit__rvhandback(void) {
  for (int f = 0; f < 10; ++f) {
    k_names[f] = PyUnicode_InternFromString(k_fields[f]);
    if (!k_names[f]) return NULL;
  }
  return PyModule_Create(&module);
}
