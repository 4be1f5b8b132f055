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

static PyObject* build(PyObject* self, PyObject* args) {
  PyObject *rec_obj, *names, *cls;
  Py_ssize_t S, dmax;
  if (!PyArg_ParseTuple(args, "OnnOO", &rec_obj, &S, &dmax, &names, &cls)) return NULL;
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
      PyObject* d = _PyDict_NewPresized(10);
      PyObject* obj = tp->tp_alloc(tp, 0);
      int bad = !d || !obj;
      for (int f = 0; f < 10; ++f) {
        if (!v[f]) bad = 1;
        if (!bad && PyDict_SetItem(d, k_names[f], v[f]) < 0) bad = 1;
        Py_XDECREF(v[f]);
      }
      if (!bad && PyObject_GenericSetDict(obj, d, NULL) < 0) bad = 1;
      Py_XDECREF(d);
      if (bad) {
        Py_XDECREF(obj);
        goto fail;
      }
      PyList_SET_ITEM(lst, i, obj);
    }
  }
  PyBuffer_Release(&buf);
  return out;
fail:
  PyBuffer_Release(&buf);
  Py_XDECREF(out);
  if (!PyErr_Occurred()) PyErr_NoMemory();
  return NULL;
}

static PyMethodDef methods[] = {
    {"build", build, METH_VARARGS,
     "build(record, S, dmax, names, Detection) -> S lists of Detection"},
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
