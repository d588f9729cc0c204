/* Fast Python -> C entry for the per-step collectives (allreduce, reduce-scatter, all-gather).
 *
 * ctypes spends ~2 us converting nine arguments per call; a training step issues one call per gradient
 * bucket, and a latency-bound allreduce is itself a few microseconds. These METH_FASTCALL functions take
 * the C entry point as an integer (its address, from the ctypes handle of libflexar.so, so there is no
 * link-time dependency and exactly one copy of the library is loaded) and call it with the GIL released.
 *
 *   ar(fn, comm, in, out, count, dtype, op, stream, algo_bytes_or_None, scale) -> rc
 *   rs(fn, comm, in, out, count, dtype, op, stream, algo_bytes_or_None) -> rc
 *   ag(fn, comm, in, out, count, dtype, stream, algo_bytes_or_None) -> rc
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stddef.h>

typedef int (*ar_fn)(void*, const void*, void*, size_t, int, int, void*, const char*, float);
typedef int (*rs_fn)(void*, const void*, void*, size_t, int, int, void*, const char*);
typedef int (*ag_fn)(void*, const void*, void*, size_t, int, void*, const char*);

static int algo_arg(PyObject* o, const char** out) {
  if (o == Py_None) { *out = NULL; return 0; }
  *out = PyBytes_AsString(o);
  return *out ? 0 : -1;
}

static PyObject* fc_ar(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  if (n != 10) { PyErr_SetString(PyExc_TypeError, "ar() takes 10 arguments"); return NULL; }
  ar_fn f = (ar_fn)PyLong_AsVoidPtr(a[0]);
  void* c = PyLong_AsVoidPtr(a[1]);
  const void* in = PyLong_AsVoidPtr(a[2]);
  void* out = PyLong_AsVoidPtr(a[3]);
  size_t count = PyLong_AsSize_t(a[4]);
  int dtype = (int)PyLong_AsLong(a[5]);
  int op = (int)PyLong_AsLong(a[6]);
  void* st = PyLong_AsVoidPtr(a[7]);
  const char* algo;
  if (algo_arg(a[8], &algo)) return NULL;
  double scale = PyFloat_AsDouble(a[9]);
  if (PyErr_Occurred()) return NULL;
  if (!f) { PyErr_SetString(PyExc_ValueError, "null entry point"); return NULL; }
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = f(c, in, out, count, dtype, op, st, algo, (float)scale);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

static PyObject* fc_rs(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  if (n != 9) { PyErr_SetString(PyExc_TypeError, "rs() takes 9 arguments"); return NULL; }
  rs_fn f = (rs_fn)PyLong_AsVoidPtr(a[0]);
  void* c = PyLong_AsVoidPtr(a[1]);
  const void* in = PyLong_AsVoidPtr(a[2]);
  void* out = PyLong_AsVoidPtr(a[3]);
  size_t count = PyLong_AsSize_t(a[4]);
  int dtype = (int)PyLong_AsLong(a[5]);
  int op = (int)PyLong_AsLong(a[6]);
  void* st = PyLong_AsVoidPtr(a[7]);
  const char* algo;
  if (algo_arg(a[8], &algo)) return NULL;
  if (PyErr_Occurred()) return NULL;
  if (!f) { PyErr_SetString(PyExc_ValueError, "null entry point"); return NULL; }
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = f(c, in, out, count, dtype, op, st, algo);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

static PyObject* fc_ag(PyObject* self, PyObject* const* a, Py_ssize_t n) {
  (void)self;
  if (n != 8) { PyErr_SetString(PyExc_TypeError, "ag() takes 8 arguments"); return NULL; }
  ag_fn f = (ag_fn)PyLong_AsVoidPtr(a[0]);
  void* c = PyLong_AsVoidPtr(a[1]);
  const void* in = PyLong_AsVoidPtr(a[2]);
  void* out = PyLong_AsVoidPtr(a[3]);
  size_t count = PyLong_AsSize_t(a[4]);
  int dtype = (int)PyLong_AsLong(a[5]);
  void* st = PyLong_AsVoidPtr(a[6]);
  const char* algo;
  if (algo_arg(a[7], &algo)) return NULL;
  if (PyErr_Occurred()) return NULL;
  if (!f) { PyErr_SetString(PyExc_ValueError, "null entry point"); return NULL; }
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = f(c, in, out, count, dtype, st, algo);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"ar", (PyCFunction)(void (*)(void))fc_ar, METH_FASTCALL, "allreduce entry"},
    {"rs", (PyCFunction)(void (*)(void))fc_rs, METH_FASTCALL, "reduce-scatter entry"},
    {"ag", (PyCFunction)(void (*)(void))fc_ag, METH_FASTCALL, "all-gather entry"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_fastcall", "flexar fast call path", -1, methods,
                                 NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fastcall(void) { return PyModule_Create(&mod); }
