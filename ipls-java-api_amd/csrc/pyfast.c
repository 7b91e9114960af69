/* ipls._fast: the per-arrival calls of ipls.Aggregator without ctypes.
 *
 * Updater._Update is called once per arriving bucket (Updater.java:115-117);
 * through ctypes each call costs ~1.5 us of argument conversion, which is on
 * the critical path of the queued (coalesced) folds: the GPU starts when the
 * queues fill.  This extension links against the in-tree libipls_agg.so
 * (rpath $ORIGIN/../lib: the same file ipls._native loads, so the loader maps
 * it once) and calls two of its C-ABI entry points directly:
 *
 *   accumulate_async(h, p, target, src, n, kind) -> ticket, or rc < 0
 *       ipls_agg_accumulate_async (include/ipls_agg.h)
 *   accumulate(h, p, target, src, n, kind)       -> rc
 *       ipls_agg_accumulate
 *   entry_points() -> the two addresses, which ipls compares with the
 *       library it bound before using this module
 *
 * h and src are addresses (a null handle is rejected by the library).  The
 * GIL is released around the call, as ctypes does: a call may wait for a
 * slot of the fold queue.  Plain C, CPython API only. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <limits.h>
#include <stdint.h>

#include "../../include/ipls_agg.h"

typedef struct {
  ipls_agg* h;
  int p, target, kind;
  const void* src;
  int64_t n;
} Args;

static int as_int(PyObject* o, int* out) {
  const long v = PyLong_AsLong(o);
  if (v == -1 && PyErr_Occurred()) return -1;
  if (v < INT_MIN || v > INT_MAX) {
    PyErr_SetString(PyExc_OverflowError, "argument out of int range");
    return -1;
  }
  *out = (int)v;
  return 0;
}

/* None or 0 is passed on as NULL: the library rejects a null handle */
static int as_ptr(PyObject* o, void** out) {
  if (o == Py_None) {
    *out = NULL;
    return 0;
  }
  *out = PyLong_AsVoidPtr(o);
  return (*out == NULL && PyErr_Occurred()) ? -1 : 0;
}

static int parse(PyObject* const* a, Py_ssize_t na, Args* x) {
  if (na != 6) {
    PyErr_Format(PyExc_TypeError, "expected 6 arguments (h, p, target, src, n, kind), got %zd", na);
    return -1;
  }
  void *h = NULL, *src = NULL;
  if (as_ptr(a[0], &h) || as_int(a[1], &x->p) || as_int(a[2], &x->target) || as_ptr(a[3], &src) ||
      as_int(a[5], &x->kind))
    return -1;
  const long long n = PyLong_AsLongLong(a[4]);
  if (n == -1 && PyErr_Occurred()) return -1;
  x->h = (ipls_agg*)h;
  x->src = src;
  x->n = (int64_t)n;
  return 0;
}

static PyObject* fast_accumulate_async(PyObject* self, PyObject* const* a, Py_ssize_t na) {
  (void)self;
  Args x;
  if (parse(a, na, &x)) return NULL;
  uint64_t ticket = 0;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = ipls_agg_accumulate_async(x.h, x.p, x.target, x.src, x.n, x.kind, &ticket);
  Py_END_ALLOW_THREADS
  if (rc < 0) return PyLong_FromLong(rc);
  return PyLong_FromUnsignedLongLong(ticket);
}

static PyObject* fast_accumulate(PyObject* self, PyObject* const* a, Py_ssize_t na) {
  (void)self;
  Args x;
  if (parse(a, na, &x)) return NULL;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = ipls_agg_accumulate(x.h, x.p, x.target, x.src, x.n, x.kind);
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

/* the addresses this module calls, so ipls can check they are the entry
 * points of the library it bound itself (one mapping of one file) */
static PyObject* fast_entry_points(PyObject* self, PyObject* unused) {
  (void)self;
  (void)unused;
  return Py_BuildValue("(KK)", (unsigned long long)(uintptr_t)&ipls_agg_accumulate_async,
                       (unsigned long long)(uintptr_t)&ipls_agg_accumulate);
}

static PyMethodDef methods[] = {
    {"entry_points", fast_entry_points, METH_NOARGS,
     "entry_points() -> (address of ipls_agg_accumulate_async, address of ipls_agg_accumulate)"},
    {"accumulate_async", (PyCFunction)(void (*)(void))fast_accumulate_async, METH_FASTCALL,
     "accumulate_async(h, p, target, src, n, kind) -> ticket (>= 0) or the library's error code (< 0)"},
    {"accumulate", (PyCFunction)(void (*)(void))fast_accumulate, METH_FASTCALL,
     "accumulate(h, p, target, src, n, kind) -> the library's return code"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fast",
                                    "Per-arrival C-ABI calls without ctypes (see csrc/pyfast.c).", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fast(void) { return PyModule_Create(&module); }
