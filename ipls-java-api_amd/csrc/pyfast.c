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
 *   accumulate_async_many(h, target, items) -> last ticket, or (rc < 0, index)
 *       ipls_agg_accumulate_async for every (p, src, n, kind) of `items`, in
 *       order, as ONE Python -> C transition: a caller that drains several
 *       arrivals at once (one peer's buckets of every partition) pays the
 *       interpreter once, not per bucket
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

typedef struct {
  int p, kind;
  const void* src;
  int64_t n;
} Item;

static PyObject* fast_accumulate_async_many(PyObject* self, PyObject* const* a, Py_ssize_t na) {
  (void)self;
  if (na != 3) {
    PyErr_Format(PyExc_TypeError, "expected 3 arguments (h, target, items), got %zd", na);
    return NULL;
  }
  void* h = NULL;
  int target;
  if (as_ptr(a[0], &h) || as_int(a[1], &target)) return NULL;
  PyObject* seq = PySequence_Fast(a[2], "items must be a sequence of (p, src, n, kind)");
  if (!seq) return NULL;
  const Py_ssize_t m = PySequence_Fast_GET_SIZE(seq);
  Item* it = (Item*)PyMem_Malloc((size_t)(m > 0 ? m : 1) * sizeof(Item));
  if (!it) {
    Py_DECREF(seq);
    return PyErr_NoMemory();
  }
  PyObject** el = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < m; ++i) {
    PyObject* t = el[i];
    void* src = NULL;
    long long n;
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) != 4 || as_int(PyTuple_GET_ITEM(t, 0), &it[i].p) ||
        as_ptr(PyTuple_GET_ITEM(t, 1), &src) || as_int(PyTuple_GET_ITEM(t, 3), &it[i].kind) ||
        ((n = PyLong_AsLongLong(PyTuple_GET_ITEM(t, 2))) == -1 && PyErr_Occurred())) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "items must be (p, src, n, kind) tuples");
      PyMem_Free(it);
      Py_DECREF(seq);
      return NULL;
    }
    it[i].src = src;
    it[i].n = (int64_t)n;
  }
  Py_DECREF(seq);
  uint64_t ticket = 0;
  int rc = 0;
  Py_ssize_t i = 0;
  Py_BEGIN_ALLOW_THREADS
  for (; i < m; ++i) {
    rc = ipls_agg_accumulate_async((ipls_agg*)h, it[i].p, target, it[i].src, it[i].n, it[i].kind, &ticket);
    if (rc < 0) break;
  }
  Py_END_ALLOW_THREADS
  PyMem_Free(it);
  if (rc < 0) return Py_BuildValue("(in)", rc, i);
  return PyLong_FromUnsignedLongLong(ticket);
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
    {"accumulate_async_many", (PyCFunction)(void (*)(void))fast_accumulate_async_many, METH_FASTCALL,
     "accumulate_async_many(h, target, [(p, src, n, kind), ...]) -> last ticket, or (rc < 0, failing index)"},
    {"accumulate", (PyCFunction)(void (*)(void))fast_accumulate, METH_FASTCALL,
     "accumulate(h, p, target, src, n, kind) -> the library's return code"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_fast",
                                    "Per-arrival C-ABI calls without ctypes (see csrc/pyfast.c).", -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fast(void) { return PyModule_Create(&module); }
