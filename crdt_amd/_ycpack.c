/* _ycpack.c — host glue for the Python mirror: ycrdt_buf arrays over Python bytes objects without
 * copying them (the ctypes path joined every update into one blob first: ~0.5 s for the 1.5 GB of a
 * 112-document C2 batch). The returned arrays point INTO the bytes objects: the caller keeps the
 * updates alive until the call that reads the array returns (crdt_amd.Batch keeps them on itself).
 *
 *   bufs(updates)          -> (array, keep)         array: bytes of n x {u64 ptr, u64 len}
 *   docs(list_of_lists)    -> (array, doc_of, keep)  doc_of: bytes of n x u32
 *
 * Non-bytes elements (bytearray, memoryview, ...) are converted to bytes once; `keep` holds those
 * copies (or is an empty list). */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

typedef struct {
  uint64_t ptr, len;
} buf_t;

/* pointer/len of one element; a non-bytes element is converted and appended to keep */
static int one(PyObject* o, PyObject* keep, buf_t* out) {
  if (!PyBytes_Check(o)) {
    PyObject* b = PyBytes_FromObject(o);
    if (!b) return -1;
    if (PyList_Append(keep, b) < 0) { Py_DECREF(b); return -1; }
    Py_DECREF(b); /* keep owns it */
    o = b;
  }
  out->ptr = (uint64_t)(uintptr_t)PyBytes_AS_STRING(o);
  out->len = (uint64_t)PyBytes_GET_SIZE(o);
  return 0;
}

static PyObject* py_bufs(PyObject* self, PyObject* arg) {
  PyObject* seq = PySequence_Fast(arg, "updates must be a sequence");
  if (!seq) return NULL;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject* arr = PyBytes_FromStringAndSize(NULL, (n ? n : 1) * (Py_ssize_t)sizeof(buf_t));
  PyObject* keep = PyList_New(0);
  if (!arr || !keep) goto fail;
  buf_t* b = (buf_t*)PyBytes_AS_STRING(arr);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < n; ++i)
    if (one(items[i], keep, &b[i]) < 0) goto fail;
  Py_DECREF(seq);
  return Py_BuildValue("(NN)", arr, keep);
fail:
  Py_XDECREF(arr);
  Py_XDECREF(keep);
  Py_DECREF(seq);
  return NULL;
}

static PyObject* py_docs(PyObject* self, PyObject* arg) {
  PyObject* outer = PySequence_Fast(arg, "docs must be a sequence of update sequences");
  if (!outer) return NULL;
  const Py_ssize_t nd = PySequence_Fast_GET_SIZE(outer);
  PyObject** docs = PySequence_Fast_ITEMS(outer);
  PyObject *arr = NULL, *doc_of = NULL, *keep = PyList_New(0);
  PyObject** inner = (PyObject**)PyMem_Calloc(nd ? nd : 1, sizeof(PyObject*));
  if (!keep || !inner) goto fail;
  Py_ssize_t n = 0;
  for (Py_ssize_t d = 0; d < nd; ++d) {
    inner[d] = PySequence_Fast(docs[d], "every document must be a sequence of updates");
    if (!inner[d]) goto fail;
    n += PySequence_Fast_GET_SIZE(inner[d]);
  }
  if (nd > 0xFFFFFFFFll) { PyErr_SetString(PyExc_ValueError, "too many documents"); goto fail; }
  arr = PyBytes_FromStringAndSize(NULL, (n ? n : 1) * (Py_ssize_t)sizeof(buf_t));
  doc_of = PyBytes_FromStringAndSize(NULL, (n ? n : 1) * (Py_ssize_t)sizeof(uint32_t));
  if (!arr || !doc_of) goto fail;
  buf_t* b = (buf_t*)PyBytes_AS_STRING(arr);
  uint32_t* dof = (uint32_t*)PyBytes_AS_STRING(doc_of);
  Py_ssize_t k = 0;
  for (Py_ssize_t d = 0; d < nd; ++d) {
    const Py_ssize_t m = PySequence_Fast_GET_SIZE(inner[d]);
    PyObject** it = PySequence_Fast_ITEMS(inner[d]);
    for (Py_ssize_t i = 0; i < m; ++i, ++k) {
      if (one(it[i], keep, &b[k]) < 0) goto fail;
      dof[k] = (uint32_t)d;
    }
  }
  for (Py_ssize_t d = 0; d < nd; ++d) Py_DECREF(inner[d]);
  PyMem_Free(inner);
  Py_DECREF(outer);
  return Py_BuildValue("(NNN)", arr, doc_of, keep);
fail:
  if (inner)
    for (Py_ssize_t d = 0; d < nd; ++d) Py_XDECREF(inner[d]);
  PyMem_Free(inner);
  Py_XDECREF(arr);
  Py_XDECREF(doc_of);
  Py_XDECREF(keep);
  Py_DECREF(outer);
  return NULL;
}

static PyMethodDef methods[] = {
    {"bufs", py_bufs, METH_O, "ycrdt_buf array over a sequence of bytes (no copy)"},
    {"docs", py_docs, METH_O, "ycrdt_buf array + document index over a list of update lists (no copy)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_ycpack", NULL, -1, methods};

PyMODINIT_FUNC PyInit__ycpack(void) { return PyModule_Create(&mod); }
