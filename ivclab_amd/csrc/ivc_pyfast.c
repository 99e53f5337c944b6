/* ivc_pyfast.c — the per-block calls of the drop-in classes in one C step (CPython + NumPy C
 * API).  The reference's exercises call DiscreteCosineTransform.transform on one (8, 8) block
 * and PatchQuant.quantize on one (3, 8, 8) stack per loop iteration
 * (exercises/ch3/E3-1_claude.py:47-60); through ctypes the argument checks and conversions
 * cost ~1.5 us of a ~10 us call.  These functions take the NumPy array, check that it is a
 * small C-contiguous array of a kernel dtype, allocate the result and call the C-ABI entry
 * point (its address handed over by ivclab_amd._native, so the process's one libivc instance
 * runs).  They return None for anything else and the Python path handles it; a failing call
 * returns the status code, which the caller turns into the library's exception.
 * Built by ivclab_amd/build.py with gcc (no HIP code here).  Host side only. */
#define PY_SSIZE_T_CLEAN
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <Python.h>
#include <numpy/arrayobject.h>
#include <stdint.h>

typedef int (*dct_fn)(const void*, int, int64_t, void*, int, int, int);
typedef int (*quant_fn)(const void*, int, int64_t, int, const double*, int, int32_t*);

static dct_fn g_dct;
static quant_fn g_quant, g_dequant;

/* ivc_dtype codes (include/ivc.h) of the NumPy type numbers, 0: not a kernel dtype */
static int dtype_code(PyArrayObject* a) {
  PyArray_Descr* d = PyArray_DESCR(a);
  if (PyArray_ISBYTESWAPPED(a)) return 0;
  switch (d->type_num) {
    case NPY_UINT8: return 1;
    case NPY_INT8: return 2;
    case NPY_UINT16: return 3;
    case NPY_INT16: return 4;
    case NPY_UINT32: return 5;
    case NPY_INT32: return 6;
    case NPY_UINT64: return 7;
    case NPY_INT64: return 8;
    case NPY_FLOAT32: return 9;
    case NPY_FLOAT64: return 10;
    default:
      /* long long on LP64 (a type number of its own, the same 8 bytes) */
      if (d->type_num == NPY_LONGLONG && sizeof(long long) == 8) return 8;
      if (d->type_num == NPY_ULONGLONG && sizeof(long long) == 8) return 7;
      return 0;
  }
}

/* the array when it is an exact ndarray, C-contiguous, aligned, with trailing (8, 8) and at
 * most max_elems elements (> 0); NULL otherwise */
static PyArrayObject* small_blocks(PyObject* o, npy_intp max_elems) {
  if (Py_TYPE(o) != &PyArray_Type) return NULL;
  PyArrayObject* a = (PyArrayObject*)o;
  const int nd = PyArray_NDIM(a);
  if (nd < 2) return NULL;
  const npy_intp* s = PyArray_DIMS(a);
  if (s[nd - 1] != 8 || s[nd - 2] != 8) return NULL;
  const npy_intp n = PyArray_SIZE(a);
  if (n <= 0 || n > max_elems) return NULL;
  if (!PyArray_IS_C_CONTIGUOUS(a) || !PyArray_ISALIGNED(a)) return NULL;
  return a;
}

/* set_entry_points(dct8x8, quantize, dequantize): the C-ABI addresses */
static PyObject* set_entry_points(PyObject* self, PyObject* args) {
  unsigned long long d, q, dq;
  if (!PyArg_ParseTuple(args, "KKK", &d, &q, &dq)) return NULL;
  g_dct = (dct_fn)(uintptr_t)d;
  g_quant = (quant_fn)(uintptr_t)q;
  g_dequant = (quant_fn)(uintptr_t)dq;
  Py_RETURN_NONE;
}

/* dct8x8(x, norm_code, inverse) -> out | status | None (dct.py:12-46: float32 stays float32,
 * every other dtype computes in float64) */
static PyObject* dct8x8(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3 || !g_dct) Py_RETURN_NONE;
  PyArrayObject* a = small_blocks(args[0], 4096);
  if (!a) Py_RETURN_NONE;
  const int code = dtype_code(a);
  if (!code) Py_RETURN_NONE;
  const long norm = PyLong_AsLong(args[1]), inv = PyLong_AsLong(args[2]);
  if (PyErr_Occurred()) return NULL;
  const int ocode = code == 9 ? 9 : 10;
  PyArrayObject* out = (PyArrayObject*)PyArray_EMPTY(PyArray_NDIM(a), PyArray_DIMS(a),
                                                     ocode == 9 ? NPY_FLOAT32 : NPY_FLOAT64, 0);
  if (!out) return NULL;
  int st;
  Py_BEGIN_ALLOW_THREADS
  st = g_dct(PyArray_DATA(a), code, (int64_t)(PyArray_SIZE(a) / 64), PyArray_DATA(out), ocode,
             (int)inv, (int)norm);
  Py_END_ALLOW_THREADS
  if (st) {
    Py_DECREF(out);
    return PyLong_FromLong(st);
  }
  return (PyObject*)out;
}

/* quant(dequantize, x, table_address, table_code) -> out | status | None, for a float32 (9) or
 * float64 (10) table (patchquant.py:44-78: the arithmetic is NumPy's result type of the two
 * arrays — float32 only for a float32 table with <= 16-bit integers or float32; C = 1
 * broadcasts over the 3 planes; the result is [..., 3, 8, 8] int32 with at least 5
 * dimensions, as the reference's broadcasting gives) */
static PyObject* quant(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 4 || !g_quant || !g_dequant) Py_RETURN_NONE;
  const int deq = PyObject_IsTrue(args[0]);
  PyArrayObject* a = small_blocks(args[1], 12288);
  if (!a) Py_RETURN_NONE;
  const int code = dtype_code(a);
  if (!code) Py_RETURN_NONE;
  const int nd = PyArray_NDIM(a);
  const npy_intp* s = PyArray_DIMS(a);
  const int C = nd == 2 ? 1 : (int)s[nd - 3];
  if (C != 1 && C != 3) Py_RETURN_NONE;
  const unsigned long long tab = PyLong_AsUnsignedLongLong(args[2]);
  const long tcode = PyLong_AsLong(args[3]);
  if (PyErr_Occurred()) return NULL;
  if (tcode != 9 && tcode != 10) Py_RETURN_NONE;
  const int cc = (tcode == 9 && (code <= 4 || code == 9)) ? 9 : 10;
  /* output: the leading dimensions, then (3, 8, 8), padded in front with 1s to 5 dimensions */
  npy_intp od[NPY_MAXDIMS];
  const int lead = nd > 3 ? nd - 3 : 0;
  const int ond = lead + 3 < 5 ? 5 : lead + 3;
  int k = 0;
  for (; k < ond - lead - 3; ++k) od[k] = 1;
  for (int i = 0; i < lead; ++i) od[k++] = s[i];
  od[k++] = 3;
  od[k++] = 8;
  od[k++] = 8;
  PyArrayObject* out = (PyArrayObject*)PyArray_EMPTY(ond, od, NPY_INT32, 0);
  if (!out) return NULL;
  const int64_t nblk = (int64_t)(PyArray_SIZE(out) / 192);
  int st;
  quant_fn f = deq ? g_dequant : g_quant;
  Py_BEGIN_ALLOW_THREADS
  st = f(PyArray_DATA(a), code, nblk, C, (const double*)(uintptr_t)tab, cc,
         (int32_t*)PyArray_DATA(out));
  Py_END_ALLOW_THREADS
  if (st) {
    Py_DECREF(out);
    return PyLong_FromLong(st);
  }
  return (PyObject*)out;
}

/* an (8, 8) table operand: an exact, C-contiguous, aligned, host-order ndarray of float32
 * (*kind = 1), float64 (2) or int64 (3) */
static const void* table_block(PyObject* o, int* kind) {
  if (Py_TYPE(o) != &PyArray_Type) return NULL;
  PyArrayObject* a = (PyArrayObject*)o;
  if (PyArray_NDIM(a) != 2 || PyArray_DIMS(a)[0] != 8 || PyArray_DIMS(a)[1] != 8) return NULL;
  if (PyArray_ISBYTESWAPPED(a) || !PyArray_IS_C_CONTIGUOUS(a) || !PyArray_ISALIGNED(a)) return NULL;
  const int t = PyArray_DESCR(a)->type_num;
  if (t == NPY_FLOAT32) {
    *kind = 1;
  } else if (t == NPY_FLOAT64) {
    *kind = 2;
  } else if (PyArray_ITEMSIZE(a) == 8 && (t == NPY_LONG || t == NPY_LONGLONG)) {
    *kind = 3;
  } else {
    return NULL;
  }
  return PyArray_DATA(a);
}

static double table_value(const void* p, int kind, int i) {
  return kind == 1 ? (double)((const float*)p)[i]
                   : kind == 2 ? ((const double*)p)[i] : (double)((const int64_t*)p)[i];
}

/* quant_lc(dequantize, x, luminance, chrominance, scale) -> out | status | None: the table
 * formed here as PatchQuant.get_quantization_table forms it (patchquant.py:39-42:
 * stack([lum, chrom, chrom]) * scale), under NumPy 2's promotion rules, when that is a float32
 * or float64 table.  The stack is float32 when both tables are, int64 when both are int64,
 * float64 otherwise.  A Python float or int scale is weak (it takes the stack's type: float32
 * multiplies in float32, an int64 stack times an int stays int64 and is declined); a float64
 * scalar is strong (the product is float64).  Ints are taken up to 2^24 (float32) / 2^53
 * (float64) in magnitude, where the conversion is exact.  NumPy converts each entry to the
 * result type and multiplies element by element, so every entry is the same correctly rounded
 * value as here.  None for anything else (other scale types, other table dtypes or layouts). */
static PyObject* quant_lc(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 5 || !g_quant || !g_dequant) Py_RETURN_NONE;
  int lk = 0, ck = 0;
  const void* lum = table_block(args[2], &lk);
  const void* chrom = table_block(args[3], &ck);
  if (!lum || !chrom) Py_RETURN_NONE;
  const int stack = lk == ck ? lk : 2;                 /* 1 float32, 2 float64, 3 int64 */
  PyObject* so = args[4];
  double sc;
  int f32;                                             /* the table's type: float32 or float64 */
  if (PyFloat_CheckExact(so)) {
    sc = PyFloat_AS_DOUBLE(so);
    f32 = stack == 1;
  } else if (PyFloat_Check(so) && PyArray_IsScalar(so, Double)) {
    sc = PyFloat_AS_DOUBLE(so);
    f32 = 0;
  } else if (PyLong_CheckExact(so) && stack != 3) {
    int ovf = 0;
    const long long v = PyLong_AsLongLongAndOverflow(so, &ovf);
    const long long lim = stack == 1 ? (1LL << 24) : (1LL << 53);
    if (ovf || v > lim || v < -lim) Py_RETURN_NONE;
    sc = (double)v;
    f32 = stack == 1;
  } else {
    Py_RETURN_NONE;
  }
  double tab[192];
  if (f32) {
    const volatile float s32 = (float)sc;
    for (int i = 0; i < 64; ++i) {
      const volatile float pl = ((const float*)lum)[i] * s32;
      const volatile float pc = ((const float*)chrom)[i] * s32;
      tab[i] = pl;
      tab[64 + i] = tab[128 + i] = pc;
    }
  } else {
    for (int i = 0; i < 64; ++i) {
      tab[i] = table_value(lum, lk, i) * sc;
      tab[64 + i] = tab[128 + i] = table_value(chrom, ck, i) * sc;
    }
  }
  PyObject* a4[4];
  a4[0] = args[0];
  a4[1] = args[1];
  PyObject* addr = PyLong_FromUnsignedLongLong((unsigned long long)(uintptr_t)tab);
  PyObject* code = PyLong_FromLong(f32 ? 9 : 10);
  if (!addr || !code) {
    Py_XDECREF(addr);
    Py_XDECREF(code);
    return NULL;
  }
  a4[2] = addr;
  a4[3] = code;
  PyObject* r = quant(self, a4, 4);
  Py_DECREF(addr);
  Py_DECREF(code);
  return r;
}

static PyMethodDef methods[] = {
    {"set_entry_points", set_entry_points, METH_VARARGS, "the C-ABI entry points"},
    {"dct8x8", (PyCFunction)(void (*)(void))dct8x8, METH_FASTCALL, "one-step DCT of small arrays"},
    {"quant", (PyCFunction)(void (*)(void))quant, METH_FASTCALL,
     "one-step (de)quantisation of small arrays"},
    {"quant_lc", (PyCFunction)(void (*)(void))quant_lc, METH_FASTCALL,
     "one-step (de)quantisation with the table formed from luminance, chrominance and scale"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_ivcfast", NULL, -1, methods};

PyMODINIT_FUNC PyInit__ivcfast(void) {
  import_array();
  return PyModule_Create(&module);
}
