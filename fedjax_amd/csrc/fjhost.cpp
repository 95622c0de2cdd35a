// fjhost.cpp — native host side of the pytree aggregation path (CPython extension).
//
// tree_mean over separate client pytrees (fedjax/core/tree_util.py:76-96, called from
// examples/fed_avg.py:82 and aggregator.py:100) spends its host time walking K pytrees
// and reading, per (client, leaf), the tensor's type / dtype / device / contiguity /
// shape and device pointer. In Python that is five attribute calls per leaf; here it
// is a handful of loads from the TensorImpl. The GPU arithmetic stays in libfjagg.so
// (include/fjagg.h); this module only builds the kernel's pointer table and weight
// vector, and never touches device memory.
//
// Everything here answers "the fast case holds" or "it does not": on any mismatch
// (structure, leaf type, dtype, shape, device, layout, an unusual weight) the caller
// falls back to the Python path, which converts what it can and raises the reference's
// errors (ValueError / TypeError). So this module never decides an error itself.
//
// Entry points (all positional):
//   gather_rows(trees, k0, spec, row0, dev_index, ptrs) -> int
//       Walk trees[k0:] against `spec` (pytree.native_spec of client 0's TreeDef) and
//       write the device pointer of client k's leaf l to ptrs[k*L + l] (int64 buffer),
//       for k = k0 .. len(trees)-1, L = len(row0). Every leaf must be a torch.Tensor on
//       cuda:dev_index (-1: host tensors, for the CPU tests), strided and contiguous,
//       with row0[l]'s dtype and shape. Also writes row0's pointers to row 0 when k0 == 1.
//       Returns 0, or -(k+1) for the first client k that does not match.
//   leaf_versions(trees, spec, L, out) -> int
//       out[k*L + l] = Tensor._version of client k's leaf l (torch's in-place modification
//       counter), walking every tree against `spec`; any tensor type. 0, or -(k+1) for the
//       first client whose structure differs. RunningMean records these at add() and checks
//       them before the buffered deltas are read (a delta updated in place after add()).
//   fold_weights(weights, f32_out, i32_out_or_None) -> (W, kinds) | None
//       For weights that are all Python int / float (not bool): f32_out[k] =
//       float32(w_k) (numpy's np.float32(w) rounding), i32_out[k] = the int32 wrap of an
//       integer weight (0 for a float one), W = sum(w) accumulated left to right from 0.0
//       in double, exactly as tree_util.py:86,95 (`sum_weight = 0.; sum_weight +=
//       weight`), kinds = bit 0: some weight is a float, bit 1: some weight is an int.
//       None when any weight is something else (numpy scalar, tensor, bool, |w| >=
//       2**53, ...): the caller then uses the Python path.
//   fold_table(row0, ptrs, w_f32, scale, has_scale, nt_min_bytes, dev_index, stream,
//              plan_fn, wsum_fn[, outs, accumulate, wsum_l2_fn, l2_ws_bytes_fn, l2sq])
//       -> (rc, outputs) | None   (l2sq: float32 [K] device tensor -> fjagg_wsum_l2_ptrs)
//       The rest of tree_mean's host work for a gathered table (ptrs from gather_rows,
//       weights from fold_weights) when every leaf is float32 and every pointer is
//       16-byte aligned: fresh output leaves shaped like row0, the plan image of
//       include/fjagg.h in pinned memory (workgroup table from fjagg_ptrs_plan), its
//       stream-ordered upload, and the fjagg_wsum_ptrs launch on `stream` (FJAGG_SCALE if
//       has_scale, FJAGG_NONTEMPORAL if the clients' bytes reach nt_min_bytes). rc is the
//       library's status. None (nothing launched) outside that case: the caller's Python
//       path then handles it.

#include <Python.h>

#include <ATen/ATen.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Walk {
  const std::vector<at::ScalarType>* dtypes;  // nullptr: record versions only (leaf_versions)
  const std::vector<c10::IntArrayRef>* sizes;
  c10::DeviceIndex dev;
  int64_t* out;  // row of L pointers (or L versions)
  size_t leaf;
  size_t cap = 0;  // leaf_versions: slots in the row
};

enum { kLeaf = 0, kNone = 1, kDict = 2, kList = 3, kTuple = 4 };

// 0: matches; 1: mismatch (no Python error set); -1: Python error set.
int leaf(PyObject* x, Walk& w) {
  if (w.dtypes == nullptr) {  // leaf_versions: any tensor, its in-place modification counter
    if (!THPVariable_Check(x) || w.leaf >= w.cap) return 1;
    w.out[w.leaf++] = static_cast<int64_t>(THPVariable_Unpack(x)._version());
    return 0;
  }
  if (Py_TYPE(x) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) return 1;
  size_t l = w.leaf++;
  if (l >= w.dtypes->size()) return 1;
  const at::Tensor& t = THPVariable_Unpack(x);
  if (t.layout() != c10::kStrided) return 1;
  if (w.dev >= 0 ? (!t.is_cuda() || t.get_device() != w.dev) : !t.is_cpu()) return 1;
  if (t.scalar_type() != (*w.dtypes)[l] || t.sizes() != (*w.sizes)[l] || !t.is_contiguous()) return 1;
  w.out[l] = reinterpret_cast<int64_t>(t.data_ptr());
  return 0;
}

int walk(PyObject* spec, PyObject* x, Walk& w) {
  if (PyLong_CheckExact(spec)) {
    long k = PyLong_AsLong(spec);
    if (k == kLeaf) return leaf(x, w);
    if (k == kNone) return x == Py_None ? 0 : 1;
    return 1;
  }
  if (!PyTuple_CheckExact(spec) || PyTuple_GET_SIZE(spec) != 3) return 1;
  long kind = PyLong_AsLong(PyTuple_GET_ITEM(spec, 0));
  PyObject* aux = PyTuple_GET_ITEM(spec, 1);
  PyObject* children = PyTuple_GET_ITEM(spec, 2);
  Py_ssize_t n = PyTuple_GET_SIZE(children);
  if (kind == kDict) {
    if (!PyDict_CheckExact(x) || PyDict_GET_SIZE(x) != n) return 1;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* v = PyDict_GetItemWithError(x, PyTuple_GET_ITEM(aux, i));  // borrowed
      if (v == nullptr) {
        if (PyErr_Occurred()) PyErr_Clear();  // e.g. an unhashable comparison: a mismatch
        return 1;
      }
      int rc = walk(PyTuple_GET_ITEM(children, i), v, w);
      if (rc) return rc;
    }
    return 0;
  }
  if (kind == kList || kind == kTuple) {
    bool ok = kind == kList ? PyList_CheckExact(x) : PyTuple_CheckExact(x);
    if (!ok || Py_SIZE(x) != n) return 1;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* v = kind == kList ? PyList_GET_ITEM(x, i) : PyTuple_GET_ITEM(x, i);
      int rc = walk(PyTuple_GET_ITEM(children, i), v, w);
      if (rc) return rc;
    }
    return 0;
  }
  return 1;
}

PyObject* gather_rows(PyObject*, PyObject* args) {
  PyObject *trees, *spec, *row0, *ptrs;
  Py_ssize_t k0;
  int dev;
  if (!PyArg_ParseTuple(args, "O!nOO!iO", &PyList_Type, &trees, &k0, &spec, &PyList_Type, &row0, &dev, &ptrs))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(trees), L = PyList_GET_SIZE(row0);
  if (k0 < 0 || k0 > K) {
    PyErr_SetString(PyExc_ValueError, "gather_rows: k0 out of range");
    return nullptr;
  }
  Py_buffer buf;
  if (PyObject_GetBuffer(ptrs, &buf, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  struct Release {
    Py_buffer* b;
    ~Release() { PyBuffer_Release(b); }
  } release{&buf};
  if (buf.len < static_cast<Py_ssize_t>(sizeof(int64_t)) * K * L) {
    PyErr_SetString(PyExc_ValueError, "gather_rows: pointer buffer smaller than K*L int64");
    return nullptr;
  }
  auto* out = static_cast<int64_t*>(buf.buf);
  try {
    std::vector<at::ScalarType> dtypes;
    std::vector<c10::IntArrayRef> sizes;
    dtypes.reserve(L);
    sizes.reserve(L);
    for (Py_ssize_t l = 0; l < L; ++l) {
      PyObject* x = PyList_GET_ITEM(row0, l);
      if (!THPVariable_Check(x)) {
        PyErr_SetString(PyExc_TypeError, "gather_rows: row0 must hold tensors");
        return nullptr;
      }
      const at::Tensor& t = THPVariable_Unpack(x);
      dtypes.push_back(t.scalar_type());
      sizes.push_back(t.sizes());
      if (k0 == 1) out[l] = reinterpret_cast<int64_t>(t.data_ptr());
    }
    Walk w{&dtypes, &sizes, static_cast<c10::DeviceIndex>(dev), nullptr, 0};
    for (Py_ssize_t k = k0; k < K; ++k) {
      w.out = out + k * L;
      w.leaf = 0;
      int rc = walk(spec, PyList_GET_ITEM(trees, k), w);
      if (rc < 0) return nullptr;
      if (rc > 0 || w.leaf != static_cast<size_t>(L)) return PyLong_FromSsize_t(-(k + 1));
    }
    return PyLong_FromLong(0);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyObject* leaf_versions(PyObject*, PyObject* args) {
  PyObject *trees, *spec, *vers;
  Py_ssize_t L;
  if (!PyArg_ParseTuple(args, "O!OnO", &PyList_Type, &trees, &spec, &L, &vers)) return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(trees);
  Py_buffer buf;
  if (PyObject_GetBuffer(vers, &buf, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  struct Release {
    Py_buffer* b;
    ~Release() { PyBuffer_Release(b); }
  } release{&buf};
  if (L < 0 || buf.len < static_cast<Py_ssize_t>(sizeof(int64_t)) * K * L) {
    PyErr_SetString(PyExc_ValueError, "leaf_versions: version buffer smaller than K*L int64");
    return nullptr;
  }
  Walk w{nullptr, nullptr, 0, nullptr, 0, static_cast<size_t>(L)};
  for (Py_ssize_t k = 0; k < K; ++k) {
    w.out = static_cast<int64_t*>(buf.buf) + k * L;
    w.leaf = 0;
    int rc = walk(spec, PyList_GET_ITEM(trees, k), w);
    if (rc < 0) return nullptr;
    if (rc > 0 || w.leaf != static_cast<size_t>(L)) return PyLong_FromSsize_t(-(k + 1));
  }
  return PyLong_FromLong(0);
}

PyObject* fold_weights(PyObject*, PyObject* args) {
  PyObject *weights, *f32, *i32;
  if (!PyArg_ParseTuple(args, "O!OO", &PyList_Type, &weights, &f32, &i32)) return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(weights);
  Py_buffer bf, bi;
  if (PyObject_GetBuffer(f32, &bf, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  bool have_i = i32 != Py_None;
  if (have_i && PyObject_GetBuffer(i32, &bi, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) {
    PyBuffer_Release(&bf);
    return nullptr;
  }
  PyObject* result = nullptr;
  if (bf.len < 4 * K || (have_i && bi.len < 4 * K)) {
    PyErr_SetString(PyExc_ValueError, "fold_weights: output buffers smaller than K");
  } else {
    auto* fo = static_cast<float*>(bf.buf);
    auto* io = have_i ? static_cast<int32_t*>(bi.buf) : nullptr;
    double W = 0.0;
    long kinds = 0;
    bool simple = true;
    for (Py_ssize_t k = 0; k < K && simple; ++k) {
      PyObject* w = PyList_GET_ITEM(weights, k);
      double d;
      if (PyLong_CheckExact(w)) {
        int overflow = 0;
        long long v = PyLong_AsLongLongAndOverflow(w, &overflow);
        // |v| < 2**53: the double is exact, so float(double) is numpy's single rounding
        if (overflow || v >= (1LL << 53) || v <= -(1LL << 53)) {
          simple = false;
          break;
        }
        d = static_cast<double>(v);
        if (io) io[k] = static_cast<int32_t>(static_cast<uint32_t>(static_cast<uint64_t>(v)));
        kinds |= 2;
      } else if (PyFloat_CheckExact(w)) {
        d = PyFloat_AS_DOUBLE(w);
        if (io) io[k] = 0;  // int32 folds take integer weights only; the caller checks the kinds
        kinds |= 1;
      } else {
        simple = false;
        break;
      }
      fo[k] = static_cast<float>(d);
      W += d;  // tree_util.py:95, Python float + int / float
    }
    if (PyErr_Occurred()) {
      result = nullptr;
    } else if (simple) {
      result = Py_BuildValue("(dl)", W, kinds);
    } else {
      Py_INCREF(Py_None);
      result = Py_None;
    }
  }
  PyBuffer_Release(&bf);
  if (have_i) PyBuffer_Release(&bi);
  return result;
}

// fjagg_ptrs_plan_leaves / fjagg_wsum_ptrs of libfjagg.so (include/fjagg.h), passed in by address
typedef int64_t (*PlanFn)(int, int, const int64_t*, const uint8_t*, int, int64_t*, int64_t);
typedef int (*WsumFn)(int, int, int, const int64_t*, int, int64_t, int64_t, const void*, float, int, void*);
typedef int64_t (*L2WsFn)(int64_t, int64_t);
typedef int (*WsumL2Fn)(int, int, int, const int64_t*, int, int64_t, int64_t, const void*, float, float*, int, void*,
                        int64_t, void*);
constexpr int kF32 = 0, kScale = 1, kAccumulate = 2, kNontemporal = 4;  // fjagg.h enums

PyObject* fold_table(PyObject*, PyObject* args) {
  PyObject *row0, *ptrs, *wf, *dst = Py_None, *l2sq = Py_None;
  double scale, nt_min_bytes;
  int has_scale, dev, accumulate = 0;
  unsigned long long stream, plan_addr, wsum_addr, l2_addr = 0, l2ws_addr = 0;
  if (!PyArg_ParseTuple(args, "O!OOdidiKKK|OiKKO", &PyList_Type, &row0, &ptrs, &wf, &scale, &has_scale,
                        &nt_min_bytes, &dev, &stream, &plan_addr, &wsum_addr, &dst, &accumulate, &l2_addr,
                        &l2ws_addr, &l2sq))
    return nullptr;
  const bool with_l2 = l2sq != Py_None;
  if (with_l2 && (!THPVariable_Check(l2sq) || !l2_addr || !l2ws_addr)) Py_RETURN_NONE;
  const Py_ssize_t L = PyList_GET_SIZE(row0);
  if (dst != Py_None && (!PyList_Check(dst) || PyList_GET_SIZE(dst) != L)) Py_RETURN_NONE;
  if (accumulate && dst == Py_None) Py_RETURN_NONE;
  Py_buffer bp, bw;
  if (PyObject_GetBuffer(ptrs, &bp, PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  if (PyObject_GetBuffer(wf, &bw, PyBUF_C_CONTIGUOUS) != 0) {
    PyBuffer_Release(&bp);
    return nullptr;
  }
  struct Release {
    Py_buffer *a, *b;
    ~Release() {
      PyBuffer_Release(a);
      PyBuffer_Release(b);
    }
  } release{&bp, &bw};
  if (L < 1 || bp.len % (8 * L) != 0) Py_RETURN_NONE;
  const int64_t K = bp.len / (8 * L);
  if (K < 1 || bw.len < 4 * K) Py_RETURN_NONE;
  const auto* in = static_cast<const int64_t*>(bp.buf);
  try {
    if (with_l2) {
      const at::Tensor& q = THPVariable_Unpack(l2sq);
      if (q.scalar_type() != at::kFloat || q.numel() != K || !q.is_contiguous() || !q.is_cuda() ||
          q.get_device() != dev)
        Py_RETURN_NONE;
    }
    // fast case only: float32 leaves (fold type and output type are then float32 for any
    // weights). A leaf with a client pointer off 16 bytes walks element units (per-leaf
    // plan); the outputs are fresh allocations, so aligned.
    std::vector<int64_t> leaf_n(L);
    int64_t total = 0;
    for (Py_ssize_t l = 0; l < L; ++l) {
      const at::Tensor& t = THPVariable_Unpack(PyList_GET_ITEM(row0, l));
      if (t.scalar_type() != at::kFloat) Py_RETURN_NONE;
      leaf_n[l] = t.numel();
      total += leaf_n[l];
    }
    if (total == 0) Py_RETURN_NONE;  // only empty leaves: the Python path (no launch at all)
    std::vector<int64_t> lbits(L, 0);
    for (int64_t k = 0; k < K; ++k)
      for (Py_ssize_t l = 0; l < L; ++l) lbits[l] |= in[k * L + l];
    std::vector<at::Tensor> outs;
    outs.reserve(L);
    std::vector<uint8_t> elem(L, 0);
    bool any_elem = false;
    for (Py_ssize_t l = 0; l < L; ++l) {
      const at::Tensor& t = THPVariable_Unpack(PyList_GET_ITEM(row0, l));
      if (dst != Py_None) {  // caller's destinations: float32, contiguous, row0's shape and device
        PyObject* o = PyList_GET_ITEM(dst, l);
        if (!THPVariable_Check(o)) Py_RETURN_NONE;
        const at::Tensor& d = THPVariable_Unpack(o);
        if (d.scalar_type() != at::kFloat || !d.is_contiguous() || d.sizes() != t.sizes() || d.device() != t.device())
          Py_RETURN_NONE;
        outs.push_back(d);
      } else {
        outs.push_back(at::empty(t.sizes(), t.options()));
      }
      elem[l] = ((lbits[l] | reinterpret_cast<int64_t>(outs.back().data_ptr())) & 15) != 0;
      any_elem = any_elem || elem[l];
    }
    auto plan = reinterpret_cast<PlanFn>(plan_addr);
    const uint8_t* mask = any_elem ? elem.data() : nullptr;
    const int64_t nblk = plan(kF32, 0, leaf_n.data(), mask, static_cast<int>(L), nullptr, 0);
    if (nblk < 0) Py_RETURN_NONE;
    // plan image (fjagg.h): in_ptrs[K*L] | out_ptrs[L] | leaf_n[L] | blocks[2*nblk] | f32 weights
    const int64_t nw = (K + 1) / 2, n = K * L + 2 * L + 2 * nblk + nw;
    at::Tensor img = at::empty({n}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
    int64_t* p = img.data_ptr<int64_t>();
    std::memcpy(p, in, sizeof(int64_t) * K * L);
    for (Py_ssize_t l = 0; l < L; ++l) {
      p[K * L + l] = reinterpret_cast<int64_t>(outs[l].data_ptr());
      p[K * L + L + l] = leaf_n[l];
    }
    if (plan(kF32, 0, leaf_n.data(), mask, static_cast<int>(L), p + K * L + 2 * L, nblk) != nblk) Py_RETURN_NONE;
    p[n - 1] = 0;
    std::memcpy(p + n - nw, bw.buf, 4 * K);
    at::Tensor dimg = img.to(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(dev)), /*non_blocking=*/true);
    const bool nt = static_cast<double>(total) * K * 4 >= nt_min_bytes;
    const int flags = (has_scale ? kScale : 0) | (nt ? kNontemporal : 0) | (accumulate ? kAccumulate : 0);
    const int64_t* dp = dimg.data_ptr<int64_t>();
    int rc;
    if (with_l2) {  // fused per-client squared l2 norms (fjagg_wsum_l2_ptrs), workspace from torch's allocator
      const at::Tensor& q = THPVariable_Unpack(l2sq);
      const int64_t need = reinterpret_cast<L2WsFn>(l2ws_addr)(K, nblk);
      if (need < 0) Py_RETURN_NONE;
      at::Tensor ws = at::empty({need > 4 ? need : 4}, dimg.options().dtype(at::kByte));
      rc = reinterpret_cast<WsumL2Fn>(l2_addr)(kF32, kF32, kF32, dp, static_cast<int>(L), K, nblk, dp + (n - nw),
                                               static_cast<float>(scale), q.data_ptr<float>(), flags,
                                               ws.data_ptr(), ws.numel(), reinterpret_cast<void*>(stream));
    } else {
      rc = reinterpret_cast<WsumFn>(wsum_addr)(kF32, kF32, kF32, dp, static_cast<int>(L), K, nblk, dp + (n - nw),
                                               static_cast<float>(scale), flags, reinterpret_cast<void*>(stream));
    }
    PyObject* list = PyList_New(L);
    if (!list) return nullptr;
    for (Py_ssize_t l = 0; l < L; ++l) PyList_SET_ITEM(list, l, THPVariable_Wrap(std::move(outs[l])));
    return Py_BuildValue("(iN)", rc, list);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyMethodDef kMethods[] = {
    {"gather_rows", gather_rows, METH_VARARGS, "pointer table of K client pytrees (see fjhost.cpp)"},
    {"leaf_versions", leaf_versions, METH_VARARGS, "torch in-place version counters of K pytrees' leaves"},
    {"fold_weights", fold_weights, METH_VARARGS, "f32/i32 weights and W of Python-number weights"},
    {"fold_table", fold_table, METH_VARARGS, "plan image + output leaves + fjagg_wsum_ptrs launch (see fjhost.cpp)"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fjhost", "native host side of the pytree aggregation path",
                       -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fjhost(void) { return PyModule_Create(&kModule); }
