// fjhost.cpp — native host side of the pytree aggregation path (CPython extension).
//
// tree_mean over separate client pytrees (fedjax/core/tree_util.py:76-96, called from
// examples/fed_avg.py:82 and aggregator.py:73) spends its host time walking K pytrees
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
//   gather_rows(trees, k0, spec, row0, dev_index, ptrs[, k1]) -> int
//       Walk trees[k0:k1] (k1 defaults to len(trees)) against `spec` (pytree.native_spec
//       of client 0's TreeDef) and write the device pointer of client k's leaf l to
//       ptrs[k*L + l] (int64 buffer), for k = k0 .. k1-1, L = len(row0). Every leaf must be a torch.Tensor on
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
#include <structmember.h>

#include <ATen/ATen.h>
#include <c10/hip/HIPFunctions.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/python_variable.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <unordered_map>
#include <vector>

#include "fjagg.h"
#include "fjtree.h"

namespace {

// Host phase timers of fold_table (host_timers() reads and resets them): where the
// per-call host time of tree_mean goes (tools/prof_tree_mean_host.py).
enum { kTSpec, kTChecks, kTOutputs, kTPlan, kTImage, kTUpload, kTLaunch, kTWrap, kTFirstLaunch, kTPhases };
double g_timers[kTPhases] = {};
long long g_timer_calls = 0;
// how fold_table's plan images reached the kernel: in the kernel arguments, or through a
// pinned staging buffer + upload (image too large, or a plan the kernarg kernels lack)
long long g_image_karg = 0, g_image_upload = 0;
struct Stamp {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(int phase) {
    auto n = std::chrono::steady_clock::now();
    g_timers[phase] += std::chrono::duration<double, std::micro>(n - t).count();
    t = n;
  }
};

// torch's in-place version counter of t. Inference tensors (torch.inference_mode) carry
// none (_version() throws): kNoVersion, and the callers that need a guard (capture,
// append_check, RunningMean) treat such a leaf as "cannot be deferred by reference".
constexpr int64_t kNoVersion = -2;
inline int64_t version_of(const at::Tensor& t) {
  return t.is_inference() ? kNoVersion : static_cast<int64_t>(t._version());
}

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
    w.out[w.leaf++] = version_of(THPVariable_Unpack(x));
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

// The leaf objects of x against spec, appended to objs (tensor leaves by exact type only; no
// tensor field is read): 0 walked, 1 mismatch, -1 Python error set.
int collect(PyObject* spec, PyObject* x, std::vector<PyObject*>& objs) {
  if (PyLong_CheckExact(spec)) {
    const long k = PyLong_AsLong(spec);
    if (k == kLeaf) {
      if (Py_TYPE(x) != reinterpret_cast<PyTypeObject*>(THPVariableClass)) return 1;
      objs.push_back(x);
      return 0;
    }
    if (k == kNone) return x == Py_None ? 0 : 1;
    return 1;
  }
  if (!PyTuple_CheckExact(spec) || PyTuple_GET_SIZE(spec) != 3) return 1;
  const long kind = PyLong_AsLong(PyTuple_GET_ITEM(spec, 0));
  PyObject* aux = PyTuple_GET_ITEM(spec, 1);
  PyObject* children = PyTuple_GET_ITEM(spec, 2);
  const Py_ssize_t n = PyTuple_GET_SIZE(children);
  if (kind == kDict) {
    if (!PyDict_CheckExact(x) || PyDict_GET_SIZE(x) != n) return 1;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* v = PyDict_GetItemWithError(x, PyTuple_GET_ITEM(aux, i));  // borrowed
      if (v == nullptr) {
        if (PyErr_Occurred()) PyErr_Clear();  // e.g. an unhashable comparison: a mismatch
        return 1;
      }
      if (int rc = collect(PyTuple_GET_ITEM(children, i), v, objs)) return rc;
    }
    return 0;
  }
  if (kind == kList || kind == kTuple) {
    const bool ok = kind == kList ? PyList_CheckExact(x) : PyTuple_CheckExact(x);
    if (!ok || Py_SIZE(x) != n) return 1;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* v = kind == kList ? PyList_GET_ITEM(x, i) : PyTuple_GET_ITEM(x, i);
      if (int rc = collect(PyTuple_GET_ITEM(children, i), v, objs)) return rc;
    }
    return 0;
  }
  return 1;
}

// Clients trees[k0, k1) against spec: every leaf a strided tensor on cuda:dev (dev < 0: on
// the host), of dtypes[l] / sizes[l], contiguous; its data pointer goes to rows[k * L + l].
// Walked in batches of 16 clients (collect the leaf objects, then check them; prefetching the
// TensorImpl / StorageImpl lines between the two measured no gain, profiles/r04j_pool/host.json).
// 0: all match; k + 1: client k
// is the first that does not; -1: a Python error is set.
int64_t gather_clients(PyObject* spec, PyObject* const* trees, int64_t k0, int64_t k1,
                       const std::vector<at::ScalarType>& dtypes, const std::vector<c10::IntArrayRef>& sizes,
                       c10::DeviceIndex dev, int64_t* rows) {
  const size_t L = dtypes.size();
  constexpr int64_t B = 16;
  thread_local std::vector<PyObject*> objs;
  for (int64_t b0 = k0; b0 < k1; b0 += B) {
    const int64_t b1 = std::min(k1, b0 + B);
    objs.clear();
    for (int64_t k = b0; k < b1; ++k) {
      const size_t before = objs.size();
      const int rc = collect(spec, trees[k], objs);
      if (rc < 0) return -1;
      if (rc > 0 || objs.size() - before != L) return k + 1;
    }
    for (int64_t k = b0; k < b1; ++k) {
      PyObject* const* row = objs.data() + (k - b0) * L;
      int64_t* out = rows + k * L;
      for (size_t l = 0; l < L; ++l) {
        const at::Tensor& t = THPVariable_Unpack(row[l]);
        if (t.layout() != c10::kStrided) return k + 1;
        if (dev >= 0 ? (!t.is_cuda() || t.get_device() != dev) : !t.is_cpu()) return k + 1;
        if (t.scalar_type() != dtypes[l] || t.sizes() != sizes[l] || !t.is_contiguous()) return k + 1;
        out[l] = reinterpret_cast<int64_t>(t.data_ptr());
      }
    }
  }
  return 0;
}

PyObject* gather_rows(PyObject*, PyObject* args) {
  PyObject *trees, *spec, *row0, *ptrs;
  Py_ssize_t k0, k1 = -1;
  int dev;
  if (!PyArg_ParseTuple(args, "O!nOO!iO|n", &PyList_Type, &trees, &k0, &spec, &PyList_Type, &row0, &dev, &ptrs,
                        &k1))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(trees), L = PyList_GET_SIZE(row0);
  if (k1 < 0) k1 = K;
  if (k0 < 0 || k0 > k1 || k1 > K) {
    PyErr_SetString(PyExc_ValueError, "gather_rows: need 0 <= k0 <= k1 <= len(trees)");
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
    const int64_t r = gather_clients(spec, &PyList_GET_ITEM(trees, 0), k0, k1, dtypes, sizes,
                                     static_cast<c10::DeviceIndex>(dev), out);
    if (r < 0) return nullptr;
    return PyLong_FromLongLong(-r);
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
// fjagg_wsum_l2_ptrs_rows: the norms straight into a chain's two norm rows (operands >= first)
typedef int (*WsumL2RowsFn)(int, int, int, const int64_t*, int, int64_t, int64_t, const void*, float, float*, float*,
                            int64_t, int, void*, int64_t, void*);
struct L2Rows {
  WsumL2RowsFn fn;
  float* sq;
  float* nrm;
  int64_t first;
  bool aligned_only = false;  // fold_core returns 2 (nothing launched) when some leaf would walk element
                              // units: a standalone lazy norm's value must come from the all-16-byte plan
};
constexpr int kF32 = 0, kScale = 1, kAccumulate = 2, kNontemporal = 4;  // fjagg.h enums

// Fresh output leaves shaped like row0: ONE allocation, each leaf its own tensor (own
// TensorImpl and version counter) over a 256-byte aligned slice — one allocator call instead
// of one per leaf on the path to the first launch. A single leaf is a plain allocation.
// The leaves share that storage: one live leaf keeps the whole result's bytes allocated, and
// torch.save of one leaf writes them all (tree_mean's and mean_aggregator's docstrings say so).
void carve_outputs(const std::vector<at::Tensor>& row0, std::vector<at::Tensor>& outs) {
  const size_t L = row0.size();
  if (L == 1) {
    outs.push_back(at::empty(row0[0].sizes(), row0[0].options()));
    return;
  }
  thread_local std::vector<int64_t> offs;
  offs.assign(L + 1, 0);
  const int64_t q = std::max<int64_t>(1, 256 / static_cast<int64_t>(row0[0].element_size()));  // 256 B in elements
  for (size_t l = 0; l < L; ++l) offs[l + 1] = offs[l] + (row0[l].numel() + q - 1) / q * q;
  at::Tensor flat = at::empty({std::max<int64_t>(offs[L], 1)}, row0[0].options());
  for (size_t l = 0; l < L; ++l) {
    at::Tensor t = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(flat.storage()), flat.key_set(),
                                                            flat.dtype());
    t.unsafeGetTensorImpl()->set_storage_offset(offs[l]);
    t.unsafeGetTensorImpl()->set_sizes_contiguous(row0[l].sizes());
    outs.push_back(std::move(t));
  }
}

// The launch part of fold_table for a gathered table: K x L pointers `in` (row 0 = row0's
// leaves), float32 weights wf[K]. outs: empty = fresh outputs shaped like row0 (appended),
// else the destinations (float32, contiguous, row0's shapes and device). Returns 0 with the
// library status in *rc (launched), 1 when the case does not hold (nothing launched), 2 when
// rows->aligned_only and some pointer is off 16 bytes (nothing launched, outs untouched).
// Throws on torch errors.
// The fused-norm workspace of (device, stream): FJAGG_ZEROED_WS layout, its 16-byte completion
// counter zeroed once on the stream when the buffer is (re)allocated and left zero by every
// launch, so the fold's last workgroup adds the norm partials (no combine launch, fjagg.h).
// Launches on one stream are ordered, so they share it; a grown buffer's predecessor goes
// back to torch's stream-ordered allocator.
// `stream` is being captured into a graph (hipStreamIsCapturing: a runtime call, ~0.1 us — asked
// once per fold or per round, never per client)
bool stream_capturing(unsigned long long stream) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(reinterpret_cast<hipStream_t>(stream), &cs) == hipSuccess &&
         cs != hipStreamCaptureStatusNone;
}

at::Tensor l2_workspace(int dev, unsigned long long stream, int64_t need) {
  if (stream_capturing(stream)) {
    // a capture records the zeroing instead of running it: a cached workspace would then reach
    // later launches with its counter unset. A workspace of the capture's own, not cached, zeroed
    // by a fill kernel every replay runs in front of the fold (a recorded hipMemsetAsync node takes
    // effect on the first replay only: measured, tools/probe_memset_node.py)
    return at::zeros({std::max<int64_t>(need, 4096)},
                     at::TensorOptions().dtype(at::kByte).device(at::kCUDA, static_cast<c10::DeviceIndex>(dev)));
  }
  static auto* m = new std::unordered_map<uint64_t, at::Tensor>();
  const uint64_t key = static_cast<uint64_t>(stream) ^ (static_cast<uint64_t>(dev) << 56);
  if (m->size() >= 16 && !m->count(key)) m->clear();  // many short-lived streams: keep the map bounded
  at::Tensor& ws = (*m)[key];
  if (!ws.defined() || ws.numel() < need) {
    ws = at::empty({std::max<int64_t>(need * 2, 4096)},
                   at::TensorOptions().dtype(at::kByte).device(at::kCUDA, static_cast<c10::DeviceIndex>(dev)));
    if (hipMemsetAsync(ws.data_ptr(), 0, 16, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
      throw std::runtime_error("fused-norm workspace: hipMemsetAsync failed");
  }
  return ws;
}

// An upload from a pinned staging tensor cannot be replayed from a graph: once the copy is recorded
// the tensor goes back to torch's host allocator, which hands the block out again, and a replay
// copies whatever the block then holds (as kernel pointers, here). While `stream` is being captured
// such an upload is refused: true with a Python error set. (Images in the kernel arguments are
// part of the recorded launch and replay as captured.)
bool upload_refused_in_capture(unsigned long long stream, const char* what) {
  if (!stream_capturing(stream)) return false;
  PyErr_Format(PyExc_RuntimeError,
               "%s: its plan image is too large for the kernel arguments and would be uploaded from a pinned "
               "staging buffer, which a graph replay cannot reuse safely; not capturable (fewer clients or "
               "leaves per call keep the image in the kernel arguments)",
               what);
  return true;
}

int fold_core(const std::vector<at::Tensor>& row0, const int64_t* in, int64_t K, const float* wf, double scale,
              bool has_scale, double nt_min_bytes, int dev, unsigned long long stream, PlanFn plan, WsumFn wsum,
              std::vector<at::Tensor>& outs, bool accumulate, WsumL2Fn l2fn, L2WsFn l2ws, float* l2p, int* rc,
              Stamp& st, const L2Rows* rows = nullptr) {
  const int64_t L = static_cast<int64_t>(row0.size());
  const bool with_l2 = l2p != nullptr || rows != nullptr;
  if (L < 1 || K < 1 || (accumulate && outs.empty())) return 1;
  // fast case only: float32 leaves (fold type and output type are then float32 for any
  // weights). A leaf with a client pointer off 16 bytes walks element units (per-leaf
  // plan); the outputs are fresh allocations, so aligned.
  std::vector<int64_t> leaf_n(L);
  int64_t total = 0;
  for (int64_t l = 0; l < L; ++l) {
    const at::Tensor& t = row0[l];
    if (t.scalar_type() != at::kFloat) return 1;
    leaf_n[l] = t.numel();
    total += leaf_n[l];
  }
  if (total == 0) return 1;  // only empty leaves: the Python path (no launch at all)
  std::vector<int64_t> lbits(L, 0);
  for (int64_t k = 0; k < K; ++k)
    for (int64_t l = 0; l < L; ++l) lbits[l] |= in[k * L + l];
  st.lap(kTChecks);
  const bool fresh = outs.empty();
  if (!fresh) {  // caller's destinations: float32, contiguous, row0's shape and device
    if (static_cast<int64_t>(outs.size()) != L) return 1;
    for (int64_t l = 0; l < L; ++l) {
      const at::Tensor& d = outs[l];
      if (d.scalar_type() != at::kFloat || !d.is_contiguous() || d.sizes() != row0[l].sizes() ||
          d.device() != row0[l].device())
        return 1;
    }
  }
  std::vector<uint8_t> elem(L, 0);
  bool any_elem = false;
  for (int64_t l = 0; l < L; ++l) any_elem = any_elem || (lbits[l] & 15) != 0;
  if (any_elem && rows && rows->aligned_only) return 2;
  if (fresh) carve_outputs(row0, outs);
  any_elem = false;
  for (int64_t l = 0; l < L; ++l) {
    elem[l] = ((lbits[l] | reinterpret_cast<int64_t>(outs[l].data_ptr())) & 15) != 0;
    any_elem = any_elem || elem[l];
  }
  if (any_elem && rows && rows->aligned_only) return 2;  // (a caller destination off 16 bytes)
  st.lap(kTOutputs);
  // a small delta and many clients: k_ptrs_narrow's LDS-staged stripes (any alignment;
  // the rule of tree_util._narrow), not with fused norms
  static const int64_t narrow_max = [] {  // FJAGG_NARROW_MAX_BYTES, as tree_util._NARROW_MAX_BYTES
    const char* e = getenv("FJAGG_NARROW_MAX_BYTES");
    return e ? (int64_t)atoll(e) : (int64_t)(256 << 10);
  }();
  const bool narrow = !with_l2 && K >= 16 && total * 4 <= narrow_max;
  const uint8_t* mask = any_elem && !narrow ? elem.data() : nullptr;
  // every pointer 16-byte aligned: the stripe pipeline (k_ptrs_stripe, fjstripe.hip) with
  // the width of tree_util._stripe_variant_for; FJAGG_STRIPE_PYTREE=0 keeps k_ptrs_narrow
  static const bool stripe_on = [] {
    const char* e = getenv("FJAGG_STRIPE_PYTREE");
    return !(e && e[0] == '0' && e[1] == 0);
  }();
  int svar = 0;
  if (narrow && stripe_on && !any_elem && K >= 512) {  // (fjagg.hip kStripeMinClients)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    int64_t s64 = 0, s32 = 0;
    for (int64_t l = 0; l < L; ++l) {
      s64 += (leaf_n[l] + 63) / 64;
      s32 += (leaf_n[l] + 31) / 32;
    }
    svar = s64 >= cus ? 20 : s32 >= cus ? 21 : 22;
  }
  const int pflags = narrow ? (FJAGG_NARROW | FJAGG_VARIANT(svar)) : 0;
  const int64_t nblk = plan(kF32, pflags, leaf_n.data(), mask, static_cast<int>(L), nullptr, 0);
  if (nblk < 0) return 1;
  // plan image (fjagg.h): in_ptrs[K*L] | out_ptrs[L] | leaf_n[L] | blocks[2*nblk] | f32 weights
  const int64_t nw = (K + 1) / 2, n = K * L + 2 * L + 2 * nblk + nw;
  st.lap(kTPlan);
  auto fill = [&](int64_t* p) {
    std::memcpy(p, in, sizeof(int64_t) * K * L);
    for (int64_t l = 0; l < L; ++l) {
      p[K * L + l] = reinterpret_cast<int64_t>(outs[l].data_ptr());
      p[K * L + L + l] = leaf_n[l];
    }
    if (plan(kF32, pflags, leaf_n.data(), mask, static_cast<int>(L), p + K * L + 2 * L, nblk) != nblk) return false;
    p[n - 1] = 0;
    std::memcpy(p + n - nw, wf, 4 * K);
    return true;
  };
  const bool nt = static_cast<double>(total) * K * 4 >= nt_min_bytes;
  // FJAGG_L2_COMBINE_LAUNCH=1 keeps the separate norm-combine launch (no FJAGG_ZEROED_WS): the
  // in-launch hand-off follows the HIP guide's measured recipe for gfx950, which HIP itself does
  // not promise; the norms are bitwise the same either way
  static const bool combine_launch = [] {
    const char* e = getenv("FJAGG_L2_COMBINE_LAUNCH");
    return e && e[0] == '1';
  }();
  const int flags = (has_scale ? kScale : 0) | (nt ? kNontemporal : 0) | (accumulate ? kAccumulate : 0) |
                    (narrow ? (FJAGG_NARROW | FJAGG_VARIANT(svar)) : 0) |
                    (with_l2 && !combine_launch ? FJAGG_ZEROED_WS : 0);
  at::Tensor ws;  // fused l2 norms: counter header + per-workgroup partials (l2_workspace)
  if (with_l2) {
    const int64_t need = l2ws(K, nblk);
    if (need < 0) return 1;
    ws = l2_workspace(dev, stream, need);
  }
  auto launch = [&](const int64_t* image, const int64_t* w, int fl) {
    if (rows)
      return rows->fn(kF32, kF32, kF32, image, static_cast<int>(L), K, nblk, w, static_cast<float>(scale), rows->sq,
                      rows->nrm, rows->first, fl, ws.data_ptr(), ws.numel(), reinterpret_cast<void*>(stream));
    if (with_l2)
      return l2fn(kF32, kF32, kF32, image, static_cast<int>(L), K, nblk, w, static_cast<float>(scale), l2p, fl,
                  ws.data_ptr(), ws.numel(), reinterpret_cast<void*>(stream));
    return wsum(kF32, kF32, kF32, image, static_cast<int>(L), K, nblk, w, static_cast<float>(scale), fl,
                reinterpret_cast<void*>(stream));
  };
  *rc = FJAGG_EUNSUPPORTED;
  if (!narrow && n <= FJAGG_KARG_MAX_WORDS) {
    // the image and weights travel in the kernel arguments (FJAGG_HOST_TABLES): no pinned
    // staging buffer and no upload on the stream in front of the fold
    thread_local std::vector<int64_t> host_img;
    host_img.resize(static_cast<size_t>(n));
    if (!fill(host_img.data())) return 1;
    st.lap(kTImage);
    *rc = launch(host_img.data(), host_img.data() + (n - nw), flags | FJAGG_HOST_TABLES);
    if (*rc != FJAGG_EUNSUPPORTED) ++g_image_karg;
  }
  if (*rc == FJAGG_EUNSUPPORTED) {  // too large for the kernel arguments: pinned image + stream-ordered upload
    if (upload_refused_in_capture(stream, "a pytree fold")) return 3;
    at::Tensor img = at::empty({n}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
    if (!fill(img.data_ptr<int64_t>())) return 1;
    st.lap(kTImage);
    at::Tensor dimg = img.to(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(dev)), /*non_blocking=*/true);
    st.lap(kTUpload);
    const int64_t* dp = dimg.data_ptr<int64_t>();
    *rc = launch(dp, dp + (n - nw), flags);
    ++g_image_upload;
  }
  st.lap(kTLaunch);
  return 0;
}

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
  Stamp st;
  ++g_timer_calls;
  try {
    std::vector<at::Tensor> r0, outs;
    r0.reserve(L);
    for (Py_ssize_t l = 0; l < L; ++l) {
      PyObject* x = PyList_GET_ITEM(row0, l);
      if (!THPVariable_Check(x)) Py_RETURN_NONE;
      r0.push_back(THPVariable_Unpack(x));
    }
    if (dst != Py_None) {
      for (Py_ssize_t l = 0; l < L; ++l) {
        PyObject* o = PyList_GET_ITEM(dst, l);
        if (!THPVariable_Check(o)) Py_RETURN_NONE;
        outs.push_back(THPVariable_Unpack(o));
      }
    }
    float* l2p = nullptr;
    if (with_l2) {
      const at::Tensor& q = THPVariable_Unpack(l2sq);
      if (q.scalar_type() != at::kFloat || q.numel() != K || !q.is_contiguous() || !q.is_cuda() ||
          q.get_device() != dev)
        Py_RETURN_NONE;
      l2p = q.data_ptr<float>();
    }
    int rc = 0;
    if (fold_core(r0, static_cast<const int64_t*>(bp.buf), K, static_cast<const float*>(bw.buf), scale,
                  has_scale != 0, nt_min_bytes, dev, stream, reinterpret_cast<PlanFn>(plan_addr),
                  reinterpret_cast<WsumFn>(wsum_addr), outs, accumulate != 0, reinterpret_cast<WsumL2Fn>(l2_addr),
                  reinterpret_cast<L2WsFn>(l2ws_addr), l2p, &rc, st) != 0) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_NONE;
    }
    PyObject* list = PyList_New(L);
    if (!list) return nullptr;
    for (Py_ssize_t l = 0; l < L; ++l) PyList_SET_ITEM(list, l, THPVariable_Wrap(std::move(outs[l])));
    st.lap(kTWrap);
    return Py_BuildValue("(iN)", rc, list);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// ------------------------------------------------------------------ per-call tree ops
// (include/fjtree.h). The K operand trees are walked in parallel, driven by tree 0:
// exact dict (keys sorted, as jax flattens) / list / tuple / None nodes, exact
// torch.Tensor leaves. Anything else is "not the fast case" (None to the caller).

// A vector of pointers with room for N inline: the per-call walks below (one client pytree of a
// few leaves and dicts per call) then allocate nothing on the heap.
template <class T, size_t N>
struct SmallVec {
  T inl[N];
  T* p = inl;
  size_t n = 0, cap = N;
  SmallVec() = default;
  SmallVec(const SmallVec&) = delete;
  SmallVec& operator=(const SmallVec&) = delete;
  ~SmallVec() {
    if (p != inl) std::free(p);
  }
  void grow() {
    const size_t c = cap * 2;
    T* q = static_cast<T*>(std::malloc(sizeof(T) * c));
    if (!q) throw std::bad_alloc();
    std::memcpy(q, p, sizeof(T) * n);
    if (p != inl) std::free(p);
    p = q;
    cap = c;
  }
  void push_back(T v) {
    if (n == cap) grow();
    p[n++] = v;
  }
  void reserve(size_t) {}
  size_t size() const { return n; }
  size_t capacity() const { return cap; }
  bool empty() const { return n == 0; }
  void clear() { n = 0; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T* data() { return p; }
  const T* data() const { return p; }
  T* begin() { return p; }
  T* end() { return p + n; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
};

struct PWalk {
  int K = 0;
  SmallVec<PyObject*, 16> leaves[FJTREE_MAX_OPERANDS];  // borrowed, flatten order
  SmallVec<PyObject*, 8> keys;                          // owned sorted key lists, pre-order
  std::vector<int64_t>* sig = nullptr;  // optional: operand 0's structure (kinds, lengths, key objects)
  std::vector<PyObject*>* dicts = nullptr;  // optional: operand 0's dict nodes, pre-order (borrowed)
  bool seq_nodes = false;                   // operand 0 has a list / tuple node
  ~PWalk() {
    for (PyObject* k : keys) Py_DECREF(k);
  }
};

// The sorted key list of dict x (a new reference, or nullptr with *unorderable set when
// sorting raised — the error is cleared — or with a Python error set). Per-call tree ops
// walk one client pytree after another, every one a dict with the same key objects in the
// same insertion order: a small cache keyed by those key pointers (held by strong
// references, so a pointer is never a reused address) gives the sorted list without a
// PyDict_Keys + sort per dict node per call. Guarded by the GIL like every entry point.
// vals (optional, room for kSortedVals): on a cache hit of a dict of at most kSortedVals
// entries, x's values in sorted-key order (borrowed), collected by the same insertion-order
// scan that matched the keys — the walk then does no hash lookups on operand 0; *have_vals
// says whether they were filled.
constexpr Py_ssize_t kSortedVals = 32;
PyObject* sorted_keys(PyObject* x, bool* unorderable, PyObject** vals = nullptr, bool* have_vals = nullptr) {
  struct Entry {
    std::vector<PyObject*> order;  // strong references, insertion order
    PyObject* sorted;              // strong reference
    std::vector<uint8_t> perm;     // sorted position j -> insertion index (dicts of <= kSortedVals keys)
  };
  static std::vector<Entry> cache;
  static size_t next_slot = 0;
  constexpr size_t kCap = 64;
  *unorderable = false;
  if (have_vals) *have_vals = false;
  const Py_ssize_t n = PyDict_GET_SIZE(x);
  PyObject* ins[kSortedVals];
  const bool collect = vals && n <= kSortedVals;
  for (const Entry& e : cache) {
    if (static_cast<Py_ssize_t>(e.order.size()) != n) continue;
    Py_ssize_t pos = 0, i = 0;
    PyObject *k, *v;
    bool same = true;
    while (PyDict_Next(x, &pos, &k, &v)) {
      if (k != e.order[i]) {
        same = false;
        break;
      }
      if (collect) ins[i] = v;
      ++i;
    }
    if (same) {
      if (collect && static_cast<Py_ssize_t>(e.perm.size()) == n) {
        for (Py_ssize_t j = 0; j < n; ++j) vals[j] = ins[e.perm[j]];
        *have_vals = true;
      }
      Py_INCREF(e.sorted);
      return e.sorted;
    }
  }
  PyObject* keys = PyDict_Keys(x);
  if (!keys) return nullptr;
  if (PyList_Sort(keys) != 0) {
    PyErr_Clear();
    Py_DECREF(keys);
    *unorderable = true;
    return nullptr;
  }
  Entry e;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(x, &pos, &k, &v)) {
    Py_INCREF(k);
    e.order.push_back(k);
  }
  if (n <= kSortedVals && static_cast<Py_ssize_t>(e.order.size()) == n && PyList_GET_SIZE(keys) == n) {
    for (Py_ssize_t j = 0; j < n; ++j) {
      Py_ssize_t i = 0;
      while (i < n && e.order[i] != PyList_GET_ITEM(keys, j)) ++i;
      if (i == n) {  // (a key compared equal but is another object: no permutation)
        e.perm.clear();
        break;
      }
      e.perm.push_back(static_cast<uint8_t>(i));
    }
  }
  Py_INCREF(keys);
  e.sorted = keys;
  if (cache.size() < kCap) {
    cache.push_back(std::move(e));
  } else {  // replace round-robin
    Entry& old = cache[next_slot];
    for (PyObject* o : old.order) Py_DECREF(o);
    Py_DECREF(old.sorted);
    old = std::move(e);
    next_slot = (next_slot + 1) % kCap;
  }
  return keys;
}

// 0: walked; 1: not the fast case / structures differ; -1: Python error set.
int pwalk(PyObject* const* xs, PWalk& w, int depth) {
  if (depth > 64) return 1;
  PyObject* x0 = xs[0];
  const int K = w.K;
  PyTypeObject* tt = reinterpret_cast<PyTypeObject*>(THPVariableClass);
  if (Py_TYPE(x0) == tt) {
    for (int k = 0; k < K; ++k) {
      if (Py_TYPE(xs[k]) != tt) return 1;
      if (w.leaves[k].size() >= FJTREE_MAX_LEAVES) return 1;
      w.leaves[k].push_back(xs[k]);
    }
    if (w.sig) w.sig->push_back(kLeaf);
    return 0;
  }
  if (x0 == Py_None) {
    for (int k = 1; k < K; ++k)
      if (xs[k] != Py_None) return 1;
    if (w.sig) w.sig->push_back(kNone);
    return 0;
  }
  PyObject* vals[FJTREE_MAX_OPERANDS];
  if (PyDict_CheckExact(x0)) {
    const Py_ssize_t n = PyDict_GET_SIZE(x0);
    for (int k = 1; k < K; ++k)
      if (!PyDict_CheckExact(xs[k]) || PyDict_GET_SIZE(xs[k]) != n) return 1;
    bool unorderable = false, have0 = false;
    PyObject* v0[kSortedVals];
    PyObject* keys = sorted_keys(x0, &unorderable, v0, &have0);
    if (!keys) return unorderable ? 1 : -1;  // unorderable keys: the Python path decides
    w.keys.push_back(keys);
    if (w.dicts) w.dicts->push_back(x0);
    if (w.sig) {
      w.sig->push_back(kDict);
      w.sig->push_back(n);
      for (Py_ssize_t i = 0; i < n; ++i) w.sig->push_back(reinterpret_cast<int64_t>(PyList_GET_ITEM(keys, i)));
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* key = PyList_GET_ITEM(keys, i);
      for (int k = 0; k < K; ++k) {
        vals[k] = (k == 0 && have0) ? v0[i] : PyDict_GetItemWithError(xs[k], key);
        if (!vals[k]) {
          if (PyErr_Occurred()) PyErr_Clear();
          return 1;
        }
      }
      if (int rc = pwalk(vals, w, depth + 1)) return rc;
    }
    return 0;
  }
  const bool is_list = PyList_CheckExact(x0), is_tuple = PyTuple_CheckExact(x0);
  if (!is_list && !is_tuple) return 1;
  w.seq_nodes = true;
  const Py_ssize_t n = Py_SIZE(x0);
  for (int k = 1; k < K; ++k)
    if (Py_TYPE(xs[k]) != Py_TYPE(x0) || Py_SIZE(xs[k]) != n) return 1;
  if (w.sig) {
    w.sig->push_back(is_list ? kList : kTuple);
    w.sig->push_back(n);
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    for (int k = 0; k < K; ++k) vals[k] = is_list ? PyList_GET_ITEM(xs[k], i) : PyTuple_GET_ITEM(xs[k], i);
    if (int rc = pwalk(vals, w, depth + 1)) return rc;
  }
  return 0;
}

// A new tree shaped like x0 whose leaves are outs[i++] (stolen references), dict keys
// in sorted order (jax's unflatten of a dict); key lists from the walk, in pre-order.
PyObject* rebuild(PyObject* x0, PyObject** outs, size_t& i, PyObject* const* keys, size_t& ki) {
  if (Py_TYPE(x0) == reinterpret_cast<PyTypeObject*>(THPVariableClass)) {
    PyObject* o = outs[i];
    outs[i++] = nullptr;
    return o;
  }
  if (x0 == Py_None) {
    Py_INCREF(Py_None);
    return Py_None;
  }
  if (PyDict_CheckExact(x0)) {
    PyObject* kl = keys[ki++];
    PyObject* d = PyDict_New();
    if (!d) return nullptr;
    for (Py_ssize_t j = 0; j < PyList_GET_SIZE(kl); ++j) {
      PyObject* key = PyList_GET_ITEM(kl, j);
      PyObject* v = rebuild(PyDict_GetItem(x0, key), outs, i, keys, ki);
      if (!v || PyDict_SetItem(d, key, v) != 0) {
        Py_XDECREF(v);
        Py_DECREF(d);
        return nullptr;
      }
      Py_DECREF(v);
    }
    return d;
  }
  const bool is_list = PyList_CheckExact(x0);
  const Py_ssize_t n = Py_SIZE(x0);
  PyObject* c = is_list ? PyList_New(n) : PyTuple_New(n);
  if (!c) return nullptr;
  for (Py_ssize_t j = 0; j < n; ++j) {
    PyObject* v = rebuild(is_list ? PyList_GET_ITEM(x0, j) : PyTuple_GET_ITEM(x0, j), outs, i, keys, ki);
    if (!v) {
      Py_DECREF(c);
      return nullptr;
    }
    if (is_list) PyList_SET_ITEM(c, j, v);
    else PyTuple_SET_ITEM(c, j, v);
  }
  return c;
}

// float32 of a Python int / float weight as numpy rounds it; false for anything else.
bool f32_weight(PyObject* w, float* out) {
  if (PyLong_CheckExact(w)) {
    int overflow = 0;
    long long v = PyLong_AsLongLongAndOverflow(w, &overflow);
    if (overflow || v >= (1LL << 53) || v <= -(1LL << 53)) {
      if (PyErr_Occurred()) PyErr_Clear();
      return false;
    }
    *out = static_cast<float>(static_cast<double>(v));
    return true;
  }
  if (PyFloat_CheckExact(w)) {
    *out = static_cast<float>(PyFloat_AS_DOUBLE(w));
    return true;
  }
  return false;
}

// Leaves of operand k: float32, strided, contiguous, on cuda:dev, leaf l shaped like
// operand 0's. Fills the version sum; *unversioned (optional) is set when some leaf is an
// inference tensor (no version counter). false: not the fast case.
bool check_leaves(const PWalk& w, int k, c10::DeviceIndex dev, int64_t* vsum, bool* unversioned = nullptr) {
  int64_t vs = 0;
  if (unversioned) *unversioned = false;
  for (size_t l = 0; l < w.leaves[k].size(); ++l) {
    const at::Tensor& t = THPVariable_Unpack(w.leaves[k][l]);
    if (t.layout() != c10::kStrided || t.scalar_type() != at::kFloat || !t.is_cuda() || t.get_device() != dev ||
        !t.is_contiguous())
      return false;
    if (k > 0 && t.sizes() != THPVariable_Unpack(w.leaves[0][l]).sizes()) return false;
    if (t.is_inference()) {
      if (unversioned) *unversioned = true;
    } else {
      vs += static_cast<int64_t>(t._version());
    }
  }
  *vsum = vs;
  return true;
}

struct WsKey {
  int dev;
  uint64_t stream;
  bool operator==(const WsKey& o) const { return dev == o.dev && stream == o.stream; }
};
struct WsHash {
  size_t operator()(const WsKey& k) const { return std::hash<uint64_t>()(k.stream ^ (uint64_t(k.dev) << 56)); }
};
// Norm workspace per (device, stream): its completion counter must start at 0, and each
// launch leaves it at 0, so launches on one stream can share it (include/fjtree.h).
std::unordered_map<WsKey, at::Tensor, WsHash>& workspaces() {
  static auto* m = new std::unordered_map<WsKey, at::Tensor, WsHash>();
  return *m;
}

typedef int (*TreeFoldFn)(const fjtree_leaves*, void*);
typedef int64_t (*TreeWsFn)(const fjtree_leaves*);
constexpr int kStale = -100;

struct SigHash {
  size_t operator()(const std::vector<int64_t>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int64_t x : v) h = (h ^ static_cast<uint64_t>(x)) * 1099511628211ull;
    return static_cast<size_t>(h ^ (h >> 29));
  }
};

// The structure token of a captured tree: equal tokens <=> the same node kinds, lengths,
// dict key OBJECTS (in sorted order), device and leaf shapes. Interned per process; the
// table holds strong references to the key objects, so a key's address is never reused
// while its entry exists. -1 once the table is full (the caller then walks both trees).
int64_t structure_token(const std::vector<int64_t>& sig, const PWalk& w) {
  static auto* table = new std::unordered_map<std::vector<int64_t>, int64_t, SigHash>();
  constexpr size_t kMaxTokens = 4096;
  // one client pytree after another has the previous one's structure: compare with it first
  // (its key objects are alive: the table entry of its token holds them)
  static std::vector<int64_t> last_sig;
  static int64_t last_tok = -1;
  if (last_tok >= 0 && sig == last_sig) return last_tok;
  auto it = table->find(sig);
  if (it != table->end()) {
    last_sig = sig;
    last_tok = it->second;
    return it->second;
  }
  if (table->size() >= kMaxTokens) return -1;
  for (PyObject* kl : w.keys)  // keep the key objects alive for as long as the entry exists
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(kl); ++i) Py_INCREF(PyList_GET_ITEM(kl, i));
  const int64_t tok = static_cast<int64_t>(table->size());
  table->emplace(sig, tok);
  return tok;
}

// capture(tree, dev) -> (leaves_tuple, version_sum, nbytes, token, data_ptrs[+ dict tags], has_tags) | None
//     (dev = -1: the first leaf's)
//     tree_weight's lazy result holds its input's leaves (strong references, flatten order)
//     and their version sum, so the fold can check that nothing changed in between; token
//     (structure_token) lets tree_add match two captured trees' structures without a walk.
// The data pointers of a capture's leaves as bytes (int64 each), element 4 of the capture.
// A `.data = other` reassignment keeps a tensor object and, with torch's set_data, its
// version counter, but moves its storage: the folds compare these pointers with the
// captured tensors' current ones and refuse a moved leaf as they refuse a modified one.
PyObject* ptr_bytes(PyObject* const* leaves, Py_ssize_t L) {
  PyObject* b = PyBytes_FromStringAndSize(nullptr, 8 * L);
  if (!b) return nullptr;
  auto* p = reinterpret_cast<int64_t*>(PyBytes_AS_STRING(b));
  for (Py_ssize_t l = 0; l < L; ++l) p[l] = reinterpret_cast<int64_t>(THPVariable_Unpack(leaves[l]).data_ptr());
  return b;
}

// captured data pointer of leaf l (capture element 4), or 0 when the capture has none
inline int64_t captured_ptr(PyObject* cap, Py_ssize_t l) {
  if (PyTuple_GET_SIZE(cap) < 5) return 0;
  PyObject* b = PyTuple_GET_ITEM(cap, 4);
  if (!PyBytes_Check(b) || PyBytes_GET_SIZE(b) < 8 * (l + 1)) return 0;
  return reinterpret_cast<const int64_t*>(PyBytes_AS_STRING(b))[l];
}

// All L captured data pointers of a capture (element 4), or nullptr when it has none: the
// per-leaf loops of the folds read them without re-checking the tuple per leaf.
inline const int64_t* captured_ptrs(PyObject* cap, Py_ssize_t L) {
  if (PyTuple_GET_SIZE(cap) < 5) return nullptr;
  PyObject* b = PyTuple_GET_ITEM(cap, 4);
  if (!PyBytes_Check(b) || PyBytes_GET_SIZE(b) < 8 * L) return nullptr;
  return reinterpret_cast<const int64_t*>(PyBytes_AS_STRING(b));
}

// The dict tags of a capture: its tree's dict nodes in pre-order as int64 pairs (address,
// CPython dict version tag), appended to element 4 after the L data pointers, element 5 then
// True (None when the tree is not dicts over leaves: a list / tuple node, or a leaf at the
// root; one bytes object per capture, not two). A dict's version tag (PEP 509) changes with
// every mutation and is never reused, so while the root is the same object and every tag is
// unchanged, walking the tree again would give the captured leaves: tree_l2_norm of the delta
// just added checks that instead of re-walking (same_tree). Visiting in pre-order means a dict
// is dereferenced only after its parent — which still holds it — was found unchanged.
bool has_dict_tags(const PWalk& w, PyObject* root) {
#if PY_VERSION_HEX < 0x030C0000
  return w.dicts && !w.seq_nodes && !w.dicts->empty() && (*w.dicts)[0] == root;
#else
  (void)w, (void)root;
  return false;
#endif
}

// Element 4 of a capture: the L data pointers, then (with_tags) the dict tags.
PyObject* ptr_tag_bytes(const PWalk& w, Py_ssize_t L, bool with_tags) {
  const Py_ssize_t n = with_tags ? static_cast<Py_ssize_t>(w.dicts->size()) : 0;
  PyObject* b = PyBytes_FromStringAndSize(nullptr, 8 * L + 16 * n);
  if (!b) return nullptr;
  auto* p = reinterpret_cast<int64_t*>(PyBytes_AS_STRING(b));
  for (Py_ssize_t l = 0; l < L; ++l) p[l] = reinterpret_cast<int64_t>(THPVariable_Unpack(w.leaves[0][l]).data_ptr());
#if PY_VERSION_HEX < 0x030C0000
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* d = (*w.dicts)[i];
    p[L + 2 * i] = reinterpret_cast<int64_t>(d);
    p[L + 2 * i + 1] = static_cast<int64_t>(reinterpret_cast<PyDictObject*>(d)->ma_version_tag);
  }
#endif
  return b;
}

// tree is the captured tree, unchanged (the capture's dict tags): true, or false = not known.
bool same_tree(PyObject* tree, PyObject* cap) {
#if PY_VERSION_HEX < 0x030C0000
  if (PyTuple_GET_SIZE(cap) < 6 || PyTuple_GET_ITEM(cap, 5) != Py_True) return false;
  PyObject* b = PyTuple_GET_ITEM(cap, 4);
  const Py_ssize_t L = PyTuple_GET_SIZE(PyTuple_GET_ITEM(cap, 0));
  if (!PyBytes_CheckExact(b) || PyBytes_GET_SIZE(b) < 8 * L + 16) return false;
  const auto* p = reinterpret_cast<const int64_t*>(PyBytes_AS_STRING(b)) + L;
  const Py_ssize_t n = (PyBytes_GET_SIZE(b) - 8 * L) / 16;
  if (p[0] != reinterpret_cast<int64_t>(tree) || !PyDict_CheckExact(tree)) return false;
  for (Py_ssize_t i = 0; i < n; ++i)
    if (static_cast<int64_t>(reinterpret_cast<PyDictObject*>(p[2 * i])->ma_version_tag) != p[2 * i + 1]) return false;
  return true;
#else
  (void)tree, (void)cap;
  return false;
#endif
}

// nbytes as a Python int: one client pytree after another has the same size, so the last
// object is handed out again (ints are immutable).
PyObject* nbytes_long(int64_t nbytes) {
  static int64_t last = -1;
  static PyObject* obj = nullptr;
  if (obj && nbytes == last) {
    Py_INCREF(obj);
    return obj;
  }
  PyObject* o = PyLong_FromLongLong(nbytes);
  if (!o) return nullptr;
  Py_XDECREF(obj);
  Py_INCREF(o);
  obj = o;
  last = nbytes;
  return o;
}

// New reference: the capture tuple, Py_None (not the fast case), or nullptr (Python error).
PyObject* capture_impl(PyObject* tree, int dev) {
  try {
    thread_local std::vector<int64_t> sig;
    thread_local std::vector<PyObject*> dicts;
    sig.clear();
    dicts.clear();
    PWalk w;
    w.K = 1;
    w.sig = &sig;
    w.dicts = &dicts;
    w.leaves[0].reserve(16);
    int rc = pwalk(&tree, w, 0);
    if (rc < 0) return nullptr;
    int64_t vs = 0;
    if (rc > 0 || w.leaves[0].empty()) Py_RETURN_NONE;
    if (dev < 0) {
      const at::Tensor& t0 = THPVariable_Unpack(w.leaves[0][0]);
      if (!t0.is_cuda()) Py_RETURN_NONE;
      dev = t0.get_device();
    }
    bool unv = false;
    // an inference tensor has no version counter to guard a lazy capture with: not deferred
    if (!check_leaves(w, 0, static_cast<c10::DeviceIndex>(dev), &vs, &unv) || unv) Py_RETURN_NONE;
    const Py_ssize_t L = static_cast<Py_ssize_t>(w.leaves[0].size());
    PyObject* tup = PyTuple_New(L);
    if (!tup) return nullptr;
    int64_t nbytes = 0;
    sig.push_back(dev);
    for (Py_ssize_t l = 0; l < L; ++l) {
      Py_INCREF(w.leaves[0][l]);
      PyTuple_SET_ITEM(tup, l, w.leaves[0][l]);
      const at::Tensor& t = THPVariable_Unpack(w.leaves[0][l]);
      nbytes += 4 * t.numel();
      sig.push_back(t.dim());
      for (int64_t s : t.sizes()) sig.push_back(s);
    }
    const int64_t tok = structure_token(sig, w);
    const bool tags = has_dict_tags(w, tree);
    PyObject* out = PyTuple_New(6);
    PyObject* a = PyLong_FromLongLong(vs);
    PyObject* b = nbytes_long(nbytes);
    PyObject* c = PyLong_FromLongLong(tok);
    PyObject* d = ptr_tag_bytes(w, L, tags);
    PyObject* e = tags ? Py_True : Py_None;
    Py_INCREF(e);
    if (!out || !a || !b || !c || !d) {
      Py_XDECREF(out), Py_XDECREF(a), Py_XDECREF(b), Py_XDECREF(c), Py_XDECREF(d), Py_DECREF(e), Py_DECREF(tup);
      return nullptr;
    }
    PyTuple_SET_ITEM(out, 0, tup);
    PyTuple_SET_ITEM(out, 1, a);
    PyTuple_SET_ITEM(out, 2, b);
    PyTuple_SET_ITEM(out, 3, c);
    PyTuple_SET_ITEM(out, 4, d);
    PyTuple_SET_ITEM(out, 5, e);
    return out;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyObject* capture(PyObject*, PyObject* args) {
  PyObject* tree;
  int dev;
  if (!PyArg_ParseTuple(args, "Oi", &tree, &dev)) return nullptr;
  return capture_impl(tree, dev);
}

// capture_probe(tree, reps) -> dict: ns per call of the parts of capture_impl over `reps` calls
// (tools/prof_capture_parts.py): the sorted walk, the leaf checks, the signature + structure
// token, the capture objects, and the whole capture.
PyObject* capture_probe(PyObject*, PyObject* args) {
  PyObject* tree;
  long long reps;
  if (!PyArg_ParseTuple(args, "OL", &tree, &reps)) return nullptr;
  using clk = std::chrono::steady_clock;
  auto ns = [&](clk::time_point t0) {
    return std::chrono::duration<double, std::nano>(clk::now() - t0).count() / static_cast<double>(reps);
  };
  try {
    double t_walk, t_check, t_sig, t_full;
    {
      auto t0 = clk::now();
      for (long long r = 0; r < reps; ++r) {
        thread_local std::vector<int64_t> sig;
        thread_local std::vector<PyObject*> dicts;
        sig.clear(), dicts.clear();
        PWalk w;
        w.K = 1;
        w.sig = &sig;
        w.dicts = &dicts;
        if (pwalk(&tree, w, 0) != 0) Py_RETURN_NONE;
      }
      t_walk = ns(t0);
    }
    PWalk w;
    w.K = 1;
    std::vector<int64_t> sig;
    std::vector<PyObject*> dicts;
    w.sig = &sig;
    w.dicts = &dicts;
    if (pwalk(&tree, w, 0) != 0 || w.leaves[0].empty()) Py_RETURN_NONE;
    const int dev = THPVariable_Unpack(w.leaves[0][0]).get_device();
    {
      auto t0 = clk::now();
      int64_t vs = 0;
      bool unv = false;
      for (long long r = 0; r < reps; ++r)
        if (!check_leaves(w, 0, static_cast<c10::DeviceIndex>(dev), &vs, &unv)) Py_RETURN_NONE;
      t_check = ns(t0);
    }
    {
      auto t0 = clk::now();
      for (long long r = 0; r < reps; ++r) {
        std::vector<int64_t> s2(sig);
        s2.push_back(dev);
        for (size_t l = 0; l < w.leaves[0].size(); ++l) {
          const at::Tensor& t = THPVariable_Unpack(w.leaves[0][l]);
          s2.push_back(t.dim());
          for (int64_t z : t.sizes()) s2.push_back(z);
        }
        (void)structure_token(s2, w);
      }
      t_sig = ns(t0);
    }
    {
      auto t0 = clk::now();
      for (long long r = 0; r < reps; ++r) {
        PyObject* c = capture_impl(tree, -1);
        if (!c) return nullptr;
        Py_DECREF(c);
      }
      t_full = ns(t0);
    }
    return Py_BuildValue("{s:d,s:d,s:d,s:d}", "walk_ns", t_walk, "check_ns", t_check, "sig_token_ns", t_sig,
                         "capture_ns", t_full);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// matches(tree, leaves_tuple, version_sum) -> bool: the same leaf objects, unmodified.
PyObject* matches(PyObject*, PyObject* args) {
  PyObject *tree, *tup;
  long long vsum;
  if (!PyArg_ParseTuple(args, "OO!L", &tree, &PyTuple_Type, &tup, &vsum)) return nullptr;
  try {
    PWalk w;
    w.K = 1;
    int rc = pwalk(&tree, w, 0);
    if (rc < 0) return nullptr;
    if (rc > 0 || static_cast<Py_ssize_t>(w.leaves[0].size()) != PyTuple_GET_SIZE(tup)) Py_RETURN_FALSE;
    int64_t vs = 0;
    for (size_t l = 0; l < w.leaves[0].size(); ++l) {
      if (w.leaves[0][l] != PyTuple_GET_ITEM(tup, l)) Py_RETURN_FALSE;
      vs += version_of(THPVariable_Unpack(w.leaves[0][l]));
    }
    if (vs != vsum) Py_RETURN_FALSE;
    Py_RETURN_TRUE;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// compatible(a, b) -> bool: the two trees have the same structure (the fast walk's node
// kinds, dict keys, lengths) and float32 device leaves of equal shapes on one device,
// i.e. tree_add(a, b) is the fast case. Nothing is launched.
PyObject* compatible(PyObject*, PyObject* args) {
  PyObject *a, *b;
  if (!PyArg_ParseTuple(args, "OO", &a, &b)) return nullptr;
  try {
    PWalk w;
    w.K = 2;
    PyObject* xs[2] = {a, b};
    int rc = pwalk(xs, w, 0);
    if (rc < 0) return nullptr;
    if (rc > 0 || w.leaves[0].empty()) Py_RETURN_FALSE;
    const at::Tensor& t0 = THPVariable_Unpack(w.leaves[0][0]);
    if (!t0.is_cuda()) Py_RETURN_FALSE;
    int64_t vs;
    if (!check_leaves(w, 0, t0.get_device(), &vs) || !check_leaves(w, 1, t0.get_device(), &vs)) Py_RETURN_FALSE;
    Py_RETURN_TRUE;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// append_check(ref, item, cap) -> cap | None | -100
//     One walk for tree_add(sum, weighted item) in deferred mode: `item` must have ref's
//     structure and float32 device leaves of ref's shapes on ref's device (else None: not the
//     fast case). cap None: returns a new capture of item (leaves_tuple, version_sum,
//     nbytes); cap given (from tree_weight): item must still hold exactly those leaves,
//     unmodified (else -100), and cap is returned.
PyObject* append_check(PyObject*, PyObject* args) {
  PyObject *ref, *item, *cap;
  if (!PyArg_ParseTuple(args, "OOO", &ref, &item, &cap)) return nullptr;
  try {
    PWalk w;
    w.K = 2;
    PyObject* xs[2] = {ref, item};
    int rc = pwalk(xs, w, 0);
    if (rc < 0) return nullptr;
    if (rc > 0 || w.leaves[0].empty()) Py_RETURN_NONE;
    const at::Tensor& t0 = THPVariable_Unpack(w.leaves[0][0]);
    if (!t0.is_cuda()) Py_RETURN_NONE;
    int64_t vs0, vs;
    bool unv = false;
    if (!check_leaves(w, 0, t0.get_device(), &vs0) || !check_leaves(w, 1, t0.get_device(), &vs, &unv) || unv)
      Py_RETURN_NONE;  // (an inference-tensor item cannot be held by reference: eager tree_add)
    const Py_ssize_t L = static_cast<Py_ssize_t>(w.leaves[1].size());
    if (cap != Py_None) {
      if (!PyTuple_Check(cap) || PyTuple_GET_SIZE(cap) < 2) Py_RETURN_NONE;
      PyObject* tup = PyTuple_GET_ITEM(cap, 0);
      bool same = PyTuple_GET_SIZE(tup) == L && PyLong_AsLongLong(PyTuple_GET_ITEM(cap, 1)) == vs;
      for (Py_ssize_t l = 0; same && l < L; ++l) {
        same = w.leaves[1][l] == PyTuple_GET_ITEM(tup, l);
        const int64_t cp = captured_ptr(cap, l);
        if (same && cp) same = cp == reinterpret_cast<int64_t>(THPVariable_Unpack(w.leaves[1][l]).data_ptr());
      }
      if (!same) return PyLong_FromLong(kStale);
      Py_INCREF(cap);
      return cap;
    }
    PyObject* tup = PyTuple_New(L);
    if (!tup) return nullptr;
    int64_t nbytes = 0;
    for (Py_ssize_t l = 0; l < L; ++l) {
      Py_INCREF(w.leaves[1][l]);
      PyTuple_SET_ITEM(tup, l, w.leaves[1][l]);
      nbytes += 4 * THPVariable_Unpack(w.leaves[1][l]).numel();
    }
    PyObject* pb = ptr_bytes(w.leaves[1].data(), L);
    if (!pb) {
      Py_DECREF(tup);
      return nullptr;
    }
    return Py_BuildValue("(NLLLN)", tup, static_cast<long long>(vs), static_cast<long long>(nbytes), -1LL, pb);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// A 0-d tensor over element `offset` of b's storage: its own TensorImpl on b's storage (no
// dispatcher round trip, unlike as_strided; not an autograd view of b, which needs none here).
at::Tensor scalar_at(const at::Tensor& b, int64_t offset) {
  at::Tensor v = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(b.storage()), b.key_set(), b.dtype());
  v.unsafeGetTensorImpl()->set_storage_offset(offset);
  v.unsafeGetTensorImpl()->set_sizes_contiguous({});
  return v;
}

// norm_view(buf, row, index, type) -> 0-d tensor of `type` (a torch.Tensor subclass) viewing
// buf[row, index]: the lazy l2-norm values of deferred sums (tree_util._NormView).
PyObject* norm_view(PyObject*, PyObject* args) {
  PyObject *buf, *type;
  long long row, index;
  if (!PyArg_ParseTuple(args, "OLLO", &buf, &row, &index, &type)) return nullptr;
  if (!THPVariable_Check(buf) || !PyType_Check(type)) {
    PyErr_SetString(PyExc_TypeError, "norm_view(tensor, row, index, type)");
    return nullptr;
  }
  try {
    const at::Tensor& b = THPVariable_Unpack(buf);
    if (b.dim() != 2 || row < 0 || row >= b.size(0) || index < 0 || index >= b.size(1)) {
      PyErr_SetString(PyExc_IndexError, "norm_view: index out of range");
      return nullptr;
    }
    return THPVariable_Wrap(scalar_at(b, b.storage_offset() + row * b.stride(0) + index * b.stride(1)),
                            reinterpret_cast<PyTypeObject*>(type));
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// table_from_caps(caps, ptrs) -> int
//     caps: list of K captures (leaves_tuple, version_sum) of L leaves each; writes leaf l of
//     capture k's device pointer to ptrs[k*L + l] (int64 buffer). Returns -1 when every
//     capture is unchanged (same versions), else the index of the first stale one.
PyObject* table_from_caps(PyObject*, PyObject* args) {
  PyObject *caps, *ptrs;
  if (!PyArg_ParseTuple(args, "O!O", &PyList_Type, &caps, &ptrs)) return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(caps);
  if (K == 0) return PyLong_FromLong(-1);
  const Py_ssize_t L = PyTuple_GET_SIZE(PyTuple_GET_ITEM(PyList_GET_ITEM(caps, 0), 0));
  Py_buffer buf;
  if (PyObject_GetBuffer(ptrs, &buf, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  struct Release {
    Py_buffer* b;
    ~Release() { PyBuffer_Release(b); }
  } release{&buf};
  if (buf.len < static_cast<Py_ssize_t>(sizeof(int64_t)) * K * L) {
    PyErr_SetString(PyExc_ValueError, "table_from_caps: pointer buffer smaller than K*L int64");
    return nullptr;
  }
  auto* out = static_cast<int64_t*>(buf.buf);
  try {
    for (Py_ssize_t k = 0; k < K; ++k) {
      PyObject* cap = PyList_GET_ITEM(caps, k);
      PyObject* tup = PyTuple_GET_ITEM(cap, 0);
      if (PyTuple_GET_SIZE(tup) != L) return PyLong_FromSsize_t(k);
      int64_t vs = 0;
      const int64_t* cps = captured_ptrs(cap, L);
      for (Py_ssize_t l = 0; l < L; ++l) {
        const at::Tensor& t = THPVariable_Unpack(PyTuple_GET_ITEM(tup, l));
        vs += version_of(t);
        out[k * L + l] = reinterpret_cast<int64_t>(t.data_ptr());
        if (cps && cps[l] != out[k * L + l]) return PyLong_FromSsize_t(k);  // storage moved (`.data =`)
      }
      if (vs != PyLong_AsLongLong(PyTuple_GET_ITEM(cap, 1))) return PyLong_FromSsize_t(k);
    }
    return PyLong_FromLong(-1);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// fold_caps(base, caps, weights, scale, has_scale, nt_min_bytes, plan_fn, wsum_fn, wsum_l2_fn,
//           l2_ws_bytes_fn, l2sq) -> (rc, tree) | k | None
//     A deferred running sum's fold (tree_util._fold_chain) in one call: caps[0] is the
//     captured base, caps[1..] the links' captures (leaves_tuple, version_sum, ...), weights
//     the K Python-number weights. Checks every capture's versions (k: the first stale one;
//     0 also when `base` no longer has the captured leaf count), builds the pointer table and
//     launches fold_core on the current stream; the result tree has base's structure (dict
//     keys sorted). l2sq: None or float32 [K] for every operand's squared norm. None: not this
//     case (nothing launched).
PyObject* fold_caps_impl(PyObject* base, PyObject* const* caps, PyObject* const* weights, Py_ssize_t K, double scale,
                         bool has_scale, double nt_min, unsigned long long plan_addr, unsigned long long wsum_addr,
                         unsigned long long l2_addr, unsigned long long l2ws_addr, PyObject* l2sq,
                         const L2Rows* rows = nullptr) {
  if (K < 1) Py_RETURN_NONE;
  Stamp st;
  ++g_timer_calls;
  try {
    thread_local std::vector<float> wf;
    wf.resize(K);
    for (Py_ssize_t k = 0; k < K; ++k)
      if (!f32_weight(weights[k], &wf[k])) Py_RETURN_NONE;
    PyObject* cap0 = caps[0];
    if (!PyTuple_Check(cap0) || PyTuple_GET_SIZE(cap0) < 2 || !PyTuple_Check(PyTuple_GET_ITEM(cap0, 0)))
      Py_RETURN_NONE;
    const Py_ssize_t L = PyTuple_GET_SIZE(PyTuple_GET_ITEM(cap0, 0));
    if (L < 1) Py_RETURN_NONE;
    PWalk w;  // base's structure now (for the result tree); its leaf objects are not used
    w.K = 1;
    const int wr = pwalk(&base, w, 0);
    if (wr < 0) return nullptr;
    if (wr > 0) Py_RETURN_NONE;
    if (static_cast<Py_ssize_t>(w.leaves[0].size()) != L) return PyLong_FromLong(0);
    thread_local std::vector<int64_t> ptrs;
    ptrs.resize(static_cast<size_t>(K * L));
    std::vector<at::Tensor> row0;
    row0.reserve(L);
    int dev = -1;
    for (Py_ssize_t k = 0; k < K; ++k) {
      PyObject* cap = caps[k];
      if (!PyTuple_Check(cap) || PyTuple_GET_SIZE(cap) < 2) Py_RETURN_NONE;
      PyObject* tup = PyTuple_GET_ITEM(cap, 0);
      if (!PyTuple_Check(tup) || PyTuple_GET_SIZE(tup) != L) return PyLong_FromSsize_t(k);
      int64_t vs = 0;
      const int64_t* cps = captured_ptrs(cap, L);
      for (Py_ssize_t l = 0; l < L; ++l) {
        PyObject* o = PyTuple_GET_ITEM(tup, l);
        if (!THPVariable_Check(o)) Py_RETURN_NONE;
        const at::Tensor& t = THPVariable_Unpack(o);
        if (k == 0) {
          if (t.scalar_type() != at::kFloat || !t.is_cuda() || !t.is_contiguous()) Py_RETURN_NONE;
          if (dev < 0) dev = t.get_device();
          if (t.get_device() != dev) Py_RETURN_NONE;
          row0.push_back(t);
        } else if (t.numel() != row0[l].numel() || t.scalar_type() != at::kFloat || !t.is_contiguous()) {
          // the links' captures were checked against the chain's structure when they were
          // taken (dtype, device, layout, shape); an in-place reshape bumps the version, but
          // a `.data` reassignment does not: the element count, dtype and layout guard the
          // fold's reads, the Python path then raises or recomputes
          Py_RETURN_NONE;
        }
        vs += version_of(t);
        ptrs[k * L + l] = reinterpret_cast<int64_t>(t.data_ptr());
        if (cps && cps[l] != ptrs[k * L + l]) return PyLong_FromSsize_t(k);  // storage moved (`.data =`)
      }
      const long long want = PyLong_AsLongLong(PyTuple_GET_ITEM(cap, 1));
      if (want == -1 && PyErr_Occurred()) return nullptr;
      if (vs != want) return PyLong_FromSsize_t(k);
    }
    float* l2p = nullptr;
    if (l2sq != Py_None) {
      if (!THPVariable_Check(l2sq)) Py_RETURN_NONE;
      const at::Tensor& q = THPVariable_Unpack(l2sq);
      if (q.scalar_type() != at::kFloat || q.numel() != K || !q.is_contiguous() || !q.is_cuda() ||
          q.get_device() != dev)
        Py_RETURN_NONE;
      l2p = q.data_ptr<float>();
    }
    const unsigned long long stream =
        reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream());
    std::vector<at::Tensor> outs;
    int rc = 0;
    if (fold_core(row0, ptrs.data(), K, wf.data(), scale, has_scale, nt_min, dev, stream,
                  reinterpret_cast<PlanFn>(plan_addr), reinterpret_cast<WsumFn>(wsum_addr), outs, false,
                  l2p ? reinterpret_cast<WsumL2Fn>(l2_addr) : nullptr,
                  (l2p || rows) ? reinterpret_cast<L2WsFn>(l2ws_addr) : nullptr, l2p, &rc, st, rows) != 0) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_NONE;
    }
    if (rc != 0) return Py_BuildValue("(iO)", rc, Py_None);
    std::vector<PyObject*> wrapped(L);
    for (Py_ssize_t l = 0; l < L; ++l) wrapped[l] = THPVariable_Wrap(std::move(outs[l]));
    size_t i = 0, ki = 0;
    PyObject* tree = rebuild(base, wrapped.data(), i, w.keys.data(), ki);
    for (PyObject* o : wrapped) Py_XDECREF(o);  // (rebuild took the ones it used)
    if (!tree) return nullptr;
    st.lap(kTWrap);
    return Py_BuildValue("(iN)", rc, tree);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyObject* fold_caps(PyObject*, PyObject* args) {
  PyObject *base, *caps, *weights, *l2sq;
  double scale, nt_min;
  int has_scale;
  unsigned long long plan_addr, wsum_addr, l2_addr, l2ws_addr;
  if (!PyArg_ParseTuple(args, "OO!O!dpdKKKKO", &base, &PyList_Type, &caps, &PyList_Type, &weights, &scale,
                        &has_scale, &nt_min, &plan_addr, &wsum_addr, &l2_addr, &l2ws_addr, &l2sq))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(caps);
  if (K < 1 || PyList_GET_SIZE(weights) != K) Py_RETURN_NONE;
  return fold_caps_impl(base, &PyList_GET_ITEM(caps, 0), &PyList_GET_ITEM(weights, 0), K, scale, has_scale != 0,
                        nt_min, plan_addr, wsum_addr, l2_addr, l2ws_addr, l2sq);
}

// leaf_fold(trees, weights, caps, scale, flags, norm_operand, dev, stream, fold_fn, ws_fn)
//     -> (rc, out_tree | None, l2sq | None, l2 | None) | None
// dev = -1: the first leaf's device; stream = 0: torch's current stream on it.
// One fjtree_fold_leaves launch over K = len(trees) operand trees (include/fjtree.h):
// out = [fl(] sum_k fl(x_k * f32(w_k)) [* scale)], plus the l2 norm of operand
// norm_operand with FJTREE_NORM (0-d float32 views of a fresh [2] tensor). caps[k] is
// None or (leaves_tuple, version_sum) from capture(): operand k must still hold exactly
// those leaf objects, unmodified, else rc = -100 (nothing launched). None: not the fast
// case (float32 leaves, <= FJTREE_MAX_LEAVES of them, Python-number weights, matching
// structures), nothing launched.
PyObject* leaf_fold(PyObject*, PyObject* args) {
  PyObject *trees, *weights, *caps;
  double scale;
  int flags, norm_operand, dev;
  unsigned long long stream, fold_addr, ws_addr;
  if (!PyArg_ParseTuple(args, "O!O!O!diiiKKK", &PyList_Type, &trees, &PyList_Type, &weights, &PyList_Type, &caps,
                        &scale, &flags, &norm_operand, &dev, &stream, &fold_addr, &ws_addr))
    return nullptr;
  const Py_ssize_t K = PyList_GET_SIZE(trees);
  if (K < 1 || K > FJTREE_MAX_OPERANDS || PyList_GET_SIZE(weights) != K || PyList_GET_SIZE(caps) != K)
    Py_RETURN_NONE;
  try {
    fjtree_leaves t;
    std::memset(&t, 0, sizeof(t));
    for (Py_ssize_t k = 0; k < K; ++k)
      if (!f32_weight(PyList_GET_ITEM(weights, k), &t.w[k])) Py_RETURN_NONE;
    PWalk w;
    w.K = static_cast<int>(K);
    PyObject* xs[FJTREE_MAX_OPERANDS];
    for (Py_ssize_t k = 0; k < K; ++k) xs[k] = PyList_GET_ITEM(trees, k);
    int rc = pwalk(xs, w, 0);
    if (rc < 0) return nullptr;
    if (rc > 0 || w.leaves[0].empty()) Py_RETURN_NONE;
    if (dev < 0) {  // the first leaf's device, and the caller's current stream on it
      const at::Tensor& t0 = THPVariable_Unpack(w.leaves[0][0]);
      if (!t0.is_cuda()) Py_RETURN_NONE;
      dev = t0.get_device();
    }
    if (stream == 0) stream = reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream(dev).stream());
    const c10::DeviceIndex di = static_cast<c10::DeviceIndex>(dev);
    for (Py_ssize_t k = 0; k < K; ++k) {
      int64_t vs = 0;
      if (!check_leaves(w, static_cast<int>(k), di, &vs)) Py_RETURN_NONE;
      PyObject* cap = PyList_GET_ITEM(caps, k);
      if (cap == Py_None) continue;
      PyObject* tup = PyTuple_GET_ITEM(cap, 0);
      long long cv = PyLong_AsLongLong(PyTuple_GET_ITEM(cap, 1));
      bool same = PyTuple_GET_SIZE(tup) == static_cast<Py_ssize_t>(w.leaves[k].size()) && cv == vs;
      for (size_t l = 0; same && l < w.leaves[k].size(); ++l) {
        same = w.leaves[k][l] == PyTuple_GET_ITEM(tup, l);
        const int64_t cp = captured_ptr(cap, static_cast<Py_ssize_t>(l));
        if (same && cp) same = cp == reinterpret_cast<int64_t>(THPVariable_Unpack(w.leaves[k][l]).data_ptr());
      }
      if (!same) return Py_BuildValue("(iOOO)", kStale, Py_None, Py_None, Py_None);
    }
    const int L = static_cast<int>(w.leaves[0].size());
    const bool norm = flags & FJTREE_NORM, out = !(flags & FJTREE_NO_OUT);
    t.K = static_cast<int>(K);
    t.L = L;
    t.scale = static_cast<float>(scale);
    t.flags = flags;
    t.norm_operand = norm_operand;
    std::vector<at::Tensor> outs;
    outs.reserve(L);
    for (int l = 0; l < L; ++l) {
      const at::Tensor& x0 = THPVariable_Unpack(w.leaves[0][l]);
      for (Py_ssize_t k = 0; k < K; ++k)
        t.x[k][l] = static_cast<const float*>(THPVariable_Unpack(w.leaves[k][l]).data_ptr());
      t.n[l] = x0.numel();
      if (out) {
        outs.push_back(at::empty(x0.sizes(), x0.options()));
        t.out[l] = outs.back().data_ptr<float>();
      }
    }
    at::Tensor nrm;
    if (norm) {
      nrm = at::empty({2}, THPVariable_Unpack(w.leaves[0][0]).options());
      t.norm_out = nrm.data_ptr<float>();
      const int64_t need = reinterpret_cast<TreeWsFn>(ws_addr)(&t);
      // (under a graph capture a workspace of the capture's own: its zeroing fill is recorded, not
      // run, so a cached one would reach later launches with its counter unset)
      at::Tensor own;
      at::Tensor* wsp = &own;
      if (stream_capturing(stream)) {
        own = at::zeros({need > 4096 ? need : 4096}, nrm.options().dtype(at::kByte));
      } else {
        wsp = &workspaces()[WsKey{dev, stream}];
        if (!wsp->defined() || wsp->numel() < need)
          *wsp = at::zeros({need > 4096 ? need * 2 : 8192}, nrm.options().dtype(at::kByte));
      }
      t.ws = wsp->data_ptr();
      t.ws_bytes = wsp->numel();
    }
    rc = reinterpret_cast<TreeFoldFn>(fold_addr)(&t, reinterpret_cast<void*>(stream));
    PyObject* tree_out = Py_None;
    Py_INCREF(Py_None);
    if (out && rc == 0) {
      std::vector<PyObject*> objs(L);
      for (int l = 0; l < L; ++l) objs[l] = THPVariable_Wrap(std::move(outs[l]));
      size_t i = 0, ki = 0;
      PyObject* r = rebuild(xs[0], objs.data(), i, w.keys.data(), ki);
      for (PyObject* o : objs) Py_XDECREF(o);
      if (!r) {
        Py_DECREF(Py_None);
        return nullptr;
      }
      Py_DECREF(Py_None);
      tree_out = r;
    }
    PyObject *sq = Py_None, *l2 = Py_None;
    if (norm && rc == 0) {
      sq = THPVariable_Wrap(nrm.select(0, 0));
      l2 = THPVariable_Wrap(nrm.select(0, 1));
    } else {
      Py_INCREF(Py_None);
      Py_INCREF(Py_None);
    }
    return Py_BuildValue("(iNNN)", rc, tree_out, sq, l2);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// ------------------------------------------------------------------ standalone lazy norms
// examples/fed_avg.py:72-82 takes tree_l2_norm(delta) of every client's delta (:79-81) before
// the tree_mean of the same deltas (:82). A delta no running sum took gets a lazy norm here: a
// 0-d view (tree_util._NormView) into a norm buffer whose value the tree_mean launch that folds
// the delta writes (fjagg_wsum_l2_ptrs_rows, mean_pairs_impl), so the round reads every delta
// once. The view's ticket is a SoloNorm node: the captured leaves (strong references, their
// in-place versions and data pointers) and the version tags of the tree's dict nodes (the mean
// recognises the same, unchanged tree without re-walking it). A view read before a mean folds
// its delta, a delta no mean folds, and the oldest nodes past the pending budget are computed
// by their own pytree-kernel launch (solo_resolve) — the same kernel and plan (every leaf in
// 16-byte units; the per-client reduction order depends on the leaf sizes only), so a norm has
// the same bits whenever it is computed. A captured leaf updated in place before the value is
// computed cannot be recovered: the node turns stale and reading its view raises RuntimeError
// (tree_util.set_lazy_norms(False) opts out, as set_deferred_sums(False) does for the sums).
constexpr int kSoloMaxDicts = 64;
constexpr int64_t kSoloCols = 4096;  // columns of a norm buffer (row 0: squared norms, row 1: norms)
enum { kSoloDone = 0, kSoloPending = 1, kSoloStale = 2 };  // (tp_alloc zeroes: a fresh node is not pending)

struct SoloObject {
  PyObject_HEAD
  PyObject* tree;  // the pytree tree_l2_norm was given (the mean matches clients by identity)
  PyObject* buf;   // float32 [2, kSoloCols] norm buffer
  long long idx;   // this node's column
  long long nbytes;
  int state;
  int L, ndicts, tagged;
  long long vsum;  // the leaves' version sum at the call
  int cap_leaves, cap_dicts;  // capacity of the arrays below (one malloc'd block, kept across reuse)
  const void* order;          // the structure's flatten permutation (solo_structure), or nullptr
  PyObject** leaves;  // [cap_leaves] the captured leaf tensors in the capture walk's order (strong while pending)
  int64_t* ptrs;      // [cap_leaves] their data pointers at the call
  int64_t* tags;      // [2 * cap_dicts] (dict node, PEP 509 version tag), pre-order (tagged)
  PyObject* weakreflist;
};

struct SoloState {
  PyTypeObject* type = nullptr;  // _fjhost.SoloNorm
  bool on = true;                // tree_util.set_lazy_norms
  long long max_pending = 16383;
  long long budget = 0;          // bytes of pending deltas; 0: automatic (py_budget(device) once)
  PyObject* py_budget = nullptr;
  // every node registered since the last compaction, in registration order, with the view handed
  // out for it (strong references both; pooled: the buffer's record holds the view too). A pending
  // node whose view nobody else references any more was dropped by the caller: its capture goes
  // (solo_compact) — the views, not the registry, decide how long a capture lives.
  struct Entry {
    PyObject* view;
    SoloObject* node;
    bool pooled;
  };
  std::vector<Entry> reg;
  long long pending = 0, pending_bytes = 0;
  long long recheck = 0;         // pending bytes at which the budget is checked again (solo_evict)
  PyObject* buf = nullptr;       // the norm buffer new columns come from
  long long next = 0;
  unsigned long long rows_fn = 0, l2ws_fn = 0, plan_fn = 0;  // libfjagg entry points (solo_config)
  long long fused = 0, eager = 0, stale = 0, launches = 0;  // counters (solo_info)
  double t_release = 0, t_compact = 0, t_refill = 0;  // host us spent after the mean's launches (solo_info)
  // Pool of pre-made (norm view, node) pairs over consecutive columns, built right after a mean
  // that fused lazy norms has issued its launches (while the GPU folds) and sized to the norms
  // the round asked for: creating a 0-d tensor subclass and a node on the critical path of the
  // example's loop costs more than the capture itself. Handed-out pairs stay listed per buffer;
  // once a buffer is full and the caller has dropped every view of it (nothing but the pool
  // references them or aliases the storage), its pairs are reused whole on the same stream.
  std::vector<std::pair<PyObject*, PyObject*>> pool;  // (view of row 1, node), ready, in column order
  size_t pool_head = 0;
  struct BufRec {
    PyObject* buf;
    unsigned long long stream;
    std::vector<std::pair<PyObject*, PyObject*>> pairs;  // handed-out pool pairs of this buffer
  };
  std::vector<BufRec> bufs;
  long long want = 0;  // row-1 norms asked for since the last refill
  long long pool_builds = 0, pool_reuses = 0;
  double refill_us = 0.0;
};
SoloState g_solo;

void solo_release(SoloObject* n, int state) {
  if (n->state == kSoloPending) {
    --g_solo.pending;
    g_solo.pending_bytes -= n->nbytes;
  }
  n->state = state;
  Py_CLEAR(n->tree);
  for (int l = 0; l < n->L; ++l) Py_CLEAR(n->leaves[l]);
}

int solo_traverse(PyObject* o, visitproc visit, void* arg) {
  auto* n = reinterpret_cast<SoloObject*>(o);
  Py_VISIT(Py_TYPE(o));
  Py_VISIT(n->tree);
  Py_VISIT(n->buf);
  for (int l = 0; l < n->L && n->leaves; ++l) Py_VISIT(n->leaves[l]);
  return 0;
}
int solo_clear(PyObject* o) {
  auto* n = reinterpret_cast<SoloObject*>(o);
  if (n->state == kSoloPending) solo_release(n, kSoloDone);  // (dropped unread: nothing to compute)
  Py_CLEAR(n->tree);
  Py_CLEAR(n->buf);
  for (int l = 0; l < n->L && n->leaves; ++l) Py_CLEAR(n->leaves[l]);
  return 0;
}
void solo_dealloc(PyObject* o) {
  PyTypeObject* tp = Py_TYPE(o);
  PyObject_GC_UnTrack(o);
  auto* n = reinterpret_cast<SoloObject*>(o);
  if (n->weakreflist) PyObject_ClearWeakRefs(o);
  solo_clear(o);
  PyMem_Free(n->leaves);
  tp->tp_free(o);
  Py_DECREF(tp);
}
// `node`: the node itself while its value is not written (flush_views then computes it, or
// raises for a stale one), None once it is — the protocol of tree_util._Ticket.node
PyObject* solo_get_node(PyObject* o, void*) {
  PyObject* r = reinterpret_cast<SoloObject*>(o)->state == kSoloDone ? Py_None : o;
  Py_INCREF(r);
  return r;
}
PyGetSetDef kSoloGetSet[] = {{const_cast<char*>("node"), solo_get_node, nullptr, nullptr, nullptr},
                             {nullptr}};
PyMemberDef kSoloMembers[] = {
    {const_cast<char*>("_tree"), T_OBJECT, offsetof(SoloObject, tree), READONLY, nullptr},
    {const_cast<char*>("_buf"), T_OBJECT, offsetof(SoloObject, buf), READONLY, nullptr},
    {const_cast<char*>("_idx"), T_LONGLONG, offsetof(SoloObject, idx), READONLY, nullptr},
    {const_cast<char*>("_state"), T_INT, offsetof(SoloObject, state), READONLY, nullptr},
    {const_cast<char*>("__weaklistoffset__"), T_PYSSIZET, offsetof(SoloObject, weakreflist), READONLY, nullptr},
    {nullptr}};
PyType_Slot kSoloSlots[] = {{Py_tp_dealloc, reinterpret_cast<void*>(solo_dealloc)},
                            {Py_tp_traverse, reinterpret_cast<void*>(solo_traverse)},
                            {Py_tp_clear, reinterpret_cast<void*>(solo_clear)},
                            {Py_tp_members, kSoloMembers},
                            {Py_tp_getset, kSoloGetSet},
                            {Py_tp_doc, const_cast<char*>("a standalone lazy l2 norm's capture (fjhost.cpp)")},
                            {0, nullptr}};
PyType_Spec kSoloSpec = {"_fjhost.SoloNorm", sizeof(SoloObject), 0, Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC,
                         kSoloSlots};

// room for L leaves and D dict tags in n's arrays (false: out of memory, no error set)
bool solo_reserve(SoloObject* n, int L, int D) {
  if (n->leaves && L <= n->cap_leaves && D <= n->cap_dicts) return true;
  const int cl = std::max(L, 16), cd = std::max(D, 8);
  void* blk = PyMem_Malloc(sizeof(PyObject*) * cl + sizeof(int64_t) * (cl + 2 * cd));
  if (!blk) return false;
  for (int l = 0; l < n->L && n->leaves; ++l) Py_CLEAR(n->leaves[l]);
  PyMem_Free(n->leaves);
  n->leaves = static_cast<PyObject**>(blk);
  n->ptrs = reinterpret_cast<int64_t*>(n->leaves + cl);
  n->tags = n->ptrs + cl;
  n->cap_leaves = cl;
  n->cap_dicts = cd;
  n->L = 0;
  std::memset(n->leaves, 0, sizeof(PyObject*) * cl);
  return true;
}

// The captured leaves still hold the values of the call: same versions, same storage.
bool solo_unchanged(const SoloObject* n) {
  int64_t vs = 0;
  for (int l = 0; l < n->L; ++l) {
    const at::Tensor& t = THPVariable_Unpack(n->leaves[l]);
    vs += static_cast<int64_t>(t._version());
    if (reinterpret_cast<int64_t>(t.data_ptr()) != n->ptrs[l]) return false;
  }
  return vs == n->vsum;
}

// The capture walk: every dict (pre-order, values in insertion order — no key sort), list / tuple
// and None node, exact torch.Tensor leaves. 0 walked; 1 not the fast case.
// sig (optional): the walked structure in walk order — kLeaf, kNone, (kList | kTuple, n, children),
// (kDict, n, then per item its key object and the child's entries) — for solo_structure.
int solo_walk(PyObject* x, std::vector<PyObject*>& lv, std::vector<PyObject*>& dv, bool& lists, int depth,
              std::vector<int64_t>* sig = nullptr) {
  if (depth > 64) return 1;
  if (Py_TYPE(x) == reinterpret_cast<PyTypeObject*>(THPVariableClass)) {
    lv.push_back(x);
    if (sig) sig->push_back(kLeaf);
    return lv.size() > static_cast<size_t>(FJTREE_MAX_LEAVES);
  }
  if (x == Py_None) {
    if (sig) sig->push_back(kNone);
    return 0;
  }
  if (PyDict_CheckExact(x)) {
    dv.push_back(x);
    if (sig) sig->push_back(kDict), sig->push_back(PyDict_GET_SIZE(x));
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(x, &pos, &k, &v)) {
      if (sig) sig->push_back(reinterpret_cast<int64_t>(k));
      if (solo_walk(v, lv, dv, lists, depth + 1, sig)) return 1;
    }
    return 0;
  }
  const bool is_list = PyList_CheckExact(x);
  if (!is_list && !PyTuple_CheckExact(x)) return 1;
  lists = lists || is_list;
  if (sig) sig->push_back(is_list ? kList : kTuple), sig->push_back(Py_SIZE(x));
  for (Py_ssize_t i = 0; i < Py_SIZE(x); ++i)
    if (solo_walk(is_list ? PyList_GET_ITEM(x, i) : PyTuple_GET_ITEM(x, i), lv, dv, lists, depth + 1, sig))
      return 1;
  return 0;
}

// The flatten order (jax's: dict keys sorted) of the capture walk's leaf order, per structure:
// structures are interned by their walk signature (the table keeps their key objects alive, so a
// key's address is never reused while its entry exists), the permutation computed once, when a
// structure is first seen (perm[f] = the walk-order index of flatten leaf f). -1: no order (keys
// that do not sort, or the table is full): not the fast case.
struct SoloStruct {
  std::vector<int32_t> perm;
};
int solo_sort_walk(const std::vector<int64_t>& sig, size_t& i, int& leaf, std::vector<int32_t>& out) {
  const int64_t kind = sig[i++];
  if (kind == kLeaf) {
    out.push_back(leaf++);
    return 0;
  }
  if (kind == kNone) return 0;
  const int64_t n = sig[i++];
  if (kind == kList || kind == kTuple) {
    for (int64_t c = 0; c < n; ++c)
      if (solo_sort_walk(sig, i, leaf, out)) return 1;
    return 0;
  }
  // a dict: its children's flatten orders, concatenated in key order
  std::vector<std::pair<PyObject*, std::vector<int32_t>>> kids(static_cast<size_t>(n));
  for (int64_t c = 0; c < n; ++c) {
    kids[c].first = reinterpret_cast<PyObject*>(sig[i++]);
    if (solo_sort_walk(sig, i, leaf, kids[c].second)) return 1;
  }
  bool bad = false;
  std::stable_sort(kids.begin(), kids.end(), [&](const auto& a, const auto& b) {
    if (bad) return false;
    const int r = PyObject_RichCompareBool(a.first, b.first, Py_LT);
    if (r < 0) {
      PyErr_Clear();
      bad = true;
      return false;
    }
    return r == 1;
  });
  if (bad) return 1;
  for (auto& k : kids) out.insert(out.end(), k.second.begin(), k.second.end());
  return 0;
}
const SoloStruct* solo_structure(const std::vector<int64_t>& sig) {
  static auto* table = new std::unordered_map<std::vector<int64_t>, int64_t, SigHash>();
  static auto* structs = new std::deque<SoloStruct>();  // (stable addresses: nodes point at entries)
  static std::vector<int64_t> last_sig;
  static int64_t last = -1;
  if (last >= 0 && sig == last_sig) return &(*structs)[last];
  auto it = table->find(sig);
  if (it != table->end()) {
    last_sig = sig;
    last = it->second;
    return it->second >= 0 ? &(*structs)[it->second] : nullptr;
  }
  if (table->size() >= 4096) return nullptr;
  SoloStruct st;
  size_t i = 0;
  int leaf = 0;
  const bool ok = solo_sort_walk(sig, i, leaf, st.perm) == 0 && i == sig.size();
  int64_t id = -1;
  if (ok) {
    id = static_cast<int64_t>(structs->size());
    structs->push_back(std::move(st));
  }
  // keep the key objects alive for as long as the entry exists (their addresses are in the sig)
  {
    size_t j = 0;
    std::function<void()> walk = [&]() {
      const int64_t kind = sig[j++];
      if (kind == kLeaf || kind == kNone) return;
      const int64_t n = sig[j++];
      for (int64_t c = 0; c < n; ++c) {
        if (kind == kDict) Py_INCREF(reinterpret_cast<PyObject*>(sig[j++]));
        walk();
      }
    };
    walk();
  }
  table->emplace(sig, id);
  last_sig = sig;
  last = id;
  return id >= 0 ? &(*structs)[id] : nullptr;
}

// The same leaf objects, in any order (L <= FJTREE_MAX_LEAVES).
bool same_leaf_set(PyObject* const* a, PyObject* const* b, int L) {
  PyObject* x[FJTREE_MAX_LEAVES];
  PyObject* y[FJTREE_MAX_LEAVES];
  std::memcpy(x, a, sizeof(PyObject*) * L);
  std::memcpy(y, b, sizeof(PyObject*) * L);
  std::sort(x, x + L);
  std::sort(y, y + L);
  return std::equal(x, x + L, y);
}

// `tree` is the node's tree and still holds exactly the captured leaves: its dict nodes' version
// tags unchanged (pre-order: a dict is read only after its parent was found unchanged, so it is
// alive), or for a tree with list nodes a walk finding the same leaf objects.
bool solo_same_tree(const SoloObject* n, PyObject* tree) {
  if (n->tree != tree) return false;
#if PY_VERSION_HEX < 0x030C0000
  if (n->tagged) {
    for (int i = 0; i < n->ndicts; ++i)
      if (static_cast<int64_t>(reinterpret_cast<PyDictObject*>(n->tags[2 * i])->ma_version_tag) != n->tags[2 * i + 1])
        return false;
    return true;
  }
#endif
  thread_local std::vector<PyObject*> lv, dv;
  lv.clear();
  dv.clear();
  bool lists = false;
  if (solo_walk(tree, lv, dv, lists, 0) != 0 || static_cast<int>(lv.size()) != n->L) return false;
  return same_leaf_set(lv.data(), n->leaves, n->L);
}

// Captures `tree` into node n (not yet pending). false: not the fast case (float32 CUDA leaves,
// strided, contiguous, one device, versioned, <= FJTREE_MAX_LEAVES, some element) or no memory.
bool solo_capture_into(SoloObject* n, PyObject* tree) {
  thread_local std::vector<PyObject*> lv, dv;
  thread_local std::vector<int64_t> sig;
  lv.clear();
  dv.clear();
  sig.clear();
  bool lists = false;
  if (solo_walk(tree, lv, dv, lists, 0, &sig) != 0 || lv.empty()) return false;
  const SoloStruct* order = solo_structure(sig);
  if (!order || order->perm.size() != lv.size()) return false;  // (keys that do not sort: the Python path)
  const int L = static_cast<int>(lv.size());
  int dev = -1;
  int64_t vs = 0, numel = 0;
  for (PyObject* x : lv) {
    const at::Tensor& t = THPVariable_Unpack(x);
    if (t.layout() != c10::kStrided || t.scalar_type() != at::kFloat || !t.is_cuda() || !t.is_contiguous() ||
        t.is_inference())
      return false;
    if (dev < 0) dev = t.get_device();
    if (t.get_device() != dev) return false;
    vs += static_cast<int64_t>(t._version());
    numel += t.numel();
  }
  if (numel == 0) return false;  // (the Python path returns a zero)
  const bool tagged = !lists && dv.size() <= static_cast<size_t>(kSoloMaxDicts);
  if (!solo_reserve(n, L, tagged ? static_cast<int>(dv.size()) : 0)) return false;
  n->L = L;
  n->vsum = vs;
  n->nbytes = 4 * numel;
  n->order = order;
  for (int l = 0; l < L; ++l) {
    Py_INCREF(lv[l]);
    n->leaves[l] = lv[l];
    n->ptrs[l] = reinterpret_cast<int64_t>(THPVariable_Unpack(lv[l]).data_ptr());
  }
#if PY_VERSION_HEX < 0x030C0000
  n->tagged = tagged;
  n->ndicts = tagged ? static_cast<int>(dv.size()) : 0;
  for (int i = 0; i < n->ndicts; ++i) {
    n->tags[2 * i] = reinterpret_cast<int64_t>(dv[i]);
    n->tags[2 * i + 1] = static_cast<int64_t>(reinterpret_cast<PyDictObject*>(dv[i])->ma_version_tag);
  }
#else
  n->tagged = 0;
  n->ndicts = 0;
#endif
  Py_INCREF(tree);
  Py_XSETREF(n->tree, tree);
  return true;
}

// The captured leaves of a node in flatten order (jax's: dict keys sorted) — the order the mean's
// fused fold reads them in, so a norm computed on its own has the fused value's bits, whether
// or not the tree has changed since the call (the permutation is the captured structure's).
void solo_flatten_order(const SoloObject* n, std::vector<PyObject*>& out) {
  const auto* st = static_cast<const SoloStruct*>(n->order);
  out.resize(static_cast<size_t>(n->L));
  for (int f = 0; f < n->L; ++f) out[f] = n->leaves[st->perm[f]];
}

// every captured pointer 16-byte aligned: the mean's fused plan (no element units) is this node's
bool solo_aligned(const SoloObject* n) {
  for (int l = 0; l < n->L; ++l)
    if (n->ptrs[l] & 15) return false;
  return true;
}

// Computes the values of `nodes` (pending ones; others are skipped) by pytree-kernel launches on
// the current stream, the leaves in flatten order (solo_flatten_order): runs of consecutive
// columns of one buffer with equal leaf shapes, every pointer aligned, fold together (the fold's
// outputs are dropped); a misaligned node folds alone (its own element-unit plan, as every
// computation of it). A node whose leaves changed turns stale. 0, or -1 with a Python error.
int solo_resolve(std::vector<SoloObject*>& nodes) {
  std::vector<SoloObject*> todo;
  for (SoloObject* n : nodes) {
    if (n->state != kSoloPending) continue;
    if (!solo_unchanged(n)) {
      solo_release(n, kSoloStale);
      ++g_solo.stale;
      continue;
    }
    todo.push_back(n);
  }
  if (todo.empty()) return 0;
  if (!g_solo.rows_fn || !g_solo.l2ws_fn || !g_solo.plan_fn) {
    PyErr_SetString(PyExc_RuntimeError, "lazy norms: libfjagg entry points not configured (solo_config)");
    return -1;
  }
  std::stable_sort(todo.begin(), todo.end(), [](const SoloObject* a, const SoloObject* b) {
    return a->buf != b->buf ? a->buf < b->buf : a->idx < b->idx;
  });
  for (SoloObject* n : todo) Py_INCREF(n);
  struct Drop {
    std::vector<SoloObject*>& v;
    ~Drop() {
      for (SoloObject* n : v) Py_DECREF(n);
    }
  } drop{todo};
  try {
    std::vector<std::vector<PyObject*>> order(todo.size());
    for (size_t i = 0; i < todo.size(); ++i) solo_flatten_order(todo[i], order[i]);
    auto same_shape = [&](size_t i, size_t j) {
      if (order[i].size() != order[j].size()) return false;
      for (size_t l = 0; l < order[i].size(); ++l)
        if (THPVariable_Unpack(order[j][l]).sizes() != THPVariable_Unpack(order[i][l]).sizes()) return false;
      return true;
    };
    size_t i = 0;
    while (i < todo.size()) {
      SoloObject* a = todo[i];
      const bool al = solo_aligned(a);
      const int dev = THPVariable_Unpack(a->leaves[0]).get_device();
      size_t j = i + 1;
      while (al && j < todo.size() && j - i < 4096 && todo[j]->buf == a->buf &&
             todo[j]->idx == a->idx + static_cast<long long>(j - i) && solo_aligned(todo[j]) && same_shape(i, j) &&
             THPVariable_Unpack(todo[j]->leaves[0]).get_device() == dev)
        ++j;
      const int64_t K = static_cast<int64_t>(j - i), L = a->L;
      std::vector<at::Tensor> row0;
      row0.reserve(L);
      for (int64_t l = 0; l < L; ++l) row0.push_back(THPVariable_Unpack(order[i][l]));
      std::vector<int64_t> ptrs(static_cast<size_t>(K * L));
      for (int64_t k = 0; k < K; ++k)
        for (int64_t l = 0; l < L; ++l)
          ptrs[k * L + l] = reinterpret_cast<int64_t>(THPVariable_Unpack(order[i + k][l]).data_ptr());
      std::vector<float> wf(static_cast<size_t>(K), 1.0f);
      const unsigned long long stream = reinterpret_cast<unsigned long long>(
          c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream());
      const at::Tensor& b = THPVariable_Unpack(a->buf);
      if (b.get_device() != dev) {
        PyErr_SetString(PyExc_RuntimeError, "lazy norms: a norm buffer on another device than its delta");
        return -1;
      }
      float* r0 = b.data_ptr<float>() + a->idx;
      L2Rows rows{reinterpret_cast<WsumL2RowsFn>(g_solo.rows_fn), r0, r0 + b.stride(0), 0};
      std::vector<at::Tensor> outs;  // (fresh, dropped: only the norms are wanted)
      int rc = 0;
      Stamp st;
      if (fold_core(row0, ptrs.data(), K, wf.data(), 1.0, false, HUGE_VAL, dev, stream,
                    reinterpret_cast<PlanFn>(g_solo.plan_fn), nullptr, outs, false, nullptr,
                    reinterpret_cast<L2WsFn>(g_solo.l2ws_fn), nullptr, &rc, st, &rows) != 0) {
        if (PyErr_Occurred()) return -1;
        PyErr_SetString(PyExc_RuntimeError, "lazy norms: the captured leaves are not a fold's case");
        return -1;
      }
      if (rc != 0) {
        PyErr_Format(PyExc_RuntimeError, "lazy norms: fjagg_wsum_l2_ptrs_rows failed (%d)", rc);
        return -1;
      }
      ++g_solo.launches;
      for (size_t q = i; q < j; ++q) {
        solo_release(todo[q], kSoloDone);
        ++g_solo.eager;
      }
      i = j;
    }
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return -1;
  }
  return 0;
}

// Drops the registry entries of nodes that are no longer pending, after releasing the capture of a
// pending node whose view only the registry (and its buffer's record) still references: the caller
// dropped it, nobody can read the value.
void solo_compact() {
  size_t o = 0;
  for (auto& e : g_solo.reg) {
    // (no view of the node left outside: the registry's view and node references, the record's
    // pair when pooled, and that view's _ticket are all that hold them)
    if (e.node->state == kSoloPending && Py_REFCNT(e.view) <= (e.pooled ? 2 : 1) &&
        Py_REFCNT(reinterpret_cast<PyObject*>(e.node)) <= (e.pooled ? 3 : 2) &&
        THPVariable_Unpack(e.view).use_count() == 1)
      solo_release(e.node, kSoloDone);
    if (e.node->state == kSoloPending) {
      g_solo.reg[o++] = e;
    } else {
      Py_DECREF(e.view);
      Py_DECREF(reinterpret_cast<PyObject*>(e.node));
    }
  }
  g_solo.reg.resize(o);
  if (g_solo.pending == 0) g_solo.recheck = 0;
}

// every pending node, oldest first (the budget's eviction and solo_resolve(None))
int solo_resolve_all() {
  solo_compact();
  std::vector<SoloObject*> v;
  for (auto& e : g_solo.reg)
    if (e.node->state == kSoloPending) v.push_back(e.node);  // (the registry holds them)
  const int rc = solo_resolve(v);
  solo_compact();
  return rc;
}

// the pending nodes whose pytree only the node holds (the deltas their views alone keep alive)
int solo_evict() {
  solo_compact();
  std::vector<SoloObject*> v;
  for (auto& e : g_solo.reg)
    if (e.node->state == kSoloPending && e.node->tree && Py_REFCNT(e.node->tree) <= 1) v.push_back(e.node);
  const int rc = solo_resolve(v);
  solo_compact();
  return rc;
}

// The mean's side: the pending node of a client's tree, checked unchanged, or nullptr. The
// registry entry after the previous match is tried first (clients in registration order); after
// a miss, a map of the pending nodes by tree (built once per mean) answers.
struct SoloMatcher {
  size_t cursor = 0;
  bool built = false;
  std::unordered_map<PyObject*, SoloObject*> by_tree;
  SoloObject* match(PyObject* tree, int L) {
    SoloObject* n = nullptr;
    const size_t R = g_solo.reg.size();
    for (size_t p = cursor; p < R && p < cursor + 2 && !n; ++p) {
      SoloObject* c = g_solo.reg[p].node;
      if (c->tree == tree && c->state == kSoloPending) {
        n = c;
        cursor = p + 1;
      }
    }
    if (!n) {
      if (!built) {
        built = true;
        for (auto& e : g_solo.reg)  // (registration order: a tree's earliest pending node)
          if (e.node->state == kSoloPending && e.node->tree) by_tree.emplace(e.node->tree, e.node);
      }
      auto it = by_tree.find(tree);
      if (it == by_tree.end() || it->second->state != kSoloPending) return nullptr;
      n = it->second;
    }
    return (n->L == L && solo_same_tree(n, tree) && solo_unchanged(n)) ? n : nullptr;
  }
};

int solo_refill(int dev, unsigned long long stream);  // (the lazy-norm pool, below: uses the view type)

// ------------------------------------------------------------------ tree_mean, whole call
// tree_mean(list of (pytree, weight)) in one native call for the common case: exact dict /
// list / tuple / None nodes over float32 CUDA tensors (contiguous, client 0's shapes, one
// device), Python int / float weights. The same launches as the Python path
// (gather_rows + fold_weights + fold_table), and the idle-stream pipeline of
// tree_util._tree_mean_pipelined. Anything else is "not this case": None (nothing launched,
// or launches whose outputs are dropped) and the Python path runs, raising the reference's
// errors.

// Walk program of tree x (the format of pytree.native_spec: 0 leaf, 1 None, (2, sorted keys,
// children) dict, (3|4, n, children) list / tuple) with its tensor leaves in flatten order
// and the sorted key list of every dict in pre-order (for rebuild). nullptr: not the fast
// case when no Python error is set.
struct SpecBuild {
  std::vector<PyObject*> leaves;  // borrowed
  std::vector<PyObject*> keys;    // owned
  ~SpecBuild() {
    for (PyObject* k : keys) Py_DECREF(k);
  }
};

PyObject* spec_of(PyObject* x, SpecBuild& b, int depth) {
  if (depth > 64) return nullptr;
  if (Py_TYPE(x) == reinterpret_cast<PyTypeObject*>(THPVariableClass)) {
    b.leaves.push_back(x);
    return PyLong_FromLong(kLeaf);
  }
  if (x == Py_None) return PyLong_FromLong(kNone);
  const bool is_dict = PyDict_CheckExact(x), is_list = PyList_CheckExact(x), is_tuple = PyTuple_CheckExact(x);
  if (!is_dict && !is_list && !is_tuple) return nullptr;
  PyObject* keys = nullptr;
  Py_ssize_t n;
  if (is_dict) {
    bool unorderable = false;
    keys = sorted_keys(x, &unorderable);
    if (!keys) return nullptr;  // (unorderable keys: no error set, the Python path decides)
    b.keys.push_back(keys);
    n = PyList_GET_SIZE(keys);
  } else {
    n = Py_SIZE(x);
  }
  PyObject* children = PyTuple_New(n);
  if (!children) return nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* c = is_dict ? PyDict_GetItem(x, PyList_GET_ITEM(keys, i))
                          : (is_list ? PyList_GET_ITEM(x, i) : PyTuple_GET_ITEM(x, i));
    PyObject* cs = c ? spec_of(c, b, depth + 1) : nullptr;
    if (!cs) {
      Py_DECREF(children);
      return nullptr;
    }
    PyTuple_SET_ITEM(children, i, cs);
  }
  PyObject* aux = is_dict ? PyList_AsTuple(keys) : PyLong_FromSsize_t(n);
  if (!aux) {
    Py_DECREF(children);
    return nullptr;
  }
  return Py_BuildValue("(lNN)", is_dict ? (long)kDict : is_list ? (long)kList : (long)kTuple, aux, children);
}

// chunk ends of mean_pairs' fold-bound pipeline as fractions of K (pipeline_fracs(); empty:
// the single `frac` argument)
std::vector<double> g_pipeline_fracs;

PyObject* pipeline_fracs(PyObject*, PyObject* arg) {
  PyObject* seq = PySequence_Fast(arg, "pipeline_fracs: a sequence of floats");
  if (!seq) return nullptr;
  std::vector<double> v;
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); ++i) {
    const double f = PyFloat_AsDouble(PySequence_Fast_GET_ITEM(seq, i));
    if (f == -1.0 && PyErr_Occurred()) {
      Py_DECREF(seq);
      return nullptr;
    }
    v.push_back(f);
  }
  Py_DECREF(seq);
  g_pipeline_fracs.swap(v);
  Py_RETURN_NONE;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// mean_pairs(pairs, may_pipeline, frac, chunk, chunk_walk_us, walk_ns_per_leaf, min_bytes,
//            narrow_max, nt_min_bytes, plan_fn, wsum_fn[, wsum_l2_fn, l2_ws_bytes_fn])
//   -> (rc, tree, job_bytes, l2sq | None) | None
// With the l2 entry points every client's squared l2 norm over all leaves comes from the
// launch that folds it (fjagg_wsum_l2_ptrs; K <= 4096, the caller checks).
// may_pipeline: the caller's host-side estimate says the stream may be idle (then the
// stream is probed). The chunking is tree_util._pipeline_bounds's.
// triples: the items are mean_aggregator().apply's (client_id, params, weight) triples
// (aggregator.py:61-75), read as (params, weight) without building the pairs list.
PyObject* mean_pairs_impl(PyObject* pairs, bool triples, int may_pipeline, double frac, long long chunk,
                          double chunk_walk_us, double walk_ns, long long min_bytes, long long narrow_max,
                          double nt_min, unsigned long long plan_addr, unsigned long long wsum_addr,
                          unsigned long long l2_addr, unsigned long long l2ws_addr) {
  const bool with_l2 = l2_addr != 0 && l2ws_addr != 0;  // tree_mean_with_l2_norms: + every client's l2sq
  if (!PyList_CheckExact(pairs) && !PyTuple_CheckExact(pairs)) Py_RETURN_NONE;
  const Py_ssize_t K = Py_SIZE(pairs);
  if (K < 1) Py_RETURN_NONE;
  PyObject* const* items = PyList_CheckExact(pairs) ? &PyList_GET_ITEM(pairs, 0) : &PyTuple_GET_ITEM(pairs, 0);
  Stamp st;
  const auto t_entry = st.t;
  ++g_timer_calls;
  try {
    // the trees are held by new references for the call: key comparisons during the walks
    // can run Python code, which could otherwise drop the caller's last reference
    struct Held {
      std::vector<PyObject*> v;
      ~Held() {
        for (PyObject* o : v) Py_XDECREF(o);
      }
    } held;
    held.v.assign(K, nullptr);
    std::vector<PyObject*>& trees = held.v;
    std::vector<float> wf(K);
    double W = 0.0;
    // pairs [parsed, k1) -> trees, f32 weights, W (tree_util.py:89,95, in order); parsed
    // chunk by chunk, so the first launch does not wait for the whole list. false: a pair
    // or weight this path does not take (the caller's Python path then does)
    Py_ssize_t parsed = 0;
    auto parse = [&](Py_ssize_t k1) {
      for (; parsed < k1; ++parsed) {  // `for pytree, weight in pytrees_and_weights`
        PyObject* pr = items[parsed];
        PyObject *t, *w;
        const Py_ssize_t o = triples ? 1 : 0, n = o + 2;
        if (PyTuple_CheckExact(pr) && PyTuple_GET_SIZE(pr) == n) {
          t = PyTuple_GET_ITEM(pr, o);
          w = PyTuple_GET_ITEM(pr, o + 1);
        } else if (PyList_CheckExact(pr) && PyList_GET_SIZE(pr) == n) {
          t = PyList_GET_ITEM(pr, o);
          w = PyList_GET_ITEM(pr, o + 1);
        } else {
          return false;
        }
        double d;
        if (PyLong_CheckExact(w)) {
          int overflow = 0;
          long long v = PyLong_AsLongLongAndOverflow(w, &overflow);
          if (PyErr_Occurred()) PyErr_Clear();
          if (overflow || v >= (1LL << 53) || v <= -(1LL << 53)) return false;
          d = static_cast<double>(v);
        } else if (PyFloat_CheckExact(w)) {
          d = PyFloat_AS_DOUBLE(w);
        } else {
          return false;
        }
        Py_INCREF(t);
        trees[parsed] = t;
        wf[parsed] = static_cast<float>(d);
        W += d;  // tree_util.py:95
      }
      return true;
    };
    if (!parse(1)) Py_RETURN_NONE;
    SpecBuild sb;
    PyObject* spec = spec_of(trees[0], sb, 0);
    if (!spec) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_NONE;
    }
    struct Ref {
      PyObject* o;
      ~Ref() { Py_DECREF(o); }
    } spec_ref{spec};
    const int64_t L = static_cast<int64_t>(sb.leaves.size());
    if (L < 1) Py_RETURN_NONE;
    std::vector<at::Tensor> row0;
    row0.reserve(L);
    std::vector<at::ScalarType> dtypes;
    std::vector<c10::IntArrayRef> sizes;
    int64_t n = 0;
    int dev = -1;
    for (PyObject* x : sb.leaves) {
      const at::Tensor& t = THPVariable_Unpack(x);
      if (t.layout() != c10::kStrided || !t.is_cuda() || t.scalar_type() != at::kFloat || !t.is_contiguous())
        Py_RETURN_NONE;
      if (dev < 0) dev = t.get_device();
      if (t.get_device() != dev) Py_RETURN_NONE;
      row0.push_back(t);
      n += t.numel();
    }
    if (n == 0) Py_RETURN_NONE;
    for (const at::Tensor& t : row0) {
      dtypes.push_back(t.scalar_type());
      sizes.push_back(t.sizes());
    }
    const double job_bytes = 4.0 * static_cast<double>(n) * static_cast<double>(K);
    const unsigned long long stream =
        reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream());
    // chunk ends (tree_util._pipeline_bounds), pipelined only on an idle stream
    std::vector<int64_t> bounds;
    if (may_pipeline && frac > 0.0 && K >= 8 && 4 * n > narrow_max && job_bytes >= static_cast<double>(min_bytes) &&
        hipStreamQuery(reinterpret_cast<hipStream_t>(stream)) == hipSuccess) {
      const double wns = walk_ns * L, fns = 4.0 * n / 8.0e12 * 1e9;
      int64_t c = 0;
      if (wns > fns && chunk > 0) {
        c = std::max<int64_t>(chunk, static_cast<int64_t>(std::ceil(chunk_walk_us * 1e3 / wns)));
        if (K <= c) c = 0;
      }
      if (c > 0) {
        for (int64_t k1 = c; k1 < K; k1 += c) bounds.push_back(k1);
      } else if (!g_pipeline_fracs.empty()) {  // pipeline_fracs(): several first chunks
        int64_t prev = 0;
        for (double f : g_pipeline_fracs) {
          const int64_t k1 = std::min<int64_t>(K - 1, std::max<int64_t>(prev + 1, static_cast<int64_t>(K * f)));
          if (k1 > prev && k1 < K) bounds.push_back(k1), prev = k1;
        }
      } else {
        bounds.push_back(std::min<int64_t>(K - 1, std::max<int64_t>(1, static_cast<int64_t>(K * frac))));
      }
    }
    bounds.push_back(K);
    st.lap(kTSpec);
    std::vector<int64_t> ptrs(static_cast<size_t>(K * L));
    for (int64_t l = 0; l < L; ++l) ptrs[l] = reinterpret_cast<int64_t>(row0[l].data_ptr());
    const double ntm = job_bytes >= nt_min ? 0.0 : HUGE_VAL;  // the whole job's bytes decide
    std::vector<at::Tensor> outs;
    at::Tensor l2sq;  // float32 [K] (with_l2): client k's squared norm from the launch that folds it
    if (with_l2) l2sq = at::empty({K}, row0[0].options());
    int64_t done = 0;
    int rc = 0;
    // standalone lazy norms of these clients (examples/fed_avg.py:79-81): a chunk whose clients
    // all have pending nodes in consecutive columns of one buffer folds with the norms written
    // straight into those columns (fjagg_wsum_l2_ptrs_rows); the nodes are done once every
    // launch is issued
    if (!with_l2 && !g_solo.reg.empty()) solo_compact();
    // (not under a graph capture: a replay would write those columns again, and a column is handed
    // out again once its view is dropped; the pending norms are computed on their own when read)
    bool solo = !with_l2 && g_solo.pending > 0 && g_solo.rows_fn && g_solo.l2ws_fn && !stream_capturing(stream);
    std::vector<SoloObject*> fused;  // held (new references) until the call returns
    struct HeldNodes {
      std::vector<SoloObject*>& v;
      ~HeldNodes() {
        for (SoloObject* n : v) Py_DECREF(n);
      }
    } held_nodes{fused};
    SoloMatcher matcher;
    SoloObject* next_node = nullptr;  // a match found past the end of the previous run (borrowed)
    bool next_none = false;           // the client past the previous run has no pending node
    for (int64_t k1 : bounds) {
      if (!parse(k1)) Py_RETURN_NONE;
      const int64_t r = gather_clients(spec, trees.data(), std::max<int64_t>(done, 1), k1, dtypes, sizes,
                                       static_cast<c10::DeviceIndex>(dev), ptrs.data());
      if (r < 0) return nullptr;
      if (r > 0) Py_RETURN_NONE;
      // the chunk folds in runs: clients whose pending nodes sit in consecutive columns of one
      // buffer fold with their norms written there, clients without one fold plainly. Any split
      // gives the same bits (accumulate mode).
      for (int64_t a = done; a < k1;) {
        int64_t b = k1;
        L2Rows rows{};
        bool use_rows = false;
        const size_t f0 = fused.size();
        if (solo) {
          SoloObject* n0 = next_node ? next_node : next_none ? nullptr : matcher.match(trees[a], static_cast<int>(L));
          next_node = nullptr;
          next_none = false;
          b = a + 1;
          if (n0) {
            Py_INCREF(n0);
            fused.push_back(n0);
            while (b < k1 && b - a < 4096) {  // (fjagg_wsum_l2_ptrs: K <= 4096)
              SoloObject* n = matcher.match(trees[b], static_cast<int>(L));
              if (!n || n->buf != n0->buf || n->idx != n0->idx + (b - a)) {
                next_node = n;
                next_none = !n;
                break;
              }
              Py_INCREF(n);
              fused.push_back(n);
              ++b;
            }
            const at::Tensor& bt = THPVariable_Unpack(n0->buf);
            float* r0 = bt.data_ptr<float>() + n0->idx;
            rows = L2Rows{reinterpret_cast<WsumL2RowsFn>(g_solo.rows_fn), r0, r0 + bt.stride(0), 0, true};
            use_rows = bt.get_device() == dev;
          } else {
            while (b < k1) {  // a run of clients without pending norms: one plain fold
              SoloObject* n = matcher.match(trees[b], static_cast<int>(L));
              if (n) {
                next_node = n;
                break;
              }
              ++b;
            }
          }
        }
        const bool last = b == K;  // (then every weight is parsed: W is complete)
        const double scale = last ? (W > 0.0 ? 1.0 / W : 0.0) : 1.0;  // tree_util.py:37,60
        const bool acc = !outs.empty();
        int got = 2;
        if (use_rows)
          got = fold_core(row0, ptrs.data() + a * L, b - a, wf.data() + a, scale, last, ntm, dev, stream,
                          reinterpret_cast<PlanFn>(plan_addr), reinterpret_cast<WsumFn>(wsum_addr), outs, acc,
                          nullptr, reinterpret_cast<L2WsFn>(g_solo.l2ws_fn), nullptr, &rc, st, &rows);
        if (got == 2) {  // (no lazy norms here, or a misaligned leaf: the plain fold, the nodes stay pending)
          for (size_t q = f0; q < fused.size(); ++q) Py_DECREF(fused[q]);
          fused.resize(f0);
          got = fold_core(row0, ptrs.data() + a * L, b - a, wf.data() + a, scale, last, ntm, dev, stream,
                          reinterpret_cast<PlanFn>(plan_addr), reinterpret_cast<WsumFn>(wsum_addr), outs, acc,
                          with_l2 ? reinterpret_cast<WsumL2Fn>(l2_addr) : nullptr,
                          with_l2 ? reinterpret_cast<L2WsFn>(l2ws_addr) : nullptr,
                          with_l2 ? l2sq.data_ptr<float>() + a : nullptr, &rc, st);
        }
        if (got != 0) {
          if (PyErr_Occurred()) return nullptr;
          Py_RETURN_NONE;
        }
        if (rc != 0) return Py_BuildValue("(iOdO)", rc, Py_None, job_bytes, Py_None);
        if (a == 0)
          g_timers[kTFirstLaunch] +=
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_entry).count();
        a = b;
      }
      done = k1;
    }
    if (!fused.empty()) {  // every launch is issued: the lazy norms these clients' views read are written
      Stamp sw;
      for (SoloObject* n : fused) solo_release(n, kSoloDone);
      g_solo.fused += static_cast<long long>(fused.size());
      const double t_rel = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - sw.t).count();
      solo_compact();
      const double t_cmp = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - sw.t).count();
      if (g_solo.want > 0 && solo_refill(dev, stream) != 0) return nullptr;  // (while the GPU folds)
      const double t_ref = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - sw.t).count();
      g_solo.t_release += t_rel, g_solo.t_compact += t_cmp - t_rel, g_solo.t_refill += t_ref - t_cmp;
    }
    std::vector<PyObject*> wrapped(L);
    for (int64_t l = 0; l < L; ++l) wrapped[l] = THPVariable_Wrap(std::move(outs[l]));
    size_t i = 0, ki = 0;
    PyObject* tree = rebuild(trees[0], wrapped.data(), i, sb.keys.data(), ki);
    for (PyObject* o : wrapped) Py_XDECREF(o);  // (rebuild took the ones it used)
    if (!tree) return nullptr;
    st.lap(kTWrap);
    PyObject* l2 = with_l2 ? THPVariable_Wrap(std::move(l2sq)) : (Py_INCREF(Py_None), Py_None);
    if (!l2) {
      Py_DECREF(tree);
      return nullptr;
    }
    return Py_BuildValue("(iNdN)", rc, tree, job_bytes, l2);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyObject* mean_pairs(PyObject*, PyObject* args) {
  PyObject* pairs;
  int may_pipeline;
  double frac, chunk_walk_us, walk_ns, nt_min;
  long long chunk, min_bytes, narrow_max;
  unsigned long long plan_addr, wsum_addr, l2_addr = 0, l2ws_addr = 0;
  if (!PyArg_ParseTuple(args, "OpdLddLLdKK|KK", &pairs, &may_pipeline, &frac, &chunk, &chunk_walk_us, &walk_ns,
                        &min_bytes, &narrow_max, &nt_min, &plan_addr, &wsum_addr, &l2_addr, &l2ws_addr))
    return nullptr;
  return mean_pairs_impl(pairs, false, may_pipeline, frac, chunk, chunk_walk_us, walk_ns, min_bytes, narrow_max, nt_min,
                         plan_addr, wsum_addr, l2_addr, l2ws_addr);
}

// ------------------------------------------------------------------ tree_mean as a builtin
// tree_util.tree_mean (tree_util.py:76-96) for a resident list / tuple of pairs, and
// mean_aggregator().apply's list of triples (aggregator.py:61-75), without a Python frame:
// the configuration of tree_util._native_mean (mean_config), the same mean_pairs_impl, and
// the host-side estimate of when the folds this process issued can have finished (the idle
// probe's gate, tree_util._BUSY_UNTIL). Anything but that case calls the Python function.
struct MeanConfig {
  bool on = false;  // mean_config() ran (tree_util sets it on its first Python-path call)
  double frac = 0.25, chunk_walk_us = 60.0, walk_ns = 35.0, nt_min = 256.0 * (1 << 20), peak = 8.0e12;
  long long chunk = 512, min_bytes = 64LL << 20, narrow_max = 256 << 10;
  unsigned long long plan = 0, wsum = 0;
  double busy_until = 0.0;  // steady-clock seconds
  PyObject* py_tree_mean = nullptr;
  PyObject* py_mean_triples = nullptr;
};
MeanConfig g_mean;

// mean_config(on, frac, chunk, chunk_walk_us, walk_ns, min_bytes, narrow_max, nt_min, peak, plan, wsum,
//             py_tree_mean, py_mean_triples, busy_until)
// busy_until: time.perf_counter() seconds (CLOCK_MONOTONIC, steady_clock's clock here)
PyObject* mean_config(PyObject*, PyObject* args) {
  int on;
  PyObject *ftm, *fmt;
  if (!PyArg_ParseTuple(args, "pdLddLLddKKOOd", &on, &g_mean.frac, &g_mean.chunk, &g_mean.chunk_walk_us,
                        &g_mean.walk_ns, &g_mean.min_bytes, &g_mean.narrow_max, &g_mean.nt_min, &g_mean.peak,
                        &g_mean.plan, &g_mean.wsum, &ftm, &fmt, &g_mean.busy_until))
    return nullptr;
  Py_INCREF(ftm), Py_INCREF(fmt);
  Py_XSETREF(g_mean.py_tree_mean, ftm);
  Py_XSETREF(g_mean.py_mean_triples, fmt);
  g_mean.on = on != 0 && g_mean.plan && g_mean.wsum;
  Py_RETURN_NONE;
}

// busy_until([t]) -> t: the time (time.perf_counter() seconds) before which the folds this
// process issued cannot have finished, at peak bandwidth — ONE estimate for the builtin
// tree_mean and tree_util's Python paths (tree_util._BUSY_UNTIL reads and writes it here).
PyObject* busy_until(PyObject*, PyObject* args) {
  double t = -1.0;
  if (!PyArg_ParseTuple(args, "|d", &t)) return nullptr;
  if (t >= 0.0) g_mean.busy_until = t;
  return PyFloat_FromDouble(g_mean.busy_until);
}

PyObject* mean_fast(PyObject* arg, bool triples) {
  const double now = now_s();
  PyObject* got = mean_pairs_impl(arg, triples, g_mean.frac > 0.0 && now >= g_mean.busy_until, g_mean.frac,
                                  g_mean.chunk, g_mean.chunk_walk_us, g_mean.walk_ns, g_mean.min_bytes,
                                  g_mean.narrow_max, g_mean.nt_min, g_mean.plan, g_mean.wsum, 0, 0);
  if (!got || got == Py_None) return got;
  // (rc, tree, job_bytes, None)
  const int rc = static_cast<int>(PyLong_AsLong(PyTuple_GET_ITEM(got, 0)));
  const double job_bytes = PyFloat_AsDouble(PyTuple_GET_ITEM(got, 2));
  g_mean.busy_until = std::max(now, g_mean.busy_until) + job_bytes / g_mean.peak;
  if (rc != 0) {  // the Python path raises the library's error (FjaggError) for it
    Py_DECREF(got);
    Py_RETURN_NONE;
  }
  PyObject* tree = PyTuple_GET_ITEM(got, 1);
  Py_INCREF(tree);
  Py_DECREF(got);
  return tree;
}

PyObject* fast_tree_mean(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  if (!g_mean.py_tree_mean) {
    PyErr_SetString(PyExc_RuntimeError, "fedjax_amd.tree_util is not installed (mean_config)");
    return nullptr;
  }
  if (g_mean.on && nargs == 1 && !kwnames && Py_SIZE(args[0]) > 0 &&
      (PyList_CheckExact(args[0]) || PyTuple_CheckExact(args[0]))) {
    PyObject* got = mean_fast(args[0], false);
    if (got != Py_None) return got;  // (a tree, or nullptr with the error set)
    Py_DECREF(got);
  }
  return PyObject_Vectorcall(g_mean.py_tree_mean, args, nargs, kwnames);
}

// mean_triples(clients) -> tree: tree_mean over (client_id, params, weight) triples
PyObject* mean_triples(PyObject*, PyObject* clients) {
  if (!g_mean.py_mean_triples) {
    PyErr_SetString(PyExc_RuntimeError, "fedjax_amd.tree_util is not installed (mean_config)");
    return nullptr;
  }
  if (g_mean.on && Py_SIZE(clients) > 0 && (PyList_CheckExact(clients) || PyTuple_CheckExact(clients))) {
    PyObject* got = mean_fast(clients, true);
    if (got != Py_None) return got;
    Py_DECREF(got);
  }
  return PyObject_CallOneArg(g_mean.py_mean_triples, clients);
}

// server_pairs(pairs, params, m, v, mean_out, desc_addr, nt_min_bytes, plan_fn, update_fn)
//   -> rc | None
// server.fused_tree_mean_update for the common case in one native call: the pairs as in
// mean_pairs (float32 CUDA deltas, Python-number weights, plain containers), and params /
// m / v / mean_out (None where absent) trees of client 0's structure with contiguous float32
// leaves of the deltas' shapes on the same device. Builds the plan image of
// fjagg_server_update_ptrs (in_ptrs | params | leaf_n | blocks | f32 weights | m | v | mean;
// per-leaf element units where a pointer is off 16 bytes), uploads it through pinned memory
// and launches on the current stream. None: not this case (nothing launched).
typedef int (*UpdFn)(int, const int64_t*, int, int64_t, int64_t, const float*, float, const void*, const int64_t*,
                     int, void*);

PyObject* server_pairs(PyObject*, PyObject* args) {
  PyObject *pairs, *params, *mt, *vt, *mo;
  double nt_min;
  unsigned long long desc_addr, plan_addr, upd_addr;
  if (!PyArg_ParseTuple(args, "OOOOOKdKK", &pairs, &params, &mt, &vt, &mo, &desc_addr, &nt_min, &plan_addr,
                        &upd_addr))
    return nullptr;
  if (!PyList_CheckExact(pairs) && !PyTuple_CheckExact(pairs)) Py_RETURN_NONE;
  const Py_ssize_t K = Py_SIZE(pairs);
  if (K < 1) Py_RETURN_NONE;
  {  // the state trees the rule reads: a missing one is never launched with a null
     // table entry; the Python path raises ValueError for it
    const auto* opt = reinterpret_cast<const fjagg_server_opt*>(desc_addr);
    if (!opt) Py_RETURN_NONE;
    const bool needs_m = opt->kind == FJAGG_OPT_MOMENTUM || opt->kind == FJAGG_OPT_ADAM || opt->kind == FJAGG_OPT_YOGI ||
                         (opt->kind == FJAGG_OPT_RMSPROP && (opt->flags & (FJAGG_OPT_F_MOMENTUM | FJAGG_OPT_F_CENTERED)));
    const bool needs_v = opt->kind >= FJAGG_OPT_ADAM;
    if ((needs_m && mt == Py_None) || (needs_v && vt == Py_None)) Py_RETURN_NONE;
  }
  PyObject* const* items = PyList_CheckExact(pairs) ? &PyList_GET_ITEM(pairs, 0) : &PyTuple_GET_ITEM(pairs, 0);
  try {
    struct Held {
      std::vector<PyObject*> v;
      ~Held() {
        for (PyObject* o : v) Py_XDECREF(o);
      }
    } held;
    held.v.assign(K, nullptr);
    std::vector<PyObject*>& trees = held.v;
    std::vector<float> wf(K);
    double W = 0.0;
    for (Py_ssize_t k = 0; k < K; ++k) {
      PyObject* pr = items[k];
      PyObject *t, *w;
      if (PyTuple_CheckExact(pr) && PyTuple_GET_SIZE(pr) == 2) {
        t = PyTuple_GET_ITEM(pr, 0);
        w = PyTuple_GET_ITEM(pr, 1);
      } else if (PyList_CheckExact(pr) && PyList_GET_SIZE(pr) == 2) {
        t = PyList_GET_ITEM(pr, 0);
        w = PyList_GET_ITEM(pr, 1);
      } else {
        Py_RETURN_NONE;
      }
      double d;
      if (PyLong_CheckExact(w)) {
        int overflow = 0;
        long long iv = PyLong_AsLongLongAndOverflow(w, &overflow);
        if (PyErr_Occurred()) PyErr_Clear();
        if (overflow || iv >= (1LL << 53) || iv <= -(1LL << 53)) Py_RETURN_NONE;
        d = static_cast<double>(iv);
      } else if (PyFloat_CheckExact(w)) {
        d = PyFloat_AS_DOUBLE(w);
      } else {
        Py_RETURN_NONE;
      }
      Py_INCREF(t);
      trees[k] = t;
      wf[k] = static_cast<float>(d);
      W += d;  // tree_util.py:95
    }
    SpecBuild sb;
    PyObject* spec = spec_of(trees[0], sb, 0);
    if (!spec) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_NONE;
    }
    struct Ref {
      PyObject* o;
      ~Ref() { Py_DECREF(o); }
    } spec_ref{spec};
    const int64_t L = static_cast<int64_t>(sb.leaves.size());
    if (L < 1) Py_RETURN_NONE;
    std::vector<at::ScalarType> dtypes;
    std::vector<c10::IntArrayRef> sizes;
    std::vector<at::Tensor> row0;
    int dev = -1;
    for (PyObject* x : sb.leaves) {
      const at::Tensor& t = THPVariable_Unpack(x);
      if (t.layout() != c10::kStrided || !t.is_cuda() || t.scalar_type() != at::kFloat || !t.is_contiguous())
        Py_RETURN_NONE;
      if (dev < 0) dev = t.get_device();
      if (t.get_device() != dev) Py_RETURN_NONE;
      row0.push_back(t);
    }
    std::vector<int64_t> leaf_n(L);
    int64_t total = 0;
    for (int64_t l = 0; l < L; ++l) {
      dtypes.push_back(at::kFloat);
      sizes.push_back(row0[l].sizes());
      leaf_n[l] = row0[l].numel();
      total += leaf_n[l];
    }
    if (total == 0) Py_RETURN_NONE;
    // params / state / mean_out leaves: client 0's structure, float32, contiguous, its shapes
    Walk w{&dtypes, &sizes, static_cast<c10::DeviceIndex>(dev), nullptr, 0};
    std::vector<int64_t> pp(L, 0), st(3 * L, 0);
    PyObject* side[4] = {params, mt, vt, mo};
    for (int i = 0; i < 4; ++i) {
      if (side[i] == Py_None) {
        if (i == 0) Py_RETURN_NONE;
        continue;
      }
      w.out = i == 0 ? pp.data() : st.data() + (i - 1) * L;
      w.leaf = 0;
      const int r = walk(spec, side[i], w);
      if (r < 0) return nullptr;
      if (r > 0 || w.leaf != static_cast<size_t>(L)) Py_RETURN_NONE;
    }
    // every client's leaf pointers
    std::vector<int64_t> ptrs(static_cast<size_t>(K * L));
    for (int64_t l = 0; l < L; ++l) ptrs[l] = reinterpret_cast<int64_t>(row0[l].data_ptr());
    for (Py_ssize_t k = 1; k < K; ++k) {
      w.out = ptrs.data() + k * L;
      w.leaf = 0;
      const int r = walk(spec, trees[k], w);
      if (r < 0) return nullptr;
      if (r > 0 || w.leaf != static_cast<size_t>(L)) Py_RETURN_NONE;
    }
    // per-leaf element units where any pointer of the leaf is off 16 bytes
    std::vector<uint8_t> elem(L, 0);
    bool any_elem = false;
    for (int64_t l = 0; l < L; ++l) {
      int64_t bits = pp[l] | st[l] | st[L + l] | st[2 * L + l];
      for (Py_ssize_t k = 0; k < K; ++k) bits |= ptrs[k * L + l];
      elem[l] = (bits & 15) != 0;
      any_elem = any_elem || elem[l];
    }
    auto plan = reinterpret_cast<PlanFn>(plan_addr);
    const uint8_t* mask = any_elem ? elem.data() : nullptr;
    const int64_t nblk = plan(kF32, 0, leaf_n.data(), mask, static_cast<int>(L), nullptr, 0);
    if (nblk < 1) Py_RETURN_NONE;
    const int64_t nw = (K + 1) / 2, n = K * L + 2 * L + 2 * nblk + nw + 3 * L;
    if (upload_refused_in_capture(reinterpret_cast<unsigned long long>(
                                      c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream()),
                                  "the server step's pytree fold"))
      return nullptr;
    at::Tensor img = at::empty({n}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
    int64_t* p = img.data_ptr<int64_t>();
    std::memcpy(p, ptrs.data(), sizeof(int64_t) * K * L);
    std::memcpy(p + K * L, pp.data(), sizeof(int64_t) * L);
    std::memcpy(p + K * L + L, leaf_n.data(), sizeof(int64_t) * L);
    if (plan(kF32, 0, leaf_n.data(), mask, static_cast<int>(L), p + K * L + 2 * L, nblk) != nblk) Py_RETURN_NONE;
    int64_t* wp = p + K * L + 2 * L + 2 * nblk;
    wp[nw - 1] = 0;
    std::memcpy(wp, wf.data(), 4 * K);
    std::memcpy(wp + nw, st.data(), sizeof(int64_t) * 3 * L);
    at::Tensor dimg = img.to(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(dev)), /*non_blocking=*/true);
    const int64_t* dp = dimg.data_ptr<int64_t>();
    const double job_bytes = 4.0 * static_cast<double>(total) * static_cast<double>(K);
    const int flags = job_bytes >= nt_min ? kNontemporal : 0;
    const float scale = static_cast<float>(W > 0.0 ? 1.0 / W : 0.0);  // tree_util.py:37,60
    const unsigned long long stream =
        reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream());
    const int rc = reinterpret_cast<UpdFn>(upd_addr)(kF32, dp, static_cast<int>(L), K, nblk,
                                                      reinterpret_cast<const float*>(dp + K * L + 2 * L + 2 * nblk),
                                                      scale, reinterpret_cast<const void*>(desc_addr),
                                                      dp + K * L + 2 * L + 2 * nblk + nw, flags,
                                                      reinterpret_cast<void*>(stream));
    return PyLong_FromLong(rc);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// ------------------------------------------------------------------ lazy results, natively
// tree_util.WeightedTree, PendingSum and _Chain are Python subclasses of the three base
// types below: their fields are these C members, their methods stay Python. The two hot
// calls of the library running-sum loop (fedjax/algorithms/fed_avg.py:137-138, and the six
// other algorithms of SURVEY §8f row 1) — tree_weight(delta, n) and tree_add(s, that) — are
// METH_FASTCALL functions here that build those objects directly; tree_util installs them as
// tree_util.tree_weight / tree_add (fast_install). Anything but the fast case calls the
// Python function they replace, which then decides exactly as before.

struct WTObject {
  PyObject_HEAD
  PyObject* tree;
  PyObject* weight;
  PyObject* cap;
  PyObject* value;
};

struct ChainObject {
  PyObject_HEAD
  PyObject* tip;
  PyObject* buf;
  PyObject* budget;
  PyObject* views;  // list: pre-made (norm view, ticket) pairs of buf's row 1 by link index, or NULL
};

struct PSObject {
  PyObject_HEAD
  PyObject* root;
  PyObject* parent;
  PyObject* cap;
  PyObject* weight;
  PyObject* value;
  PyObject* chain;
  PyObject* ticket;
  PyObject* ref;
  PyObject* bcap;
  long long n, bytes, idx, tok;
  PyObject* weakreflist;
};

#define FJ_OBJ_MEMBER(T, f) {const_cast<char*>("_" #f), T_OBJECT, offsetof(T, f), 0, nullptr}
#define FJ_LL_MEMBER(T, f) {const_cast<char*>("_" #f), T_LONGLONG, offsetof(T, f), 0, nullptr}

PyMemberDef kWTMembers[] = {FJ_OBJ_MEMBER(WTObject, tree), FJ_OBJ_MEMBER(WTObject, weight),
                            FJ_OBJ_MEMBER(WTObject, cap), FJ_OBJ_MEMBER(WTObject, value), {nullptr}};
PyMemberDef kChainMembers[] = {{const_cast<char*>("tip"), T_OBJECT, offsetof(ChainObject, tip), 0, nullptr},
                               {const_cast<char*>("buf"), T_OBJECT, offsetof(ChainObject, buf), 0, nullptr},
                               {const_cast<char*>("budget"), T_OBJECT, offsetof(ChainObject, budget), 0, nullptr},
                               {const_cast<char*>("views"), T_OBJECT, offsetof(ChainObject, views), 0, nullptr},
                               {nullptr}};
PyMemberDef kPSMembers[] = {FJ_OBJ_MEMBER(PSObject, root),   FJ_OBJ_MEMBER(PSObject, parent),
                            FJ_OBJ_MEMBER(PSObject, cap),    FJ_OBJ_MEMBER(PSObject, weight),
                            FJ_OBJ_MEMBER(PSObject, value),  FJ_OBJ_MEMBER(PSObject, chain),
                            FJ_OBJ_MEMBER(PSObject, ticket), FJ_OBJ_MEMBER(PSObject, ref),
                            FJ_OBJ_MEMBER(PSObject, bcap),   FJ_LL_MEMBER(PSObject, n),
                            FJ_LL_MEMBER(PSObject, bytes),   FJ_LL_MEMBER(PSObject, idx),
                            FJ_LL_MEMBER(PSObject, tok),
                            {const_cast<char*>("__weaklistoffset__"), T_PYSSIZET, offsetof(PSObject, weakreflist),
                             READONLY, nullptr},
                            {nullptr}};

int wt_traverse(PyObject* o, visitproc visit, void* arg) {
  auto* x = reinterpret_cast<WTObject*>(o);
  Py_VISIT(Py_TYPE(o));
  Py_VISIT(x->tree);
  Py_VISIT(x->weight);
  Py_VISIT(x->cap);
  Py_VISIT(x->value);
  return 0;
}
int wt_clear(PyObject* o) {
  auto* x = reinterpret_cast<WTObject*>(o);
  Py_CLEAR(x->tree);
  Py_CLEAR(x->weight);
  Py_CLEAR(x->cap);
  Py_CLEAR(x->value);
  return 0;
}
void wt_dealloc(PyObject* o) {
  PyTypeObject* tp = Py_TYPE(o);
  PyObject_GC_UnTrack(o);
  wt_clear(o);
  tp->tp_free(o);
  Py_DECREF(tp);
}

int chain_traverse(PyObject* o, visitproc visit, void* arg) {
  auto* x = reinterpret_cast<ChainObject*>(o);
  Py_VISIT(Py_TYPE(o));
  Py_VISIT(x->tip);
  Py_VISIT(x->buf);
  Py_VISIT(x->budget);
  Py_VISIT(x->views);
  return 0;
}
int chain_clear(PyObject* o) {
  auto* x = reinterpret_cast<ChainObject*>(o);
  Py_CLEAR(x->tip);
  Py_CLEAR(x->buf);
  Py_CLEAR(x->budget);
  Py_CLEAR(x->views);
  return 0;
}
void chain_dealloc(PyObject* o) {
  PyTypeObject* tp = Py_TYPE(o);
  PyObject_GC_UnTrack(o);
  chain_clear(o);
  tp->tp_free(o);
  Py_DECREF(tp);
}

int ps_traverse(PyObject* o, visitproc visit, void* arg) {
  auto* x = reinterpret_cast<PSObject*>(o);
  Py_VISIT(Py_TYPE(o));
  Py_VISIT(x->root);
  Py_VISIT(x->parent);
  Py_VISIT(x->cap);
  Py_VISIT(x->weight);
  Py_VISIT(x->value);
  Py_VISIT(x->chain);
  Py_VISIT(x->ticket);
  Py_VISIT(x->ref);
  Py_VISIT(x->bcap);
  return 0;
}
int ps_clear(PyObject* o) {
  auto* x = reinterpret_cast<PSObject*>(o);
  Py_CLEAR(x->root);
  Py_CLEAR(x->parent);
  Py_CLEAR(x->cap);
  Py_CLEAR(x->weight);
  Py_CLEAR(x->value);
  Py_CLEAR(x->chain);
  Py_CLEAR(x->ticket);
  Py_CLEAR(x->ref);
  Py_CLEAR(x->bcap);
  return 0;
}
void ps_dealloc(PyObject* o) {
  PyTypeObject* tp = Py_TYPE(o);
  PyObject_GC_UnTrack(o);
  if (reinterpret_cast<PSObject*>(o)->weakreflist) PyObject_ClearWeakRefs(o);
  ps_clear(o);
  tp->tp_free(o);
  Py_DECREF(tp);
}

PyType_Slot kWTSlots[] = {{Py_tp_dealloc, reinterpret_cast<void*>(wt_dealloc)},
                          {Py_tp_traverse, reinterpret_cast<void*>(wt_traverse)},
                          {Py_tp_clear, reinterpret_cast<void*>(wt_clear)},
                          {Py_tp_members, kWTMembers},
                          {Py_tp_new, reinterpret_cast<void*>(PyType_GenericNew)},
                          {Py_tp_doc, const_cast<char*>("fields of tree_util.WeightedTree")},
                          {0, nullptr}};
PyType_Slot kChainSlots[] = {{Py_tp_dealloc, reinterpret_cast<void*>(chain_dealloc)},
                             {Py_tp_traverse, reinterpret_cast<void*>(chain_traverse)},
                             {Py_tp_clear, reinterpret_cast<void*>(chain_clear)},
                             {Py_tp_members, kChainMembers},
                             {Py_tp_new, reinterpret_cast<void*>(PyType_GenericNew)},
                             {Py_tp_doc, const_cast<char*>("fields of tree_util._Chain")},
                             {0, nullptr}};
PyType_Slot kPSSlots[] = {{Py_tp_dealloc, reinterpret_cast<void*>(ps_dealloc)},
                          {Py_tp_traverse, reinterpret_cast<void*>(ps_traverse)},
                          {Py_tp_clear, reinterpret_cast<void*>(ps_clear)},
                          {Py_tp_members, kPSMembers},
                          {Py_tp_new, reinterpret_cast<void*>(PyType_GenericNew)},
                          {Py_tp_doc, const_cast<char*>("fields of tree_util.PendingSum")},
                          {0, nullptr}};
constexpr unsigned kBaseFlags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE | Py_TPFLAGS_HAVE_GC;
PyType_Spec kWTSpec = {"_fjhost.WeightedBase", sizeof(WTObject), 0, kBaseFlags, kWTSlots};
PyType_Spec kChainSpec = {"_fjhost.ChainBase", sizeof(ChainObject), 0, kBaseFlags, kChainSlots};
PyType_Spec kPSSpec = {"_fjhost.PendingBase", sizeof(PSObject), 0, kBaseFlags, kPSSlots};

struct FastState {
  PyTypeObject* ticket = nullptr;    // tree_util._Ticket
  PyTypeObject* norm_view = nullptr;  // tree_util._NormView
  PyObject* py_l2[2] = {nullptr, nullptr};  // tree_util._tree_l2_squared_py / _tree_l2_norm_py
  PyObject* py_fold_ticket = nullptr;        // tree_util._fold_ticket (flush_views)
  PyTypeObject* wt = nullptr;     // tree_util.WeightedTree
  PyTypeObject* ps = nullptr;     // tree_util.PendingSum
  PyTypeObject* chain = nullptr;  // tree_util._Chain
  PyObject* py_tree_weight = nullptr;  // the Python functions the fast calls fall back to
  PyObject* py_tree_add = nullptr;
  // tree_util.set_deferred_sums
  bool defer = true;
  long long max_clients = 4095, flush_bytes = 256LL << 20, flush_clients = 64;  // (set by fast_config)
  PyObject* last = nullptr;  // weak reference to the most recent PendingSum link
  // Lazy-norm pool: a norm buffer [2, max_clients + 1] and a list of pre-made (view of
  // buf[1, i], ticket) pairs for i < the norms the last round asked for. Creating a 0-d
  // tensor subclass object costs ~0.3 us of host time, on the critical path of the library
  // loop (one tree_l2_norm per client, fed_avg.py:142-144); the pool is built right after a
  // round's final fold is launched (fold_chain with the 1/W scale), while the GPU folds, and
  // the next chain that takes a norm takes the pool as its buffer (fast_l2).
  PyObject* pool_buf = nullptr;
  PyObject* pool_views = nullptr;  // the pairs still to hand out (items become None)
  PyObject* pool_all = nullptr;    // every pair of the pool, in order (never modified)
  // pools a chain took: (buf, all pairs). Once the caller has dropped every view of one and
  // nothing else holds its buffer, the next refill reuses it whole (no new objects).
  std::vector<std::pair<PyObject*, PyObject*>> retired;
  std::vector<unsigned long long> retired_stream;  // the stream each retired pool's norms were written on
  unsigned long long pool_stream = 0;              // the stream the current pool was built on
  PyObject* d_view_ticket = nullptr;  // _NormView._ticket and _Ticket.node slot descriptors
  PyObject* d_ticket_node = nullptr;
  long long pool_want = 0;  // norms (row 1) the current round's chains asked for: the next pool's size
  double refill_us = 0.0;   // host time of the last refill (pool_info)
  long long pool_reuses = 0, pool_builds = 0;
};
FastState g_fast;

// fast_install(WeightedTree, PendingSum, _Chain, py_tree_weight, py_tree_add)
PyObject* fast_install(PyObject*, PyObject* args) {
  PyObject *wt, *ps, *ch, *ftw, *fta;
  if (!PyArg_ParseTuple(args, "O!O!O!OO", &PyType_Type, &wt, &PyType_Type, &ps, &PyType_Type, &ch, &ftw, &fta))
    return nullptr;
  if (!PyCallable_Check(ftw) || !PyCallable_Check(fta)) {
    PyErr_SetString(PyExc_TypeError, "fast_install: fallbacks must be callable");
    return nullptr;
  }
  Py_INCREF(wt), Py_INCREF(ps), Py_INCREF(ch), Py_INCREF(ftw), Py_INCREF(fta);
  Py_XSETREF(g_fast.wt, reinterpret_cast<PyTypeObject*>(wt));
  Py_XSETREF(g_fast.ps, reinterpret_cast<PyTypeObject*>(ps));
  Py_XSETREF(g_fast.chain, reinterpret_cast<PyTypeObject*>(ch));
  Py_XSETREF(g_fast.py_tree_weight, ftw);
  Py_XSETREF(g_fast.py_tree_add, fta);
  Py_RETURN_NONE;
}

// fast_config(enabled, max_clients, flush_bytes, flush_clients): tree_util.set_deferred_sums
PyObject* fast_config(PyObject*, PyObject* args) {
  int en;
  long long mc, fb, fc;
  if (!PyArg_ParseTuple(args, "pLLL", &en, &mc, &fb, &fc)) return nullptr;
  g_fast.defer = en != 0;
  g_fast.max_clients = mc;
  g_fast.flush_bytes = fb;
  g_fast.flush_clients = fc;
  Py_RETURN_NONE;
}

// set_last(node) / last() -> node | None: the most recent PendingSum link (weakly held),
// whose delta a following tree_l2_norm may take from the chain's fold (tree_util._lazy_norm)
PyObject* set_last(PyObject*, PyObject* node) {
  PyObject* wr = PyWeakref_NewRef(node, nullptr);
  if (!wr) return nullptr;
  Py_XSETREF(g_fast.last, wr);
  Py_RETURN_NONE;
}
PyObject* last(PyObject*, PyObject*) {
  PyObject* o = g_fast.last ? PyWeakref_GetObject(g_fast.last) : Py_None;
  Py_INCREF(o);
  return o;
}

// Python int / float weight that tree_weight defers (|int| < 2**53: exact in float32's path)
inline int deferrable_weight(PyObject* w) {
  if (PyFloat_CheckExact(w)) return 1;
  if (!PyLong_CheckExact(w)) return 0;
  int of = 0;
  const long long v = PyLong_AsLongLongAndOverflow(w, &of);
  if (v == -1 && PyErr_Occurred()) return -1;
  return (!of && v > -(1LL << 53) && v < (1LL << 53)) ? 1 : 0;
}

// tree_weight(pytree, weight): tree_util.tree_weight (tree_util.py:29-32). A Python-number
// weight and a pytree of float32 device tensors give a WeightedTree holding the capture;
// anything else is the Python function's.
PyObject* fast_tree_weight(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  if (!g_fast.wt || !g_fast.py_tree_weight) {
    PyErr_SetString(PyExc_RuntimeError, "fedjax_amd.tree_util is not installed (fast_install)");
    return nullptr;
  }
  if (nargs == 2 && kwnames == nullptr) {
    const int ok = deferrable_weight(args[1]);
    if (ok < 0) return nullptr;
    if (ok) {
      PyObject* cap = capture_impl(args[0], -1);
      if (!cap) return nullptr;
      if (cap != Py_None) {
        auto* o = reinterpret_cast<WTObject*>(g_fast.wt->tp_alloc(g_fast.wt, 0));
        if (!o) {
          Py_DECREF(cap);
          return nullptr;
        }
        Py_INCREF(args[0]);
        o->tree = args[0];
        Py_INCREF(args[1]);
        o->weight = args[1];
        o->cap = cap;
        return reinterpret_cast<PyObject*>(o);
      }
      Py_DECREF(cap);
    }
  }
  return PyObject_Vectorcall(g_fast.py_tree_weight, args, nargs, kwnames);
}

// Should the pending run ending at p be folded before the next link is appended (an early
// flush)? It holds >= flush_bytes in >= flush_clients links. tree_util._flush_due states the
// same rule.
inline bool flush_due(const PSObject* p) { return p->bytes >= g_fast.flush_bytes && p->n >= g_fast.flush_clients; }

// tree_add(left, right): tree_util.tree_add (tree_util.py:47-50). The fast case is the
// running sum's append, s = tree_add(s, tree_weight(x, n)) with s a live PendingSum at the
// tip of its chain, the capture's structure token equal to the sum's, and no chain limit
// reached (tree_util._defer's checks): the new link is built here, exactly as PendingSum's
// __init__ builds it. Anything else is the Python function's.
PyObject* fast_tree_add(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  if (!g_fast.ps || !g_fast.py_tree_add) {
    PyErr_SetString(PyExc_RuntimeError, "fedjax_amd.tree_util is not installed (fast_install)");
    return nullptr;
  }
  if (nargs == 2 && kwnames == nullptr && g_fast.defer && Py_TYPE(args[1]) == g_fast.wt &&
      Py_TYPE(args[0]) == g_fast.ps) {
    auto* r = reinterpret_cast<WTObject*>(args[1]);
    auto* p = reinterpret_cast<PSObject*>(args[0]);
    auto* ch = reinterpret_cast<ChainObject*>(p->chain);
    if (r->tree && r->tree != Py_None && r->cap && PyTuple_CheckExact(r->cap) && PyTuple_GET_SIZE(r->cap) >= 4 &&
        (!p->value || p->value == Py_None) && p->tok >= 0 && ch && Py_TYPE(ch) == g_fast.chain &&
        ch->tip == args[0] && ch->budget && PyLong_CheckExact(ch->budget)) {
      const long long tok = PyLong_AsLongLong(PyTuple_GET_ITEM(r->cap, 3));
      const long long nb = PyLong_AsLongLong(PyTuple_GET_ITEM(r->cap, 2));
      const long long budget = PyLong_AsLongLong(ch->budget);
      if (PyErr_Occurred()) return nullptr;
      if (tok == p->tok && p->n + 1 <= g_fast.max_clients && p->bytes + nb <= budget && !flush_due(p)) {
        auto* q = reinterpret_cast<PSObject*>(g_fast.ps->tp_alloc(g_fast.ps, 0));
        if (!q) return nullptr;
        Py_INCREF(p);
        q->parent = args[0];
        Py_INCREF(r->cap);
        q->cap = r->cap;
        Py_INCREF(r->weight);
        q->weight = r->weight;
        Py_INCREF(ch);
        q->chain = reinterpret_cast<PyObject*>(ch);
        Py_XINCREF(p->ref);
        q->ref = p->ref;
        q->n = p->n + 1;
        q->bytes = p->bytes + nb;
        q->idx = p->idx + 1;
        q->tok = p->tok;
        Py_INCREF(q);
        Py_XSETREF(ch->tip, reinterpret_cast<PyObject*>(q));
        PyObject* wr = PyWeakref_NewRef(reinterpret_cast<PyObject*>(q), nullptr);
        if (!wr) {
          Py_DECREF(q);
          return nullptr;
        }
        Py_XSETREF(g_fast.last, wr);
        return reinterpret_cast<PyObject*>(q);
      }
    }
  }
  return PyObject_Vectorcall(g_fast.py_tree_add, args, nargs, kwnames);
}


// fast_install_norms(_Ticket, _NormView, py_tree_l2_squared, py_tree_l2_norm[, py_fold_ticket])
PyObject* fast_install_norms(PyObject*, PyObject* args) {
  PyObject *tk, *nv, *f0, *f1, *ft = Py_None;
  if (!PyArg_ParseTuple(args, "O!O!OO|O", &PyType_Type, &tk, &PyType_Type, &nv, &f0, &f1, &ft)) return nullptr;
  Py_INCREF(tk), Py_INCREF(nv), Py_INCREF(f0), Py_INCREF(f1), Py_INCREF(ft);
  Py_XSETREF(g_fast.ticket, reinterpret_cast<PyTypeObject*>(tk));
  Py_XSETREF(g_fast.norm_view, reinterpret_cast<PyTypeObject*>(nv));
  Py_XSETREF(g_fast.py_l2[0], f0);
  Py_XSETREF(g_fast.py_l2[1], f1);
  Py_XSETREF(g_fast.py_fold_ticket, ft);
  // the slots' descriptors, so setting / reading them skips the attribute lookup
  PyObject* dv = PyObject_GetAttrString(nv, "_ticket");
  PyObject* dn = dv ? PyObject_GetAttrString(tk, "node") : nullptr;
  if (!dv || !dn || !Py_TYPE(dv)->tp_descr_set || !Py_TYPE(dn)->tp_descr_set || !Py_TYPE(dv)->tp_descr_get) {
    Py_XDECREF(dv), Py_XDECREF(dn);
    PyErr_Clear();
    PyErr_SetString(PyExc_TypeError, "fast_install_norms: _NormView._ticket and _Ticket.node must be __slots__");
    return nullptr;
  }
  Py_XSETREF(g_fast.d_view_ticket, dv);
  Py_XSETREF(g_fast.d_ticket_node, dn);
  Py_RETURN_NONE;
}

// obj.<slot> = v through the slot's descriptor (0, or -1 with a Python error)
inline int slot_set(PyObject* descr, PyObject* obj, PyObject* v) { return Py_TYPE(descr)->tp_descr_set(descr, obj, v); }

PyObject* solo_stale_error() {
  PyErr_SetString(PyExc_RuntimeError,
                  "a client delta passed to tree_l2_norm / tree_l2_squared was modified (a leaf updated in place) "
                  "before its lazy norm was computed; the reference takes the norm of the value at that call. Add "
                  "copies, or call fedjax_amd.tree_util.set_lazy_norms(False)");
  return nullptr;
}

// solo_config(on, max_pending, budget_bytes, rows_fn, l2ws_fn, plan_fn, py_budget): tree_util's
// set_lazy_norms and the library's entry points (0: keep the current one)
PyObject* solo_config(PyObject*, PyObject* args) {
  int on;
  long long mp, bb;
  unsigned long long rf, wf, pf;
  PyObject* pb;
  if (!PyArg_ParseTuple(args, "pLLKKKO", &on, &mp, &bb, &rf, &wf, &pf, &pb)) return nullptr;
  g_solo.on = on != 0;
  g_solo.max_pending = std::max<long long>(1, std::min<long long>(mp, 1LL << 20));
  g_solo.budget = std::max<long long>(0, bb);
  if (rf) g_solo.rows_fn = rf;
  if (wf) g_solo.l2ws_fn = wf;
  if (pf) g_solo.plan_fn = pf;
  if (pb != Py_None) {
    Py_INCREF(pb);
    Py_XSETREF(g_solo.py_budget, pb);
  }
  Py_RETURN_NONE;
}

// solo_resolve(nodes | None) -> None: compute these pending standalone norms now (None: every
// pending one); raises for a stale one among them
PyObject* solo_resolve_py(PyObject*, PyObject* arg) {
  if (arg == Py_None) {
    if (solo_resolve_all() != 0) return nullptr;
    Py_RETURN_NONE;
  }
  PyObject* seq = PySequence_Fast(arg, "solo_resolve: a sequence of SoloNorm nodes or None");
  if (!seq) return nullptr;
  std::vector<SoloObject*> v;
  for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); ++i) {
    PyObject* o = PySequence_Fast_GET_ITEM(seq, i);
    if (Py_TYPE(o) == g_solo.type) v.push_back(reinterpret_cast<SoloObject*>(o));
  }
  const int rc = solo_resolve(v);
  bool stale = false;
  for (SoloObject* n : v) stale = stale || n->state == kSoloStale;
  Py_DECREF(seq);
  if (rc != 0) return nullptr;
  solo_compact();
  if (stale) return solo_stale_error();
  Py_RETURN_NONE;
}

// solo_info() -> dict: pending nodes and bytes, registry size, norms fused into a mean, computed
// on their own (and their launches), stale nodes
PyObject* solo_info(PyObject*, PyObject*) {
  solo_compact();
  return Py_BuildValue("{s:L,s:L,s:n,s:L,s:L,s:L,s:L,s:L,s:L,s:n,s:L,s:L,s:d,s:n}", "pending", g_solo.pending,
                       "pending_bytes", g_solo.pending_bytes, "registry", static_cast<Py_ssize_t>(g_solo.reg.size()),
                       "fused", g_solo.fused, "eager", g_solo.eager, "eager_launches", g_solo.launches, "stale",
                       g_solo.stale, "budget", g_solo.budget, "column", g_solo.buf ? g_solo.next : kSoloCols,
                       "pool_ready", static_cast<Py_ssize_t>(g_solo.pool.size() - g_solo.pool_head), "pool_builds",
                       g_solo.pool_builds, "pool_reuses", g_solo.pool_reuses, "refill_us", g_solo.refill_us,
                       "buffers", static_cast<Py_ssize_t>(g_solo.bufs.size()));
}
PyObject* solo_times(PyObject*, PyObject*) {
  PyObject* r = Py_BuildValue("{s:d,s:d,s:d}", "release_us", g_solo.t_release, "compact_us", g_solo.t_compact,
                              "refill_us", g_solo.t_refill);
  g_solo.t_release = g_solo.t_compact = g_solo.t_refill = 0;
  return r;
}

// solo_norm_py(tree, which) -> view | None: the standalone lazy norm for tree_util's Python path
PyObject* solo_norm(PyObject* tree, int which);
PyObject* solo_norm_py(PyObject*, PyObject* args) {
  PyObject* tree;
  int which;
  if (!PyArg_ParseTuple(args, "Oi", &tree, &which)) return nullptr;
  if (!g_solo.on || !g_solo.type || !g_solo.rows_fn || !g_fast.norm_view || !g_fast.d_view_ticket ||
      Py_TYPE(tree) == g_fast.wt || Py_TYPE(tree) == g_fast.ps)
    Py_RETURN_NONE;
  return solo_norm(tree, which != 0 ? 1 : 0);
}

// flush_views(obj): tree_util._flush_views natively — every lazy norm view (tree_util._NormView)
// in obj (nested lists / tuples / dict values) whose ticket still names an unfolded link gets
// its chain folded (py_fold_ticket(ticket)), so no torch function reads its buffer early.
// Views already filled cost a dict lookup each.
PyObject* flush_views(PyObject*, PyObject* arg) {
  if (!g_fast.norm_view || !g_fast.py_fold_ticket || g_fast.py_fold_ticket == Py_None) {
    PyErr_SetString(PyExc_RuntimeError, "fedjax_amd.tree_util is not installed (fast_install_norms)");
    return nullptr;
  }
  static PyObject* node_name = PyUnicode_InternFromString("node");
  std::vector<SoloObject*> solo_wait;  // pending standalone norms met on the way (new references)
  struct HeldSolo {
    std::vector<SoloObject*>& v;
    ~HeldSolo() {
      for (SoloObject* n : v) Py_DECREF(n);
    }
  } held_solo{solo_wait};
  std::vector<std::pair<PyObject*, int>> st;  // (not shared: a fold may run Python code that calls back)
  Py_INCREF(arg);  // (every stacked object is held: folding runs Python code)
  st.emplace_back(arg, 0);
  struct Held {
    std::vector<std::pair<PyObject*, int>>& v;
    ~Held() {
      for (auto& e : v) Py_DECREF(e.first);
      v.clear();
    }
  } held{st};
  while (!st.empty()) {
    PyObject* x = st.back().first;
    const int depth = st.back().second;
    st.pop_back();
    struct Drop {
      PyObject* o;
      ~Drop() { Py_DECREF(o); }
    } drop{x};
    PyTypeObject* t = Py_TYPE(x);
    if (t == g_fast.norm_view) {
      PyObject* tk = Py_TYPE(g_fast.d_view_ticket)->tp_descr_get(g_fast.d_view_ticket, x,
                                                                  reinterpret_cast<PyObject*>(t));
      if (!tk) {  // the slot was never set: no ticket
        if (!PyErr_ExceptionMatches(PyExc_AttributeError)) return nullptr;
        PyErr_Clear();
        continue;
      }
      struct DropTk {
        PyObject* o;
        ~DropTk() { Py_DECREF(o); }
      } drop_tk{tk};
      if (tk == Py_None) continue;
      if (Py_TYPE(tk) == g_solo.type) {  // a standalone lazy norm: computed below, with the others
        const int stt = reinterpret_cast<SoloObject*>(tk)->state;
        if (stt == kSoloStale) return solo_stale_error();
        if (stt == kSoloPending) {
          Py_INCREF(tk);
          solo_wait.push_back(reinterpret_cast<SoloObject*>(tk));
        }
        continue;
      }
      PyObject* node = PyObject_GetAttr(tk, node_name);
      if (!node) return nullptr;
      const bool live = node != Py_None;
      Py_DECREF(node);
      if (live) {
        PyObject* r = PyObject_CallOneArg(g_fast.py_fold_ticket, tk);
        if (!r) return nullptr;
        Py_DECREF(r);
      }
    } else if (depth < 64 && (t == &PyList_Type || t == &PyTuple_Type)) {
      for (Py_ssize_t i = Py_SIZE(x) - 1; i >= 0; --i) {
        PyObject* c = t == &PyList_Type ? PyList_GET_ITEM(x, i) : PyTuple_GET_ITEM(x, i);
        Py_INCREF(c);
        st.emplace_back(c, depth + 1);
      }
    } else if (depth < 64 && t == &PyDict_Type) {
      Py_ssize_t pos = 0;
      PyObject *k, *v;
      while (PyDict_Next(x, &pos, &k, &v)) {
        Py_INCREF(v);
        st.emplace_back(v, depth + 1);
      }
    }
  }
  if (!solo_wait.empty()) {  // one launch per run of them (solo_resolve)
    if (solo_resolve(solo_wait) != 0) return nullptr;
    solo_compact();
    for (SoloObject* n : solo_wait)
      if (n->state == kSoloStale) return solo_stale_error();
  }
  Py_RETURN_NONE;
}

void retire_pool(PyObject* buf, PyObject* all);

// A new _Ticket naming `node` (tree_util._Ticket, without its Python __init__ frame).
PyObject* new_ticket(PyObject* node) {
  PyObject* t = g_fast.ticket->tp_alloc(g_fast.ticket, 0);
  if (t && slot_set(g_fast.d_ticket_node, t, node) != 0) Py_CLEAR(t);
  return t;
}

// The device's pending budget (bytes): set_lazy_norms' value, else tree_util's automatic one
// (min(4 GiB, 1/8 of the free memory), asked once).
long long solo_budget(int dev) {
  if (g_solo.budget > 0) return g_solo.budget;
  static long long autob = 0;
  if (autob <= 0 && g_solo.py_budget) {
    PyObject* r = PyObject_CallFunction(g_solo.py_budget, "i", dev);
    if (r) {
      autob = PyLong_AsLongLong(r);
      Py_DECREF(r);
    }
    if (PyErr_Occurred()) PyErr_Clear();
  }
  return autob > 0 ? autob : (1LL << 30);
}

// The next free column of the current norm buffer (a new buffer, and its pool record, when it
// is full or on another device). false: a Python error is set.
bool solo_column(int dev, PyObject** buf, long long* idx) {
  if (!g_solo.buf || g_solo.next >= kSoloCols || THPVariable_Unpack(g_solo.buf).get_device() != dev) {
    at::Tensor b = at::empty({2, kSoloCols}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
    PyObject* bo = THPVariable_Wrap(std::move(b));
    if (!bo) return false;
    Py_XSETREF(g_solo.buf, bo);
    g_solo.next = 0;
    Py_INCREF(bo);
    g_solo.bufs.push_back(SoloState::BufRec{
        bo, reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream()),
        {}});
    if (g_solo.bufs.size() > 6) {  // (bounded: the oldest record lets its pairs go)
      auto& old = g_solo.bufs.front();
      for (auto& pr : old.pairs) Py_DECREF(pr.first), Py_DECREF(pr.second);
      Py_DECREF(old.buf);
      g_solo.bufs.erase(g_solo.bufs.begin());
    }
  }
  *buf = g_solo.buf;
  *idx = g_solo.next++;
  return true;
}

// A view of row `row`, column idx of n's buffer, whose _ticket is n (new reference or nullptr).
PyObject* solo_view(SoloObject* n, int row) {
  const at::Tensor& b = THPVariable_Unpack(n->buf);
  PyObject* v = THPVariable_Wrap(scalar_at(b, b.storage_offset() + row * b.stride(0) + n->idx * b.stride(1)),
                                 g_fast.norm_view);
  if (v && slot_set(g_fast.d_view_ticket, v, reinterpret_cast<PyObject*>(n)) != 0) Py_CLEAR(v);
  return v;
}

// A full, non-current buffer whose handed-out pool pairs nobody but its record references (the
// views dropped by the caller, the nodes done, no fresh node on it, no alias of the storage) and
// whose last norms were written on `stream`: its pairs can take new norms.
bool solo_recyclable(const SoloState::BufRec& r, unsigned long long stream) {
  if (r.buf == g_solo.buf || r.stream != stream || r.pairs.empty() ||
      Py_REFCNT(r.buf) != 1 + static_cast<Py_ssize_t>(r.pairs.size()))
    return false;
  const at::Tensor& b = THPVariable_Unpack(r.buf);
  if (b.use_count() != 1 || static_cast<size_t>(b.storage().use_count()) != r.pairs.size() + 1) return false;
  for (const auto& pr : r.pairs) {
    if (Py_REFCNT(pr.first) != 1 || Py_REFCNT(pr.second) != 2 || THPVariable_Unpack(pr.first).use_count() != 1 ||
        reinterpret_cast<SoloObject*>(pr.second)->state == kSoloPending)
      return false;
  }
  return true;
}

// Builds the pool for the next round (see SoloState): as many pairs as the last round took,
// recycled from a buffer nobody reads any more, else new. Runs right after a mean's launches
// (the GPU folds meanwhile). 0, or -1 with a Python error.
int solo_refill(int dev, unsigned long long stream) {
  Stamp clock;
  const long long m = std::min<long long>(g_solo.want, kSoloCols);
  g_solo.want = 0;
  if (m <= 0 || !g_solo.type || !g_fast.norm_view || !g_fast.d_view_ticket) return 0;
  solo_compact();
  // pairs handed out since the last refill already moved to their buffers' records; drop the
  // taken slots, keep the rest when they are enough and on this device
  g_solo.pool.erase(g_solo.pool.begin(), g_solo.pool.begin() + static_cast<std::ptrdiff_t>(g_solo.pool_head));
  g_solo.pool_head = 0;
  if (!g_solo.pool.empty()) {
    const auto* n0 = reinterpret_cast<SoloObject*>(g_solo.pool.front().second);
    if (static_cast<long long>(g_solo.pool.size()) >= m && THPVariable_Unpack(n0->buf).get_device() == dev) return 0;
    for (auto& pr : g_solo.pool) Py_DECREF(pr.first), Py_DECREF(pr.second);
    g_solo.pool.clear();
  }
  for (auto& r : g_solo.bufs) {
    if (THPVariable_Unpack(r.buf).get_device() != dev || static_cast<long long>(r.pairs.size()) < m ||
        !solo_recyclable(r, stream))
      continue;
    g_solo.pool.swap(r.pairs);  // (column order: handed out in order)
    ++g_solo.pool_reuses;
    g_solo.refill_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - clock.t).count();
    return 0;
  }
  g_solo.pool.reserve(static_cast<size_t>(m));
  for (long long i = 0; i < m; ++i) {
    PyObject* buf;
    long long idx;
    if (!solo_column(dev, &buf, &idx)) return -1;
    auto* n = reinterpret_cast<SoloObject*>(g_solo.type->tp_alloc(g_solo.type, 0));
    if (!n) return -1;
    Py_INCREF(buf);
    n->buf = buf;
    n->idx = idx;
    if (!solo_reserve(n, 16, 8)) {
      Py_DECREF(n);
      PyErr_NoMemory();
      return -1;
    }
    PyObject* v = solo_view(n, 1);
    if (!v) {
      Py_DECREF(n);
      return -1;
    }
    g_solo.pool.emplace_back(v, reinterpret_cast<PyObject*>(n));
  }
  ++g_solo.pool_builds;
  g_solo.refill_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - clock.t).count();
  return 0;
}

// solo_probe(tree, reps) -> dict: ns per call of the standalone lazy norm's capture steps on one
// tree, repeated (caches warm): the walk with its signature, the structure lookup, the leaf checks,
// the data-pointer reads (data_ptr / const_data_ptr) and the whole capture into a scratch node.
// (tools/prof_capture_parts.py; profiling only)
PyObject* solo_probe(PyObject*, PyObject* args) {
  PyObject* tree;
  long long reps;
  if (!PyArg_ParseTuple(args, "OL", &tree, &reps)) return nullptr;
  if (!g_solo.type) Py_RETURN_NONE;
  using clk = std::chrono::steady_clock;
  auto ns = [&](clk::time_point t0) {
    return std::chrono::duration<double, std::nano>(clk::now() - t0).count() / static_cast<double>(reps);
  };
  try {
    std::vector<PyObject*> lv, dv;
    std::vector<int64_t> sig;
    bool lists = false;
    auto t0 = clk::now();
    for (long long r = 0; r < reps; ++r) {
      lv.clear(), dv.clear(), sig.clear();
      if (solo_walk(tree, lv, dv, lists, 0, &sig) != 0) Py_RETURN_NONE;
    }
    const double t_walk = ns(t0);
    t0 = clk::now();
    const SoloStruct* st = nullptr;
    for (long long r = 0; r < reps; ++r) st = solo_structure(sig);
    const double t_struct = ns(t0);
    if (!st || lv.empty()) Py_RETURN_NONE;
    t0 = clk::now();
    int64_t acc = 0;
    for (long long r = 0; r < reps; ++r)
      for (PyObject* x : lv) {
        const at::Tensor& t = THPVariable_Unpack(x);
        acc += t.layout() == c10::kStrided && t.scalar_type() == at::kFloat && t.is_cuda() && t.is_contiguous() &&
               !t.is_inference();
        acc += t.get_device() + static_cast<int64_t>(t._version()) + t.numel();
      }
    const double t_check = ns(t0);
    t0 = clk::now();
    for (long long r = 0; r < reps; ++r)
      for (PyObject* x : lv) acc += reinterpret_cast<int64_t>(THPVariable_Unpack(x).data_ptr());
    const double t_ptr = ns(t0);
    t0 = clk::now();
    for (long long r = 0; r < reps; ++r)
      for (PyObject* x : lv) acc += reinterpret_cast<int64_t>(THPVariable_Unpack(x).const_data_ptr());
    const double t_cptr = ns(t0);
    auto* n = reinterpret_cast<SoloObject*>(g_solo.type->tp_alloc(g_solo.type, 0));
    if (!n) return nullptr;
    t0 = clk::now();
    for (long long r = 0; r < reps; ++r) {
      if (!solo_capture_into(n, tree)) {
        Py_DECREF(n);
        Py_RETURN_NONE;
      }
      solo_release(n, kSoloDone);
    }
    const double t_cap = ns(t0);
    Py_DECREF(n);
    return Py_BuildValue("{s:d,s:d,s:d,s:d,s:d,s:d,s:L}", "walk_sig_ns", t_walk, "structure_ns", t_struct,
                         "leaf_checks_ns", t_check, "data_ptr_ns", t_ptr, "const_data_ptr_ns", t_cptr,
                         "capture_into_ns", t_cap, "_", static_cast<long long>(acc & 1));
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// tree_l2_norm / tree_l2_squared (which 1 / 0) of a delta no running sum took: a lazy view of a
// SoloNorm node (see "standalone lazy norms"). The most recent node answers for its own tree
// when unchanged (the norm and the squared norm of one delta share a column); a norm takes the
// pool's next pair. Py_None: not the fast case; nullptr: a Python error.
PyObject* solo_norm(PyObject* tree, int which) {
  try {
    // Under a graph capture the norm is computed now, by the launch that computes it whenever it is
    // read alone (solo_resolve: the same kernel and plan, so the same bits), which the graph records:
    // a node with a column of its own (a direct column is never handed out again, a pooled one is
    // once its view is dropped, and every replay writes the column). Asked at the first norm of a
    // round (nothing pending), not per client.
    if (g_solo.pending == 0 &&
        stream_capturing(reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream().stream()))) {
      auto* c = reinterpret_cast<SoloObject*>(g_solo.type->tp_alloc(g_solo.type, 0));
      if (!c) return nullptr;
      struct DropC {
        SoloObject* n;
        ~DropC() { Py_DECREF(n); }
      } drop_c{c};
      if (!solo_capture_into(c, tree)) {
        if (PyErr_Occurred()) return nullptr;
        Py_RETURN_NONE;
      }
      PyObject* buf;
      long long idx;
      if (!solo_column(THPVariable_Unpack(c->leaves[0]).get_device(), &buf, &idx)) return nullptr;
      Py_INCREF(buf);
      Py_XSETREF(c->buf, buf);
      c->idx = idx;
      PyObject* v = solo_view(c, which);
      if (!v) return nullptr;
      c->state = kSoloPending;
      ++g_solo.pending;
      g_solo.pending_bytes += c->nbytes;
      std::vector<SoloObject*> one{c};
      if (solo_resolve(one) != 0) {
        solo_release(c, kSoloDone);
        Py_DECREF(v);
        return nullptr;
      }
      return v;
    }
    if (!g_solo.reg.empty()) {
      SoloObject* c = g_solo.reg.back().node;
      if (c->state == kSoloPending && c->tree == tree && solo_same_tree(c, tree) && solo_unchanged(c))
        return solo_view(c, which);
    }
    SoloObject* n = nullptr;   // (a new reference)
    PyObject* view = nullptr;  // the pool's view for n (a new reference)
    bool pooled = false;       // (its buffer's record holds the view too)
    if (which == 1 && g_solo.pool_head < g_solo.pool.size()) {
      const auto pr = g_solo.pool[g_solo.pool_head];
      auto* pn = reinterpret_cast<SoloObject*>(pr.second);
      if (!solo_capture_into(pn, tree)) {
        if (PyErr_Occurred()) return nullptr;
        Py_RETURN_NONE;  // (the pair stays in the pool)
      }
      if (THPVariable_Unpack(pn->leaves[0]).get_device() == THPVariable_Unpack(pn->buf).get_device()) {
        ++g_solo.pool_head;  // the pool's references to the pair move to its buffer's record
        SoloState::BufRec* rec = nullptr;
        for (auto& r : g_solo.bufs)
          if (r.buf == pn->buf) rec = &r;
        if (rec) {
          rec->pairs.push_back(pr);
          Py_INCREF(pr.first);
          Py_INCREF(pr.second);
        }
        view = pr.first;
        n = pn;
        pooled = rec != nullptr;
      } else {
        solo_release(pn, kSoloDone);  // (a pool on another device: this delta takes a fresh node)
      }
    }
    if (!n) {
      n = reinterpret_cast<SoloObject*>(g_solo.type->tp_alloc(g_solo.type, 0));
      if (!n) return nullptr;
      if (!solo_capture_into(n, tree)) {
        Py_DECREF(n);
        if (PyErr_Occurred()) return nullptr;
        Py_RETURN_NONE;
      }
    }
    struct DropN {
      SoloObject* n;
      ~DropN() { Py_DECREF(n); }
    } drop_n{n};
    const int dev = THPVariable_Unpack(n->leaves[0]).get_device();
    // the pending limits: past max_pending every pending norm is computed now (one launch per
    // run); past the byte budget, the ones whose pytree nobody but the node holds any more (the
    // deltas the views alone keep alive), rechecked after every further quarter budget
    int er = 0;
    if (g_solo.pending + 1 > g_solo.max_pending) {
      er = solo_resolve_all();
    } else if (g_solo.pending_bytes + n->nbytes > solo_budget(dev) && g_solo.pending_bytes + n->nbytes >= g_solo.recheck) {
      er = solo_evict();
      g_solo.recheck = g_solo.pending_bytes + n->nbytes + solo_budget(dev) / 4;
    }
    if (er != 0) {
      Py_XDECREF(view);
      solo_release(n, kSoloDone);
      return nullptr;
    }
    if (!view) {
      PyObject* buf;
      long long idx;
      if (!solo_column(dev, &buf, &idx)) return nullptr;
      Py_INCREF(buf);
      Py_XSETREF(n->buf, buf);
      n->idx = idx;
    }
    if (!view) {
      view = solo_view(n, which);
      if (!view) {
        solo_release(n, kSoloDone);
        return nullptr;
      }
    }
    n->state = kSoloPending;
    ++g_solo.pending;
    g_solo.pending_bytes += n->nbytes;
    if (g_solo.reg.size() >= 2 * static_cast<size_t>(g_solo.pending) + 64) solo_compact();
    Py_INCREF(view);  // (the registry's references: the view and the node)
    Py_INCREF(reinterpret_cast<PyObject*>(n));
    g_solo.reg.push_back(SoloState::Entry{view, n, pooled});
    if (which == 1) ++g_solo.want;
    return view;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// tree_l2_squared / tree_l2_norm (tree_util.py:105-114) of the delta the running sum just
// took: a lazy 0-d view into its chain's norm buffer, which the chain's fold fills
// (tree_util._lazy_norm, built here without a Python frame). The tree must hold exactly the
// captured leaves of the most recent PendingSum link, unmodified — known without a walk when
// it is the captured dict tree with every dict version tag unchanged (same_tree) — and the
// chain must have a norm buffer: its own, or the pool's (FastState), which a chain without
// one takes for its first norm; the pool's views and tickets are handed out by link index.
// Anything else: the Python function.
PyObject* fast_l2(PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames, int which) {
  PyObject* py = g_fast.py_l2[which];
  if (!py) {
    PyErr_SetString(PyExc_RuntimeError, "fedjax_amd.tree_util is not installed (fast_install_norms)");
    return nullptr;
  }
  bool chain_delta = false;  // the running sum's last delta (its chain's norm, by the Python path)
  if (nargs == 1 && !kwnames && g_fast.defer && g_fast.last && g_fast.norm_view && g_fast.ticket &&
      Py_TYPE(args[0]) != g_fast.wt && Py_TYPE(args[0]) != g_fast.ps) {
    PyObject* no = PyWeakref_GetObject(g_fast.last);
    if (no && Py_TYPE(no) == g_fast.ps) {
      auto* node = reinterpret_cast<PSObject*>(no);
      auto* ch = reinterpret_cast<ChainObject*>(node->chain);
      if ((!node->value || node->value == Py_None) && node->cap && PyTuple_CheckExact(node->cap) &&
          PyTuple_GET_SIZE(node->cap) >= 2 && ch && Py_TYPE(ch) == g_fast.chain) {
        Py_INCREF(no);  // (held for the check: the walk below could run Python code)
        struct Drop {
          PyObject* o;
          ~Drop() { Py_DECREF(o); }
        } drop{no};
        try {
          PyObject* tup = PyTuple_GET_ITEM(node->cap, 0);
          bool same = PyTuple_Check(tup) && PyTuple_GET_SIZE(tup) > 0;
          if (same && !same_tree(args[0], node->cap)) {
            PWalk w;
            w.K = 1;
            w.leaves[0].reserve(16);
            PyObject* tree = args[0];
            const int rc = pwalk(&tree, w, 0);
            if (rc < 0) return nullptr;
            same = rc == 0 && static_cast<Py_ssize_t>(w.leaves[0].size()) == PyTuple_GET_SIZE(tup);
            for (size_t l = 0; same && l < w.leaves[0].size(); ++l) same = w.leaves[0][l] == PyTuple_GET_ITEM(tup, l);
            // the captured leaf objects, unmodified since tree_weight (version and storage)
            int64_t vs = 0;
            for (Py_ssize_t l = 0; same && l < PyTuple_GET_SIZE(tup); ++l) {
              const at::Tensor& t = THPVariable_Unpack(PyTuple_GET_ITEM(tup, l));
              vs += version_of(t);
              const int64_t cp = captured_ptr(node->cap, l);
              if (cp && cp != reinterpret_cast<int64_t>(t.data_ptr())) same = false;
            }
            same = same && vs == PyLong_AsLongLong(PyTuple_GET_ITEM(node->cap, 1));
          }
          // (the captured tree itself, unchanged dicts: its leaves' versions and storages are not
          // re-read here — the chain's fold checks every captured leaf before it launches and
          // raises for one modified since tree_weight, so a view is either filled from the
          // values tree_weight saw or never filled)
          if (same) {
            chain_delta = true;
            if ((!ch->buf || ch->buf == Py_None) && which == 1 && g_fast.pool_buf && g_fast.pool_views &&
                !stream_capturing(reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream().stream()))) {
              // (not under a graph capture: replays would write the pool's columns, which are handed
              // out again once their views are dropped; the chain then takes a buffer of its own)
              // the chain's first norm: take the pool as the chain's buffer and views (same device,
              // the current chain size)
              const at::Tensor& pb = THPVariable_Unpack(g_fast.pool_buf);
              const at::Tensor& t0 = THPVariable_Unpack(PyTuple_GET_ITEM(tup, 0));
              if (pb.get_device() == t0.get_device() && pb.dim() == 2 && pb.size(1) == g_fast.max_clients + 1) {
                retire_pool(g_fast.pool_buf, g_fast.pool_all);
                Py_XSETREF(ch->buf, g_fast.pool_buf);
                Py_XSETREF(ch->views, g_fast.pool_views);
                Py_CLEAR(g_fast.pool_all);
                g_fast.pool_buf = g_fast.pool_views = nullptr;
              }
            }
            PyObject* buf = ch->buf;
            if (buf && THPVariable_Check(buf)) {
              const at::Tensor& b = THPVariable_Unpack(buf);
              const int row = which;  // row 0 = squared norms, row 1 = norms
              if (b.dim() == 2 && node->idx < b.size(1)) {
                if (which == 1 && node->idx + 1 > g_fast.pool_want) g_fast.pool_want = node->idx + 1;
                PyObject* pair = nullptr;  // a pool (view, ticket) for this link, if one is left
                if (which == 1 && (!node->ticket || node->ticket == Py_None) && ch->views &&
                    PyList_CheckExact(ch->views) && node->idx < PyList_GET_SIZE(ch->views)) {
                  pair = PyList_GET_ITEM(ch->views, node->idx);
                  if (pair != Py_None && PyTuple_CheckExact(pair) && PyTuple_GET_SIZE(pair) == 2) {
                    // handed out once: the list's reference moves to this call (PyList_SET_ITEM
                    // does not release the item it overwrites)
                    Py_INCREF(Py_None);
                    PyList_SET_ITEM(ch->views, node->idx, Py_None);
                  } else {
                    pair = nullptr;
                  }
                }
                if (pair) {
                  struct DropPair {
                    PyObject* o;
                    ~DropPair() { Py_DECREF(o); }
                  } drop_pair{pair};
                  PyObject* v = PyTuple_GET_ITEM(pair, 0);
                  PyObject* t = PyTuple_GET_ITEM(pair, 1);
                  if (slot_set(g_fast.d_ticket_node, t, no) != 0) return nullptr;
                  Py_INCREF(t);
                  Py_XSETREF(node->ticket, t);
                  Py_INCREF(v);
                  return v;  // (its _ticket was set to t when the pool was built)
                }
                if (!node->ticket || node->ticket == Py_None) {
                  PyObject* t = new_ticket(no);
                  if (!t) return nullptr;
                  Py_XSETREF(node->ticket, t);
                }
                PyObject* v = THPVariable_Wrap(
                    scalar_at(b, b.storage_offset() + row * b.stride(0) + node->idx * b.stride(1)), g_fast.norm_view);
                if (!v) return nullptr;
                if (slot_set(g_fast.d_view_ticket, v, node->ticket) != 0) {
                  Py_DECREF(v);
                  return nullptr;
                }
                return v;
              }
            }
          }
        } catch (const std::exception& e) {
          PyErr_SetString(PyExc_RuntimeError, e.what());
          return nullptr;
        }
      }
    }
  }
  if (!chain_delta && nargs == 1 && !kwnames && g_fast.defer && g_solo.on && g_solo.type && g_solo.rows_fn && g_fast.norm_view &&
      g_fast.d_view_ticket && Py_TYPE(args[0]) != g_fast.wt && Py_TYPE(args[0]) != g_fast.ps) {
    PyObject* v = solo_norm(args[0], which);
    if (v != Py_None) return v;  // (a lazy view, or nullptr with the error set)
    Py_DECREF(v);
  }
  return PyObject_Vectorcall(py, args, nargs, kwnames);
}

void clear_pool() {
  Py_CLEAR(g_fast.pool_buf);
  Py_CLEAR(g_fast.pool_views);
  Py_CLEAR(g_fast.pool_all);
}

// a chain took (buf, all): keep them (new references) for reuse, at most 4 (the oldest goes),
// with the stream the pool was built on (its norms are written and read there)
void retire_pool(PyObject* buf, PyObject* all) {
  if (!buf || !all) return;
  Py_INCREF(buf);
  Py_INCREF(all);
  g_fast.retired.emplace_back(buf, all);
  g_fast.retired_stream.push_back(g_fast.pool_stream);
  if (g_fast.retired.size() > 4) {
    Py_DECREF(g_fast.retired.front().first);
    Py_DECREF(g_fast.retired.front().second);
    g_fast.retired.erase(g_fast.retired.begin());
    g_fast.retired_stream.erase(g_fast.retired_stream.begin());
  }
}

// A retired pool is reusable when nothing but the pool itself references it: the buffer
// object and every pair, view and ticket are held only by the pool (the caller dropped the
// views, the chain is gone) and the buffer's storage has no alias outside the pool's own
// tensors — so writing new norms into it cannot change a value anybody can still read.
bool reusable(PyObject* buf, PyObject* all, c10::DeviceIndex dev, long long m) {
  if (Py_REFCNT(buf) != 1 || !THPVariable_Check(buf) || !PyList_CheckExact(all) || PyList_GET_SIZE(all) < m)
    return false;
  const at::Tensor& b = THPVariable_Unpack(buf);
  if (b.get_device() != dev || b.dim() != 2 || b.size(1) != g_fast.max_clients + 1 || b.use_count() != 1 ||
      static_cast<long long>(b.storage().use_count()) != PyList_GET_SIZE(all) + 1)
    return false;
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(all); ++i) {
    PyObject* pair = PyList_GET_ITEM(all, i);
    if (Py_REFCNT(pair) != 1) return false;
    PyObject* v = PyTuple_GET_ITEM(pair, 0);
    PyObject* t = PyTuple_GET_ITEM(pair, 1);
    if (Py_REFCNT(v) != 1 || THPVariable_Unpack(v).use_count() != 1 || Py_REFCNT(t) != 2) return false;
  }
  return true;
}

// Builds the lazy-norm pool (FastState) for the next round: a retired pool nobody references
// any more, reused whole (every ticket's node reset to None), or a fresh norm buffer on device
// dev and g_fast.pool_want (view of buf[1, i], ticket) pairs, each view's _ticket set to its
// ticket (ticket.node None until fast_l2 hands the pair out). 0, or -1 with a Python error.
int refill_pool(c10::DeviceIndex dev) {
  Stamp clock;
  const long long m = std::min<long long>(g_fast.pool_want, g_fast.max_clients + 1);
  g_fast.pool_want = 0;
  if (m <= 0 || !g_fast.norm_view || !g_fast.ticket || !g_fast.d_view_ticket) return 0;
  if (g_fast.pool_buf) {  // an unused pool: kept if a chain on this device could still take it
    const at::Tensor& pb = THPVariable_Unpack(g_fast.pool_buf);
    if (pb.get_device() == dev && pb.size(1) == g_fast.max_clients + 1 && g_fast.pool_views &&
        PyList_GET_SIZE(g_fast.pool_views) >= m)
      return 0;
    clear_pool();
  }
  const unsigned long long stream =
      reinterpret_cast<unsigned long long>(c10::hip::getCurrentHIPStream(dev).stream());
  for (size_t r = 0; r < g_fast.retired.size(); ++r) {
    auto [buf, all] = g_fast.retired[r];
    // (only on the stream its earlier norms were written on: a kernel on another stream that
    // reads a dropped view may not have run yet, and the new norms must not overtake it)
    if (g_fast.retired_stream[r] != stream || !reusable(buf, all, dev, m)) continue;
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(all); ++i)
      if (slot_set(g_fast.d_ticket_node, PyTuple_GET_ITEM(PyList_GET_ITEM(all, i), 1), Py_None) != 0) return -1;
    PyObject* views = PyList_GetSlice(all, 0, PyList_GET_SIZE(all));
    if (!views) return -1;
    g_fast.retired.erase(g_fast.retired.begin() + static_cast<std::ptrdiff_t>(r));
    g_fast.retired_stream.erase(g_fast.retired_stream.begin() + static_cast<std::ptrdiff_t>(r));
    g_fast.pool_stream = stream;
    g_fast.pool_buf = buf;  // (the retired entry's references move to the pool)
    g_fast.pool_all = all;
    g_fast.pool_views = views;
    ++g_fast.pool_reuses;
    g_fast.refill_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - clock.t).count();
    return 0;
  }
  at::Tensor b = at::empty({2, g_fast.max_clients + 1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
  PyObject* views = PyList_New(m);
  if (!views) return -1;
  for (long long i = 0; i < m; ++i) {
    PyObject* v = THPVariable_Wrap(scalar_at(b, b.size(1) + i), g_fast.norm_view);
    PyObject* t = v ? new_ticket(Py_None) : nullptr;
    if (!t || slot_set(g_fast.d_view_ticket, v, t) != 0) {
      Py_XDECREF(v), Py_XDECREF(t), Py_DECREF(views);
      return -1;
    }
    PyObject* pair = PyTuple_Pack(2, v, t);
    Py_DECREF(v), Py_DECREF(t);
    if (!pair) {
      Py_DECREF(views);
      return -1;
    }
    PyList_SET_ITEM(views, i, pair);
  }
  g_fast.pool_buf = THPVariable_Wrap(b);
  g_fast.pool_views = g_fast.pool_buf ? PyList_GetSlice(views, 0, m) : nullptr;
  if (!g_fast.pool_buf || !g_fast.pool_views) {
    Py_DECREF(views);
    clear_pool();
    return -1;
  }
  g_fast.pool_all = views;
  g_fast.pool_stream = stream;
  ++g_fast.pool_builds;
  g_fast.refill_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - clock.t).count();
  return 0;
}

// drop_pool(): forget the lazy-norm pool (tests; tree_util.set_deferred_sums)
PyObject* drop_pool(PyObject*, PyObject*) {
  clear_pool();
  for (auto& e : g_fast.retired) {
    Py_DECREF(e.first);
    Py_DECREF(e.second);
  }
  g_fast.retired.clear();
  g_fast.retired_stream.clear();
  g_fast.pool_want = 0;
  Py_RETURN_NONE;
}

// pool_info() -> (pool views ready, pool_want, host us of the last refill, retired pools,
//                 refills that reused a retired pool, refills that built one)
PyObject* pool_info(PyObject*, PyObject*) {
  return Py_BuildValue("(nLdnLL)", g_fast.pool_views ? PyList_GET_SIZE(g_fast.pool_views) : Py_ssize_t(0),
                       g_fast.pool_want, g_fast.refill_us, static_cast<Py_ssize_t>(g_fast.retired.size()),
                       g_fast.pool_reuses, g_fast.pool_builds);
}

PyObject* fast_tree_l2_squared(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  return fast_l2(args, nargs, kwnames, 0);
}
PyObject* fast_tree_l2_norm(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  return fast_l2(args, nargs, kwnames, 1);
}

// zeros_like(tree) -> tree | None: tree_util.tree_zeros_like (tree_util.py:41-44) for a plain
// dict / list / tuple / None pytree of float32 device tensors (<= 64 leaves, one device): ONE
// zeroed allocation, and every leaf its own tensor over a 256-byte aligned slice of it (its
// own TensorImpl and in-place version counter, not a view: writing one leaf does not bump
// the others' versions). The result's dict keys are sorted, as jax.tree.map builds them.
// None: not this case (the Python path decides).
PyObject* zeros_like(PyObject*, PyObject* tree) {
  try {
    PWalk w;
    w.K = 1;
    w.leaves[0].reserve(16);
    const int rc = pwalk(&tree, w, 0);
    if (rc < 0) return nullptr;
    const size_t L = w.leaves[0].size();
    if (rc > 0 || L == 0) Py_RETURN_NONE;
    std::vector<int64_t> offs(L + 1, 0);
    int dev = -1;
    for (size_t l = 0; l < L; ++l) {
      const at::Tensor& t = THPVariable_Unpack(w.leaves[0][l]);
      if (t.layout() != c10::kStrided || t.scalar_type() != at::kFloat || !t.is_cuda()) Py_RETURN_NONE;
      if (dev < 0) dev = t.get_device();
      if (t.get_device() != dev) Py_RETURN_NONE;
      offs[l + 1] = offs[l] + (t.numel() + 63) / 64 * 64;
    }
    const at::Tensor& t0 = THPVariable_Unpack(w.leaves[0][0]);
    // zeroed by one hipMemsetAsync on the current stream (at::zeros would add a dispatched fill);
    // under a graph capture by a fill kernel: a recorded memset node takes effect on the graph's
    // first replay only (measured, tools/probe_memset_node.py)
    at::Tensor flat = at::empty({std::max<int64_t>(offs[L], 1)}, t0.options());
    const hipStream_t zs = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(dev)).stream();
    if (stream_capturing(reinterpret_cast<unsigned long long>(zs))) {
      flat.zero_();
    } else if (hipMemsetAsync(flat.data_ptr(), 0, static_cast<size_t>(flat.numel()) * 4, zs) != hipSuccess) {
      PyErr_SetString(PyExc_RuntimeError, "tree_zeros_like: hipMemsetAsync failed");
      return nullptr;
    }
    std::vector<PyObject*> wrapped(L, nullptr);
    struct Drop {
      std::vector<PyObject*>& v;
      ~Drop() {
        for (PyObject* o : v) Py_XDECREF(o);  // (rebuild takes the ones it uses)
      }
    } drop{wrapped};
    for (size_t l = 0; l < L; ++l) {
      at::Tensor leaf = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(flat.storage()), flat.key_set(),
                                                                 flat.dtype());
      leaf.unsafeGetTensorImpl()->set_storage_offset(offs[l]);
      leaf.unsafeGetTensorImpl()->set_sizes_contiguous(THPVariable_Unpack(w.leaves[0][l]).sizes());
      wrapped[l] = THPVariable_Wrap(std::move(leaf));
      if (!wrapped[l]) return nullptr;
    }
    size_t i = 0, ki = 0;
    return rebuild(tree, wrapped.data(), i, w.keys.data(), ki);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// fold_chain(node, scale, has_scale, nt_min_bytes, plan_fn, wsum_fn, wsum_l2_fn, l2_ws_bytes_fn)
//     -> (rc, tree) | k | None
// tree_util._fold_chain for a PendingSum link, walked natively: the unfolded links from the
// nearest folded ancestor (or the chain's root), the base (the root's tree, or the folded
// ancestor's value), then fold_caps over [base capture, link captures] with weights
// [1, n_1 .. n_k]; the squared norms of the links a lazy norm view waits on come from the same
// launch and are written into the chains' norm buffers (tree_util._fill_norms). None (nothing
// launched) when the run has no captured base; k: capture k is stale.
PyObject* fold_chain(PyObject*, PyObject* args) {
  PyObject* node;
  double scale, nt_min;
  int has_scale;
  unsigned long long plan_addr, wsum_addr, l2_addr, l2ws_addr, fill_addr = 0, rows_addr = 0;
  if (!PyArg_ParseTuple(args, "OdpdKKKK|KK", &node, &scale, &has_scale, &nt_min, &plan_addr, &wsum_addr, &l2_addr,
                        &l2ws_addr, &fill_addr, &rows_addr))
    return nullptr;
  if (!g_fast.ps || Py_TYPE(node) != g_fast.ps) Py_RETURN_NONE;
  thread_local std::vector<PSObject*> links;
  links.clear();
  PyObject* base = nullptr;
  for (auto* p = reinterpret_cast<PSObject*>(node);;) {
    if (p->value && p->value != Py_None) {
      base = p->value;
      break;
    }
    links.push_back(p);
    if (!p->parent || p->parent == Py_None) {
      base = p->root;
      break;
    }
    if (Py_TYPE(p->parent) != g_fast.ps) Py_RETURN_NONE;
    p = reinterpret_cast<PSObject*>(p->parent);
  }
  if (links.empty() || !base) Py_RETURN_NONE;
  std::reverse(links.begin(), links.end());
  PyObject* bcap = links[0]->bcap;
  if (!bcap || bcap == Py_None) Py_RETURN_NONE;
  const Py_ssize_t K = static_cast<Py_ssize_t>(links.size()) + 1;
  thread_local std::vector<PyObject*> caps, weights;
  caps.resize(K);
  weights.resize(K);
  static PyObject* one = PyLong_FromLong(1);
  caps[0] = bcap;
  weights[0] = one;
  for (Py_ssize_t j = 1; j < K; ++j) {
    caps[j] = links[j - 1]->cap;
    weights[j] = links[j - 1]->weight;
    if (!caps[j] || !weights[j]) Py_RETURN_NONE;
  }
  // lazy norms waiting on links of this run (tree_util._NormView tickets): every operand's
  // squared norm comes from the same launch (fjagg_wsum_l2_ptrs) and is copied into the chains'
  // norm buffers, as tree_util._fill_norms does
  static PyObject* node_name = PyUnicode_InternFromString("node");
  thread_local std::vector<size_t> waiting;
  waiting.clear();
  for (size_t j = 0; j < links.size(); ++j) {
    PyObject* tk = links[j]->ticket;
    if (!tk || tk == Py_None) continue;
    PyObject* tn = (Py_TYPE(tk) == g_fast.ticket && g_fast.d_ticket_node)
                       ? Py_TYPE(g_fast.d_ticket_node)->tp_descr_get(g_fast.d_ticket_node, tk, nullptr)
                       : PyObject_GetAttr(tk, node_name);
    if (!tn) return nullptr;
    const bool w = tn != Py_None;
    Py_DECREF(tn);
    if (w) waiting.push_back(j);
  }
  try {
    // the common case: the run is consecutive links of ONE chain whose norm buffer covers them —
    // the fold's norm combine writes the buffer's two rows itself (fjagg_wsum_l2_ptrs_rows,
    // operand 0, the base, skipped): no l2 tensor and no fill launch
    L2Rows rows{};
    bool use_rows = false;
    c10::DeviceIndex rows_dev = -1;
    if (!waiting.empty() && rows_addr) {
      PyObject* ch0 = links[0]->chain;
      bool one = ch0 && Py_TYPE(ch0) == g_fast.chain;
      for (size_t j = 1; one && j < links.size(); ++j)
        one = links[j]->chain == ch0 && links[j]->idx == links[0]->idx + static_cast<long long>(j);
      PyObject* buf = one ? reinterpret_cast<ChainObject*>(ch0)->buf : nullptr;
      if (buf && THPVariable_Check(buf)) {
        const at::Tensor& b = THPVariable_Unpack(buf);
        const int64_t i0 = links[0]->idx, n = static_cast<int64_t>(links.size());
        // (the fold's device: its base capture's first leaf; a buffer elsewhere takes the fill path)
        PyObject* bt0 = PyTuple_Check(bcap) && PyTuple_GET_SIZE(bcap) > 0 ? PyTuple_GET_ITEM(bcap, 0) : nullptr;
        const int fold_dev = bt0 && PyTuple_Check(bt0) && PyTuple_GET_SIZE(bt0) > 0 &&
                                     THPVariable_Check(PyTuple_GET_ITEM(bt0, 0))
                                 ? THPVariable_Unpack(PyTuple_GET_ITEM(bt0, 0)).get_device()
                                 : -2;
        if (b.dim() == 2 && b.size(0) == 2 && b.is_contiguous() && b.scalar_type() == at::kFloat && b.is_cuda() &&
            b.get_device() == fold_dev && i0 >= 0 && i0 + n <= b.size(1)) {
          float* row0 = b.data_ptr<float>() + i0;
          rows = L2Rows{reinterpret_cast<WsumL2RowsFn>(rows_addr), row0, row0 + b.size(1), 1};
          use_rows = true;
          rows_dev = b.get_device();
        }
      }
    }
    at::Tensor l2;
    PyObject* l2obj = Py_None;
    if (!waiting.empty() && !use_rows) {
      PyObject* t0 = PyTuple_Check(bcap) && PyTuple_GET_SIZE(bcap) > 0 ? PyTuple_GET_ITEM(bcap, 0) : nullptr;
      if (!t0 || !PyTuple_Check(t0) || PyTuple_GET_SIZE(t0) < 1 || !THPVariable_Check(PyTuple_GET_ITEM(t0, 0)))
        Py_RETURN_NONE;
      l2 = at::empty({K}, THPVariable_Unpack(PyTuple_GET_ITEM(t0, 0)).options().dtype(at::kFloat));
      l2obj = THPVariable_Wrap(l2);
      if (!l2obj) return nullptr;
    }
    Py_INCREF(base);  // (the walk's references are borrowed from the chain, which `node` holds)
    PyObject* got = fold_caps_impl(base, caps.data(), weights.data(), K, scale, has_scale != 0, nt_min, plan_addr,
                                   wsum_addr, l2_addr, l2ws_addr, l2obj, use_rows ? &rows : nullptr);
    if (got && PyTuple_Check(got)) {  // launched: this fold's bytes extend the busy estimate
      const double now = now_s();
      const auto* tip = reinterpret_cast<PSObject*>(node);
      const double bytes = static_cast<double>(tip->bytes) * (1.0 + 1.0 / std::max<long long>(1, tip->n));
      g_mean.busy_until = std::max(now, g_mean.busy_until) + bytes / g_mean.peak;
    }
    Py_DECREF(base);
    if (l2obj != Py_None) Py_DECREF(l2obj);
    if (!got || waiting.empty() || !PyTuple_Check(got) || PyLong_AsLong(PyTuple_GET_ITEM(got, 0)) != 0) return got;
    // runs of consecutive links of one chain: one fjtree_norms_fill launch each (or, without
    // its address, a copy and a sqrt)
    typedef int (*FillFn)(const float*, float*, float*, int64_t, void*);
    auto fill = reinterpret_cast<FillFn>(fill_addr);
    for (size_t j = use_rows ? links.size() : 0; j < links.size();) {
      PyObject* ch = links[j]->chain;
      const size_t j0 = j;
      while (j < links.size() && links[j]->chain == ch &&
             links[j]->idx == links[j0]->idx + static_cast<long long>(j - j0))
        ++j;
      PyObject* buf = ch && Py_TYPE(ch) == g_fast.chain ? reinterpret_cast<ChainObject*>(ch)->buf : nullptr;
      if (buf && THPVariable_Check(buf)) {
        const at::Tensor& b = THPVariable_Unpack(buf);
        // (links past the buffer's end — a chain continued across folds — have no views)
        const int64_t i0 = links[j0]->idx, n = std::min<int64_t>(static_cast<int64_t>(j - j0), b.size(1) - i0);
        if (n <= 0) continue;
        if (fill && b.is_contiguous() && b.scalar_type() == at::kFloat && b.is_cuda() &&
            b.get_device() == l2.get_device()) {
          float* row0 = b.data_ptr<float>() + i0;
          const hipStream_t s = c10::hip::getCurrentHIPStream(l2.get_device()).stream();
          const int rc = fill(l2.data_ptr<float>() + 1 + j0, row0, row0 + b.size(1), n, s);
          if (rc != 0) {
            Py_DECREF(got);
            PyErr_Format(PyExc_RuntimeError, "fjtree_norms_fill failed (%d)", rc);
            return nullptr;
          }
          continue;
        }
        const at::Tensor src = l2.narrow(0, 1 + static_cast<int64_t>(j0), n);
        b.select(0, 0).narrow(0, i0, n).copy_(src);
        at::Tensor dst = b.select(0, 1).narrow(0, i0, n);
        at::sqrt_out(dst, src);
      }
    }
    for (size_t j : waiting) {
      PyObject* tk = links[j]->ticket;
      if ((Py_TYPE(tk) == g_fast.ticket && g_fast.d_ticket_node ? slot_set(g_fast.d_ticket_node, tk, Py_None)
                                                                 : PyObject_SetAttr(tk, node_name, Py_None)) != 0) {
        Py_DECREF(got);
        return nullptr;
      }
      Py_CLEAR(links[j]->ticket);
    }
    // the round's final fold (tree_inverse_weight: the 1/W scale) is in flight: the chain, now
    // folded to its tip, lets go of its norm buffer (its views hold their own references; a sum
    // continued from here starts a new chain), and the next round's lazy-norm pool is built
    // while the GPU folds
    if (has_scale) {
      auto* ch = reinterpret_cast<ChainObject*>(links.back()->chain);
      if (ch && Py_TYPE(ch) == g_fast.chain && ch->tip == node) {
        Py_CLEAR(ch->buf);
        Py_CLEAR(ch->views);
      }
      if (refill_pool(use_rows ? rows_dev : l2.get_device()) != 0) {
        Py_DECREF(got);
        return nullptr;
      }
    }
    return got;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyObject* image_paths(PyObject*, PyObject*) {
  return Py_BuildValue("{s:L,s:L}", "kernel_args", g_image_karg, "uploaded", g_image_upload);
}

PyObject* host_timers(PyObject*, PyObject*) {
  static const char* names[kTPhases] = {"spec",  "checks", "outputs", "plan",           "image",
                                        "upload", "launch", "wrap",    "first_launch_at"};
  PyObject* d = PyDict_New();
  if (!d) return nullptr;
  for (int i = 0; i < kTPhases; ++i) {
    PyObject* v = PyFloat_FromDouble(g_timer_calls ? g_timers[i] / g_timer_calls : 0.0);
    PyDict_SetItemString(d, names[i], v);
    Py_DECREF(v);
    g_timers[i] = 0.0;
  }
  PyObject* c = PyLong_FromLongLong(g_timer_calls);
  PyDict_SetItemString(d, "calls", c);
  Py_DECREF(c);
  g_timer_calls = 0;
  return d;
}

PyMethodDef kMethods[] = {
    {"host_timers", host_timers, METH_NOARGS, "mean per-call microseconds of fold_table's phases (resets)"},
    {"image_paths", image_paths, METH_NOARGS, "fold_table launches with the image in kernel arguments / uploaded"},
    {"gather_rows", gather_rows, METH_VARARGS, "pointer table of K client pytrees (see fjhost.cpp)"},
    {"leaf_versions", leaf_versions, METH_VARARGS, "torch in-place version counters of K pytrees' leaves"},
    {"fold_weights", fold_weights, METH_VARARGS, "f32/i32 weights and W of Python-number weights"},
    {"capture", capture, METH_VARARGS, "leaves + version sum of a tree for a lazy tree_weight"},
    {"capture_probe", capture_probe, METH_VARARGS, "ns per call of capture's parts (profiling)"},
    {"solo_probe", solo_probe, METH_VARARGS, "ns per call of the lazy norm capture's parts (profiling)"},
    {"matches", matches, METH_VARARGS, "tree holds exactly the captured leaves, unmodified"},
    {"compatible", compatible, METH_VARARGS, "tree_add(a, b) is the fast case (structure, float32 leaves)"},
    {"append_check", append_check, METH_VARARGS, "deferred tree_add: structure + capture check in one walk"},
    {"norm_view", norm_view, METH_VARARGS, "0-d view of buf[row, index] as a tensor subclass"},
    {"table_from_caps", table_from_caps, METH_VARARGS, "pointer table of captured leaves, version check"},
    {"fold_caps", fold_caps, METH_VARARGS, "a deferred running sum's fold from its captures, one call"},
    {"leaf_fold", leaf_fold, METH_VARARGS, "fjtree_fold_leaves over 1-2 operand trees (see fjhost.cpp)"},
    {"fold_table", fold_table, METH_VARARGS, "plan image + output leaves + fjagg_wsum_ptrs launch (see fjhost.cpp)"},
    {"mean_pairs", mean_pairs, METH_VARARGS, "tree_mean of (pytree, weight) pairs in one native call (see fjhost.cpp)"},
    {"server_pairs", server_pairs, METH_VARARGS, "fused_tree_mean_update in one native call (see fjhost.cpp)"},
    {"zeros_like", zeros_like, METH_O, "tree_zeros_like of a float32 device pytree: one allocation, own leaves"},
    {"mean_config", mean_config, METH_VARARGS, "configuration of the builtin tree_mean (tree_util._native_mean)"},
    {"tree_mean", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_tree_mean)), METH_FASTCALL | METH_KEYWORDS,
     "tree_mean(pytrees_and_weights)\n--\n\nReturns (weighted) mean of input trees and weights "
     "(fedjax/core/tree_util.py:76-96).\n\nA resident list / tuple of (float32 device pytree, Python-number weight) "
     "pairs is folded by one native call\n(the pytree kernel, pipelined with the walk on an idle GPU); every other "
     "input is\nfedjax_amd.tree_util._tree_mean_py's (one-shot iterables stream in chunks).\n\nThe result's "
     "float32 leaves are slices of one allocation (each its own tensor and\nversion counter): one live leaf keeps "
     "all of them allocated, and torch.save of one\nleaf writes every leaf's bytes (clone a leaf to keep it alone)."},
    {"mean_triples", mean_triples, METH_O, "tree_mean over (client_id, params, weight) triples (aggregator.py:61-75)"},
    {"pipeline_fracs", pipeline_fracs, METH_O, "chunk ends (fractions of K) of tree_mean's fold-bound pipeline"},
    {"busy_until", busy_until, METH_VARARGS, "the shared estimate of when this process's folds finish ([set])"},
    {"fold_chain", fold_chain, METH_VARARGS, "a PendingSum's deferred fold, its links walked natively"},
    {"flush_views", flush_views, METH_O, "fold the chains lazy norm views in an object still wait on"},
    {"fast_install_norms", fast_install_norms, METH_VARARGS, "register tree_util's lazy norm classes and fallbacks"},
    {"drop_pool", drop_pool, METH_NOARGS, "forget the lazy-norm pool"},
    {"solo_config", solo_config, METH_VARARGS, "standalone lazy norms: switch, limits, library entry points"},
    {"solo_resolve", solo_resolve_py, METH_O, "compute pending standalone lazy norms now (None: all)"},
    {"solo_info", solo_info, METH_NOARGS, "standalone lazy norms: pending, fused, computed alone, stale"},
    {"solo_norm", solo_norm_py, METH_VARARGS, "the standalone lazy norm view of a tree, or None"},
    {"solo_times", solo_times, METH_NOARGS, "host us the means spent releasing, compacting, refilling (resets)"},
    {"pool_info", pool_info, METH_NOARGS, "(pool views ready, norms asked for since the last refill)"},
    {"tree_l2_squared", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_tree_l2_squared)),
     METH_FASTCALL | METH_KEYWORDS,
     "tree_l2_squared(pytree)\n--\n\nReturns squared l2 norm of tree (fedjax/core/tree_util.py:105-108), a 0-d "
     "float32 tensor.\n\nThe delta a deferred running sum just took gets a lazy view its fold fills; anything "
     "else is\nfedjax_amd.tree_util._tree_l2_squared_py."},
    {"tree_l2_norm", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_tree_l2_norm)),
     METH_FASTCALL | METH_KEYWORDS,
     "tree_l2_norm(pytree)\n--\n\nReturns l2 norm of tree (fedjax/core/tree_util.py:111-114), a 0-d float32 "
     "tensor.\n\nThe delta a deferred running sum just took gets a lazy view its fold fills; anything else "
     "is\nfedjax_amd.tree_util._tree_l2_norm_py."},
    {"fast_install", fast_install, METH_VARARGS, "register tree_util's lazy classes and Python fallbacks"},
    {"fast_config", fast_config, METH_VARARGS, "deferred-sum settings (tree_util.set_deferred_sums)"},
    {"set_last", set_last, METH_O, "remember the most recent PendingSum link (weakly)"},
    {"last", last, METH_NOARGS, "the most recent PendingSum link, or None"},
    {"tree_weight", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_tree_weight)),
     METH_FASTCALL | METH_KEYWORDS,
     "tree_weight(pytree, weight)\n--\n\nWeights tree leaves by weight (fedjax/core/tree_util.py:29-32).\n\n"
     "Float32 device pytrees (<= 64 leaves) with a Python-number weight give a WeightedTree\n"
     "(deferred, fused into the tree_add that consumes it); anything else is computed now\n"
     "by the pytree kernel (fedjax_amd.tree_util._tree_weight_py)."},
    {"tree_add", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_tree_add)), METH_FASTCALL | METH_KEYWORDS,
     "tree_add(left, right)\n--\n\nAdds two trees together (fedjax/core/tree_util.py:47-50).\n\n"
     "The running sum s = tree_add(s, tree_weight(x, n)) appends to a deferred PendingSum\n"
     "(one launch folds the round); every other case is fedjax_amd.tree_util._tree_add_py."},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fjhost", "native host side of the pytree aggregation path",
                       -1, kMethods};

}  // namespace

// The torch this extension was compiled against (fedjax_amd._lib.torch_stamp(), passed by
// __graft_entry__.build()): fjhost reaches into torch's TensorImpl / THPVariable layout, so
// _lib.host() refuses to use it under any other torch (a layout mismatch would not fail
// loudly by itself).
#ifndef FJHOST_TORCH_STAMP
#define FJHOST_TORCH_STAMP "unstamped"
#endif

PyMODINIT_FUNC PyInit__fjhost(void) {
  PyObject* m = PyModule_Create(&kModule);
  if (!m) return nullptr;
  if (PyModule_AddStringConstant(m, "TORCH_STAMP", FJHOST_TORCH_STAMP) != 0) {
    Py_DECREF(m);
    return nullptr;
  }
  const std::pair<const char*, PyType_Spec*> types[] = {
      {"WeightedBase", &kWTSpec}, {"ChainBase", &kChainSpec}, {"PendingBase", &kPSSpec}, {"SoloNorm", &kSoloSpec}};
  for (const auto& t : types) {
    PyObject* tp = PyType_FromSpec(t.second);
    if (tp && t.second == &kSoloSpec) {
      Py_INCREF(tp);
      g_solo.type = reinterpret_cast<PyTypeObject*>(tp);
    }
    if (!tp || PyModule_AddObject(m, t.first, tp) != 0) {
      Py_XDECREF(tp);
      Py_DECREF(m);
      return nullptr;
    }
  }
  return m;
}
