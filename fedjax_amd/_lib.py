"""ctypes binding of ``libfjagg.so`` — the C ABI declared in ``include/fjagg.h``
(aggregation), ``include/fjcomp.h`` (compression aggregators) and
``include/fjcomm.h`` (client-sharded aggregation over RCCL, timing events) and
``include/fjtree.h`` (per-call tree ops, leaf table in the kernel arguments) and
``include/fjopt.h`` (the adafactor server step).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950) into
``fedjax_amd/_build/libfjagg.so``. It links against the HIP runtime by soname
(``libamdhip64.so.7``); ``torch`` is imported first so that the library binds to
the HIP runtime torch already loaded (one runtime per process, so torch's
streams and device pointers are valid inside the library). ``load()`` verifies
that exactly one HIP runtime is mapped.

There is no fallback: if the library is missing or fails to load, every entry
point raises :class:`FjaggError`.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FJAGG_LIB", os.path.join(_HERE, "_build", "libfjagg.so"))

# enum fjagg_dtype
F32, BF16, I32 = 0, 1, 2
# enum fjagg_flags
SCALE, ACCUMULATE, NONTEMPORAL, UNALIGNED, UNBALANCED, NARROW, HOST_TABLES = 1, 2, 4, 8, 16, 32, 64
ZEROED_WS = 128  # fused-norm calls: the workspace's 16-byte completion counter is zero (fjagg.h)
KARG_MAX_WEIGHTS, KARG_MAX_WORDS = 1024, 3584
# enum fjagg_mode
MODE_EXACT, MODE_SPLIT = 0, 1
ABI_VERSION = 3
COMP_ABI_VERSION = 1
COMM_ABI_VERSION = 1
COMM_ID_BYTES = 128
COMM_MAX_BUCKETS = 64
COMM_MAX_DEVICES = 16
TREE_ABI_VERSION = 1
TREE_MAX_LEAVES, TREE_MAX_OPERANDS = 64, 2
TREE_NORM, TREE_NO_OUT = 1 << 8, 1 << 9
TREE_ORDERED = 1 << 10  # FJTREE_ORDERED: norm combine by release/acquire atomics (fjtree.h)
# include/fjcomp.h
COMP_UNIFORM, COMP_TERNGRAD, COMP_BINARY = 1, 2, 3
WHT_PLAIN, WHT_ROTATE, WHT_UNROTATE, WHT_UNROTATE_DRIVE = 0, 1, 2, 3
STATS_CHUNK = 16384

# every symbol include/fjagg.h declares: (name, restype, argtypes)
_i64, _i32, _f32, _vp, _u64 = ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint64
_u32 = ctypes.c_uint32
_SIGNATURES = {
    "fjagg_last_error": (ctypes.c_char_p, []),
    "fjagg_abi_version": (_i32, []),
    "fjagg_wsum_dense": (_i32, [_i32, _i32, _i32, _vp, _i64, _i64, _i64, _vp, _f32, _vp, _i32, _i32, _vp, _i64, _vp]),
    "fjagg_split_workspace_bytes": (_i64, [_i64, _i64]),
    "fjagg_ptrs_plan": (_i64, [_i32, _i32, _vp, _i32, _vp, _i64]),
    "fjagg_ptrs_plan_leaves": (_i64, [_i32, _i32, _vp, _vp, _i32, _vp, _i64]),
    "fjagg_wsum_ptrs": (_i32, [_i32, _i32, _i32, _vp, _i32, _i64, _i64, _vp, _f32, _i32, _vp]),
    "fjagg_karg_image_words": (_i64, [_i64, _i32, _i64]),
    "fjagg_wsum_l2_ptrs_workspace_bytes": (_i64, [_i64, _i64]),
    "fjagg_wsum_l2_ptrs": (_i32, [_i32, _i32, _i32, _vp, _i32, _i64, _i64, _vp, _f32, _vp, _i32, _vp, _i64, _vp]),
    "fjagg_wsum_l2_ptrs_rows": (_i32, [_i32, _i32, _i32, _vp, _i32, _i64, _i64, _vp, _f32, _vp, _vp, _i64, _i32, _vp,
                                       _i64, _vp]),
    "fjagg_server_update_dense": (_i32, [_i32, _vp, _i64, _i64, _i64, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _i32, _vp]),
    "fjagg_server_update_ptrs": (_i32, [_i32, _vp, _i32, _i64, _i64, _vp, _f32, _vp, _vp, _i32, _vp]),
    "fjagg_wsum_l2_workspace_bytes": (_i64, [_i64, _i64]),
    "fjagg_wsum_l2_dense": (_i32, [_i32, _i32, _i32, _vp, _i64, _i64, _i64, _vp, _f32, _vp, _vp, _i32, _vp, _i64, _vp]),
    "fjagg_l2sq_workspace_bytes": (_i64, [_i64, _i64]),
    "fjagg_l2sq_dense": (_i32, [_i32, _vp, _i64, _i64, _i64, _vp, _vp, _i64, _vp]),
    "fjagg_l2sq_rows_workspace_bytes": (_i64, [_i64, _i64]),
    "fjagg_l2sq_rows": (_i32, [_i32, _vp, _i64, _i64, _i64, _i32, _vp, _vp, _i64, _vp]),
    "fjagg_fill_synth": (_i32, [_i32, _vp, _i64, _i64, _i64, _i64, _u64, _f32, _vp]),
    # include/fjcomp.h
    "fjcomp_abi_version": (_i32, []),
    "fjcomp_threefry2x32": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "fjcomp_random_split": (_i32, [_vp, _i64, _i64, _vp]),
    "fjcomp_prng_sequence": (_i32, [_vp, _i64, _vp]),
    "fjcomp_random_bits": (_i32, [_u32, _u32, _i64, _vp, _vp]),
    "fjcomp_uniform": (_i32, [_u32, _u32, _i64, _vp, _vp]),
    "fjcomp_rademacher": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp]),
    "fjcomp_row_stats_workspace_bytes": (_i64, [_i64]),
    "fjcomp_row_stats": (_i32, [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _i64, _vp]),
    "fjcomp_stats_combine": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "fjcomp_quant_fold": (_i32, [_i32, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _i64, _i32, _f32, _i32, _vp,
                                 _vp, _vp]),
    "fjcomp_wht_tiles": (_i64, [_i32, _i32]),
    "fjcomp_wht": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp]),
    # include/fjcomm.h
    "fjcomm_abi_version": (_i32, []),
    "fjcomm_unique_id": (_i32, [_vp]),
    "fjcomm_init": (_i32, [_vp, _vp, _i32, _i32]),
    "fjcomm_destroy": (_i32, [_vp]),
    "fjcomm_abort": (_i32, [_vp]),
    "fjcomm_test_block": (_i32, [_i64, _vp]),
    "fjcomm_sharded_wsum_dense": (_i32, [_vp, _i32, _vp, _i64, _i64, _i64, _vp, _f32, _vp, _i32, _i32, _i32, _vp,
                                         _vp]),
    "fjcomm_sharded_wsum_dense_edges": (_i32, [_vp, _i32, _vp, _i64, _i64, _i64, _vp, _f32, _vp, _vp, _i32, _i32,
                                               _i32, _vp, _vp]),
    "fjcomm_init_all": (_i32, [_vp, _i32, _vp]),
    "fjcomm_multi_wsum_dense": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _i64, _vp, _f32, _vp, _vp, _i32, _i32, _i32,
                                       _vp]),
    "fjagg_event_create": (_i32, [_vp]),
    "fjagg_event_destroy": (_i32, [_vp]),
    "fjagg_event_record": (_i32, [_vp, _vp]),
    "fjagg_event_elapsed_ms": (_i32, [_vp, _vp, _vp]),
    # include/fjtree.h
    "fjtree_abi_version": (_i32, []),
    "fjtree_workspace_bytes": (_i64, [_vp]),
    "fjtree_fold_leaves": (_i32, [_vp, _vp]),
    "fjtree_norms_fill": (_i32, [_vp, _vp, _vp, _i64, _vp]),
    # include/fjopt.h
    "fjopt_abi_version": (_i32, []),
    "fjopt_adafactor_plan": (_i64, [_vp, _i32, _vp, _vp, _i64, _vp]),
    "fjopt_adafactor_step": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp]),
    # include/fjalloc.h (opt-in delta-memory segments, fedjax_amd.memory)
    "fjalloc_alloc": (_vp, [ctypes.c_ssize_t, _i32, _vp]),
    "fjalloc_free": (None, [_vp, ctypes.c_size_t, _i32, _vp]),
    "fjalloc_stats": (_i32, [_i32, _vp]),
    "fjalloc_configure": (_i32, [_i64, _i64, _i32, _i64]),
}
SYMBOLS = tuple(_SIGNATURES)


class ServerOpt(ctypes.Structure):
    """struct fjagg_server_opt (include/fjagg.h)."""
    _fields_ = [("kind", ctypes.c_int), ("nesterov", ctypes.c_int), ("neg_lr", ctypes.c_float),
                ("decay", ctypes.c_float), ("one_minus_b1", ctypes.c_float), ("b1", ctypes.c_float),
                ("one_minus_b2", ctypes.c_float), ("b2", ctypes.c_float), ("bc1", ctypes.c_float),
                ("bc2", ctypes.c_float), ("eps", ctypes.c_float), ("eps_root", ctypes.c_float),
                ("flags", ctypes.c_int)]


OPT_SGD, OPT_MOMENTUM, OPT_ADAM, OPT_ADAGRAD, OPT_RMSPROP, OPT_YOGI = 1, 2, 3, 4, 5, 6
OPT_F_MOMENTUM, OPT_F_CENTERED = 1, 2


class AfLeaf(ctypes.Structure):
    """struct fjopt_af_leaf (include/fjopt.h)."""
    _fields_ = [("g", _vp), ("p", _vp), ("v_row", _vp), ("v_col", _vp), ("v", _vp), ("m", _vp), ("n", _i64),
                ("dims", _i64 * 5), ("factored", _i32), ("d0_is_lo", _i32), ("decay_weights", _i32),
                ("reserved", _i32)]


class AfHparams(ctypes.Structure):
    """struct fjopt_af_hparams (include/fjopt.h)."""
    _fields_ = [("decay_rate_t", _f32), ("one_minus_decay", _f32), ("eps", _f32), ("clip", _i32),
                ("clip_threshold", _f32), ("has_lr", _i32), ("lr", _f32), ("param_scale", _i32),
                ("min_scale", _f32), ("momentum", _i32), ("mom_decay", _f32), ("one_minus_mom", _f32),
                ("weight_decay", _i32), ("wd", _f32)]


OPT_ABI_VERSION = 1


class TreeLeaves(ctypes.Structure):
    """struct fjtree_leaves (include/fjtree.h)."""
    _fields_ = [("K", ctypes.c_int), ("L", ctypes.c_int),
                ("x", (ctypes.c_void_p * 64) * 2), ("out", ctypes.c_void_p * 64), ("n", ctypes.c_int64 * 64),
                ("w", ctypes.c_float * 2), ("scale", ctypes.c_float), ("flags", ctypes.c_int),
                ("norm_operand", ctypes.c_int), ("norm_out", ctypes.c_void_p), ("ws", ctypes.c_void_p),
                ("ws_bytes", ctypes.c_int64)]


class FjaggError(RuntimeError):
    """A libfjagg call failed (message from ``fjagg_last_error``) or the library
    could not be loaded."""


_lib = None
_lock = threading.Lock()


def hip_runtimes_mapped() -> list:
    """Distinct libamdhip64 files mapped into this process."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})
    except OSError:  # pragma: no cover
        return []


def load() -> ctypes.CDLL:
    """Load libfjagg.so once; raise FjaggError if it is missing or inconsistent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise FjaggError(
                f"{LIB_PATH} is missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` from the repo root")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise FjaggError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                raise FjaggError(f"{LIB_PATH} does not export {name}")
            fn.restype, fn.argtypes = res, args
        got = (lib.fjagg_abi_version(), lib.fjcomp_abi_version(), lib.fjcomm_abi_version(),
               lib.fjtree_abi_version())
        want = (ABI_VERSION, COMP_ABI_VERSION, COMM_ABI_VERSION, TREE_ABI_VERSION)
        if got != want:
            raise FjaggError(f"ABI mismatch: library {got} != {want}")
        runtimes = hip_runtimes_mapped()
        if len(runtimes) > 1:
            raise FjaggError(f"two HIP runtimes mapped into one process: {runtimes}")
        _lib = lib
        return lib


HOST_PATH = os.path.join(_HERE, "_build", "_fjhost.so")
_host = None
_REBUILD = "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'` from the repo root"


def torch_stamp() -> str:
    """The torch build _fjhost.so must be compiled against: version, git revision, HIP
    version and C++ ABI flag (fjhost.cpp uses torch's TensorImpl / THPVariable layout)."""
    import sys

    ver = getattr(torch, "version", None)
    return (f"torch {torch.__version__} git {getattr(ver, 'git_version', '?')} hip {getattr(ver, 'hip', None)} "
            f"cxx11abi {int(torch._C._GLIBCXX_USE_CXX11_ABI)} py {sys.version_info[0]}.{sys.version_info[1]}")


def host_stamp_path(path: str = None) -> str:
    """The stamp file build() writes beside _fjhost.so (read before the library is loaded)."""
    return (path or HOST_PATH) + ".torch"


def host():
    """The native host helper ``_fjhost`` (fedjax_amd/csrc/fjhost.cpp: pytree walk and
    pointer table, weight packing; no device work). Raises FjaggError if it is missing or
    was built against another torch: its stamp file (checked before the library is loaded,
    since a mismatched build can fail inside dlopen or misread torch's objects) and the
    TORCH_STAMP compiled into it must both equal :func:`torch_stamp`."""
    global _host
    if _host is None:
        import importlib.machinery
        import importlib.util

        if not os.path.exists(HOST_PATH):
            raise FjaggError(f"{HOST_PATH} is missing: {_REBUILD}")
        want = torch_stamp()
        try:
            with open(host_stamp_path()) as f:
                built = f.read().strip()
        except OSError:
            built = None
        if built != want:
            raise FjaggError(f"{HOST_PATH} was built against [{built or 'no stamp file'}], this process runs "
                             f"[{want}]: {_REBUILD}")
        loader = importlib.machinery.ExtensionFileLoader("_fjhost", HOST_PATH)
        spec = importlib.util.spec_from_file_location("_fjhost", HOST_PATH, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        if getattr(mod, "TORCH_STAMP", None) != want:
            raise FjaggError(f"{HOST_PATH} was compiled against [{getattr(mod, 'TORCH_STAMP', None)}], this "
                             f"process runs [{want}] (its stamp file says otherwise): {_REBUILD}")
        _host = mod
    return _host


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().fjagg_last_error().decode(errors="replace")
        raise FjaggError(f"{what} failed ({rc}): {msg}")


def call(name: str, *args):
    """Call an int-returning entry point and raise on a non-zero status."""
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc


def upload(host: "torch.Tensor", device) -> "torch.Tensor":
    """``host`` on ``device`` through pinned memory, ordered on the current stream (the plan images
    and weights the kernels read). Refused while that stream is being captured into a graph: once
    the copy is recorded, the pinned staging tensor goes back to torch's host allocator, which hands
    the block out again, and a replay would copy whatever it then holds (kernel pointers, weights)."""
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("fedjax_amd: this call uploads a host table through a pinned staging buffer, "
                           "which a graph replay cannot reuse safely; not capturable (the dense fold with "
                           "device weights and the kernel-argument paths are)")
    return host.pin_memory().to(device, non_blocking=True)
