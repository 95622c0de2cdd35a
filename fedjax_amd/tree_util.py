"""``fedjax.tree_util`` for device-resident torch pytrees, computed by HIP kernels.

Drop-in for google/fedjax 0.0.17 ``fedjax/core/tree_util.py`` (re-exported as
``fedjax.tree_util``, fedjax/__init__.py:22). Same names, arguments, return
structure and error behaviour; leaves are ``torch`` tensors on a ROCm device
(host tensors, numpy arrays and Python scalars are copied to the device first —
the host-resident deployment path).

Every arithmetic op goes through ``libfjagg.so`` (``fedjax_amd.kernels``). There
is no CPU / PyTorch fallback: without the library or a GPU these raise.

Semantics follow the reference under JAX's defaults (x64 disabled):

* the fold of :func:`tree_mean` is the reference's exact op sequence —
  ``t_k = fl(x_k * f32(w_k))``, ``s_0 = t_0``, ``s_k = fl(s_{k-1} + t_k)``,
  ``y = fl(s * f32(1/W))`` with ``W`` summed on the host exactly as
  tree_util.py:86,95 does — so float32 results are bitwise equal to FedJAX's;
* Python numbers are weakly typed (take the leaf's dtype), int64/float64 leaves
  canonicalise to int32/float32, int32 leaves with Python-int weights fold in
  wrapping int32 and become float32 only at the final ``1/W`` scale;
* bfloat16 leaves are folded in float32 and rounded once (DESIGN.md §4 states the
  bound against an f64 oracle); ``set_bf16_semantics("reference")`` instead rounds
  every product and sum to bfloat16 as the reference's jnp ops do, bit for bit.
"""

from __future__ import annotations

import copy
import ctypes
import numbers
import os
import time
import weakref
from typing import Any, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from fedjax_amd import _lib, kernels, pytree
from fedjax_amd.typing import PyTree

__all__ = [
    "tree_weight", "tree_inverse_weight", "tree_zeros_like", "tree_add", "tree_sum",
    "tree_mean", "tree_size", "tree_l2_squared", "tree_l2_norm", "tree_clip_by_global_norm",
    "tree_l2_norms", "tree_mean_with_l2_norms", "WeightedTree", "PendingSum", "set_deferred_sums",
    "set_lazy_norms", "set_bf16_semantics", "bf16_semantics",
]

# Non-temporal loads pay off once the deltas cannot stay in the 256 MiB Infinity
# Cache (interleaved A/B, profiles/r01_probe2.jsonl + r01_pytree_c2b.json: +10 % at
# 17 GB, +13 % at 618 MB on the 16-byte vector path).
NONTEMPORAL_MIN_BYTES = 256 << 20

_CANONICAL = {
    torch.float32: torch.float32, torch.bfloat16: torch.bfloat16, torch.int32: torch.int32,
    torch.int64: torch.int32, torch.float64: torch.float32,
}


# --------------------------------------------------------------------------- leaves
def _default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise _lib.FjaggError("fedjax_amd aggregates on a ROCm GPU; torch.cuda.is_available() is False")
    return torch.device("cuda", torch.cuda.current_device())


def _find_device(leaves: Iterable[Any]) -> torch.device:
    for x in leaves:
        if isinstance(x, torch.Tensor) and x.is_cuda:
            return x.device
    return _default_device()


def _to_tensor(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x
    if hasattr(x, "__dlpack__") and not isinstance(x, (np.ndarray, np.generic)):
        return torch.from_dlpack(x)  # e.g. a jax.Array on the ROCm device: zero-copy
    if isinstance(x, (bool, np.bool_)):
        raise TypeError("boolean leaves are not supported")
    if isinstance(x, numbers.Integral) and not isinstance(x, np.generic):
        return torch.tensor(x, dtype=torch.int32)
    if isinstance(x, numbers.Real) and not isinstance(x, np.generic):
        return torch.tensor(x, dtype=torch.float32)
    a = np.asarray(x)
    if not a.flags.writeable or not a.flags.c_contiguous:
        a = np.ascontiguousarray(a).copy()
    return torch.from_numpy(a)


_NATIVE = (torch.float32, torch.bfloat16, torch.int32)
pytree.register_leaf_type(torch.Tensor)
pytree.register_leaf_type(np.ndarray)


def _device_index(device: torch.device) -> int:
    """x.get_device() value of tensors on ``device`` (-1 for the host)."""
    if device.type != "cuda":
        return -1
    return device.index if device.index is not None else torch.cuda.current_device()


def _device_leaf(x, device: torch.device, index: Optional[int] = None) -> torch.Tensor:
    """Leaf as a contiguous device tensor of a canonical dtype (jnp.asarray rules)."""
    if index is None:
        index = _device_index(device)
    if type(x) is torch.Tensor and x.dtype in _NATIVE and x.get_device() == index and x.is_contiguous():
        return x  # the common case: a delta already on the GPU (cheapest accessors first)
    t = _to_tensor(x)
    dt = _CANONICAL.get(t.dtype)
    if dt is None:
        raise TypeError(f"leaf dtype {t.dtype} is not supported (float32, bfloat16, int32; "
                        "int64/float64 canonicalise to 32 bits)")
    if t.device != device:
        t = t.to(device, non_blocking=t.is_pinned())
    if t.dtype != dt:
        t = t.to(dt)
    if not t.is_contiguous():
        t = t.contiguous()
    return t


# -------------------------------------------------------------------------- weights
_WEAK_INT, _WEAK_FLOAT, _STRONG_INT, _STRONG_FLOAT = range(4)


def _host_weight(w):
    """A weight as the host value the reference would compute with: Python numbers
    stay Python numbers (weakly typed); arrays/tensors become numpy scalars."""
    if type(w) is int or type(w) is float:
        return w
    if isinstance(w, torch.Tensor):
        if w.numel() != 1:
            raise ValueError("weights must be scalars")
        a = w.detach().reshape(()).cpu().numpy()
        return a[()]
    if isinstance(w, np.ndarray):
        if w.size != 1:
            raise ValueError("weights must be scalars")
        return w.reshape(())[()]
    return w


def _weight_kind(w) -> int:
    t = type(w)
    if t is int:
        return _WEAK_INT
    if t is float:
        return _WEAK_FLOAT
    if isinstance(w, np.generic):
        if isinstance(w, np.bool_):
            return _STRONG_INT
        return _STRONG_INT if isinstance(w, np.integer) else _STRONG_FLOAT
    if isinstance(w, numbers.Integral):  # includes bool
        return _WEAK_INT
    if isinstance(w, numbers.Real):
        return _WEAK_FLOAT
    raise TypeError(f"weight {w!r} is not a real scalar")


def _inverse(W):
    """tree_util.py:37,60: ``(1. / weight) if weight > 0. else 0.`` on the host."""
    return (1.0 / W) if W > 0.0 else 0.0


# ----------------------------------------------------------------------- fold engine
_BF16 = {"mode": "f32"}


def set_bf16_semantics(mode: str) -> None:
    """How folds over bfloat16 leaves round (tree_mean, tree_sum, tree_add, tree_weight,
    tree_inverse_weight, RunningMean, ClientDeltaSlab.mean).

    ``"f32"`` (default): accumulate in float32 and round once to bfloat16 — far more
    accurate than the reference, within the bound of DESIGN.md §4 of the exact value.
    ``"reference"``: the reference's arithmetic bit for bit — jnp on bf16 leaves with
    weakly typed weights (tree_util.py:32,50,60): each weight and ``1/W`` become bf16 and
    every product and every sum is rounded to bf16 (fjagg acc dtype FJAGG_BF16).
    A strongly typed float32 weight promotes the fold to float32 in both modes, as in
    the reference."""
    if mode not in ("f32", "reference"):
        raise ValueError(f"bf16 semantics must be 'f32' or 'reference', got {mode!r}")
    _BF16["mode"] = mode


def bf16_semantics() -> str:
    """The current :func:`set_bf16_semantics` mode."""
    return _BF16["mode"]


def _leaf_rule(dt: torch.dtype, kinds: Sequence[int], scaled_kind: Optional[int]):
    """(in_code, acc_code, out_dtype) of one leaf position under JAX promotion."""
    strong_float = any(k == _STRONG_FLOAT for k in kinds) or scaled_kind == _STRONG_FLOAT
    if dt == torch.float32:
        return _lib.F32, _lib.F32, torch.float32
    if dt == torch.bfloat16:
        if strong_float:
            return _lib.BF16, _lib.F32, torch.float32
        return _lib.BF16, (_lib.BF16 if _BF16["mode"] == "reference" else _lib.F32), torch.bfloat16
    # int32 leaves: int * int folds in int32; int * float promotes to float32
    if all(k in (_WEAK_INT, _STRONG_INT) for k in kinds):
        return _lib.I32, _lib.I32, (torch.int32 if scaled_kind is None else torch.float32)
    return _lib.I32, _lib.F32, torch.float32


def _fold(rows, weights, *, scale=None,
          out: Optional[List[torch.Tensor]] = None, accumulate: bool = False,
          nontemporal: Optional[bool] = None, validated: bool = False,
          l2sq: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    """y_l = [out_l +] sum_k fl(rows[k][l] * w_k) [* scale] for every leaf l, one
    kernel launch per (input, fold, output) dtype group. ``out`` gives the
    destination tensors (fresh ones otherwise); ``accumulate`` folds into them.
    ``rows``: K lists of L leaves, or a :class:`_Table` (client 0's leaves + the K x L
    pointer table). ``weights``: host weights, or a :class:`_Weights` (already packed).
    ``validated``: rows come from _client_rows / _client_table (shapes and dtypes
    already checked). ``l2sq`` (float32 [K]): also write every client's squared l2 norm
    over all leaves, from the same pass (fjagg_wsum_l2_ptrs; float leaves of one dtype)."""
    if accumulate and out is None:
        raise ValueError("accumulate needs out")
    table = rows if isinstance(rows, _Table) else None
    if (table is not None and nontemporal is None and isinstance(weights, _Weights) and table.row0):
        outs = _native_fold(table, weights, scale, out, accumulate, l2sq)
        if outs is not None:
            return outs
    if table is not None:
        rows, validated = [table.row0], True  # built by _client_table, which checked every client
    K, L = (len(rows) if table is None else table.ptrs.shape[0]), len(rows[0])
    packed = weights if isinstance(weights, _Weights) else None
    kinds = packed.kinds if packed is not None else [_weight_kind(w) for w in weights]
    scaled_kind = None if scale is None else _weight_kind(scale)
    device = rows[0][0].device if L else None
    outs: List[Optional[torch.Tensor]] = [None] * L
    groups = {}
    if not validated:
        # x.size() is ~8x cheaper than x.shape; this loop runs once per (client, leaf)
        sig0 = [(x.size(), x.dtype) for x in rows[0]]
        for k in range(1, K):  # rows are on `device` already (_client_rows)
            if [(x.size(), x.dtype) for x in rows[k]] != sig0:
                _check_row(k, rows[k], sig0)
    rules = {}  # leaf dtype -> (in, acc, out dtype): the rule depends on the weights only
    for l in range(L):
        x0 = rows[0][l]
        rule = rules.get(x0.dtype)
        if rule is None:
            rule = rules[x0.dtype] = _leaf_rule(x0.dtype, kinds, scaled_kind)
        in_c, acc_c, out_dt = rule
        if out is not None:
            o = out[l]
            if o.dtype != out_dt or o.size() != x0.size() or not o.is_contiguous() or o.device != device:
                raise ValueError(f"leaf {l}: destination must be a contiguous {out_dt} tensor "
                                 f"of shape {tuple(x0.shape)} on {device}")
        else:
            o = torch.empty(x0.size(), dtype=out_dt, device=device)
        outs[l] = o
        groups.setdefault((in_c, acc_c, kernels.dtype_code(out_dt)), []).append(l)

    if l2sq is not None:
        if len(groups) != 1 or next(iter(groups))[1] != _lib.F32 or next(iter(groups))[0] == _lib.I32:
            # (a bf16 reference fold has no fused-norm kernel: callers take two passes)
            raise TypeError("fused l2 norms need float leaves of one dtype and a float fold")
        if l2sq.dtype != torch.float32 or l2sq.numel() != K or l2sq.device != device:
            raise ValueError(f"l2sq must be a float32 [{K}] tensor on {device}")
    for (in_c, acc_c, out_c), ls in groups.items():
        leaf_n = np.array([rows[0][l].numel() for l in ls], dtype=np.int64)
        if not leaf_n.any():
            if l2sq is not None:
                l2sq.zero_()
            continue
        if table is not None:
            in_ptrs = table.ptrs if len(ls) == L else table.ptrs[:, ls]
        elif len(ls) == L:
            in_ptrs = np.array([[x.data_ptr() for x in row] for row in rows], dtype=np.int64)
        else:
            in_ptrs = np.array([[rows[k][l].data_ptr() for l in ls] for k in range(K)], dtype=np.int64)
        out_ptrs = np.array([outs[l].data_ptr() for l in ls], dtype=np.int64)
        narrow = _narrow(K, leaf_n, in_c) and l2sq is None
        svar = 0
        if narrow:
            # k_ptrs_stripe when every pointer is 16-byte aligned (k_ptrs_narrow otherwise)
            if _STRIPE_PYTREE and K >= 512 and not ((in_ptrs & 15).any() or (out_ptrs & 15).any()):
                svar = _stripe_variant_for(leaf_n, device)
            blocks, unaligned = _ptrs_plan(in_c, leaf_n, ("narrow", svar), device), False
        else:
            blocks, unaligned = _leaf_plan(in_c, leaf_n, in_ptrs, out_ptrs, device)
        if packed is not None:
            w_host = packed.i32 if acc_c == _lib.I32 else packed.f32
        elif acc_c != _lib.I32:  # F32, or BF16 (the kernel rounds each f32 weight to bf16)
            w_host = np.array([np.float32(w) for w in weights], dtype=np.float32)
        else:
            w_host = np.array([np.int64(w) for w in weights], dtype=np.int64).astype(np.int32)
        w_words = np.zeros((K + 1) // 2, dtype=np.int64)
        w_words.view(np.uint8)[: 4 * K] = w_host.view(np.uint8)
        image = np.concatenate([in_ptrs.ravel(), out_ptrs, leaf_n, blocks, w_words])
        image_dev = _lib.upload(torch.from_numpy(image), device)
        w_dev_ptr = image_dev.data_ptr() + 8 * (image.size - w_words.size)
        total_bytes = int(leaf_n.sum()) * K * (2 if in_c == _lib.BF16 else 4)
        nt = (total_bytes >= NONTEMPORAL_MIN_BYTES) if nontemporal is None else nontemporal
        flags = (_lib.SCALE if scale is not None else 0) | (_lib.ACCUMULATE if accumulate else 0)
        flags |= (_lib.UNALIGNED if unaligned else 0) | (_lib.NONTEMPORAL if nt else 0)
        flags |= (_lib.NARROW | ((svar & 0xFF) << 8)) if narrow else 0
        nblk = len(blocks) // 2
        sc = float(np.float32(scale) if scale is not None else 1.0)
        stream = torch.cuda.current_stream(device).cuda_stream
        if l2sq is None:
            _lib.call("fjagg_wsum_ptrs", in_c, acc_c, out_c, image_dev.data_ptr(), len(ls), K, nblk,
                      w_dev_ptr, sc, flags, stream)
        else:
            need = int(_lib.load().fjagg_wsum_l2_ptrs_workspace_bytes(K, nblk))
            ws = torch.empty(max(need, 4), dtype=torch.uint8, device=device)
            _lib.call("fjagg_wsum_l2_ptrs", in_c, acc_c, out_c, image_dev.data_ptr(), len(ls), K, nblk,
                      w_dev_ptr, sc, l2sq.data_ptr(), flags, ws.data_ptr(), ws.numel(), stream)
    return outs


_ENTRY_ADDRS = None  # (plan_leaves, wsum_ptrs, wsum_l2_ptrs, l2 workspace bytes) addresses for fjhost.fold_table


_FILL_ADDR = 0  # fjtree_norms_fill, for fjhost.fold_chain's lazy-norm fill
_ROWS_ADDR = 0  # fjagg_wsum_l2_ptrs_rows: fjhost.fold_chain's norms straight into a chain's norm rows


def _native_fold_addrs() -> None:
    global _ENTRY_ADDRS, _FILL_ADDR, _ROWS_ADDR
    lib = _lib.load()
    _ENTRY_ADDRS = tuple(ctypes.cast(getattr(lib, f), ctypes.c_void_p).value
                         for f in ("fjagg_ptrs_plan_leaves", "fjagg_wsum_ptrs", "fjagg_wsum_l2_ptrs",
                                   "fjagg_wsum_l2_ptrs_workspace_bytes"))
    _FILL_ADDR = ctypes.cast(lib.fjtree_norms_fill, ctypes.c_void_p).value
    _ROWS_ADDR = ctypes.cast(lib.fjagg_wsum_l2_ptrs_rows, ctypes.c_void_p).value
    _mean_config()
    _solo_config()


def set_nontemporal_min_bytes(nbytes: int) -> None:
    """Folds whose client deltas total at least ``nbytes`` use non-temporal loads (default
    256 MiB, the Infinity Cache's size: :data:`NONTEMPORAL_MIN_BYTES`). Sets the module value
    and the builtin tree_mean's copy of it together."""
    global NONTEMPORAL_MIN_BYTES
    NONTEMPORAL_MIN_BYTES = int(nbytes)
    _mean_config()


def _mean_config() -> None:
    """Configure the builtin tree_mean (fjhost.tree_mean / mean_triples): the same settings
    _native_mean passes, the library's entry points once loaded (until then the builtin
    calls the Python function, which loads them), and the Python fallbacks."""
    on = _NATIVE_MEAN and _ENTRY_ADDRS is not None
    _HOST.mean_config(on, _PIPELINE_FRAC, _PIPELINE_CHUNK, _CHUNK_WALK_US, _WALK_NS_PER_LEAF, _PIPELINE_MIN_BYTES,
                      _NARROW_MAX_BYTES, float(NONTEMPORAL_MIN_BYTES), _PEAK_BYTES_PER_S,
                      _ENTRY_ADDRS[0] if on else 0, _ENTRY_ADDRS[1] if on else 0, _tree_mean_py, _mean_triples_py,
                      _BUSY_UNTIL[0])


def _native_fold(table: "_Table", packed: "_Weights", scale, out=None,
                 accumulate: bool = False, l2sq: Optional[torch.Tensor] = None) -> Optional[List[torch.Tensor]]:
    """The common case of :func:`_fold` in one native call (fjhost.fold_table): float32
    leaves, Python-number weights, fresh outputs or the caller's float32 ``out`` leaves
    (``accumulate`` folds into them; misaligned leaves get the per-leaf plan); with ``l2sq``
    also every client's squared l2 norm (fjagg_wsum_l2_ptrs). It builds the same plan
    image and launches the same kernel as the Python path below; None when the case does
    not hold (nothing launched)."""
    if _ENTRY_ADDRS is None:
        _native_fold_addrs()
    dev = table.row0[0].device
    if dev.type != "cuda":
        return None
    sc = float(np.float32(scale)) if scale is not None else 1.0
    got = _lib.host().fold_table(table.row0, table.ptrs, packed.f32, sc, scale is not None,
                                 float(NONTEMPORAL_MIN_BYTES), dev.index, torch.cuda.current_stream(dev).cuda_stream,
                                 _ENTRY_ADDRS[0], _ENTRY_ADDRS[1], list(out) if out is not None else None,
                                 1 if accumulate else 0, _ENTRY_ADDRS[2], _ENTRY_ADDRS[3], l2sq)
    if got is None:
        return None
    rc, outs = got
    _lib.check(rc, "fjagg_wsum_ptrs")
    return outs


_PLANS = {}  # (in dtype, leaf sizes, unaligned) -> workgroup table (the device is fixed per process)


# A small client delta and many clients: the LDS-staged stripes of k_ptrs_narrow keep more
# loads in flight than 16-byte units spread over the few lanes a narrow tree has. Up to
# 256 KiB per client (a 48.7 K-param model at 1,024-4,096 clients: 0.44 -> 0.33 ms); at
# ~430 KiB the balanced 16-byte plan is as fast or faster (profiles/r02k_narrow_pytree.txt).
_NARROW_MAX_BYTES = int(os.environ.get("FJAGG_NARROW_MAX_BYTES", 256 << 10))  # 0: never (A/B runs)


def _narrow(K: int, leaf_n: np.ndarray, in_c: int) -> bool:
    return K >= 16 and int(leaf_n.sum()) * (2 if in_c == _lib.BF16 else 4) <= _NARROW_MAX_BYTES


# Narrow plans over 16-byte aligned leaves run the stripe pipeline (k_ptrs_stripe,
# fjstripe.hip) instead of k_ptrs_narrow; FJAGG_STRIPE_PYTREE=0 keeps k_ptrs_narrow (A/B).
_STRIPE_PYTREE = os.environ.get("FJAGG_STRIPE_PYTREE", "1") != "0"
_CUS = {}


def _stripe_variant_for(leaf_n: np.ndarray, device: torch.device) -> int:
    """FJAGG_VARIANT of the stripe width for these leaves (kernels.stripe_variant over the
    stripes of every leaf: each leaf starts a new stripe)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    cus = _CUS.get(idx)
    if cus is None:
        cus = _CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    for v, c in ((20, 64), (21, 32)):
        if int(((leaf_n + c - 1) // c).sum()) >= cus:
            return v
    return 22


def _ptrs_plan(in_c: int, leaf_n: np.ndarray, unaligned, device: torch.device) -> np.ndarray:
    """Cached :func:`kernels.ptrs_plan`; ``unaligned`` is a bool, a per-leaf mask,
    "narrow" (the k_ptrs_narrow stripes) or ("narrow", v) (v = 20 / 21 / 22: the
    k_ptrs_stripe stripes; 0: k_ptrs_narrow's)."""
    key = (in_c, leaf_n.tobytes(), unaligned if isinstance(unaligned, (bool, str, tuple)) else
           np.asarray(unaligned, dtype=np.uint8).tobytes(), device)
    blocks = _PLANS.get(key)
    if blocks is None:
        if isinstance(unaligned, tuple):  # ("narrow", stripe variant or 0)
            blocks = kernels.ptrs_plan(in_c, leaf_n, False, narrow=True, stripe_variant=unaligned[1])
        elif isinstance(unaligned, str):
            blocks = kernels.ptrs_plan(in_c, leaf_n, False, narrow=True)
        else:
            blocks = kernels.ptrs_plan(in_c, leaf_n, unaligned)
        if len(_PLANS) < 1024:
            _PLANS[key] = blocks
    return blocks


def _leaf_plan(in_c: int, leaf_n: np.ndarray, in_ptrs: np.ndarray, *more_ptrs) -> tuple:
    """Plan for a [K, L] table of client leaf pointers plus per-leaf output pointers
    (``more_ptrs``: [L] or [m, L] int64 arrays, then the device). Leaves whose pointers
    are not all 16-byte aligned walk element units; the others keep 16-byte units
    (fjagg_ptrs_plan_leaves). Returns (blocks, launch-wide UNALIGNED flag) — the flag is
    never needed now that the choice is per leaf, so it is always False."""
    *arrs, device = more_ptrs
    bits = np.bitwise_or.reduce(in_ptrs, axis=0) if in_ptrs.shape[0] else np.zeros(len(leaf_n), np.int64)
    for a in arrs:
        a = np.asarray(a, dtype=np.int64).reshape(-1, len(leaf_n))
        bits = bits | np.bitwise_or.reduce(a, axis=0)
    bad = (bits & 15) != 0
    return _ptrs_plan(in_c, leaf_n, bad if bad.any() else False, device), False


class _Table:
    """K clients' leaves as client 0's canonical device leaves + an int64 [K, L] table of
    every client's leaf pointers (built natively by fjhost.gather_rows)."""

    __slots__ = ("row0", "ptrs")

    def __init__(self, row0: List[torch.Tensor], ptrs: np.ndarray):
        self.row0, self.ptrs = row0, ptrs

    def __len__(self):
        return self.ptrs.shape[0]

    def __getitem__(self, k):
        """``rows[0]`` is client 0's leaves in both representations; other clients exist
        only as pointers (:func:`_ptr_table`)."""
        if k != 0:
            raise TypeError("a _Table holds client 0's leaves only; use _ptr_table for the others")
        return self.row0


def _ptr_table(rows, dtype=np.int64) -> np.ndarray:
    """[K, L] leaf pointers of rows (a _Table or K lists of leaves)."""
    if isinstance(rows, _Table):
        return rows.ptrs if dtype == np.int64 else rows.ptrs.astype(dtype)
    return np.array([[x.data_ptr() for x in r] for r in rows], dtype=dtype)


class _Weights:
    """Weights that were all Python numbers, packed by fjhost.fold_weights: float32 and
    int32 vectors, their weak-type kinds, and W summed as tree_util.py:86,95 does."""

    __slots__ = ("f32", "i32", "kinds", "total")

    def __init__(self, f32, i32, kinds, total):
        self.f32, self.i32, self.kinds, self.total = f32, i32, kinds, total


def _pack_weights(weights: List[Any]) -> Optional[_Weights]:
    """_Weights of ``weights`` when they are all Python int / float, else None."""
    K = len(weights)
    f32, i32 = np.empty(K, dtype=np.float32), np.empty(K, dtype=np.int32)
    got = _lib.host().fold_weights(weights, f32, i32)
    if got is None:
        return None
    total, bits = got
    kinds = ([_WEAK_FLOAT] if bits & 1 else []) + ([_WEAK_INT] if bits & 2 else [])
    return _Weights(f32, i32, kinds, total)


def _client_table(trees: Sequence[PyTree], first=None):
    """(treedef, rows) like :func:`_client_rows`; rows is a :class:`_Table` when every
    client's leaves are already contiguous device tensors of client 0's dtypes and
    shapes on client 0's device (the common case, checked natively), else lists.
    ``first``: pytree.flatten(trees[0]) when already computed."""
    leaves0, td = pytree.flatten(trees[0]) if first is None else first
    device = _find_device(leaves0)
    idx = _device_index(device)
    row0 = [_device_leaf(x, device, idx) for x in leaves0]
    spec = pytree.native_spec(td) if row0 else None
    if spec is not None:
        ptrs = np.empty((len(trees), len(row0)), dtype=np.int64)
        if _lib.host().gather_rows(trees if type(trees) is list else list(trees), 1, spec, row0, idx, ptrs) == 0:
            return td, _Table(row0, ptrs)
    return _client_rows(trees, (leaves0, td, row0))


def _check_row(k: int, row: List[torch.Tensor], sig0) -> None:
    for l, x in enumerate(row):
        if x.size() != sig0[l][0]:
            raise ValueError(f"leaf {l}: client {k} has shape {tuple(x.shape)}, "
                             f"client 0 has {tuple(sig0[l][0])}")
        if x.dtype != sig0[l][1]:
            raise TypeError(f"leaf {l}: client {k} has dtype {x.dtype}, client 0 has {sig0[l][1]}")


def _client_rows(trees: Sequence[PyTree], first=None) -> Tuple[pytree.TreeDef, List[List[torch.Tensor]]]:
    """Flatten every client's pytree into canonical device leaves, checking that all
    clients match client 0's structure, leaf shapes and dtypes (what _fold assumes).
    ``first``: (leaves, treedef, canonical leaves) of client 0 when already computed."""
    dl, T, flat = _device_leaf, torch.Tensor, pytree.flatten_as
    if first is None:
        leaves0, td = pytree.flatten(trees[0])
        device = _find_device(leaves0)
        row0 = [dl(x, device, _device_index(device)) for x in leaves0]
    else:
        leaves0, td, row0 = first
        device = row0[0].device if row0 else _find_device(leaves0)
    idx = _device_index(device)
    rows = [row0]
    dt0 = [x.dtype for x in row0]
    sz0 = [x.size() for x in row0]
    for k in range(1, len(trees)):
        r = flat(td, trees[k])
        # the common case in one pass per (client, leaf): already a contiguous device tensor
        # of client 0's dtype and shape (_device_leaf's fast path + _fold's signature check)
        if not all([type(x) is T and x.dtype is d and x.get_device() == idx and x.is_contiguous() and x.size() == s
                    for x, d, s in zip(r, dt0, sz0)]):
            r = [dl(x, device, idx) for x in r]
            _check_row(k, r, list(zip(sz0, dt0)))
        rows.append(r)
    return td, rows


# ------------------------------------------------------------------------ public API
def _fold_trees(trees: Sequence[PyTree], weights: List[Any]) -> PyTree:
    """Fold of whole pytrees with host weights: the native table and weight packing
    (fjhost) when they apply, the Python fold otherwise (same kernel, same bits)."""
    td, rows = _client_table(trees)
    if not rows[0]:
        return pytree.unflatten(td, [])
    packed = _pack_weights(weights)
    return pytree.unflatten(td, _fold(rows, packed if packed is not None else [_host_weight(w) for w in weights],
                                      validated=True))


# ------------------------------------------------------- per-call tree ops (fjtree.h)
# The running-sum loop of FedJAX's algorithms (fedjax/algorithms/fed_avg.py:132-146 and
# six others) calls tree_add(s, tree_weight(delta, n)) and tree_l2_norm(delta) once per
# client. For pytrees of float32 device tensors (<= 64 leaves) each call is ONE launch of
# fjtree_fold_leaves with the leaf table in the kernel arguments (fjhost.leaf_fold):
# tree_weight is deferred (WeightedTree) and folded into the tree_add that consumes it,
# and that launch also sums the squares of the weighted delta, which tree_l2_norm of the
# same, unmodified delta then returns without another pass.
_TREE_ADDRS = None
_STALE = -100  # fjhost.leaf_fold: a captured operand changed since tree_weight
_NORMS: "collections.deque" = None  # (capture, l2sq, l2) of the last fused tree_add calls


def _tree_addrs():
    global _TREE_ADDRS, _NORMS
    if _TREE_ADDRS is None:
        import collections
        lib = _lib.load()
        _NORMS = collections.deque(maxlen=2)
        _TREE_ADDRS = tuple(ctypes.cast(getattr(lib, f), ctypes.c_void_p).value
                            for f in ("fjtree_fold_leaves", "fjtree_workspace_bytes"))
    return _TREE_ADDRS


# How the per-call norm's workgroup partials are ordered before the last workgroup reads
# them (include/fjtree.h): "handoff" = write-through partials drained before
# a relaxed counter add (gfx950's hand-off form, the default); "ordered" = an acquire-release
# counter add (HIP memory model; a whole-L2 write-back per workgroup). Same bits either way.
_NORM_COMBINE = os.environ.get("FJTREE_NORM_COMBINE", "handoff")


def set_norm_combine(mode: str) -> None:
    """Select the cross-workgroup ordering of the per-call fused norm: ``"handoff"``
    (default) or ``"ordered"`` (release/acquire atomics, FJTREE_ORDERED)."""
    global _NORM_COMBINE
    if mode not in ("handoff", "ordered"):
        raise ValueError("norm combine is 'handoff' or 'ordered'")
    _NORM_COMBINE = mode


def _leaf_fold(trees, weights, caps, scale=None, norm_operand=-1, no_out=False):
    """fjhost.leaf_fold: (out_tree, l2sq, l2) from one fjtree launch; None when the call
    is not the fast case (nothing launched). Raises when a captured operand is stale."""
    fold, ws = _TREE_ADDRS or _tree_addrs()
    flags = ((_lib.SCALE if scale is not None else 0) | (_lib.TREE_NORM if norm_operand >= 0 else 0)
             | (_lib.TREE_NO_OUT if no_out else 0)
             | (_lib.TREE_ORDERED if norm_operand >= 0 and _NORM_COMBINE == "ordered" else 0))
    got = _lib.host().leaf_fold(trees, weights, caps, 1.0 if scale is None else float(scale), flags,
                                max(norm_operand, 0), -1, 0, fold, ws)
    if got is None:
        return None
    rc, out, sq, l2 = got
    if rc == _STALE:
        raise RuntimeError("a pytree passed to tree_weight was modified (a leaf replaced or updated in "
                           "place) before its weighted value was used; the reference computes "
                           "tree_weight eagerly")
    _lib.check(rc, "fjtree_fold_leaves")
    return out, sq, l2


_HOST = _lib.host()  # the _fjhost module: native walks, and the base types of the lazy results below


class WeightedTree(_HOST.WeightedBase):
    """``tree_weight(tree, w)`` of a pytree of float32 device tensors, not yet computed.

    The multiply is deferred so that ``tree_add(s, tree_weight(x, n))`` — the running sum
    of fed_avg.py:137-138 — is one fused launch (bitwise ``fl(s + fl(x * f32(n)))``). Any
    other use computes it: indexing, iteration, attribute access and every pytree walk of
    this package (``pytree.flatten``, ``tree_util.*``) see the weighted pytree itself, and
    ``materialize()`` returns it. The input's leaf objects and their in-place versions are
    captured at ``tree_weight``. A deferred running sum (``tree_add`` into a sum of the
    same structure) takes the captured leaves, so a leaf replaced in the input afterwards
    does not change the sum — the value the reference's eager tree_weight computed; a
    captured leaf modified in place makes the sum's fold raise RuntimeError. Any other use
    (including ``tree_add`` with deferral off)
    raises RuntimeError when a leaf was replaced or modified in between (the reference's
    arrays are immutable).
    The guard is torch's in-place version counter: writes that bypass it (through
    ``tensor.data``, or by native code writing the tensor's memory) are not seen, and the
    deferred multiply then reads the new values. Inference tensors, which have no version
    counter, are weighted eagerly.
    ``isinstance(w, dict)`` is False: call ``materialize()`` where the concrete container
    type matters.
    """

    __slots__ = ()  # fields _tree, _weight, _cap, _value: fjhost's WeightedBase

    def __init__(self, tree, weight, cap):
        self._tree, self._weight, self._cap, self._value = tree, weight, cap, None

    def materialize(self) -> PyTree:
        if self._value is None:
            from fedjax_amd import memory
            with memory.producing(self._cap[0][0].device if memory.default_enabled() else None):
                got = _leaf_fold([self._tree], [self._weight], [self._cap])
            if got is None:
                raise RuntimeError("the pytree passed to tree_weight changed structure before use")
            self._value = got[0]
            self._tree = self._cap = None
        return self._value

    def __getitem__(self, key):
        return self.materialize()[key]

    def __iter__(self):
        return iter(self.materialize())

    def __len__(self):
        return len(self.materialize())

    def __contains__(self, key):
        return key in self.materialize()

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return getattr(self.materialize(), name)

    def __repr__(self):
        return f"WeightedTree({self.materialize()!r})"

    # pickled and copied as the pytree it stands for (the reference's tree_weight / tree_add
    # return plain pytrees): the capture and the chain stay behind
    def __reduce_ex__(self, proto):
        return copy.copy, (self.materialize(),)  # (unpickled without fedjax_amd)

    def __deepcopy__(self, memo):
        return copy.deepcopy(self.materialize(), memo)

    def __copy__(self):
        return copy.copy(self.materialize())


pytree.register_lazy_type(WeightedTree, WeightedTree.materialize)
_F32_EXACT_INT = 1 << 53

# Deferred running sums (PendingSum): on by default; see set_deferred_sums.
# budget_bytes None = automatic: min(4 GiB, 1/8 of the device's free memory when the
# process first defers a sum on it), see _defer_budget
_DEFER = {"enabled": True, "budget_bytes": None, "max_clients": 4095,
          # fold the pending part early once it holds this much in >= flush_clients links: that
          # launch runs while the caller's loop goes on, and fewer deltas stay referenced. With
          # the native chain fold a flush costs ~10-25 us of host time; at configs[1] (about 4.8
          # MB per client) a flush at 256 MiB takes a synchronised round 0.21 -> 0.17 ms with
          # rounds back to back unchanged (profiles/r04p_flush/host.json). Each flush also reads
          # and writes the running sum once more: where the GPU bounds the loop (configs[2]'s
          # 16 MiB clients) a flush every 16 clients costs 17 % (2.60 -> 3.08 ms per round), one
          # every >= 64 clients ~1.5 % (profiles/r04q_check/flush_large.json) — hence 64
          "flush_bytes": 256 << 20, "flush_clients": 64}
_AUTO_BUDGET = {}  # device index -> automatic budget in bytes


def set_deferred_sums(enabled: bool = True, *, budget_bytes: Optional[int] = None,
                      max_clients: Optional[int] = None, flush_bytes: Optional[int] = None,
                      flush_clients: Optional[int] = None) -> None:
    """Configure how ``tree_add(s, tree_weight(x, n))`` runs.

    Enabled (default): the sum is deferred (:class:`PendingSum`) and folded by ONE
    pytree-kernel launch when it is used, at most ``budget_bytes`` of pending deltas or
    ``max_clients`` (<= 4095) clients per launch (an older part of the chain is folded
    first when a limit would be passed, so memory stays bounded). Once the pending part
    holds >= 256 MiB of deltas in >= 64 clients it is folded at the next ``tree_add``
    (``flush_bytes`` / ``flush_clients``): that launch overlaps the rest of the caller's
    loop, and the deltas it covers are released. Any split gives the same bits. Disabled: every call is
    one fused launch (fjtree_fold_leaves), which also suits loops that update delta
    tensors in place between clients. Both give the reference's bits.

    Memory: a deferred chain keeps its clients' deltas alive until its fold, where the
    reference's loop frees each delta after its ``tree_add`` (tree_util.py:85-96). The
    default budget is therefore min(4 GiB, 1/8 of the device memory free when the process
    first defers a sum there), per chain; a loop that keeps several running sums at once
    holds up to that much per sum — pass a smaller ``budget_bytes`` (or disable deferral)
    on a device close to full. ``budget_bytes=0`` restores the automatic value. A new
    budget applies to running sums started after the call.

    Semantics: deferral holds each delta by reference, guarded by torch's in-place
    version counter (a modified delta makes the fold raise). Writes that bypass that
    counter — ``tensor.data`` writes, native code or kernels writing the memory — are not
    detected, and the deferred fold reads the new values: loops that write deltas that
    way must disable deferral."""
    _DEFER["enabled"] = bool(enabled)
    if budget_bytes is not None:
        _DEFER["budget_bytes"] = int(budget_bytes) if int(budget_bytes) > 0 else None
    if max_clients is not None:
        _DEFER["max_clients"] = min(4095, max(1, int(max_clients)))
    if flush_bytes is not None:
        _DEFER["flush_bytes"] = max(0, int(flush_bytes))
    if flush_clients is not None:
        _DEFER["flush_clients"] = max(1, int(flush_clients))
    _HOST.fast_config(_DEFER["enabled"], _DEFER["max_clients"], _DEFER["flush_bytes"], _DEFER["flush_clients"])
    _HOST.drop_pool()  # (the lazy-norm pool's buffer is sized by max_clients)


# Standalone lazy norms (fjhost.cpp "standalone lazy norms"): tree_l2_norm(delta) of a delta no
# running sum took — examples/fed_avg.py:79-81, before the tree_mean of :82 — is a lazy view
# whose value the tree_mean launch folding that delta writes. budget_bytes None = automatic (the
# deferred sums' budget): past it, or past max_pending views, the oldest are computed at once.
_LAZY = {"enabled": os.environ.get("FJAGG_LAZY_NORMS", "1") != "0", "budget_bytes": None, "max_pending": 16383}


def set_lazy_norms(enabled: bool = True, *, budget_bytes: Optional[int] = None,
                   max_pending: Optional[int] = None) -> None:
    """Configure ``tree_l2_norm`` / ``tree_l2_squared`` of a float32 device pytree that no
    deferred running sum just took (examples/fed_avg.py:79-81 takes the norm of each client's
    delta before the round's ``tree_mean``, :82).

    Enabled (default, with deferred sums on): the call returns a lazy 0-d view and holds the
    delta's leaves; a later ``tree_mean`` / ``mean_aggregator().apply`` that folds the same,
    unmodified pytree writes the norm from the same pass over the delta (so the round reads
    each delta once). Reading the view first (any torch function or method, ``float``,
    ``print``), or a delta no mean folds, computes it with its own launch of the same kernel:
    the value does not depend on when it is read (f32 sum of squares in a fixed order,
    DESIGN.md §4). At most ``max_pending`` norms (default 16383) wait at once, past which all
    are computed; once the waiting deltas pass ``budget_bytes`` (default: the deferred sums'
    budget), those whose pytree only the lazy norm still holds are computed (checked again
    after every further quarter budget), so the views never keep much more than that alive on
    their own. A delta leaf
    updated in place before its norm is computed makes reading the view raise RuntimeError
    (the value at the call is gone); writes that bypass torch's version counter are not
    detected, as for deferred sums. Disabled (or ``set_deferred_sums(False)``): every call
    computes at once, as the reference does."""
    _LAZY["enabled"] = bool(enabled)
    if budget_bytes is not None:
        _LAZY["budget_bytes"] = int(budget_bytes) if int(budget_bytes) > 0 else None
    if max_pending is not None:
        _LAZY["max_pending"] = max(1, min(1 << 20, int(max_pending)))
    _solo_config()


def _solo_budget(dev: int) -> int:
    return _defer_budget(torch.device("cuda", dev))


def _solo_config() -> None:
    """set_lazy_norms' settings and the library's entry points, into fjhost (once loaded)."""
    if _ENTRY_ADDRS is None:
        _HOST.solo_config(_LAZY["enabled"], _LAZY["max_pending"], _LAZY["budget_bytes"] or 0, 0, 0, 0, _solo_budget)
        return
    _HOST.solo_config(_LAZY["enabled"], _LAZY["max_pending"], _LAZY["budget_bytes"] or 0, _ROWS_ADDR,
                      _ENTRY_ADDRS[3], _ENTRY_ADDRS[0], _solo_budget)


def _defer_budget(device: torch.device) -> int:
    """Bytes of deltas one deferred chain may hold on ``device`` (see set_deferred_sums)."""
    b = _DEFER["budget_bytes"]
    if b is not None:
        return b
    idx = device.index if device.index is not None else torch.cuda.current_device()
    got = _AUTO_BUDGET.get(idx)
    if got is None:
        free, _ = torch.cuda.mem_get_info(idx)
        got = _AUTO_BUDGET[idx] = int(min(4 << 30, max(64 << 20, free // 8)))
    return got


class _Chain(_HOST.ChainBase):
    """The linear run of PendingSum links one norm buffer serves: float32 [2, n] on the
    device, row 0 = squared l2 norms, row 1 = l2 norms of the clients, by link index."""

    __slots__ = ()  # fields tip, buf, budget: fjhost's ChainBase

    def __init__(self):
        self.tip, self.buf, self.budget = None, None, None  # budget: _defer_budget, on first use


class _Ticket:
    """What a lazy norm view needs to get its value: the link whose fold writes it
    (dropped once written, so views never keep client deltas alive)."""

    __slots__ = ("node",)

    def __init__(self, node):
        self.node = node


class _NormView(torch.Tensor):
    """0-d float32 l2 norm (or its square) of a client delta added to a deferred sum: a
    view into the chain's norm buffer, written by the chain's fold. Every torch function
    or method that touches it (``float(v)``, ``v.item()``, ``print(v)``, ``torch.stack``,
    arithmetic) first runs that fold if it has not run, then computes on plain tensors —
    so no read can see the buffer before the value is there."""

    __slots__ = ("_ticket",)  # (no per-view __dict__: fjhost sets the slot through its descriptor)

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        _HOST.flush_views(args)
        if kwargs:
            _HOST.flush_views(kwargs)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **(kwargs or {}))

    def __format__(self, spec):
        _HOST.flush_views(self)
        with torch._C.DisableTorchFunctionSubclass():
            return self.item().__format__(spec) if self.dim() == 0 else torch.Tensor.__format__(self, spec)

    def _value(self) -> torch.Tensor:
        """The value as a plain tensor of its own (computed first if pending): no ticket and no
        view of the norm buffer."""
        _HOST.flush_views(self)
        with torch._C.DisableTorchFunctionSubclass():
            return self.detach().clone()

    def __reduce_ex__(self, proto):
        # pickled (torch.save, multiprocessing, copy.copy) as its value, as the reference's jnp
        # scalar is: a capture's node cannot travel, and the view would carry the whole buffer
        return torch.Tensor.__reduce_ex__(self._value(), proto)

    def __deepcopy__(self, memo):
        return self._value()


def _fold_ticket(ticket) -> None:
    """Fold the chain a waiting lazy norm's ticket names (fjhost.flush_views calls this); a
    standalone norm's ticket (a SoloNorm node) is computed by its own launch."""
    if type(ticket) is _HOST.SoloNorm:
        _HOST.solo_resolve([ticket])
    elif ticket.node is not None:
        ticket.node._chain.tip.materialize()  # folds every pending link of the chain


def _flush_views(x) -> None:
    """The Python statement of fjhost.flush_views (which the views use)."""
    t = type(x)
    if t is _NormView:
        ticket = getattr(x, "_ticket", None)
        if type(ticket) is _HOST.SoloNorm:
            if ticket.node is not None:
                _HOST.solo_resolve([ticket])  # (raises for a stale one)
        elif ticket is not None and ticket.node is not None:
            ticket.node._chain.tip.materialize()  # folds every pending link of the chain
    elif t is list or t is tuple:
        for y in x:
            _flush_views(y)
    elif t is dict:
        for y in x.values():
            _flush_views(y)


class PendingSum(_HOST.PendingBase):
    """``s = tree_add(s, tree_weight(x, n))`` repeated over clients, not yet computed.

    FedJAX's algorithms build the round's running sum this way, one client at a time
    (fedjax/algorithms/fed_avg.py:132-146). Each ``tree_add`` here appends the client's
    delta (its leaves, captured at ``tree_weight``) and weight to a chain in O(1) host
    work; the chain is folded when the sum is used — by ``tree_inverse_weight`` (which
    also applies the ``1/W`` scale in the same launch), by indexing, iteration, attribute
    access, ``materialize()`` or any pytree walk of this package. The fold is the pytree
    kernel over [base, x_1 .. x_k] with weights [1, n_1 .. n_k]: per element
    ``fl(...fl(fl(base*1) + fl(x_1 n_1)) ... + fl(x_k n_k))``, the reference's sequence of
    ``jnp.add`` calls, bit for bit. ``tree_l2_norm(x)`` of the delta just added returns a
    lazy view whose value the same fold computes (fjagg_wsum_l2_ptrs): the per-client
    ``delta_l2_norm`` of fed_avg.py:142-144 without another pass over the delta.

    The deltas stay referenced until the fold (bounded by :func:`set_deferred_sums`). A
    delta modified in place after its tree_weight makes the fold raise RuntimeError (the
    reference's arrays are immutable); loops that reuse delta buffers should call
    ``set_deferred_sums(False)``. The check is torch's in-place version counter, so a
    write that bypasses it — through ``tensor.data``, or by native code / a kernel writing
    the tensor's memory — is NOT detected: the fold then sums the new values where the
    reference summed the old ones. Such loops must use ``set_deferred_sums(False)`` (or add
    copies). Inference tensors have no version counter and are never deferred. ``isinstance(s, dict)`` is False: call
    ``materialize()`` where the concrete container type matters.
    """

    # fields _root, _parent, _cap, _weight, _n, _bytes, _value, _chain, _idx, _ticket, _ref, _bcap,
    # _tok and weak-reference support: fjhost's PendingBase (fjhost.tree_add builds links natively)
    __slots__ = ()

    def __init__(self, root, parent, cap, weight, ref, bcap=None, tok=-1):
        self._root, self._parent, self._cap, self._weight, self._value = root, parent, cap, weight, None
        self._ref = ref  # a tree with the sum's structure (the chain's base): O(1) structure checks
        self._bcap = bcap  # capture of the base tree when this link starts a run (parent not pending)
        self._tok = tok  # the sum's structure token (fjhost.capture), -1 if unknown
        self._ticket = None
        live = parent is not None and parent._value is None
        self._n = 1 + (parent._n if live else 0)
        self._bytes = cap[2] + (parent._bytes if live else 0)
        if parent is not None and parent._chain.tip is parent and (
                live or (parent._chain.buf is not None and parent._idx + 1 < parent._chain.buf.shape[1])):
            # (a parent folded early — an early flush, or a bounded chain — keeps its chain when
            # the chain's norm buffer has room: the next lazy norm needs no new buffer)
            self._chain, self._idx = parent._chain, parent._idx + 1
        else:
            self._chain, self._idx = _Chain(), 0
        self._chain.tip = self

    def _links(self):
        """(base tree, the unfolded links from the nearest folded ancestor, in order)."""
        links = []
        p = self
        while p is not None and p._value is None:
            links.append(p)
            if p._parent is None:
                base = p._root
            p = p._parent
        if p is not None:
            base = p._value
        links.reverse()
        return base, links

    def materialize(self) -> PyTree:
        if self._value is None:
            self._value = _fold_pending(self, None)
            self._root = self._parent = self._cap = self._ref = self._bcap = None  # the deltas can go
        return self._value

    __getitem__ = WeightedTree.__getitem__
    __iter__ = WeightedTree.__iter__
    __len__ = WeightedTree.__len__
    __contains__ = WeightedTree.__contains__
    __getattr__ = WeightedTree.__getattr__
    __reduce_ex__ = WeightedTree.__reduce_ex__
    __deepcopy__ = WeightedTree.__deepcopy__
    __copy__ = WeightedTree.__copy__

    def __repr__(self):
        return f"PendingSum({self.materialize()!r})"


pytree.register_lazy_type(PendingSum, PendingSum.materialize)


_FOLD_CAPS = os.environ.get("FJAGG_FOLD_CAPS", "1") != "0"  # 0: the Python path below (A/B runs)


def _fold_pending(node: "PendingSum", scale):
    """The fold of a PendingSum's unfolded links [* f32(scale)]: fjhost.fold_chain walks the
    links natively and folds them in one launch (fold_caps); when a lazy norm waits on a
    link, or the run has no captured base, the Python walk below (_fold_chain) does it."""
    if _FOLD_CAPS:
        if _ENTRY_ADDRS is None:
            _native_fold_addrs()
        got = _HOST.fold_chain(node, float(np.float32(scale)) if scale is not None else 1.0, scale is not None,
                               float(NONTEMPORAL_MIN_BYTES), *_ENTRY_ADDRS, _FILL_ADDR, _ROWS_ADDR)
        if type(got) is int:
            _stale_chain(got)
        if got is not None:
            rc, tree = got
            _lib.check(rc, "fjagg_wsum_ptrs")
            return tree
    base, links = node._links()
    return _fold_chain(base, links, scale)


def _fold_chain(base, links, scale):
    """fl(...fl(fl(base*1) + fl(x_1 w_1)) ... + fl(x_k w_k)) [* f32(scale)]: one pytree-kernel
    launch over the base tree's leaves and the captured leaves of every link; with the
    per-client squared norms from the same pass when a lazy norm view waits on a link.
    A captured base (the common case) goes through one native call (fjhost.fold_caps: the
    version checks, the pointer table, the launch and the result tree)."""
    bcap = links[0]._bcap
    if _FOLD_CAPS and bcap is not None:
        waiting = [n for n in links if n._ticket is not None and n._ticket.node is not None]
        l2sq = None
        if waiting:
            l2sq = torch.empty(1 + len(links), dtype=torch.float32, device=bcap[0][0].device)
        if _ENTRY_ADDRS is None:
            _native_fold_addrs()
        sc = float(np.float32(scale)) if scale is not None else 1.0
        got = _HOST.fold_caps(base, [bcap] + [n._cap for n in links], [1] + [n._weight for n in links], sc,
                              scale is not None, float(NONTEMPORAL_MIN_BYTES), *_ENTRY_ADDRS, l2sq)
        if type(got) is int:
            _stale_chain(got)
        if got is not None:
            rc, tree = got
            _lib.check(rc, "fjagg_wsum_ptrs")
            if waiting:
                _fill_norms(links, waiting, l2sq)
            return tree
    leaves0, td = pytree.flatten(base)
    L = len(leaves0)
    caps = [n._cap for n in links]
    ptrs = np.empty((1 + len(caps), L), dtype=np.int64)
    bcap = links[0]._bcap
    if bcap is not None:
        # the base as it was at the first tree_add: its captured leaves, checked unmodified
        if len(bcap[0]) != L:
            bad = 0
        else:
            leaves0 = list(bcap[0])
            bad = _lib.host().table_from_caps([bcap] + caps, ptrs)
    else:
        ptrs[0] = [x.data_ptr() for x in leaves0]
        bad = _lib.host().table_from_caps(caps, ptrs[1:])
        bad = bad + 1 if bad >= 0 else bad
    if bad >= 0:
        _stale_chain(bad)
    packed = _pack_weights([1] + [n._weight for n in links])
    waiting = [n for n in links if n._ticket is not None and n._ticket.node is not None]
    l2sq = None
    if waiting:
        l2sq = torch.empty(1 + len(links), dtype=torch.float32, device=leaves0[0].device)
    outs = _fold(_Table(list(leaves0), ptrs), packed, scale=scale, validated=True, l2sq=l2sq)
    if waiting:
        _fill_norms(links, waiting, l2sq)
    return pytree.unflatten(td, outs)


def _stale_chain(bad: int):
    """Raise for operand ``bad`` of a chain's fold (0: the base) found modified."""
    if bad == 0:
        raise RuntimeError("the running sum passed to tree_add was modified (a leaf replaced or updated in "
                           "place) before the pending sum was used; the reference adds its value at tree_add. "
                           "Call fedjax_amd.tree_util.set_deferred_sums(False) for loops that do this")
    raise RuntimeError(f"client {bad - 1} of a pending tree_add sum was modified (a leaf updated in place) "
                       "after its tree_weight / tree_add; the reference sums each delta's value at that "
                       "call. Add copies, or call fedjax_amd.tree_util.set_deferred_sums(False)")


def _fill_norms(links, waiting, l2sq):
    """Copy the fold's per-operand squared norms (l2sq[1 + j] for link j) into the chains'
    norm buffers the waiting lazy views read, and release the views' tickets."""
    # per chain, the links form one run of consecutive indices: two small launches each
    j = 0
    while j < len(links):
        ch, j0 = links[j]._chain, j
        while j < len(links) and links[j]._chain is ch and links[j]._idx == links[j0]._idx + (j - j0):
            j += 1
        if ch.buf is not None:
            # (links past the buffer's end — a chain continued across folds — have no views)
            i0 = links[j0]._idx
            n = min(j - j0, ch.buf.shape[1] - i0)
            if n > 0:  # buf[0, i] = l2sq, buf[1, i] = sqrt(l2sq), one launch (include/fjtree.h)
                src, cols = l2sq[1 + j0:1 + j0 + n], ch.buf.shape[1]
                _lib.check(_lib.load().fjtree_norms_fill(
                    src.data_ptr(), ch.buf.data_ptr() + 4 * i0, ch.buf.data_ptr() + 4 * (cols + i0), n,
                    torch.cuda.current_stream(src.device).cuda_stream), "fjtree_norms_fill")
    for n in waiting:
        n._ticket.node = None
        n._ticket = None


def _lazy_norm(pytree_, row: int):
    """A _NormView of the delta just added to a deferred sum, or None."""
    node = _HOST.last()  # the most recent PendingSum link (weakly held by fjhost)
    if node is None or node._value is not None or node._cap is None:
        return None
    host = _HOST
    if not host.matches(pytree_, node._cap[0], node._cap[1]):
        return None
    ch = node._chain
    if ch.buf is None:
        ch.buf = torch.empty((2, _DEFER["max_clients"] + 1), dtype=torch.float32, device=node._cap[0][0].device)
    if node._idx >= ch.buf.shape[1]:
        return None
    if node._ticket is None:
        node._ticket = _Ticket(node)
    v = host.norm_view(ch.buf, row, node._idx, _NormView)
    v._ticket = node._ticket
    return v


def _defer(sum_side, item, item_weight, item_cap):
    """PendingSum for tree_add(sum_side, weighted item), or None when not applicable.

    When the item comes from tree_weight (``item_cap``, its capture) and the sum's structure
    token equals the capture's, the structures and leaf shapes are known to match without a
    walk: the link holds the captured leaves — the values tree_weight saw, as the
    reference's eager tree_weight would — and the fold checks their versions. Otherwise
    ``fjhost.append_check`` walks the sum and the item together."""
    host = _HOST
    if type(sum_side) is PendingSum:
        parent, root = sum_side, None
        live = sum_side._value is None
        ref = sum_side._ref if live else sum_side._value
    else:
        ref, parent, root, live = sum_side, None, sum_side, False
    bcap = None
    if live:
        tok = parent._tok
    else:  # this link starts a run: capture its base (its leaves, versions and structure token)
        bcap = host.capture(ref, -1)
        tok = bcap[3] if bcap is not None else -1
    if item_cap is not None and tok >= 0 and item_cap[3] == tok:
        cap = item_cap
    else:
        cap = host.append_check(ref, item, item_cap)
        if cap is None:
            return None
        if type(cap) is int:
            raise RuntimeError("a pytree passed to tree_weight was modified (a leaf replaced or updated in "
                               "place) before its weighted value was used; the reference computes "
                               "tree_weight eagerly")
    if live:
        budget = parent._chain.budget
        if budget is None:
            budget = parent._chain.budget = _defer_budget(cap[0][0].device)
        if parent._n + 1 > _DEFER["max_clients"] or parent._bytes + cap[2] > budget or _flush_due(parent):
            parent.materialize()  # bound the chain: fold what is pending, continue from it
            bcap = host.capture(parent._value, -1)
    node = PendingSum(root, parent, cap, item_weight, ref, bcap, tok)
    host.set_last(node)
    return node


def _flush_due(p: "PendingSum") -> bool:
    """An early flush of the pending run ending at ``p`` before the next link (fjhost's
    flush_due): it holds flush_bytes in flush_clients links. (A second flush at half the
    thresholds while the GPU is idle was measured and dropped in round 5: synchronised
    configs[1] rounds 0.218 -> 0.266 ms with norms, profiles/r05_norm_loop/k_ab_idle_flush.jsonl.)"""
    return p._bytes >= _DEFER["flush_bytes"] and p._n >= _DEFER["flush_clients"]


def _tree_weight_py(pytree_: PyTree, weight: float) -> PyTree:
    """Weights tree leaves by weight (tree_util.py:29-32).

    Float32 device pytrees (<= 64 leaves) with a Python-number weight give a
    :class:`WeightedTree` (deferred, fused into the tree_add that consumes it);
    anything else is computed now by the pytree kernel. :func:`tree_weight` is the native
    fjhost.tree_weight, which builds the WeightedTree itself in the fast case and calls
    this function otherwise."""
    tw = type(weight)
    w = weight if (tw is float or tw is int) else _host_weight(weight)
    if (type(w) is float or (type(w) is int and -_F32_EXACT_INT < w < _F32_EXACT_INT)):
        cap = _HOST.capture(pytree_, -1)
        if cap is not None:
            return WeightedTree(pytree_, w, cap)
    return _fold_trees([pytree_], [w])


def _eager(t):
    return t.materialize() if type(t) is WeightedTree or type(t) is PendingSum else t


def tree_inverse_weight(pytree_: PyTree, weight: float) -> PyTree:
    """Weights tree leaves by ``1 / weight`` (tree_util.py:35-38); computed now. A
    :class:`PendingSum` is folded with the ``1/W`` scale in the same launch
    (``fl(s * f32(1/W))``, the reference's bits) — fed_avg.py:145-146 in one pass."""
    inv = _inverse(weight if type(weight) is float or type(weight) is int else _host_weight(weight))
    if type(pytree_) is PendingSum and pytree_._value is None:
        return _fold_pending(pytree_, inv)
    pytree_ = _eager(pytree_)
    if type(inv) is float:
        got = _leaf_fold([pytree_], [inv], [None])
        if got is not None:
            return got[0]
    return _fold_trees([pytree_], [inv])


def tree_zeros_like(pytree_: PyTree) -> PyTree:
    """Creates a tree with zeros with same structure as the input (tree_util.py:41-44).

    A plain pytree of float32 device tensors (the running-sum base of fed_avg.py:132) is
    zeroed as ONE allocation (fjhost.zeros_like: one allocation and one memset instead of
    one per leaf). Each leaf is still its own tensor with its own in-place version counter
    over a 256-byte aligned slice of that storage, so writing one leaf never marks the
    others modified. The slices share one storage: a leaf kept alive keeps the whole
    buffer alive, and ``torch.save`` of a single leaf writes every leaf's bytes. Other
    pytrees get one ``torch.zeros`` per leaf."""
    got = _HOST.zeros_like(pytree_)
    if got is not None:
        return got
    leaves, td = pytree.flatten(pytree_)
    device = _find_device(leaves)
    out = []
    for x in leaves:
        t = _to_tensor(x)
        dt = _CANONICAL.get(t.dtype)
        if dt is None:
            raise TypeError(f"leaf dtype {t.dtype} is not supported")
        out.append(torch.zeros(t.shape, dtype=dt, device=device))
    return pytree.unflatten(td, out)


def _tree_add_py(left: PyTree, right: PyTree) -> PyTree:
    """Adds two trees together (tree_util.py:47-50): x*1 is exact, so a K=2 fold
    with unit weights is the reference's ``jnp.add``. A :class:`WeightedTree` operand
    is folded in the same launch (``fl(s + fl(x * f32(n)))``), which also sums the
    squares of its input for a following ``tree_l2_norm`` of that input. :func:`tree_add`
    is the native fjhost.tree_add, which appends the running sum's link itself in the
    common case (tree_add(s, tree_weight(x, n)) with s a live deferred sum) and calls this
    function otherwise."""
    tl, tr = type(left) is WeightedTree, type(right) is WeightedTree
    if tr and not tl and right._tree is not None and _DEFER["enabled"]:
        # the running sum of fed_avg.py:137-138: s = tree_add(s, tree_weight(x, n))
        got = _defer(left, right._tree, right._weight, right._cap)
        if got is not None:
            return got
    pl, pr = type(left) is PendingSum, type(right) is PendingSum
    if _DEFER["enabled"] and (tl != tr or pl != pr) and not (pl and pr):
        # the running-sum pattern: defer (x + y == y + x exactly, so the sum may be either side)
        if tr and right._tree is not None and not tl:
            got = _defer(left, right._tree, right._weight, right._cap)
        elif tl and left._tree is not None and not tr:
            got = _defer(right, left._tree, left._weight, left._cap)
        elif pl and not tr:
            got = _defer(left, right, 1, None)
        elif pr and not tl:
            got = _defer(right, left, 1, None)
        else:
            got = None
        if got is not None:
            return got
    left, right = (left.materialize() if pl else left), (right.materialize() if pr else right)
    if tl or tr:
        ops = [left._tree if tl else left, right._tree if tr else right]
        if ops[0] is None or ops[1] is None:  # already materialized
            return _fold_trees([_eager(left), _eager(right)], [1, 1])
        ws = [left._weight if tl else 1, right._weight if tr else 1]
        caps = [left._cap if tl else None, right._cap if tr else None]
        norm_op = 1 if tr else 0
    else:
        ops, ws, caps, norm_op = [left, right], [1, 1], [None, None], -1
    got = _leaf_fold(ops, ws, caps, norm_operand=norm_op)
    if got is not None:
        out, sq, l2 = got
        if norm_op >= 0:
            _NORMS.appendleft((caps[norm_op], sq, l2))
        return out
    return _fold_trees([_eager(left), _eager(right)], [1, 1])


# The hot pair of the running-sum loop, native (fjhost.tree_weight / fjhost.tree_add): the
# fast case builds the WeightedTree / PendingSum link in C, everything else calls the Python
# functions above. Per client this is one builtin call each instead of a Python frame, the
# type tests and a Python object construction.
_HOST.fast_install(WeightedTree, PendingSum, _Chain, _tree_weight_py, _tree_add_py)
_HOST.fast_config(_DEFER["enabled"], _DEFER["max_clients"], _DEFER["flush_bytes"], _DEFER["flush_clients"])
# set_deferred_sums(True, **DEFERRED_SUM_DEFAULTS) restores the defaults
DEFERRED_SUM_DEFAULTS = {"max_clients": _DEFER["max_clients"], "flush_bytes": _DEFER["flush_bytes"],
                         "flush_clients": _DEFER["flush_clients"], "budget_bytes": 0}
tree_weight = _HOST.tree_weight
tree_add = _HOST.tree_add


def tree_sum(pytrees: Iterable[PyTree]) -> PyTree:
    """Sums multiple trees together (tree_util.py:64-73); ``None`` if empty."""
    trees = list(pytrees)
    if not trees:
        return None
    return _fold_trees(trees, [1] * len(trees))


def _collect_pairs(pairs):
    """Consume (tree, weight) pairs once: (trees, weights, W) with W summed as
    tree_util.py:86,95 (a Python float from 0.0; numpy scalars keep their type).
    ``weights`` is a :class:`_Weights` when every weight is a Python number."""
    if type(pairs) is not list:
        pairs = list(pairs)
    trees = [tree for tree, _ in pairs]  # unpacks each pair as `for pytree, weight in ...` does
    weights = [weight for _, weight in pairs]
    packed = _pack_weights(weights) if trees else None
    if packed is not None:
        return trees, packed, packed.total
    sum_weight = 0.0
    for i, w in enumerate(weights):
        w = weights[i] = _host_weight(w)
        sum_weight += w  # tree_util.py:95
    return trees, weights, sum_weight


# A synchronous tree_mean on an idle GPU waits for the whole host walk (every client's
# leaves checked, K x L pointers) before the fold starts. When the stream is idle the call
# walks the clients in chunks and launches each chunk's fold as soon as its pointers are
# gathered, accumulating into the first chunk's sums, with 1/W applied by the last launch
# (accumulate mode: the same per-element sequence, the same bits). Two shapes:
#   * the fold is the longer part (configs[1]: ~0.35 us of walk vs ~0.6 us of fold per
#     client): two launches, the first over _PIPELINE_FRAC of the clients;
#   * the walk is the longer part (many clients, many leaves per client): launches of
#     >= _PIPELINE_CHUNK clients, each chunk's fold hidden behind the next chunk's walk.
# Deltas of <= 256 KiB (the narrow plans, whose images are uploaded per launch) are not
# pipelined: there the per-launch upload costs more than the overlap gives.
# A busy stream gets one launch (the host work hides behind the queued kernels anyway).
# The idle probe (hipStreamQuery) puts a marker on the stream, ~3 us of GPU time per call
# when calls run back to back, so it is gated by a host-side estimate: the time the folds
# this module issued would finish at the 8 TB/s peak; before that the stream is busy with
# them and is not probed. FJAGG_PIPELINE_FRAC=0 turns the pipeline off (A/B runs).
# (0.2: profiles/r04p_flush/host.json, sync call 0.115-0.116 ms vs 0.117-0.118 at 0.25 and
# 0.122 at 0.1, two interleaved sweeps; round 3 picked 0.25 before the walk got faster)
_PIPELINE_FRAC = float(os.environ.get("FJAGG_PIPELINE_FRAC", "0.2"))
_PIPELINE_CHUNK = int(os.environ.get("FJAGG_PIPELINE_CHUNK", "512"))
_PIPELINE_MIN_BYTES = 64 << 20  # below this the first launch is too short to hide the walk
_WALK_NS_PER_LEAF = 35.0  # native walk + checks per (client, leaf), MI355X host
_PEAK_BYTES_PER_S = 8.0e12
class _BusyUntil:
    """perf_counter() time before which this module's issued folds cannot have finished:
    the builtin tree_mean's own estimate (fjhost.busy_until), so the native and the Python
    paths keep ONE (``_BUSY_UNTIL[0]`` reads it, ``_BUSY_UNTIL[0] = t`` sets it)."""

    __slots__ = ()

    def __getitem__(self, i):
        return _HOST.busy_until()

    def __setitem__(self, i, t):
        _HOST.busy_until(float(t))


_BUSY_UNTIL = _BusyUntil()


# The whole call in one native function (fjhost.mean_pairs) for the common case — plain
# dict / list / tuple pytrees of float32 CUDA tensors, Python-number weights: the same
# launches as below (gather, fold_table, the pipeline), without the Python walk of client 0,
# the pair collection and the unflatten. FJAGG_NATIVE_MEAN=0 keeps the Python path (A/B).
_NATIVE_MEAN = os.environ.get("FJAGG_NATIVE_MEAN", "1") != "0"


def _native_mean(pairs, with_l2: bool = False):
    """fjhost.mean_pairs: the tree (with_l2: (tree, l2sq)), or None when not its case."""
    if _ENTRY_ADDRS is None:
        _native_fold_addrs()
    now = time.perf_counter()
    extra = (_ENTRY_ADDRS[2], _ENTRY_ADDRS[3]) if with_l2 else ()
    got = _lib.host().mean_pairs(pairs, _PIPELINE_FRAC > 0.0 and now >= _BUSY_UNTIL[0], _PIPELINE_FRAC,
                                 _PIPELINE_CHUNK, _CHUNK_WALK_US, _WALK_NS_PER_LEAF, _PIPELINE_MIN_BYTES,
                                 _NARROW_MAX_BYTES, float(NONTEMPORAL_MIN_BYTES), _ENTRY_ADDRS[0], _ENTRY_ADDRS[1],
                                 *extra)
    if got is None:
        return None
    rc, tree, job_bytes, l2sq = got
    _BUSY_UNTIL[0] = max(now, _BUSY_UNTIL[0]) + job_bytes / _PEAK_BYTES_PER_S
    _lib.check(rc, "fjagg_wsum_l2_ptrs" if with_l2 else "fjagg_wsum_ptrs")
    return (tree, l2sq) if with_l2 else tree


def _stream_idle(stream: torch.cuda.Stream) -> bool:
    return stream.query()


_CHUNK_WALK_US = 60.0  # walk per chunk that amortises a launch's host cost (~15-20 us with its plan image)


def _pipeline_bounds(K: int, n: int, L: int) -> List[int]:
    """Chunk ends [k_1, ..., K] of the pipelined fold (see _PIPELINE_FRAC). Walk-bound
    calls take chunks of at least _PIPELINE_CHUNK clients and at least _CHUNK_WALK_US of
    walk each (profiles/r03g_pipeline/)."""
    walk_ns, fold_ns = _WALK_NS_PER_LEAF * L, 4.0 * n / _PEAK_BYTES_PER_S * 1e9
    if walk_ns > fold_ns and _PIPELINE_CHUNK > 0:
        c = max(_PIPELINE_CHUNK, int(np.ceil(_CHUNK_WALK_US * 1e3 / walk_ns)))
        if K > c:
            return list(range(c, K, c)) + [K]
    return [min(K - 1, max(1, int(K * _PIPELINE_FRAC))), K]


def _tree_mean_pipelined(trees: List[PyTree], packed: "_Weights", W, first) -> Optional[PyTree]:
    """tree_mean of float32 device pytrees in chunked launches overlapping the host walk
    (see _PIPELINE_FRAC); None (nothing launched, or launches whose outputs are dropped)
    when the case does not hold, and the caller then takes the one-launch path, which also
    raises the reference's errors. ``first``: pytree.flatten(trees[0])."""
    leaves0, td = first
    if not leaves0:
        return None
    x0 = leaves0[0]
    if type(x0) is not torch.Tensor or not x0.is_cuda:
        return None
    device = x0.device
    idx = x0.get_device()
    n = 0
    for x in leaves0:
        if type(x) is not torch.Tensor or x.dtype is not torch.float32 or x.get_device() != idx \
                or not x.is_contiguous():
            return None
        n += x.numel()
    K = len(trees)
    # small deltas (<= _NARROW_MAX_BYTES) fold through plan images uploaded per launch: chunked
    # launches there cost more than the overlap gives (profiles/r03g_pipeline/narrow2.jsonl)
    if 4 * n <= _NARROW_MAX_BYTES or 4 * n * K < _PIPELINE_MIN_BYTES:
        return None
    now = time.perf_counter()
    busy = now < _BUSY_UNTIL[0]
    _BUSY_UNTIL[0] = max(now, _BUSY_UNTIL[0]) + 4 * n * K / _PEAK_BYTES_PER_S  # this call's fold, either way
    stream = torch.cuda.current_stream(device)
    if busy or not _stream_idle(stream):
        return None  # kernels still queued: the walk already overlaps them
    spec = pytree.native_spec(td)
    if spec is None:
        return None
    host = _lib.host()
    if _ENTRY_ADDRS is None:
        _native_fold_addrs()
    plan, wsum, *_ = _ENTRY_ADDRS
    nt_min = 0.0 if 4 * n * K >= NONTEMPORAL_MIN_BYTES else float("inf")  # the whole job's bytes decide
    s = stream.cuda_stream
    ptrs = np.empty((K, len(leaves0)), dtype=np.int64)
    scale = float(np.float32(_inverse(W)))
    outs, done = None, 0  # clients [0, done) folded; client 0's row comes from the gather at k0 = 1
    for k1 in _pipeline_bounds(K, n, len(leaves0)):
        if host.gather_rows(trees, max(done, 1), spec, leaves0, idx, ptrs, k1) != 0:
            return None
        last = k1 == K
        got = host.fold_table(leaves0, ptrs[done:k1], packed.f32[done:k1], scale if last else 1.0, last, nt_min,
                              idx, s, plan, wsum, outs, 0 if outs is None else 1)
        if got is None:
            return None
        _lib.check(got[0], "fjagg_wsum_ptrs")
        outs, done = got[1], k1
    return pytree.unflatten(td, outs)


# tree_mean over a one-shot iterable holds at most this many bytes of client deltas
# (float32 leaves) before folding them into the running sum (see tree_mean).
STREAM_BUDGET_BYTES = 4 << 30


def _tree_mean_py(pytrees_and_weights: Iterable[Tuple[PyTree, float]]) -> PyTree:
    """Returns (weighted) mean of input trees and weights (tree_util.py:76-96).

    All K clients are folded by ONE kernel launch per leaf-dtype group; the result
    is bitwise equal to the reference's sequential jit fold for float32 leaves.
    The iterable is consumed once (it may be a generator, compression.py:191).

    A list or tuple is folded in one launch (its deltas are resident anyway). Any other
    iterable of float32 pytrees is consumed in chunks of at most
    :data:`STREAM_BUDGET_BYTES` of deltas, each folded into the running sum in
    accumulate mode (the same per-element sequence, so the same bits), with the ``1/W``
    scale fused into the last chunk's launch. Like the reference, which holds one client
    at a time, a generator of host-resident or freshly produced deltas therefore never
    needs all K deltas on the GPU at once; below the budget it is still one launch.

    Storage: the native path's float32 result leaves are slices of one allocation (each its
    own tensor and version counter, 256-byte aligned): one live leaf keeps every leaf's bytes
    allocated, and ``torch.save`` of one leaf writes them all — ``clone()`` a leaf to keep it
    on its own.
    """
    if type(pytrees_and_weights) is not list and type(pytrees_and_weights) is not tuple:
        return _tree_mean_stream(iter(pytrees_and_weights))
    if _NATIVE_MEAN and pytrees_and_weights:
        got = _native_mean(pytrees_and_weights)
        if got is not None:
            return got
    trees, weights, sum_weight = _collect_pairs(pytrees_and_weights)
    if not trees:
        return None  # tree_util.py:96 maps over None
    first = None
    if _PIPELINE_FRAC > 0.0 and len(trees) >= 8 and isinstance(weights, _Weights):
        first = pytree.flatten(trees[0])
        got = _tree_mean_pipelined(trees, weights, sum_weight, first)
        if got is not None:
            return got
    td, rows = _client_table(trees, first)
    if not rows[0]:
        return pytree.unflatten(td, [])
    inv = _inverse(sum_weight)
    return pytree.unflatten(td, _fold(rows, weights, scale=inv, validated=True))


def _mean_triples_py(clients) -> PyTree:
    """tree_mean over mean_aggregator().apply's (client_id, params, weight) triples
    (aggregator.py:61-75) when fjhost.mean_triples declines them."""
    return _tree_mean_py([(param, weight) for _, param, weight in clients])


# tree_mean is the native fjhost.tree_mean: a resident list / tuple of float32 device pytrees
# with Python-number weights is one native call (no Python frame); everything else is
# _tree_mean_py. mean_of_triples serves mean_aggregator().apply the same way.
tree_mean = _HOST.tree_mean
mean_of_triples = _HOST.mean_triples
_mean_config()  # the fallbacks now; the library's entry points once _native_fold_addrs runs


def _f32_tree_bytes(tree) -> Optional[int]:
    """4 x elements of a pytree whose leaves are all float32 (tensors or arrays), else None."""
    n = 0
    for x in pytree.leaves_of(tree):
        dt = getattr(x, "dtype", None)
        if dt is not torch.float32 and dt != np.float32:
            return None
        n += x.numel() if isinstance(x, torch.Tensor) else int(np.size(x))
    return 4 * n


def _tree_mean_stream(it) -> PyTree:
    first = next(it, None)
    if first is None:
        return None
    tree0, _ = first
    per_client = _f32_tree_bytes(tree0)
    if not per_client:  # other dtypes (whose fold type may depend on every weight): all at once
        return tree_mean([first] + list(it))
    B = max(1, STREAM_BUDGET_BYTES // per_client)
    chunk, out, td, sum_weight = [first], None, None, 0.0
    while True:
        done = False
        while len(chunk) < B:
            nxt = next(it, None)
            if nxt is None:
                done = True
                break
            chunk.append(nxt)
        if done and out is None and _NATIVE_MEAN:
            # the whole iterable fit one chunk (mean_aggregator().apply over resident clients):
            # the one-call native path, as tree_mean(list) takes
            got = _native_mean(chunk)
            if got is not None:
                return got
        trees = [t for t, _ in chunk]
        weights = [w for _, w in chunk]
        for i, w in enumerate(weights):
            w = weights[i] = _host_weight(w)
            sum_weight += w  # tree_util.py:95, in arrival order across chunks
        ctd, rows = _client_table(trees)
        if td is None:
            td = ctd
            if not rows[0]:
                list(it)  # consume the rest, as the reference's loop does
                return pytree.unflatten(td, [])
        elif ctd != td:
            raise ValueError(f"pytree structure mismatch: expected {td!r}, got {ctd!r}")
        packed = _pack_weights(weights)
        out = _fold(rows, packed if packed is not None else weights, out=out, accumulate=out is not None,
                    scale=_inverse(sum_weight) if done else None, validated=True)
        if done:
            return pytree.unflatten(td, out)
        chunk = []
        nxt = next(it, None)
        if nxt is None:  # the iterable ended exactly at a chunk boundary: scale what was folded
            return tree_inverse_weight(pytree.unflatten(td, out), sum_weight)
        chunk.append(nxt)


def tree_mean_with_l2_norms(pytrees_and_weights: Iterable[Tuple[PyTree, float]]):
    """``(tree_mean(pairs), [tree_l2_norm(tree) for tree, _ in pairs])`` from ONE pass over
    the client deltas (fjagg_wsum_l2_ptrs): the mean of examples/fed_avg.py:82 and the
    per-client ``delta_l2_norm`` diagnostic of :79-81 (tree_util.py:105-114).

    The mean is bitwise :func:`tree_mean`'s. The norms (float32 [K] on the device) sum
    squares in f32 in a fixed order; float leaves of one dtype.
    Returns ``(None, None)`` for no clients."""
    if (_NATIVE_MEAN and type(pytrees_and_weights) in (list, tuple)
            and 0 < len(pytrees_and_weights) <= _L2_MAX_CLIENTS):
        got = _native_mean(pytrees_and_weights, with_l2=True)
        if got is not None:
            return got[0], _sqrt_rn(got[1])
    trees, weights, sum_weight = _collect_pairs(pytrees_and_weights)
    if not trees:
        return None, None
    td, rows = _client_table(trees)
    if not rows[0]:
        return pytree.unflatten(td, []), torch.zeros(len(trees), dtype=torch.float32, device=_default_device())
    float_one = len({x.dtype for x in rows[0]}) == 1 and rows[0][0].dtype in (torch.float32, torch.bfloat16)
    if float_one and rows[0][0].dtype == torch.bfloat16:
        kinds = weights.kinds if isinstance(weights, _Weights) else [_weight_kind(w) for w in weights]
        float_one = _leaf_rule(torch.bfloat16, kinds, _WEAK_FLOAT)[1] == _lib.F32
    if len(trees) > _L2_MAX_CLIENTS or not float_one:
        # the fused pass keeps K partial norms per workgroup in LDS (K <= 4096) and sums one
        # float dtype: otherwise the mean and the norms take one pass each
        outs = _fold(rows, weights, scale=_inverse(sum_weight), validated=True)
        return pytree.unflatten(td, outs), tree_l2_norms(trees)
    l2sq = torch.empty(len(trees), dtype=torch.float32, device=rows[0][0].device)
    outs = _fold(rows, weights, scale=_inverse(sum_weight), validated=True, l2sq=l2sq)
    return pytree.unflatten(td, outs), _sqrt_rn(l2sq)


def _sqrt_rn(l2sq: torch.Tensor) -> torch.Tensor:
    """Correctly rounded float32 square roots of a device vector (jnp.sqrt of the reference's
    tree_l2_norm, tree_util.py:111-114): one fjtree_norms_fill launch (its f64 route; the
    single-precision device sqrt can be 1 ulp off)."""
    out = torch.empty_like(l2sq)
    _lib.check(_lib.load().fjtree_norms_fill(l2sq.data_ptr(), l2sq.data_ptr(), out.data_ptr(), l2sq.numel(),
                                             torch.cuda.current_stream(l2sq.device).cuda_stream), "fjtree_norms_fill")
    return out


_L2_MAX_CLIENTS = 4096  # fjagg_wsum_l2_ptrs (kL2MaxClients in fjagg.hip)


def _l2sq_mixed(row: List[torch.Tensor]) -> torch.Tensor:
    """``sum(jnp.vdot(x, x) for x in leaves)`` (tree_util.py:105-108) for leaves of mixed or
    integer dtypes: int32 leaves square and sum in wrapping int32 (exact in any order,
    computed mod 2**32), float leaves in float32; the per-leaf values are added in leaf
    order from Python's int 0 with jnp's promotion (int32 + float32 -> float32)."""
    acc = None
    for x in row:
        if x.dtype == torch.int32:
            v = (x.long() * x.long()).sum() & 0xFFFFFFFF
            v = torch.where(v >= 2 ** 31, v - 2 ** 32, v).to(torch.int32)
        else:
            xf = x.float()
            v = torch.dot(xf.reshape(-1), xf.reshape(-1))
        acc = v if acc is None else acc + v
    return acc if acc is not None else torch.zeros((), dtype=torch.int32)


def tree_size(pytree_: PyTree) -> int:
    """Returns total size of all tree leaves (tree_util.py:99-102)."""
    return int(sum(_to_tensor(x).numel() for x in pytree.leaves_of(pytree_)))


def _l2_rows(rows: List[List[torch.Tensor]], take_sqrt: bool) -> torch.Tensor:
    K, L = len(rows), len(rows[0])
    device = rows[0][0].device
    out = torch.empty(K, dtype=torch.float32, device=device)
    for row in rows:
        for x in row:
            if x.dtype not in (torch.float32, torch.bfloat16):
                raise TypeError(f"l2 norms support float32/bfloat16 leaves, not {x.dtype}")
    if any(x.dtype != rows[0][0].dtype for row in rows for x in row):
        raise TypeError("l2 norms need one leaf dtype across the tree")
    ptrs = np.array([x.data_ptr() for row in rows for x in row], dtype=np.int64)
    ns = np.array([x.numel() for row in rows for x in row], dtype=np.int64)
    image_dev = _lib.upload(torch.from_numpy(np.concatenate([ptrs, ns])), device)
    max_n = int(ns.max()) if ns.size else 0
    need = int(_lib.load().fjagg_l2sq_rows_workspace_bytes(K * L, max_n))
    ws = torch.empty(max(need, 4), dtype=torch.uint8, device=device)
    _lib.call("fjagg_l2sq_rows", kernels.dtype_code(rows[0][0].dtype), image_dev.data_ptr(), K * L,
              max_n, L, 1 if take_sqrt else 0, out.data_ptr(), ws.data_ptr(), ws.numel(),
              torch.cuda.current_stream(device).cuda_stream)
    return out


def _l2_fast(pytree_, which: int):
    """(l2sq, l2)[which] of a float32 device pytree: the fused value of a preceding
    tree_add(s, tree_weight(pytree_, n)) when pytree_ is unchanged since; with deferral on,
    else a standalone lazy norm (set_lazy_norms) that the tree_mean folding pytree_ computes;
    else one fjtree launch (same reduction order as the fused tree_add, so the same bits).
    None: not the fast case."""
    if _TREE_ADDRS is None:
        _tree_addrs()
    if _DEFER["enabled"]:
        v = _lazy_norm(pytree_, which)
        if v is not None:
            return v
    host = _lib.host()
    for cap, sq, l2 in _NORMS:
        if host.matches(pytree_, cap[0], cap[1]):
            return sq if which == 0 else l2
    if _DEFER["enabled"] and _LAZY["enabled"]:
        if _ENTRY_ADDRS is None:
            _native_fold_addrs()
        v = host.solo_norm(pytree_, which)
        if v is not None:
            return v
    got = _leaf_fold([pytree_], [1], [None], norm_operand=0, no_out=True)
    return None if got is None else got[1 + which]


def _tree_l2_squared_py(pytree_: PyTree) -> torch.Tensor:
    """Returns squared l2 norm of tree (tree_util.py:105-108), a 0-d float32 tensor.
    :func:`tree_l2_squared` is the native fjhost.tree_l2_squared, which returns the lazy
    view of the delta a deferred sum just took itself and calls this function otherwise."""
    pytree_ = _eager(pytree_)
    got = _l2_fast(pytree_, 0)
    if got is not None:
        return got
    _, rows = _client_rows([pytree_])
    if not rows[0]:
        return torch.zeros((), dtype=torch.float32, device=_default_device())
    if len({x.dtype for x in rows[0]}) > 1 or rows[0][0].dtype == torch.int32:
        return _l2sq_mixed(rows[0])
    return _l2_rows(rows, take_sqrt=False).reshape(())


def _tree_l2_norm_py(pytree_: PyTree) -> torch.Tensor:
    """Returns l2 norm of tree (tree_util.py:111-114), a 0-d float32 tensor.
    :func:`tree_l2_norm` is the native fjhost.tree_l2_norm (see _tree_l2_squared_py)."""
    pytree_ = _eager(pytree_)
    got = _l2_fast(pytree_, 1)
    if got is not None:
        return got
    _, rows = _client_rows([pytree_])
    if not rows[0]:
        return torch.zeros((), dtype=torch.float32, device=_default_device())
    if len({x.dtype for x in rows[0]}) > 1 or rows[0][0].dtype == torch.int32:
        return torch.sqrt(_l2sq_mixed(rows[0]).float())  # jnp.sqrt of an int32 sum is float32
    return _l2_rows(rows, take_sqrt=True).reshape(())


# The per-client delta_l2_norm of the running-sum loops (fed_avg.py:142-144), native: the lazy
# view of the delta the running sum just took, without a Python frame (fjhost.tree_l2_norm).
_HOST.fast_install_norms(_Ticket, _NormView, _tree_l2_squared_py, _tree_l2_norm_py, _fold_ticket)
_solo_config()  # set_lazy_norms' defaults (FJAGG_LAZY_NORMS=0: off); the entry points once the library loads
tree_l2_squared = _HOST.tree_l2_squared
tree_l2_norm = _HOST.tree_l2_norm


def tree_l2_norms(pytrees: Sequence[PyTree]) -> torch.Tensor:
    """l2 norm of each of K trees in ONE launch (float32[K]) — the per-client
    ``delta_l2_norm`` diagnostic of examples/fed_avg.py:79-81 batched."""
    trees = list(pytrees)
    _, rows = _client_rows(trees)
    if len({x.dtype for x in rows[0]}) > 1 or rows[0][0].dtype == torch.int32:
        return torch.stack([torch.sqrt(_l2sq_mixed(r).float()) for r in rows])
    return _l2_rows(rows, take_sqrt=True)


def tree_clip_by_global_norm(pytree_: PyTree, max_norm: float) -> PyTree:
    """Clips a pytree of arrays using their global norm (tree_util.py:117-133).

    ``scale = min(1, max_norm / norm)`` is formed in float32 as the reference does;
    it is read back to the host to parameterise the weighting launch.
    """
    norm = np.float32(tree_l2_norm(pytree_).item())
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.minimum(np.float32(1), np.float32(max_norm) / norm)
    return _eager(tree_weight(pytree_, np.float32(scale)))
