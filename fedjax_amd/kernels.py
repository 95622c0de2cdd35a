"""Tensor-level wrappers over the C ABI (include/fjagg.h).

Every function here takes device-resident ``torch`` tensors (only the weights of
:func:`weighted_sum_dense` may be host arrays), launches on torch's current HIP
stream and returns without synchronising (like a JAX dispatch). They are the only
route from Python to the kernels; there is no CPU or PyTorch fallback: host client
deltas, an unsupported dtype or a missing library raise.
"""

from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from fedjax_amd import _lib

_EUNSUPPORTED = -3  # FJAGG_EUNSUPPORTED: the launch was refused, nothing was issued
# how host weights reached the dense folds: in the kernel arguments, or uploaded because
# the launch was not built that way (tests and bench.py read these)
HOST_WEIGHT_PATHS = {"kernel_args": 0, "uploaded": 0}
_CODES = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16, torch.int32: _lib.I32}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _CODES[dt]
    except KeyError:
        raise TypeError(f"fedjax_amd kernels support float32, bfloat16 and int32, not {dt}") from None


class Event:
    """HIP timing event created without the system-scope fence (``fjagg_event_create``,
    include/fjcomm.h): recording one does not write back or invalidate the caches, so
    bracketing every launch leaves the launches themselves unperturbed (a default
    ``torch.cuda.Event`` record costs ~30 us of cache write-back on MI355X)."""

    def __init__(self):
        import ctypes
        h = ctypes.c_void_p()
        _lib.call("fjagg_event_create", ctypes.byref(h))
        self.handle = h.value

    def record(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream()
        _lib.call("fjagg_event_record", self.handle, s.cuda_stream)

    def elapsed_time(self, end: "Event") -> float:
        """Milliseconds from this event to ``end`` (waits for ``end``)."""
        import ctypes
        ms = ctypes.c_float()
        _lib.call("fjagg_event_elapsed_ms", ctypes.byref(ms), self.handle, end.handle)
        return float(ms.value)

    def __del__(self):
        if getattr(self, "handle", None):
            _lib.load().fjagg_event_destroy(self.handle)
            self.handle = None


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _require_device(*ts: torch.Tensor) -> torch.device:
    dev = None
    for t in ts:
        if not t.is_cuda:
            raise ValueError("fedjax_amd kernels need device tensors (got a host tensor); "
                             "move client deltas to the GPU first")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"tensors on different devices: {dev} and {t.device}")
    return dev


def stripe_variant(total_cols: int, cus: int) -> int:
    """The stripe width k_dense_stripe / k_ptrs_stripe use for ``total_cols`` columns
    (fjstripe.hip stripe_cols): 64 while every CU still gets a stripe, then 32, else 16,
    as FJAGG_VARIANT 20 / 21 / 22."""
    if (total_cols + 63) // 64 >= cus:
        return 20
    if (total_cols + 31) // 32 >= cus:
        return 21
    return 22


def weighted_sum_dense(x: torch.Tensor, w: torch.Tensor, *, scale: Optional[float] = None,
                       out: Optional[torch.Tensor] = None, out_dtype: Optional[torch.dtype] = None,
                       accumulate: bool = False, mode: str = "exact",
                       workspace: Optional[torch.Tensor] = None, nontemporal: bool = False,
                       variant: int = 0, balanced: bool = True, reference_bf16: bool = False) -> torch.Tensor:
    """Fold a client-major slab ``x[K, P]`` (row stride ``x.stride(0)``, unit column
    stride) with per-client weights ``w[K]`` into ``out[P]``.

    ``w`` is float32 (float fold) or int32 (integer fold; int32 ``x`` only): a device
    tensor, or host weights (a numpy array or CPU tensor), which then travel in the
    kernel arguments (``FJAGG_HOST_TABLES``: no upload in front of the fold on the
    stream) when the library builds that launch, and are uploaded otherwise.
    ``scale`` multiplies the fold at the end (tree_mean's f32(1/W)).
    ``accumulate`` starts the fold from ``out``'s current contents.
    ``reference_bf16`` (bfloat16 ``x`` and ``out``, float32 ``w``): the reference's
    bfloat16 arithmetic — weights and scale rounded to bf16, every product and sum
    rounded to bf16 (acc dtype FJAGG_BF16) — instead of a float32 fold.
    """
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be a [K, P] tensor with unit column stride")
    K, P = x.shape
    if isinstance(w, np.ndarray):
        w = torch.from_numpy(w)
    if tuple(w.shape) != (K,):
        raise ValueError(f"w must have shape ({K},), got {tuple(w.shape)}")
    acc = _lib.I32 if w.dtype == torch.int32 else _lib.F32
    if w.dtype not in (torch.float32, torch.int32) or not w.is_contiguous():
        raise TypeError("w must be a contiguous float32 or int32 tensor")
    if reference_bf16:
        if x.dtype != torch.bfloat16 or w.dtype != torch.float32:
            raise TypeError("reference_bf16 folds bfloat16 deltas with float32 weights")
        acc = _lib.BF16
    if out is None:
        if out_dtype is None:
            if acc == _lib.BF16:
                out_dtype = torch.bfloat16
            elif acc == _lib.F32:  # int32 leaves * float weights promote to float32
                out_dtype = torch.float32 if x.dtype == torch.int32 else x.dtype
            else:
                out_dtype = torch.float32 if scale is not None else torch.int32
        out = torch.empty(P, dtype=out_dtype, device=x.device)
    if out.numel() != P or not out.is_contiguous():
        raise ValueError("out must be a contiguous tensor of P elements")
    dev = _require_device(x, out) if not w.is_cuda else _require_device(x, w, out)
    flags = (_lib.SCALE if scale is not None else 0) | (_lib.ACCUMULATE if accumulate else 0)
    flags |= (_lib.NONTEMPORAL if nontemporal else 0) | ((variant & 0xFF) << 8)
    flags |= 0 if balanced else _lib.UNBALANCED
    m = {"exact": _lib.MODE_EXACT, "split": _lib.MODE_SPLIT}[mode]
    ld = x.stride(0) if K > 1 else P
    sc = float(scale if scale is not None else 1.0)
    if not w.is_cuda:
        w = w.contiguous()
        if m == _lib.MODE_EXACT:
            rc = _lib.load().fjagg_wsum_dense(dtype_code(x.dtype), acc, dtype_code(out.dtype), x.data_ptr(), ld, K, P,
                                              w.data_ptr(), sc, out.data_ptr(), flags | _lib.HOST_TABLES, m, None, 0,
                                              _stream_handle(dev))
            if rc != _EUNSUPPORTED:
                _lib.check(rc, "fjagg_wsum_dense")
                HOST_WEIGHT_PATHS["kernel_args"] += 1
                return out
        w = _lib.upload(w, dev)  # not built with kernel-argument weights
        HOST_WEIGHT_PATHS["uploaded"] += 1
    ws_ptr, ws_bytes = None, 0
    if m == _lib.MODE_SPLIT:
        need = split_workspace_bytes(K, P)
        if need:
            if workspace is None:
                workspace = torch.empty(need, dtype=torch.uint8, device=dev)
            ws_ptr, ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    _lib.call("fjagg_wsum_dense", dtype_code(x.dtype), acc, dtype_code(out.dtype), x.data_ptr(), ld,
              K, P, w.data_ptr(), sc, out.data_ptr(), flags, m, ws_ptr, ws_bytes, _stream_handle(dev))
    return out


def weighted_sum_l2_dense(x: torch.Tensor, w: torch.Tensor, *, scale: Optional[float] = None,
                          out: Optional[torch.Tensor] = None, l2sq: Optional[torch.Tensor] = None,
                          accumulate: bool = False, nontemporal: bool = False,
                          workspace: Optional[torch.Tensor] = None):
    """``weighted_sum_dense`` (exact mode, float fold) plus every client's squared
    L2 norm from the same pass: returns ``(out[P], l2sq[K])``."""
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be a [K, P] tensor with unit column stride")
    K, P = x.shape
    if w.shape != (K,) or w.dtype != torch.float32 or not w.is_contiguous():
        raise TypeError(f"w must be a contiguous float32 tensor of shape ({K},)")
    if out is None:
        out = torch.empty(P, dtype=x.dtype, device=x.device)
    if l2sq is None:
        l2sq = torch.empty(K, dtype=torch.float32, device=x.device)
    dev = _require_device(x, w, out, l2sq)
    need = int(_lib.load().fjagg_wsum_l2_workspace_bytes(K, P))
    flags = (_lib.SCALE if scale is not None else 0) | (_lib.ACCUMULATE if accumulate else 0)
    flags |= _lib.NONTEMPORAL if nontemporal else 0
    if workspace is None and not _L2_COMBINE_LAUNCH:  # a zeroed-counter workspace: the fold's last
        # workgroup combines. The stream's cached one, or under a graph capture one of the capture's
        # own: a capture records the zeroing instead of running it (torch.zeros: a fill kernel every
        # replay runs; a recorded memset acts on the first replay only)
        workspace = (torch.zeros(max(need, 4096), dtype=torch.uint8, device=dev)
                     if torch.cuda.is_current_stream_capturing() else _l2_workspace(dev, need))
        flags |= _lib.ZEROED_WS
    elif workspace is None:
        workspace = torch.empty(max(need, 4), dtype=torch.uint8, device=dev)
    elif workspace.numel() * workspace.element_size() < need:  # (a caller's workspace: two launches)
        workspace = torch.empty(max(need, 4), dtype=torch.uint8, device=dev)
    ld = x.stride(0) if K > 1 else P
    _lib.call("fjagg_wsum_l2_dense", dtype_code(x.dtype), _lib.F32, dtype_code(out.dtype), x.data_ptr(),
              ld, K, P, w.data_ptr(), float(scale if scale is not None else 1.0), out.data_ptr(),
              l2sq.data_ptr(), flags, workspace.data_ptr(), workspace.numel() * workspace.element_size(),
              _stream_handle(dev))
    return out, l2sq


_L2_WS = {}  # (device index, stream handle) -> fused-norm workspace, counter header zero
# FJAGG_L2_COMBINE_LAUNCH=1: keep the separate norm-combine launch (as fjhost; include/fjagg.h
# FJAGG_ZEROED_WS): the in-launch hand-off follows the HIP guide's measured gfx950 recipe
_L2_COMBINE_LAUNCH = os.environ.get("FJAGG_L2_COMBINE_LAUNCH", "0") == "1"


def _l2_workspace(dev: torch.device, need: int) -> torch.Tensor:
    """The FJAGG_ZEROED_WS workspace of ``dev``'s current stream (fjagg.h): zeroed when it is
    (re)allocated; every fused-norm launch leaves its 16-byte completion counter zero, and
    launches on one stream are ordered, so they share it."""
    key = (dev.index, _stream_handle(dev))
    ws = _L2_WS.get(key)
    if ws is None and len(_L2_WS) >= 16:  # many short-lived streams: keep the cache bounded
        _L2_WS.clear()
    if ws is None or ws.numel() < need:
        ws = _L2_WS[key] = torch.zeros(max(2 * need, 4096), dtype=torch.uint8, device=dev)
    return ws


def split_workspace_bytes(K: int, P: int) -> int:
    return int(_lib.load().fjagg_split_workspace_bytes(K, P))


def ptrs_plan(in_code: int, leaf_n: Sequence[int], unaligned, narrow: bool = False,
              stripe_variant: int = 0) -> np.ndarray:
    """Workgroup table of the pytree kernel (host int64 array, 2 words per workgroup).

    ``unaligned``: a bool for the whole launch (True = element units everywhere; launch
    with ``unaligned=True``), or a per-leaf boolean array: the marked leaves take
    element units, the others 16-byte units (``fjagg_ptrs_plan_leaves``; launch with
    ``unaligned=False``). ``narrow``: 64-element stripes for k_ptrs_narrow (any
    alignment; launch with ``FJAGG_NARROW``); with ``stripe_variant`` 20 / 21 / 22:
    64 / 32 / 16-element stripes for k_ptrs_stripe (16-byte aligned pointers; launch with
    ``FJAGG_NARROW | FJAGG_VARIANT(stripe_variant)``)."""
    lib = _lib.load()
    n = np.ascontiguousarray(leaf_n, dtype=np.int64)
    if narrow:
        flags, mask = _lib.NARROW | ((stripe_variant & 0xFF) << 8), None
    elif isinstance(unaligned, (bool, np.bool_)):
        flags, mask = (_lib.UNALIGNED if unaligned else 0), None
    else:
        mask = np.ascontiguousarray(unaligned, dtype=np.uint8)
        if mask.shape != n.shape:
            raise ValueError(f"per-leaf mask of {mask.shape[0] if mask.ndim else 0} entries for {n.size} leaves")
        flags = 0
    mp = mask.ctypes.data if mask is not None else None
    need = lib.fjagg_ptrs_plan_leaves(in_code, flags, n.ctypes.data, mp, len(n), None, 0)
    _lib.check(0 if need >= 0 else int(need), "fjagg_ptrs_plan_leaves")
    blocks = np.empty(2 * max(need, 1), dtype=np.int64)
    got = lib.fjagg_ptrs_plan_leaves(in_code, flags, n.ctypes.data, mp, len(n), blocks.ctypes.data, need)
    _lib.check(0 if got >= 0 else int(got), "fjagg_ptrs_plan_leaves")
    return blocks[:2 * need]


def weighted_sum_ptrs(in_code: int, acc_code: int, out_code: int, image_dev: torch.Tensor,
                      L: int, K: int, nblk: int, w_dev: torch.Tensor, scale: Optional[float],
                      accumulate: bool = False, unaligned: bool = False,
                      nontemporal: bool = False, narrow: bool = False, stripe_variant: int = 0) -> None:
    """Launch the pytree kernel over a device plan image (see include/fjagg.h); ``narrow`` /
    ``stripe_variant`` as the plan was built (:func:`ptrs_plan`)."""
    dev = _require_device(image_dev, w_dev)
    flags = (_lib.SCALE if scale is not None else 0) | (_lib.ACCUMULATE if accumulate else 0)
    flags |= (_lib.UNALIGNED if unaligned else 0) | (_lib.NONTEMPORAL if nontemporal else 0)
    flags |= (_lib.NARROW | ((stripe_variant & 0xFF) << 8)) if narrow else 0
    _lib.call("fjagg_wsum_ptrs", in_code, acc_code, out_code, image_dev.data_ptr(), L, K, nblk,
              w_dev.data_ptr(), float(scale if scale is not None else 1.0), flags,
              _stream_handle(dev))


def l2_squared_dense(x: torch.Tensor, out: Optional[torch.Tensor] = None,
                     workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-client sum of squares of a [K, P] slab -> float32[K] (tree_util.py:105-108)."""
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be a [K, P] tensor with unit column stride")
    K, P = x.shape
    dev = _require_device(x)
    if out is None:
        out = torch.empty(K, dtype=torch.float32, device=dev)
    need = int(_lib.load().fjagg_l2sq_workspace_bytes(K, P))
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(max(need, 4), dtype=torch.uint8, device=dev)
    ld = x.stride(0) if K > 1 else P
    _lib.call("fjagg_l2sq_dense", dtype_code(x.dtype), x.data_ptr(), ld, K, P, out.data_ptr(),
              workspace.data_ptr(), workspace.numel() * workspace.element_size(), _stream_handle(dev))
    return out


def fill_synth(x: torch.Tensor, *, k0: int = 0, seed: int = 0, amp: float = 0.01) -> torch.Tensor:
    """Synthetic deltas x[k, p] = amp * u(seed, k0 + k, p) (tests/bench only)."""
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be a [K, P] tensor with unit column stride")
    dev = _require_device(x)
    K, P = x.shape
    ld = x.stride(0) if K > 1 else P
    _lib.call("fjagg_fill_synth", dtype_code(x.dtype), x.data_ptr(), ld, K, P, k0, seed, amp,
              _stream_handle(dev))
    return x
