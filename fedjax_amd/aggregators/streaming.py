"""Streaming weighted mean: the running-sum pattern of FedJAX's algorithms.

fedjax/algorithms/fed_avg.py:132-146 (and fed_prox.py:127-140, mime.py:186-197,
mime_lite.py:129-148, agnostic_fed_avg.py:278-289, apfl.py:207-220,
hyp_cluster.py:284-304) aggregate clients as they arrive from a generator::

    delta_params_sum = tree_util.tree_zeros_like(server_state.params)
    num_examples_sum = 0.
    for client_id, delta_params in train_for_each_client(...):
        delta_params_sum = tree_util.tree_add(
            delta_params_sum, tree_util.tree_weight(delta_params, num_examples))
        num_examples_sum += num_examples
    mean_delta_params = tree_util.tree_inverse_weight(delta_params_sum, num_examples_sum)

That is 2 XLA dispatches and ~5P element transfers per client. :class:`RunningMean`
keeps the running sum on the GPU and folds each arriving batch of B clients with
ONE launch of the pytree kernel in accumulate mode
(``s = fl(s + fl(x_b * w_b))`` for b = 0..B-1, in arrival order) — the same
rounding sequence as the loop above, so the result is bitwise equal, at
(B + 2)·P element transfers per B clients.
"""

from __future__ import annotations

from typing import Any, List, Optional

import numpy as np
import torch

from fedjax_amd import pytree, tree_util
from fedjax_amd.typing import PyTree


_NO_VERSION = -2  # fjhost.cpp kNoVersion: an inference tensor (no in-place version counter)


def _version_of(x) -> int:
    """In-place version counter of a tensor leaf; -1 for host arrays and scalars, and
    _NO_VERSION for inference tensors (``torch.inference_mode``), whose ``_version`` raises."""
    if not isinstance(x, torch.Tensor):
        return -1
    return _NO_VERSION if x.is_inference() else int(x._version)


class RunningMean:
    """Running weighted sum of client deltas with the structure of ``template``.

    ``add(delta, weight)`` may be called with device or host pytrees; deltas are
    buffered and folded ``buffer_clients`` at a time (default: as many as fit
    ``tree_util.STREAM_BUDGET_BYTES``, so usually once per round). ``result()`` returns
    ``tree_inverse_weight(sum, total_weight)`` (tree_util.py:35-38).

    Buffering holds references, not copies. The reference's loop reads each delta at
    its ``tree_add``, so a caller that updates a delta tensor in place after ``add()``
    (reusing one buffer for every client, as torch loops often do) would change the
    sum here but not there. Each tensor leaf's in-place version counter is recorded
    at ``add()`` and checked before the buffer is read: a changed leaf raises
    ``RuntimeError``. The guard watches the tensors, not the containers: putting a
    different tensor into a buffered dict or list after ``add()`` is not detected.
    ``copy_on_add=True`` clones every delta (into a fresh container) at ``add()``
    instead (one extra device copy per client; safe for any reuse). Inference tensors
    (``torch.inference_mode``) have no version counter, so their leaves are always
    cloned at ``add()``.
    """

    def __init__(self, template: PyTree, *, buffer_clients: Optional[int] = None,
                 device: Optional[torch.device] = None, copy_on_add: bool = False):
        leaves, self.treedef = pytree.flatten(template)
        self.device = device or tree_util._find_device(leaves)
        self._sum: List[torch.Tensor] = self._zero_sum(leaves)  # fed_avg.py:132
        self.total_weight: Any = 0.0  # fed_avg.py:133 (num_examples_sum = 0.)
        self.num_clients = 0
        if buffer_clients is None:
            # as many clients as tree_mean streams per launch (STREAM_BUDGET_BYTES of deltas,
            # at most 4096): one fold per round for most models (configs[1]: 888 clients)
            per = max(1, 4 * sum(int(x.numel()) for x in self._sum))
            buffer_clients = min(4096, max(1, tree_util.STREAM_BUDGET_BYTES // per))
        self.buffer_clients = max(1, int(buffer_clients))
        self._trees: List[PyTree] = []
        self._weights: List[Any] = []
        self.copy_on_add = bool(copy_on_add)
        self._spec = pytree.native_spec(self.treedef)
        self._nleaves = len(self._sum)
        # versions recorded at add(): row k belongs to self._trees[k] (grown by doubling)
        self._vrows = np.empty((min(self.buffer_clients, 64), self._nleaves), dtype=np.int64)
        self._host = None

    def _zero_sum(self, leaves) -> List[torch.Tensor]:
        """tree_zeros_like(template) on the device, as leaves. An all-float32 template gets
        one zeroed allocation carved into 256-byte-aligned contiguous leaf views (one
        allocation and one memset per round instead of one per leaf)."""
        shapes = [tuple(x.shape) for x in leaves]
        if leaves and all(isinstance(x, torch.Tensor) and x.dtype == torch.float32 or
                          isinstance(x, np.ndarray) and x.dtype == np.float32 for x in leaves):
            sizes = [int(np.prod(s, dtype=np.int64)) for s in shapes]
            offs = np.concatenate([[0], np.cumsum([(n + 63) // 64 * 64 for n in sizes])])
            flat = torch.zeros(int(offs[-1]), dtype=torch.float32, device=self.device)
            return [flat[int(o):int(o) + n].view(s) for o, n, s in zip(offs, sizes, shapes)]
        zeros = tree_util.tree_zeros_like(pytree.unflatten(self.treedef, [
            tree_util._device_leaf(x, self.device) for x in leaves]))
        return pytree.leaves_of(zeros)

    def _leaf_versions(self, trees: List[PyTree]):
        """int64 [len(trees), L] in-place version counters of every tensor leaf (-1 for
        host arrays and scalars, which carry none); ValueError on a structure mismatch."""
        L = self._nleaves
        v = np.empty((len(trees), L), dtype=np.int64)
        if self._spec is not None:
            from fedjax_amd import _lib
            if _lib.host().leaf_versions(trees, self._spec, L, v) == 0:
                return v
        for k, t in enumerate(trees):  # other leaf types or node kinds; raises on mismatch
            v[k] = [_version_of(x) for x in pytree.flatten_as(self.treedef, t)]
        return v

    def _record_versions(self, delta: PyTree) -> None:
        """_leaf_versions([delta]) into row len(self._trees) of self._vrows; the native
        walk writes the row in place (no per-client array: add() is on the client loop)."""
        i = len(self._trees)
        if i >= self._vrows.shape[0]:
            self._vrows = np.concatenate([self._vrows, np.empty_like(self._vrows)])
        row = self._vrows[i]
        if self._spec is not None:
            if self._host is None:
                from fedjax_amd import _lib
                self._host = _lib.host()
            if self._host.leaf_versions([delta], self._spec, self._nleaves, row) == 0:
                return
        row[:] = self._leaf_versions([delta])[0]

    def add(self, delta: PyTree, weight) -> None:
        """tree_add(sum, tree_weight(delta, weight)); fed_avg.py:137-139. The delta is
        buffered by reference (a clone with ``copy_on_add``); its leaves are read when
        the buffer is folded, after checking that none was modified in place since."""
        w = tree_util._host_weight(weight)
        if self.copy_on_add:
            delta = pytree.unflatten(self.treedef, [
                x.clone() if isinstance(x, torch.Tensor) else x for x in pytree.flatten_as(self.treedef, delta)])
        else:
            self._record_versions(delta)
            if (self._vrows[len(self._trees)] == _NO_VERSION).any():
                # inference tensors carry no version counter to guard the reference with:
                # buffer a snapshot of those leaves instead (their values at add(), as the
                # reference reads them)
                delta = pytree.unflatten(self.treedef, [
                    x.clone() if isinstance(x, torch.Tensor) and x.is_inference() else x
                    for x in pytree.flatten_as(self.treedef, delta)])
                self._vrows[len(self._trees)] = self._leaf_versions([delta])[0]
        self._trees.append(delta)
        self._weights.append(w)
        self.total_weight += w
        self.num_clients += 1
        if len(self._trees) >= self.buffer_clients:
            self.flush()

    def flush(self) -> None:
        """Fold the buffered clients into the running sum: ONE pytree-kernel launch in
        accumulate mode. The K x L pointer table comes from the native gather
        (tree_util._client_table) when every buffered delta is already a pytree of
        contiguous device tensors shaped like the sum; otherwise each delta is
        flattened against the template and copied to the device first."""
        if not self._trees:
            return
        trees, weights = self._trees, self._weights
        self._trees, self._weights = [], []
        if not self._sum:  # dtype rules checked by _fold (the sum has the template's dtypes)
            return
        if not self.copy_on_add and not np.array_equal(self._leaf_versions(trees), self._vrows[:len(trees)]):
            raise RuntimeError("a buffered client delta was modified in place after RunningMean.add(); "
                               "the reference would have summed its value at add() time. Add a copy, "
                               "or construct RunningMean(..., copy_on_add=True)")
        td, rows = tree_util._client_table(trees)
        if not (td == self.treedef and isinstance(rows, tree_util._Table)
                and rows.row0[0].device == self.device):
            rows = [[tree_util._device_leaf(x, self.device) for x in pytree.flatten_as(self.treedef, t)]
                    for t in trees]
        packed = tree_util._pack_weights(weights)
        tree_util._fold(rows, packed if packed is not None else weights, out=self._sum, accumulate=True)

    def sum(self) -> PyTree:
        """The running weighted sum (flushes pending clients)."""
        self.flush()
        return pytree.unflatten(self.treedef, self._sum)

    def result(self) -> PyTree:
        """tree_inverse_weight(sum, total_weight); fed_avg.py:145-146."""
        return tree_util.tree_inverse_weight(self.sum(), self.total_weight)


__all__ = ["RunningMean"]
