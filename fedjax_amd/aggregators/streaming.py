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

import torch

from fedjax_amd import pytree, tree_util
from fedjax_amd.typing import PyTree


class RunningMean:
    """Running weighted sum of client deltas with the structure of ``template``.

    ``add(delta, weight)`` may be called with device or host pytrees; deltas are
    buffered (references only) and folded ``buffer_clients`` at a time. ``result()``
    returns ``tree_inverse_weight(sum, total_weight)`` (tree_util.py:35-38).
    """

    def __init__(self, template: PyTree, *, buffer_clients: int = 8,
                 device: Optional[torch.device] = None):
        leaves, self.treedef = pytree.flatten(template)
        self.device = device or tree_util._find_device(leaves)
        zeros = tree_util.tree_zeros_like(pytree.unflatten(self.treedef, [
            tree_util._device_leaf(x, self.device) for x in leaves]))
        self._sum: List[torch.Tensor] = pytree.leaves_of(zeros)  # fed_avg.py:132
        self.total_weight: Any = 0.0  # fed_avg.py:133 (num_examples_sum = 0.)
        self.num_clients = 0
        self.buffer_clients = max(1, int(buffer_clients))
        self._trees: List[PyTree] = []
        self._weights: List[Any] = []

    def add(self, delta: PyTree, weight) -> None:
        """tree_add(sum, tree_weight(delta, weight)); fed_avg.py:137-139. The delta is
        buffered by reference; its leaves are read when the buffer is folded."""
        w = tree_util._host_weight(weight)
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
