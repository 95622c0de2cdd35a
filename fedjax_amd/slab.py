"""Client-major delta slab: the HBM layout of K client deltas for one round.

The reference keeps one pytree per client (examples/fed_avg.py:72-76 holds all K
at once in a Python list). On MI355X the fold is fastest when every client's
delta is one contiguous row of a single allocation::

    slab[K, P]   row k = client k's leaves back to back, jax flatten order
                 (dict keys sorted), row stride padded to 16 bytes

so one launch of the dense kernel streams K*P elements with 1 KiB coalesced
wave loads and writes one P-element result. 288 GB of HBM holds e.g. 1024
clients x 4 M f32 params (17 GB) or 1024 x 125 M bf16 (256 GB) per GPU.

``client(k)`` returns a pytree of views into row k, so client training (or an
H2D copy of a host-resident delta) writes straight into the slab; those views
also work with :func:`fedjax_amd.tree_util.tree_mean` (pytree path).
"""

from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from fedjax_amd import _lib, kernels, pytree, tree_util
from fedjax_amd.typing import PyTree


class ClientDeltaSlab:
    """K client deltas sharing one pytree structure, as one [K, P] device tensor."""

    def __init__(self, template: PyTree, num_clients: int, *, dtype: torch.dtype = torch.float32,
                 device: Optional[torch.device] = None):
        if dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("slab dtype must be float32 or bfloat16")
        leaves, self.treedef = pytree.flatten(template)
        self.shapes = [tuple(tree_util._to_tensor(x).shape) for x in leaves]
        self.sizes = [int(np.prod(s, dtype=np.int64)) for s in self.shapes]
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        self.num_params = int(self.offsets[-1])
        self.num_clients = int(num_clients)
        self.dtype = dtype
        self.device = device if device is not None else tree_util._default_device()
        vw = 16 // torch.empty((), dtype=dtype).element_size()
        self.row_stride = max(vw, (self.num_params + vw - 1) // vw * vw)
        from fedjax_amd import memory

        with memory.producing(self.device):  # the delta pool under memory.set_default(True)
            self.storage = torch.empty(self.num_clients, self.row_stride, dtype=dtype, device=self.device)
        if self.row_stride > self.num_params:
            self.storage[:, self.num_params:].zero_()

    # ------------------------------------------------------------------ views
    @property
    def rows(self) -> torch.Tensor:
        """[K, P] view of the deltas (row stride = ``row_stride``)."""
        return self.storage[:, : self.num_params]

    def unflatten(self, flat: torch.Tensor) -> PyTree:
        """Pytree of views into a flat P-element tensor."""
        views = [flat[o:o + n].view(s) for o, n, s in zip(self.offsets[:-1], self.sizes, self.shapes)]
        return pytree.unflatten(self.treedef, views)

    def client(self, k: int) -> PyTree:
        """Pytree of views into client k's row (write a delta through them)."""
        return self.unflatten(self.storage[k])

    def set_client(self, k: int, delta: PyTree) -> None:
        """Copy one client's delta (device or host pytree) into row k."""
        for dst, src in zip(pytree.leaves_of(self.client(k)), pytree.flatten_as(self.treedef, delta)):
            dst.copy_(tree_util._to_tensor(src), non_blocking=True)

    def fill_synthetic(self, *, seed: int = 0, amp: float = 0.01, k0: int = 0) -> "ClientDeltaSlab":
        """x[k, p] = amp * u(seed, k0 + k, p): the synthetic deltas of bench.py."""
        kernels.fill_synth(self.rows, seed=seed, amp=amp, k0=k0)
        return self

    # ------------------------------------------------------------- aggregation
    def host_weights(self, weights: Sequence) -> np.ndarray:
        """float32 weights f32(w_k) on the host."""
        if len(weights) != self.num_clients:
            raise ValueError(f"need {self.num_clients} weights, got {len(weights)}")
        return np.array([np.float32(tree_util._host_weight(x)) for x in weights], dtype=np.float32)

    def weight_vector(self, weights: Sequence) -> torch.Tensor:
        """float32 weights f32(w_k) on the device (pinned H2D, stream-ordered)."""
        return _lib.upload(torch.from_numpy(self.host_weights(weights)), self.device)

    def weighted_sum_flat(self, w_dev: torch.Tensor, *, scale=None, out: Optional[torch.Tensor] = None,
                          accumulate: bool = False, mode: str = "exact",
                          nontemporal: Optional[bool] = None, variant: int = 0,
                          reference_bf16: Optional[bool] = None) -> torch.Tensor:
        """Flat P-element fold of the slab (one launch). ``w_dev``: device weights, or host
        float32 weights (carried in the kernel arguments when the launch allows it, see
        :func:`kernels.weighted_sum_dense`). A bfloat16
        slab folds with the reference's bf16 arithmetic when ``reference_bf16`` (default:
        ``tree_util.set_bf16_semantics("reference")`` is in force and mode is exact)."""
        nbytes = self.rows.numel() * self.rows.element_size()
        nt = nbytes >= tree_util.NONTEMPORAL_MIN_BYTES if nontemporal is None else nontemporal
        if reference_bf16 is None:
            reference_bf16 = (self.dtype == torch.bfloat16 and mode == "exact"
                              and tree_util.bf16_semantics() == "reference")
        return kernels.weighted_sum_dense(
            self.rows, w_dev, scale=None if scale is None else float(np.float32(scale)), out=out,
            accumulate=accumulate, mode=mode, nontemporal=nt, variant=variant, reference_bf16=reference_bf16)

    def mean(self, weights: Sequence, *, out: Optional[torch.Tensor] = None, mode: str = "exact",
             with_norms: bool = False):
        """Weighted mean of the K rows — ``tree_mean(zip(clients, weights))`` with the
        reference's W and f32(1/W) (tree_util.py:86-96), one dense launch.

        ``with_norms=True`` also returns every client's delta l2 norm (float32[K],
        the ``delta_l2_norm`` diagnostic of examples/fed_avg.py:79-81) computed in
        the same pass over the slab: ``(mean, norms)``."""
        W = 0.0
        for x in weights:
            W += tree_util._host_weight(x)
        scale = tree_util._inverse(W)
        if with_norms and self.dtype == torch.bfloat16 and tree_util.bf16_semantics() == "reference":
            # no fused-norm kernel for the bf16 reference fold: the mean, then the norms
            if mode != "exact":
                raise ValueError("fused norms run in exact mode")
            flat = self.weighted_sum_flat(self.host_weights(weights), scale=scale, out=out)
            return self.unflatten(flat), self.l2_norms()
        if with_norms:
            if mode != "exact":
                raise ValueError("fused norms run in exact mode")
            nbytes = self.rows.numel() * self.rows.element_size()
            flat, l2sq = kernels.weighted_sum_l2_dense(
                self.rows, self.weight_vector(weights), scale=float(np.float32(scale)), out=out,
                nontemporal=nbytes >= tree_util.NONTEMPORAL_MIN_BYTES)
            return self.unflatten(flat), torch.sqrt(l2sq)
        flat = self.weighted_sum_flat(self.host_weights(weights), scale=scale, out=out, mode=mode)
        return self.unflatten(flat)

    def l2_norms(self) -> torch.Tensor:
        """Per-client delta l2 norms (float32[K]) in one pass over the slab."""
        return torch.sqrt(kernels.l2_squared_dense(self.rows))


__all__ = ["ClientDeltaSlab"]
