"""Server optimizer step fused with the aggregation.

The step after the mean in every FedJAX algorithm is the server update
(examples/fed_avg.py:97-101, fedjax/algorithms/fed_avg.py:150-154):
``opt_state, params = server_optimizer.apply(mean_delta, opt_state, params)``
with ``fedjax.optimizers.sgd`` or ``adam`` (fedjax/core/optimizers.py:148-250, optax).
:func:`fused_mean_update` folds the round's client deltas and applies that update
in the same kernel (``fjagg_server_update_dense``): the mean stays in registers,
params / momentum / second moments are read and written once.

Arithmetic restates optax's op order with IEEE single-precision ops; constants are
rounded to float32 on the host the way JAX's weak typing rounds Python floats.
Bitwise parity holds against the numpy restatement in tests/test_gpu_parity.py;
against XLA it is unpinned (XLA:CPU may contract mul+add, and evaluates
``b1 ** count`` with its own pow).
"""

from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import numpy as np
import torch

from fedjax_amd import _lib, kernels, tree_util
from fedjax_amd.slab import ClientDeltaSlab


@dataclasses.dataclass(frozen=True)
class ServerOptimizer:
    """Hyperparameters of fedjax.optimizers.sgd / adam (optimizers.py:148-250)."""
    kind: int
    learning_rate: float
    momentum: Optional[float] = None
    nesterov: bool = False
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    eps_root: float = 0.0

    def init(self, params: torch.Tensor) -> dict:
        """Optimizer state for flat float32 device params (optax init: zeros, count 0)."""
        st = {"count": 0}
        if self.kind in (_lib.OPT_MOMENTUM, _lib.OPT_ADAM):
            st["m"] = torch.zeros_like(params)
        if self.kind == _lib.OPT_ADAM:
            st["v"] = torch.zeros_like(params)
        return st

    def descriptor(self, count: int) -> _lib.ServerOpt:
        """struct fjagg_server_opt for the step whose incremented count is ``count``."""
        f32 = np.float32
        d = _lib.ServerOpt()
        d.kind = self.kind
        d.nesterov = int(self.nesterov)
        d.neg_lr = f32(-self.learning_rate)  # scale_by_learning_rate: scale(-lr)
        d.decay = f32(self.momentum or 0.0)
        d.one_minus_b1, d.b1 = f32(1 - self.b1), f32(self.b1)
        d.one_minus_b2, d.b2 = f32(1 - self.b2), f32(self.b2)
        # bias_correction: 1 - decay ** count, in float32
        d.bc1 = f32(1) - np.power(f32(self.b1), f32(count))
        d.bc2 = f32(1) - np.power(f32(self.b2), f32(count))
        d.eps, d.eps_root = f32(self.eps), f32(self.eps_root)
        return d


def sgd(learning_rate: float, momentum: Optional[float] = None, nesterov: bool = False) -> ServerOptimizer:
    """fedjax.optimizers.sgd (optimizers.py:227-250)."""
    kind = _lib.OPT_SGD if momentum is None else _lib.OPT_MOMENTUM
    return ServerOptimizer(kind, learning_rate, momentum=momentum, nesterov=nesterov)


def adam(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
         eps_root: float = 0.0) -> ServerOptimizer:
    """fedjax.optimizers.adam (optimizers.py:148-178)."""
    return ServerOptimizer(_lib.OPT_ADAM, learning_rate, b1=b1, b2=b2, eps=eps, eps_root=eps_root)


def fused_mean_update(slab: ClientDeltaSlab, weights: Sequence, opt: ServerOptimizer,
                      params: torch.Tensor, state: dict, *, mean_out: Optional[torch.Tensor] = None,
                      nontemporal: Optional[bool] = None) -> dict:
    """One server round on the GPU: mean of the slab's K deltas (tree_mean
    semantics, tree_util.py:76-96) -> ``opt`` update of ``params`` in place.

    ``params`` is the flat float32 [P] server parameter vector in the slab's leaf
    order (``slab.unflatten(params)`` gives the pytree). Returns the new state
    (moments updated in place, count incremented). ``mean_out`` optionally
    receives the mean itself.
    """
    if params.dtype != torch.float32 or params.numel() != slab.num_params or not params.is_contiguous():
        raise ValueError(f"params must be a contiguous float32 tensor of {slab.num_params} elements")
    W = 0.0
    for x in weights:
        W += tree_util._host_weight(x)
    scale = np.float32(tree_util._inverse(W))
    count = state["count"] + 1  # optax safe_int32_increment
    desc = opt.descriptor(count)
    m, v = state.get("m"), state.get("v")
    rows = slab.rows
    nbytes = rows.numel() * rows.element_size()
    nt = nbytes >= tree_util.NONTEMPORAL_MIN_BYTES if nontemporal is None else nontemporal
    w_dev = slab.weight_vector(weights)
    ld = rows.stride(0) if rows.shape[0] > 1 else rows.shape[1]
    ptr = lambda t: None if t is None else t.data_ptr()
    _lib.call("fjagg_server_update_dense", kernels.dtype_code(rows.dtype), rows.data_ptr(), ld,
              rows.shape[0], rows.shape[1], w_dev.data_ptr(), float(scale), ctypes.byref(desc),
              params.data_ptr(), ptr(m), ptr(v), ptr(mean_out), _lib.NONTEMPORAL if nt else 0,
              torch.cuda.current_stream(params.device).cuda_stream)
    new = dict(state)
    new["count"] = count
    return new


__all__ = ["ServerOptimizer", "adam", "fused_mean_update", "sgd"]
