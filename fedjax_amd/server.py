"""Server optimizer step fused with the aggregation.

The step after the mean in every FedJAX algorithm is the server update
(examples/fed_avg.py:97-101, fedjax/algorithms/fed_avg.py:150-154):
``opt_state, params = server_optimizer.apply(mean_delta, opt_state, params)``
with any of ``fedjax.optimizers.sgd``, ``adam``, ``adagrad``, ``rmsprop`` (centered without momentum too),
``yogi`` or ``adafactor`` (fedjax/core/optimizers.py:117-348, optax).
:func:`fused_mean_update` folds the round's client deltas and applies that update
in the same kernel (``fjagg_server_update_dense``): the mean stays in registers,
params / momentum / second moments are read and written once.

Arithmetic restates optax's op order with IEEE single-precision ops; constants are
rounded to float32 on the host the way JAX's weak typing rounds Python floats.
``learning_rate`` is a float or a schedule (``ScalarOrSchedule``, optimizers.py:114):
a schedule is evaluated on the host once per round, at optax's pre-increment step count
(``optax.scale_by_schedule``), into the kernel's descriptor. :func:`ignore_grads_haiku`
(optimizers.py:69-109) freezes haiku parameters: their leaves are left out of the fused
launch, so params and optimizer state pass through untouched.
:func:`adafactor` needs whole-leaf reductions (factored second moments, block RMS), so
it runs after the fold as its own short launch chain over all leaves (include/fjopt.h).
Bitwise parity holds against the numpy restatement in tests/test_gpu_parity.py;
against XLA it is unpinned (XLA:CPU may contract mul+add, and evaluates
``b1 ** count`` with its own pow).
"""

from __future__ import annotations

import ctypes
import dataclasses
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from fedjax_amd import _lib, kernels, pytree, tree_util
from fedjax_amd.slab import ClientDeltaSlab


@dataclasses.dataclass(frozen=True)
class ServerOptimizer:
    """Hyperparameters of fedjax.optimizers.sgd / adam / adagrad / rmsprop / yogi
    (optimizers.py:117-281). ``b2`` is rmsprop's ``decay``; ``momentum`` its trace decay;
    ``init_m`` / ``init_v`` the initial values of the state (adagrad's
    initial_accumulator_value, rmsprop's initial_scale, yogi's 1e-6). ``learning_rate`` is
    a float or a schedule ``count -> float`` (ScalarOrSchedule, optimizers.py:114);
    ``frozen`` holds the haiku ``(module_name, name)`` pairs of ignore_grads_haiku."""
    kind: int
    learning_rate: Union[float, Callable[[int], float]]
    momentum: Optional[float] = None
    nesterov: bool = False
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    eps_root: float = 0.0
    init_m: float = 0.0
    init_v: float = 0.0
    frozen: Tuple[Tuple[str, str], ...] = ()
    centered: bool = False

    def lr(self, count: int) -> float:
        """The learning rate of the step whose INCREMENTED count is ``count``: a schedule is
        evaluated at the count before the step (optax.scale_by_schedule reads state.count,
        then increments it)."""
        if callable(self.learning_rate):
            return float(np.asarray(self.learning_rate(count - 1), dtype=np.float64))
        return float(self.learning_rate)

    def needs_m(self) -> bool:
        return self.kind in (_lib.OPT_MOMENTUM, _lib.OPT_ADAM, _lib.OPT_YOGI) or (
            self.kind == _lib.OPT_RMSPROP and (self.momentum is not None or self.centered))

    def needs_v(self) -> bool:
        return self.kind >= _lib.OPT_ADAM

    def init(self, params) -> dict:
        """Optimizer state (optax init, count 0) for flat float32 device params or a pytree
        of them (then m / v are pytrees of the same structure)."""
        def full(value):
            if isinstance(params, torch.Tensor):
                return torch.full_like(params, float(np.float32(value)))
            z = tree_util.tree_zeros_like(params)
            if value != 0.0:
                for x in pytree.flatten(z)[0]:
                    x.fill_(float(np.float32(value)))
            return z
        st = {"count": 0}
        if self.needs_m():
            st["m"] = full(self.init_m)
        if self.needs_v():
            st["v"] = full(self.init_v)
        return st

    def descriptor(self, count: int) -> _lib.ServerOpt:
        """struct fjagg_server_opt for the step whose incremented count is ``count``."""
        f32 = np.float32
        d = _lib.ServerOpt()
        d.kind = self.kind
        d.nesterov = int(self.nesterov)
        d.neg_lr = f32(-self.lr(count))  # scale_by_learning_rate: scale(-lr) / scale_by_schedule(-lr(t))
        d.decay = f32(self.momentum or 0.0)
        d.one_minus_b1, d.b1 = f32(1 - self.b1), f32(self.b1)
        d.one_minus_b2, d.b2 = f32(1 - self.b2), f32(self.b2)
        # bias_correction: 1 - decay ** count, in float32
        d.bc1 = f32(1) - np.power(f32(self.b1), f32(count))
        d.bc2 = f32(1) - np.power(f32(self.b2), f32(count))
        d.eps, d.eps_root = f32(self.eps), f32(self.eps_root)
        d.flags = 0
        if self.kind == _lib.OPT_RMSPROP:
            d.flags = (_lib.OPT_F_MOMENTUM if self.momentum is not None else 0) | (
                _lib.OPT_F_CENTERED if self.centered else 0)
        return d


def sgd(learning_rate: float, momentum: Optional[float] = None, nesterov: bool = False) -> ServerOptimizer:
    """fedjax.optimizers.sgd (optimizers.py:227-250)."""
    kind = _lib.OPT_SGD if momentum is None else _lib.OPT_MOMENTUM
    return ServerOptimizer(kind, learning_rate, momentum=momentum, nesterov=nesterov)


def adam(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
         eps_root: float = 0.0) -> ServerOptimizer:
    """fedjax.optimizers.adam (optimizers.py:148-178)."""
    return ServerOptimizer(_lib.OPT_ADAM, learning_rate, b1=b1, b2=b2, eps=eps, eps_root=eps_root)


def adagrad(learning_rate: float, initial_accumulator_value: float = 0.1, eps: float = 1e-6) -> ServerOptimizer:
    """fedjax.optimizers.adagrad (optimizers.py:117-145): optax.scale_by_rss, then -lr."""
    return ServerOptimizer(_lib.OPT_ADAGRAD, learning_rate, eps=eps, init_v=initial_accumulator_value)


def rmsprop(learning_rate: float, decay: float = 0.9, eps: float = 1e-8, initial_scale: float = 0.,
            centered: bool = False, momentum: Optional[float] = None, nesterov: bool = False) -> ServerOptimizer:
    """fedjax.optimizers.rmsprop (optimizers.py:181-224) = optax.rmsprop: scale_by_rms
    (centered: scale_by_stddev, state m = mu), scale_by_learning_rate, then [trace] of the
    lr-scaled update (state m = the trace)."""
    if centered and momentum is not None:
        raise NotImplementedError("centered rmsprop with momentum keeps three states (mu, nu, trace); the fused "
                                  "server step has two")
    return ServerOptimizer(_lib.OPT_RMSPROP, learning_rate, momentum=momentum, nesterov=nesterov, b2=decay,
                           eps=eps, init_v=initial_scale, centered=bool(centered))


def yogi(learning_rate: float, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-3) -> ServerOptimizer:
    """fedjax.optimizers.yogi (optimizers.py:253-281): optax.scale_by_yogi (eps_root 0,
    initial_accumulator_value 1e-6 for both moments), then -lr."""
    return ServerOptimizer(_lib.OPT_YOGI, learning_rate, b1=b1, b2=b2, eps=eps, init_m=1e-6, init_v=1e-6)


def ignore_grads_haiku(optimizer, non_trainable_names: List[Tuple[str, str]]):
    """fedjax.optimizers.ignore_grads_haiku (optimizers.py:69-109): ``optimizer`` with the
    haiku parameters ``params[module_name][name]`` for every pair in ``non_trainable_names``
    frozen. The reference maps them to ``None`` for the update and puts the old values
    back; here their leaves are left out of the fused launch (no fold, no update), so the
    params and the optimizer state of those leaves pass through untouched. The step count
    still advances, as optax's does."""
    return dataclasses.replace(optimizer, frozen=tuple((str(m), str(n)) for m, n in non_trainable_names))


def _frozen_leaves(opt, params, treedef) -> np.ndarray:
    """bool [L]: leaf l (flatten order of ``treedef``) is one of opt.frozen. ``params`` is
    a haiku-style ``{module_name: {name: leaf}}`` mapping, as the reference requires."""
    L = treedef.num_leaves
    if not opt.frozen:
        return np.zeros(L, dtype=bool)
    for m, n in opt.frozen:  # optimizers.py:103 indexes params[module_name][name]
        params[m][n]  # noqa: B018 - KeyError for a name the params do not have
    marks = {m: ({n: (m, n) in opt.frozen for n in sub} if isinstance(sub, dict) else False)
             for m, sub in params.items()}
    mask = np.array(pytree.flatten_as(treedef, marks), dtype=bool)
    assert mask.size == L
    return mask


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
    if isinstance(opt, Adafactor):  # needs whole-leaf reductions: the mean first, then the step
        # (state = opt.init(slab.unflatten(params)): optax's per-leaf statistics)
        mean = mean_out if mean_out is not None else torch.empty_like(params)
        slab.mean(weights, out=mean)
        return opt.apply(slab.unflatten(mean), state, slab.unflatten(params))[0]
    _require_state(opt, state)
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
    # ignore_grads_haiku: frozen leaves are column ranges of the slab; the fused step runs
    # over each maximal run of trainable leaves (one launch without frozen leaves)
    frozen = _frozen_leaves(opt, slab.unflatten(params), slab.treedef)
    runs, l0 = [], 0
    for l in range(len(frozen) + 1):
        if l == len(frozen) or frozen[l]:
            if l > l0:
                runs.append((int(slab.offsets[l0]), int(slab.offsets[l])))
            l0 = l + 1
    esz = rows.element_size()
    ptr = lambda t, o: None if t is None else t.data_ptr() + 4 * o
    for c0, c1 in runs:
        if c1 == c0:
            continue
        _lib.call("fjagg_server_update_dense", kernels.dtype_code(rows.dtype), rows.data_ptr() + esz * c0, ld,
                  rows.shape[0], c1 - c0, w_dev.data_ptr(), float(scale), ctypes.byref(desc),
                  params.data_ptr() + 4 * c0, ptr(m, c0), ptr(v, c0), ptr(mean_out, c0), _lib.NONTEMPORAL if nt else 0,
                  torch.cuda.current_stream(params.device).cuda_stream)
    if mean_out is not None:  # the mean of frozen leaves too (no update consumes it)
        for l in np.flatnonzero(frozen):
            c0, c1 = int(slab.offsets[l]), int(slab.offsets[l + 1])
            if c1 > c0:
                kernels.weighted_sum_dense(rows[:, c0:c1], w_dev, scale=float(scale), out=mean_out[c0:c1],
                                           nontemporal=nt)
    new = dict(state)
    new["count"] = count
    return new


_UPDATE_ADDRS = None


def _update_addrs():
    """(fjagg_ptrs_plan_leaves, fjagg_server_update_ptrs) addresses for fjhost.server_pairs."""
    global _UPDATE_ADDRS
    if _UPDATE_ADDRS is None:
        lib = _lib.load()
        _UPDATE_ADDRS = tuple(ctypes.cast(getattr(lib, f), ctypes.c_void_p).value
                              for f in ("fjagg_ptrs_plan_leaves", "fjagg_server_update_ptrs"))
    return _UPDATE_ADDRS


def _require_state(opt: "ServerOptimizer", state: dict) -> None:
    """The moments ``opt``'s rule reads must be in ``state`` (e.g. a state from
    ``rmsprop(centered=False).init`` given to a centered rmsprop has no 'm'): raise instead
    of launching the fused step with an absent state tree."""
    for key, need in (("m", opt.needs_m()), ("v", opt.needs_v())):
        if need and state.get(key) is None:
            raise ValueError(f"optimizer state has no {key!r}, which this optimizer's update reads; "
                             f"use opt.init(params) of the same optimizer")


def fused_tree_mean_update(pytrees_and_weights, opt: ServerOptimizer, params, state: dict, *,
                           mean_out=None, nontemporal: Optional[bool] = None) -> dict:
    """:func:`fused_mean_update` on the pytree path: ``tree_mean`` of the clients' delta
    pytrees (tree_util.py:76-96) and ``opt``'s update of the ``params`` pytree (float32
    device leaves, the deltas' structure and shapes, updated in place) in ONE kernel
    (``fjagg_server_update_ptrs``) — examples/fed_avg.py:82 + :97-101. ``state`` is
    ``opt.init(params)``; returns the new state. ``mean_out`` (optional pytree of float32
    leaves) also receives the mean."""
    if isinstance(opt, Adafactor):  # needs whole-leaf reductions: the mean first, then the step
        mean = tree_util.tree_mean(pytrees_and_weights) if mean_out is None else None
        if mean_out is not None:
            trees, weights, W = tree_util._collect_pairs(pytrees_and_weights)
            if not trees:
                raise ValueError("no clients to aggregate")
            td, rows = tree_util._client_table(trees)
            tree_util._fold(rows, weights, scale=tree_util._inverse(W), out=pytree.flatten_as(td, mean_out),
                            validated=True)
            mean = mean_out
        elif mean is None:
            raise ValueError("no clients to aggregate")
        return opt.apply(mean, state, params)[0]
    _require_state(opt, state)
    if (not opt.frozen and nontemporal is None and type(pytrees_and_weights) in (list, tuple)
            and pytrees_and_weights):
        # the common case in one native call (fjhost.server_pairs): same image, same launch
        count = state["count"] + 1
        desc = opt.descriptor(count)
        rc = _lib.host().server_pairs(pytrees_and_weights, params, state.get("m"), state.get("v"), mean_out,
                                      ctypes.addressof(desc), float(tree_util.NONTEMPORAL_MIN_BYTES),
                                      *_update_addrs())
        if rc is not None:
            _lib.check(rc, "fjagg_server_update_ptrs")
            new = dict(state)
            new["count"] = count
            return new
    trees, weights, W = tree_util._collect_pairs(pytrees_and_weights)
    if not trees:
        raise ValueError("no clients to aggregate")
    td, rows = tree_util._client_table(trees)
    row0 = rows[0]
    K, L = len(trees), len(row0)
    if L == 0:
        return dict(state, count=state["count"] + 1)
    dt = row0[0].dtype
    if dt not in (torch.float32, torch.bfloat16) or any(x.dtype != dt for x in row0):
        raise TypeError("the fused server step takes float32 or bfloat16 deltas of one dtype")
    device = row0[0].device

    def leaves(tree, what):
        ls = pytree.flatten_as(td, tree)
        for x, d in zip(ls, row0):
            if not (isinstance(x, torch.Tensor) and x.dtype == torch.float32 and x.is_contiguous()
                    and x.device == device and x.shape == d.shape):
                raise ValueError(f"{what} leaves must be contiguous float32 device tensors shaped like the deltas")
        return ls

    p = leaves(params, "params")
    m = leaves(state["m"], "state m") if "m" in state else None
    v = leaves(state["v"], "state v") if "v" in state else None
    mo = leaves(mean_out, "mean_out") if mean_out is not None else None
    count = state["count"] + 1  # optax safe_int32_increment
    desc = opt.descriptor(count)
    in_c = kernels.dtype_code(dt)
    # ignore_grads_haiku: a frozen leaf gets no workgroups (leaf_n 0 in the plan), so its
    # params and state are never read or written
    frozen = _frozen_leaves(opt, params, td)
    leaf_n = np.array([0 if f else x.numel() for x, f in zip(row0, frozen)], dtype=np.int64)
    in_ptrs = tree_util._ptr_table(rows)
    out_ptrs = np.array([x.data_ptr() for x in p], dtype=np.int64)
    st = np.zeros(3 * L, dtype=np.int64)
    for i, ls in enumerate((m, v, mo)):
        if ls is not None:
            st[i * L:(i + 1) * L] = [x.data_ptr() for x in ls]
    blocks, unaligned = tree_util._leaf_plan(in_c, leaf_n, in_ptrs, out_ptrs, st.reshape(3, L), device)
    w32 = weights.f32 if isinstance(weights, tree_util._Weights) else np.array(
        [np.float32(w) for w in weights], np.float32)
    w_words = np.zeros((K + 1) // 2, dtype=np.int64)
    w_words.view(np.uint8)[:4 * K] = w32.view(np.uint8)
    image = np.concatenate([in_ptrs.ravel(), out_ptrs, leaf_n, blocks, w_words, st])
    image_dev = _lib.upload(torch.from_numpy(image), device)
    base = image_dev.data_ptr()
    w_ptr = base + 8 * (K * L + 2 * L + blocks.size)
    st_ptr = w_ptr + 8 * w_words.size
    nbytes = int(leaf_n.sum()) * K * row0[0].element_size()
    nt = nbytes >= tree_util.NONTEMPORAL_MIN_BYTES if nontemporal is None else nontemporal
    flags = (_lib.NONTEMPORAL if nt else 0) | (_lib.UNALIGNED if unaligned else 0)
    if blocks.size:
        _lib.call("fjagg_server_update_ptrs", in_c, base, L, K, blocks.size // 2, w_ptr,
                  float(np.float32(tree_util._inverse(W))), ctypes.byref(desc), st_ptr, flags,
                  torch.cuda.current_stream(device).cuda_stream)
    if mo is not None and frozen.any():  # the mean of frozen leaves too (no update consumes it)
        idx = np.flatnonzero(frozen)
        if isinstance(rows, tree_util._Table):  # every leaf is already the caller's device tensor
            sub = [[pytree.flatten_as(td, t)[i] for i in idx] for t in trees]
        else:
            sub = [[r[i] for i in idx] for r in rows]
        tree_util._fold(sub, weights, scale=tree_util._inverse(W), out=[mo[i] for i in idx])
    new = dict(state)
    new["count"] = count
    return new


# --------------------------------------------------------------------------- adafactor
def _factored_dims(shape, factored: bool, min_dim_size_to_factor: int):
    """optax factorized._factored_dims: (d1, d0) = the second-largest and the largest axis
    (numpy argsort order, as optax computes it), or None."""
    if not factored or len(shape) < 2:
        return None
    sorted_dims = np.argsort(shape)
    if shape[sorted_dims[-2]] < min_dim_size_to_factor:
        return None
    return int(sorted_dims[-2]), int(sorted_dims[-1])


@dataclasses.dataclass(frozen=True)
class Adafactor:
    """fedjax.optimizers.adafactor (optimizers.py:284-348): optax.adafactor's chain
    (include/fjopt.h) on the GPU, ``fjopt_adafactor_step`` over every leaf at once.

    ``init(params)`` gives optax's state shapes (per leaf ``v_row`` / ``v_col`` for factored
    leaves, ``v`` otherwise, each with a (1,) placeholder for the other kind, and the ema
    ``m`` when ``momentum`` is set); ``apply(grads, state, params)`` updates ``params`` and
    the state tensors in place and returns ``(state, params)`` (the reference's
    ``Optimizer.apply`` returns new arrays). Params, grads and state are float32 device
    tensors. Means are float64 sums in a fixed order (parity unpinned)."""
    learning_rate: Union[None, float, Callable[[int], float]]
    min_dim_size_to_factor: int = 128
    decay_rate: float = 0.8
    decay_offset: int = 0
    multiply_by_parameter_scale: bool = True
    clipping_threshold: Optional[float] = 1.0
    momentum: Optional[float] = None
    dtype_momentum: torch.dtype = torch.float32
    weight_decay_rate: Optional[float] = None
    eps: float = 1e-30
    factored: bool = True
    weight_decay_mask: object = None
    frozen: Tuple[Tuple[str, str], ...] = ()
    _plans: dict = dataclasses.field(default_factory=dict, compare=False, repr=False)

    def init(self, params) -> dict:
        leaves, td = pytree.flatten(params)
        vr, vc, v, m = [], [], [], []
        for p in leaves:
            if not (isinstance(p, torch.Tensor) and p.dtype == torch.float32):
                raise TypeError("adafactor takes float32 tensor params")
            z1 = torch.zeros(1, dtype=torch.float32, device=p.device)
            fd = _factored_dims(tuple(p.shape), self.factored, self.min_dim_size_to_factor)
            if fd is not None:
                d1, d0 = fd
                vr.append(torch.zeros(tuple(np.delete(p.shape, d0)), dtype=torch.float32, device=p.device))
                vc.append(torch.zeros(tuple(np.delete(p.shape, d1)), dtype=torch.float32, device=p.device))
                v.append(z1)
            else:
                vr.append(z1)
                vc.append(z1.clone())
                v.append(torch.zeros_like(p))
            if self.momentum is not None:
                m.append(torch.zeros_like(p))
        st = {"count": 0, "v_row": pytree.unflatten(td, vr), "v_col": pytree.unflatten(td, vc),
              "v": pytree.unflatten(td, v)}
        if self.momentum is not None:
            if self.dtype_momentum != torch.float32:
                raise NotImplementedError("the fused adafactor keeps a float32 momentum (dtype_momentum)")
            st["m"] = pytree.unflatten(td, m)
        return st

    def hparams(self, count: int) -> _lib.AfHparams:
        """struct fjopt_af_hparams of the step taken at (pre-increment) count ``count``."""
        f32 = np.float32
        h = _lib.AfHparams()
        d = f32(1) - np.power(f32(count - self.decay_offset + 1), f32(-self.decay_rate))  # _decay_rate_pow
        h.decay_rate_t, h.one_minus_decay, h.eps = d, f32(1) - d, f32(self.eps)
        h.clip = int(self.clipping_threshold is not None)
        h.clip_threshold = f32(self.clipping_threshold or 1.0)
        h.has_lr = int(self.learning_rate is not None)
        if self.learning_rate is not None:  # scale_by_schedule reads its pre-increment count
            lr = self.learning_rate(count) if callable(self.learning_rate) else self.learning_rate
            h.lr = f32(np.asarray(lr, dtype=np.float64))
        h.param_scale, h.min_scale = int(bool(self.multiply_by_parameter_scale)), f32(1e-3)
        h.momentum = int(self.momentum is not None)
        if self.momentum is not None:
            h.mom_decay, h.one_minus_mom = f32(self.momentum), f32(1.0 - self.momentum)
        h.weight_decay = int(self.weight_decay_rate is not None)
        h.wd = f32(self.weight_decay_rate or 0.0)
        return h

    def _mask(self, params, td) -> List[bool]:
        if self.weight_decay_rate is None or self.weight_decay_mask is None:
            return [True] * td.num_leaves
        mask = self.weight_decay_mask(params) if callable(self.weight_decay_mask) else self.weight_decay_mask
        flags = pytree.flatten_as(td, mask)  # a full tree of booleans (prefix trees are not supported)
        return [bool(f) for f in flags]

    def apply(self, grads, state: dict, params):
        """One step: ``(state, params)`` with params and state updated in place."""
        p, td = pytree.flatten(params)
        g = pytree.flatten_as(td, grads)
        vr = pytree.flatten_as(td, state["v_row"])
        vc = pytree.flatten_as(td, state["v_col"])
        v = pytree.flatten_as(td, state["v"])
        m = pytree.flatten_as(td, state["m"]) if self.momentum is not None else [None] * len(p)
        count = int(state["count"])
        hp = self.hparams(count)
        if p:
            device = p[0].device
            mask = self._mask(params, td)
            frozen = _frozen_leaves(self, params, td)  # ignore_grads_haiku: left out of the step
            recs = []
            for l, (pl, gl) in enumerate(zip(p, g)):
                if frozen[l]:
                    continue
                for what, t in (("grads", gl), ("params", pl)):
                    if not (isinstance(t, torch.Tensor) and t.dtype == torch.float32 and t.is_contiguous()
                            and t.device == device and t.shape == pl.shape):
                        raise ValueError(f"leaf {l}: {what} must be contiguous float32 tensors on {device} "
                                         f"shaped like the params")
                rec = _lib.AfLeaf()
                rec.g, rec.p, rec.n = gl.data_ptr(), pl.data_ptr(), pl.numel()
                shape = tuple(pl.shape)
                fd = _factored_dims(shape, self.factored, self.min_dim_size_to_factor)
                if fd is not None:
                    d1, d0 = fd
                    lo, hi = min(d0, d1), max(d0, d1)
                    prod = lambda s: int(np.prod(s, dtype=np.int64))
                    dims = (prod(shape[:lo]), shape[lo], prod(shape[lo + 1:hi]), shape[hi], prod(shape[hi + 1:]))
                    if tuple(vr[l].shape) != tuple(np.delete(shape, d0)) or \
                            tuple(vc[l].shape) != tuple(np.delete(shape, d1)):
                        raise ValueError(f"leaf {l}: state v_row / v_col do not have optax's factored shapes")
                    rec.factored, rec.d0_is_lo = 1, int(d0 == lo)
                    rec.v_row, rec.v_col = vr[l].data_ptr(), vc[l].data_ptr()
                else:
                    dims = (1, pl.numel(), 1, 1, 1)
                    if v[l].shape != pl.shape:
                        raise ValueError(f"leaf {l}: state v must have the params' shape")
                    rec.v = v[l].data_ptr()
                for s_ in (vr[l], vc[l], v[l]) + ((m[l],) if m[l] is not None else ()):
                    if s_.dtype != torch.float32 or not s_.is_contiguous() or s_.device != device:
                        raise ValueError(f"leaf {l}: state must be contiguous float32 tensors on {device}")
                if m[l] is not None:
                    if m[l].shape != pl.shape:
                        raise ValueError(f"leaf {l}: state m must have the params' shape")
                    rec.m = m[l].data_ptr()
                rec.dims[:] = dims
                rec.decay_weights = int(mask[l])
                recs.append(rec)
            # The plan is keyed on what shapes it (leaf shapes, factoring, flags, mask) and on
            # the stream, not on the pointers: the mean delta is a fresh tensor every round
            # (ADVICE r3). The pointers are rewritten into the cached table, and uploaded into
            # its device copy on this stream, only when they change; the workspace belongs to
            # the (plan, stream) entry, so calls on two streams never share one.
            stream = torch.cuda.current_stream(device)
            shape_key = []
            for rec in recs:
                z = _lib.AfLeaf.from_buffer_copy(rec)
                z.g = z.p = z.v_row = z.v_col = z.v = z.m = None
                shape_key.append(bytes(z))
            key = (hp.clip, hp.param_scale, hp.momentum, hp.weight_decay, hp.has_lr, tuple(shape_key),
                   device, stream.cuda_stream)
            ptr_key = tuple(bytes(rec) for rec in recs)
            if not recs:
                return dict(state, count=count + 1), params
            plan = self._plans.get(key)
            lib = _lib.load()
            arr = None
            if plan is None:
                arr = (_lib.AfLeaf * len(recs))(*recs)
                ws_bytes = ctypes.c_int64()
                words = int(lib.fjopt_adafactor_plan(arr, len(recs), ctypes.byref(hp), None, 0, ctypes.byref(ws_bytes)))
                _lib.check(min(words, 0), "fjopt_adafactor_plan")
                table = np.zeros(max(words, 1), dtype=np.int64)
                table_dev = torch.empty(table.size, dtype=torch.int64, device=device)
                ws = torch.empty(max(int(ws_bytes.value), 1), dtype=torch.uint8, device=device)
                if len(self._plans) >= 8:
                    self._plans.clear()
                plan = self._plans[key] = [None, table, table_dev, ws]
            if plan[0] != ptr_key:  # new pointers: rewrite the host table, upload it on this stream
                if arr is None:
                    arr = (_lib.AfLeaf * len(recs))(*recs)
                ws_bytes = ctypes.c_int64()
                words = int(lib.fjopt_adafactor_plan(arr, len(recs), ctypes.byref(hp), plan[1].ctypes.data,
                                                     plan[1].size, ctypes.byref(ws_bytes)))
                _lib.check(min(words, 0), "fjopt_adafactor_plan")
                plan[2].copy_(_lib.upload(torch.from_numpy(plan[1]), plan[2].device), non_blocking=True)
                plan[0] = ptr_key
            _, table, table_dev, ws = plan
            _lib.call("fjopt_adafactor_step", table.ctypes.data, table_dev.data_ptr(), ctypes.byref(hp),
                      ws.data_ptr(), ws.numel(), stream.cuda_stream)
        new = dict(state)
        new["count"] = count + 1
        return new, params


def adafactor(learning_rate, min_dim_size_to_factor: int = 128, decay_rate: float = 0.8, decay_offset: int = 0,
              multiply_by_parameter_scale: bool = True, clipping_threshold: Optional[float] = 1.0,
              momentum: Optional[float] = None, dtype_momentum=torch.float32,
              weight_decay_rate: Optional[float] = None, eps: float = 1e-30, factored: bool = True,
              weight_decay_mask=None) -> Adafactor:
    """fedjax.optimizers.adafactor (optimizers.py:284-348), same arguments and defaults."""
    return Adafactor(learning_rate, min_dim_size_to_factor, decay_rate, decay_offset, multiply_by_parameter_scale,
                     clipping_threshold, momentum, dtype_momentum, weight_decay_rate, eps, factored,
                     weight_decay_mask)


__all__ = ["Adafactor", "ServerOptimizer", "adafactor", "adagrad", "adam", "fused_mean_update",
           "fused_tree_mean_update", "ignore_grads_haiku", "rmsprop", "sgd", "yogi"]
