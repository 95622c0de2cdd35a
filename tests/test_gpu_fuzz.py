"""Seeded random sweep of the aggregation surface against the numpy oracle.

Each case draws a pytree structure (nested dicts / lists / tuples, 1-70 leaves), leaf
shapes from sizes that sit on every boundary the kernels care about (empty, 1, the 4- and
8-element units, 64 / 256 lanes, 4096-element fjtree chunks), a placement (separate
allocations, views at random element offsets into one buffer — so 4-byte but not 16-byte
aligned rows —, non-contiguous views, host numpy leaves), a leaf dtype (float32, int32,
bfloat16),
K clients, weights (Python ints, Python floats, numpy float32 scalars, a zero total) and
a sprinkle of NaN / inf / -0. Every case runs the reference surface that SURVEY §8(a)
lists and compares it with oracle/tree_util_ref.py (fedjax/core/tree_util.py:29-114
restated op for op):

* tree_mean over a list (one launch: k_ptrs, k_ptrs_narrow, element units, tails),
  over a generator (the streaming path, with a budget that forces several chunks),
  mean_aggregator().apply — bitwise;
* tree_sum — bitwise;
* the library loop s = tree_add(s, tree_weight(x, n)) ... tree_inverse_weight(s, W),
  deferred (PendingSum) and eager (fjtree launches) — bitwise;
* tree_mean_with_l2_norms — mean bitwise, norms within 2e-6 of the f64 oracle.

bfloat16 leaves are checked against the documented deviation instead of the reference's
bf16-rounded op sequence: a float32 fold rounded once, restated in numpy
here (_bf16_fold); with a strongly typed float32 weight both agree (the reference promotes
to float32).

Bitwise means equal bit patterns, except that any NaN matches any NaN (the GPU's
default NaN is positive, x86's negative; the reference gives whichever its backend does).
"""
import math

import os

import numpy as np
import pytest
import torch

import fedjax_amd
from fedjax_amd import pytree, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025,
         4095, 4096, 4097, 8191, 12289, 65537]
# FJ_FUZZ_CASES / FJ_FUZZ_SEED0: a longer campaign over other seeds (the suite runs the defaults)
NCASES = int(os.environ.get("FJ_FUZZ_CASES", "200"))
SEED0 = int(os.environ.get("FJ_FUZZ_SEED0", "1000"))


def _shape(rs, n):
    """A 1-3 dim shape with n elements."""
    if n == 0 or rs.rand() < 0.5:
        return (n,)
    for d in (2, 3, 4, 5, 7, 8, 16, 31, 64):
        if n % d == 0 and rs.rand() < 0.5:
            return (d, n // d)
    return (n,)


def _structure(rs, nleaves):
    """A nested container holding leaf slots 0..nleaves-1 (dict keys sorted != insertion)."""
    slots = list(range(nleaves))

    def build(items, depth):
        if len(items) == 1 and (depth > 0 or rs.rand() < 0.3):
            return ("leaf", items[0])
        kind = rs.choice(["dict", "list", "tuple"]) if depth < 3 else "dict"
        parts = max(1, min(len(items), int(rs.randint(1, 5))))
        cuts = sorted(rs.choice(np.arange(1, len(items)), size=parts - 1, replace=False)) if len(items) > 1 and parts > 1 else []
        groups = [items[a:b] for a, b in zip([0] + list(cuts), list(cuts) + [len(items)])]
        kids = [build(g, depth + 1) for g in groups]
        if kind == "dict":
            keys = ["k%02d" % v for v in rs.permutation(100)[:len(kids)]]
            return ("dict", dict(zip(keys, kids)))
        return (kind, kids)
    return build(slots, 0)


def _realize(node, leaves):
    kind, v = node
    if kind == "leaf":
        return leaves[v]
    if kind == "dict":
        return {k: _realize(c, leaves) for k, c in v.items()}
    kids = [_realize(c, leaves) for c in v]
    return kids if kind == "list" else tuple(kids)


def _bf16_bits(a):
    """float32 -> bfloat16 bits, round to nearest even (NaN stays NaN)."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(np.isnan(a), np.uint16(0x7FC0), r)


def _bf16_f32(bits):
    return (np.asarray(bits, np.uint32) << 16).view(np.float32)


def _values(rs, n, dtype, special):
    if dtype == np.int32:
        return rs.randint(-1000, 1000, size=n).astype(np.int32)
    a = ((rs.rand(n) * 2 - 1) * 10.0 ** rs.randint(-3, 2)).astype(np.float32)
    if special and n:
        for v in (np.nan, np.inf, -np.inf, -0.0):
            if rs.rand() < 0.3:
                a[rs.randint(n)] = v
    if dtype == "bf16":  # float32 arrays holding bfloat16 values (exact)
        a = _bf16_f32(_bf16_bits(a))
    return a


def _case(seed):
    rs = np.random.RandomState(seed)
    nleaves = 70 if seed % 12 == 5 else int(rs.choice([1, 2, 3, 5, 8, 12, 40], p=[.12, .12, .12, .16, .2, .2, .08]))
    K = int(rs.choice([1, 2, 3, 5, 16, 17, 33, 64, 130]))
    u = rs.rand()
    dtype = np.int32 if u < 0.12 else ("bf16" if u < 0.24 else np.float32)
    sizes = [int(rs.choice(SIZES)) for _ in range(nleaves)]
    budget = 6_000_000 // max(1, K)  # keep the numpy oracle quick
    while sum(sizes) > budget:
        i = int(np.argmax(sizes))
        sizes[i] //= 3
    shapes = [_shape(rs, n) for n in sizes]
    struct = _structure(rs, nleaves)
    placement = rs.choice(["separate", "offset_views", "noncontig", "host"], p=[.4, .35, .1, .15])
    if dtype == "bf16" and placement == "host":
        placement = "separate"  # numpy has no bfloat16
    wkind = rs.choice(["int", "float", "np32", "mixed", "zero"], p=[.35, .25, .15, .15, .1])
    special = dtype != np.int32 and rs.rand() < 0.2
    host = [[_values(rs, n, dtype, special).reshape(s) for n, s in zip(sizes, shapes)] for _ in range(K)]
    if wkind == "int":
        ws = [int(v) for v in rs.randint(1, 501, size=K)]
    elif wkind == "float":
        ws = [float(v) for v in rs.rand(K) * 3]
    elif wkind == "np32":
        ws = [np.float32(v) for v in rs.rand(K) * 3]
    elif wkind == "mixed":
        ws = [int(rs.randint(1, 9)) if rs.rand() < 0.5 else float(rs.rand()) for _ in range(K)]
    else:
        ws = [0] * K
    return dict(rs=rs, K=K, dtype=dtype, shapes=shapes, struct=struct, placement=placement, host=host,
                ws=ws, wkind=wkind)


def _place(c, dev):
    """Client pytrees (torch device tensors or numpy) for the case's placement."""
    rs, out = c["rs"], []
    tdt = {np.int32: torch.int32, np.float32: torch.float32, "bf16": torch.bfloat16}[c["dtype"]]

    def dev_leaf(a):
        if tdt is torch.bfloat16:
            return torch.from_numpy(_bf16_bits(a).view(np.int16)).view(torch.bfloat16).to(dev)
        return torch.from_numpy(a.copy()).to(dev)
    for leaves in c["host"]:
        if c["placement"] == "host":
            xs = [np.array(a) for a in leaves]
        elif c["placement"] == "separate":
            xs = [dev_leaf(a) for a in leaves]
        elif c["placement"] == "offset_views":
            total = sum(a.size for a in leaves) + 4 * len(leaves) + 3
            buf = torch.empty(total, dtype=tdt, device=dev)
            off, xs = int(rs.randint(0, 4)), []
            for a in leaves:
                v = buf[off:off + a.size].view(a.shape)
                v.copy_(dev_leaf(a))
                xs.append(v)
                off += a.size + int(rs.randint(0, 4))
        else:  # non-contiguous: every other element of a buffer twice as long
            xs = []
            for a in leaves:
                b = torch.zeros(2 * a.size, dtype=tdt, device=dev)
                b[::2] = dev_leaf(a.reshape(-1))
                xs.append(b[::2].view(a.shape) if a.ndim == 1 else b[::2].reshape(a.shape))
        out.append(_realize(c["struct"], xs))
    return out


def _rnd_bf16(a):
    return _bf16_f32(_bf16_bits(a))


def _bf16_ref_fold(np_trees, ws, scale, zero_init=False):
    """The reference's bf16 sequence: t_k = bf16(x_k * bf16(f32(w_k))), s_0 = t_0 (or
    bf16(0 + t_0) for the running sum from tree_zeros_like), s_k = bf16(s + t_k),
    y = bf16(s * bf16(f32(scale))); bfloat16 bits out."""
    per = [ref.flatten(t)[0] for t in np_trees]
    out = []
    for l in range(len(per[0])):
        s = np.zeros(per[0][l].shape, np.float32) if zero_init else None
        for k, w in enumerate(ws):
            t = _rnd_bf16(per[k][l].astype(np.float32) * _rnd_bf16(np.float32(w)))
            s = t if s is None else _rnd_bf16(s + t)
        if scale is not None:
            s = _rnd_bf16(s * _rnd_bf16(np.float32(scale)))
        out.append(_bf16_bits(s))
    return ref.unflatten(ref.flatten(np_trees[0])[1], out)


def _np_leaves(t):
    def host(x):
        if isinstance(x, torch.Tensor):
            x = x.detach().cpu()
            return x.view(torch.int16).numpy().view(np.uint16) if x.dtype == torch.bfloat16 else x.numpy()
        return np.asarray(x)
    return [host(x).reshape(-1) for x in pytree.leaves_of(t)]


def _bf16_fold(np_trees, ws, scale, out_bf16):
    """The documented bf16 semantics (tree_util module docstring): fold in
    float32 — t_k = fl(x_k * f32(w_k)), s_0 = t_0, s_k = fl(s_{k-1} + t_k), y = fl(s *
    f32(scale)) — and round once to bfloat16 (float32 out when a weight is strongly typed)."""
    per = [ref.flatten(t)[0] for t in np_trees]
    out = []
    for l in range(len(per[0])):
        s = None
        for k, w in enumerate(ws):
            t = per[k][l].astype(np.float32) * np.float32(w)
            s = t if s is None else s + t
        if scale is not None:
            s = s * np.float32(scale)
        out.append(_bf16_bits(s) if out_bf16 else s.astype(np.float32))
    return ref.unflatten(ref.flatten(np_trees[0])[1], out)


def _same(got, want, what):
    g, w = _np_leaves(got), [np.asarray(x).reshape(-1) for x in ref.flatten(want)[0]]
    assert len(g) == len(w), what
    for i, (a, b) in enumerate(zip(g, w)):
        assert a.dtype == b.dtype, f"{what}: leaf {i} dtype {a.dtype} != {b.dtype}"
        if a.dtype == np.float32:
            nan = np.isnan(a) & np.isnan(b)
            ok = (a.view(np.uint32) == b.view(np.uint32)) | nan
        elif a.dtype == np.uint16:  # bfloat16 bits
            nan = np.isnan(_bf16_f32(a)) & np.isnan(_bf16_f32(b))
            ok = (a == b) | nan
        else:
            ok = a == b
        assert ok.all(), f"{what}: leaf {i} differs at {np.flatnonzero(~ok)[:5]}"


@pytest.mark.filterwarnings("ignore::RuntimeWarning")  # inf - inf in the oracle's numpy
@pytest.mark.parametrize("seed", range(NCASES))
def test_random_case_matches_oracle(cuda, seed, monkeypatch):
    c = _case(SEED0 + seed)
    trees = _place(c, cuda)
    np_trees = [_realize(c["struct"], leaves) for leaves in c["host"]]
    ws, K = c["ws"], c["K"]
    bf16 = c["dtype"] == "bf16"
    strong = any(isinstance(w, np.generic) for w in ws)
    if bf16:
        W = 0.0
        for w in ws:
            W += w  # tree_util.py:95
        want = _bf16_fold(np_trees, ws, (1.0 / W) if W > 0.0 else 0.0, out_bf16=not strong)
        want_sum = _bf16_fold(np_trees, [1] * K, None, out_bf16=True)
    else:
        want = ref.tree_mean(list(zip(np_trees, ws)))
        want_sum = ref.tree_sum(np_trees)
    _same(tu.tree_mean(list(zip(trees, ws))), want, "tree_mean(list)")
    # the idle-stream pipeline (tree_util._tree_mean_pipelined) forced on whatever this case
    # is: chunks of about a third of the clients, each accumulating into the first's sums
    with monkeypatch.context() as mp:
        mp.setattr(tu, "_PIPELINE_MIN_BYTES", 0)
        mp.setattr(tu, "_NARROW_MAX_BYTES", 0)
        mp.setattr(tu, "_CHUNK_WALK_US", 0.0)
        mp.setattr(tu, "_PIPELINE_CHUNK", max(1, K // 3))
        mp.setattr(tu, "_BUSY_UNTIL", [0.0])
        tu._mean_config()  # (the builtin tree_mean's copy of these settings)
        try:
            torch.cuda.synchronize()
            _same(tu.tree_mean(list(zip(trees, ws))), want, "tree_mean(list), pipelined")
        finally:
            mp.undo()
            tu._mean_config()
    # generator input: chunks of about two clients' worth of deltas
    per = max(1, sum(int(np.prod(s)) for s in c["shapes"])) * 4
    monkeypatch.setattr(tu, "STREAM_BUDGET_BYTES", 2 * per + 1)
    _same(tu.tree_mean((t, w) for t, w in zip(trees, ws)), want, "tree_mean(generator)")
    agg = fedjax_amd.aggregators.mean_aggregator()
    got, _ = agg.apply(((f"c{k}", t, w) for k, (t, w) in enumerate(zip(trees, ws))), agg.init())
    _same(got, want, "mean_aggregator().apply")
    _same(tu.tree_sum(trees), want_sum, "tree_sum")
    if bf16 and not strong:
        # the reference's own bf16 arithmetic (set_bf16_semantics("reference")): every weight,
        # 1/W, product and sum rounded to bf16 (tests/test_gpu_bf16_reference.py restates it)
        tu.set_bf16_semantics("reference")
        try:
            _same(tu.tree_mean(list(zip(trees, ws))),
                  _bf16_ref_fold(np_trees, ws, (1.0 / W) if W > 0.0 else 0.0), "tree_mean (bf16 reference)")
            _same(tu.tree_sum(trees), _bf16_ref_fold(np_trees, [1] * K, None), "tree_sum (bf16 reference)")
            s = tu.tree_zeros_like(trees[0])
            for t, w in zip(trees, ws):
                s = tu.tree_add(s, tu.tree_weight(t, w))
            _same(tu.tree_inverse_weight(s, W), _bf16_ref_fold(np_trees, ws, (1.0 / W) if W > 0.0 else 0.0,
                                                                zero_init=True), "library loop (bf16 reference)")
        finally:
            tu.set_bf16_semantics("f32")
    if c["dtype"] != np.int32 and c["placement"] != "host" and any(int(np.prod(s)) for s in c["shapes"]):
        # one pass: the mean and every client's l2 norm
        mean, norms = tu.tree_mean_with_l2_norms(list(zip(trees, ws)))
        _same(mean, want, "tree_mean_with_l2_norms")
        n64 = np.array([math.sqrt(sum(float(np.dot(a.astype(np.float64).ravel(), a.astype(np.float64).ravel()))
                                      for a in leaves)) for leaves in c["host"]])
        got = norms.cpu().numpy().astype(np.float64)
        fin = np.isfinite(n64)
        assert np.all(np.abs(got[fin] - n64[fin]) <= 2e-6 * n64[fin] + 1e-30), "l2 norms"
        assert np.all(~np.isfinite(got[~fin])), "l2 norms of non-finite deltas"
    if c["dtype"] == np.float32:
        # the library algorithms' running sum (fed_avg.py:132-146), deferred and eager
        W = 0.0
        acc = ref.tree_zeros_like(np_trees[0])
        for t, w in zip(np_trees, ws):
            acc = ref.tree_add(acc, ref.tree_weight(t, w))
            W += w
        want_loop = ref.tree_inverse_weight(acc, W)
        for deferred in (True, False):
            tu.set_deferred_sums(deferred)
            try:
                s, W2 = tu.tree_zeros_like(trees[0]), 0.0
                for t, w in zip(trees, ws):
                    s = tu.tree_add(s, tu.tree_weight(t, w))
                    W2 += w
                _same(tu.tree_inverse_weight(s, W2), want_loop, f"library loop (deferred={deferred})")
            finally:
                tu.set_deferred_sums(True)


def test_cases_cover_the_kernel_matrix():
    """The sweep reaches every plan the host can pick (checked on the case generator, so a
    change to the generator cannot silently drop a path)."""
    cs = [_case(1000 + s) for s in range(NCASES)]
    assert {c["placement"] for c in cs} == {"separate", "offset_views", "noncontig", "host"}
    assert any(c["dtype"] == np.int32 for c in cs) and any(c["dtype"] == "bf16" for c in cs)
    assert any(len(c["shapes"]) > 64 for c in cs)  # beyond one fjtree launch
    assert any(c["K"] >= 16 and sum(int(np.prod(s)) for s in c["shapes"]) * 4 <= (256 << 10) for c in cs)  # narrow
    assert any(c["wkind"] == "zero" for c in cs) and any(c["wkind"] == "np32" for c in cs)
