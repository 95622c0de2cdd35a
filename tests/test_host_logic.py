"""Host logic of the product path that needs no GPU: weight semantics, dtype
rules, block planning, sharding and bucketing."""
import numpy as np
import pytest
import torch

from fedjax_amd import _lib, distributed, kernels, tree_util as tu
from oracle import tree_util_ref as ref


def test_total_weight_follows_reference_types():
    # Python numbers: f64 accumulation (tree_util.py:86,95)
    W = 0.0
    for w in [1, 2.5, 3]:
        W += tu._host_weight(w)
    assert type(W) is float and W == 6.5
    # float32 tensors/arrays: stays float32 (NEP 50 == jax weak typing)
    W = 0.0
    for w in [torch.tensor(0.1), np.float32(0.2)]:
        W += tu._host_weight(w)
    assert isinstance(W, np.float32)
    assert tu._inverse(W) == np.float32(1) / W and isinstance(tu._inverse(W), np.float32)
    assert tu._inverse(0.0) == 0.0 and tu._inverse(-3.0) == 0.0


def test_inverse_matches_oracle_mean_scale():
    for ws in ([3, 4, 5], [0.1, 0.7, 1e-3], [500] * 1024):
        W = 0.0
        for w in ws:
            W += w
        assert np.float32(tu._inverse(W)) == ref.mean_scale(ws)


def test_weight_kinds_and_leaf_rules():
    K = tu._weight_kind
    assert [K(1), K(1.0), K(np.int32(1)), K(np.float32(1))] == [0, 1, 2, 3]
    with pytest.raises(TypeError):
        K("1")
    R = tu._leaf_rule
    assert R(torch.float32, [0, 1], None) == (_lib.F32, _lib.F32, torch.float32)
    assert R(torch.bfloat16, [0, 1], 1) == (_lib.BF16, _lib.F32, torch.bfloat16)
    assert R(torch.bfloat16, [3], 1) == (_lib.BF16, _lib.F32, torch.float32)  # bf16 * strong f32
    assert R(torch.int32, [0, 2], None) == (_lib.I32, _lib.I32, torch.int32)  # tree_sum of ints
    assert R(torch.int32, [0, 0], 1) == (_lib.I32, _lib.I32, torch.float32)  # tree_mean of ints
    assert R(torch.int32, [1], None) == (_lib.I32, _lib.F32, torch.float32)  # int * 2.0


def test_leaf_canonicalisation_rules():
    assert tu._to_tensor(3).dtype == torch.int32
    assert tu._to_tensor(2.5).dtype == torch.float32
    assert tu._CANONICAL[torch.int64] == torch.int32 and tu._CANONICAL[torch.float64] == torch.float32
    with pytest.raises(TypeError):
        tu._to_tensor(True)


def _decode(blocks):
    b = blocks.reshape(-1, 2).tolist()
    return [((w0 >> 40) & 0x3FFFFF, bool((w0 >> 62) & 1), w0 & ((1 << 40) - 1), w1) for w0, w1 in b]


@pytest.mark.parametrize("unaligned", [False, True])
def test_ptrs_plan_covers_every_unit_once(unaligned):
    leaf_n = [32, 288, 64, 18432, 128, 1179648, 62, 7936, 0, 3, 1]
    V = 1 if unaligned else 4
    blocks = kernels.ptrs_plan(_lib.F32, leaf_n, unaligned)
    dec = _decode(blocks)
    # tails come first (latency-bound blocks start early)
    first_main = next((i for i, d in enumerate(dec) if not d[1]), len(dec))
    assert all(d[1] for d in dec[:first_main]) and not any(d[1] for d in dec[first_main:])
    tails = {d[0] for d in dec if d[1]}
    ranges = {l: [] for l in range(len(leaf_n))}
    for leaf, tail, u0, u1 in dec:
        if not tail:
            assert u0 < u1
            ranges[leaf].append((u0, u1))
    sizes = [u1 - u0 for r in ranges.values() for u0, u1 in r]
    for l, n in enumerate(leaf_n):
        r = sorted(ranges[l])
        covered = [u for u0, u1 in r for u in (u0, u1)]
        nunits = n // V
        if nunits:
            assert r[0][0] == 0 and r[-1][1] == nunits
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        else:
            assert not r
        assert (l in tails) == (n % V != 0)
    # balanced: every range is at most the common share S (a multiple of 64 units)
    S = max(sizes)
    assert S % 64 == 0 and all(sz <= S for sz in sizes)


def test_ptrs_plan_per_leaf_units():
    """fjagg_ptrs_plan_leaves: marked leaves walk element units (flag bit 63, no tail
    block, ranges of at most S elements); the other leaves keep 16-byte units and tails."""
    leaf_n = [32, 288, 64, 18432, 128, 1179648, 62, 7936, 5, 3]
    mask = np.array([0, 0, 0, 1, 0, 1, 1, 0, 0, 1], dtype=bool)
    blocks = kernels.ptrs_plan(_lib.F32, leaf_n, mask).reshape(-1, 2)
    elem = (blocks[:, 0].view(np.uint64) >> np.uint64(63)).astype(bool)
    w0 = blocks[:, 0] & ((1 << 63) - 1)
    dec = _decode(np.stack([w0, blocks[:, 1]], 1).ravel())
    first_main = next(i for i, d in enumerate(dec) if not d[1])
    assert all(d[1] for d in dec[:first_main]) and not any(d[1] for d in dec[first_main:])
    S = max(u1 - u0 for (_, t, u0, u1), e in zip(dec, elem) if not t and not e)
    for l, n in enumerate(leaf_n):
        mine = [(d, e) for d, e in zip(dec, elem) if d[0] == l]
        assert all(e == mask[l] for _, e in mine)
        tails = [d for d, _ in mine if d[1]]
        r = sorted((d[2], d[3]) for d, _ in mine if not d[1])
        units = n if mask[l] else n // 4
        assert len(tails) == (0 if mask[l] else int(n % 4 != 0))
        assert r[0][0] == 0 and r[-1][1] == units and all(a[1] == b[0] for a, b in zip(r, r[1:]))
        assert all(u1 - u0 <= S for u0, u1 in r)  # element ranges keep the unit count
    # no marked leaf: the same table as the launch-wide aligned plan
    assert np.array_equal(kernels.ptrs_plan(_lib.F32, leaf_n, np.zeros(len(leaf_n), bool)),
                          kernels.ptrs_plan(_lib.F32, leaf_n, False))
    with pytest.raises(ValueError):
        kernels.ptrs_plan(_lib.F32, leaf_n, mask[:-1])


def test_ptrs_plan_bf16_units():
    blocks = kernels.ptrs_plan(_lib.BF16, [17], False)
    dec = _decode(blocks)
    assert dec == [(0, True, 0, 0), (0, False, 0, 2)]  # 2 units of 8 + a 1-element tail


def test_shard_range_partitions_clients():
    for K in (1, 7, 1024, 1025):
        for G in (1, 2, 3, 8):
            ranges = [distributed.shard_range(K, g, G) for g in range(G)]
            assert ranges[0][0] == 0 and ranges[-1][1] == K
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_bucket_edges_are_aligned_and_cover():
    for P in (1, 1000, 1206590, 4194304):
        for nb in (1, 4, 7):
            e = distributed.bucket_edges(P, nb)
            assert e[0][0] == 0 and e[-1][1] == P
            assert all(a[1] == b[0] for a, b in zip(e, e[1:]))
            assert all(p0 % distributed.BUCKET_ALIGN == 0 for p0, _ in e)


def test_tapered_bucket_edges():
    A = distributed.BUCKET_ALIGN
    P = 4 * 1024 * 1024
    assert distributed.bucket_edges(P, (4, 2, 1)) == [(0, 2397184), (2397184, 3595264), (3595264, P)]
    assert distributed.bucket_edges(P, (3, 1)) == [(0, 3 * P // 4), (3 * P // 4, P)]
    assert distributed.bucket_edges(P, (1, 1)) == distributed.bucket_edges(P, 2)
    for P in (1, 1000, 5000, 1206590, 4194304):
        for spec in ((3, 1), (7, 1), (4, 2, 1), (8, 4, 2, 1), (0.5, 0.25)):
            e = distributed.bucket_edges(P, spec)
            assert e[0][0] == 0 and e[-1][1] == P and len(e) <= len(spec)
            assert all(a[1] == b[0] and a[0] < a[1] for a, b in zip(e, e[1:]))
            assert all(p0 % A == 0 for p0, _ in e)
    assert distributed.bucket_edges(0, (3, 1)) == []
    assert distributed.bucket_name((4, 2, 1)) == "4:2:1" and distributed.bucket_name(2) == "2"
    with pytest.raises(ValueError):
        distributed.bucket_edges(100, (1, 0))


def test_server_descriptor_constants_follow_jax_weak_typing():
    from fedjax_amd import server
    opt = server.adam(10 ** -2.5, b1=0.9, b2=0.999, eps=1e-4)
    d = opt.descriptor(3)
    f = np.float32
    assert d.kind == _lib.OPT_ADAM
    assert d.neg_lr == f(-(10 ** -2.5))
    assert d.one_minus_b1 == f(1 - 0.9) and d.b1 == f(0.9)  # Python-float 1-b1, then f32
    assert d.bc1 == f(1) - np.power(f(0.9), f(3)) and d.bc2 == f(1) - np.power(f(0.999), f(3))
    s = server.sgd(0.1, momentum=0.9, nesterov=True)
    assert s.kind == _lib.OPT_MOMENTUM and s.descriptor(1).nesterov == 1
    assert server.sgd(1.0).kind == _lib.OPT_SGD


def test_bf16_semantics_switch_and_leaf_rule():
    """set_bf16_semantics("reference") selects the bf16 fold (acc FJAGG_BF16) for bf16
    leaves with weakly typed weights only; strongly typed float32 weights promote to f32."""
    from fedjax_amd import tree_util as tu
    assert tu.bf16_semantics() == "f32"
    W, S = tu._WEAK_INT, tu._STRONG_FLOAT
    assert tu._leaf_rule(torch.bfloat16, [W], None) == (_lib.BF16, _lib.F32, torch.bfloat16)
    tu.set_bf16_semantics("reference")
    try:
        assert tu._leaf_rule(torch.bfloat16, [W, tu._WEAK_FLOAT], tu._WEAK_FLOAT) == (_lib.BF16, _lib.BF16,
                                                                                       torch.bfloat16)
        assert tu._leaf_rule(torch.bfloat16, [S], None) == (_lib.BF16, _lib.F32, torch.float32)
        assert tu._leaf_rule(torch.float32, [W], None) == (_lib.F32, _lib.F32, torch.float32)
        assert tu._leaf_rule(torch.int32, [W], None) == (_lib.I32, _lib.I32, torch.int32)
    finally:
        tu.set_bf16_semantics("f32")
    with pytest.raises(ValueError):
        tu.set_bf16_semantics("bf16")


def test_server_schedule_and_frozen_mask_host_side():
    """ScalarOrSchedule (optimizers.py:114): the descriptor of the step whose incremented
    count is c carries f32(-lr(c - 1)) (optax.scale_by_schedule reads the count before
    incrementing it); ignore_grads_haiku (optimizers.py:69-109) marks the frozen leaves in
    flatten order and raises KeyError for a name the params do not have."""
    from fedjax_amd import pytree, server
    sched = lambda c: 0.1 * 0.5 ** c
    opt = server.sgd(sched)
    for c in (1, 2, 3):
        assert opt.descriptor(c).neg_lr == np.float32(-sched(c - 1))
    assert server.sgd(0.3).descriptor(7).neg_lr == np.float32(-0.3)
    params = {"linear_1": {"w": np.zeros(3)}, "linear_2": {"w": np.zeros(3), "b": np.zeros(3)}}
    _, td = pytree.flatten(params)
    ig = server.ignore_grads_haiku(server.adam(sched), [("linear_1", "w"), ("linear_2", "b")])
    assert ig.kind == server.adam(0.1).kind and ig.frozen == (("linear_1", "w"), ("linear_2", "b"))
    # flatten order: linear_1/w, linear_2/b, linear_2/w
    assert server._frozen_leaves(ig, params, td).tolist() == [True, True, False]
    assert server._frozen_leaves(server.adam(0.1), params, td).tolist() == [False] * 3
    with pytest.raises(KeyError):
        server._frozen_leaves(server.ignore_grads_haiku(ig, [("linear_3", "w")]), params, td)


def test_nontemporal_threshold_setter():
    """tree_util.set_nontemporal_min_bytes sets the module value the Python folds and fold_chain
    read, and re-configures the builtin tree_mean with it (fjhost.mean_config), so a runtime
    change reaches every path; the default is restored after."""
    old = tu.NONTEMPORAL_MIN_BYTES
    try:
        tu.set_nontemporal_min_bytes(12345)
        assert tu.NONTEMPORAL_MIN_BYTES == 12345 and isinstance(tu.NONTEMPORAL_MIN_BYTES, int)
        tu.set_nontemporal_min_bytes(float(1 << 20))
        assert tu.NONTEMPORAL_MIN_BYTES == 1 << 20
    finally:
        tu.set_nontemporal_min_bytes(old)
    assert tu.NONTEMPORAL_MIN_BYTES == old
