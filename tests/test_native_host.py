"""The native host helper of the pytree path (fedjax_amd/csrc/fjhost.cpp): pointer
table and weight packing must agree with the Python path they replace, and must
decline (never decide) every case that path handles differently. Host tensors
(dev_index -1) stand in for device tensors; no GPU needed."""
import collections

import numpy as np
import pytest
import torch

from fedjax_amd import _lib, pytree, tree_util as tu

H = _lib.host()


def _tree(seed):
    g = torch.Generator().manual_seed(seed)
    return {"b": {"w": torch.randn(3, 4, generator=g), "b": torch.randn(4, generator=g)},
            "a": [torch.randn(5, generator=g), (torch.randn(2, 2, generator=g), None)]}


def _table(trees):
    leaves0, td = pytree.flatten(trees[0])
    spec = pytree.native_spec(td)
    ptrs = np.full((len(trees), len(leaves0)), -7, dtype=np.int64)
    rc = H.gather_rows(trees, 1, spec, leaves0, -1, ptrs)
    return rc, ptrs


def test_pointer_table_matches_python_flatten():
    trees = [_tree(k) for k in range(6)]
    rc, ptrs = _table(trees)
    assert rc == 0
    want = [[x.data_ptr() for x in pytree.flatten(t)[0]] for t in trees]
    assert ptrs.tolist() == want


def test_spec_encodes_flatten_order():
    _, td = pytree.flatten(_tree(0))
    # dict keys sorted, list/tuple positional, None kept as an empty node
    assert pytree.native_spec(td) == (2, ("a", "b"), ((3, 2, (0, (4, 2, (0, 1)))), (2, ("b", "w"), (0, 0))))
    nt = collections.namedtuple("nt", "x y")
    for t in (nt(torch.zeros(1), torch.zeros(1)), collections.OrderedDict(x=torch.zeros(1))):
        assert pytree.native_spec(pytree.flatten(t)[1]) is None  # Python walk


@pytest.mark.parametrize("mutate", [
    lambda t: t["b"].pop("w"),                                   # structure
    lambda t: t["b"].__setitem__("x", t["b"].pop("w")),          # key
    lambda t: t["a"].__setitem__(0, t["a"][0].double()),          # dtype
    lambda t: t["a"].__setitem__(0, torch.zeros(6)),              # shape
    lambda t: t["b"].__setitem__("w", torch.zeros(4, 3).t()),     # not contiguous
    lambda t: t["a"].__setitem__(0, np.zeros(5, np.float32)),     # not a tensor
    lambda t: t["a"].__setitem__(1, [t["a"][1][0], None]),        # tuple -> list
    lambda t: t["a"].__setitem__(1, (t["a"][1][0], torch.zeros(1))),  # None -> leaf
    lambda t: t["a"].__setitem__(0, torch.nn.Parameter(t["a"][0])),   # tensor subclass
])
def test_mismatch_is_declined_at_the_first_bad_client(mutate):
    trees = [_tree(k) for k in range(5)]
    mutate(trees[3])
    rc, _ = _table(trees)
    assert rc == -(3 + 1)


def test_device_index_must_match():
    trees = [_tree(k) for k in range(3)]
    leaves0, td = pytree.flatten(trees[0])
    ptrs = np.empty((3, len(leaves0)), dtype=np.int64)
    assert H.gather_rows(trees, 1, pytree.native_spec(td), leaves0, 0, ptrs) == -2  # host tensors, cuda:0 asked


def test_pointer_buffer_is_checked():
    trees = [_tree(k) for k in range(3)]
    leaves0, td = pytree.flatten(trees[0])
    with pytest.raises(ValueError):
        H.gather_rows(trees, 1, pytree.native_spec(td), leaves0, -1, np.empty(4, dtype=np.int64))


@pytest.mark.parametrize("ws", [
    [1, 2, 3], [0.1, 0.7, 1e-3], [3, 0.5, 7], [2**31 + 5, -(2**40) - 3, 1], [-0.0, 0.0], [2**53 - 1, 1],
    [float("inf"), 1.0], [16777217, 33554435],
])
def test_packed_weights_equal_python_semantics(ws):
    got = tu._pack_weights(list(ws))
    W = 0.0
    for w in ws:
        W += w  # tree_util.py:95
    assert got is not None and got.total == W or (np.isnan(W) and np.isnan(got.total))
    assert got.f32.view(np.uint32).tolist() == np.array([np.float32(w) for w in ws]).view(np.uint32).tolist()
    ints = [w for w in ws if type(w) is int]
    if len(ints) == len(ws):
        assert got.i32.tolist() == np.array([np.int64(w) for w in ws], dtype=np.int64).astype(np.int32).tolist()
    want_kinds = sorted({tu._weight_kind(w) for w in ws})
    assert sorted(got.kinds) == want_kinds


@pytest.mark.parametrize("ws", [[1, np.float32(2)], [True, 1], [torch.tensor(1.0)], [2**53], [1, "x"]])
def test_other_weights_take_the_python_path(ws):
    assert tu._pack_weights(list(ws)) is None


def test_collect_pairs_consumes_a_generator_once():
    trees = [_tree(k) for k in range(3)]
    gen = ((t, w) for t, w in zip(trees, [1, 2, 3]))
    got_trees, weights, W = tu._collect_pairs(gen)
    assert got_trees == trees and W == 6.0 and isinstance(weights, tu._Weights)
    _, weights, W = tu._collect_pairs(zip(trees, [np.float32(1), np.float32(2), np.float32(0.5)]))
    assert isinstance(weights, list) and isinstance(W, np.float32) and W == np.float32(3.5)


def test_leaf_versions_track_in_place_updates():
    """fjhost.leaf_versions (RunningMean's reuse guard): torch's version counters in
    flatten order; an in-place update bumps exactly that leaf; structure mismatch is
    reported at the first bad client."""
    trees = [_tree(k) for k in range(3)]
    leaves0, td = pytree.flatten(trees[0])
    spec, L = pytree.native_spec(td), len(leaves0)
    v0 = np.empty((3, L), dtype=np.int64)
    assert H.leaf_versions(trees, spec, L, v0) == 0
    assert v0.tolist() == [[x._version for x in pytree.flatten(t)[0]] for t in trees]
    trees[1]["b"]["w"].add_(1.0)
    v1 = np.empty((3, L), dtype=np.int64)
    assert H.leaf_versions(trees, spec, L, v1) == 0
    changed = np.argwhere(v1 != v0).tolist()
    pos = [i for i, x in enumerate(pytree.flatten(trees[1])[0]) if x is trees[1]["b"]["w"]][0]
    assert changed == [[1, pos]]
    trees[2]["b"].pop("w")
    assert H.leaf_versions(trees, spec, L, v1) == -3
    with pytest.raises(ValueError):
        H.leaf_versions(trees, spec, L, np.empty(2, dtype=np.int64))


def _mean_pairs(pairs):
    """fjhost.mean_pairs with the tree_util knobs; plan / launch addresses are never
    reached on the host (every case here declines first)."""
    return _lib.host().mean_pairs(pairs, False, 0.25, 512, 60.0, 35.0, 64 << 20, 256 << 10, float(256 << 20), 0, 0)


@pytest.mark.parametrize("pairs", [
    [],                                                                 # no clients
    [({"w": torch.zeros(5)}, 1)] * 3,                                   # host tensors
    [({"w": torch.zeros(5)}, np.float32(1))] * 3,                       # a numpy weight
    [({"w": torch.zeros(5)}, True)] * 3,                                # a bool weight
    [({"w": torch.zeros(5)}, 2 ** 60)] * 3,                             # a weight past 2**53
    [({"w": torch.zeros(5)},)] * 3,                                     # not a pair
    [({1: torch.zeros(5), "a": torch.zeros(5)}, 1)] * 3,                # unorderable dict keys
    [(collections.OrderedDict(w=torch.zeros(5)), 1)] * 3,              # a node kind it does not take
    [({"w": np.zeros(5, np.float32)}, 1)] * 3,                          # a numpy leaf
    [({"w": None}, 1)] * 3,                                             # no leaves
])
def test_native_whole_call_declines(pairs):
    """tree_mean's one-call native path (fjhost.mean_pairs) answers None, launching
    nothing and raising nothing, for every input it does not take: the Python path then
    runs (and raises the reference's errors where there are any)."""
    assert _mean_pairs(pairs) is None
    assert _mean_pairs(tuple(pairs)) is None
    assert _lib.host().server_pairs(pairs, {"w": torch.zeros(5)}, None, None, None, 0, 0.0, 0, 0) is None


def test_walk_visits_dict_values_in_sorted_key_order_on_every_call():
    """The native walk's sorted-key cache also hands out operand 0's dict values in sorted-key
    order (fjhost sorted_keys: the insertion-order scan that matches the key objects collects
    them). The same key objects in different insertion orders, dicts up to and past the 32 keys
    that path serves, the cache-miss walk and the cache-hit ones: every walk visits the leaves in
    jax's flatten order (fjhost.matches compares them with the flatten-order leaf tuple)."""
    import random
    rnd = random.Random(5)
    for n in (1, 2, 5, 31, 32, 33, 40):
        names = [f"k{i:02d}" for i in range(n)]  # one set of key objects per size
        inner = ["w", "b", "a"] if n <= 16 else ["w"]  # (the fast walk takes <= 64 leaves)
        for _ in range(3):
            order, inner_order = names[:], inner[:]
            rnd.shuffle(order)
            rnd.shuffle(inner_order)
            tree = {k: {j: torch.zeros(1) for j in inner_order} for k in order}
            flat = tuple(tree[k][j] for k in sorted(names) for j in sorted(inner))
            assert flat == tuple(pytree.flatten(tree)[0])
            vs = sum(x._version for x in flat)
            for _ in range(3):
                assert H.matches(tree, flat, vs)
            assert not H.matches(tree, flat[::-1], vs)
