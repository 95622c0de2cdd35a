"""Host-side pytree logic (no GPU)."""
import collections

import pytest

import fedjax_amd
from fedjax_amd import pytree


def test_dict_keys_sorted_like_jax():
    leaves, td = pytree.flatten({"b": 1, "a": {"z": 2, "c": 3}, "c": [4, (5, None)]})
    assert leaves == [3, 2, 1, 4, 5]
    assert pytree.unflatten(td, leaves) == {"b": 1, "a": {"z": 2, "c": 3}, "c": [4, (5, None)]}


def test_emnist_param_order():
    # fedjax/models/emnist.py:59-72 haiku params, jax flatten order
    params = {"linear": {"w": 5, "b": 4}, "conv2_d": {"w": 1, "b": 0}, "conv2_d_1": {"w": 3, "b": 2},
              "linear_1": {"w": 7, "b": 6}}
    assert pytree.flatten(params)[0] == [0, 1, 2, 3, 4, 5, 6, 7]


def test_namedtuple_and_ordereddict():
    NT = collections.namedtuple("NT", ["y", "x"])
    t = NT(y=1, x=collections.OrderedDict([("q", 2), ("a", 3)]))
    leaves, td = pytree.flatten(t)
    assert leaves == [1, 2, 3]
    assert pytree.unflatten(td, [10, 20, 30]) == NT(10, collections.OrderedDict([("q", 20), ("a", 30)]))


def test_dataclass_is_pytree_and_frozen():
    @fedjax_amd.dataclass
    class State:
        params: dict
        step: int

    s = State(params={"w": 1.0}, step=3)
    leaves, td = pytree.flatten(s)
    assert leaves == [1.0, 3]
    assert pytree.unflatten(td, [2.0, 4]) == State(params={"w": 2.0}, step=4)
    assert s.replace(step=5).step == 5
    with pytest.raises(Exception):
        s.step = 1


def test_structure_mismatch_raises():
    _, td = pytree.flatten({"a": 1, "b": 2})
    with pytest.raises(ValueError):
        pytree.flatten_as(td, {"a": 1, "c": 2})
    with pytest.raises(ValueError):
        pytree.flatten_as(td, {"a": 1})


def test_tree_map_and_none():
    assert pytree.tree_map(lambda a, b: a + b, (1, None, [2]), (10, None, [20])) == (11, None, [22])
    assert pytree.flatten(None)[0] == []


def test_aggregator_is_pytree_dataclass():
    agg = fedjax_amd.aggregators.mean_aggregator()
    assert callable(agg.init) and callable(agg.apply)
    leaves, _ = pytree.flatten(agg)
    assert len(leaves) == 2
    assert isinstance(agg.init(), fedjax_amd.aggregators.MeanAggregatorState)


def test_treedefs_are_interned():
    """Flattens of one structure share one TreeDef object (per-structure caches hit by
    identity); different structures stay different; unhashable aux data is not interned."""
    import numpy as np
    a = {"b": {"w": np.zeros(3), "b": np.zeros(2)}, "a": [np.zeros(1), (np.zeros(1), None)]}
    b = {"a": [np.ones(1), (np.ones(1), None)], "b": {"b": np.ones(2), "w": np.ones(3)}}
    la, ta = pytree.flatten(a)
    lb, tb = pytree.flatten(b)
    assert ta is tb and len(la) == len(lb) == 4
    _, tc = pytree.flatten({"a": [np.zeros(1), [np.zeros(1), None]], "b": {"w": 0, "b": 0}})
    assert tc != ta and tc is not ta
    assert pytree.unflatten(ta, lb)["b"]["w"] is b["b"]["w"]

    class Box:
        def __init__(self, v, meta):
            self.v, self.meta = v, meta
    pytree.register_pytree_node(Box, lambda x: ([x.v], x.meta), lambda aux, ch: Box(ch[0], aux))
    t1 = pytree.flatten(Box(np.zeros(2), {"unhashable": 1}))[1]
    t2 = pytree.flatten(Box(np.zeros(2), {"unhashable": 1}))[1]
    assert t1 is not t2  # aux is a dict: built fresh each time
    assert pytree.unflatten(t1, [np.ones(2)]).meta == {"unhashable": 1}


def test_flatten_as_keys_without_expression_repr():
    """dict keys whose repr is not a Python expression (numpy strings, enums)
    go through the compiled accessor as objects."""
    import enum

    import numpy as np

    from fedjax_amd import pytree

    class Color(enum.Enum):
        RED = 1

    t = {np.str_("a"): np.zeros(2), Color.RED: np.ones(1)}
    try:
        leaves, td = pytree.flatten(t)
    except TypeError:  # unorderable mixed keys: jax refuses such dicts too
        t = {np.str_("a"): np.zeros(2), np.str_("b"): np.ones(1)}
        leaves, td = pytree.flatten(t)
    got = pytree.flatten_as(td, t)
    assert all(a is b for a, b in zip(got, leaves))
    t2 = {np.str_("a"): np.zeros(2), np.str_("b"): np.ones(1)}
    leaves2, td2 = pytree.flatten(t2)
    assert [x is y for x, y in zip(pytree.flatten_as(td2, t2), leaves2)] == [True, True]
