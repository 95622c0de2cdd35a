"""The native running-sum objects and calls (fjhost.WeightedBase / PendingBase / ChainBase,
fjhost.tree_weight / tree_add), on the CPU: the link fjhost.tree_add builds
is the one PendingSum.__init__ builds, every case outside the fast one reaches the Python
function, and the objects are freed (cycles, long chains). No device work: captures are
built by hand here; the GPU tests (test_gpu_tree_ops.py, test_gpu_algorithms.py) run the
same calls on real deltas, bitwise against the oracle."""
import gc
import inspect
import weakref

import pytest
import torch

from fedjax_amd import tree_util as tu

H = tu._HOST


def _cap(tok, nbytes=400, leaves=None):
    leaves = leaves if leaves is not None else (torch.zeros(100),)
    return (leaves, 0, nbytes, tok)


def _root(tok=7, budget=1 << 30):
    tree = {"w": torch.zeros(100)}
    p = tu.PendingSum(tree, None, _cap(tok), 3, tree, _cap(tok), tok)
    p._chain.budget = budget
    return p


@pytest.fixture()
def stubs():
    """fjhost's fallbacks replaced by recorders for the test, then restored."""
    calls = []

    def tw(*a, **k):
        calls.append(("tree_weight", a, k))
        return "py-tree-weight"

    def ta(*a, **k):
        calls.append(("tree_add", a, k))
        return "py-tree-add"

    H.fast_install(tu.WeightedTree, tu.PendingSum, tu._Chain, tw, ta)
    yield calls
    H.fast_install(tu.WeightedTree, tu.PendingSum, tu._Chain, tu._tree_weight_py, tu._tree_add_py)
    tu.set_deferred_sums(True)


def test_public_calls_are_the_native_ones():
    assert tu.tree_weight is H.tree_weight and tu.tree_add is H.tree_add
    assert list(inspect.signature(tu.tree_weight).parameters) == ["pytree", "weight"]
    assert list(inspect.signature(tu.tree_add).parameters) == ["left", "right"]
    assert issubclass(tu.WeightedTree, H.WeightedBase) and issubclass(tu.PendingSum, H.PendingBase)
    assert issubclass(tu._Chain, H.ChainBase)


def test_native_link_equals_the_python_link(stubs):
    p = _root()
    wt = tu.WeightedTree({"w": torch.zeros(100)}, 5, _cap(7, nbytes=400))
    q = tu.tree_add(p, wt)
    assert stubs == []  # built natively
    assert type(q) is tu.PendingSum
    # PendingSum.__init__ on the same arguments, on a twin root (the Python path's link)
    p2 = _root()
    ref = tu.PendingSum(None, p2, wt._cap, wt._weight, p2._ref, None, p2._tok)
    twin = {"_parent": (p, p2), "_chain": (p._chain, p2._chain), "_ref": (p._ref, p2._ref)}
    for f in ("_root", "_parent", "_cap", "_weight", "_value", "_chain", "_ticket", "_ref", "_bcap"):
        mine, theirs = twin.get(f, (getattr(ref, f), getattr(ref, f)))
        assert getattr(q, f) is mine and getattr(ref, f) is theirs, f
    for f in ("_n", "_bytes", "_idx", "_tok"):
        assert getattr(q, f) == getattr(ref, f), f
    ch_tip = p._chain.tip
    assert (q._n, q._bytes, q._idx) == (2, 800, 1)
    assert ch_tip is q  # the native call moved the chain's tip
    assert H.last() is q
    del ref


@pytest.mark.parametrize("case", ["token", "limit", "budget", "flush", "folded", "not_tip", "disabled", "kw"])
def test_declined_cases_reach_the_python_function(stubs, case):
    p = _root()
    wt = tu.WeightedTree({"w": torch.zeros(100)}, 5, _cap(8 if case == "token" else 7))
    if case == "limit":
        tu.set_deferred_sums(True, max_clients=1)
    elif case == "budget":
        p._chain.budget = 500
    elif case == "flush":
        tu.set_deferred_sums(True, flush_bytes=100, flush_clients=1)
    elif case == "folded":
        p._value = {"w": torch.zeros(100)}
    elif case == "not_tip":
        tu.tree_add(p, tu.WeightedTree({"w": torch.zeros(100)}, 1, _cap(7)))  # p is no longer the tip
        stubs.clear()
    elif case == "disabled":
        tu.set_deferred_sums(False)
    if case == "kw":
        got = tu.tree_add(left=p, right=wt)
    else:
        got = tu.tree_add(p, wt)
    assert got == "py-tree-add"
    assert len(stubs) == 1 and stubs[0][0] == "tree_add"
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)


def test_tree_weight_declines_to_python(stubs):
    tree = {"w": torch.zeros(3)}  # host tensors: no capture, the Python function decides
    assert tu.tree_weight(tree, 2) == "py-tree-weight"
    assert tu.tree_weight(tree, 2.5) == "py-tree-weight"
    assert tu.tree_weight(tree, 1 << 60) == "py-tree-weight"  # beyond float32's exact-int path
    assert tu.tree_weight(pytree=tree, weight=2) == "py-tree-weight"
    assert [c[0] for c in stubs] == ["tree_weight"] * 4


def test_chains_are_freed():
    p = _root()
    wr_root = weakref.ref(p)
    q = p
    for _ in range(4000):  # a long chain: freeing it must not recurse 4000 deep unguarded
        q = tu.tree_add(q, tu.WeightedTree({"w": None}, 1, _cap(7, nbytes=1)))
    wr_tip = weakref.ref(q)
    assert q._n == 4001
    del p, q
    gc.collect()  # node -> chain -> tip -> node is a cycle: the collector frees it
    assert wr_root() is None and wr_tip() is None
    assert H.last() is None


def test_flush_views_folds_only_waiting_chains():
    """fjhost.flush_views (what every torch function on a lazy norm view runs first) folds
    the chain of a view whose ticket still names a link, walks nested lists / tuples / dict
    values, and leaves filled views (ticket node None) and other objects alone."""
    buf = torch.arange(8, dtype=torch.float32).view(2, 4)
    folded = []

    class Tip:
        def materialize(self):
            folded.append(1)
            t1.node = None  # (a fold clears the tickets it fills)

    class Chain:
        tip = Tip()

    class Node:
        _chain = Chain()

    t1, t2 = tu._Ticket(Node()), tu._Ticket(None)
    v1, v2, v3 = (H.norm_view(buf, 1, i, tu._NormView) for i in range(3))
    v1._ticket, v2._ticket = t1, t2  # v3: no ticket at all
    H.flush_views([v3, (1, {"a": [v2]}), "x"])
    assert folded == []
    H.flush_views({"k": [(v2, v1)], "j": v3})
    assert folded == [1]
    H.flush_views([v1, v1])  # filled now: no second fold
    assert folded == [1]
    with torch._C.DisableTorchFunctionSubclass():
        assert float(v1) == 4.0  # buf[1, 0]: a view of the chain buffer
