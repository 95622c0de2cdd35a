"""Golden fixtures are consistent with the oracle restatement (CPU)."""
import numpy as np
import pytest

from oracle import tree_util_ref as ref
from tests import golden_cases as gc


def test_fixture_set_is_complete():
    assert len(gc.NAMES) >= 15, gc.NAMES


@pytest.mark.parametrize("name", [n for n in gc.NAMES if not n.startswith("bf16")])
def test_oracle_reproduces_fixture(name):
    c = gc.load(name)
    x, shapes = c["x"], c["shapes"]
    trees = [gc.split_leaves(x[k], shapes) for k in range(x.shape[0])]
    with np.errstate(invalid="ignore"):
        m = ref.tree_mean(zip(trees, c["weight_list"]))
    got = np.concatenate([np.asarray(v, np.float32).ravel() for v in m])
    assert np.array_equal(got.view(np.uint32), c["y"].view(np.uint32)), name


def test_bf16_fixture_bounds(coracle):
    c = gc.load("bf16_k16_p1024")
    y64 = coracle.wsum_bf16_f64(c["x"], np.float64(c["weight_list"]), 1.0 / sum(c["weight_list"]))
    assert np.array_equal(y64, c["y_f64"])
