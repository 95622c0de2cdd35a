"""tree_mean on an idle stream folds in chunked launches that overlap the host walk
(tree_util._tree_mean_pipelined): the first launch folds clients [0, k1) as soon as their
pointers are gathered, later ones accumulate into the same sums, the last applies 1/W.
Accumulate mode keeps the per-element sequence of fedjax/core/tree_util.py:85-96, so the
result must be bitwise the one-launch fold and the oracle's; errors must be the one-launch
path's (the second walk falls back to it)."""
import numpy as np
import pytest
import torch

from fedjax_amd import _lib, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu
EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def _tmap(f, t):
    return {k: _tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def _clients(K, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [_tmap(lambda s: torch.rand(s, device="cuda", generator=g) - 0.5, EMNIST) for _ in range(K)]


def _flat(tree):
    return np.concatenate([x.detach().cpu().numpy().ravel() for x in ref.flatten(tree)[0]])


def _launches():  # fold_table launches (image in the kernel arguments or uploaded)
    p = _lib.host().image_paths()
    return p["kernel_args"] + p["uploaded"]


@pytest.fixture
def chunk(tu_settings):
    def set_(v):
        tu_settings(_PIPELINE_CHUNK=v)
    return set_


@pytest.fixture
def frac(tu_settings):
    def set_(v):
        tu_settings(_PIPELINE_FRAC=v)
    return set_


@pytest.mark.parametrize("K", [16, 29, 128])
def test_pipelined_tree_mean_bitwise(K, frac, cuda):
    clients = _clients(K, seed=K)
    weights = np.random.RandomState(K).randint(1, 501, size=K).tolist()
    weights[3] = 2.5  # a float weight among ints (weak float kinds)
    pairs = list(zip(clients, weights))
    frac(0.0)
    one = _flat(tu.tree_mean(pairs))
    for f in (0.01, 0.33, 0.5, 0.99):
        frac(f)
        torch.cuda.synchronize()  # idle stream: the pipelined path
        n0 = _launches()
        got = _flat(tu.tree_mean(pairs))
        assert _launches() - n0 == 2, f"frac {f}: expected the two-launch pipeline"
        np.testing.assert_array_equal(got.view(np.uint32), one.view(np.uint32))
    if K == 29:  # the oracle on every element (29 x 1.2 M)
        host = [(_tmap(lambda x: x.cpu().numpy(), c), w) for c, w in pairs]
        want = np.concatenate([np.asarray(x).ravel() for x in ref.flatten(ref.tree_mean(host))[0]])
        np.testing.assert_array_equal(one.view(np.uint32), want.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("K,c", [(1500, 512), (1500, 100), (600, 256)])
def test_chunked_pipeline_small_model_bitwise(K, c, frac, chunk, cuda, tu_settings):
    """A small model (48,670 params: the walk, not the fold, is the longer part), with the
    narrow-delta exclusion lifted: launches of c clients, each accumulating into the first's
    sums (stripe / narrow plans per chunk)."""
    tu_settings(_CHUNK_WALK_US=0.0)  # chunks of exactly c clients
    tu_settings(_NARROW_MAX_BYTES=0)  # (the fold still picks its narrow plans natively)
    g = torch.Generator(device="cuda").manual_seed(K + c)
    shapes = {"w": (784, 62), "b": (62,)}
    clients = [{k: torch.rand(s, device="cuda", generator=g) - 0.5 for k, s in shapes.items()} for _ in range(K)]
    pairs = list(zip(clients, np.random.RandomState(c).randint(1, 501, size=K).tolist()))
    frac(0.0)
    one = _flat(tu.tree_mean(pairs))
    frac(0.25)
    chunk(c)
    torch.cuda.synchronize()
    n0 = _launches()
    got = _flat(tu.tree_mean(pairs))
    assert _launches() - n0 == -(-K // c)
    np.testing.assert_array_equal(got.view(np.uint32), one.view(np.uint32))
    if K == 600:
        host = [({k: v.cpu().numpy() for k, v in t.items()}, w) for t, w in pairs]
        want = np.concatenate([np.asarray(x).ravel() for x in ref.flatten(ref.tree_mean(host))[0]])
        np.testing.assert_array_equal(one.view(np.uint32), want.astype(np.float32).view(np.uint32))


def test_busy_stream_takes_one_launch(frac, cuda):
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    frac(0.33)
    K = 16
    pairs = list(zip(_clients(K), [1.0 + k for k in range(K)]))
    ref_out = _flat(tu.tree_mean(pairs))
    torch.cuda.synchronize()
    torch.cuda._sleep(50_000_000)  # keeps the stream busy while tree_mean is issued
    n0 = _launches()
    out = tu.tree_mean(pairs)
    assert _launches() - n0 == 1
    np.testing.assert_array_equal(_flat(out).view(np.uint32), ref_out.view(np.uint32))


@pytest.mark.parametrize("where", [2, 13])  # before / after the first chunk's clients (k1 = 5)
def test_pipelined_errors_are_the_one_launch_paths(where, frac, cuda):
    frac(0.33)
    K = 16
    clients = _clients(K)
    clients[where]["linear"]["w"] = torch.zeros(9216, 127, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match="shape"):
        tu.tree_mean(list(zip(clients, [1] * K)))
    clients = _clients(K)
    clients[where]["linear"]["b"] = clients[where]["linear"]["b"].to(torch.bfloat16)
    torch.cuda.synchronize()
    with pytest.raises(TypeError, match="dtype"):
        tu.tree_mean(list(zip(clients, [1] * K)))


def test_pipelined_declines_what_it_does_not_cover(frac, cuda):
    """numpy-scalar weights, host leaves, a small delta (the narrow plans): one launch,
    the same bits as with the pipeline off."""
    frac(0.33)
    K = 16
    clients = _clients(K)
    cases = {
        "numpy weights": list(zip(clients, [np.float32(1 + k) for k in range(K)])),
        "host client 0": [(_tmap(lambda x: x.cpu(), clients[0]), 1)] + [(c, 1) for c in clients[1:]],
        "small delta": [({"w": c["linear_1"]["w"]}, 1 + k) for k, c in enumerate(clients)],
    }
    for name, pairs in cases.items():
        frac(0.0)
        want = _flat(tu.tree_mean(pairs))
        frac(0.33)
        torch.cuda.synchronize()
        n0 = _launches()
        got = _flat(tu.tree_mean(pairs))
        assert _launches() - n0 <= 1, name
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg=name)


def test_native_whole_call_equals_python_path(frac, cuda, tu_settings):
    """fjhost.mean_pairs (the whole tree_mean call natively) against the Python path
    (FJAGG_NATIVE_MEAN off): bitwise, for dict / list / tuple / None nodes, pairs given as
    tuples or lists, int and float weights, pipelined or not; declined cases (a namedtuple
    node, a numpy weight, a bf16 leaf) still give the Python path's result."""
    import collections
    g = torch.Generator(device="cuda").manual_seed(7)
    r = lambda *s: torch.rand(*s, device="cuda", generator=g) - 0.5
    NT = collections.namedtuple("NT", "a b")
    K = 12
    cases = {
        "nested": [({"z": [r(70_000), None, (r(3), r(5, 2))], "a": {"q": r(8), "p": r(100_000)}}, 1 + k)
                   for k in range(K)],
        "list pairs, float weights": [[[r(90_000), r(4)], 0.5 + k] for k in range(K)],
        "emnist": list(zip(_clients(K, seed=3), [7] * K)),
        "namedtuple": [(NT(r(80_000), r(3)), k + 1) for k in range(K)],
        "numpy weight": [({"w": r(80_000)}, np.float32(k + 1)) for k in range(K)],
        "bf16": [({"w": r(80_000).to(torch.bfloat16)}, k + 1) for k in range(K)],
    }
    for name, pairs in cases.items():
        tu_settings(_NATIVE_MEAN=False)
        frac(0.0)
        want = tu.tree_mean(pairs)
        tu_settings(_NATIVE_MEAN=True)
        for f in (0.0, 0.5):
            frac(f)
            tu_settings(_PIPELINE_MIN_BYTES=0)
            torch.cuda.synchronize()
            got = tu.tree_mean(pairs)
            assert ref.flatten(got)[1] == ref.flatten(want)[1], name
            assert type(got) is type(want), name
            for a, b in zip(ref.flatten(got)[0], ref.flatten(want)[0]):
                assert a.dtype == b.dtype and a.shape == b.shape, name
                assert torch.equal(a.view(torch.int16 if a.dtype == torch.bfloat16 else torch.int32),
                                   b.view(torch.int16 if b.dtype == torch.bfloat16 else torch.int32)), name
    # structure / shape / dtype errors: the Python path's
    bad = [({"w": r(80_000)}, 1) for _ in range(K)]
    bad[9] = ({"w": r(80_001)}, 1)
    with pytest.raises(ValueError):
        tu.tree_mean(bad)
    bad[9] = ({"v": r(80_000)}, 1)
    with pytest.raises(ValueError):
        tu.tree_mean(bad)


def test_native_mean_with_l2_norms_equals_python_path(frac, cuda, tu_settings):
    """tree_mean_with_l2_norms through fjhost.mean_pairs (one launch, or the pipelined
    chunks, each giving its clients' norms) against the Python path: mean and norms bitwise."""
    K = 40
    pairs = list(zip(_clients(K, seed=9), [1 + (k % 7) for k in range(K)]))
    tu_settings(_NATIVE_MEAN=False)
    want_mean, want_norms = tu.tree_mean_with_l2_norms(pairs)
    tu_settings(_NATIVE_MEAN=True)
    for f in (0.0, 0.3):
        frac(f)
        torch.cuda.synchronize()
        n0 = _launches()
        mean, norms = tu.tree_mean_with_l2_norms(pairs)
        assert _launches() - n0 == (1 if f == 0.0 else 2)
        np.testing.assert_array_equal(_flat(mean).view(np.uint32), _flat(want_mean).view(np.uint32))
        np.testing.assert_array_equal(norms.cpu().numpy().view(np.uint32), want_norms.cpu().numpy().view(np.uint32))
