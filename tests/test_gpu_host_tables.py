"""FJAGG_HOST_TABLES: weights (dense) and whole plan images (pytree) carried in the
kernel arguments instead of a pinned upload on the stream. The kernels and the fold
order are the ones of the device-table launches, so every result here must be bitwise
the device-table result and the oracle's, and every refusal must leave
nothing launched (the callers then upload the tables, same bits).
"""
import numpy as np
import pytest
import torch

from fedjax_amd import _lib, kernels, tree_util as tu
from oracle import tree_util_ref as ref

pytestmark = pytest.mark.gpu

EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def u32(t):
    return t.detach().cpu().contiguous().view(torch.int32).numpy()


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


@pytest.mark.parametrize("K,P,dt,out_dt,offset", [
    (128, 1206590, torch.float32, torch.float32, 0),   # configs[1] slab: E8U4 burst
    (1024, 300_003, torch.float32, torch.float32, 0),  # E4U4 with an element tail
    (40, 200_000, torch.float32, torch.float32, 1),    # misaligned rows: element units (V = 1)
    (8, 70_000, torch.float32, torch.float32, 0),      # K < 16: E1U8, not the narrow kernel
    (64, 600_000, torch.bfloat16, torch.bfloat16, 0),
    (64, 600_000, torch.bfloat16, torch.float32, 0),
])
def test_dense_host_weights_bitwise(K, P, dt, out_dt, offset, cuda, coracle):
    x = torch.empty(K, P + 8 + offset, dtype=dt, device=cuda)[:, offset:offset + P]
    kernels.fill_synth(x, seed=7)
    w = np.float32(ref.fedavg_weights(K, seed=2))
    r = float(np.float32(1.0 / float(w.astype(np.float64).sum())))
    before = dict(kernels.HOST_WEIGHT_PATHS)
    got = kernels.weighted_sum_dense(x, w, scale=r, out_dtype=out_dt, nontemporal=K * P > (1 << 26))
    assert kernels.HOST_WEIGHT_PATHS["kernel_args"] == before["kernel_args"] + 1
    assert kernels.HOST_WEIGHT_PATHS["uploaded"] == before["uploaded"]
    want = kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), scale=r, out_dtype=out_dt,
                                      nontemporal=K * P > (1 << 26))
    assert np.array_equal(u32(got.float() if out_dt == torch.bfloat16 else got),
                          u32(want.float() if out_dt == torch.bfloat16 else want))
    if dt == torch.float32 and K * P <= 50_000_000:
        xo = coracle.synth_f32(K, P, seed=7)
        assert np.array_equal(u32(got), coracle.wsum_f32(xo, w, scale=r).astype(np.float32).view(np.int32))


def test_dense_host_weights_accumulate_and_cpu_tensor(cuda, coracle):
    K, P = 33, 250_000
    x = torch.empty(K, P, device=cuda)
    kernels.fill_synth(x, seed=4)
    w = torch.from_numpy(np.float32(ref.fedavg_weights(K, seed=6)))  # a CPU tensor works too
    init = torch.full((P,), 0.25, device=cuda)
    out = init.clone()
    kernels.weighted_sum_dense(x, w, out=out, accumulate=True)
    xo = coracle.synth_f32(K, P, seed=4)
    want = coracle.wsum_f32(xo, w.numpy(), init=np.full(P, 0.25, np.float32))
    assert np.array_equal(u32(out), want.astype(np.float32).view(np.int32))


def test_dense_host_weights_refused_then_uploaded(cuda, coracle):
    """K > 1024, the narrow kernel's shapes, split mode, an int32 fold and the bf16
    reference fold are not built with kernel-argument weights: the C ABI refuses before
    launching anything and weighted_sum_dense uploads the weights instead (same bits)."""
    lib = _lib.load()
    cases = [(2000, 140_000, torch.float32, {}), (64, 20_000, torch.float32, {}),
             (64, 200_000, torch.float32, {"mode": "split"}), (32, 200_000, torch.bfloat16, {"reference_bf16": True})]
    for K, P, dt, kw in cases:
        x = torch.empty(K, P, dtype=dt, device=cuda)
        kernels.fill_synth(x, seed=1)
        w = np.float32(ref.fedavg_weights(K, seed=1))
        before = dict(kernels.HOST_WEIGHT_PATHS)
        got = kernels.weighted_sum_dense(x, w, scale=1e-4, **kw)
        assert kernels.HOST_WEIGHT_PATHS["uploaded"] == before["uploaded"] + 1, (K, P, kw)
        want = kernels.weighted_sum_dense(x, torch.from_numpy(w).to(cuda), scale=1e-4, **kw)
        assert torch.equal(got.float().view(torch.int32), want.float().view(torch.int32)), (K, P, kw)
    # the C ABI refuses up front with FJAGG_EUNSUPPORTED and a message
    x = torch.empty(4, 1024, dtype=torch.int32, device=cuda)
    wi = np.ones(4, np.int32)
    rc = lib.fjagg_wsum_dense(_lib.I32, _lib.I32, _lib.I32, x.data_ptr(), 1024, 4, 1024, wi.ctypes.data, 1.0,
                              x.data_ptr(), _lib.HOST_TABLES, 0, None, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == -3 and b"HOST_TABLES" in lib.fjagg_last_error()


def test_dense_host_weights_graph_capture(cuda, coracle):
    """A captured fold holds the weights it was captured with (the kernel arguments are
    copied into the graph node); the host array may change afterwards."""
    K, P = 64, 400_000
    x = torch.empty(K, P, device=cuda)
    kernels.fill_synth(x, seed=12)
    w = np.float32(ref.fedavg_weights(K, seed=12))
    out = torch.empty(P, device=cuda)
    s = torch.cuda.Stream()
    kernels.weighted_sum_dense(x, w, scale=1e-3, out=out)  # warm (residency query outside capture)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        kernels.weighted_sum_dense(x, w, scale=1e-3, out=out)
    w[:] = 0.0
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    want = coracle.wsum_f32(coracle.synth_f32(K, P, seed=12), np.float32(ref.fedavg_weights(K, seed=12)), scale=1e-3)
    assert np.array_equal(u32(out), want.astype(np.float32).view(np.int32))


def _emnist_clients(K, cuda, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [tmap(lambda s: (torch.rand(s, generator=g) * 2 - 1).to(cuda), EMNIST) for _ in range(K)]


def test_pytree_image_in_kernel_args_configs1(cuda, tu_settings):
    """configs[1] (128 clients x the 8 EMNIST-CNN leaves, separate allocations): tree_mean's
    native path carries the whole plan image (~13 KB) in the kernel arguments; the mean and
    the fused norms are bitwise the device-image launches of the Python path, and the mean
    is bitwise the oracle's."""
    tu_settings(_PIPELINE_FRAC=0.0)  # one launch per call (tests/test_gpu_pipeline.py: two)
    K = 128
    trees = _emnist_clients(K, cuda, 1)
    weights = [int(v) for v in ref.fedavg_weights(K, seed=5)]
    host = _lib.host()
    p0 = host.image_paths()
    got = tu.tree_mean(list(zip(trees, weights)))
    got_l2, norms = tu.tree_mean_with_l2_norms(list(zip(trees, weights)))
    p1 = host.image_paths()
    assert p1["kernel_args"] - p0["kernel_args"] == 2 and p1["uploaded"] == p0["uploaded"]
    # the Python path builds the same image in device memory (fjagg_wsum_ptrs without the flag)
    _, rows = tu._client_table(trees)
    leaves = [tu.pytree.leaves_of(t) for t in trees]
    slow = tu._fold(leaves, weights, scale=tu._inverse(float(sum(weights))), validated=True)
    q = torch.empty(K, device=cuda)
    slow_l2 = tu._fold(leaves, weights, scale=tu._inverse(float(sum(weights))), validated=True, l2sq=q)
    for a, b, c, d in zip(tu.pytree.leaves_of(got), slow, tu.pytree.leaves_of(got_l2), slow_l2):
        assert np.array_equal(u32(a), u32(b)) and np.array_equal(u32(c), u32(d)) and np.array_equal(u32(a), u32(c))
    assert np.array_equal(u32(norms), np.sqrt(q.cpu().numpy()).view(np.int32))  # correctly rounded sqrt
    want = ref.tree_mean([([x.cpu().numpy() for x in lv], w) for lv, w in zip(leaves, weights)])
    for a, b in zip(tu.pytree.leaves_of(got), want):
        assert np.array_equal(u32(a), b.view(np.int32))


def test_pytree_image_too_large_is_uploaded(cuda, tu_settings):
    """An image beyond FJAGG_KARG_MAX_WORDS (here 640 clients x 8 leaves) takes the
    pinned upload; misaligned leaves (per-leaf element units) still fit the kernel
    arguments. Both bitwise the Python path."""
    tu_settings(_PIPELINE_FRAC=0.0)  # one launch per call
    host = _lib.host()
    g = torch.Generator(device="cpu").manual_seed(2)
    # 280 KB per client (above the narrow plan's 256 KiB), 5,120 client leaves
    trees = [{"a": torch.randn(70_000, generator=g).to(cuda), "b": [torch.randn(50, generator=g).to(cuda)] * 7}
             for _ in range(640)]
    w = list(range(1, 641))
    p0 = host.image_paths()
    got = tu.tree_mean(list(zip(trees, w)))
    p1 = host.image_paths()
    assert p1["uploaded"] - p0["uploaded"] == 1 and p1["kernel_args"] == p0["kernel_args"]
    leaves = [tu.pytree.leaves_of(t) for t in trees]
    slow = tu._fold(leaves, w, scale=tu._inverse(float(sum(w))), validated=True)
    for a, b in zip(tu.pytree.leaves_of(got), slow):
        assert np.array_equal(u32(a), u32(b))
    base = torch.randn(9, 20_003, generator=g).to(cuda)
    odd = [{"a": base[k, 1:10_001], "b": base[k, 10_001:]} for k in range(9)]  # 4-byte offsets
    p0 = host.image_paths()
    got = tu.tree_mean(list(zip(odd, w[:9])))
    assert host.image_paths()["kernel_args"] - p0["kernel_args"] == 1
    slow = tu._fold([tu.pytree.leaves_of(t) for t in odd], w[:9], scale=tu._inverse(45.0), validated=True)
    for a, b in zip(tu.pytree.leaves_of(got), slow):
        assert np.array_equal(u32(a), u32(b))
