"""HIP graph capture of the launches whose arguments live on the device or in the kernel
arguments (no allocation or synchronisation inside the library).

A server that runs the same round shape every round can capture the aggregation once
and replay it (torch.cuda.CUDAGraph = hipGraph on ROCm): the dense slab fold (weights on
the device), the per-call tree ops (fjtree: the leaf table is in the kernel arguments), and
the pytree folds of tree_mean and the deferred running sum while their plan image fits the
kernel arguments. A plan image too large for them would be uploaded from a pinned staging
buffer that torch hands out again after the capture: such a capture is refused with an error.
Replays must give the eager launch's bits on the new contents of the same buffers.
"""
import numpy as np
import pytest
import torch

from fedjax_amd import kernels, pytree, tree_util as tu

pytestmark = pytest.mark.gpu


def test_dense_fold_replays_bitwise(cuda):
    K, P = 64, 100_003
    x = torch.empty(K, P + 1, device=cuda)[:, :P]
    w = torch.tensor(np.float32(np.random.RandomState(0).randint(1, 501, size=K)), device=cuda)
    out = torch.empty(P, device=cuda)
    scale = float(np.float32(1.0 / float(w.double().sum())))
    kernels.fill_synth(x, seed=1)
    kernels.weighted_sum_dense(x, w, scale=scale, out=out)  # warm-up outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            kernels.weighted_sum_dense(x, w, scale=scale, out=out)
    for seed in (2, 3):
        kernels.fill_synth(x, seed=seed)
        g.replay()
        torch.cuda.synchronize()
        want = kernels.weighted_sum_dense(x, w, scale=scale)
        assert torch.equal(out.view(torch.int32), want.view(torch.int32))


def test_per_call_tree_ops_replay_bitwise(cuda):
    """tree_add(a, tree_weight(b, 3)) and tree_l2_norm(b) in eager mode (one fjtree launch
    each) captured once, replayed on new contents of a and b."""
    tu.set_deferred_sums(False)
    try:
        g0 = torch.Generator(device=cuda).manual_seed(0)
        a = {"u": torch.rand(5000, device=cuda, generator=g0), "v": torch.rand(33, 9, device=cuda, generator=g0)}
        b = {"u": torch.rand(5000, device=cuda, generator=g0), "v": torch.rand(33, 9, device=cuda, generator=g0)}
        tu.tree_add(a, tu.tree_weight(b, 3))  # warm-up: workspaces, plans
        tu.tree_l2_norm(b)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            tu.tree_add(a, tu.tree_weight(b, 3))  # this stream's norm workspace exists before capture
            tu.tree_l2_norm(b)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                out = tu.tree_add(a, tu.tree_weight(b, 3))
                nrm = tu.tree_l2_norm(b)
        for k in range(2):
            with torch.no_grad():
                for t in (a, b):
                    for leaf in pytree.leaves_of(t):
                        leaf.copy_(torch.rand(leaf.shape, device=cuda, generator=g0))
            g.replay()
            torch.cuda.synchronize()
            want = tu.tree_add(a, tu.tree_weight(b, 3))
            want_n = tu.tree_l2_norm(b)
            for x, y in zip(pytree.leaves_of(out), pytree.leaves_of(want)):
                assert torch.equal(x.view(torch.int32), y.view(torch.int32))
            assert torch.equal(nrm.view(torch.int32), want_n.view(torch.int32))
    finally:
        tu.set_deferred_sums(True)


def test_default_settings_capture_replays_or_refuses(cuda):
    """With the defaults (deferred running sums, lazy norms) a captured library-loop round and a
    small tree_mean record their launches with the plan images in the kernel arguments and replay
    bitwise on new contents. A tree_mean whose image is too large for the kernel arguments would
    upload it through a pinned staging buffer, which torch's host allocator hands out again after
    the capture: that capture is refused with an error (nothing is recorded that a replay could
    not reuse), and the stream works normally afterwards."""
    g0 = torch.Generator(device=cuda).manual_seed(5)
    xs = [{"u": torch.rand(5000, device=cuda, generator=g0), "v": torch.rand(33, 9, device=cuda, generator=g0)}
          for _ in range(6)]
    W = float(sum(range(1, 7)))

    def loop():
        s = tu.tree_zeros_like(xs[0])
        for k, x in enumerate(xs):
            s = tu.tree_add(s, tu.tree_weight(x, k + 1))
        return tu.tree_inverse_weight(s, W)

    def mean():
        return tu.tree_mean([(x, k + 1) for k, x in enumerate(xs)])

    for fn in (loop, mean):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                out = fn()
        for _ in range(2):
            with torch.no_grad():
                for x in xs:
                    for leaf in pytree.leaves_of(x):
                        leaf.copy_(torch.rand(leaf.shape, device=cuda, generator=g0))
            g.replay()
            torch.cuda.synchronize()
            want = fn()
            for a, b in zip(pytree.leaves_of(out), pytree.leaves_of(want)):
                assert torch.equal(a.view(torch.int32), b.view(torch.int32)), fn.__name__
    big = [{"u": torch.rand(64, device=cuda, generator=g0), "v": torch.rand(8, device=cuda, generator=g0)}
           for _ in range(2000)]
    pairs = [(t, 1 + k % 7) for k, t in enumerate(big)]
    want = tu.tree_mean(pairs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with pytest.raises(RuntimeError, match="not capturable"):
            with torch.cuda.graph(g, stream=s):
                tu.tree_mean(pairs)
    torch.cuda.synchronize()
    again = tu.tree_mean(pairs)
    for a, b in zip(pytree.leaves_of(again), pytree.leaves_of(want)):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_captured_rounds_with_norms_replay(cuda):
    """examples/fed_avg.py's round (tree_l2_norm per client, then tree_mean) and the library loop
    with its per-client norms (fed_avg.py:132-146), captured with the default settings. Under a
    capture the norms come from launches recorded in the graph (no pooled norm columns, which a
    replay would overwrite after they are handed out again; fjhost stream_capturing), so every
    replay refreshes the mean and the norms: the bits of an eager round on the new contents.
    Eager rounds on the capture stream afterwards keep their own bits."""
    g0 = torch.Generator(device=cuda).manual_seed(9)
    xs = [{"u": torch.rand(5000, device=cuda, generator=g0), "v": torch.rand(33, 9, device=cuda, generator=g0)}
          for _ in range(6)]
    ws = [3, 1, 4, 1, 5, 9]

    def example():
        norms = [tu.tree_l2_norm(x) for x in xs]
        return tu.tree_mean(list(zip(xs, ws))), norms

    def library():
        s, norms = tu.tree_zeros_like(xs[0]), []
        for x, w in zip(xs, ws):
            s = tu.tree_add(s, tu.tree_weight(x, w))
            norms.append(tu.tree_l2_norm(x))
        return tu.tree_inverse_weight(s, float(sum(ws))), norms

    def same(a, b):
        return all(torch.equal(x.reshape(-1).view(torch.int32), y.reshape(-1).view(torch.int32))
                   for x, y in zip(pytree.leaves_of(a), pytree.leaves_of(b)))

    for fn in (example, library):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                mean, norms = fn()
        for _ in range(2):
            with torch.no_grad():
                for x in xs:
                    for leaf in pytree.leaves_of(x):
                        leaf.copy_(torch.rand(leaf.shape, device=cuda, generator=g0))
            g.replay()
            torch.cuda.synchronize()
            want, want_norms = fn()
            assert same(mean, want), fn.__name__
            assert same(norms, want_norms), fn.__name__
        with torch.cuda.stream(st):
            again, again_norms = fn()
        st.synchronize()
        assert same(again, want) and same(again_norms, want_norms), fn.__name__


def test_recorded_zeroing_runs_on_every_replay(cuda):
    """On this ROCm a hipMemsetAsync recorded into a graph takes effect on the first replay only
    (tools/probe_memset_node.py), so what the captured calls zero, they zero with a kernel:
    tree_zeros_like's running-sum base (eager mode: one fused fjtree launch per tree_add, which
    reads it) and the split-mode dense fold's unit weights. Both replay bitwise three times on
    new contents."""
    g0 = torch.Generator(device=cuda).manual_seed(13)
    xs = [{"u": torch.rand(5000, device=cuda, generator=g0), "v": torch.rand(33, 9, device=cuda, generator=g0)}
          for _ in range(6)]
    tu.set_deferred_sums(False)
    try:
        def loop():
            s = tu.tree_zeros_like(xs[0])
            for k, x in enumerate(xs):
                s = tu.tree_add(s, tu.tree_weight(x, k + 1))
            return s
        loop()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            loop()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                out = loop()
        for _ in range(3):
            with torch.no_grad():
                for x in xs:
                    for leaf in pytree.leaves_of(x):
                        leaf.copy_(torch.rand(leaf.shape, device=cuda, generator=g0))
            g.replay()
            torch.cuda.synchronize()
            want = loop()
            for a, b in zip(pytree.leaves_of(out), pytree.leaves_of(want)):
                assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    finally:
        tu.set_deferred_sums(True)
    K, P = next((k, p) for k, p in ((4096, 2048), (8192, 1024), (16384, 512), (2048, 4096))
                if kernels.split_workspace_bytes(k, p) > 0)
    x = torch.empty(K, P, device=cuda)
    w = torch.tensor(np.float32(np.random.RandomState(3).randint(1, 501, size=K)), device=cuda)
    scale = float(np.float32(1.0 / float(w.double().sum())))
    ws = torch.empty(kernels.split_workspace_bytes(K, P), dtype=torch.uint8, device=cuda)
    out = torch.empty(P, device=cuda)
    kernels.fill_synth(x, seed=1)
    kernels.weighted_sum_dense(x, w, scale=scale, out=out, mode="split", workspace=ws)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            kernels.weighted_sum_dense(x, w, scale=scale, out=out, mode="split", workspace=ws)
    for seed in (2, 3, 4):
        kernels.fill_synth(x, seed=seed)
        g.replay()
        torch.cuda.synchronize()
        want = kernels.weighted_sum_dense(x, w, scale=scale, mode="split")
        assert torch.equal(out.view(torch.int32), want.view(torch.int32)), seed


def test_dense_fused_norms_capture_on_a_fresh_stream(cuda):
    """kernels.weighted_sum_l2_dense without a workspace uses the stream's cached zeroed-counter
    workspace; first used inside a capture, that workspace would be zeroed by a recorded fill that
    has not run yet. The capture gets a workspace of its own: replays give the eager bits, and eager
    calls on the capture stream afterwards (before and after a replay) do too."""
    K, P = 64, 100_003
    x = torch.empty(K, P + 1, device=cuda)[:, :P]
    w = torch.tensor(np.float32(np.random.RandomState(5).randint(1, 501, size=K)), device=cuda)
    scale = float(np.float32(1.0 / float(w.double().sum())))
    out = torch.empty(P, device=cuda)
    l2 = torch.empty(K, device=cuda)
    kernels.fill_synth(x, seed=1)
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()  # (a stream no fused-norm call has used yet)
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            kernels.weighted_sum_l2_dense(x, w, scale=scale, out=out, l2sq=l2)

    def eager_on(stream):
        with torch.cuda.stream(stream):
            o, n = kernels.weighted_sum_l2_dense(x, w, scale=scale)
        stream.synchronize()
        return o, n

    o0, n0 = eager_on(st)  # before any replay
    o1, n1 = kernels.weighted_sum_l2_dense(x, w, scale=scale, workspace=torch.empty(1, dtype=torch.uint8, device=cuda))
    torch.cuda.synchronize()  # (a caller's workspace: two launches, the same bits)
    assert torch.equal(o0.view(torch.int32), o1.view(torch.int32)) and torch.equal(n0.view(torch.int32), n1.view(torch.int32))
    for seed in (2, 3, 4):
        kernels.fill_synth(x, seed=seed)
        g.replay()
        torch.cuda.synchronize()
        want_o, want_n = eager_on(st)
        assert torch.equal(out.view(torch.int32), want_o.view(torch.int32)), seed
        assert torch.equal(l2.view(torch.int32), want_n.view(torch.int32)), seed


def test_c_abi_zeroed_counter_captured_after_zeroing(cuda):
    """The FJAGG_ZEROED_WS contract for a C caller (include/fjagg.h): a workspace whose counter was
    zeroed before the capture stays zero across replays (every launch leaves it zero), so a
    captured fjagg_wsum_l2_ptrs with its norm combine in the last workgroup replays the eager
    two-launch call's mean and norms bitwise, three times, on new contents."""
    import ctypes

    from fedjax_amd import _lib
    lib = _lib.load()
    shapes = [(32,), (3, 3, 1, 32), (9216, 16), (62,)]
    K, L = 24, 4
    rows = [[torch.empty(int(np.prod(s)), device=cuda) for s in shapes] for _ in range(K)]
    leaf_n = np.array([int(np.prod(s)) for s in shapes], dtype=np.int64)
    outs = [torch.empty(int(n), device=cuda) for n in leaf_n]
    nb = lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, leaf_n.ctypes.data, None, L, None, 0)
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(_lib.F32, 0, leaf_n.ctypes.data, None, L, blocks.ctypes.data, nb)
    img = torch.from_numpy(np.concatenate([np.array([[x.data_ptr() for x in r] for r in rows], np.int64).ravel(),
                                           np.array([o.data_ptr() for o in outs], np.int64), leaf_n, blocks])).to(cuda)
    w = torch.tensor(np.float32(np.arange(1, K + 1)), device=cuda)
    l2 = torch.empty(K, device=cuda)
    need = max(16, int(lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)))
    ws = torch.zeros(need, dtype=torch.uint8, device=cuda)  # zeroed before the capture
    torch.cuda.synchronize()

    def call(l2_out, flags, work, stream):
        _lib.check(lib.fjagg_wsum_l2_ptrs(_lib.F32, _lib.F32, _lib.F32, img.data_ptr(), L, K, nb, w.data_ptr(),
                                          ctypes.c_float(0.01), l2_out.data_ptr(), flags, work.data_ptr(),
                                          work.numel(), ctypes.c_void_p(stream.cuda_stream)), "fjagg_wsum_l2_ptrs")

    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            call(l2, _lib.SCALE | _lib.ZEROED_WS, ws, st)
    for seed in (1, 2, 3):
        for k, r in enumerate(rows):
            for x in r:
                kernels.fill_synth(x.view(1, -1), seed=seed, k0=k)
        g.replay()
        torch.cuda.synchronize()
        got_mean = torch.cat([o.clone() for o in outs])
        want_l2 = torch.empty(K, device=cuda)
        call(want_l2, _lib.SCALE, torch.empty(need, dtype=torch.uint8, device=cuda), torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert torch.equal(l2.view(torch.int32), want_l2.view(torch.int32)), seed
        assert torch.equal(got_mean.view(torch.int32), torch.cat(outs).view(torch.int32)), seed
        assert int(ws[:8].view(torch.int32)[0]) == 0 and int(ws[:8].view(torch.int32)[1]) == 0  # counter, error word
