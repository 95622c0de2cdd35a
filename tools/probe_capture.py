"""What the default settings (deferred sums, lazy norms) do under HIP graph capture, and what a
capture-status query costs: hipStreamIsCapturing on the current stream (ns per call), then the
library loop (fed_avg.py:132-146) and tree_mean captured once and replayed on new contents,
compared with the eager results. Prints one JSON line; exploration only."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import pytree, tree_util as tu  # noqa: E402

dev = torch.device("cuda:0")
res = {}
hip = ctypes.CDLL("libamdhip64.so")
st = torch.cuda.current_stream(dev)
status = ctypes.c_int(0)
n = 100000
t0 = time.perf_counter()
for _ in range(n):
    hip.hipStreamIsCapturing(ctypes.c_void_p(st.cuda_stream), ctypes.byref(status))
res["hipStreamIsCapturing_ctypes_ns"] = round((time.perf_counter() - t0) / n * 1e9, 1)
t0 = time.perf_counter()
for _ in range(n):
    torch.cuda.is_current_stream_capturing()
res["torch_is_current_stream_capturing_ns"] = round((time.perf_counter() - t0) / n * 1e9, 1)

g0 = torch.Generator(device=dev).manual_seed(0)
xs = [{"u": torch.rand(5000, device=dev, generator=g0), "v": torch.rand(33, 9, device=dev, generator=g0)}
      for _ in range(6)]
W = float(sum(range(1, 7)))


def loop():
    s = tu.tree_zeros_like(xs[0])
    for k, x in enumerate(xs):
        s = tu.tree_add(s, tu.tree_weight(x, k + 1))
    return tu.tree_inverse_weight(s, W)


def mean():
    return tu.tree_mean([(x, k + 1) for k, x in enumerate(xs)])


def refill():
    with torch.no_grad():
        for x in xs:
            for leaf in pytree.leaves_of(x):
                leaf.copy_(torch.rand(leaf.shape, device=dev, generator=g0))


for name, fn in (("library_loop", loop), ("tree_mean", mean)):
    try:
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                out = fn()
        ok = []
        for _ in range(2):
            refill()
            g.replay()
            torch.cuda.synchronize()
            want = fn()
            ok.append(all(torch.equal(a.view(torch.int32), b.view(torch.int32))
                          for a, b in zip(pytree.leaves_of(out), pytree.leaves_of(want))))
        res[name] = {"replays_bitwise": ok, "out_type": type(out).__name__}
    except Exception as e:  # noqa: BLE001
        res[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
print(json.dumps(res))
