"""One server round at configs[1] (128 clients x EMNIST-CNN, separate allocations), synchronous
and back to back: tree_mean then a separate Adam step through the fused kernel's own path,
versus fused_tree_mean_update (fold + Adam in one launch). Prints one JSON line (us, medians)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import server, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def timed(fn, n=100):
    for _ in range(5):
        fn()
    sync = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        sync.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round(float(np.median(sync)), 1), round((time.perf_counter() - t0) / n * 1e6, 1)


def main(K=128):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    clients = [tmap(lambda s: (torch.rand(s, device=dev, generator=g) - 0.5) * 0.01, SHAPES) for _ in range(K)]
    pairs = list(zip(clients, np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    params = tmap(lambda s: torch.randn(s, device=dev, generator=g), SHAPES)
    opt = server.adam(1e-3)
    st = [opt.init(params)]

    def fused():
        st[0] = server.fused_tree_mean_update(pairs, opt, params, st[0])

    res = {}
    res["fused_tree_mean_update_sync_us"], res["fused_tree_mean_update_b2b_us"] = timed(fused)
    res["tree_mean_sync_us"], res["tree_mean_b2b_us"] = timed(lambda: tu.tree_mean(pairs))
    print(json.dumps({"workload": "configs[1] server round, Adam", **res}), flush=True)


if __name__ == "__main__":
    main()
