"""cProfile of the library running-sum loop (fedjax/algorithms/fed_avg.py:132-146) at
configs[1]: where the host time of tree_weight / tree_add goes. Prints the top entries."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def rounds(deltas, weights, params, n):
    for _ in range(n):
        s = tu.tree_zeros_like(params)
        for d, w in zip(deltas, weights):
            s = tu.tree_add(s, tu.tree_weight(d, w))
        tu.tree_inverse_weight(s, float(sum(weights)))
    torch.cuda.synchronize()


def main(K=128):
    if len(sys.argv) > 1:  # flush_bytes of the deferred chain (tree_util.set_deferred_sums)
        tu.set_deferred_sums(True, flush_bytes=int(sys.argv[1]))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    deltas = [tmap(lambda s: torch.rand(s, device=dev, generator=g) - 0.5, SHAPES) for _ in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    params = tmap(lambda s: torch.zeros(s, device=dev), SHAPES)
    rounds(deltas, weights, params, 5)
    t0 = time.perf_counter()
    rounds(deltas, weights, params, 50)
    print(f"round_ms {(time.perf_counter() - t0) / 50 * 1e3:.4f} flush_bytes {tu._DEFER['flush_bytes']}", flush=True)
    if os.environ.get("CPROF", "1") == "0":
        return
    pr = cProfile.Profile()
    pr.enable()
    rounds(deltas, weights, params, 50)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
