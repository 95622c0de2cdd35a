"""Host cost of an early flush of a deferred running sum (tree_util.set_deferred_sums
flush_bytes) at configs[1]: the library loop (fed_avg.py:132-146, 128 clients x EMNIST-CNN)
with the chain folded every ~53 clients, each _fold_chain call and its pieces timed with
perf_counter (wrappers around the module's functions). Prints one JSON line per setting."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import pytree, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
pc = time.perf_counter
T = {}


def timed(name, f):
    def w(*a, **k):
        t0 = pc()
        try:
            return f(*a, **k)
        finally:
            T.setdefault(name, []).append((pc() - t0) * 1e6)
    return w


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main(K=128):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    deltas = [tmap(lambda s: torch.rand(s, device=dev, generator=g) - 0.5, SHAPES) for _ in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    params = tmap(lambda s: torch.zeros(s, device=dev), SHAPES)
    for fb in (1 << 30, 256 << 20, 128 << 20):
        tu.set_deferred_sums(True, flush_bytes=fb)
        walls = []
        for r in range(25):
            if r == 5:
                T.clear()
                tu._fold_chain = timed("fold_chain", orig_chain)
                tu._fold = timed("fold", orig_fold)
                pytree.unflatten = timed("unflatten", orig_unflatten)
                tu.PendingSum.materialize = timed("materialize", orig_mat)
            torch.cuda.synchronize()
            t0 = pc()
            s = tu.tree_zeros_like(params)
            for d, w in zip(deltas, weights):
                s = tu.tree_add(s, tu.tree_weight(d, w))
            tu.tree_inverse_weight(s, float(sum(weights)))
            torch.cuda.synchronize()
            if r >= 5:
                walls.append((pc() - t0) * 1e3)
        tu._fold_chain, tu._fold, pytree.unflatten, tu.PendingSum.materialize = (orig_chain, orig_fold,
                                                                                 orig_unflatten, orig_mat)
        print(json.dumps({"flush_bytes": fb, "round_ms_median": round(float(np.median(walls)), 4),
                          **{f"{k}_us": [len(v) // 20, round(float(np.median(v)), 2)] for k, v in T.items()}}),
              flush=True)
    tu.set_deferred_sums(True, flush_bytes=1 << 30)


orig_chain, orig_fold, orig_unflatten, orig_mat = tu._fold_chain, tu._fold, pytree.unflatten, tu.PendingSum.materialize

if __name__ == "__main__":
    main()
