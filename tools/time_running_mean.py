"""configs[1] (128 x EMNIST-CNN, 8 separate leaves per client) through the streaming
running sum of fedjax/algorithms/fed_avg.py:132-146 (aggregators.RunningMean) at
several buffer sizes B, next to tree_mean over the same clients. Wall time per round
(every client added, result() taken, synchronised). Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import aggregators, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def wall(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main(K=128, reps=20):
    dev = torch.device("cuda:0")
    template = tmap(lambda s: np.zeros(s, np.float32), SHAPES)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    P = slab.num_params
    clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    tmpl = clients[0]
    res = {"workload": "configs[1] 128 x EMNIST-CNN through RunningMean (fed_avg.py:132-146)",
           "tree_mean_ms": round(wall(lambda: tu.tree_mean(zip(clients, weights)), reps), 4)}
    ref = tu.tree_mean(zip(clients, weights))
    for B in (1, 8, 32, 128, None):
        def rnd():
            rm = aggregators.RunningMean(tmpl, buffer_clients=B, device=dev)
            for c, w in zip(clients, weights):
                rm.add(c, w)
            return rm.result()
        ms = wall(rnd, max(3, reps // (4 if B == 1 else 1)))
        out = rnd()
        same = all(torch.equal(a, b) for a, b in zip(fedjax_amd.pytree.leaves_of(out), fedjax_amd.pytree.leaves_of(ref)))
        res[f"B{B}_ms"] = round(ms, 4)
        res[f"B{B}_GBs"] = round(K * P * 4 / ms / 1e6, 1)
        res[f"B{B}_bitwise_eq_tree_mean"] = same
    # the reference loop itself, through this package's tree_util (fed_avg.py:132-146)
    def literal():
        s = tu.tree_zeros_like(tmpl)
        n = 0.
        for c, w in zip(clients, weights):
            s = tu.tree_add(s, tu.tree_weight(c, w))
            n += w
        return tu.tree_inverse_weight(s, n)
    res["literal_loop_ms"] = round(wall(literal, 10), 4)

    def literal_norms():  # + the per-client delta_l2_norm diagnostic of fed_avg.py:142-144
        s = tu.tree_zeros_like(tmpl)
        n, norms = 0., []
        for c, w in zip(clients, weights):
            s = tu.tree_add(s, tu.tree_weight(c, w))
            n += w
            norms.append(tu.tree_l2_norm(c))
        return tu.tree_inverse_weight(s, n)
    res["literal_loop_with_l2_norms_ms"] = round(wall(literal_norms, 10), 4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    literal_norms()
    res["literal_loop_with_l2_norms_host_issue_ms"] = round((time.perf_counter() - t0) * 1e3, 4)
    torch.cuda.synchronize()
    out = literal()
    res["literal_loop_bitwise_eq_tree_mean"] = all(
        torch.equal(a, b) for a, b in zip(fedjax_amd.pytree.leaves_of(out), fedjax_amd.pytree.leaves_of(ref)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
