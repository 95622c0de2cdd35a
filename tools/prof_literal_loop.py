"""Host-side cost of each call in the literal running-sum loop of
fedjax/algorithms/fed_avg.py:132-146 at configs[1] (128 clients x EMNIST-CNN, 8 separate
leaves each), through fedjax_amd.tree_util:

    s = tree_zeros_like(params)
    for each client: s = tree_add(s, tree_weight(delta, n)); tree_l2_norm(delta)
    mean = tree_inverse_weight(s, sum n)

Prints one JSON line: per-call host microseconds (median over rounds) of tree_weight,
tree_add and tree_l2_norm, the round's wall time (synchronised) and its host issue
time, and the GPU time of the launches (HIP events around one round)."""
import json
import os
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


def main(K=128, rounds=15):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    deltas = [tmap(lambda s: (torch.rand(s, device=dev, generator=g) - 0.5) * 0.02, SHAPES) for _ in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    params = tmap(lambda s: torch.zeros(s, device=dev), SHAPES)
    per = {"tree_weight": [], "tree_add": [], "tree_l2_norm": [], "round_wall": [], "round_issue": []}
    pc = time.perf_counter
    for r in range(rounds + 3):
        torch.cuda.synchronize()
        t_round = pc()
        tw = ta = tn = 0.0
        s = tu.tree_zeros_like(params)
        n_sum = 0.
        for d, n in zip(deltas, weights):
            t0 = pc()
            wt = tu.tree_weight(d, n)
            t1 = pc()
            s = tu.tree_add(s, wt)
            t2 = pc()
            tu.tree_l2_norm(d)
            t3 = pc()
            tw += t1 - t0
            ta += t2 - t1
            tn += t3 - t2
            n_sum += n
        mean = tu.tree_inverse_weight(s, n_sum)
        t_issue = pc() - t_round
        torch.cuda.synchronize()
        t_wall = pc() - t_round
        if r >= 3:
            per["tree_weight"].append(tw / K * 1e6)
            per["tree_add"].append(ta / K * 1e6)
            per["tree_l2_norm"].append(tn / K * 1e6)
            per["round_issue"].append(t_issue * 1e3)
            per["round_wall"].append(t_wall * 1e3)
    del mean
    res = {"workload": "configs[1] literal loop (fed_avg.py:132-146) incl. tree_l2_norm, K=128",
           "host_us_per_call": {k: round(float(np.median(per[k])), 2) for k in ("tree_weight", "tree_add",
                                                                               "tree_l2_norm")},
           "round_issue_ms": round(float(np.median(per["round_issue"])), 4),
           "round_wall_ms": round(float(np.median(per["round_wall"])), 4)}
    print(json.dumps(res), flush=True)
    if os.environ.get("CPROF", "0") == "1":  # where the per-call host time goes
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(20):
            s = tu.tree_zeros_like(params)
            for d, n in zip(deltas, weights):
                s = tu.tree_add(s, tu.tree_weight(d, n))
                tu.tree_l2_norm(d)
            tu.tree_inverse_weight(s, float(sum(weights)))
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(16)


if __name__ == "__main__":
    main()
