"""Host cost of examples/fed_avg.py:72-82's round at configs[1] (128 EMNIST-CNN deltas, one
allocation per (client, leaf)): per-call tree_l2_norm host time, one synchronous round with the
norms (lazy views the mean fills), the same tree_mean without norms, and the eager norms
(set_lazy_norms(False)) for comparison. Rounds alternate; medians. Prints one JSON line.

usage: python tools/time_example_round.py [--rounds 40] [--clients 128]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import kernels, tree_util as tu  # noqa: E402

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--clients", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    K = a.clients

    def tree(k):
        out, seed = {}, 1
        for mod, leaves in SHAPES.items():
            out[mod] = {}
            for name, shp in leaves.items():
                x = torch.empty(1, int(np.prod(shp)), device=dev)
                kernels.fill_synth(x, seed=seed, k0=k)
                out[mod][name] = x.view(shp)
                seed += 1
        return out

    pairs = [(tree(k), 1 + (k * 37) % 500) for k in range(K)]
    pc = time.perf_counter
    H = tu._HOST
    res = {"clients": K}
    modes = ["norms", "mean_only", "eager_norms"]
    t = {m: [] for m in modes}
    parts = {"loop": [], "mean_call": [], "wait": []}
    for i in range(3 * (a.rounds + 2)):
        m = modes[i % 3]
        tu.set_lazy_norms(m != "eager_norms")
        diag = lst = None  # (the previous round's diagnostics are freed outside the timed region)
        torch.cuda.synchronize()
        t0 = pc()
        if m == "mean_only":
            tu.tree_mean(pairs)
            t1 = t0
            t2 = pc()
        else:
            diag, lst = {}, []
            for cid, (d, n) in enumerate(pairs):
                lst.append((d, n))
                diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
            t1 = pc()
            tu.tree_mean(lst)
            t2 = pc()
        torch.cuda.synchronize()
        t3 = pc()
        if i >= 6:
            t[m].append(t3 - t0)
            if m == "norms":
                parts["loop"].append(t1 - t0)
                parts["mean_call"].append(t2 - t1)
                parts["wait"].append(t3 - t2)
            elif m == "mean_only":
                parts.setdefault("plain_mean_call", []).append(t2 - t1)
                parts.setdefault("plain_wait", []).append(t3 - t2)
    tu.set_lazy_norms(True)
    for m in modes:
        res[m + "_ms"] = round(float(np.median(t[m])) * 1e3, 4)
    for k, v in parts.items():
        res["norms_round_" + k + "_us"] = round(float(np.median(v)) * 1e6, 1)
    res["norm_call_us"] = round(res["norms_round_loop_us"] / K, 3)
    only = []
    for i in range(a.rounds):  # norm rounds back to back (no other mode in between)
        torch.cuda.synchronize()
        t0 = pc()
        diag, lst = {}, []
        for cid, (d, n) in enumerate(pairs):
            lst.append((d, n))
            diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
        tu.tree_mean(lst)
        torch.cuda.synchronize()
        only.append(pc() - t0)
    res["norms_only_rounds_ms"] = round(float(np.median(only)) * 1e3, 4)
    # the example's loop without the norm call (its own Python: enumerate, append, the dict), and the
    # same loop calling the native tree_l2_norm, back to back with nothing on the GPU: the norm's share
    floor, calls = [], []
    for i in range(2 * a.rounds):
        diag = lst = None
        torch.cuda.synchronize()
        t0 = pc()
        diag, lst = {}, []
        if i % 2 == 0:
            for cid, (d, n) in enumerate(pairs):
                lst.append((d, n))
                diag[cid] = {"delta_l2_norm": d}
        else:
            for cid, (d, n) in enumerate(pairs):
                lst.append((d, n))
                diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
        (floor if i % 2 == 0 else calls).append(pc() - t0)
        if i % 2:
            tu.tree_mean(lst)  # (fills the views: the registry does not grow)
            torch.cuda.synchronize()
    # the same 128 calls on two trees in turn (their metadata stays in cache): the call's own work
    warm = []
    two = [pairs[0][0], pairs[1][0]]
    for i in range(a.rounds):
        diag = None
        torch.cuda.synchronize()
        t0 = pc()
        diag = {}
        for cid in range(K):
            diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(two[cid & 1])}
        warm.append(pc() - t0)
        tu.tree_mean([(t, 1) for t in two])
        torch.cuda.synchronize()
    res["example_loop_norm_calls_on_two_warm_trees_us"] = round(float(np.median(warm)) * 1e6, 1)
    res["example_loop_without_norm_call_us"] = round(float(np.median(floor)) * 1e6, 1)
    res["example_loop_with_norm_call_us"] = round(float(np.median(calls)) * 1e6, 1)
    res["ratio_norms_vs_mean_only"] = round(res["norms_ms"] / res["mean_only_ms"], 4)
    res["solo_info"] = H.solo_info()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
