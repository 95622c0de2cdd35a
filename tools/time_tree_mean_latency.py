"""Single-call latency of tree_mean at configs[1] (128 clients x EMNIST-CNN, one allocation
per client leaf): the device is idle before each call and the call is waited for, as a
server that aggregates once per round sees it. Also the pipelined rate (calls back to back)
for comparison. Prints one JSON line per pipeline fraction (microseconds, medians):
    python tools/time_tree_mean_latency.py [FRAC ...]   (tree_util._PIPELINE_FRAC values,
    measured in interleaved rounds; default: the module's own; a negative FRAC = |FRAC|
    with the idle probe answering "busy": the probe's own cost, never pipelined)"""
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


def measure(pairs, reps):
    pc = time.perf_counter
    single, issue = [], []
    for i in range(reps + 10):
        torch.cuda.synchronize()
        t0 = pc()
        out = tu.tree_mean(pairs)
        t1 = pc()
        torch.cuda.synchronize()
        t2 = pc()
        if i >= 10:
            issue.append((t1 - t0) * 1e6)
            single.append((t2 - t0) * 1e6)
        del out
    torch.cuda.synchronize()
    t0 = pc()
    for _ in range(reps):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    piped = (pc() - t0) / reps * 1e6
    return single, issue, piped


def main(fracs, K=128, reps=100, rounds=3):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    clients = [tmap(lambda s: torch.rand(s, device=dev, generator=g), SHAPES) for _ in range(K)]
    pairs = list(zip(clients, np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    res = {f: ([], [], []) for f in fracs}
    idle = tu._stream_idle
    for _ in range(rounds):
        for f in fracs:
            if f is not None:
                tu._PIPELINE_FRAC = abs(f)
                tu._mean_config()  # (the builtin tree_mean keeps its own copy)
                tu._stream_idle = (lambda s: False) if f < 0 else idle
            s, i, p = measure(pairs, reps)
            res[f][0].extend(s)
            res[f][1].extend(i)
            res[f][2].append(p)
    for f, (s, i, p) in res.items():
        print(json.dumps({"K": K, "pipeline_frac": tu._PIPELINE_FRAC if f is None else f,
                          "single_call_us": round(float(np.median(s)), 1),
                          "single_call_host_issue_us": round(float(np.median(i)), 1),
                          "back_to_back_us_per_call": round(float(np.median(p)), 1)}), flush=True)


if __name__ == "__main__":
    main([float(a) for a in sys.argv[1:]] or [None])
