"""One synchronous fedjax_amd.tree_util.tree_mean call at configs[1] (128 clients x EMNIST-CNN,
one allocation per client leaf, the drop-in `examples/fed_avg.py:82` call): wall time per call
(device idle before each, synchronised after) and the builtin's host phases per call
(fjhost.host_timers: spec = client walk before the first launch, checks, outputs, plan, image,
launch, wrap; first_launch_at = host microseconds from the call's start to its first launch).
One JSON line. usage: python tools/prof_sync_tree_mean.py [calls]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import _lib, kernels, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tree(k, dev):
    out, seed = {}, 1
    for mod, leaves in SHAPES.items():
        out[mod] = {}
        for name, shp in leaves.items():
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=seed, k0=k)
            out[mod][name] = x.view(shp)
            seed += 1
    return out


def main(calls=200, K=128):
    dev = torch.device("cuda:0")
    pairs = list(zip([tree(k, dev) for k in range(K)], np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    for _ in range(20):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    host = _lib.host()
    host.host_timers()
    wall, back = [], []
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = tu.tree_mean(pairs)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        wall.append((t2 - t0) * 1e6)
        back.append((t1 - t0) * 1e6)
        del m
    phases = {k: round(v, 2) for k, v in host.host_timers().items()}
    print(json.dumps({"workload": "configs[1] synchronous tree_mean, separate leaf allocations",
                      "call_us_median": round(float(np.median(wall)), 1),
                      "returns_after_us_median": round(float(np.median(back)), 1),
                      "host_phases_us_per_call": phases}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
