"""Where a tree_mean that fuses standalone lazy norms spends its host time, against the same
tree_mean without norms (configs[1], 128 clients): fjhost.host_timers() phases and the image
paths (kernel arguments / uploaded) of each, over 20 rounds."""
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
dev = torch.device("cuda:0")


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


pairs = [(tree(k), 1 + k % 50) for k in range(128)]
H = tu._HOST
res = {}
for mode in ("plain", "norms", "plain", "norms"):
    H.host_timers()
    H.solo_times()
    p0 = H.image_paths()
    calls = []
    for _ in range(20):
        diag = None
        torch.cuda.synchronize()
        if mode == "norms":
            diag = [tu.tree_l2_norm(d) for d, _ in pairs]
        t0 = time.perf_counter()
        tu.tree_mean(pairs)
        calls.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    p1 = H.image_paths()
    res[mode] = {"mean_call_us": round(float(np.median(calls)) * 1e6, 1), "timers": H.host_timers(),
                 "image_paths": {k: p1[k] - p0[k] for k in p1},
                 "solo_times_per_call": {k: round(v / 20, 2) for k, v in H.solo_times().items()}}
print(json.dumps(res))
