"""Synchronous configs[1] tree_mean (128 EMNIST-CNN clients, separate leaf allocations) under
several first-chunk schedules of the fold-bound pipeline (fjhost.pipeline_fracs: chunk ends as
fractions of K; [] = the single 0.2 first chunk), interleaved, medians; bitwise checked."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import kernels, pytree, tree_util as tu  # noqa: E402

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


pairs = [(tree(k), 1 + (k * 37) % 500) for k in range(128)]
H = tu._HOST
SCHEDULES = [[], [0.06, 0.2], [0.08, 0.25, 0.6], [0.05, 0.15, 0.4], [0.1, 0.35], [0.04, 0.12, 0.32, 0.7]]
if len(sys.argv) > 1:  # e.g. '[[], [0.1], [0.15], [0.3]]': single first chunks of other sizes
    SCHEDULES = json.loads(sys.argv[1])
ref = [x.clone() for x in pytree.leaves_of(tu.tree_mean(pairs))]
times = {str(s): [] for s in SCHEDULES}
pc = time.perf_counter
for rep in range(60):
    for s in SCHEDULES:
        H.pipeline_fracs(s)
        torch.cuda.synchronize()
        t0 = pc()
        m = tu.tree_mean(pairs)
        torch.cuda.synchronize()
        times[str(s)].append(pc() - t0)
        if rep == 0:
            assert all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(pytree.leaves_of(m), ref))
H.pipeline_fracs([])
print(json.dumps({k: round(float(np.median(v[5:])) * 1e3, 4) for k, v in times.items()}))
