"""ns per call of tree_weight's capture parts (fjhost.capture_probe) on a configs[1] EMNIST-CNN
delta: one tree repeated (caches warm) and 128 different trees in turn (as the library loop
walks them), plus the whole tree_weight and tree_l2_norm calls per client over the 128; the same
for the standalone lazy norm's capture (fjhost.solo_probe)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import tree_util as tu  # noqa: E402

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
dev = torch.device("cuda:0")
trees = []
for k in range(128):
    trees.append({m: {n: torch.empty(1, int(np.prod(s)), device=dev).view(s) for n, s in lv.items()}
                  for m, lv in SHAPES.items()})
H = tu._HOST
res = {"one_tree": H.capture_probe(trees[0], 20000), "solo_one_tree": H.solo_probe(trees[0], 20000)}
parts = {}
for t in trees:
    for k, v in H.capture_probe(t, 1).items():
        parts.setdefault(k, []).append(v)
res["128_trees_median"] = {k: round(float(np.median(v)), 1) for k, v in parts.items()}
parts = {}
for t in trees:
    for k, v in H.solo_probe(t, 1).items():
        parts.setdefault(k, []).append(v)
res["solo_128_trees_median"] = {k: round(float(np.median(v)), 1) for k, v in parts.items()}
pc = time.perf_counter
for name, fn in (("tree_weight", lambda t: tu.tree_weight(t, 3)), ("tree_l2_norm", tu.tree_l2_norm)):
    best = 1e9
    for _ in range(20):
        t0 = pc()
        keep = [fn(t) for t in trees]
        best = min(best, (pc() - t0) / len(trees) * 1e9)
        del keep
    res[name + "_ns_per_client"] = round(best, 1)
print(json.dumps(res))
