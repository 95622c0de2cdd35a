"""Per-call host cost of a standalone lazy tree_l2_norm (fjhost solo_norm) and its parts, on
the configs[1] EMNIST-CNN delta shape: the whole call, the capture alone (fjhost.capture, the
running sum's tree_weight capture), tree_weight, and whether any Python frame runs in the call."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import tree_util as tu  # noqa: E402

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
dev = torch.device("cuda:0")
trees = [{m: {n: torch.zeros(s, device=dev) for n, s in lv.items()} for m, lv in SHAPES.items()} for _ in range(128)]
tu.tree_mean([(t, 1) for t in trees[:2]])  # loads the library's entry points
H = tu._HOST
pc = time.perf_counter
res = {}


def per_call(fn, reps=20):
    best = 1e9
    for _ in range(reps):
        t0 = pc()
        keep = [fn(t) for t in trees]
        dt = (pc() - t0) / len(trees) * 1e6
        best = min(best, dt)
        del keep
        H.solo_resolve(None)
    return round(best, 3)


calls = []
sys.setprofile(lambda f, e, a: calls.append((e, f.f_code.co_name)) if e == "call" else None)
v = tu.tree_l2_norm(trees[0])
sys.setprofile(None)
res["python_frames_in_call"] = sorted({c[1] for c in calls})
res["view_ticket"] = type(v._ticket).__name__
del v
res["tree_l2_norm_us"] = per_call(tu.tree_l2_norm)
res["capture_us"] = per_call(lambda t: H.capture(t, -1))
res["tree_weight_us"] = per_call(lambda t: tu.tree_weight(t, 1))
res["solo_norm_direct_us"] = per_call(lambda t: H.solo_norm(t, 1))
res["info"] = H.solo_info()
print(json.dumps(res))
