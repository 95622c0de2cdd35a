"""Where the host time of examples/fed_avg.py:79-81's norms goes inside a synchronous round:
per-call durations of tree_l2_norm over 128 configs[1] deltas (views of [1, n] allocations, as
bench.py builds them), their percentiles, with the GC on and off, and the same loop calling
fjhost.capture only."""
import gc
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
tu.tree_mean(pairs)
H = tu._HOST
pc = time.perf_counter
res = {}


def rounds(fn, n=30, sync=True, mean=True):
    per, tot = [], []
    for _ in range(n):
        if sync:
            torch.cuda.synchronize()
        diag, lst = {}, []
        t0 = pc()
        for cid, (d, w) in enumerate(pairs):
            a = pc()
            lst.append((d, w))
            diag[cid] = {"delta_l2_norm": fn(d)}
            per.append(pc() - a)
        tot.append(pc() - t0)
        if mean:
            tu.tree_mean(lst)
        else:
            H.solo_resolve(None)
    per = np.array(per) * 1e6
    return {"p10": round(float(np.percentile(per, 10)), 3), "p50": round(float(np.median(per)), 3),
            "p90": round(float(np.percentile(per, 90)), 3), "max": round(float(per.max()), 2),
            "loop_us_median": round(float(np.median(tot)) * 1e6, 1)}


res["norm"] = rounds(tu.tree_l2_norm)
gc.disable()
res["norm_gc_off"] = rounds(tu.tree_l2_norm)
gc.enable()
res["norm_nosync"] = rounds(tu.tree_l2_norm, sync=False)
res["capture"] = rounds(lambda t: H.capture(t, -1))
res["tree_weight"] = rounds(lambda t: tu.tree_weight(t, 1))
print(json.dumps(res))
