"""Timeline of one synchronised library-loop round (fedjax/algorithms/fed_avg.py:132-146) at
configs[1]: the client loop's host time (tree_weight + tree_add [+ tree_l2_norm] per client),
the final tree_inverse_weight call, and the wait for the GPU; per-call costs of tree_weight and
tree_add measured inside the loop. Medians over rounds; one JSON line."""
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
W = float(sum(w for _, w in pairs))
pc = time.perf_counter
res = {}
for with_norms in (False, True, False, True):
    parts = {"loop": [], "final_call": [], "wait": [], "round": [], "tw": [], "ta": [], "nrm": []}
    for r in range(30):
        diag = None
        torch.cuda.synchronize()
        t0 = pc()
        s, diag = tu.tree_zeros_like(pairs[0][0]), {}
        for cid, (t, w) in enumerate(pairs):
            a = pc()
            wt = tu.tree_weight(t, w)
            b = pc()
            s = tu.tree_add(s, wt)
            c = pc()
            if with_norms:
                diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(t)}
            d = pc()
            if r >= 5:
                parts["tw"].append(b - a), parts["ta"].append(c - b), parts["nrm"].append(d - c)
        t1 = pc()
        mean = tu.tree_inverse_weight(s, W)
        t2 = pc()
        torch.cuda.synchronize()
        t3 = pc()
        if r >= 5:
            parts["loop"].append(t1 - t0), parts["final_call"].append(t2 - t1), parts["wait"].append(t3 - t2)
            parts["round"].append(t3 - t0)
    res["with_norms" if with_norms else "without_norms"] = {k: round(float(np.median(v)) * 1e6, 2)
                                                            for k, v in parts.items()}
print(json.dumps(res))
