"""Host cost of the pieces of tree_weight's native capture at configs[1] (one EMNIST-CNN client
pytree, 8 leaves in 5 dicts): fjhost.capture (walk + leaf checks + structure token + the
capture tuple), tree_weight (capture + the WeightedTree object), fjhost.matches (walk + leaf
identity + versions), tree_add of a tree_weight into a live chain, and an empty FASTCALL for
scale. Microseconds per call, median of `reps` batches of 1,000 calls. One JSON line.
usage: python tools/prof_capture.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import kernels, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def main(reps=15, n=1000):
    dev = torch.device("cuda:0")
    t = {m: {k: torch.zeros(int(np.prod(s)), device=dev).view(s) for k, s in lv.items()} for m, lv in SHAPES.items()}
    H = tu._HOST
    cap = H.capture(t, -1)
    pc = time.perf_counter

    def per_call(fn):
        vals = []
        for _ in range(reps):
            t0 = pc()
            for _ in range(n):
                fn()
            vals.append((pc() - t0) / n * 1e6)
        return round(float(np.median(vals)), 3)

    res = {"empty_builtin_len": per_call(lambda: len(t)),
           "capture": per_call(lambda: H.capture(t, -1)),
           "tree_weight": per_call(lambda: tu.tree_weight(t, 3)),
           "matches": per_call(lambda: H.matches(t, cap[0], cap[1]))}
    wt = tu.tree_weight(t, 3)
    tu.set_deferred_sums(True, max_clients=4095, flush_bytes=1 << 40)

    def adds():
        s = tu.tree_zeros_like(t)
        t0 = pc()
        for _ in range(200):
            s = tu.tree_add(s, wt)
        dt = (pc() - t0) / 200 * 1e6
        del s
        return dt
    res["tree_add_append"] = round(float(np.median([adds() for _ in range(reps)])), 3)
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 15)
