"""A/B of the running sum's second early flush (tree_util._flush_due: half the thresholds while
the GPU is idle) on the library loop at configs[1] (fed_avg.py:132-146, 128 clients x
EMNIST-CNN), with and without the per-client tree_l2_norm: synchronised rounds, the four modes
interleaved round by round, median ms per mode. One JSON line.
usage: python tools/ab_idle_flush.py [rounds]"""
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


def main(rounds=40, K=128):
    dev = torch.device("cuda:0")
    pairs = list(zip([tree(k, dev) for k in range(K)], np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    W = float(sum(w for _, w in pairs))
    modes = [(n, i) for n in (True, False) for i in (True, False)]
    times = {m: [] for m in modes}
    for r in range(rounds + 3):
        for norms, idle in modes:
            tu.set_deferred_sums(True, idle_flush=idle)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s, diag = tu.tree_zeros_like(pairs[0][0]), {}
            for cid, (t, w) in enumerate(pairs):
                s = tu.tree_add(s, tu.tree_weight(t, w))
                if norms:
                    diag[cid] = tu.tree_l2_norm(t)
            m = tu.tree_inverse_weight(s, W)
            torch.cuda.synchronize()
            if r >= 3:
                times[(norms, idle)].append((time.perf_counter() - t0) * 1e3)
            del s, m, diag
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    print(json.dumps({f"{'norms' if n else 'plain'}_idle_flush_{'on' if i else 'off'}_ms":
                      round(float(np.median(v)), 4) for (n, i), v in times.items()}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
