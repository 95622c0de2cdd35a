"""The early-flush client threshold of the deferred running sum (tree_util._DEFER["flush_clients"],
fjhost flush_due) against the synchronised library-loop round at configs[1] (128 clients x
EMNIST-CNN, fedjax/algorithms/fed_avg.py:132-146 with the per-client tree_l2_norm) and at a
GPU-bound shape (128 clients x 16 MiB f32, one leaf). Thresholds interleaved round by round;
median microseconds per round. One JSON line per shape.
usage: python tools/ab_flush_clients.py [rounds]"""
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
THRESHOLDS = (48, 64, 80, 96, 4095)


def emnist(k, dev):
    out, seed = {}, 1
    for mod, leaves in SHAPES.items():
        out[mod] = {}
        for name, shp in leaves.items():
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=seed, k0=k)
            out[mod][name] = x.view(shp)
            seed += 1
    return out


def big(k, dev):
    x = torch.empty(1, 4 << 20, dtype=torch.float32, device=dev)
    kernels.fill_synth(x, seed=3, k0=k)
    return {"w": x.view(-1)}


def run(make, K, rounds, dev):
    pairs = list(zip([make(k, dev) for k in range(K)], np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    W = float(sum(w for _, w in pairs))
    times = {t: [] for t in THRESHOLDS}
    for r in range(rounds + 3):
        for t in THRESHOLDS:
            tu.set_deferred_sums(True, **dict(tu.DEFERRED_SUM_DEFAULTS, flush_clients=t))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s, diag = tu.tree_zeros_like(pairs[0][0]), {}
            for cid, (d, w) in enumerate(pairs):
                s = tu.tree_add(s, tu.tree_weight(d, w))
                diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
            m = tu.tree_inverse_weight(s, W)
            torch.cuda.synchronize()
            if r >= 3:
                times[t].append((time.perf_counter() - t0) * 1e6)
            del m, diag, s
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    return {str(t): round(float(np.median(v)), 1) for t, v in times.items()}


def main(rounds=30):
    dev = torch.device("cuda:0")
    print(json.dumps({"shape": "configs[1] 128 x EMNIST-CNN", "round_us_by_flush_clients": run(emnist, 128, rounds, dev)}),
          flush=True)
    torch.cuda.empty_cache()
    print(json.dumps({"shape": "128 x 16 MiB", "round_us_by_flush_clients": run(big, 128, rounds, dev)}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
