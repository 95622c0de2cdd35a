"""Early-flush sweep of the deferred running sum (tree_util.set_deferred_sums flush_bytes /
flush_clients) on the library loop at configs[1] (fedjax/algorithms/fed_avg.py:132-146: 128
EMNIST-CNN deltas, one allocation per (client, leaf)): one synchronous round of
tree_add(s, tree_weight(delta, n)) x K + tree_inverse_weight, with and without the per-client
tree_l2_norm, as bench.py times it. Settings interleave round by round; medians. Every
setting's mean is checked bitwise against the default's. Prints one JSON line.

usage: python tools/ab_flush_small.py [--rounds 40]  (tools/ab_flush_clients.py: the 48-96 sweep, round 4)
"""
import argparse
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
SETTINGS = [(256 << 20, 64), (0, 48), (0, 32), (0, 24), (0, 16), (0, 96)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    a = ap.parse_args()
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

    K = 128
    pairs = [(tree(k), 1 + (k * 37) % 500) for k in range(K)]
    W = float(sum(w for _, w in pairs))
    pc = time.perf_counter
    t = {(s, m): [] for s in SETTINGS for m in (False, True)}
    ref, same = None, {}
    for i in range(a.rounds + 3):
        for s in SETTINGS:
            tu.set_deferred_sums(True, flush_bytes=s[0], flush_clients=s[1])
            for with_norms in (False, True):
                diag = None
                torch.cuda.synchronize()
                t0 = pc()
                acc, diag = tu.tree_zeros_like(pairs[0][0]), {}
                for cid, (d, w) in enumerate(pairs):
                    acc = tu.tree_add(acc, tu.tree_weight(d, w))
                    if with_norms:
                        diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
                mean = tu.tree_inverse_weight(acc, W)
                torch.cuda.synchronize()
                if i >= 3:
                    t[(s, with_norms)].append(pc() - t0)
                if i == 0:
                    bits = torch.cat([x.reshape(-1) for x in pytree.leaves_of(mean)]).view(torch.int32)
                    if ref is None:
                        ref = bits.clone()
                    same[str(s)] = same.get(str(s), True) and bool(torch.equal(bits, ref))
                del acc, mean
    tu.set_deferred_sums(True, flush_bytes=256 << 20, flush_clients=64)
    res = {}
    for s in SETTINGS:
        res[f"flush_bytes={s[0]},flush_clients={s[1]}"] = {
            "without_norms_ms": round(float(np.median(t[(s, False)])) * 1e3, 4),
            "with_norms_ms": round(float(np.median(t[(s, True)])) * 1e3, 4),
            "mean_bits_equal_default": same[str(s)]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
