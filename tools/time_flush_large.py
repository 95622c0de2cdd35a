"""The library running-sum loop (fedjax/algorithms/fed_avg.py:132-146) on a model where the
GPU, not the host, bounds the round: configs[2]'s shape, 1024 clients x one 4 Mi float32
leaf (16 MiB per client, separate allocations). An early flush of the deferred sum reads and
writes the running base once more (2 x 16 MiB per flush), so its cost here is HBM traffic, not
host time; this sweeps set_deferred_sums(flush_bytes=, flush_clients=) against that.

Prints one JSON line: per setting [synchronised round ms, rounds back to back ms], twice
(interleaved). usage: python tools/time_flush_large.py [rounds] [clients]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import kernels, tree_util as tu

SETTINGS = ((1 << 30, 16), (256 << 20, 16), (256 << 20, 48), (256 << 20, 64), (1 << 62, 1 << 30))


def main(rounds=10, K=1024, P=1 << 22):
    dev = torch.device("cuda:0")
    trees = []
    for k in range(K):
        x = torch.empty(1, P, dtype=torch.float32, device=dev)
        kernels.fill_synth(x, seed=1, k0=k)
        trees.append({"w": x.view(P)})
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    W = float(sum(weights))
    pc = time.perf_counter

    def one_round():
        s = tu.tree_zeros_like(trees[0])
        for t, w in zip(trees, weights):
            s = tu.tree_add(s, tu.tree_weight(t, w))
        return tu.tree_inverse_weight(s, W)

    res = {"workload": f"{K} clients x {P} f32 (one leaf, separate allocations)", "bytes_per_round": K * P * 4}
    ref = None
    out = {}
    for rep in range(2):
        for fb, fc in SETTINGS:
            tu.set_deferred_sums(True, flush_bytes=fb, flush_clients=fc)
            m = one_round()
            bits = m["w"][:: 4099].cpu().numpy().view(np.uint32)
            ref = bits if ref is None else ref
            assert np.array_equal(bits, ref), "early flush changed the bits"
            walls = []
            for _ in range(rounds):
                torch.cuda.synchronize()
                t0 = pc()
                m = one_round()
                torch.cuda.synchronize()
                walls.append((pc() - t0) * 1e3)
            t0 = pc()
            for _ in range(rounds):
                m = one_round()
            torch.cuda.synchronize()
            b2b = (pc() - t0) / rounds * 1e3
            name = "never" if fb >= 1 << 60 else f"{fb >> 20}MiB/{fc}"
            out.setdefault(name, []).append([round(float(np.median(walls)), 3), round(b2b, 3)])
            del m
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    res["flush_sweep_ms"] = out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
