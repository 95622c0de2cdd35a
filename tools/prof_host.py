"""Host-side cost of tree_mean at configs[1] (128 clients x 8 EMNIST-CNN leaves):
cProfile of 300 calls, top entries by own time. The kernel takes ~95 us per call, so
everything above that in wall time is host work.

usage (GPU box): python tools/prof_host.py
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fedjax_amd  # noqa: E402
from fedjax_amd import tree_util as tu  # noqa: E402

EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main():
    dev = torch.device("cuda:0")
    K = 128
    template = tmap(lambda s: np.zeros(s, np.float32), EMNIST)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
    w = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    pairs = list(zip(clients, w))
    for _ in range(20):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(300):
        tu.tree_mean(pairs)
    issue = (time.perf_counter() - t0) / 300
    torch.cuda.synchronize()
    print(f"host issue per call: {issue * 1e6:.1f} us")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        tu.tree_mean(pairs)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
