"""Host profile of the per-client tree ops of fedjax/algorithms/fed_avg.py:137-139
(tree_add(s, tree_weight(delta, n))) on configs[1] pytrees: wall per client and the
cProfile top entries."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


dev = torch.device("cuda:0")
clients = [tmap(lambda s: torch.randn(s, device=dev), SHAPES) for _ in range(16)]
s = tu.tree_zeros_like(clients[0])


def loop(n):
    global s
    for i in range(n):
        s = tu.tree_add(s, tu.tree_weight(clients[i % 16], 3))


loop(50)
torch.cuda.synchronize()
t0 = time.perf_counter()
loop(500)
torch.cuda.synchronize()
print(f"per client (tree_weight + tree_add): {(time.perf_counter() - t0) / 500 * 1e6:.1f} us")
pr = cProfile.Profile()
pr.enable()
loop(500)
pr.disable()
out = io.StringIO()
pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(25)
print(out.getvalue())
