"""Five tree_mean calls on configs[1] client pytrees (128 x EMNIST-CNN, one allocation per
(client, leaf)) for rocprofv3 --pmc: the k_ptrs launches' HBM traffic (tools/pmc_summary.py)."""
import os
import sys

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
K = 128
slab = fedjax_amd.ClientDeltaSlab(tmap(lambda s: np.zeros(s, np.float32), SHAPES), K, device=dev).fill_synthetic(seed=0)
clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
del slab
weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
for _ in range(5):
    tu.tree_mean(zip(clients, weights))
torch.cuda.synchronize()
print("ok")
