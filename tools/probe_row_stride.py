"""Does the pytree fold's speed depend on the byte stride between clients' rows? 128
clients' linear/w leaves (1,179,648 f32 each) carved from one buffer at several row
strides, folded by tree_mean; GPU ms per call (events around 50 back-to-back calls).
4,826,368 B is the slab's row stride (views), 4,718,592 B = 9 x 512 KiB is what the
caching allocator gives back-to-back 4.5 MiB allocations."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd  # noqa: F401
from fedjax_amd import tree_util as tu

N, K = 1179648, 128
dev = torch.device("cuda:0")
weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
res = {}
for stride in (4826368, 4718592, 4718592 + 4096, 4718592 + 65536, 4 << 20 << 1, 5 << 20):
    buf = torch.empty(K * stride // 4 + N, device=dev)
    buf.normal_()
    clients = [{"w": buf[k * stride // 4:k * stride // 4 + N]} for k in range(K)]
    pairs = list(zip(clients, weights))
    for _ in range(5):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        tu.tree_mean(pairs)
    e.record()
    e.synchronize()
    res[str(stride)] = round(s.elapsed_time(e) / 50 * 1e3, 1)
    del buf, clients, pairs
print(json.dumps({"probe": "row stride vs k_ptrs time (us per call, linear/w x 128 clients)", "us": res}))
