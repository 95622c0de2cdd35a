"""Where DeltaIngestor's end-to-end rate goes (128 x 4 Mi f32 host deltas): host time of
the put loop, wall time to ready(), and back-to-back async pinned H2D row copies on one
stream (the DMA bound for the same rows)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import ingest

K, P = 128, 4 * 1024 * 1024
dev = torch.device("cuda:0")
slab = fedjax_amd.ClientDeltaSlab({"w": np.zeros(P, np.float32)}, K, device=dev)
rs = np.random.RandomState(0)
host = [{"w": (rs.standard_normal(P).astype(np.float32) * 0.01)} for _ in range(4)]
res = {}
for depth, th in ((8, 16), (8, 8), (8, 4), (8, 2), (16, 4)):
    torch.set_num_threads(th)
    ing = ingest.DeltaIngestor(slab, depth=depth)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tw = 0.0
        for k in range(K):
            i = ing.n % len(ing.staging)
            if ing.events[i] is not None:
                a = time.perf_counter()
                ing.events[i].synchronize()
                tw += time.perf_counter() - a
            ing.put(k, host[k % 4])
        t1 = time.perf_counter()
        ing.ready()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    res[f"depth{depth}_threads{th}"] = {"host_loop_ms": round((t1 - t0) * 1e3, 2), "waiting_on_dma_ms": round(tw * 1e3, 2),
                            "wall_ms": round((t2 - t0) * 1e3, 2), "GBs": round(K * P * 4 / (t2 - t0) / 1e9, 2)}
pinned = [torch.empty(P * 4, dtype=torch.uint8).pin_memory() for _ in range(4)]
s = torch.cuda.Stream(dev)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for k in range(K):
            slab.storage[k].view(torch.uint8)[: P * 4].copy_(pinned[k % 4], non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
res["async_row_copies_GBs"] = round(K * P * 4 / t / 1e9, 2)
print(json.dumps(res))
