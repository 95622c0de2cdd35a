"""End-to-end rate with host-resident client deltas: host pytrees or
msgpack payloads -> pinned ring -> slab rows (copy stream) -> fold. Prints JSON."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import ingest

K, P = int(sys.argv[1]) if len(sys.argv) > 1 else 128, int(sys.argv[2]) if len(sys.argv) > 2 else 4 * 1024 * 1024
dev = torch.device("cuda:0")
template = {"w": np.zeros(P, np.float32)}
slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev)
rs = np.random.RandomState(0)
host = [{"w": (rs.standard_normal(P).astype(np.float32) * 0.01)} for _ in range(4)]  # reuse 4 host deltas
payloads = [ingest.msgpack_serialize(h) for h in host]
weights = list(rs.randint(1, 501, size=K))
weights = [int(w) for w in weights]
res = {}
for mode in ("pytree", "msgpack"):
    for depth in (2, 4, 8):
        ing = ingest.DeltaIngestor(slab, depth=depth)
        best = 1e9
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                ing.put(k, host[k % 4] if mode == "pytree" else payloads[k % 4])
            ing.ready()
            m = slab.mean(weights)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        res[f"{mode}_depth{depth}"] = round(K * P * 4 / best / 1e9, 2)
# plain pinned H2D of the whole slab (upper bound)
pinned = torch.empty(K, P, dtype=torch.float32).pin_memory()
torch.cuda.synchronize()
t0 = time.perf_counter()
slab.rows.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
res["pinned_h2d_bound"] = round(K * P * 4 / (time.perf_counter() - t0) / 1e9, 2)
print(json.dumps({"probe": "e2e_ingest", "K": K, "P": P, "GBs": res}))
