"""tree_mean over many clients of a small model (a narrow parameter axis through the pytree
kernel): an EMNIST logistic-regression-sized tree {w: (784, 62), b: (62,)} (48,670 params)
and a 2-layer MLP {l1/w: (784, 128), l1/b, l2/w: (128, 62), l2/b} (108,606 params), each
(client, leaf) its own allocation. Prints one JSON line per shape: GPU ms per call (events
around back-to-back calls), GB/s of client deltas, and the median wall time of one
synchronous call on an idle GPU. The FJAGG_PIPELINE_* environment selects the host pipeline
(tree_util._tree_mean_pipelined; FJAGG_PIPELINE_FRAC=0: off)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import tree_util as tu

MODELS = {
    "logreg": {"w": (784, 62), "b": (62,)},
    "mlp": {"l1": {"w": (784, 128), "b": (128,)}, "l2": {"w": (128, 62), "b": (62,)}},
}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, shapes in MODELS.items():
        for K in (256, 1024, 4096):
            clients = [tmap(lambda s: torch.rand(s, device=dev, generator=g), shapes) for _ in range(K)]
            P = sum(int(np.prod(s)) for s in [x.shape for x in __import__("fedjax_amd").pytree.leaves_of(clients[0])])
            pairs = list(zip(clients, np.random.RandomState(1).randint(1, 501, size=K).tolist()))
            for _ in range(3):
                tu.tree_mean(pairs)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            s.record()
            for _ in range(reps):
                tu.tree_mean(pairs)
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / reps
            sync = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tu.tree_mean(pairs)
                torch.cuda.synchronize()
                sync.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps({"model": name, "clients": K, "params": P, "ms_per_call": round(ms, 4),
                              "GBs": round(K * P * 4 / ms / 1e6, 1),
                              "sync_call_ms": round(float(np.median(sync)), 4),
                              "pipeline": [tu._PIPELINE_FRAC, tu._PIPELINE_CHUNK]}), flush=True)
            del clients, pairs


if __name__ == "__main__":
    main()
