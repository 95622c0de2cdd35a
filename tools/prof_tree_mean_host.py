"""Host-side phases of one tree_mean call at configs[1] (128 clients x EMNIST-CNN, one
allocation per client leaf): pair collection + weight packing, client table (flatten of
client 0 + native gather of the K x L pointers), native fold (outputs, plan image, upload,
launch), unflatten. Median microseconds over many calls; the GPU runs behind (no sync
inside the timed phases). Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import pytree, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main(K=128, reps=200, sync=False):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    clients = [tmap(lambda s: torch.rand(s, device=dev, generator=g), SHAPES) for _ in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    pairs = list(zip(clients, weights))
    ph = {"collect_pairs": [], "client_table": [], "fold": [], "unflatten": [], "total": []}
    pc = time.perf_counter
    for i in range(reps + 20):
        t0 = pc()
        trees, w, W = tu._collect_pairs(pairs)
        t1 = pc()
        td, rows = tu._client_table(trees)
        t2 = pc()
        outs = tu._fold(rows, w, scale=tu._inverse(W), validated=True)
        t3 = pc()
        pytree.unflatten(td, outs)
        t4 = pc()
        tu.tree_mean(pairs)
        t5 = pc()
        if i >= 20:
            for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
                ph[k].append(v * 1e6)
        if sync or i % 50 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    from fedjax_amd import _lib
    _lib.host().host_timers()  # reset: the phases below are of the timed calls only
    for i in range(reps):
        td, rows = tu._client_table(trees)
        if sync:
            torch.cuda.synchronize()
        tu._fold(rows, w, scale=tu._inverse(W), validated=True)
    torch.cuda.synchronize()
    inner = {k: round(v, 2) for k, v in _lib.host().host_timers().items()}
    print(json.dumps({"workload": f"configs[1] tree_mean host phases (us, median), K={K}, sync={sync}",
                      **{k: round(float(np.median(v)), 2) for k, v in ph.items()},
                      "fold_table_phases_us_mean": inner}), flush=True)


if __name__ == "__main__":  # argv: K, then "sync" (idle GPU before every call)
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 128, sync="sync" in sys.argv[2:])
