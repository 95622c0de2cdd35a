"""Is the configs[1] pytree fold slower than the slab fold because of the kernel or
because of where the leaves live? Folds the same 128 x EMNIST-CNN deltas through
tree_mean with three placements, then as the dense slab:

  views  - every client leaf is a view into the one padded slab allocation;
  clones - one allocation per (client, leaf), as a reference caller holds them;
  packed - one contiguous allocation per client, leaves as views into it
           (what the msgpack decoder / DeltaIngestor produce).

Prints one JSON line with the per-call GPU time (events around 50 back-to-back
calls; tree_mean's host issue is shorter than the kernel, so the GPU stays busy).
Run under rocprofv3 --kernel-trace for the exact k_ptrs durations: each mode
issues WARM + REPS calls in the order above.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import kernels, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
WARM, REPS = 5, 50


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def packed_copy(tree, dev):
    leaves = []
    tmap(leaves.append, tree)
    buf = torch.empty(sum(x.numel() for x in leaves) + 4 * len(leaves), device=dev)
    it = iter(range(len(leaves)))
    offs = [0]
    for x in leaves:  # keep every leaf 16-byte aligned
        offs.append(offs[-1] + (x.numel() + 3) // 4 * 4)

    def place(x):
        i = next(it)
        v = buf[offs[i]:offs[i] + x.numel()].view(x.shape)
        v.copy_(x)
        return v
    return tmap(place, tree)


def gpu_ms(fn):
    for _ in range(WARM):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / REPS


def main(K=128):
    dev = torch.device("cuda:0")
    template = tmap(lambda s: np.zeros(s, np.float32), SHAPES)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    P = slab.num_params
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    placements = {
        "views": [slab.client(k) for k in range(K)],
        "clones": [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)],
        "packed": [packed_copy(slab.client(k), dev) for k in range(K)],
    }
    # is the gap in the big leaf or in the seven small ones? clones of linear/w alone vs its views
    big = {"views_linear_w_only": [{"w": c["linear"]["w"]} for c in placements["views"]],
           "clones_linear_w_only": [{"w": c["linear"]["w"]} for c in placements["clones"]]}
    res = {"workload": "configs[1] 128 x EMNIST-CNN, 8 leaves", "bytes": K * P * 4}
    for name, clients in big.items():
        pairs = list(zip(clients, weights))
        res[name] = {"ms": round(gpu_ms(lambda: tu.tree_mean(pairs)), 4)}
    ref = None
    for name, clients in placements.items():
        pairs = list(zip(clients, weights))
        ms = gpu_ms(lambda: tu.tree_mean(pairs))
        out = tu.tree_mean(pairs)
        flat = torch.cat([x.reshape(-1) for x in [out[a][b] for a in sorted(out) for b in sorted(out[a])]])
        if ref is None:
            ref = flat
        res[name] = {"ms": round(ms, 4), "GBs": round(K * P * 4 / ms / 1e6, 1),
                     "bitwise_equal_to_views": bool(torch.equal(flat, ref))}
    wd = slab.weight_vector(weights)
    r = float(np.float32(1.0 / sum(weights)))
    o = torch.empty(P, device=dev)
    ms = gpu_ms(lambda: kernels.weighted_sum_dense(slab.rows, wd, scale=r, out=o, nontemporal=True))
    res["slab"] = {"ms": round(ms, 4), "GBs": round(K * P * 4 / ms / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
