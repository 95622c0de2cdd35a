"""Counter study of the configs[1] pytree fold (k_ptrs) by leaf placement (VERDICT r1
next #5): the same 128 x EMNIST-CNN deltas folded by tree_mean with the clients' leaves

  views   - views into one padded slab allocation (the fast case, ~88 us);
  clones  - one allocation per (client, leaf), as a reference caller holds them (~94 us);
  rows2m  - one allocation, every client's leaves packed at its own 2 MiB-aligned offset
            (the clones' alignment inside a single allocation);
  bigseg  - one allocation per client, each made 32 MiB (above the caching allocator's
            20 MiB segments, so each is its own hipMalloc);
  expseg  - one allocation per (client, leaf) like clones, under torch's expandable-segments
            allocator (PYTORCH_HIP_ALLOC_CONF=expandable_segments:True, set before torch loads):
            the caller's allocation pattern unchanged, the leaves mapped into one growing
            virtual range. This torch build refuses it on ROCm (a warning; the run is then
            the clones case, profiles/r02s_placement/).

usage: python tools/probe_ptrs_pmc.py MODE [calls]   (run under rocprofv3 --kernel-trace or
--pmc; every k_ptrs dispatch of the run is of MODE's placement)
"""
import os
import sys

if len(sys.argv) > 1 and sys.argv[1] == "expseg":
    os.environ["PYTORCH_HIP_ALLOC_CONF"] = "expandable_segments:True"
    os.environ["PYTORCH_CUDA_ALLOC_CONF"] = "expandable_segments:True"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def packed_into(buf, base, tree):
    """tree's leaves copied into buf[base:], each leaf 16-byte aligned."""
    off = [base]

    def place(x):
        v = buf[off[0]:off[0] + x.numel()].view(x.shape)
        v.copy_(x)
        off[0] += (x.numel() + 3) // 4 * 4
        return v
    return tmap(place, tree)


def main(mode, calls=20, K=128):
    dev = torch.device("cuda:0")
    template = tmap(lambda s: np.zeros(s, np.float32), SHAPES)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    P = slab.num_params
    per = (P + 4 * 8 + 3) // 4 * 4
    if mode == "views":
        clients = [slab.client(k) for k in range(K)]
    elif mode in ("clones", "expseg"):
        clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
    elif mode == "rows2m":
        stride = -(-per * 4 // (2 << 20)) * (2 << 20) // 4
        buf = torch.empty(K * stride, device=dev)
        clients = [packed_into(buf, k * stride, slab.client(k)) for k in range(K)]
    elif mode == "bigseg":
        bufs = [torch.empty((32 << 20) // 4, device=dev) for _ in range(K)]
        clients = [packed_into(bufs[k], 0, slab.client(k)) for k in range(K)]
    else:
        raise SystemExit(f"unknown mode {mode}")
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    pairs = list(zip(clients, weights))
    torch.cuda.synchronize()
    for _ in range(calls):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    print(f"{mode}: {calls} tree_mean calls", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
