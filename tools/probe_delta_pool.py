"""k_ptrs at configs[1] with the clients' leaves allocated three ways:

  clones - one torch allocation per (client, leaf), default caching allocator (what callers hold)
  pool   - the same allocations made under fedjax_amd.memory.delta_allocation() (fjalloc:
           segments mapped into one reserved virtual range per device)
  views  - views into one padded slab (the placement the fold is fastest on)

Prints one JSON line per mode: tree_mean calls back to back (kernel-bound), ms per call, and
the bits of the mean (equal across modes). Run it under rocprofv3 --kernel-trace / --pmc to
get the k_ptrs durations and translation counters per mode.
usage: python tools/probe_delta_pool.py [modes,comma,separated] [calls]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import memory, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main(modes, calls=50, K=128):
    dev = torch.device("cuda:0")
    if os.environ.get("FJALLOC_STAGGER_KIB") is not None:  # A/B of the segment stagger (fjalloc_configure)
        from fedjax_amd import _lib
        assert _lib.load().fjalloc_configure(1 << 30, 64 << 10, 2, int(os.environ["FJALLOC_STAGGER_KIB"]) << 10) == 0
    template = tmap(lambda s: np.zeros(s, np.float32), SHAPES)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    ref_bits = None
    for mode in modes:
        if mode == "views":
            clients = [slab.client(k) for k in range(K)]
        elif mode == "clones":
            clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
        elif mode == "pool":
            with memory.delta_allocation(dev):
                clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
        else:
            raise SystemExit(f"unknown mode {mode}")
        pairs = list(zip(clients, weights))
        for _ in range(5):
            m = tu.tree_mean(pairs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            m = tu.tree_mean(pairs)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / calls * 1e3
        bits = np.concatenate([x.reshape(-1).cpu().numpy().view(np.uint32) for x in tu.pytree.leaves_of(m)])
        same = True if ref_bits is None else bool(np.array_equal(bits, ref_bits))
        ref_bits = bits if ref_bits is None else ref_bits
        ptrs = sorted(x.data_ptr() for t in clients for x in tu.pytree.leaves_of(t))
        rec = {"mode": mode, "calls": calls, "ms_per_call": round(ms, 4), "same_bits_as_first_mode": same,
               "leaf_address_span_MiB": round((ptrs[-1] - ptrs[0]) / 2**20, 1)}
        if mode == "pool":
            rec["fjalloc"] = memory.stats(dev)
        print(json.dumps(rec), flush=True)
        del clients, pairs, m
        torch.cuda.synchronize()


if __name__ == "__main__":
    main(sys.argv[1].split(",") if len(sys.argv) > 1 else ["clones", "pool", "views"],
         int(sys.argv[2]) if len(sys.argv) > 2 else 50)
