"""Round-1 probe 2: interleaved NT A/B, simulated 8-way shard compute, configs[4]
per-GPU bf16 shard. Prints JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import distributed as fd, kernels

dev = torch.device("cuda:0")


def ev_time(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def ab_nt(K, P, rounds=5, reps=10):
    x = torch.empty(K, P, device=dev)
    kernels.fill_synth(x, seed=0)
    w = torch.rand(K, device=dev)
    out = torch.empty(P, device=dev)
    res = {}
    for _ in range(rounds):
        for v in (0, 1, 2):
            for nt in (False, True):
                t = ev_time(lambda: kernels.weighted_sum_dense(x, w, scale=0.5, out=out, nontemporal=nt, variant=v), reps)
                res.setdefault(f"v{v}_nt{int(nt)}", []).append(K * P * 4 / t / 1e9)
    print(json.dumps({"probe": "nt_ab", "K": K, "P": P,
                      "GBs_median": {k: round(float(np.median(v)), 1) for k, v in res.items()},
                      "GBs_min": {k: round(float(np.min(v)), 1) for k, v in res.items()}}), flush=True)
    del x


def shard8(K=128, P=4 * 1024 * 1024, buckets=4, reps=20):
    """One rank of the 8-way strong-scaling run: its fold of 4 buckets, no collective."""
    x = torch.empty(K, P, device=dev)
    kernels.fill_synth(x, seed=0)
    w = torch.rand(K, device=dev)
    out = torch.empty(P, device=dev)
    res = {}
    for nb in (1, 2, 4, 8):
        for nt in (False, True):
            def f():
                for p0, p1 in fd.bucket_edges(P, nb):
                    kernels.weighted_sum_dense(x[:, p0:p1], w, scale=0.5, out=out[p0:p1], nontemporal=nt)
            t = ev_time(f, reps)
            res[f"b{nb}_nt{int(nt)}"] = {"ms": round(t * 1e3, 4), "GBs": round(K * P * 4 / t / 1e9, 1)}
    print(json.dumps({"probe": "shard8_rank_compute", "K": K, "P": P, "res": res}), flush=True)
    del x


def c5_shard(K=1024, P=125_000_000, reps=3):
    free, total = torch.cuda.mem_get_info()
    need = K * P * 2 + P * 4
    if need > free - (4 << 30):
        print(json.dumps({"probe": "c5_shard", "skipped": f"need {need/2**30:.1f} GiB, free {free/2**30:.1f}"}))
        return
    x = torch.empty(K, P, dtype=torch.bfloat16, device=dev)
    t0 = time.perf_counter()
    kernels.fill_synth(x, seed=0)
    torch.cuda.synchronize()
    fill_s = time.perf_counter() - t0
    w = torch.rand(K, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    res = {}
    for nt in (True, False):
        t = ev_time(lambda: kernels.weighted_sum_dense(x, w, scale=0.5, out=out, nontemporal=nt), reps)
        res[f"nt{int(nt)}"] = {"ms": round(t * 1e3, 3), "GBs": round(K * P * 2 / t / 1e9, 1)}
    print(json.dumps({"probe": "c5_shard", "K": K, "P": P, "dtype": "bf16->f32 partial",
                      "bytes": K * P * 2, "fill_s": round(fill_s, 2), "res": res}), flush=True)
    del x


if __name__ == "__main__":
    ab_nt(128, 1206590)
    ab_nt(1024, 4 * 1024 * 1024, rounds=3, reps=5)
    shard8()
    c5_shard()
