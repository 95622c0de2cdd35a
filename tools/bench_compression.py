"""Time the compression aggregators' rounds on the GPU.

One "round" = ``aggregator.apply`` over K device-resident client deltas with the
EMNIST-CNN tree (configs[1]: 128 clients x 1,206,590 float32 params), timed with
HIP events on the launch stream around the whole apply (host table building, key
schedule and every launch included), after warmup. Prints one JSON line per
aggregator with the round time and the delta bytes consumed per second.

usage: python tools/bench_compression.py [--clients 128] [--rounds 10] [--only uniform,terngrad,...]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import fedjax_amd
from fedjax_amd import random
from fedjax_amd.aggregators import compression as comp

EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--only", default="uniform,uniform_arith,terngrad,rotated,drive")
    ap.add_argument("--cpu-sample", type=int, default=2, help="clients in the numpy-oracle CPU sample (0: skip)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    K = args.clients
    template = tmap(lambda s: np.zeros(s, np.float32), EMNIST)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    P = slab.num_params
    w = [int(x) for x in np.random.RandomState(1).randint(1, 500, K)]
    clients = [(b"c%d" % k, slab.client(k), w[k]) for k in range(K)]
    aggs = {
        "uniform": lambda: comp.uniform_stochastic_quantizer(16, random.PRNGKey(0)),
        "uniform_arith": lambda: comp.uniform_stochastic_quantizer(16, random.PRNGKey(0), "arithmetic"),
        "terngrad": lambda: comp.terngrad_quantizer(random.PRNGKey(0)),
        "rotated": lambda: comp.rotated_uniform_stochastic_quantizer(16, random.PRNGKey(0)),
        "drive": lambda: comp.structured_drive_quantizer(random.PRNGKey(0)),
    }
    stream = torch.cuda.current_stream(dev)
    for name in args.only.split(","):
        agg = aggs[name]()
        st = agg.init()
        for _ in range(args.warmup):
            _, st = agg.apply(clients, st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.rounds):
            _, st = agg.apply(clients, st)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.rounds
        ms = e0.elapsed_time(e1) / args.rounds
        rec = {"aggregator": name, "clients": K, "params": P, "rounds": args.rounds, "ms_per_round": round(ms, 4),
               "wall_ms_per_round": round(wall * 1e3, 4), "delta_GBps": round(K * P * 4 / (ms * 1e-3) / 1e9, 1)}
        if args.cpu_sample:
            rec["cpu_baseline"] = cpu_baseline(name, template, args.cpu_sample, K, P)
        print(json.dumps(rec), flush=True)


def cpu_baseline(name, template, k_sample, K, P):
    """The numpy restatement (oracle) on a bounded client sample, scaled to K clients."""
    from oracle import compression_ref as cref
    from oracle import jax_random_ref as jr
    rs = np.random.RandomState(0)
    cl = [("c", tmap(lambda x: (rs.standard_normal(x.shape) * 0.01).astype(np.float32), template), 1 + i)
          for i in range(k_sample)]
    make = {"uniform": lambda: cref.uniform_stochastic_quantizer(16, jr.prng_key(0)),
            "uniform_arith": lambda: cref.uniform_stochastic_quantizer(16, jr.prng_key(0), "arithmetic"),
            "terngrad": lambda: cref.terngrad_quantizer(jr.prng_key(0)),
            "rotated": lambda: cref.rotated_uniform_stochastic_quantizer(16, jr.prng_key(0)),
            "drive": lambda: cref.structured_drive_quantizer(jr.prng_key(0))}[name]
    init, apply = make()
    t0 = time.perf_counter()
    apply(cl, init())
    dt = time.perf_counter() - t0
    per_round = dt * K / k_sample
    return {"kind": "port", "cores": 1, "sample": f"{k_sample} clients, numpy oracle, scaled x{K / k_sample:g}",
            "ms_per_round": round(per_round * 1e3, 1), "delta_GBps": round(K * P * 4 / per_round / 1e9, 3)}


if __name__ == "__main__":
    main()
