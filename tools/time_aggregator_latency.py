"""Synchronous and back-to-back latency of mean_aggregator().apply at configs[1] (128 clients x
EMNIST-CNN, separate allocations), with the native whole-call path off / on (interleaved)."""
import os, sys, json, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import fedjax_amd
from fedjax_amd import tree_util as tu
SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
def tmap(f, t): return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)
dev = torch.device("cuda:0"); g = torch.Generator(device=dev).manual_seed(0)
K = 128
triples = [(f"c{k}", tmap(lambda s: torch.rand(s, device=dev, generator=g), SHAPES), int(w))
           for k, w in enumerate(np.random.RandomState(1).randint(1, 501, size=K))]
agg = fedjax_amd.aggregators.mean_aggregator(); st = agg.init()
for native in (False, True, False, True):
    tu._NATIVE_MEAN = native
    tu._mean_config()  # (the builtin tree_mean keeps its own copy)
    for _ in range(5): agg.apply(triples, st)
    ts = []
    for _ in range(100):
        torch.cuda.synchronize(); t0 = time.perf_counter(); agg.apply(triples, st); torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(100): agg.apply(triples, st)
    torch.cuda.synchronize(); b2b = (time.perf_counter() - t0) / 100 * 1e6
    print(json.dumps({"native": native, "mean_aggregator_apply_sync_us": round(float(np.median(ts)), 1), "back_to_back_us": round(b2b, 1)}), flush=True)
