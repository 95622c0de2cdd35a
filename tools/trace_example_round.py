"""One mode of tools/time_example_round.py's configs[1] round, repeated, for a kernel trace:
``norms`` (examples/fed_avg.py:79-81's per-client tree_l2_norm, then tree_mean) or
``mean_only``. Rounds are separated by a synchronize and a 200 us host sleep, so a trace
splits them at the gaps; --summarize turns a rocprofv3 kernel_trace.csv into per-round GPU
spans (first kernel start to last kernel end), kernel counts and per-kernel durations.

usage: python tools/trace_example_round.py --mode norms --rounds 30
       python tools/trace_example_round.py --summarize DIR/..._kernel_trace.csv
"""
import argparse
import csv
import json
import os
import sys
import time


def summarize(path):
    import numpy as np
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rounds, cur = [], []
    for s, e, n in rows:
        if cur and s - cur[-1][1] > 100_000:  # a gap of > 100 us: the next round
            rounds.append(cur)
            cur = []
        cur.append((s, e, n))
    if cur:
        rounds.append(cur)
    rounds = [r for r in rounds if any("k_ptrs" in n or "k_dense" in n for _, _, n in r)][5:]
    span = [(r[-1][1] - r[0][0]) / 1e3 for r in rounds]
    busy = [sum(e - s for s, e, _ in r) / 1e3 for r in rounds]
    per = {}
    for r in rounds:
        for i, (s, e, n) in enumerate(r):  # (keyed by position in the round: chunk 1, chunk 2, ...)
            name = n.replace("(anonymous namespace)::", "")
            name = name[5:] if name.startswith("void ") else name
            per.setdefault(f"{i}: " + name.split("(")[0][:110], []).append((e - s) / 1e3)
    out = {"rounds": len(rounds), "span_us_median": round(float(np.median(span)), 2),
           "busy_us_median": round(float(np.median(busy)), 2),
           "kernels_per_round": round(sum(len(r) for r in rounds) / max(1, len(rounds)), 2),
           "kernels": {k: {"n_per_round": round(len(v) / max(1, len(rounds)), 2),
                           "median_us": round(float(np.median(v)), 2)} for k, v in per.items()}}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["norms", "mean_only"], default="norms")
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--clients", type=int, default=128)
    ap.add_argument("--summarize")
    a = ap.parse_args()
    if a.summarize:
        return summarize(a.summarize)
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fedjax_amd import kernels, tree_util as tu
    shapes = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
              "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
    dev = torch.device("cuda:0")

    def tree(k):
        out, seed = {}, 1
        for mod, leaves in shapes.items():
            out[mod] = {}
            for name, shp in leaves.items():
                x = torch.empty(1, int(np.prod(shp)), device=dev)
                kernels.fill_synth(x, seed=seed, k0=k)
                out[mod][name] = x.view(shp)
                seed += 1
        return out

    pairs = [(tree(k), 1 + (k * 37) % 500) for k in range(a.clients)]
    pc = time.perf_counter
    t = []
    for i in range(a.rounds):
        diag = lst = None
        torch.cuda.synchronize()
        time.sleep(2e-4)
        t0 = pc()
        if a.mode == "mean_only":
            tu.tree_mean(pairs)
        else:
            diag, lst = {}, []
            for cid, (d, n) in enumerate(pairs):
                lst.append((d, n))
                diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
            tu.tree_mean(lst)
        torch.cuda.synchronize()
        t.append(pc() - t0)
    print(json.dumps({"mode": a.mode, "round_ms_median": round(float(np.median(t[5:])) * 1e3, 4),
                      "solo_info": tu._HOST.solo_info()}))


if __name__ == "__main__":
    main()
