"""HBM traffic of one examples/fed_avg.py:72-82 round (configs[1]: 128 EMNIST-CNN deltas,
one allocation per (client, leaf)), for rocprofv3 --pmc passes:

    rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python tools/pmc_example_round.py MODE
    python tools/pmc_example_round.py --summarize FETCH_DIR WRITE_DIR ROUNDS

MODE: norms (the example: per-client tree_l2_norm, then tree_mean; lazy norms), eager (the
same with set_lazy_norms(False): one norm pass per client), mean_only (tree_mean alone).
Each mode runs 2 warm-up rounds, then ROUNDS (default 10) rounds; --summarize sums the
counters of every fold / norm dispatch (fill_synth excluded) over the last ROUNDS rounds and
reports bytes per round against the algorithmic K*P*4 read (gfx950: read = 2 x FETCH_SIZE x
1024, write = WRITE_SIZE x 1024)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
K, P = 128, 1206590


def run(mode, rounds=10):
    import numpy as np
    import torch
    from fedjax_amd import kernels, tree_util as tu
    dev = torch.device("cuda:0")

    def tree(k):
        out, seed = {}, 1
        for mod, leaves in SHAPES.items():
            out[mod] = {}
            for name, shp in leaves.items():
                x = torch.empty(1, int(np.prod(shp)), device=dev)
                kernels.fill_synth(x, seed=seed, k0=k)
                out[mod][name] = x.view(shp)
                seed += 1
        return out
    pairs = [(tree(k), 1 + k % 50) for k in range(K)]
    tu.set_lazy_norms(mode != "eager")
    for _ in range(2 + rounds):
        torch.cuda.synchronize()
        if mode == "mean_only":
            tu.tree_mean(pairs)
        else:
            diag, lst = {}, []
            for cid, (d, n) in enumerate(pairs):
                lst.append((d, n))
                diag[cid] = {"delta_l2_norm": tu.tree_l2_norm(d)}
            tu.tree_mean(lst)
            float(diag[0]["delta_l2_norm"])
    torch.cuda.synchronize()


def summarize(fdir, wdir, rounds):
    """Counters of the fold / norm kernels (k_ptrs*, k_leaves* — fjtree, k_l2_combine) summed over all 2 + ROUNDS rounds
    (the warm-up rounds are the same work) and divided by their number."""
    def total(d, counter):
        agg, names = {}, {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r.get("Kernel_Name", "")
                    if r.get("Counter_Name") == counter and ("k_ptrs" in name or "k_leaves" in name or "k_l2" in name):
                        did = int(r["Dispatch_Id"])
                        agg[did] = agg.get(did, 0.0) + float(r["Counter_Value"])
                        names[did] = name.replace("void ", "").split("<")[0]
        return sum(agg.values()), len(agg), sorted(set(names.values()))
    f, nf, kn = total(fdir, "FETCH_SIZE")
    w, _, _ = total(wdir, "WRITE_SIZE")
    n = rounds + 2
    alg = K * P * 4
    res = {"rounds": n, "dispatches_per_round": nf / n, "kernels": kn,
           "read_bytes_per_round": 2 * f * 1024 / n, "write_bytes_per_round": w * 1024 / n,
           "algorithmic_read_bytes": alg, "read_over_algorithmic": round(2 * f * 1024 / n / alg, 4),
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024"}
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "--summarize":
        summarize(sys.argv[2], sys.argv[3], int(sys.argv[4]))
    else:
        run(sys.argv[1])
