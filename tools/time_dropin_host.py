"""Host cost of the drop-in calls at configs[1] (128 clients x EMNIST-CNN, one allocation
per (client, leaf)), the numbers behind bench.py's drop_in record, split by phase:

* the library running-sum loop of fedjax/algorithms/fed_avg.py:132-146
  (tree_zeros_like; tree_add(s, tree_weight(delta, n)) x K; tree_inverse_weight):
  per-call host us of tree_weight / tree_add, the zeros and the final fold call, the
  synchronised round and rounds back to back;
* one synchronous tree_mean (examples/fed_avg.py:82) and mean_aggregator().apply
  (aggregator.py:73) on an idle GPU: wall, and the host time until the call returns;
* fjhost.host_timers() phases of the native folds.

Prints one JSON line. usage: python tools/time_dropin_host.py [rounds]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import _lib, kernels, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tree(k, dev):
    out, seed = {}, 1
    for mod, leaves in SHAPES.items():
        out[mod] = {}
        for name, shp in leaves.items():
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=seed, k0=k)
            out[mod][name] = x.view(shp)
            seed += 1
    return out


def med(v):
    return round(float(np.median(v)), 3)


def main(rounds=30, K=128):
    dev = torch.device("cuda:0")
    pairs = list(zip([tree(k, dev) for k in range(K)],
                     np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    W = float(sum(w for _, w in pairs))
    pc = time.perf_counter
    host = _lib.host()
    res = {"workload": f"configs[1]: {K} clients x EMNIST-CNN, separate leaf allocations"}
    # ---- library loop, per call
    tw, ta, tz, tf, wall = [], [], [], [], []
    for r in range(rounds + 5):
        torch.cuda.synchronize()
        t0 = pc()
        s = tu.tree_zeros_like(pairs[0][0])
        t1 = pc()
        a = b = 0.0
        for t, w in pairs:
            u0 = pc()
            x = tu.tree_weight(t, w)
            u1 = pc()
            s = tu.tree_add(s, x)
            u2 = pc()
            a += u1 - u0
            b += u2 - u1
        t2 = pc()
        m = tu.tree_inverse_weight(s, W)
        t3 = pc()
        torch.cuda.synchronize()
        t4 = pc()
        if r >= 5:
            tz.append((t1 - t0) * 1e6)
            tw.append(a / K * 1e6)
            ta.append(b / K * 1e6)
            tf.append((t3 - t2) * 1e6)
            wall.append((t4 - t0) * 1e3)
    del s, m
    # without per-call timers: the round as the bench times it, and back to back
    sync_round = []
    for r in range(rounds + 5):
        torch.cuda.synchronize()
        t0 = pc()
        s = tu.tree_zeros_like(pairs[0][0])
        for t, w in pairs:
            s = tu.tree_add(s, tu.tree_weight(t, w))
        m = tu.tree_inverse_weight(s, W)
        torch.cuda.synchronize()
        if r >= 5:
            sync_round.append((pc() - t0) * 1e3)
    torch.cuda.synchronize()
    t0 = pc()
    for r in range(rounds):
        s = tu.tree_zeros_like(pairs[0][0])
        for t, w in pairs:
            s = tu.tree_add(s, tu.tree_weight(t, w))
        m = tu.tree_inverse_weight(s, W)
    torch.cuda.synchronize()
    b2b = (pc() - t0) / rounds * 1e3
    host.host_timers()
    for r in range(rounds):
        s = tu.tree_zeros_like(pairs[0][0])
        for t, w in pairs:
            s = tu.tree_add(s, tu.tree_weight(t, w))
        m = tu.tree_inverse_weight(s, W)
        torch.cuda.synchronize()
    res["library_loop"] = {"tree_weight_us": med(tw), "tree_add_us": med(ta), "zeros_like_us": med(tz),
                           "fold_call_us": med(tf), "round_sync_ms_timed_calls": med(wall),
                           "round_sync_ms": med(sync_round), "round_back_to_back_ms": round(b2b, 4),
                           "fold_phases_us": {k: round(v, 2) for k, v in host.host_timers().items()}}
    del s, m
    # the loop as fedjax/algorithms/fed_avg.py:132-146 writes it: + tree_l2_norm(delta) per client
    # (the norms read back once after the round, as client_diagnostics are)
    tn, norm_round = [], []
    for r in range(rounds + 5):
        torch.cuda.synchronize()
        t0 = pc()
        s = tu.tree_zeros_like(pairs[0][0])
        norms, c = [], 0.0
        for t, w in pairs:
            s = tu.tree_add(s, tu.tree_weight(t, w))
            u0 = pc()
            norms.append(tu.tree_l2_norm(t))
            c += pc() - u0
        m = tu.tree_inverse_weight(s, W)
        vals = torch.stack(norms).cpu()  # (one read of the round's norms)
        torch.cuda.synchronize()
        if r >= 5:
            norm_round.append((pc() - t0) * 1e3)
            tn.append(c / K * 1e6)
    res["library_loop"]["with_l2_norms"] = {"tree_l2_norm_us": med(tn), "round_sync_ms": med(norm_round)}
    del s, m, norms, vals
    nsweep = {}
    for rep in range(2):
        for fb in (1 << 30, 256 << 20):
            tu.set_deferred_sums(True, flush_bytes=fb)
            walls = []
            for r in range(rounds):
                torch.cuda.synchronize()
                t0 = pc()
                s, norms = tu.tree_zeros_like(pairs[0][0]), []
                for t, w in pairs:
                    s = tu.tree_add(s, tu.tree_weight(t, w))
                    norms.append(tu.tree_l2_norm(t))
                m = tu.tree_inverse_weight(s, W)
                vals = torch.stack(norms).cpu()
                torch.cuda.synchronize()
                walls.append((pc() - t0) * 1e3)
            nsweep.setdefault(f"{fb >> 20}MiB", []).append(med(walls))
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    res["library_loop"]["with_l2_norms"]["flush_sweep_round_sync_ms"] = nsweep
    del s, m, norms, vals
    # ---- synchronous tree_mean / mean_aggregator().apply
    agg = fedjax_amd.aggregators.mean_aggregator()
    triples = [(f"c{k}", t, w) for k, (t, w) in enumerate(pairs)]
    state = agg.init()
    for name, call in (("tree_mean", lambda: tu.tree_mean(pairs)),
                       ("mean_aggregator_apply", lambda: agg.apply(triples, state))):
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        host.host_timers()
        walls, issue = [], []
        for _ in range(5 * rounds):
            torch.cuda.synchronize()
            t0 = pc()
            call()
            t1 = pc()
            torch.cuda.synchronize()
            walls.append((pc() - t0) * 1e3)
            issue.append((t1 - t0) * 1e6)
        res[name] = {"sync_call_ms": med(walls), "host_issue_us": med(issue),
                     "fold_phases_us": {k: round(v, 2) for k, v in host.host_timers().items()}}
        torch.cuda.synchronize()
        t0 = pc()
        for _ in range(5 * rounds):
            call()
        torch.cuda.synchronize()
        res[name]["back_to_back_ms"] = round((pc() - t0) / (5 * rounds) * 1e3, 4)
    # chunk schedules of the synchronous call's pipeline (fjhost.pipeline_fracs)
    sweep = {}
    for rep in range(2):  # the schedules interleaved, twice
        for fr in [(), (0.1,), (0.15,), (0.2,), (0.3,), (0.1, 0.3), (0.15, 0.45)]:
            host.pipeline_fracs(list(fr))
            walls = []
            for _ in range(3 * rounds):
                torch.cuda.synchronize()
                t0 = pc()
                tu.tree_mean(pairs)
                torch.cuda.synchronize()
                walls.append((pc() - t0) * 1e3)
            sweep.setdefault(",".join(map(str, fr)) or "0.25 (frac)", []).append(med(walls))
    host.pipeline_fracs([])
    res["tree_mean_sync_sweep_ms"] = sweep
    # early flushes of the running sum (set_deferred_sums(flush_bytes=, flush_clients=)): the
    # pending part is folded during the loop, so only the last part's fold follows the loop
    flush = {}
    for rep in range(2):
        for fb, fc in ((1 << 30, 16), (128 << 20, 16), (256 << 20, 16), (256 << 20, 48), (256 << 20, 64)):
            tu.set_deferred_sums(True, flush_bytes=fb, flush_clients=fc)
            walls = []
            for _ in range(2 * rounds):
                torch.cuda.synchronize()
                t0 = pc()
                s = tu.tree_zeros_like(pairs[0][0])
                for t, w in pairs:
                    s = tu.tree_add(s, tu.tree_weight(t, w))
                m = tu.tree_inverse_weight(s, W)
                torch.cuda.synchronize()
                walls.append((pc() - t0) * 1e3)
            torch.cuda.synchronize()
            t0 = pc()
            for _ in range(rounds):
                s = tu.tree_zeros_like(pairs[0][0])
                for t, w in pairs:
                    s = tu.tree_add(s, tu.tree_weight(t, w))
                m = tu.tree_inverse_weight(s, W)
            torch.cuda.synchronize()
            b2b = (pc() - t0) / rounds * 1e3
            flush.setdefault(f"{fb >> 20}MiB/{fc}", []).append([med(walls), round(b2b, 4)])
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    res["library_round_flush_sweep_ms"] = flush  # [synchronised round, rounds back to back]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
