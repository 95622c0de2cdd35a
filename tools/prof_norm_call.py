"""Host cost of the per-client tree_l2_norm in the library loop (fedjax/algorithms/fed_avg.py:
137-144) at configs[1], split into its parts: the loop with and without the norm call, and the
pieces the native fast path does per call (the structure walk against the capture, the 0-d view
TensorImpl, wrapping it as the _NormView subclass, the _ticket attribute), and the fold phases of
each round's final call (fjhost.host_timers: checks, outputs, plan, image, launch, ...). Host time only:
microseconds per client, median of `reps` rounds of 128 clients. One JSON line.
usage: python tools/prof_norm_call.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import kernels, tree_util as tu

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


def main(reps=40, K=128):
    dev = torch.device("cuda:0")
    pairs = list(zip([tree(k, dev) for k in range(K)], np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    W = float(sum(w for _, w in pairs))
    pc = time.perf_counter
    host = tu._HOST
    buf = torch.empty((2, 257), dtype=torch.float32, device=dev)
    res = {}

    phases = {}
    timers = {}  # norm -> fjhost.host_timers() of each round's final call (fold_chain's phases)

    def loop(norm):
        torch.cuda.synchronize()
        tz = pc()
        s, norms = tu.tree_zeros_like(pairs[0][0]), []
        t0 = pc()
        for t, w in pairs:
            s = tu.tree_add(s, tu.tree_weight(t, w))
            if norm:
                norms.append(tu.tree_l2_norm(t))
        t1 = pc()
        host.host_timers()  # reset: the final call's fold phases only
        m = tu.tree_inverse_weight(s, W)
        t2 = pc()
        timers.setdefault(norm, []).append(host.host_timers())
        torch.cuda.synchronize()
        t3 = pc()
        key = "norms" if norm else "plain"
        phases.setdefault(key, []).append((t0 - tz, t1 - t0, t2 - t1, t3 - t2, t3 - tz,
                                           host.pool_info()[2] if norm else 0.0))
        del m, norms
        return (t1 - t0) / K * 1e6

    parts = {
        "loop_plain": lambda: loop(False),
        "loop_norms": lambda: loop(True),
    }

    def per_call(fn):
        t0 = pc()
        for i in range(K):
            fn(i)
        return (pc() - t0) / K * 1e6

    cap_t = pairs[0][0]
    parts["norm_view_subclass"] = lambda: per_call(lambda i: host.norm_view(buf, 1, i, tu._NormView))
    parts["norm_view_tensor"] = lambda: per_call(lambda i: host.norm_view(buf, 1, i, torch.Tensor))

    def view_and_ticket(i):
        v = host.norm_view(buf, 1, i, tu._NormView)
        v._ticket = None

    parts["norm_view_subclass_setattr"] = lambda: per_call(view_and_ticket)
    parts["tree_weight_only"] = lambda: per_call(lambda i: tu.tree_weight(cap_t, 3))
    for name, fn in parts.items():
        for _ in range(3):
            fn()
        vals = [fn() for _ in range(reps)]
        res[name + "_us_per_client"] = round(float(np.median(vals)), 3)
    res["norm_call_us_per_client"] = round(res["loop_norms_us_per_client"] - res["loop_plain_us_per_client"], 3)
    for key, rows in phases.items():  # median host microseconds of each phase of a synchronised round
        a = np.median(np.array(rows[3:]), axis=0) * 1e6
        res[f"round_{key}_us"] = {"zeros": round(a[0], 1), "loop": round(a[1], 1), "final_call": round(a[2], 1),
                                  "sync_wait": round(a[3], 1), "total": round(a[4], 1),
                                  "pool_refill_in_final_call": round(a[5] / 1e6, 1)}
    for norm, rows in timers.items():
        keys = [k for k in rows[0] if k != "calls"]
        res[f"final_call_fold_phases_{'norms' if norm else 'plain'}_us"] = {
            k: round(float(np.median([r[k] for r in rows[3:]])), 2) for k in keys}
    info = host.pool_info()
    res["pool"] = {"refills_reusing_a_pool": info[4], "refills_building_one": info[5], "retired": info[3]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
