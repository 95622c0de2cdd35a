"""Config 2 (128 clients x EMNIST-CNN, 8 leaves) through the pytree path:
tree_mean wall time (host planning + H2D + launch) and kernel time (HIP events),
plus the same deltas as a dense slab. Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import kernels, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main(K=128, reps=20):
    dev = torch.device("cuda:0")
    template = tmap(lambda s: np.zeros(s, np.float32), SHAPES)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    P = slab.num_params
    # separate allocations per (client, leaf), as a reference caller holds them
    clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    pairs = list(zip(clients, weights))
    for _ in range(3):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    # kernel-only time: events around the launch inside tree_mean
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ks = []
    for _ in range(reps):
        s.record()
        tu.tree_mean(pairs)
        e.record()
        e.synchronize()
        ks.append(s.elapsed_time(e))
    wd = slab.weight_vector(weights)
    r = float(np.float32(1.0 / sum(weights)))
    out = torch.empty(P, device=dev)
    dense = {}
    for nt in (False, True):
        for v in (0, 1, 2, 3):
            kernels.weighted_sum_dense(slab.rows, wd, scale=r, out=out, nontemporal=nt, variant=v)
            s.record()
            for _ in range(reps):
                kernels.weighted_sum_dense(slab.rows, wd, scale=r, out=out, nontemporal=nt, variant=v)
            e.record()
            e.synchronize()
            dense[f"v{v}_nt{int(nt)}"] = round(K * P * 4 / (s.elapsed_time(e) / reps / 1e3) / 1e9, 1)
    # fused per-client l2 norms on the same pytree path (fjagg_wsum_l2_ptrs)
    for _ in range(3):
        tu.tree_mean_with_l2_norms(pairs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tu.tree_mean_with_l2_norms(pairs)
    torch.cuda.synchronize()
    wall_l2 = (time.perf_counter() - t0) / reps
    # tree_mean + server Adam step in one kernel on the same pytrees (fjagg_server_update_ptrs)
    from fedjax_amd import server
    opt = server.adam(10 ** -2.5, b1=0.9, b2=0.999, eps=1e-4)
    params = tmap(lambda v: torch.zeros(v.shape, device=dev), clients[0])
    st = opt.init(params)
    for _ in range(3):
        st = server.fused_tree_mean_update(pairs, opt, params, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        st = server.fused_tree_mean_update(pairs, opt, params, st)
    torch.cuda.synchronize()
    wall_opt = (time.perf_counter() - t0) / reps
    # the reference surface: mean_aggregator().apply over (client_id, delta, weight) triples
    agg = fedjax_amd.aggregators.mean_aggregator()
    state = agg.init()
    triples = [(f"c{k}", c, w) for k, (c, w) in enumerate(pairs)]
    for _ in range(3):
        agg.apply(triples, state)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        agg.apply(triples, state)
    torch.cuda.synchronize()
    wall_apply = (time.perf_counter() - t0) / reps
    # host cost per call: time to issue `reps` calls with the GPU idle at the start
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tu.tree_mean(pairs)
    host = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    nbytes = K * P * 4
    print(json.dumps({"workload": "configs[1] 128 x EMNIST-CNN (1,206,590 params, 8 leaves)",
                      "tree_mean_with_l2_norms_wall_ms": round(wall_l2 * 1e3, 4),
                      "fused_tree_mean_adam_wall_ms": round(wall_opt * 1e3, 4),
                      "tree_mean_wall_ms": round(wall * 1e3, 4),
                      "tree_mean_host_issue_ms": round(host * 1e3, 4),
                      "mean_aggregator_apply_wall_ms": round(wall_apply * 1e3, 4),
                      "tree_mean_wall_GBs": round(nbytes / wall / 1e9, 1),
                      "tree_mean_gpu_ms_median": round(float(np.median(ks)), 4),
                      "tree_mean_gpu_GBs": round(nbytes / (np.median(ks) / 1e3) / 1e9, 1),
                      "dense_slab_GBs": dense}))


def main_c3(K=1024, P=4 * 1024 * 1024, reps=5):
    """configs[2] through tree_mean with every client delta its own allocation."""
    dev = torch.device("cuda:0")
    base = torch.empty(K, P, device=dev)
    kernels.fill_synth(base, seed=0)
    clients = [{"w": base[k]} for k in range(K)]  # separate rows = separate device pointers
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    pairs = list(zip(clients, weights))
    tu.tree_mean(pairs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    print(json.dumps({"workload": "configs[2] via tree_mean, 1024 client tensors x 4 Mi f32",
                      "tree_mean_wall_ms": round(wall * 1e3, 3),
                      "tree_mean_wall_GBs": round(K * P * 4 / wall / 1e9, 1)}))


if __name__ == "__main__":
    main()
    main_c3()
