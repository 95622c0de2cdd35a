"""Benchmark of the aggregation hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2] [--e2e]

``--gpus N`` > 1 works bare (this process spawns N ranks through a
``torch.distributed.run`` child and forwards rank 0's JSON line) or under an
outer ``torch.distributed.run`` (WORLD_SIZE set: this process is one rank).

One step = one weighted mean of the round's client deltas, already resident in
HBM: host W and f32 weights (4 KiB pinned H2D) + the fold kernel, exactly what
``ClientDeltaSlab.mean`` / ``sharded_weighted_mean`` do per round.

* N = 1: BASELINE configs[2], 1024 clients x 4,194,304 fp32 params (17.2 GB) on
  one MI355X — the configuration the north-star target is quoted on.
* N > 1 (torchrun, one rank per GPU): the same 1024 clients sharded N ways
  (configs[3]); each rank folds its 1024/N clients, already scaled by f32(1/W),
  and the partials are summed by a bucketed RCCL reduce to rank 0 that overlaps
  the next bucket's fold. Strong scaling: total work is fixed.

value = K*P*4 bytes of client deltas / wall time of the K timed steps (max over
ranks). roofline.achieved = the same algorithmic bytes per fold launch / the
launch's mean duration from HIP events on the launch stream. cpu_baseline =
the oracle's C restatement of the reference op sequence (oracle/fold_ref.c,
``oracle_tree_mean_refseq_f32``) on a bounded sample, rank 0, N = 1 only.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# N>1 auto-tune: 1 = no overlap; more = shorter exposed reduce tail; tapered relative sizes
# (fd.bucket_edges) hide each reduce behind the next, smaller fold and expose only the last.
# Tapers whose buckets are whole multiples of 1 Mi f32 keep every bucket's fold on a full
# grid (2:1:1 of 4 Mi = 2 Mi + 1 Mi + 1 Mi); 3:1 or 7:1 cut buckets the balanced grid
# covers with part-empty tiles (profiles/r01t_probe_bucket.jsonl, r01t_shard_rehearsal.jsonl)
BUCKET_CANDIDATES = (1, 2, 4, 8, (2, 1, 1), (4, 2, 1, 1))
METRIC = "device-resident aggregated client-delta GB/s, K clients × P fp32 params"
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
WORKLOADS = {  # name: (clients, params, dtype, description)
    "c3": (1024, 4 * 1024 * 1024, torch.float32,
           "configs[2]: mean aggregator, 1024 clients x 4 M-param (4,194,304) fp32 deltas"),
    "c2": (128, 1206590, torch.float32,
           "configs[1]: mean aggregator, 128 clients x 1,206,590-param EMNIST-CNN fp32 deltas"),
    "c5": (8192, 125_000_000, torch.bfloat16,
           "configs[4]: 8192 clients x 125 M-param bf16 deltas, client-sharded (needs >= 8 GPUs)"),
    "c5s": (1024, 125_000_000, torch.bfloat16,
            "configs[4] per-GPU shard: 1024 clients x 125 M-param bf16 deltas on one GPU"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_LAST_PHASE = ["started"]


def phase(rank, name):
    """One stderr line per phase of a rank's run (communicator init, each auto-tune
    candidate, warmup, timed loop, e2e, done), and the rank's current phase in the file a
    spawning parent named in FJ_BENCH_PHASES (spawn_ranks reads them on a timeout to name
    the ranks that had not finished, and where each one stopped)."""
    _LAST_PHASE[0] = name
    log(f"[bench rank {rank}] {name}")
    d = os.environ.get("FJ_BENCH_PHASES")
    if d:
        try:
            with open(os.path.join(d, f"rank{rank}"), "w") as f:
                f.write(name)
        except OSError:
            pass


def fedavg_weights(K, seed=1):
    return np.random.RandomState(seed).randint(1, 501, size=K).tolist()


def _cgroup_cpus():
    """CPUs the cgroup quota grants this process (cpu.max), or None without a quota."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else max(1, int(round(int(quota) / int(period))))
    except (OSError, ValueError):
        return None


def _oracle():
    """The oracle's C restatement (oracle/fold_ref.c through tests/coracle.py). TEST
    INFRASTRUCTURE: loaded only by the cpu_baseline leg (the reported CPU baseline) and by
    check_result (the checker of the timed output, after the timed region); the measured
    path never touches it."""
    from tests import coracle as co

    lib_path = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib_path):
        import __graft_entry__
        __graft_entry__.build()
    return co.load(lib_path)


def check_cols(P, n=2000, edges=(), seed=0):
    """Columns the check compares: n random ones, both ends of the row, and both sides of
    every bucket edge of the exchange (fd.bucket_edges)."""
    rs = np.random.RandomState(seed)
    extra = [0, 1, 2, 3, P - 4, P - 3, P - 2, P - 1]
    for e in edges:
        extra += [e - 1, e, e + 1]
    c = np.concatenate([rs.randint(0, P, n), np.asarray(extra, dtype=np.int64)])
    return np.unique(c[(c >= 0) & (c < P)]).astype(np.int64)


def _bf16_bits(a):
    """float32 -> bfloat16 bits (RNE; finite inputs), as the kernels' f32_to_bf16."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def _ulps(a, b):
    """Distance in float32 ulps (ordered bit patterns)."""
    def ordered(x):
        i = np.ascontiguousarray(x, dtype=np.float32).view(np.int32).astype(np.int64)
        return np.where(i < 0, -(i & 0x7FFFFFFF), i)
    return np.abs(ordered(a) - ordered(b))


def check_result(y, *, K, P, k0, k1, weights, W, dtype, seed=0, exact=True, nranks=1, edges=(),
                 reference_bf16=False, f32_mean=None):
    """Checks the timed run's result against the oracle, after the timed region (VERDICT r4
    next #1): the synthetic deltas are a counter hash of (client, column), so the host
    regenerates exactly the ~2,000 sampled columns it compares (oracle_synth_cols_f32) and
    folds them with the oracle's restatement of tree_util.py:76-96 (oracle_wsum_f32).

    * ``exact``: ``y`` (the mean, or at a rehearsal rank 0's scaled partial over clients
      k0..k1) must be bitwise the oracle's sequential fold — f32 out, bf16 out (the fold's
      one RNE rounding), or with ``reference_bf16`` the reference's bf16 op sequence;
    * otherwise (N > 1 ranks, rank 0 after the exchange): the f32 mean over all K clients
      within SURVEY §8(c)'s bound with the N-way combine's extra roundings,
      |y - y_ref| <= (K+N+2) 2^-24 r sum_k |w_k x_k| + 2^-24 |y_ref|, with
      max-abs and max-ulp reported; for bf16 deltas (configs[4]) ``y`` is the bf16 mean and
      ``f32_mean`` the f32 mean before the cast: the cast is checked bitwise, and the bf16
      mean against the f64 oracle within 2^-8 |y64| + that bound.
    Returns (status, detail): status "bitwise", "within_tolerance" or "FAILED"."""
    o = _oracle()
    cols = check_cols(P, edges=edges)
    ct = torch.from_numpy(cols).to(y.device)
    bf16 = dtype == torch.bfloat16
    got = y.index_select(0, ct)
    got = (got.view(torch.int16).cpu().numpy().view(np.uint16) if y.dtype == torch.bfloat16
           else got.cpu().numpy())
    kc = (k1 - k0) if exact else K
    x = o.synth_cols_f32(kc, cols, seed=seed, k0=k0 if exact else 0, bf16=bf16)
    w = np.float32(weights[k0:k1] if exact else weights)
    r = np.float32(1.0 / W) if W > 0 else np.float32(0.0)
    detail = {"columns": int(cols.size), "clients": int(kc),
              "oracle": "oracle/fold_ref.c (sequential fold, tree_util.py:76-96) on host-regenerated columns"}
    if exact:
        if reference_bf16:
            xu = (x.view(np.uint32) >> 16).astype(np.uint16)
            want = o.wsum_bf16_refsem(xu, w, r)
        else:
            want = o.wsum_f32(x, w, scale=r)
            if y.dtype == torch.bfloat16:
                want = _bf16_bits(want)
        bad = int(np.count_nonzero(got.view(np.uint16 if want.dtype == np.uint16 else np.uint32)
                                   != want.view(np.uint16 if want.dtype == np.uint16 else np.uint32)))
        detail["compare"] = "bitwise"
        detail["mismatches"] = bad
        return ("bitwise" if bad == 0 else "FAILED"), detail
    want = o.wsum_f32(x, w, scale=r)
    grow = (K + nranks + 2) / (K + 2)
    bound = o.bound_f32(x, w, r, want) * grow
    ym = got if f32_mean is None else f32_mean.index_select(0, ct).cpu().numpy()
    err = np.abs(ym.astype(np.float64) - want.astype(np.float64))
    ok = bool(np.all(err <= bound))
    detail.update({"compare": f"f32 mean within the (K+N+2) sequential-sum bound, N={nranks}",
                   "max_abs": float(err.max()), "max_ulp": int(_ulps(ym, want).max()),
                   "max_err_over_bound": float((err / np.maximum(bound, 1e-300)).max()),
                   "bitwise_columns": int(np.count_nonzero(ym.view(np.uint32) == want.view(np.uint32)))})
    if f32_mean is not None:  # bf16 deltas: the cast of the f32 mean, and the bf16 mean vs f64
        cast_ok = bool(np.array_equal(got, _bf16_bits(ym)))
        xu = (x.view(np.uint32) >> 16).astype(np.uint16)
        y64 = o.wsum_bf16_f64(xu, w.astype(np.float64), float(r))
        fb = (K + nranks + 3) * 2.0 ** -24 * float(r) * np.abs(x.astype(np.float64) * w[:, None]).sum(0) \
            + 2.0 ** -24 * np.abs(y64)
        yb = (got.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        b_ok = bool(np.all(np.abs(yb - y64) <= 2.0 ** -8 * np.abs(y64) + fb))
        detail.update({"bf16_cast_bitwise": cast_ok, "bf16_mean_within_f64_bound": b_ok,
                       "bf16_max_abs_vs_f64": float(np.abs(yb - y64).max())})
        ok = ok and cast_ok and b_ok
    return ("within_tolerance" if ok else "FAILED"), detail


def cpu_baseline(K, seconds=6.0):
    """Reference op sequence (per client: fresh w*x buffer, in-place add; final
    scale) on the host, bounded sample, timed at 1 thread, at the cgroup's CPU
    share and at every core this process may run on (os.sched_getaffinity, SURVEY
    §8(d)). ``value`` / ``cores`` are the fastest of those runs (on a box whose cgroup
    quota is below its visible cores, the quota's thread count beats all cores);
    ``sweep`` holds every run."""
    o = _oracle()
    Ps = 1 << 18  # sample: all K clients x 262,144 params (1 GiB for K = 1024)
    x = o.synth_f32(K, Ps, seed=0)
    w = np.float32(fedavg_weights(K))
    r = np.float32(1.0 / float(sum(fedavg_weights(K))))
    cores = len(os.sched_getaffinity(0))
    share = _cgroup_cpus()
    res = {}
    for nt in sorted({1, cores} | ({min(share, cores)} if share else set())):
        reps, t = 0, 0.0
        while t < seconds / 3 or reps < 2:
            t0 = time.perf_counter()
            o.refseq_f32(x, w, r, nthreads=nt)
            t += time.perf_counter() - t0
            reps += 1
        res[nt] = K * Ps * 4 * reps / t / 1e9
    best = max(res, key=res.get)
    return {"value": round(res[best], 2), "unit": "GB/s", "cores": best, "kind": "port",
            "single_thread_value": round(res[1], 2),
            "all_cores_value": round(res[cores], 2), "visible_cores": cores,
            "sweep": {str(n): round(v, 2) for n, v in sorted(res.items())},
            "cgroup_cpu_share": share,
            "sample": f"{K} clients x {Ps} params fp32 ({K * Ps * 4 / 2**30:.2f} GiB), reference op "
                      f"sequence (tree_util.py:85-96) restated in C, oracle/fold_ref.c; "
                      f"{os.uname().machine} host; fastest of 1 thread / the cgroup quota / all "
                      f"{cores} cores in sched_getaffinity: {best} threads"
                      + (f" (cgroup quota: {share} CPUs)" if share else "")}


def _back_to_back_ms(call, n, batches=5):
    """Milliseconds per call of `call` issued back to back: the median over `batches` batches of
    n // batches calls, each bracketed by a device synchronize (one host stall — a garbage
    collection, a pinned-memory release — then moves one batch, not the figure)."""
    per = max(1, n // batches)
    vals = []
    for _ in range(batches):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(per):
            call()
        torch.cuda.synchronize()
        vals.append((time.perf_counter() - t0) / per * 1e3)
    return float(np.median(vals))


def dropin_surface(dev, calls=20):
    """The drop-in surface itself, timed in the same run as the headline but outside its
    timed region: what examples/fed_avg.py:82 (tree_mean) and
    fedjax/aggregators/aggregator.py:73 (mean_aggregator().apply) call, over caller-held
    pytrees rather than the bench's slab.

    * configs[2] as 1024 separately allocated 4 Mi float32 tensors through
      ``mean_aggregator().apply`` (calls back to back);
    * configs[1] as 128 EMNIST-CNN pytrees, every (client, leaf) its own allocation,
      through ``tree_mean``: calls back to back, and one synchronous call on an idle GPU
      (the latency a server aggregating once per round sees);
    * the same clients through the library algorithms' running sum (fed_avg.py:132-146),
      one synchronous round.

    GB/s = the K*P*4 algorithmic bytes of client deltas / the time per call."""
    import fedjax_amd
    from fedjax_amd import kernels, tree_util as tu

    res = {}
    pc = time.perf_counter
    # configs[2]: 1024 x 4 Mi as separate tensors through the Aggregator surface
    K, P = 1024, 4 * 1024 * 1024
    clients = []
    for k in range(K):
        t = torch.empty(P, dtype=torch.float32, device=dev)
        kernels.fill_synth(t.view(1, P), seed=0, k0=k)
        clients.append(t)
    triples = [(f"c{k}", t, w) for k, (t, w) in enumerate(zip(clients, fedavg_weights(K)))]
    agg = fedjax_amd.aggregators.mean_aggregator()
    state = agg.init()
    for _ in range(3):
        agg.apply(triples, state)
    torch.cuda.synchronize()
    t0 = pc()
    for _ in range(calls):
        out, state = agg.apply(triples, state)
    torch.cuda.synchronize()
    ms = (pc() - t0) / calls * 1e3
    res["c2_mean_aggregator_apply_ms"] = round(ms, 4)
    res["c2_mean_aggregator_apply_GBs"] = round(K * P * 4 / ms / 1e6, 1)
    del clients, triples, out
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    # configs[1]: 128 EMNIST-CNN pytrees, one allocation per (client, leaf)
    shapes = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
              "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
    K, P = 128, 1206590

    def tree(k):
        out, seed = {}, 1
        for mod, leaves in shapes.items():
            out[mod] = {}
            for name, shp in leaves.items():
                n = int(np.prod(shp))
                x = torch.empty(1, n, dtype=torch.float32, device=dev)
                kernels.fill_synth(x, seed=seed, k0=k)
                out[mod][name] = x.view(shp)
                seed += 1
        return out

    pairs = list(zip([tree(k) for k in range(K)], fedavg_weights(K)))
    for _ in range(5):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    n = 5 * calls
    ms = _back_to_back_ms(lambda: tu.tree_mean(pairs), n)
    res["c1_tree_mean_back_to_back_ms"] = round(ms, 4)
    res["c1_tree_mean_back_to_back_GBs"] = round(K * P * 4 / ms / 1e6, 1)
    single = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = pc()
        tu.tree_mean(pairs)
        torch.cuda.synchronize()
        single.append(pc() - t0)
    ms = float(np.median(single)) * 1e3
    res["c1_tree_mean_sync_call_ms"] = round(ms, 4)
    res["c1_tree_mean_sync_call_GBs"] = round(K * P * 4 / ms / 1e6, 1)
    # the same clients through the Aggregator surface (aggregator.py:61-75), one synchronous call
    agg, single = fedjax_amd.aggregators.mean_aggregator(), []
    triples = [(f"c{k}", t, w) for k, (t, w) in enumerate(pairs)]
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = pc()
        agg.apply(triples, state)
        torch.cuda.synchronize()
        single.append(pc() - t0)
    ms = float(np.median(single)) * 1e3
    res["c1_mean_aggregator_apply_sync_call_ms"] = round(ms, 4)
    res["c1_mean_aggregator_apply_sync_call_GBs"] = round(K * P * 4 / ms / 1e6, 1)
    del triples
    # the library algorithms' running sum (fedjax/algorithms/fed_avg.py:132-146): one
    # synchronous round of tree_add(s, tree_weight(delta, n)) x K + tree_inverse_weight,
    # (a) as fed_avg.py:132-146 writes it, with the per-client delta_l2_norm kept in
    # client_diagnostics (:142-144), and (b) without the norm (the aggregation alone)
    W = float(sum(w for _, w in pairs))
    import gc
    gc.collect()
    loops = {True: [], False: []}
    for i in range(2 * (calls + 2)):  # rounds with and without the norms alternate (box drift hits both)
        with_norms = i % 2 == 0
        torch.cuda.synchronize()
        t0 = pc()
        s, client_diagnostics = tu.tree_zeros_like(pairs[0][0]), {}
        for cid, (t, w) in enumerate(pairs):
            s = tu.tree_add(s, tu.tree_weight(t, w))
            if with_norms:
                client_diagnostics[cid] = {"delta_l2_norm": tu.tree_l2_norm(t)}
        mean = tu.tree_inverse_weight(s, W)
        torch.cuda.synchronize()
        if i >= 4:
            loops[with_norms].append(pc() - t0)
        if with_norms and i == 2 * (calls + 2) - 2:  # the kept norms hold the values: vs one batched launch
            got = torch.stack([client_diagnostics[c]["delta_l2_norm"] for c in range(K)])
            ref = tu.tree_l2_norms([t for t, _ in pairs])
            res["c1_library_loop_norms_max_rel_diff"] = float(((got - ref).abs() / ref).max())
            del got, ref
    del s, mean, client_diagnostics
    for with_norms in (True, False):
        ms = float(np.median(loops[with_norms])) * 1e3
        key = "c1_library_loop_with_norms_round" if with_norms else "c1_library_loop_without_norms_round"
        res[key + "_ms"] = round(ms, 4)
        res[key + "_GBs"] = round(K * P * 4 / ms / 1e6, 1)
    # examples/fed_avg.py:72-82 as written: per client the (delta, n) pair appended and
    # tree_l2_norm(delta) kept in client_diagnostics, then tree_mean of the list. The norms are
    # lazy views the mean's launch fills (tree_util.set_lazy_norms): one pass over the deltas.
    # Rounds alternate with the same synchronous tree_mean without the norms (same box drift).
    H = tu._HOST
    for Kx in (K, 10):
        sub, sfx = pairs[:Kx], "" if Kx == K else f"_k{Kx}"
        times, fused0, rounds = {True: [], False: []}, H.solo_info()["fused"], 0
        for i in range(2 * (calls + 2)):
            with_norms = i % 2 == 0
            torch.cuda.synchronize()
            t0 = pc()
            if with_norms:
                client_diagnostics, client_delta_params_weights = {}, []
                for cid, (delta_params, n_) in enumerate(sub):
                    client_delta_params_weights.append((delta_params, n_))
                    client_diagnostics[cid] = {"delta_l2_norm": tu.tree_l2_norm(delta_params)}
                mean = tu.tree_mean(client_delta_params_weights)
                rounds += 1
            else:
                mean = tu.tree_mean(sub)
            torch.cuda.synchronize()
            if i >= 4:
                times[with_norms].append(pc() - t0)
        got = torch.stack([client_diagnostics[c]["delta_l2_norm"] for c in range(Kx)])
        ref = tu.tree_l2_norms([t for t, _ in sub])
        res[f"c1_example_norms_max_rel_diff{sfx}"] = float(((got - ref).abs() / ref).max())
        res[f"c1_example_norms_fused_frac{sfx}"] = round((H.solo_info()["fused"] - fused0) / (rounds * Kx), 4)
        for with_norms in (True, False):
            ms = float(np.median(times[with_norms])) * 1e3
            key = "c1_example_round_with_norms" if with_norms else "c1_example_round_mean_only"
            res[key + sfx + "_ms"] = round(ms, 4)
            res[key + sfx + "_GBs"] = round(Kx * P * 4 / ms / 1e6, 1)
        del got, ref, mean, client_diagnostics, client_delta_params_weights
    # the same clients as fedjax_amd produces them under the process-wide switch
    # memory.set_default(True): host deltas copied to the device leaf by leaf
    # (memory.to_device), from the delta pool (include/fjalloc.h) — still one tensor per
    # (client, leaf), placed in shared chunks
    from fedjax_amd import memory, pytree
    host_trees = []
    for t, _ in pairs:
        lv, td = pytree.flatten(t)
        host_trees.append(pytree.unflatten(td, [x.cpu().pin_memory() for x in lv]))
    memory.set_default(True)
    try:
        pooled = list(zip([memory.to_device(t, dev) for t in host_trees], fedavg_weights(K)))
    finally:
        memory.set_default(False)
    del host_trees
    for _ in range(5):
        tu.tree_mean(pooled)
    torch.cuda.synchronize()
    res["c1_default_pool_tree_mean_back_to_back_ms"] = round(_back_to_back_ms(lambda: tu.tree_mean(pooled), n), 4)
    single = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = pc()
        tu.tree_mean(pooled)
        torch.cuda.synchronize()
        single.append(pc() - t0)
    res["c1_default_pool_tree_mean_sync_call_ms"] = round(float(np.median(single)) * 1e3, 4)
    res["c1_default_pool_tree_mean_sync_call_GBs"] = round(K * P * 4 / float(np.median(single)) / 1e9, 1)
    got = tu.tree_mean(pooled)  # the same bits as the default allocations' mean
    ref = tu.tree_mean(pairs)
    res["c1_default_pool_bitwise"] = all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in
                                         zip(pytree.leaves_of(got), pytree.leaves_of(ref)))
    del got, ref
    del pooled
    res["note"] = ("caller-held pytrees, separate allocations; timed after the headline, outside its "
                   "timed region; GB/s = K*P*4 client-delta bytes per call (library loop: per round); "
                   "c1_library_loop_with_norms: fed_avg.py:132-146 as written (tree_l2_norm per client into "
                   "client_diagnostics), c1_library_loop_without_norms: the same loop without the norm; "
                   "c1_example_round_with_norms[_k10]: examples/fed_avg.py:72-82 as written (128 / 10 clients: "
                   "tree_l2_norm per client into client_diagnostics, then tree_mean of the list; the norms are lazy "
                   "views the mean's launch fills), c1_example_round_mean_only: the same synchronous tree_mean "
                   "without the norms, rounds alternating; "
                   "c1_default_pool_*: the same clients produced by fedjax_amd.memory.to_device under "
                   "fedjax_amd.memory.set_default(True) (the delta pool)")
    del pairs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def drain_stream(stream, seconds: float) -> bool:
    """Wait (polling) until `stream` has no pending work, at most `seconds`."""
    done = torch.cuda.Event()
    done.record(stream)
    t0 = time.perf_counter()
    while not done.query():
        if time.perf_counter() - t0 > seconds:
            return False
        time.sleep(0.001)
    return True


def autotune_exchange(cands, measure, abort_native, dev, rank):
    """Time every exchange candidate (engine, collective, buckets) on every rank and agree on
    each outcome over the process group: ({candidate: ms, max over ranks}, {candidate: why
    dropped}). ``measure(cand)`` returns this rank's ms per step, None past its host deadline,
    or raises. A candidate that failed or missed its deadline on ANY rank is dropped on every
    rank; a missed deadline on the library's own communicator ("native" engine) makes every
    rank call ``abort_native()`` (fjcomm_abort) and skip the remaining native candidates, so one
    hung collective costs one deadline instead of the run (reference analogue: the pmap
    gather of fedjax/core/for_each_client.py:266-357, which has no such bound)."""
    import torch.distributed as dist
    tune, dropped, native_dead = {}, {}, False
    for cand in cands:
        if cand[0] == "native" and native_dead:
            dropped[cand] = "skipped: communicator aborted"
            continue
        status, ms = 0.0, 0.0  # 0 ok, 1 raised, 2 missed the deadline
        try:
            got = measure(cand)
            if got is None:
                status = 2.0
                log(f"[bench rank {rank}] auto-tune candidate {cand[0]}/{cand[1]}/{cand[2]} missed its deadline")
            else:
                ms = float(got)
        except Exception as e:  # noqa: BLE001
            status = 1.0
            log(f"[bench rank {rank}] auto-tune candidate {cand[0]}/{cand[1]}/{cand[2]} failed: {e}")
        if status == 2.0 and cand[0] == "native":
            abort_native()  # before the agreement: its collective may hold the GPU until then
        flag = torch.tensor([status, ms], dtype=torch.float64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        worst, slowest = float(flag[0].item()), float(flag[1].item())
        if worst == 0.0:
            tune[cand] = slowest
            continue
        dropped[cand] = "dropped: missed the deadline" if worst == 2.0 else "dropped: raised"
        if worst == 2.0 and cand[0] == "native":
            if status != 2.0:
                abort_native()  # (another rank missed it: this rank stops using the communicator too)
            native_dead = True
    return tune, dropped


def rank_timeout(args) -> float:
    """Seconds a spawned N-rank run may take before spawn_ranks kills it: process start,
    rendezvous and communicator init (300 s), plus every step the ranks run — warmup,
    timed steps, the exchange auto-tune (24 candidates x 7 steps) and the e2e repeats —
    at a pessimistic 0.5 TB/s per rank for that rank's share of the deltas, times 4."""
    K, P, dtype, _ = WORKLOADS[args.workload]
    K = args.clients or K
    esize = torch.empty((), dtype=dtype).element_size()
    per_rank_s = (K + args.gpus - 1) // args.gpus * P * esize / 0.5e12
    steps = args.warmup + args.steps + 24 * 7 + 6
    # (+ one missed auto-tune deadline, the abort's stream drain and the communicator's teardown)
    return 300.0 + 4.0 * steps * per_rank_s + 2.0 * args.candidate_deadline + 70.0


def start_rank_watchdog(rank: int, seconds: float):
    """Ranks started by an outer launcher (the driver's ``torch.distributed.run``, no
    spawn_ranks parent to time them): past ``seconds`` without reaching "done" the rank
    names the phase it is stuck in and exits with status 124, so the launcher tears the
    job down instead of waiting on a stuck rendezvous or collective. A process exit, not
    an exec. Returns the timer (cancelled at "done")."""
    import threading

    def expire():
        log(f"[bench rank {rank}] watchdog: not done within {seconds:.0f} s, stuck in phase "
            f"'{_LAST_PHASE[0]}'; exiting with status 124")
        os._exit(124)

    t = threading.Timer(seconds, expire)
    t.daemon = True
    t.start()
    return t


def _rank_phases(d: str, nproc: int):
    out = {}
    for r in range(nproc):
        try:
            with open(os.path.join(d, f"rank{r}")) as f:
                out[r] = f.read().strip() or "started"
        except OSError:
            out[r] = "not started"
    return out


def spawn_ranks(nproc: int, argv, script: str = None, timeout: float = None) -> int:
    """Run ``script argv`` as ``nproc`` ranks of one node and forward rank 0's JSON line.

    A bare ``python bench.py --gpus N`` (no WORLD_SIZE in the environment) lands here
    before anything touches the GPU. The ranks are children of this process
    (``python -m torch.distributed.run``, rendezvous on 127.0.0.1, in a process group of
    their own): nothing is exec'd. Every rank's stderr passes through; stdout is collected
    and only the JSON line (rank 0's) is printed. Returns the launcher's exit status,
    non-zero if any rank failed or no JSON line came back. Rank 0 writes its line to the
    file named in FJ_BENCH_JSON (emit_json); the shared stdout pipe is the fallback for
    scripts that do not.

    ``timeout`` (seconds, None = none): past it the whole process group is terminated
    (SIGTERM, then SIGKILL after 10 s), the ranks that had not reached their "done" phase
    are named with the last phase each one wrote (FJ_BENCH_PHASES, bench.phase), and the
    return status is 124."""
    import shutil
    import signal
    import subprocess
    import tempfile

    # --standalone: the launcher's c10d rendezvous binds its TCP store on port 0 and keeps it,
    # and the ranks join through that store (TORCHELASTIC_USE_AGENT_STORE). Until round 4 a
    # port found by binding 0 and closing the socket was passed as --master-port; another
    # process could take it in between (the intermittent rc=1 of test_spawn_forwards_rank0_json).
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--local-addr=127.0.0.1", script or os.path.abspath(__file__), *argv]
    fd, json_path = tempfile.mkstemp(prefix="fj_bench_", suffix=".json")
    os.close(fd)
    phase_dir = tempfile.mkdtemp(prefix="fj_bench_phases_")
    env = dict(os.environ, FJ_BENCH_LAUNCHER="bench.py -> torch.distributed.run child", FJ_BENCH_JSON=json_path,
               FJ_BENCH_PHASES=phase_dir)
    log("+", " ".join(cmd) + (f"   (timeout {timeout:.0f} s)" if timeout else ""))
    try:
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, start_new_session=True)
        try:
            out, _ = proc.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            phases = _rank_phases(phase_dir, nproc)
            stuck = [r for r, p in phases.items() if p != "done"]
            log(f"bench: spawned ranks did not finish within {timeout:.0f} s; ranks {stuck} had not finished "
                f"(last phase per rank: {phases}); terminating the launcher's process group")
            for sig, wait in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
                try:
                    os.killpg(proc.pid, sig)  # the group this call started (start_new_session)
                except ProcessLookupError:
                    break
                try:
                    proc.wait(timeout=wait)
                    break
                except subprocess.TimeoutExpired:
                    continue
            return 124
        with open(json_path) as f:
            filed = f.read().strip()
    finally:
        os.unlink(json_path)
        shutil.rmtree(phase_dir, ignore_errors=True)
    if proc.returncode != 0:
        log(f"bench: spawn_ranks returns {proc.returncode}: the rank launcher exited with that status "
            f"(a rank failed; its stderr is above)")
        return proc.returncode
    if filed:  # rank 0's line from its own file: nothing else can be interleaved into it
        lines = [filed]
    else:  # a script that does not write FJ_BENCH_JSON: rank 0's JSON object on the shared pipe
        lines = []
        for ln in out.decode(errors="replace").splitlines():
            i = ln.find('{"')  # another rank's unterminated banner can precede the JSON
            if i >= 0:
                try:
                    json.loads(ln[i:])
                    lines.append(ln[i:])
                except ValueError:
                    pass
    if len(lines) != 1:
        log(f"bench: spawn_ranks returns 1: expected one JSON line from rank 0, got {len(lines)} "
            f"(rank 0's file {'was empty' if not filed else 'held a line'}; stdout {len(out)} bytes)")
        return 1
    sys.stdout.write(lines[0] + "\n")
    sys.stdout.flush()
    return 0


def emit_json(json_fd, res):
    """Rank 0's result line: to the saved stdout, and to the file a spawning parent named in
    FJ_BENCH_JSON (ranks share one stdout pipe, where a line longer than PIPE_BUF could be
    interleaved with another rank's output)."""
    line = json.dumps(res) + "\n"
    path = os.environ.get("FJ_BENCH_JSON")
    if path:
        with open(path, "w") as f:
            f.write(line)
    os.write(json_fd, line.encode())


def load_traffic(workload, path=None):
    """HBM bytes per launch of the dominant kernel from the PMC passes in
    profiles/traffic_<workload>.json, with where they came from: the build (sha256 of the
    libfjagg.so the counters ran) and whether it is the build running now. None: no file."""
    p = path or os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_summary import build_tag

    now = build_tag()
    src = {"file": os.path.relpath(p, ROOT), "measured_in_this_run": False,
           "method": d.get("method", "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_full.sh)"),
           "correction": d.get("correction"), "build": d.get("build", d.get("collected")),
           "this_build": now, "same_build": d.get("build") == now, "collected": d.get("collected")}
    return d.get("hbm_bytes_per_launch"), src


def measure_traffic(workload, dst=None):
    """--measure-traffic: the FETCH_SIZE and WRITE_SIZE passes run here, each as its own
    rocprofv3 child over a short bench run of the same workload (no cpu baseline, no
    drop-in), summarised by tools/pmc_summary.py into profiles/traffic_<workload>.json.
    Returns (bytes per launch, source record) for this run's line."""
    import subprocess
    import tempfile

    out = tempfile.mkdtemp(prefix="fj_pmc_")
    cmd = [sys.executable, os.path.abspath(__file__), "--workload", workload, "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-dropin"]
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        log(f"[bench] PMC pass {counter}")
        subprocess.run(["rocprofv3", "--pmc", counter, "-d", os.path.join(out, counter), "-o", "run",
                        "--output-format", "csv", "--", *cmd], check=True, timeout=300,
                       stdout=subprocess.DEVNULL)
    dst = dst or os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), os.path.join(out, "FETCH_SIZE"),
                    os.path.join(out, "WRITE_SIZE"), dst], check=True, timeout=120, stdout=subprocess.DEVNULL)
    b, src = load_traffic(workload, dst)
    if src is not None:
        src["measured_in_this_run"] = True
    return b, src


# host RAM one rank may pin for its shard in the e2e leg (a configs[4] shard is 256 GB)
E2E_MAX_PINNED_BYTES = 64 << 30
# N = 1 default e2e sample: the first 256 clients of the slab (4.3 GB at configs[2]); --e2e: all
E2E_SAMPLE_CLIENTS = 256


def host_resident_rate(x, w_local, sharded_step, out, scale, nt, dev, rank, sharded, job_bytes, reps=3):
    """The deployment rate (north star): every rank's client deltas start in
    its own pinned host memory and go over its own PCIe link (H2D into the resident slab),
    then the fold — at N>1 the whole sharded step, fold + RCCL reduce — and the mean comes
    back to the host (D2H on rank 0). Rate = all clients' bytes / the max-over-ranks wall
    time of ``reps`` such rounds. Every rank decides together whether its shard fits the
    pinned budget (one all_reduce), so either all ranks run the leg or none does. At N = 1
    ``x`` may be the first clients of the slab only (a sub-sample: the rate is PCIe-bound
    and does not depend on the client count; ``job_bytes`` are that sample's bytes)."""
    from fedjax_amd import kernels

    nbytes = x.shape[0] * x.shape[1] * x.element_size()
    ok = nbytes <= E2E_MAX_PINNED_BYTES
    xh = None
    if ok:
        try:
            xh = torch.empty(x.shape, dtype=x.dtype).pin_memory()
            xh.copy_(x)  # D2H straight into the pinned buffer
        except RuntimeError as e:  # pinned allocation refused: skip the leg on every rank
            log(f"[bench rank {rank}] e2e: pinned host buffer of {nbytes / 2**30:.1f} GiB refused ({e})")
            ok, xh = False, None
    if sharded:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())
    if not ok:
        return {"e2e_host_resident_GBs": None,
                "e2e_note": f"skipped: a rank's shard ({nbytes / 2**30:.1f} GiB) exceeds the "
                            f"{E2E_MAX_PINNED_BYTES >> 30} GiB pinned-host budget or was refused"}
    yh = torch.empty(out.shape, dtype=out.dtype).pin_memory()
    wd = torch.from_numpy(np.float32(w_local[:x.shape[0]])).to(dev)

    def one():
        x.copy_(xh, non_blocking=True)
        if sharded:
            sharded_step()
        else:
            kernels.weighted_sum_dense(x, wd, scale=scale, out=out, nontemporal=nt)
        if rank == 0:
            yh.copy_(out, non_blocking=True)

    one()  # warm (first pinned transfers map the buffers)
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    ts = time.perf_counter()
    for _ in range(reps):
        one()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    t = time.perf_counter() - ts
    if sharded:
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    del xh
    return {"e2e_host_resident_GBs": round(job_bytes * reps / t / 1e9, 2),
            "e2e_ms_per_round": round(t / reps * 1e3, 4),
            "e2e_note": "each rank's deltas in its own pinned host memory -> its own PCIe link (H2D) -> "
                        + (f"fold + {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} exchange"
                           if sharded else "fold") + " -> mean D2H on rank 0; "
                        "bytes = all clients' deltas; max over ranks"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--candidate-deadline", type=float, default=60.0,
                    help="host seconds one exchange auto-tune measurement may take before the library's own "
                         "communicator is aborted and its candidates dropped (torch-engine candidates run first)")
    ap.add_argument("--buckets", default="0",
                    help="N>1: parameter buckets of the fold/reduce pipeline, a count or relative sizes "
                         "like 4:2:1; 0 = pick the fastest of BUCKET_CANDIDATES during warmup (max over ranks)")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--nontemporal", type=int, default=-1, help="-1 auto, 0 off, 1 on")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in surface sub-record (mean_aggregator().apply / tree_mean over "
                         "caller-held pytrees, timed after the headline)")
    ap.add_argument("--e2e", action="store_true",
                    help="N=1: time host-resident deltas (H2D + fold + D2H) over ALL the clients (default: "
                         f"the first {E2E_SAMPLE_CLIENTS} clients' deltas, a stated sub-sample)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-resident end-to-end leg")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the check of the timed result against the oracle (sampled columns)")
    ap.add_argument("--measure-traffic", action="store_true",
                    help="N=1: run the FETCH_SIZE / WRITE_SIZE rocprofv3 passes from this run (child processes) "
                         "and report their HBM bytes as roofline.traffic (default: profiles/traffic_<workload>.json "
                         "with its build tag)")
    ap.add_argument("--traffic-out", default="",
                    help="--measure-traffic: where the summary goes (default profiles/traffic_<workload>.json)")
    ap.add_argument("--timeout", type=float, default=0,
                    help="bare --gpus N: seconds before the spawned ranks are killed (0 = derived from the "
                         "workload and steps, rank_timeout)")
    ap.add_argument("--backend", default="nccl", help="nccl (RCCL) for runs; gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--all-ranks", action="store_true",
                    help="every rank needs the mean: all_reduce only (default: the mean is needed on rank 0, and "
                         "the auto-tune may still pick all_reduce when RCCL runs it faster than reduce)")
    ap.add_argument("--engine", choices=["auto", "native", "torch"], default="auto",
                    help="N>1 exchange: native RCCL pipeline (include/fjcomm.h), torch.distributed, or the "
                         "faster of the two measured during warmup")
    ap.add_argument("--server", choices=["none", "sgd", "adam"], default="none",
                    help="fuse the server optimizer step into the fold (N=1; examples/fed_avg.py:97-101)")
    ap.add_argument("--rehearse-shard", type=int, default=0, metavar="N",
                    help="one GPU, world 1: run rank 0's share of an N-way shard through the full sharded "
                         "step (RCCL communicator of one rank). Timing rehearsal only: no cross-GPU traffic")
    ap.add_argument("--clients", type=int, default=0, help="override the workload's client count (experiments)")
    ap.add_argument("--single-process", action="store_true",
                    help="N GPUs driven by ONE process (fjcomm_init_all / fjcomm_multi_wsum_dense, grouped RCCL "
                         "reduce): the shape of FedJAX's server over jax.local_devices(); no launcher")
    ap.add_argument("--with-norms", action="store_true",
                    help="fuse every client's delta l2 norm into the fold (examples/fed_avg.py:79-81)")
    ap.add_argument("--reference-bf16", action="store_true",
                    help="bf16 workloads: the reference's bf16 arithmetic (every product and sum rounded to bf16, "
                         "tree_util.set_bf16_semantics('reference')) instead of the f32 fold")
    ap.add_argument("--device-weights", action="store_true",
                    help="upload the weights each step (pinned H2D in front of the fold) instead of passing "
                         "them in the kernel arguments (A/B of FJAGG_HOST_TABLES)")
    args = ap.parse_args()
    if args.single_process:
        return single_process(args)
    if args.reference_bf16 and (WORKLOADS[args.workload][2] != torch.bfloat16 or args.gpus > 1 or args.with_norms):
        raise SystemExit("--reference-bf16 runs a bf16 workload (c5s) at N=1 without fused norms")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # bare `python bench.py --gpus N`: one rank per GPU as child processes (nothing in
        # this process touches the GPU runtime, not even a device count — the ranks check
        # that there are enough GPUs — and nothing is exec'd)
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:],
                                     timeout=args.timeout if args.timeout > 0 else rank_timeout(args)))
    # stdout carries exactly one line, rank 0's JSON: native libraries write banners to fd 1
    # (RCCL's version block, gloo's connection notes), so fd 1 is pointed at stderr for the
    # rest of the run and the JSON goes to a saved copy of the original stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            raise SystemExit("launch N>1 with torch.distributed.run (one rank per GPU)")
    ngpu = torch.cuda.device_count()
    if world > 1 and args.backend == "nccl" and ngpu < world:
        raise SystemExit(f"--gpus {world} needs {world} visible GPUs for RCCL (found {ngpu}); "
                         f"--backend gloo rehearses on fewer")
    watchdog = None
    if world > 1 and "FJ_BENCH_PHASES" not in os.environ:  # (under spawn_ranks the parent times the ranks)
        watchdog = start_rank_watchdog(rank, args.timeout if args.timeout > 0 else rank_timeout(args))
    dev = torch.device("cuda", local_rank % max(1, ngpu))
    torch.cuda.set_device(dev)
    nshard = world
    if args.rehearse_shard > 1:
        if world != 1:
            raise SystemExit("--rehearse-shard runs as a single process")
        nshard = args.rehearse_shard
    sharded = nshard > 1
    if sharded:
        phase(rank, f"init process group ({args.backend}, world {world})")
        kw = {"device_id": dev} if args.backend == "nccl" else {}
        if world == 1:  # the one-GPU rehearsal: its own store, bound on port 0 and held (no port race)
            kw["store"] = dist.TCPStore("127.0.0.1", 0, 1, True)
        dist.init_process_group(args.backend, rank=rank, world_size=world, **kw)

    import fedjax_amd  # noqa: F401
    from fedjax_amd import distributed as fd, kernels, tree_util as tu

    K, P, dtype, desc = WORKLOADS[args.workload]
    if args.clients:
        K, desc = args.clients, desc + f" [clients overridden: {args.clients}]"
    esize = torch.empty((), dtype=dtype).element_size()
    weights = fedavg_weights(K)
    W = 0.0
    for w in weights:
        W += w  # tree_util.py:95
    k0, k1 = fd.shard_range(K, rank, nshard)
    Kl = k1 - k0
    if Kl > 1024 and dtype == torch.bfloat16:
        raise SystemExit(f"{args.workload}: {Kl} clients x {P} params per GPU exceed 288 GB; use more GPUs")
    # ClientDeltaSlab layout: rows padded to 16 bytes (vector path)
    vw = 16 // esize
    ld = (P + vw - 1) // vw * vw
    x = torch.empty(Kl, ld, dtype=dtype, device=dev)[:, :P]
    phase(rank, f"fill {Kl} clients x {P} params")
    kernels.fill_synth(x, seed=0, k0=k0)  # the same global client k on every N
    w_local = [weights[k] for k in range(k0, k1)]
    out = torch.empty(P, dtype=dtype if not sharded else torch.float32, device=dev)
    final = torch.empty(P, dtype=dtype, device=dev) if (sharded and dtype != torch.float32) else None
    ones = torch.ones(1, dtype=torch.float32, device=dev)
    nbytes_local = Kl * P * esize
    nt = (nbytes_local >= tu.NONTEMPORAL_MIN_BYTES) if args.nontemporal < 0 else bool(args.nontemporal)
    scale = float(np.float32(tu._inverse(W)))
    stream = torch.cuda.current_stream(dev)
    l2sq = torch.empty(Kl, dtype=torch.float32, device=dev) if args.with_norms else None
    kernel_ms = []

    def fold(xs, wd, o, events):
        if events is not None:
            e0, e1 = kernels.Event(), kernels.Event()
            e0.record(stream)
        if args.with_norms:
            kernels.weighted_sum_l2_dense(xs, wd, scale=scale, out=o, l2sq=l2sq, nontemporal=nt)
        else:
            kernels.weighted_sum_dense(xs, wd, scale=scale, out=o, nontemporal=nt, variant=args.variant,
                                       reference_bf16=args.reference_bf16)
        if events is not None:
            e1.record(stream)
            events.append((e0, e1, xs.shape[0] * xs.shape[1] * esize))

    if args.server != "none":
        if sharded or dtype != torch.float32:
            raise SystemExit("--server runs at N=1 on f32 slabs")
        from fedjax_amd import _lib as flib, server as fsrv
        sopt = fsrv.sgd(10 ** -1.5) if args.server == "sgd" else fsrv.adam(10 ** -2.5, b1=0.9, b2=0.999, eps=1e-4)
        sparams = torch.zeros(P, dtype=torch.float32, device=dev)
        sstate = sopt.init(sparams)

    # N>1 exchange engines: "native" = one fjcomm_sharded_wsum_dense call per step (own RCCL
    # communicator, device-scope events between fold and reduce buckets); "torch" = per-bucket
    # HIP fold + torch.distributed collective (ProcessGroupNCCL)
    comm = None
    if sharded and args.backend == "nccl" and args.engine in ("auto", "native") and not args.with_norms:
        phase(rank, "native RCCL communicator init")
        try:
            comm = fd.RcclCommunicator(device=dev)
        except Exception as e:  # noqa: BLE001 - the torch engine still runs
            if args.engine == "native":
                raise
            log(f"native RCCL communicator unavailable ({e}); using torch.distributed")
    engine = "native" if comm is not None else "torch"
    buckets = (tuple(float(v) for v in args.buckets.split(":")) if ":" in args.buckets
               else int(args.buckets)) or 1
    root = 0
    collective = "all_reduce" if args.all_ranks else "reduce"  # the exchange of the partials

    def step(events=None):
        # the round's weights: host float32, carried in the fold's kernel arguments
        # (FJAGG_HOST_TABLES) when the launch allows it; uploaded (pinned H2D on the stream)
        # for the fused-norm / server-step kernels and with --device-weights
        wd = np.float32(w_local)
        if args.device_weights or args.server != "none" or args.with_norms:
            wd = torch.from_numpy(wd).pin_memory().to(dev, non_blocking=True)
        if args.server != "none":
            desc = sopt.descriptor(1)  # copied by value into the kernel arguments at launch
            if events is not None:
                e0, e1 = kernels.Event(), kernels.Event()
                e0.record(stream)
            flib.call("fjagg_server_update_dense", flib.F32, x.data_ptr(), x.stride(0), Kl, P, wd.data_ptr(),
                      scale, ctypes.byref(desc), sparams.data_ptr(),
                      sstate.get("m").data_ptr() if "m" in sstate else None,
                      sstate.get("v").data_ptr() if "v" in sstate else None, None,
                      flib.NONTEMPORAL if nt else 0, stream.cuda_stream)
            if events is not None:
                e1.record(stream)
                events.append((e0, e1, Kl * P * esize))
        elif not sharded:
            fold(x, wd, out, events)
        elif engine == "native":
            evs, spans = None, fd.bucket_edges(P, buckets)
            if events is not None:
                evs = [kernels.Event() for _ in range(2 * len(spans))]
            fd.sharded_weighted_mean(x, wd, W, buckets=buckets, out=out, all_ranks=collective == "all_reduce",
                                     comm=comm, nontemporal=nt, fold_events=evs)
            if evs is not None:
                for i, (p0, p1) in enumerate(spans):
                    events.append((evs[2 * i], evs[2 * i + 1], Kl * (p1 - p0) * esize))
        else:
            fd.sharded_weighted_mean(x, wd, W, buckets=buckets, out=out, all_ranks=collective == "all_reduce",
                                     partial_fn=lambda xs, wdd, sc, o: fold(xs, wdd, o, events))
        if sharded and final is not None and (rank == root or collective == "all_reduce"):  # f32 mean -> leaf dtype
            kernels.weighted_sum_dense(out.view(1, P), ones, out=final)

    def wall(nsteps):
        """Max-over-ranks wall time of nsteps steps, bracketed like the timed region."""
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def wall_local(nsteps, deadline_s):
        """This rank's wall time of nsteps steps, or None when they have not completed within
        deadline_s (polled: no blocking wait on a collective that may never end). No
        collective runs after the steps: the ranks compare results in autotune_exchange."""
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step()
        done = torch.cuda.Event()
        done.record(stream)  # (the steps end on `stream`: the last bucket reduces there)
        while not done.query():
            if time.perf_counter() - t0 > deadline_s:
                return None
            time.sleep(0.0002)
        return time.perf_counter() - t0

    tune = {}
    if sharded and args.buckets == "0":
        # every rank measures every candidate and the ranks agree on each result (max over
        # ranks), so all pick the same (engine, collective, buckets). The mean is needed on rank
        # 0 only, so all_reduce is a candidate next to reduce: RCCL may run it faster (its
        # all-reduce algorithms are the most tuned), and it leaves the same mean on rank 0
        # (within the tolerance of DESIGN.md §4). The torch engine's candidates run first; the
        # library's own communicator's run under a host deadline — past it every rank aborts
        # that communicator (fjcomm_abort) and its remaining candidates are skipped.
        engines = ["torch", "native"] if comm is not None and args.engine == "auto" else [engine]
        colls = ["all_reduce"] if args.all_ranks else ["reduce", "all_reduce"]
        cands = [(eng, col, b) for eng in engines for col in colls for b in BUCKET_CANDIDATES
                 if len(fd.bucket_edges(P, b)) >= (b if isinstance(b, int) else len(b))]
        deadline_s = args.candidate_deadline

        def measure(cand):
            nonlocal engine, collective, buckets
            engine, collective, buckets = cand
            phase(rank, f"auto-tune candidate {cand[0]}/{cand[1]}/{fd.bucket_name(cand[2])}")
            if wall_local(2, deadline_s) is None:
                return None
            t = wall_local(5, deadline_s)
            return None if t is None else t / 5 * 1e3

        def abort_native():
            if comm is not None:
                try:
                    comm.abort()
                except Exception as e:  # noqa: BLE001
                    log(f"[bench rank {rank}] fjcomm_abort: {e}")
            if not drain_stream(stream, 60.0):
                log(f"[bench rank {rank}] the stream did not drain within 60 s after fjcomm_abort")
                sys.stdout.flush()
                os._exit(124)

        tune, dropped = autotune_exchange(cands, measure, abort_native, dev, rank)
        if not tune:
            raise SystemExit("every exchange candidate failed (see the auto-tune lines above)")
        engine, collective, buckets = min(tune, key=tune.get)
        tune = {f"{e}/{c}/{fd.bucket_name(b)}": round(t, 4) for (e, c, b), t in tune.items()}
        tune.update({f"{e}/{c}/{fd.bucket_name(b)}": why for (e, c, b), why in dropped.items()})
        log(f"exchange auto-tune (ms/step, max over ranks): {tune} -> "
            f"{engine}/{collective}/{fd.bucket_name(buckets)}")
    phase(rank, f"warmup ({args.warmup} steps)")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    phase(rank, f"timed loop ({args.steps} steps)")
    events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(events)
    t_issue = time.perf_counter() - t0  # host time to enqueue the steps (host-bound if ~ elapsed)
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if sharded:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = [e0.elapsed_time(e1) for e0, e1, _ in events]
    bytes_per_launch = float(np.mean([b for _, _, b in events]))
    mean_kernel_s = float(np.mean(kernel_ms)) / 1e3
    achieved = bytes_per_launch / mean_kernel_s / 1e9

    # the timed result against the oracle (rank 0, after the timed region)
    check, check_detail = None, None
    if rank == 0 and not args.no_check:
        if args.server != "none":
            check_detail = {"skipped": "the fused server step writes params, not the mean"}
        else:
            phase(rank, "check the result against the oracle (sampled columns)")
            exact = nshard != world or not sharded  # one fold, or rank 0's share in a rehearsal
            edges = [p0 for p0, _ in fd.bucket_edges(P, buckets)[1:]] if sharded else []
            check, check_detail = check_result(
                final if (final is not None and not exact) else out, K=K, P=P, k0=k0, k1=k1, weights=weights,
                W=W, dtype=dtype, exact=exact, nranks=nshard, edges=edges, reference_bf16=args.reference_bf16,
                f32_mean=out if (final is not None and not exact) else None)
            check_detail["wall_s"] = round(time.perf_counter() - t1, 2)
            log(f"[bench rank 0] check: {check} {check_detail}")

    e2e = None
    if not args.no_e2e and args.server == "none" and not args.with_norms:
        phase(rank, "e2e: host-resident deltas (pinned H2D + fold [+ reduce] + D2H)")
        ns = Kl if (sharded or args.e2e) else min(Kl, E2E_SAMPLE_CLIENTS)
        e2e = host_resident_rate(x[:ns], w_local, step if sharded else None, out, scale, nt, dev, rank, sharded,
                                 K * P * esize if (sharded and nshard == world) else ns * P * esize)
        if not sharded:
            e2e["e2e_sample"] = (f"the first {ns} of the {Kl} clients ({ns * P * esize / 1e9:.2f} GB)"
                                 if ns < Kl else f"all {Kl} clients ({ns * P * esize / 1e9:.2f} GB)")

    traffic = (None, None)
    if rank == 0 and not sharded and not args.with_norms and args.server == "none" and not args.variant \
            and not args.clients:
        traffic = (measure_traffic(args.workload, args.traffic_out or None) if args.measure_traffic
                   else load_traffic(args.workload))
    if rank == 0:
        value = (K if nshard == world else Kl) * P * esize * args.steps / elapsed / 1e9
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "ranks": world,
            "rccl_ranks": world if (sharded and args.backend == "nccl" and nshard == world) else 0,
            "launcher": os.environ.get("FJ_BENCH_LAUNCHER",
                                       "torch.distributed.run" if "WORLD_SIZE" in os.environ else "direct"),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "host_issue_ms_per_step": round(t_issue / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
            "data": "synthetic: counter-hash client deltas 0.01*u[-1,1), integer weights in [1,500]",
            "config": {"workload": desc, "clients": K, "params": P, "clients_per_gpu": Kl,
                       "parallelism": f"client-sharded x{nshard}" + (
                           f" + {'RCCL' if args.backend == 'nccl' else args.backend} "
                           f"{collective}" if sharded else "") + (
                           " (REHEARSAL: one GPU runs rank 0's share, RCCL world 1)" if nshard != world else ""),
                       "buckets": (buckets if isinstance(buckets, int) else fd.bucket_name(buckets))
                       if sharded else 1,
                       "exchange_engine": engine if sharded else None,
                       "exchange_collective": collective if sharded else None,
                       "exchange_autotune_ms": {k: round(t, 4) for k, t in tune.items()} or None,
                       "weights_path": {k: v for k, v in kernels.HOST_WEIGHT_PATHS.items() if v} or "device tensor",
                       "nontemporal": nt,
                       "variant": args.variant, "fused_l2_norms": bool(args.with_norms),
                       "bf16_arithmetic": ("reference (every op rounded to bf16)" if args.reference_bf16 else
                                           "f32 fold, one rounding") if dtype == torch.bfloat16 else None,
                       "fused_server_step": args.server},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4),
                         "traffic": traffic[0], "traffic_source": traffic[1],
                         "kernel": ("k_dense_opt fold + server " + args.server if args.server != "none" else
                                    "k_dense_l2 fold + per-client l2" if args.with_norms else "k_dense weighted fold"),
                         "bytes_per_launch": bytes_per_launch,
                         "mean_launch_ms": round(mean_kernel_s * 1e3, 4)},
        }
        res["check"] = check
        res["check_detail"] = check_detail
        if e2e is not None:
            res.update(e2e)
        if nshard != world:
            res["rehearsal_projected_whole_job_GBs"] = round(value * nshard, 2)
        if (not sharded and not args.no_dropin and args.workload == "c3" and not args.clients
                and args.server == "none" and not args.with_norms):
            res["drop_in"] = dropin_surface(dev)
        if not sharded and not args.no_cpu_baseline and dtype == torch.float32:
            res["cpu_baseline"] = cpu_baseline(K)
        emit_json(json_fd, res)
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if sharded:
        dist.destroy_process_group()
    phase(rank, "done")
    if watchdog is not None:
        watchdog.cancel()
    if check == "FAILED":
        log("bench: the timed result does NOT match the oracle (check_detail in the JSON line)")
        raise SystemExit(3)


def single_process(args):
    """``--single-process``: one process folds each GPU's client share and sums the
    partials with one grouped RCCL reduce per bucket (include/fjcomm.h,
    fjcomm_multi_wsum_dense). Strong scaling over the same 1024 x 4 Mi workload."""
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    from fedjax_amd import distributed as fd, kernels, tree_util as tu

    N = args.gpus
    if torch.cuda.device_count() < N:
        raise SystemExit(f"--single-process --gpus {N}: only {torch.cuda.device_count()} GPUs visible")
    K, P, dtype, desc = WORKLOADS[args.workload]
    if args.clients:
        K = args.clients
    esize = torch.empty((), dtype=dtype).element_size()
    weights = fedavg_weights(K)
    W = 0.0
    for w in weights:
        W += w
    devs = [torch.device("cuda", d) for d in range(N)]
    xs, ws = [], []
    for d, dev in enumerate(devs):
        k0, k1 = fd.shard_range(K, d, N)
        vw = 16 // esize
        x = torch.empty(k1 - k0, (P + vw - 1) // vw * vw, dtype=dtype, device=dev)[:, :P]
        kernels.fill_synth(x, seed=0, k0=k0)
        xs.append(x)
        ws.append(weights[k0:k1])
    comm = fd.MultiDeviceCommunicator(devs)
    outs = [torch.empty(P, dtype=torch.float32, device=dev) for dev in devs]
    buckets = (tuple(float(v) for v in args.buckets.split(":")) if ":" in args.buckets
               else int(args.buckets)) or 1

    def sync():
        for dev in devs:
            torch.cuda.synchronize(dev)

    def step():  # the round's weights on the host, per device (kernel arguments of the folds)
        fd.multi_device_weighted_mean(xs, [np.float32(w) for w in ws], W, comm=comm, buckets=buckets, outs=outs,
                                      all_devices=args.all_ranks)

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    comm.close()
    check, check_detail = None, None
    if not args.no_check:  # device 0's mean over all K clients vs the oracle, after the timed region
        check, check_detail = check_result(outs[0], K=K, P=P, k0=0, k1=K, weights=weights, W=W, dtype=dtype,
                                           exact=False, nranks=N,
                                           edges=[p0 for p0, _ in fd.bucket_edges(P, buckets)[1:]])
    res = {"metric": METRIC, "value": round(K * P * esize * args.steps / elapsed / 1e9, 2), "unit": "GB/s",
           "n_gpus": N, "ranks": 1, "rccl_ranks": N, "launcher": "single process (fjcomm_init_all)",
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
           "data": "synthetic: counter-hash client deltas 0.01*u[-1,1), integer weights in [1,500]",
           "config": {"workload": desc, "clients": K, "params": P,
                      "parallelism": f"client-sharded x{N}, one process, grouped RCCL "
                                     f"{'all_reduce' if args.all_ranks else 'reduce'}",
                      "buckets": fd.bucket_name(buckets)},
           "check": check, "check_detail": check_detail}
    emit_json(json_fd, res)
    if check == "FAILED":
        raise SystemExit(3)


if __name__ == "__main__":
    main()
