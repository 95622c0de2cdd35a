"""A/B timing of the pytree fold (k_ptrs via tree_mean) and the compression fold
(k_quant_fold via the quantizer aggregators) for the library FJAGG_LIB points to.

configs[1] shapes: 128 clients x EMNIST-CNN (8 leaves, 1,206,590 f32 params), every
(client, leaf) its own device tensor; plus configs[2] as 1024 separate 4 Mi tensors.
HIP events around back-to-back calls on the launch stream; prints one JSON line.

usage (GPU box): FJAGG_LIB=path/to/libfjagg.so python tools/ab_kernels.py [tag]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fedjax_amd  # noqa: E402
from fedjax_amd import _lib, kernels, random, tree_util as tu  # noqa: E402
from fedjax_amd.aggregators import compression as comp  # noqa: E402

EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def per_call_ms(fn, reps, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = kernels.Event(), kernels.Event()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    return e0.elapsed_time(e1) / reps


def main(tag):
    if tag == "base":  # the previous library predates this entry point (not used here)
        _lib._SIGNATURES.pop("fjcomm_sharded_wsum_dense_edges", None)
    dev = torch.device("cuda:0")
    K = 128
    template = tmap(lambda s: np.zeros(s, np.float32), EMNIST)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    P = slab.num_params
    clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
    w = np.random.RandomState(1).randint(1, 501, size=K).tolist()
    pairs = list(zip(clients, w))
    res = {"lib": tag, "lib_path": _lib.LIB_PATH}
    ms = per_call_ms(lambda: tu.tree_mean(pairs), 50)
    res["c1_tree_mean_ms"] = round(ms, 4)
    res["c1_tree_mean_GBs"] = round(K * P * 4 / ms / 1e6, 1)
    trip = [(b"c%d" % k, slab.client(k), w[k]) for k in range(K)]
    for name, make in (("uniform", lambda: comp.uniform_stochastic_quantizer(16, random.PRNGKey(0))),
                       ("terngrad", lambda: comp.terngrad_quantizer(random.PRNGKey(0))),
                       ("uniform_arith",
                        lambda: comp.uniform_stochastic_quantizer(16, random.PRNGKey(0), "arithmetic"))):
        agg = make()
        st = [agg.init()]

        def rnd():
            _, st[0] = agg.apply(trip, st[0])
        res[f"c1_{name}_round_ms"] = round(per_call_ms(rnd, 10), 4)
    del clients, pairs, slab
    torch.cuda.empty_cache()
    Kc, Pc = 1024, 4 * 1024 * 1024
    base = torch.empty(Kc, Pc, device=dev)
    kernels.fill_synth(base, seed=0)
    pairs = [({"w": base[k]}, int(v)) for k, v in enumerate(np.random.RandomState(1).randint(1, 501, size=Kc))]
    ms = per_call_ms(lambda: tu.tree_mean(pairs), 5, warmup=1)
    res["c2_tree_mean_ms"] = round(ms, 4)
    res["c2_tree_mean_GBs"] = round(Kc * Pc * 4 / ms / 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "new")
