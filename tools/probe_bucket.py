"""Fold time of one parameter bucket of a sharded step: K client rows of a [K, 4 Mi]
f32 slab (row stride 16 MB), columns [0, n), for several bucket widths and kernel
variants, with the library FJAGG_LIB points to. Prints one JSON line.

usage (GPU box): FJAGG_LIB=... python tools/probe_bucket.py TAG [K]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedjax_amd import _lib, kernels  # noqa: E402


def main(tag, K):
    if tag == "base":
        _lib._SIGNATURES.pop("fjcomm_sharded_wsum_dense_edges", None)
    dev = torch.device("cuda:0")
    P = 4 * 1024 * 1024
    x = torch.empty(K, P, device=dev)
    kernels.fill_synth(x, seed=0)
    w = torch.rand(K, device=dev)
    out = torch.empty(P, device=dev)
    res = {"lib": tag, "K": K}
    for n in (1 << 20, 1 << 21, 3 << 20, 1 << 22):
        for v in ((0, 5, 12, 13) if tag == "base" else (0, 5, 12, 13, 16, 17)):
            f = lambda: kernels.weighted_sum_dense(x[:, :n], w, scale=0.5, out=out[:n], nontemporal=True,
                                                   variant=v)
            for _ in range(3):
                f()
            e0, e1 = kernels.Event(), kernels.Event()
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            ms = e0.elapsed_time(e1) / 20
            res[f"{n >> 10}Ki_v{v}"] = round(K * n * 4 / ms / 1e6, 1)
    del x
    # configs[1] as a padded slab (one contiguous row per client)
    n = 1206590
    x = torch.empty(K, 1206592, device=dev)[:, :n]
    kernels.fill_synth(x, seed=0)
    for v in (0, 5, 12, 13, 16, 17):
        if v >= 16 and tag == "base":
            continue
        f = lambda: kernels.weighted_sum_dense(x, w, scale=0.5, out=out[:n], nontemporal=True, variant=v)
        for _ in range(3):
            f()
        e0, e1 = kernels.Event(), kernels.Event()
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        res[f"c1slab_v{v}"] = round(K * n * 4 / (e0.elapsed_time(e1) / 20) / 1e6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 128)
