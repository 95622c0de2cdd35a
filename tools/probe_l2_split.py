"""Fused-norm pytree fold (fjagg_wsum_l2_ptrs) vs the plain fold (fjagg_wsum_ptrs) at configs[1]
(128 clients x EMNIST-CNN, separate leaf allocations) with the library's plan and with every
non-tail workgroup range split into s pieces (more, shorter workgroups): is the fused-norm
fold short of waves per CU? Device-uploaded images (no kernel-argument path), HIP events on
the stream around `calls` launches. Prints one JSON line per split.
usage: python tools/probe_l2_split.py [calls]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import _lib, kernels

SHAPES = [(32,), (3, 3, 1, 32), (64,), (3, 3, 32, 64), (128,), (9216, 128), (62,), (128, 62)]
F32, SCALE, NONTEMPORAL = 0, 1, 4  # fjagg.h (tree_mean passes NONTEMPORAL for jobs >= 256 MiB)


def split(blocks, s):
    out = []
    for i in range(0, len(blocks), 2):
        w0, u1 = int(blocks[i]), int(blocks[i + 1])
        tail = (w0 >> 62) & 1
        u0 = w0 & ((1 << 40) - 1)
        if tail or s == 1 or u1 - u0 < s:
            out += [w0, u1]
            continue
        hi = w0 & ~((1 << 40) - 1)
        edges = [u0 + (u1 - u0) * j // s for j in range(s + 1)]
        for a, b in zip(edges[:-1], edges[1:]):
            out += [hi | a, b]
    return np.array(out, dtype=np.int64)


def main(calls=50, K=128):
    dev = torch.device("cuda:0")
    lib = _lib.load()
    leaves = []
    for k in range(K):
        row = []
        for l, shp in enumerate(SHAPES):
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=l + 1, k0=k)
            row.append(x)
        leaves.append(row)
    L = len(SHAPES)
    leaf_n = np.array([int(np.prod(s)) for s in SHAPES], dtype=np.int64)
    outs = [torch.empty(n, dtype=torch.float32, device=dev) for n in leaf_n]
    nb = lib.fjagg_ptrs_plan_leaves(F32, 0, leaf_n.ctypes.data, None, L, None, 0)
    base = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(F32, 0, leaf_n.ctypes.data, None, L, base.ctypes.data, nb)
    in_ptrs = np.array([[x.data_ptr() for x in r] for r in leaves], dtype=np.int64).ravel()
    out_ptrs = np.array([o.data_ptr() for o in outs], dtype=np.int64)
    w = torch.tensor(np.random.RandomState(1).randint(1, 501, size=K), dtype=torch.float32, device=dev)
    l2 = torch.empty(K, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    # the same clients through tree_mean (plan image in the kernel arguments), same box
    from fedjax_amd import tree_util as tu
    pairs = list(zip(leaves, w.cpu().numpy().astype(int).tolist()))
    for _ in range(5):
        tu.tree_mean(pairs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(calls):
        tu.tree_mean(pairs)
    e1.record(stream)
    torch.cuda.synchronize()
    print(json.dumps({"tree_mean_karg_us_per_call": round(e0.elapsed_time(e1) / calls * 1e3, 2)}), flush=True)
    ref_out, ref_l2 = None, None
    for s in (1, 2, 3, 4):
        blocks = split(base, s)
        n = len(blocks) // 2
        img = torch.from_numpy(np.concatenate([in_ptrs, out_ptrs, leaf_n, blocks])).to(dev)
        ws = torch.empty(max(1, lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, n)), dtype=torch.uint8, device=dev)
        res = {"split": s, "workgroups": n}
        for name in ("plain", "l2"):
            def go():
                if name == "plain":
                    return lib.fjagg_wsum_ptrs(F32, F32, F32, img.data_ptr(), L, K, n, w.data_ptr(),
                                               ctypes.c_float(1e-3), SCALE | NONTEMPORAL, ctypes.c_void_p(stream.cuda_stream))
                return lib.fjagg_wsum_l2_ptrs(F32, F32, F32, img.data_ptr(), L, K, n, w.data_ptr(),
                                              ctypes.c_float(1e-3), l2.data_ptr(), SCALE | NONTEMPORAL, ws.data_ptr(), ws.numel(),
                                              ctypes.c_void_p(stream.cuda_stream))
            for _ in range(5):
                _lib.check(go(), name)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(calls):
                go()
            e1.record(stream)
            torch.cuda.synchronize()
            res[f"{name}_us"] = round(e0.elapsed_time(e1) / calls * 1e3, 2)
            got = torch.cat(outs).cpu().numpy().view(np.uint32)
            if ref_out is None:
                ref_out = got
            res[f"{name}_mean_bits_equal"] = bool(np.array_equal(got, ref_out))
        g2 = l2.cpu().numpy()
        ref_l2 = g2 if ref_l2 is None else ref_l2
        res["l2_max_rel_diff_vs_split1"] = float(np.max(np.abs(g2 - ref_l2) / np.maximum(np.abs(ref_l2), 1e-30)))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
