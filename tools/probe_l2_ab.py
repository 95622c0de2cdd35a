"""Fused-norm folds against the plain folds, same inputs, same box:

* pytree: fjagg_wsum_l2_ptrs vs fjagg_wsum_ptrs over configs[1]'s 128 clients x EMNIST-CNN
  (separate leaf allocations), and over the 64-client chunk an early flush folds;
* dense: fjagg_wsum_l2_dense vs fjagg_wsum_dense at configs[1] as a slab and configs[2].

Device-uploaded plan images, HIP events on the stream around `calls` launches, interleaved
plain / l2 passes (median of `passes`). Two fused variants: "l2" = the norm combine in the
fold's last workgroup (FJAGG_ZEROED_WS workspace, the library's default), "l2_two_launch" =
the separate k_l2_combine launch (a caller's workspace). The means must be bitwise equal to
the plain fold's and the two variants' norms bitwise equal to each other; the norms are
compared with float64 norms of the same inputs (max relative error). One JSON line per case.
usage: python tools/probe_l2_ab.py [calls] [passes]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import _lib, kernels

SHAPES = [(32,), (3, 3, 1, 32), (64,), (3, 3, 32, 64), (128,), (9216, 128), (62,), (128, 62)]
F32, SCALE, NONTEMPORAL, ZEROED_WS = 0, 1, 4, 128  # include/fjagg.h


def timed(go, calls, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(calls):
        go()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / calls * 1e3


def pytree_case(K, calls, passes, dev, stream, lib):
    L = len(SHAPES)
    leaves = []
    for k in range(K):
        row = []
        for l, shp in enumerate(SHAPES):
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=l + 1, k0=k)
            row.append(x)
        leaves.append(row)
    leaf_n = np.array([int(np.prod(s)) for s in SHAPES], dtype=np.int64)
    outs = [torch.empty(n, dtype=torch.float32, device=dev) for n in leaf_n]
    nb = lib.fjagg_ptrs_plan_leaves(F32, 0, leaf_n.ctypes.data, None, L, None, 0)
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(F32, 0, leaf_n.ctypes.data, None, L, blocks.ctypes.data, nb)
    in_ptrs = np.array([[x.data_ptr() for x in r] for r in leaves], dtype=np.int64).ravel()
    out_ptrs = np.array([o.data_ptr() for o in outs], dtype=np.int64)
    img = torch.from_numpy(np.concatenate([in_ptrs, out_ptrs, leaf_n, blocks])).to(dev)
    w = torch.tensor(np.random.RandomState(1).randint(1, 501, size=K), dtype=torch.float32, device=dev)
    l2 = torch.empty(K, dtype=torch.float32, device=dev)
    l2b = torch.empty(K, dtype=torch.float32, device=dev)
    ws = torch.zeros(max(1, lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)), dtype=torch.uint8, device=dev)
    ws2 = torch.empty_like(ws)
    s = ctypes.c_void_p(stream.cuda_stream)
    plain = lambda: lib.fjagg_wsum_ptrs(F32, F32, F32, img.data_ptr(), L, K, nb, w.data_ptr(), ctypes.c_float(1e-3),
                                        SCALE | NONTEMPORAL, s)
    fused = lambda: lib.fjagg_wsum_l2_ptrs(F32, F32, F32, img.data_ptr(), L, K, nb, w.data_ptr(), ctypes.c_float(1e-3),
                                           l2.data_ptr(), SCALE | NONTEMPORAL | ZEROED_WS, ws.data_ptr(), ws.numel(), s)
    two = lambda: lib.fjagg_wsum_l2_ptrs(F32, F32, F32, img.data_ptr(), L, K, nb, w.data_ptr(), ctypes.c_float(1e-3),
                                         l2b.data_ptr(), SCALE | NONTEMPORAL, ws2.data_ptr(), ws2.numel(), s)
    _lib.check(plain(), "plain")
    torch.cuda.synchronize()
    ref = torch.cat(outs).clone()
    _lib.check(fused(), "l2")
    torch.cuda.synchronize()
    bits_equal = bool(torch.equal(torch.cat(outs).view(torch.int32), ref.view(torch.int32)))
    _lib.check(two(), "l2 two launches")
    torch.cuda.synchronize()
    bits_equal = bits_equal and bool(torch.equal(torch.cat(outs).view(torch.int32), ref.view(torch.int32)))
    want = np.array([sum(float((x.double() ** 2).sum()) for x in r) for r in leaves])
    rel = float(np.max(np.abs(l2.double().cpu().numpy() - want) / want))
    tp, tf, t2 = [], [], []
    for _ in range(3):
        plain(), fused(), two()
    torch.cuda.synchronize()
    for _ in range(passes):
        tp.append(timed(plain, calls, stream))
        tf.append(timed(fused, calls, stream))
        t2.append(timed(two, calls, stream))
    norms_equal = bool(torch.equal(l2.view(torch.int32), l2b.view(torch.int32)))
    counter_zero = int(ws[:16].count_nonzero()) == 0
    p, f, f2 = float(np.median(tp)), float(np.median(tf)), float(np.median(t2))
    return {"case": f"pytree configs[1] K={K}", "workgroups": int(nb), "plain_us": round(p, 2), "l2_us": round(f, 2),
            "l2_over_plain": round(f / p, 4), "l2_two_launch_us": round(f2, 2),
            "l2_two_launch_over_plain": round(f2 / p, 4), "mean_bits_equal": bits_equal,
            "norms_bits_equal_two_launch": norms_equal, "counter_left_zero": counter_zero,
            "norm_max_rel_err_vs_f64": rel}


def dense_case(K, P, calls, passes, dev, stream):
    x = torch.empty(K, (P + 3) // 4 * 4, dtype=torch.float32, device=dev)[:, :P]
    kernels.fill_synth(x, seed=0)
    w = torch.tensor(np.random.RandomState(1).randint(1, 501, size=K), dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    l2 = torch.empty(K, dtype=torch.float32, device=dev)
    l2b = torch.empty(K, dtype=torch.float32, device=dev)
    need = int(_lib.load().fjagg_wsum_l2_workspace_bytes(K, P))
    ws = torch.empty(max(need, 4), dtype=torch.uint8, device=dev)
    nt = K * P * 4 >= (256 << 20)
    plain = lambda: kernels.weighted_sum_dense(x, w, scale=1e-3, out=out, nontemporal=nt)
    fused = lambda: kernels.weighted_sum_l2_dense(x, w, scale=1e-3, out=out, l2sq=l2, nontemporal=nt)
    two = lambda: kernels.weighted_sum_l2_dense(x, w, scale=1e-3, out=out, l2sq=l2b, nontemporal=nt, workspace=ws)
    plain()
    torch.cuda.synchronize()
    ref = out.clone()
    fused()
    torch.cuda.synchronize()
    bits_equal = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
    two()
    torch.cuda.synchronize()
    bits_equal = bits_equal and bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
    norms_equal = bool(torch.equal(l2.view(torch.int32), l2b.view(torch.int32)))
    kk = min(K, 64)  # norms of the first 64 clients, from float64 sums of their rows
    want = (x[:kk].double() ** 2).sum(1).cpu().numpy()
    rel = float(np.max(np.abs(l2[:kk].double().cpu().numpy() - want) / want))
    for _ in range(2):
        plain(), fused(), two()
    torch.cuda.synchronize()
    tp, tf, t2 = [], [], []
    for _ in range(passes):
        tp.append(timed(plain, calls, stream))
        tf.append(timed(fused, calls, stream))
        t2.append(timed(two, calls, stream))
    p, f, f2 = float(np.median(tp)), float(np.median(tf)), float(np.median(t2))
    del x
    return {"case": f"dense {K}x{P}", "plain_us": round(p, 2), "l2_us": round(f, 2), "l2_over_plain": round(f / p, 4),
            "l2_two_launch_us": round(f2, 2), "l2_two_launch_over_plain": round(f2 / p, 4),
            "plain_GBs": round(K * P * 4 / p / 1e3, 1), "l2_GBs": round(K * P * 4 / f / 1e3, 1),
            "mean_bits_equal": bits_equal, "norms_bits_equal_two_launch": norms_equal,
            "norm_max_rel_err_vs_f64_first64": rel}


def main(calls=50, passes=5):
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    lib = _lib.load()
    for K in (128, 64):
        print(json.dumps(pytree_case(K, calls, passes, dev, stream, lib)), flush=True)
        torch.cuda.empty_cache()
    print(json.dumps(dense_case(128, 1206590, calls, passes, dev, stream)), flush=True)
    torch.cuda.empty_cache()
    print(json.dumps(dense_case(1024, 4 * 1024 * 1024, max(5, calls // 10), passes, dev, stream)), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
