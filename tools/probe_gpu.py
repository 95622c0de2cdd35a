"""Quick GPU probe: parity of every dense variant vs the numpy oracle on a small
shape, then per-variant bandwidth on the 1024 x 4M f32 slab (hip events).

usage (GPU box): python tools/probe_gpu.py [--big]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from fedjax_amd import kernels
from oracle import tree_util_ref as ref


def parity():
    dev = torch.device("cuda:0")
    for K, P in [(37, 10007), (1, 5), (3, 4), (130, 4096 * 3 + 3)]:
        x = torch.empty(K, P, dtype=torch.float32, device=dev)
        kernels.fill_synth(x, seed=7)
        xh = ref.synth(K, P, seed=7)
        assert np.array_equal(x.cpu().numpy().view(np.uint32), xh.view(np.uint32)), "synth mismatch"
        wi = ref.fedavg_weights(K)
        w = torch.tensor(wi.astype(np.float32), device=dev)
        r = ref.mean_scale([int(v) for v in wi])
        want = ref.wsum_dense(xh, wi.astype(np.float32), scale=r)
        for v in range(8):
            for nt in (False, True):
                y = kernels.weighted_sum_dense(x, w, scale=float(r), variant=v, nontemporal=nt)
                g = y.cpu().numpy()
                ok = np.array_equal(g.view(np.uint32), want.view(np.uint32))
                print(f"parity K={K} P={P} variant={v} nt={nt}: {'OK' if ok else 'MISMATCH'}", flush=True)
                if not ok:
                    bad = np.nonzero(g != want)[0]
                    print("   first bad", bad[:5], g[bad[:5]], want[bad[:5]])
        y = kernels.weighted_sum_dense(x, w, scale=float(r), mode="split")
        err = np.max(np.abs(y.cpu().numpy() - want))
        print(f"split K={K} P={P}: max abs err {err:.3e}", flush=True)


def bench(K=1024, P=4 * 1024 * 1024, reps=10):
    dev = torch.device("cuda:0")
    x = torch.empty(K, P, dtype=torch.float32, device=dev)
    kernels.fill_synth(x, seed=0)
    w = torch.tensor(ref.fedavg_weights(K).astype(np.float32), device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    nbytes = K * P * 4
    res = {}
    for rnd in range(3):
        for v in range(8):
            for nt in (False, True):
                kernels.weighted_sum_dense(x, w, scale=0.001, out=out, variant=v, nontemporal=nt)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    kernels.weighted_sum_dense(x, w, scale=0.001, out=out, variant=v, nontemporal=nt)
                e.record()
                e.synchronize()
                ms = s.elapsed_time(e) / reps
                res.setdefault((v, nt), []).append(nbytes / ms / 1e6)
    for (v, nt), gbs in sorted(res.items()):
        print(f"K={K} P={P} variant={v} nt={nt}: GB/s " + " ".join(f"{g:.0f}" for g in gbs), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    parity()
    bench()
    if "--big" in sys.argv:
        bench(K=128, P=1206590)
    print("total s", time.time() - t0)
