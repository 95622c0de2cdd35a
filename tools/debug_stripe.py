"""Probe k_dense_stripe (variants 20/21/22) with structured inputs; prints mismatch summaries."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import kernels

dev = torch.device("cuda:0")
for variant, C, TT in ((20, 64, 192), (21, 32, 384), (22, 16, 768)):
    for K in (TT, 2 * TT, 3 * TT + 5, 16384):
        P = 4 * C
        # 1) ones: every column must be K
        x = torch.ones(K, P, device=dev)
        w = torch.ones(K, device=dev)
        y = kernels.weighted_sum_dense(x, w, variant=variant).cpu().numpy()
        ok1 = np.all(y == K)
        # 2) one selected client k*: y[c] = x[k*][c] = 1000 * (k* % 1000) + c
        res = []
        for ks in (0, 1, 3, 4, 5, 17, TT - 1, TT, K - 1):
            if ks >= K:
                continue
            kk = torch.arange(K, device=dev, dtype=torch.float32)[:, None]
            cc = torch.arange(P, device=dev, dtype=torch.float32)[None, :]
            x = (kk % 1000) * 1000 + cc
            w = torch.zeros(K, device=dev)
            w[ks] = 1
            y = kernels.weighted_sum_dense(x, w, variant=variant).cpu().numpy()
            want = (ks % 1000) * 1000 + np.arange(P)
            bad = np.flatnonzero(y != want)
            if bad.size:
                res.append((ks, bad.size, [(int(b), float(y[b]), float(want[b])) for b in bad[:4]]))
        print(f"C={C} K={K}: ones {'ok' if ok1 else 'BAD ' + str(np.unique(y)[:8])}; select: {res or 'ok'}", flush=True)
