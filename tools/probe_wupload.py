"""What does the per-round weight upload cost in front of the configs[1] fold?
A: fold only; B: pinned 512-B H2D + fold (bench/slab today); C: a tiny kernel + fold
(stand-in for passing the weights as kernel arguments). ms per step, 200 steps."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedjax_amd import kernels  # noqa: E402

dev = torch.device("cuda:0")
K, P = 128, 1206590
x = torch.empty(K, 1206592, device=dev)[:, :P]
kernels.fill_synth(x, seed=0)
w_np = np.float32(np.random.RandomState(1).randint(1, 501, size=K))
wd = torch.from_numpy(w_np).to(dev)
out = torch.empty(P, device=dev)


def fold(w):
    kernels.weighted_sum_dense(x, w, scale=1e-4, out=out, nontemporal=True)


def A():
    fold(wd)


def B():
    fold(torch.from_numpy(w_np).pin_memory().to(dev, non_blocking=True))


def C():
    wd.fill_(1.0)
    fold(wd)


res = {}
for r in range(2):
    for name, f in (("A_fold_only", A), ("B_pinned_h2d", B), ("C_tiny_kernel", C)):
        for _ in range(20):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            f()
        torch.cuda.synchronize()
        res[f"{name}_{r}"] = round((time.perf_counter() - t0) / 200 * 1e3, 4)
print(json.dumps(res))
