"""Interleaved variant x NT sweep of the dense fold (one process, rounds x reps).
usage: python tools/sweep.py K P dtype [rounds] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import kernels

K, P = int(sys.argv[1]), int(sys.argv[2])
dt = {"f32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3]]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
dev = torch.device("cuda:0")
es = torch.empty((), dtype=dt).element_size()
vw = 16 // es
x = torch.empty(K, (P + vw - 1) // vw * vw, dtype=dt, device=dev)[:, :P]
kernels.fill_synth(x, seed=0)
w = torch.rand(K, device=dev)
out = torch.empty(P, dtype=dt, device=dev)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {}
VARIANTS = [int(v) for v in os.environ.get("SWEEP_VARIANTS", ",".join(map(str, range(1, 16)))).split(",")]
for _ in range(rounds):
    for v in VARIANTS:
        for bal in ((True,) if os.environ.get("SWEEP_BALANCED_ONLY") else (False, True)):
            nt = True
            f = lambda: kernels.weighted_sum_dense(x, w, scale=0.5, out=out, nontemporal=nt, variant=v,
                                                   balanced=bal)
            f()
            s.record()
            for _ in range(reps):
                f()
            e.record()
            e.synchronize()
            res.setdefault(f"v{v}_bal{int(bal)}", []).append(K * P * es / (s.elapsed_time(e) / reps / 1e3) / 1e9)
print(json.dumps({"sweep": f"{K}x{P} {sys.argv[3]}", "GBs_median": {k: round(float(np.median(v)), 1) for k, v in res.items()}}))
