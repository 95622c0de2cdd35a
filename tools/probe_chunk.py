"""Does folding the client axis in <= C GB chunks (f32 running sum, ACCUMULATE)
recover bandwidth on >32 GB slabs? Prints JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fedjax_amd import kernels

dev = torch.device("cuda:0")
K, P = int(sys.argv[1]), int(sys.argv[2])
dt = {"f32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3]]
es = torch.empty((), dtype=dt).element_size()
vw = 16 // es
x = torch.empty(K, (P + vw - 1) // vw * vw, dtype=dt, device=dev)[:, :P]
kernels.fill_synth(x, seed=0)
w = torch.rand(K, device=dev)
acc = torch.empty(P, dtype=torch.float32, device=dev)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def run(chunk):
    for k0 in range(0, K, chunk):
        k1 = min(K, k0 + chunk)
        kernels.weighted_sum_dense(x[k0:k1], w[k0:k1], out=acc, accumulate=k0 > 0, nontemporal=True,
                                   scale=0.5 if k1 == K else None)


res = {}
ref = None
for rnd in range(2):
    for chunk in (K, K // 2, K // 4, K // 8, K // 16):
        if chunk < 1:
            continue
        run(chunk)
        s.record()
        for _ in range(2):
            run(chunk)
        e.record()
        e.synchronize()
        res.setdefault(chunk, []).append(K * P * es / (s.elapsed_time(e) / 2 / 1e3) / 1e9)
        if ref is None:
            ref = acc.clone()
        else:
            assert torch.equal(ref.view(torch.int32), acc.view(torch.int32)), "chunked fold not bitwise"
print(json.dumps({"probe": "client_chunks", "K": K, "P": P, "dtype": sys.argv[3],
                  "GBs_by_chunk": {str(k): round(max(v), 1) for k, v in res.items()}}))
