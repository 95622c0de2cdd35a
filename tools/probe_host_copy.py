"""Host side of DeltaIngestor.put: how fast does a 16 MiB client row reach a pinned
staging row? torch copy_ at several thread counts, and the pinned H2D DMA of one row."""
import json
import os
import time

import numpy as np
import torch

P = 4 * 1024 * 1024
src = [np.random.RandomState(i).standard_normal(P).astype(np.float32) for i in range(4)]
dst = torch.empty(P * 4, dtype=torch.uint8).pin_memory()
res = {"cpus_affinity": len(os.sched_getaffinity(0)), "omp": os.environ.get("OMP_NUM_THREADS"),
       "torch_threads": torch.get_num_threads()}


def rate(fn, n=40):
    fn(0)
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    return round(n * P * 4 / (time.perf_counter() - t0) / 1e9, 2)


for th in (1, 4, 8, 16, 32):
    torch.set_num_threads(th)
    res[f"torch_copy_t{th}"] = rate(lambda i: dst.copy_(torch.from_numpy(src[i % 4]).view(torch.uint8)))
res["np_copyto"] = rate(lambda i: np.copyto(dst.numpy(), src[i % 4].view(np.uint8)))
dev = torch.device("cuda:0")
d = torch.empty(P * 4, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()


def h2d(i):
    d.copy_(dst, non_blocking=True)
    torch.cuda.synchronize()


res["h2d_one_row"] = rate(h2d)
print(json.dumps(res))
