"""bench.dropin_surface's library-loop round under two early-flush thresholds of the deferred
sum (tree_util.set_deferred_sums(flush_bytes=...)), interleaved, one process."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

import bench
from fedjax_amd import tree_util as tu

dev = torch.device("cuda:0")
for fb in (1 << 30, 256 << 20, 1 << 30, 256 << 20):
    tu.set_deferred_sums(True, flush_bytes=fb)
    r = bench.dropin_surface(dev)
    print(json.dumps({"flush_bytes": fb, **{k: v for k, v in r.items() if k.startswith("c1")}}), flush=True)
