import os, sys, json, time
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import bench
from fedjax_amd import tree_util as tu
dev = torch.device("cuda:0")
for f in (0.0, 0.25, 0.0, 0.25):
    tu._PIPELINE_FRAC = f
    tu._mean_config()  # (the builtin tree_mean keeps its own copy)
    r = bench.dropin_surface(dev)
    print(json.dumps({"frac": f, **{k: v for k, v in r.items() if k.startswith("c1")}}), flush=True)
