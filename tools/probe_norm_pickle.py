"""Exploration: do lazy norm views survive pickle / torch.save / copy.deepcopy (client
diagnostics sent to a logging process or saved with a checkpoint)? Prints one JSON line."""
import copy
import io
import json
import os
import pickle
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import tree_util as tu  # noqa: E402

dev = torch.device("cuda:0")
g0 = torch.Generator(device=dev).manual_seed(1)
xs = [{"u": torch.rand(5000, device=dev, generator=g0), "v": torch.rand(33, 9, device=dev, generator=g0)}
      for _ in range(4)]
res = {}
for kind in ("example", "library"):
    if kind == "example":
        diag = {i: {"delta_l2_norm": tu.tree_l2_norm(x)} for i, x in enumerate(xs)}
        tu.tree_mean([(x, 1) for x in xs])
    else:
        s, diag = tu.tree_zeros_like(xs[0]), {}
        for i, x in enumerate(xs):
            s = tu.tree_add(s, tu.tree_weight(x, i + 1))
            diag[i] = {"delta_l2_norm": tu.tree_l2_norm(x)}
        tu.tree_inverse_weight(s, 10.0)
    want = [float(diag[i]["delta_l2_norm"]) for i in range(4)]
    for how, fn in (("pickle", lambda d: pickle.loads(pickle.dumps(d))),
                    ("torch.save", lambda d: torch.load(io.BytesIO(_save(d)), weights_only=False)),
                    ("deepcopy", copy.deepcopy), ("copy", lambda d: {k: copy.copy(v) for k, v in d.items()})):
        def _save(d):
            b = io.BytesIO()
            torch.save(d, b)
            return b.getvalue()
        try:
            got = fn(diag)
            vals = [float(got[i]["delta_l2_norm"]) for i in range(4)]
            res[f"{kind}_{how}"] = {"ok": vals == want, "type": type(got[0]["delta_l2_norm"]).__name__}
        except Exception as e:  # noqa: BLE001
            res[f"{kind}_{how}"] = {"error": f"{type(e).__name__}: {e}"[:200]}
print(json.dumps(res))
