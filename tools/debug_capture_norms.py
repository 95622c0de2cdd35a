"""Debug: six standalone lazy norms captured into a graph (default settings), replayed on new
contents; per replay, which captured norms equal the norms of the new contents computed alone.
Prints one JSON line per replay."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedjax_amd import pytree, tree_util as tu  # noqa: E402

dev = torch.device("cuda:0")
H = tu._HOST
g0 = torch.Generator(device=dev).manual_seed(9)
xs = [{"u": torch.rand(5000, device=dev, generator=g0), "v": torch.rand(33, 9, device=dev, generator=g0)}
      for _ in range(6)]


def bits(v):
    return int(v.detach().reshape(()).view(torch.int32).item())


mode = sys.argv[1] if len(sys.argv) > 1 else "norms"
[tu.tree_l2_norm(x) for x in xs]
tu.tree_mean([(x, 1) for x in xs])
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    torch.cuda.synchronize()
    before = H.solo_info()
    with torch.cuda.graph(g, stream=st):
        norms = [tu.tree_l2_norm(x) for x in xs]
    after = H.solo_info()
print(json.dumps({"eager_launches": after["eager_launches"] - before["eager_launches"],
                  "eager": after["eager"] - before["eager"], "pending": after["pending"],
                  "columns": [int(v._ticket._idx) if hasattr(v, "_ticket") and v._ticket is not None else None
                              for v in norms]}))
for rep in range(3):
    with torch.no_grad():
        for x in xs:
            for leaf in pytree.leaves_of(x):
                leaf.copy_(torch.rand(leaf.shape, device=dev, generator=g0))
    g.replay()
    torch.cuda.synchronize()
    want = [bits(tu.tree_l2_norm(x)) for x in xs]
    got = [bits(v) for v in norms]
    print(json.dumps({"replay": rep, "equal": [a == b for a, b in zip(got, want)]}))
