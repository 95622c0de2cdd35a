"""Host time of one compression round's apply() (GPU idle before the call, no sync inside the timing): if it is close to the round's GPU time, the round is host-bound. Prints one JSON line per aggregator."""
import sys, time, json
sys.path.insert(0, '.')
import numpy as np, torch
import fedjax_amd
from fedjax_amd import random
from fedjax_amd.aggregators import compression as comp
EMNIST = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}
def tmap(f, t): return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)
dev = torch.device("cuda", 0)
K = 128
slab = fedjax_amd.ClientDeltaSlab(tmap(lambda s: np.zeros(s, np.float32), EMNIST), K, device=dev).fill_synthetic(seed=0)
w = [int(x) for x in np.random.RandomState(1).randint(1, 500, K)]
clients = [(b"c%d" % k, slab.client(k), w[k]) for k in range(K)]
for name, mk in [("uniform", lambda: comp.uniform_stochastic_quantizer(16, random.PRNGKey(0))),
                 ("terngrad", lambda: comp.terngrad_quantizer(random.PRNGKey(0))),
                 ("rotated", lambda: comp.rotated_uniform_stochastic_quantizer(16, random.PRNGKey(0))),
                 ("drive", lambda: comp.structured_drive_quantizer(random.PRNGKey(0)))]:
    agg = mk(); st = agg.init()
    for _ in range(3): _, st = agg.apply(clients, st)
    torch.cuda.synchronize()
    # host issue: apply calls with the GPU idle before each (so no back-pressure)
    hs = []
    for _ in range(10):
        torch.cuda.synchronize(); t0 = time.perf_counter(); _, st = agg.apply(clients, st); hs.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(json.dumps({"aggregator": name, "host_issue_ms": round(1e3 * float(np.median(hs)), 3)}))
