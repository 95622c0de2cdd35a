"""Where the per-client tree_l2_norm adds time to the configs[1] running-sum round
(fedjax/algorithms/fed_avg.py:132-146 with its delta_l2_norm): the synchronised round
  plain      tree_add(s, tree_weight(x, n)) x K + tree_inverse_weight
  norms      + tree_l2_norm(x) per client, the views left unread
  read       + one torch.stack(norms).cpu() after the round (as bench tools read them)
  read_each  + float(v) for every view after the round
  *_1g       the same without the early flush (flush_bytes 1 GiB)
and the host time of each phase. Prints one JSON line. usage: python tools/time_norms_loop.py [rounds]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import kernels, tree_util as tu

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tree(k, dev):
    out, seed = {}, 1
    for mod, leaves in SHAPES.items():
        out[mod] = {}
        for name, shp in leaves.items():
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=seed, k0=k)
            out[mod][name] = x.view(shp)
            seed += 1
    return out


def main(rounds=30, K=128):
    dev = torch.device("cuda:0")
    pairs = list(zip([tree(k, dev) for k in range(K)], np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    W = float(sum(w for _, w in pairs))
    pc = time.perf_counter
    res = {}
    for rep in range(2):
        for mode in ("plain", "norms", "read", "read_each", "norms_1g", "read_1g"):
            tu.set_deferred_sums(True, flush_bytes=(1 << 30) if mode.endswith("_1g") else tu.DEFERRED_SUM_DEFAULTS["flush_bytes"])
            walls, loop_us, fold_us, read_us = [], [], [], []
            for r in range(rounds + 3):
                torch.cuda.synchronize()
                t0 = pc()
                s, norms = tu.tree_zeros_like(pairs[0][0]), []
                for t, w in pairs:
                    s = tu.tree_add(s, tu.tree_weight(t, w))
                    if mode != "plain":
                        norms.append(tu.tree_l2_norm(t))
                t1 = pc()
                m = tu.tree_inverse_weight(s, W)
                t2 = pc()
                if mode.startswith("read") and mode != "read_each":
                    torch.stack(norms).cpu()
                elif mode == "read_each":
                    [float(v) for v in norms]
                t3 = pc()
                torch.cuda.synchronize()
                t4 = pc()
                if r >= 3:
                    walls.append((t4 - t0) * 1e3)
                    loop_us.append((t1 - t0) * 1e6)
                    fold_us.append((t2 - t1) * 1e6)
                    read_us.append((t3 - t2) * 1e6)
            med = lambda v: round(float(np.median(v)), 3)
            res.setdefault(mode, []).append({"round_sync_ms": med(walls), "loop_us": med(loop_us),
                                             "fold_call_us": med(fold_us), "read_us": med(read_us)})
            del s, m, norms
    tu.set_deferred_sums(True, **tu.DEFERRED_SUM_DEFAULTS)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
