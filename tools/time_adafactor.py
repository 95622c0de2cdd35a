"""Adafactor server step at configs[1]'s model (EMNIST CNN, 1,206,590 params: the 9216 x 128
dense weight is factored, the other leaves are not): milliseconds per apply (the
fjopt_adafactor_step chain alone, inputs resident) and per fused_tree_mean_update over 128
clients (fold + step). Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import server

SHAPES = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
          "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def main(K=128, reps=50):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda s: torch.randn(s, device=dev, generator=g) * 0.01
    clients = [tmap(rnd, SHAPES) for _ in range(K)]
    pairs = list(zip(clients, np.random.RandomState(1).randint(1, 501, size=K).tolist()))
    params = tmap(lambda s: torch.randn(s, device=dev, generator=g), SHAPES)
    res = {}
    for name, opt in (("adafactor", server.adafactor(0.01)),
                      ("adafactor_momentum_wd", server.adafactor(0.01, momentum=0.9, weight_decay_rate=1e-4)),
                      ("adam", server.adam(0.01))):
        st = opt.init(params)
        mean = tmap(rnd, SHAPES)
        if isinstance(opt, server.Adafactor):
            for _ in range(3):
                st, _ = opt.apply(mean, st, params)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                st, _ = opt.apply(mean, st, params)
            torch.cuda.synchronize()
            res[f"{name}_apply_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
        for _ in range(3):
            st = server.fused_tree_mean_update(pairs, opt, params, st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            st = server.fused_tree_mean_update(pairs, opt, params, st)
        torch.cuda.synchronize()
        res[f"{name}_fused_round_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
    print(json.dumps({"workload": "configs[1] server step, 128 clients x EMNIST-CNN", **res}), flush=True)


if __name__ == "__main__":
    main()
