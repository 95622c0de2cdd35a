"""cProfile of one configs[1] round through aggregators.RunningMean (B = 128: every
client buffered, one fold at result()): where the host time over tree_mean goes.
Prints the top functions by own time."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import fedjax_amd
from fedjax_amd import aggregators
from tools.time_running_mean import SHAPES, tmap


def main(K=128, rounds=200):
    dev = torch.device("cuda:0")
    template = tmap(lambda s: np.zeros(s, np.float32), SHAPES)
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=dev).fill_synthetic(seed=0)
    clients = [tmap(lambda v: v.clone(), slab.client(k)) for k in range(K)]
    weights = np.random.RandomState(1).randint(1, 501, size=K).tolist()

    def rnd():
        rm = aggregators.RunningMean(clients[0], buffer_clients=K, device=dev)
        for c, w in zip(clients, weights):
            rm.add(c, w)
        return rm.result()

    for _ in range(5):
        rnd()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(rounds):
        rnd()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
