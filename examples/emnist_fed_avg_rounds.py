"""FedAvg rounds with FedJAX's EMNIST setup on the MI355X aggregation path.

Mirrors the round structure of the reference's examples/emnist_fed_avg.py:32-98 and
examples/fed_avg.py:64-101 for the part this project owns:
  * 10 clients per round (emnist_fed_avg.py:66-67), each contributing a delta with
    the EMNIST-CNN parameter tree (fedjax/models/emnist.py:59-72, 1,206,590 params)
    and weight len(client_dataset) (fed_avg.py:76);
  * per-client delta_l2_norm diagnostics (fed_avg.py:79-81);
  * tree_mean of the deltas (fed_avg.py:82);
  * the server Adam step, lr=10**-2.5, b1=0.9, b2=0.999, eps=10**-4
    (emnist_fed_avg.py:52-54).
Client training is JAX autodiff in the reference and out of scope here: synthetic
deltas stand in for it (no datasets are downloadable in this environment).

Three equivalent paths are run each round and checked against each other:
  A. the reference surface: mean_aggregator().apply over per-client pytrees, then the
     server step on the mean;
  B. the fused slab path: ClientDeltaSlab + fjagg_server_update_dense (one kernel for
     mean + Adam) and the norms from the same pass;
  C. the library algorithm's loop written literally (fedjax/algorithms/fed_avg.py:132-146:
     tree_zeros_like, tree_add(s, tree_weight(delta, n)), tree_l2_norm(delta),
     tree_inverse_weight) through fedjax_amd.tree_util — deferred into one fold.
     Its mean is a running sum from zeros, which equals A's tree_mean bit for bit.

usage: python examples/emnist_fed_avg_rounds.py [rounds]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

import fedjax_amd
from fedjax_amd import kernels, server, tree_util

# fedjax/models/emnist.py:59-72 (haiku names; jax flatten order sorts them)
EMNIST_CNN = {"conv2_d": {"b": (32,), "w": (3, 3, 1, 32)}, "conv2_d_1": {"b": (64,), "w": (3, 3, 32, 64)},
              "linear": {"b": (128,), "w": (9216, 128)}, "linear_1": {"b": (62,), "w": (128, 62)}}


def tmap(f, t):
    return {k: tmap(f, v) for k, v in t.items()} if isinstance(t, dict) else f(t)


def run(rounds=5, clients_per_round=10, seed=0, verbose=True):
    dev = torch.device("cuda", torch.cuda.current_device())
    template = tmap(lambda s: np.zeros(s, np.float32), EMNIST_CNN)
    slab = fedjax_amd.ClientDeltaSlab(template, clients_per_round, device=dev)
    P = slab.num_params
    assert P == 1206590  # fedjax/models/emnist_test.py:45
    opt = server.adam(learning_rate=10 ** -2.5, b1=0.9, b2=0.999, eps=10 ** -4)
    params_a = torch.zeros(P, device=dev)  # path A server params (flat, slab leaf order)
    params_b = params_a.clone()  # path B
    state_b = opt.init(params_b)
    m_a, v_a = torch.zeros(P, device=dev), torch.zeros(P, device=dev)
    rs = np.random.RandomState(seed)
    agg = fedjax_amd.aggregators.mean_aggregator()
    agg_state = agg.init()
    history = []
    for rnd in range(1, rounds + 1):
        # stand-in for client_update: deltas written straight into the slab rows
        slab.fill_synthetic(seed=seed * 1000 + rnd)
        weights = [int(n) for n in rs.randint(10, 400, size=clients_per_round)]  # len(client_dataset)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # A: reference surface
        clients = [(b"c%d" % k, slab.client(k), weights[k]) for k in range(clients_per_round)]
        norms_a = tree_util.tree_l2_norms([c for _, c, _ in clients])
        mean_tree, agg_state = agg.apply(clients, agg_state)
        mean_flat = torch.cat([x.reshape(-1) for x in fedjax_amd.pytree.leaves_of(mean_tree)])
        # server step on the mean (same kernel family: a K=1 fold of the mean with weight 1)
        one = fedjax_amd.ClientDeltaSlab({"g": np.zeros(P, np.float32)}, 1, device=dev)
        one.rows[0].copy_(mean_flat)
        state_a = {"count": rnd - 1, "m": m_a, "v": v_a}
        server.fused_mean_update(one, [1], opt, params_a, state_a)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        # B: fused slab path (norms from the fold's pass, mean + Adam in one kernel)
        mean_b = torch.empty(P, device=dev)
        _, norms_b = slab.mean(weights, with_norms=True)
        state_b = server.fused_mean_update(slab, weights, opt, params_b, state_b, mean_out=mean_b)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        # C: the library FedAvg loop, literally
        s = tree_util.tree_zeros_like(slab.client(0))
        n_sum, norms_c = 0., []
        for k in range(clients_per_round):
            delta = slab.client(k)
            s = tree_util.tree_add(s, tree_util.tree_weight(delta, weights[k]))
            n_sum += weights[k]
            norms_c.append(tree_util.tree_l2_norm(delta))
        mean_c = tree_util.tree_inverse_weight(s, n_sum)
        mean_c_flat = torch.cat([x.reshape(-1) for x in fedjax_amd.pytree.leaves_of(mean_c)])
        norms_c = torch.stack(norms_c)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        same_mean = torch.equal(mean_b.view(torch.int32), mean_flat.view(torch.int32))
        same_mean_c = torch.equal(mean_c_flat.view(torch.int32), mean_flat.view(torch.int32))
        norm_rel_c = float(((norms_a - norms_c).abs() / norms_a).max())
        same_params = torch.equal(params_a.view(torch.int32), params_b.view(torch.int32))
        norm_rel = float(((norms_a - norms_b).abs() / norms_a).max())
        history.append({"round": rnd, "same_mean": same_mean, "same_params": same_params,
                        "same_mean_library_loop": same_mean_c, "norm_rel_diff": norm_rel,
                        "norm_rel_diff_library_loop": norm_rel_c, "ms_reference_surface": (t1 - t0) * 1e3,
                        "ms_fused": (t2 - t1) * 1e3, "ms_library_loop": (t3 - t2) * 1e3})
        if verbose:
            print(f"[round {rnd}] mean bitwise={same_mean} params bitwise={same_params} "
                  f"library loop mean bitwise={same_mean_c} norm rel diff={max(norm_rel, norm_rel_c):.1e}  "
                  f"surface {1e3 * (t1 - t0):.2f} ms  fused {1e3 * (t2 - t1):.2f} ms  "
                  f"library loop {1e3 * (t3 - t2):.2f} ms")
    return history


if __name__ == "__main__":
    run(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
