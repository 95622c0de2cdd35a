"""Numpy restatement of the FedAvg plumbing around the aggregation path (test
infrastructure): the client SGD loop of examples/fed_avg.py:86-95 and
fedjax/algorithms/fed_avg.py (via create_train_for_each_client), with the
aggregation delegated to a ``tree_util`` module — the oracle's or fedjax_amd's.

Client training is NOT on the path (SURVEY.md §3 hot loop #1); it is restated
only so the reference's integration known-answer tests
(examples/fed_avg_test.py:52-56, fedjax/algorithms/fed_avg_test.py:57-61) can pin
the aggregation inside a real round.
"""

import numpy as np


def shuffle_repeat_batch_indices(n, batch_size, num_epochs=1, seed=None):
    """fedjax/core/client_datasets.py:478-537 (ShuffleRepeatBatchView.__iter__)."""
    num_steps = (n * num_epochs + batch_size - 1) // batch_size
    buf = np.arange(n, dtype=np.int32)
    i = n
    rng = np.random.RandomState(seed)
    for _ in range(num_steps):
        indices = np.zeros((batch_size,), dtype=np.int32)
        filled = 0
        while filled < batch_size:
            available = n - i
            if available == 0:
                rng.shuffle(buf)
                i = 0
                available = n
            used = min(available, batch_size - filled)
            indices[filled:filled + used] = buf[i:i + used]
            i += used
            filled += used
        yield indices


def client_update(server_params, x, batch_size, num_epochs, seed):
    """examples/fed_avg.py:86-95 with the test's grad_fn (fed_avg_test.py:27-29,
    l / sum(batch['x'])) and sgd(learning_rate=1.0)."""
    params = {k: np.asarray(v, np.float32) for k, v in server_params.items()}
    for idx in shuffle_repeat_batch_indices(len(x), batch_size, num_epochs, seed):
        s = np.sum(x[idx], dtype=np.float32)
        grads = {k: v / s for k, v in params.items()}
        params = {k: v + (np.float32(-1.0) * grads[k]) for k, v in params.items()}
    return {k: server_params[k] - params[k] for k in params}


def fed_avg_example_round(tu, to_leaf, to_numpy, server_params, clients, batch_size, num_epochs, seed):
    """examples/fed_avg.py:64-84: list of (delta, len) -> tree_mean -> sgd server step."""
    pairs, norms = [], {}
    for cid, x in clients:
        delta = client_update(server_params, x, batch_size, num_epochs, seed)
        dl = {k: to_leaf(v) for k, v in delta.items()}
        pairs.append((dl, len(x)))
        norms[cid] = float(to_numpy(tu.tree_l2_norm(dl)))
    mean = tu.tree_mean(pairs)
    new = {k: server_params[k] + np.float32(-1.0) * to_numpy(mean[k]) for k in server_params}
    return new, norms


def fed_avg_library_round(tu, to_leaf, to_numpy, server_params, clients, batch_size, num_epochs, seed):
    """fedjax/algorithms/fed_avg.py:120-148: running weighted sum (zeros_like, add(weight)),
    then tree_inverse_weight."""
    s = tu.tree_zeros_like({k: to_leaf(v) for k, v in server_params.items()})
    num_examples_sum = 0.0
    norms = {}
    for cid, x in clients:
        delta = client_update(server_params, x, batch_size, num_epochs, seed)
        dl = {k: to_leaf(v) for k, v in delta.items()}
        s = tu.tree_add(s, tu.tree_weight(dl, len(x)))
        num_examples_sum += len(x)
        norms[cid] = float(to_numpy(tu.tree_l2_norm(dl)))
    mean = tu.tree_inverse_weight(s, num_examples_sum)
    new = {k: server_params[k] + np.float32(-1.0) * to_numpy(mean[k]) for k in server_params}
    return new, norms


# The reference's integration KATs: (name, round fn, batch_size, num_epochs, params, norms)
KATS = [
    ("examples/fed_avg_test.py:52-56", fed_avg_example_round, 2, 2,
     [0., 1.4425802, 2.8851604], {b"cid0": 1.7553135, b"cid1": 0.48310122}),
    ("fedjax/algorithms/fed_avg_test.py:57-61", fed_avg_library_round, 2, 1,
     [0., 1.5655555, 3.131111], {b"cid0": 1.4534444262, b"cid1": 0.2484521282}),
]
SERVER_PARAMS = {"w": np.array([0., 2., 4.], np.float32)}
CLIENTS = [(b"cid0", np.array([2., 4., 6.], np.float32)), (b"cid1", np.array([8., 10.], np.float32))]
