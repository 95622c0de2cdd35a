"""Numpy restatement of the client steps of the other FedJAX algorithms whose server
side is the running-sum path (test infrastructure, like tests/fedavg_restated.py):

* FedProx            fedjax/algorithms/fed_prox.py:43-151, KAT fed_prox_test.py:36-65
* Mime               fedjax/algorithms/mime.py:42-211,     KAT mime_test.py:38-63
* Mime Lite          fedjax/algorithms/mime_lite.py:45-170, KATs mime_lite_test.py:38-66, :92-119
* AgnosticFedAvg     fedjax/algorithms/agnostic_fed_avg.py:39-311, KAT agnostic_fed_avg_test.py:34-78
* APFL               fedjax/algorithms/apfl.py:88-231,     KAT apfl_test.py:50-98
* stateful FedAvg    examples/stateful_fed_avg.py:139-186, KAT stateful_fed_avg_test.py:46-67
* HypCluster         fedjax/algorithms/hyp_cluster.py:89-301, KATs hyp_cluster_test.py:366-403, :405-472
  (one running sum per cluster, interleaved)

Client training (the gradients, the client SGD steps, the domain statistics) is NOT on
the aggregation path; it is restated in float32 numpy, following JAX's reverse-mode
order for these linear losses, only so that the reference's known-answer values pin the
aggregation calls of a real round. Every aggregation call — ``tree_zeros_like``,
``tree_add(s, tree_weight(delta, w))``, ``tree_inverse_weight``, ``tree_sum``,
``tree_l2_norm``, ``tree_clip_by_global_norm`` — goes through the ``tu`` module passed
in: the oracle (oracle/tree_util_ref.py) on the CPU, ``fedjax_amd.tree_util`` on the
GPU. ``to_leaf`` turns a host array into that module's leaf, ``to_weight`` turns a
0-d float32/int32 array weight (a jnp array in the reference) into that module's
strongly typed scalar, ``to_numpy`` reads a leaf or 0-d result back.
"""

import numpy as np

from tests.fedavg_restated import shuffle_repeat_batch_indices

F = np.float32


def padded_batches(x, batch_size, extra=None):
    """fedjax/core/client_datasets.py:448-459 (PaddedBatchView, one batch-size bucket):
    sequential batches, the final one zero-padded with a False mask."""
    n = len(x)
    for start in range(0, n, batch_size):
        stop = min(start + batch_size, n)
        xb = np.zeros(batch_size, F)
        xb[:stop - start] = x[start:stop]
        mask = np.zeros(batch_size, bool)
        mask[:stop - start] = True
        out = {"x": xb, "__mask__": mask}
        if extra is not None:
            e = np.zeros(batch_size, extra.dtype)
            e[:stop - start] = extra[start:stop]
            out["domain_id"] = e
        yield out


def shuffled_batches(x, batch_size, num_epochs, seed, extra=None):
    """client_datasets.py:478-536 (ShuffleRepeatBatchView), via fedavg_restated."""
    for idx in shuffle_repeat_batch_indices(len(x), batch_size, num_epochs, seed):
        yield (x[idx], None if extra is None else extra[idx])


def _sum_seq(v):
    s = F(0)
    first = True
    for a in np.asarray(v, F):
        s = a if first else F(s + a)
        first = False
    return s


def grad_mean_linear(x):
    """d/dw of jnp.mean(x * w) (models.py:537-549, unpadded): the mean's cotangent
    f32(1/n) per example, then the broadcast's reduce_sum of ct * x."""
    ct = F(F(1) / F(len(x)))
    return _sum_seq(np.asarray(x, F) * ct)


def grad_masked_linear(x, mask):
    """d/dw of safe_div(vdot(x * w, mask), sum(mask)) (models.py:539-542)."""
    num = int(np.sum(mask))
    ct = F(F(1) / F(num)) if num else F(0)
    return _sum_seq(np.asarray(x, F) * (mask.astype(F) * ct))


def sgd_step(w, g, lr=1.0):
    """optax.sgd: u = -lr * g, p + u (fedjax/core/optimizers.py:227-250)."""
    return F(w + F(F(-lr) * g))


def _leaf_tree(to_leaf, w):
    return {"w": to_leaf(np.asarray(w, F).reshape(()))}


def _w(tree, to_numpy):
    return F(to_numpy(tree["w"]))


# ------------------------------------------------------------------------- FedProx
def fed_prox_round(tu, to_leaf, to_numpy, to_weight, proximal_weight=0.01):
    """fed_prox.py:115-143 with fed_prox_test.py:27-31's loss x * w, client and server
    sgd(1.0), ShuffleRepeatBatchHParams(batch_size=2, num_epochs=1, seed=0)."""
    s = F(4.0)
    clients = [(b"cid0", np.array([2., 4., 6.], F)), (b"cid1", np.array([8., 10.], F))]
    c = F(0.5 * proximal_weight)  # 0.5 * proximal_weight (Python) times an f32 array: weak
    delta_sum = tu.tree_zeros_like(_leaf_tree(to_leaf, s))
    num_examples_sum = 0.0
    norms = {}
    for cid, x in clients:
        w = s
        for xb, _ in shuffled_batches(x, 2, 1, 0):
            d = F(s - w)
            # grad of mean(x*w + c*l2sq(s - w)): sum 0.5*x_i, plus the proximal term's
            # cotangent 2*(c*d) through d = s - w (negated)
            g = F(grad_mean_linear(xb) + F(-F(F(c * d) * F(2))))
            w = sgd_step(w, g)
        delta = _leaf_tree(to_leaf, F(s - w))
        delta_sum = tu.tree_add(delta_sum, tu.tree_weight(delta, len(x)))
        num_examples_sum += len(x)
        norms[cid] = F(to_numpy(tu.tree_l2_norm(delta)))
    mean = tu.tree_inverse_weight(delta_sum, num_examples_sum)
    m = _w(mean, to_numpy)
    return {"params": sgd_step(s, m), "mean_delta": m, "norms": norms}


# ---------------------------------------------------------------------------- Mime
def _mime_server_grads(tu, to_leaf, to_numpy, to_weight, s, clients, batch_size):
    """mime.py:42-74 (create_grads_for_each_client) + :169-174: per client
    grads_sum = tree_add(tree_weight(grads, num), grads_sum) over padded batches, then
    tree_sum of (grads_sum, num_sum) over clients and tree_inverse_weight."""
    outs = []
    for cid, x in clients:
        grads_sum = tu.tree_zeros_like(_leaf_tree(to_leaf, s))
        num_sum = 0.0
        for b in padded_batches(x, batch_size):
            g = grad_masked_linear(b["x"], b["__mask__"])
            num = np.int32(np.sum(b["__mask__"]))  # jnp.sum of a bool mask: int32
            grads_sum = tu.tree_add(tu.tree_weight(_leaf_tree(to_leaf, g), to_weight(num)), grads_sum)
            num_sum = num_sum + F(num)  # 0. + int32 array -> float32
        outs.append((grads_sum, to_weight(F(num_sum))))
    grads_sum_total, num_sum_total = tu.tree_sum(outs)
    return tu.tree_inverse_weight(grads_sum_total, num_sum_total)


def mime_round(tu, to_leaf, to_numpy, to_weight, server_learning_rate=0.2):
    """mime.py:163-211 with mime_test.py:28-30's loss, sgd(1.0), train batches of 2
    (1 epoch, seed 0), grads batches PaddedBatchHParams(batch_size=2)."""
    s = F(4.0)
    clients = [(b"cid0", np.array([2., 4., 6.], F)), (b"cid1", np.array([8., 10.], F))]
    server_grads = _mime_server_grads(tu, to_leaf, to_numpy, to_weight, s, clients, 2)
    c = _w(server_grads, to_numpy)
    delta_sum = tu.tree_zeros_like(_leaf_tree(to_leaf, s))
    num_examples_sum = 0.0
    norms = {}
    for cid, x in clients:
        w = s
        for xb, _ in shuffled_batches(x, 2, 1, 0):
            cc = grad_mean_linear(xb)  # grad at init params (mime.py:92-93)
            g = grad_mean_linear(xb)  # grad at params: the loss is linear, same value
            w = sgd_step(w, F(F(g - cc) + c))  # g - cc + c (mime.py:95-97)
        delta = _leaf_tree(to_leaf, F(s - w))
        delta_sum = tu.tree_add(delta_sum, tu.tree_weight(delta, len(x)))
        num_examples_sum += len(x)
        norms[cid] = F(to_numpy(tu.tree_l2_norm(delta)))
    mean = tu.tree_inverse_weight(delta_sum, num_examples_sum)
    m = _w(mean, to_numpy)
    return {"params": F(s - F(F(server_learning_rate) * m)), "mean_delta": m, "norms": norms,
            "server_grads": c}


# ----------------------------------------------------------------------- Mime Lite
def mime_lite_round(tu, to_leaf, to_numpy, to_weight, server_learning_rate=0.2, client_delta_clip_norm=None):
    """mime_lite.py:114-170 with mime_lite_test.py:28-30's loss, sgd(1.0), train batches
    of 2 (1 epoch, seed 0), grads batches of 2; optional client delta clipping (:137-144)."""
    s = F(4.0)
    clients = [(b"cid0", np.array([0.2, 0.4, 0.6], F)), (b"cid1", np.array([0.8, 0.1], F))]
    delta_sum = tu.tree_zeros_like(_leaf_tree(to_leaf, s))
    num_examples_sum = 0.0
    norms, clipped = {}, {}
    for cid, x in clients:
        w = s
        for xb, _ in shuffled_batches(x, 2, 1, 0):
            w = sgd_step(w, grad_mean_linear(xb))
        delta = _leaf_tree(to_leaf, F(s - w))
        norms[cid] = F(to_numpy(tu.tree_l2_norm(delta)))
        if client_delta_clip_norm is not None:
            delta = tu.tree_clip_by_global_norm(delta, client_delta_clip_norm)
            clipped[cid] = F(to_numpy(tu.tree_l2_norm(delta)))
        delta_sum = tu.tree_add(delta_sum, tu.tree_weight(delta, len(x)))
        num_examples_sum += len(x)
    mean = tu.tree_inverse_weight(delta_sum, num_examples_sum)
    m = _w(mean, to_numpy)
    server_grads = _mime_server_grads(tu, to_leaf, to_numpy, to_weight, s, clients, 2)
    return {"params": F(s - F(F(server_learning_rate) * m)), "mean_delta": m, "norms": norms,
            "clipped_norms": clipped, "server_grads": _w(server_grads, to_numpy)}


def mime_lite_clip_round(tu, to_leaf, to_numpy, to_weight):
    return mime_lite_round(tu, to_leaf, to_numpy, to_weight, client_delta_clip_norm=0.5)


# ------------------------------------------------------------------ AgnosticFedAvg
def _segment_sum(v, ids, n):
    out = np.zeros(n, F)
    for a, i in zip(np.asarray(v, F), ids):
        out[i] = F(out[i] + a)
    return out


def agnostic_fed_avg_round(tu, to_leaf, to_numpy, to_weight):
    """agnostic_fed_avg.py:252-311 with agnostic_fed_avg_test.py:34-78's setup: loss x*w,
    client sgd(1.0), server sgd(0.1), train batches of 3 (1 epoch, seed 0), domain
    batches PaddedBatchHParams(3), domain weights [.1,.2,.3,.4], window 2 of [1,2,3,4],
    'eg' with domain learning rate 0.01. The client weights are the float32 arrays
    beta (:282-285), so W = 0. + beta_0 + beta_1 is float32 (SURVEY A4's array branch)."""
    s = F(4.0)
    nd = 4
    domain_weights = np.array([0.1, 0.2, 0.3, 0.4], F)
    window = [np.array([1., 2., 3., 4.], F)] * 2
    clients = [(b"cid0", np.array([1., 2., 4., 3., 6., 1.], F), np.array([1, 0, 0, 0, 2, 2], np.int32)),
               (b"cid1", np.array([8., 10., 5.], F), np.array([1, 3, 1], np.int32))]
    mean_window = np.zeros(nd, F)
    for wv in window:
        mean_window = F(mean_window + wv)
    mean_window = F(mean_window / F(len(window)))
    alpha = F(domain_weights / mean_window)
    metrics = {}
    for cid, x, dom in clients:  # create_domain_metrics_for_each_client (:39-81)
        dl, dn = np.zeros(nd, F), np.zeros(nd, F)
        for b in padded_batches(x, 3, dom):
            mask = b["__mask__"].astype(F)
            dl = F(dl + _segment_sum(F(F(b["x"] * s) * mask), b["domain_id"], nd))
            dn = F(dn + _segment_sum(mask, b["domain_id"], nd))
        metrics[cid] = {"domain_loss": dl, "domain_num": dn, "beta": _sum_seq(F(alpha * dn))}
    delta_sum = tu.tree_zeros_like(_leaf_tree(to_leaf, s))
    weight_sum = 0.0
    norms = {}
    for cid, x, dom in clients:  # create_train_for_each_client (:105-144)
        beta = metrics[cid]["beta"]
        w = s
        for xb, db in shuffled_batches(x, 3, 1, 0, dom):
            ct = F(F(1) / beta)  # jnp.sum(alpha * dsl) / beta: the division's cotangent
            per_domain = F(alpha * ct)
            g = _sum_seq(F(xb * per_domain[db]))
            w = sgd_step(w, g)
        delta = _leaf_tree(to_leaf, F(s - w))
        weight = to_weight(beta)
        delta_sum = tu.tree_add(delta_sum, tu.tree_weight(delta, weight))
        weight_sum = weight_sum + weight  # 0. + f32 array -> float32
        norms[cid] = F(to_numpy(tu.tree_l2_norm(delta)))
    mean = tu.tree_inverse_weight(delta_sum, weight_sum)
    m = _w(mean, to_numpy)
    sum_loss = tu.tree_sum(to_leaf(metrics[c]["domain_loss"]) for c, _, _ in clients)
    sum_num = tu.tree_sum(to_leaf(metrics[c]["domain_num"]) for c, _, _ in clients)
    sum_loss, sum_num = np.asarray(to_numpy(sum_loss), F), np.asarray(to_numpy(sum_num), F)
    with np.errstate(divide="ignore", invalid="ignore"):  # util.safe_div
        mean_loss = np.where(sum_num != 0, sum_loss / np.where(sum_num != 0, sum_num, F(1)), F(0)).astype(F)
    nw = F(domain_weights * np.exp(F(F(0.01) * mean_loss)))  # update_domain_weights 'eg' (:147-160)
    nw = np.maximum(nw, np.zeros_like(nw))
    nw = F(nw / _sum_seq(nw))
    return {"params": sgd_step(s, m, lr=0.1), "mean_delta": m, "norms": norms,
            "domain_weights": nw, "domain_window": [window[1], sum_num],
            "betas": {c: metrics[c]["beta"] for c, _, _ in clients}}


# ---------------------------------------------------------------------------- APFL
def apfl_round(tu, to_leaf, to_numpy, to_weight, client_coefficient=0.5):
    """apfl.py:185-231 with apfl_test.py:28-31's grad_fn (l / sum(batch['x'])), client and
    server sgd(1.0), batches of 2 (1 epoch, seed 0), client_coefficient 0.5. Each client
    trains the server track, its own params and the interpolation coefficient
    (create_train_for_each_client, :88-154); the running sum takes the server track's delta."""
    from tests.fedavg_restated import CLIENTS, SERVER_PARAMS
    s0 = np.asarray(SERVER_PARAMS["w"], F)
    delta_sum = tu.tree_zeros_like({"w": to_leaf(s0)})
    num_examples_sum = 0.0
    norms, cparams, coefs = {}, {}, {}
    for cid, x in CLIENTS:
        s, c, a = s0.copy(), s0.copy(), 0.5  # client_default_state: params, coefficient (Python float)
        for idx in shuffle_repeat_batch_indices(len(x), 2, 1, 0):
            S = np.sum(x[idx], dtype=F)
            p = (F(a) * c + F(1 - a) * s).astype(F)  # interpolate_params: a * b + (1 - a) * c
            sg, cg = (s / S).astype(F), (p / S).astype(F)
            ig = F(np.tensordot((c - s).astype(F), cg, axes=1))  # interpolation_grad_fn
            s = (s + F(-1.0) * sg).astype(F)
            c = (c + F(-1.0) * cg).astype(F)
            a = np.clip(F(F(a) + F(-1.0) * ig), 0, 1)
        delta = {"w": to_leaf((s0 - s).astype(F))}
        delta_sum = tu.tree_add(delta_sum, tu.tree_weight(delta, len(x)))
        num_examples_sum += len(x)
        norms[cid] = F(to_numpy(tu.tree_l2_norm(delta)))
        cparams[cid], coefs[cid] = c, np.asarray([a], F)
    mean = np.asarray(to_numpy(tu.tree_inverse_weight(delta_sum, num_examples_sum)["w"]), F)
    return {"params": (s0 + F(-1.0) * mean).astype(F), "mean_delta": mean, "norms": norms,
            "client_params": cparams, "client_coefficients": coefs}


# ------------------------------------------------------------- stateful FedAvg example
def stateful_fed_avg_round(tu, to_leaf, to_numpy, to_weight):
    """examples/stateful_fed_avg.py:139-186: FedAvg's client update with a per-client step
    counter (client state; not aggregated) and the same running sum (stateful_fed_avg_test.py
    :46-67, grad_fn l / sum(batch['x']), batches of 2, 1 epoch, seed 0)."""
    from tests.fedavg_restated import CLIENTS, SERVER_PARAMS, fed_avg_library_round
    new, norms = fed_avg_library_round(tu, to_leaf, to_numpy, SERVER_PARAMS, CLIENTS, 2, 1, 0)
    steps = {cid: len(list(shuffle_repeat_batch_indices(len(x), 2, 1, 0))) for cid, x in CLIENTS}
    return {"params": np.asarray(new["w"], F), "norms": {k: F(v) for k, v in norms.items()}, "num_steps": steps}


# --------------------------------------------------------------------------- HypCluster
_HC_CLIENTS = [(b"0", np.array([1.1], F)), (b"1", np.array([0.9, 0.9], F)), (b"2", np.array([-1.1], F)),
               (b"3", np.array([-0.9, -0.9, -0.9], F))]


def _hc_delta(p, x, lr=0.5, epochs=5):
    """ClientDeltaTrainer (hyp_cluster.py:200-210) with models.grad of jnp.square(params - x),
    sgd(lr), batches of 1 for `epochs` epochs: initial params - final params. (The test's
    clients repeat one value, so the unseeded shuffle order does not matter.)"""
    w = F(p)
    for _ in range(epochs * len(x)):
        for xi in x[:1]:
            g = F(F(2) * F(w - xi))  # integer_pow's jvp: 2 * z, times the mean's cotangent 1.0
            w = F(w + F(F(-lr) * g))
    return F(F(p) - w)


def _hc_expectation(tu, to_leaf, to_numpy, cluster_params, ids, clients):
    """hyp_cluster.expectation_step (hyp_cluster.py:268-301): one running sum per cluster,
    the clients' tree_add calls interleaved across the sums; None for a cluster no client
    chose."""
    sums = [tu.tree_zeros_like(to_leaf(np.asarray(p, F))) for p in cluster_params]
    nsum = [0 for _ in cluster_params]
    for cid, x in clients:
        cl = ids[cid]
        d = _hc_delta(cluster_params[cl], x)
        sums[cl] = tu.tree_add(sums[cl], tu.tree_weight(to_leaf(np.asarray(d, F)), len(x)))
        nsum[cl] += len(x)
    return [F(to_numpy(tu.tree_inverse_weight(s, n))) if n > 0 else None for s, n in zip(sums, nsum)]


def hyp_cluster_expectation_round(tu, to_leaf, to_numpy, to_weight):
    """hyp_cluster_test.py:366-403: three clusters [1, -1, 3.14], clients 0, 1, 4 in cluster
    0 and 2, 3 in cluster 1, none in cluster 2."""
    clients = _HC_CLIENTS + [(b"4", np.array([-0.1], F))]
    ids = {b"0": 0, b"1": 0, b"2": 1, b"3": 1, b"4": 0}
    deltas = _hc_expectation(tu, to_leaf, to_numpy, [1., -1., 3.14], ids, clients)
    return {"cluster_deltas": deltas[:2], "empty_cluster": deltas[2]}


def hyp_cluster_round(tu, to_leaf, to_numpy, to_weight):
    """hyp_cluster.py:89-128 with hyp_cluster_test.py:405-472's setup: clusters [1, -1], the
    maximization step's assignment (argmin over clusters of the mean loss (p - x)^2, regularizer
    0; hyp_cluster.py:224-260), the expectation step's running sums, then sgd(0.25) per cluster."""
    params = [F(1.), F(-1.)]
    ids = {}
    for cid, x in _HC_CLIENTS:
        losses = [np.mean(np.square((F(p) - x).astype(F)), dtype=F) for p in params]
        ids[cid] = int(np.argmin(losses))
    deltas = _hc_expectation(tu, to_leaf, to_numpy, params, ids, _HC_CLIENTS)
    new = [p if d is None else F(p + F(F(-0.25) * d)) for p, d in zip(params, deltas)]
    return {"cluster_params": new, "cluster_ids": ids}


# The reference's KATs: (name, round fn, {result key: expected}); npt.assert_allclose's
# default rtol (1e-7) is the reference's tolerance for every value listed, unless the
# reference's test gives one: (value, rtol).
KATS = [
    ("fedjax/algorithms/fed_prox_test.py:62-65", fed_prox_round,
     {"params": -3.77, "norms": {b"cid0": 6.95, b"cid1": 9.}}),
    ("fedjax/algorithms/mime_test.py:60-63", mime_round,
     {"params": 2.08, "norms": {b"cid0": 12., b"cid1": 6.}}),
    ("fedjax/algorithms/mime_lite_test.py:61-66", mime_lite_round,
     {"params": 3.8799999, "norms": {b"cid0": 0.70000005, b"cid1": 0.45000005}}),
    ("fedjax/algorithms/mime_lite_test.py:113-119", mime_lite_clip_round,
     {"params": 3.904, "clipped_norms": {b"cid0": 0.5, b"cid1": 0.45000005}}),
    ("fedjax/algorithms/agnostic_fed_avg_test.py:69-78", agnostic_fed_avg_round,
     {"params": 3.5555556, "norms": {b"cid0": 2.8333335, b"cid1": 7.666667},
      "domain_weights": [0.08702461, 0.18604803, 0.2663479, 0.46057943],
      "domain_window": [[1., 2., 3., 4.], [3., 3., 2., 1.]]}),
    ("fedjax/algorithms/apfl_test.py:77-98", apfl_round,
     {"params": [0., 1.5655555, 3.131111], "norms": {b"cid0": 1.4534444262, b"cid1": 0.2484521282},
      "client_params": {b"cid0": [0., 1.35, 2.7], b"cid1": [0., 1.888889, 3.777778]},
      "client_coefficients": {b"cid0": [0.5], b"cid1": [0.5]}}),
    ("examples/stateful_fed_avg_test.py:57-64", stateful_fed_avg_round,
     {"params": [0., 1.5655555, 3.131111], "norms": {b"cid0": 1.4534444262, b"cid1": 0.2484521282},
      "num_steps": {b"cid0": 2, b"cid1": 1}}),
    ("fedjax/algorithms/hyp_cluster_test.py:393-403", hyp_cluster_expectation_round,
     {"cluster_deltas": [(-0.1 + 0.1 * 2 + 1.1) / 4, ((0.1 - 0.1 * 3) / 4, 1e-6)]}),
    ("fedjax/algorithms/hyp_cluster_test.py:452-472", hyp_cluster_round,
     {"cluster_params": [1. - 0.25 * 0.1 / 3, -1. + 0.25 * 0.2 / 4],
      "cluster_ids": {b"0": 0, b"1": 0, b"2": 1, b"3": 1}}),
]


def check_kat(name, got, want, rtol=1e-7):
    """npt.assert_allclose of every listed value at the reference's tolerance (an entry
    (value, rtol) carries the reference test's own rtol)."""
    import numpy.testing as npt

    def close(g, e, msg):
        e, r = e if isinstance(e, tuple) else (e, rtol)
        npt.assert_allclose(np.asarray(g, np.float64), e, rtol=r, err_msg=msg)

    for key, v in want.items():
        if isinstance(v, dict):
            for cid, e in v.items():
                close(got[key][cid], e, f"{name} {key} {cid!r}")
        elif isinstance(v, list) and any(isinstance(e, tuple) for e in v):
            assert len(got[key]) == len(v), (name, key)
            for i, e in enumerate(v):
                close(got[key][i], e, f"{name} {key}[{i}]")
        else:
            close(got[key], v, f"{name} {key}")
