"""bench.check_result, the check of the timed output against the oracle (CPU): the host
regenerates the sampled columns of the counter-hash deltas and folds them with the oracle.
Here the "device" result is built on the CPU from the whole slab, so the test also pins that
the sampled regeneration (oracle_synth_cols_f32) is the full generator restricted to columns."""
import numpy as np
import torch

import bench
from tests.coracle import bf16_to_f32


def _full_mean(co, K, P, w, W, bf16=False, seed=0):
    x = co.synth_f32(K, P, seed=seed)
    if bf16:
        x = bf16_to_f32(co.synth_bf16(K, P, seed=seed))
    return x, co.wsum_f32(x, np.float32(w), scale=np.float32(1.0 / W))


def test_synth_cols_is_the_generator_restricted(coracle):
    K, P = 5, 1000
    cols = np.array([0, 3, 17, 998, 999])
    full = coracle.synth_f32(K, P, seed=7, k0=11)
    assert np.array_equal(coracle.synth_cols_f32(K, cols, seed=7, k0=11).view(np.uint32),
                          full[:, cols].view(np.uint32))
    fb = bf16_to_f32(coracle.synth_bf16(K, P, seed=7, k0=11))
    assert np.array_equal(coracle.synth_cols_f32(K, cols, seed=7, k0=11, bf16=True).view(np.uint32),
                          fb[:, cols].view(np.uint32))


def test_exact_check_passes_and_catches_one_flipped_bit(coracle):
    K, P = 40, 9001
    w = [int(v) for v in np.random.RandomState(1).randint(1, 501, size=K)]
    W = float(sum(w))
    _, y = _full_mean(coracle, K, P, w, W)
    st, d = bench.check_result(torch.from_numpy(y), K=K, P=P, k0=0, k1=K, weights=w, W=W, dtype=torch.float32)
    assert st == "bitwise" and d["mismatches"] == 0 and d["columns"] > 1000
    cols = bench.check_cols(P)
    y2 = y.copy()
    y2[cols[5]] = np.nextafter(y2[cols[5]], np.float32(1))
    st, d = bench.check_result(torch.from_numpy(y2), K=K, P=P, k0=0, k1=K, weights=w, W=W, dtype=torch.float32)
    assert st == "FAILED" and d["mismatches"] == 1


def test_exact_check_of_a_rehearsal_share_and_bf16_out(coracle):
    K, P, k0, k1 = 64, 3000, 16, 32
    w = [int(v) for v in np.random.RandomState(2).randint(1, 501, size=K)]
    W = float(sum(w))
    x = coracle.synth_f32(k1 - k0, P, seed=0, k0=k0)
    part = coracle.wsum_f32(x, np.float32(w[k0:k1]), scale=np.float32(1.0 / W))
    st, _ = bench.check_result(torch.from_numpy(part), K=K, P=P, k0=k0, k1=k1, weights=w, W=W,
                               dtype=torch.float32)
    assert st == "bitwise"
    # bf16 deltas, bf16 out: the f32 fold rounded once (RNE)
    xb, yf = _full_mean(coracle, K, P, w, W, bf16=True)
    yb = torch.from_numpy(bench._bf16_bits(yf).view(np.int16)).view(torch.bfloat16)
    st, _ = bench.check_result(yb, K=K, P=P, k0=0, k1=K, weights=w, W=W, dtype=torch.bfloat16)
    assert st == "bitwise"


def test_sharded_check_accepts_a_combined_order_and_rejects_a_wrong_mean(coracle):
    K, P, N = 96, 5000, 4
    w = [int(v) for v in np.random.RandomState(3).randint(1, 501, size=K)]
    W = float(sum(w))
    r = np.float32(1.0 / W)
    x = coracle.synth_f32(K, P, seed=0)
    parts = [coracle.wsum_f32(x[g * 24:(g + 1) * 24], np.float32(w[g * 24:(g + 1) * 24]), scale=r) for g in range(N)]
    y = parts[0]
    for p in parts[1:]:
        y = (y + p).astype(np.float32)
    st, d = bench.check_result(torch.from_numpy(y), K=K, P=P, k0=0, k1=K, weights=w, W=W, dtype=torch.float32,
                               exact=False, nranks=N, edges=[1024, 2048])
    assert st == "within_tolerance", d
    assert d["max_err_over_bound"] <= 1.0 and d["max_ulp"] >= 0
    bad = y.copy()
    bad[bench.check_cols(P, edges=[1024, 2048])[3]] *= np.float32(1.001)
    st, _ = bench.check_result(torch.from_numpy(bad), K=K, P=P, k0=0, k1=K, weights=w, W=W, dtype=torch.float32,
                               exact=False, nranks=N)
    assert st == "FAILED"
    # bf16 deltas with the f32 mean and its bf16 cast (configs[4]'s shape)
    xb = bf16_to_f32(coracle.synth_bf16(K, P, seed=0))
    parts = [coracle.wsum_f32(xb[g * 24:(g + 1) * 24], np.float32(w[g * 24:(g + 1) * 24]), scale=r)
             for g in range(N)]
    yf = parts[0]
    for p in parts[1:]:
        yf = (yf + p).astype(np.float32)
    yb = torch.from_numpy(bench._bf16_bits(yf).view(np.int16)).view(torch.bfloat16)
    st, d = bench.check_result(yb, K=K, P=P, k0=0, k1=K, weights=w, W=W, dtype=torch.bfloat16, exact=False,
                               nranks=N, f32_mean=torch.from_numpy(yf))
    assert st == "within_tolerance", d
    assert d["bf16_cast_bitwise"] and d["bf16_mean_within_f64_bound"]
