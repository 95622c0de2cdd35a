"""Generate the golden fixtures in tests/golden/*.npz (run from the repo root:
``python tests/golden/make_golden.py``).

JAX is not installed here, so the expected outputs come from the numpy
restatement in oracle/tree_util_ref.py, which tests/test_oracle.py pins against
every known-answer test of the reference. Each fixture holds data only:

  x        [K, P] client deltas (float32, int32 or bfloat16 bits as uint16)
  leaf_shapes  [L, 4] leaf shapes (-1 padded) splitting P in flatten order
  weights  [K] float64 values, weight_is_int [K] (Python int vs float weight)
  y        [P] expected tree_mean output (float32 / bfloat16 bits)
  y_f64    [P] (bf16 only) f64 oracle, y_refsem: reference bf16-semantics output
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import tree_util_ref as ref  # noqa: E402


def shapes_array(shapes):
    a = -np.ones((len(shapes), 4), np.int64)
    for i, s in enumerate(shapes):
        a[i, :len(s)] = s
    return a


def tree_mean_flat(x, shapes, weights):
    sizes = [int(np.prod(s)) for s in shapes]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    trees = [[x[k, offs[i]:offs[i + 1]].reshape(s) for i, s in enumerate(shapes)] for k in range(x.shape[0])]
    m = ref.tree_mean(zip(trees, weights))
    return np.concatenate([np.asarray(v).ravel() for v in m])


def save(name, x, shapes, weights, y, **extra):
    wi = np.array([isinstance(w, int) for w in weights])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x, leaf_shapes=shapes_array(shapes),
                        weights=np.array(weights, np.float64), weight_is_int=wi, y=y, **extra)
    print(name, x.shape, x.dtype, "->", y.dtype)


def main():
    # fedjax/aggregators/aggregator_test.py:24-37
    x = np.array([[1., 2., 3.], [2., 4., 6.], [1., 3., 5.]], np.float32)
    w = [2., 4., 2.]
    save("aggregator_kat", x, [(3,)], w, tree_mean_flat(x, [(3,)], w))

    # fedjax/core/tree_util_test.py:53-62 (int leaves, float weights)
    x = np.array([[0, 1], [2, 3], [4, 5]], np.int32)
    w = [6., 7., 8.]
    save("tree_mean_kat", x, [(), ()], w, tree_mean_flat(x, [(), ()], w))

    # tail-only row (P < 4): exercises the 1-element units
    x = ref.synth(1, 7, seed=1)
    save("k1_p7", x, [(7,)], [3], tree_mean_flat(x, [(7,)], [3]))

    # signed zeros survive the fold exactly as in the reference
    x = np.array([[-0.0, 0.0, -0.0, 1.0], [-0.0, -0.0, 0.0, -1.0], [-0.0, 0.0, 0.0, 0.0]], np.float32)
    w = [1, 2, 3]
    save("signed_zero", x, [(4,)], w, tree_mean_flat(x, [(4,)], w))

    # EMNIST-CNN leaf layout (fedjax/models/emnist.py:59-72) at 1/128 scale, 10 clients
    shapes = [(32,), (3, 3, 1, 32), (64,), (3, 3, 2, 8), (128,), (72, 128), (62,), (1, 62)]
    P = sum(int(np.prod(s)) for s in shapes)
    x = ref.synth(10, P, seed=17)
    w = [int(v) for v in ref.fedavg_weights(10, seed=4)]
    save("k10_emnist_1of128", x, shapes, w, tree_mean_flat(x, shapes, w))

    # dense, integer weights (len(client_dataset))
    x = ref.synth(64, 2048, seed=5)
    w = [int(v) for v in ref.fedavg_weights(64, seed=6)]
    save("k64_p2048_intw", x, [(2048,)], w, tree_mean_flat(x, [(2048,)], w))

    # float weights, ragged P
    rs = np.random.RandomState(7)
    x = ref.synth(33, 1001, seed=8)
    w = [float(v) for v in rs.uniform(0.1, 10.0, 33)]
    save("k33_p1001_floatw", x, [(1001,)], w, tree_mean_flat(x, [(1001,)], w))

    # NaN / inf propagate; W = 0 -> s * 0 (NaN where s is NaN or inf)
    x = np.array([[np.nan, np.inf, 1.0, -np.inf, 2.0, 0.5, 3.0, 4.0],
                  [1.0, 1.0, np.inf, np.inf, -2.0, 0.25, 1.0, 1.0]], np.float32)
    save("nan_inf", x, [(8,)], [2, 3], tree_mean_flat(x, [(8,)], [2, 3]))
    save("zero_total_weight", x, [(8,)], [1, -1], tree_mean_flat(x, [(8,)], [1, -1]))
    save("negative_total_weight", x[:, 4:], [(4,)], [1.5, -2.5], tree_mean_flat(x[:, 4:], [(4,)], [1.5, -2.5]))

    # f32 subnormals: IEEE arithmetic, no flush (XLA:CPU flush mode is unpinned)
    x = np.array([[1e-39, -3e-40, 1e-45, 2e-38], [1e-39, 5e-40, 1e-45, -1e-38]], np.float32)
    save("subnormal", x, [(4,)], [1, 1], tree_mean_flat(x, [(4,)], [1, 1]))

    # int leaves: Python-int weights fold in int32 (wrapping), float weights in f32
    xi = (ref.synth(5, 64, seed=9) * 1e5).astype(np.int32)
    save("int_leaves_intw", xi, [(64,)], [3, 1, 4, 1, 5], tree_mean_flat(xi, [(64,)], [3, 1, 4, 1, 5]))
    save("int_leaves_floatw", xi, [(64,)], [0.5, 1.5, 2.0, 1.0, 0.25],
         tree_mean_flat(xi, [(64,)], [0.5, 1.5, 2.0, 1.0, 0.25]))
    big = np.array([[2 ** 30, -(2 ** 30), 7], [2 ** 30, -(2 ** 30), 9]], np.int32)
    save("int_wraparound", big, [(3,)], [3, 2], tree_mean_flat(big, [(3,)], [3, 2]))

    # bf16: the build folds in f32 and rounds once; expected = f64 oracle (tolerance)
    from tests import coracle
    root = os.path.dirname(os.path.dirname(HERE))
    co = coracle.load(os.path.join(root, "oracle", "_build", "liboracle.so"))
    xb = co.synth_bf16(16, 1024, seed=12)
    wb = [int(v) for v in ref.fedavg_weights(16, seed=13)]
    r = 1.0 / float(sum(wb))
    y64 = co.wsum_bf16_f64(xb, np.float64(wb), r)
    yrs = co.wsum_bf16_refsem(xb, np.float32(wb), np.float32(r))
    save("bf16_k16_p1024", xb, [(1024,)], wb, y64.astype(np.float32), y_f64=y64, y_refsem=yrs)


if __name__ == "__main__":
    main()
