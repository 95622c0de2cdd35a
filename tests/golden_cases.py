"""Loader for tests/golden/*.npz (see tests/golden/make_golden.py)."""
import glob
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, "*.npz")))


def load(name):
    d = np.load(os.path.join(HERE, name + ".npz"))  # allow_pickle=False (default)
    shapes = [tuple(int(v) for v in row if v >= 0) for row in d["leaf_shapes"]]
    weights = [int(w) if is_int else float(w) for w, is_int in zip(d["weights"], d["weight_is_int"])]
    return {k: d[k] for k in d.files} | {"shapes": shapes, "weight_list": weights}


def split_leaves(row, shapes):
    sizes = [int(np.prod(s)) for s in shapes]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    return [row[offs[i]:offs[i + 1]].reshape(s) for i, s in enumerate(shapes)]
