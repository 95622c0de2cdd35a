"""A workload for the PMC traffic passes of the fused-norm pytree fold: `calls` launches of
fjagg_wsum_l2_ptrs (last-workgroup combine, FJAGG_ZEROED_WS) over configs[1]'s 128 clients x
EMNIST-CNN, one allocation per (client, leaf), nothing else on the GPU after the setup fills.
Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (one pass each) and summarise with
`tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json k_ptrs`; algorithmic bytes per launch =
128 x 1,206,590 x 4 read + 1,206,590 x 4 written.
usage: python tools/probe_l2_traffic.py [calls]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fedjax_amd import _lib, kernels

SHAPES = [(32,), (3, 3, 1, 32), (64,), (3, 3, 32, 64), (128,), (9216, 128), (62,), (128, 62)]
F32, SCALE, NONTEMPORAL, ZEROED_WS = 0, 1, 4, 128  # include/fjagg.h


def main(calls=8, K=128):
    dev = torch.device("cuda:0")
    lib = _lib.load()
    L = len(SHAPES)
    leaves = []
    for k in range(K):
        row = []
        for l, shp in enumerate(SHAPES):
            x = torch.empty(1, int(np.prod(shp)), dtype=torch.float32, device=dev)
            kernels.fill_synth(x, seed=l + 1, k0=k)
            row.append(x)
        leaves.append(row)
    leaf_n = np.array([int(np.prod(s)) for s in SHAPES], dtype=np.int64)
    outs = [torch.empty(n, dtype=torch.float32, device=dev) for n in leaf_n]
    nb = lib.fjagg_ptrs_plan_leaves(F32, 0, leaf_n.ctypes.data, None, L, None, 0)
    blocks = np.empty(2 * nb, dtype=np.int64)
    lib.fjagg_ptrs_plan_leaves(F32, 0, leaf_n.ctypes.data, None, L, blocks.ctypes.data, nb)
    in_ptrs = np.array([[x.data_ptr() for x in r] for r in leaves], dtype=np.int64).ravel()
    out_ptrs = np.array([o.data_ptr() for o in outs], dtype=np.int64)
    img = torch.from_numpy(np.concatenate([in_ptrs, out_ptrs, leaf_n, blocks])).to(dev)
    w = torch.tensor(np.random.RandomState(1).randint(1, 501, size=K), dtype=torch.float32, device=dev)
    l2 = torch.empty(K, dtype=torch.float32, device=dev)
    ws = torch.zeros(max(1, lib.fjagg_wsum_l2_ptrs_workspace_bytes(K, nb)), dtype=torch.uint8, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    for _ in range(calls):
        _lib.check(lib.fjagg_wsum_l2_ptrs(F32, F32, F32, img.data_ptr(), L, K, nb, w.data_ptr(), ctypes.c_float(1e-3),
                                          l2.data_ptr(), SCALE | NONTEMPORAL | ZEROED_WS, ws.data_ptr(), ws.numel(), s),
                   "fused-norm fold")
    torch.cuda.synchronize()
    print(f"{calls} fused-norm folds, K={K}, {int(leaf_n.sum())} params, {nb} workgroups", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
