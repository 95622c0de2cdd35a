"""Read bandwidth by column-segment width (tools/segbw.hip): a 16384 x 4096 float32 slab
(268 MB, the 16384 x 4 Ki stripe-fold shape) and a 4096 x 16384 one, read as segments of
64 ... 1024 bytes per client row, ~1024 workgroups in every case. Prints one JSON line per
(shape, segment, mapping): GB/s, median of 20 timed launches (HIP events)."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "_build", "libsegbw.so")
if not os.path.exists(so):
    os.makedirs(os.path.dirname(so), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-mcode-object-version=5", "-O3",
                    "-std=c++17", "-fPIC", "-shared", os.path.join(HERE, "segbw.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
lib.segbw.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
sink = torch.zeros(4, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream().cuda_stream
for K, P in [(16384, 4096), (4096, 16384)]:
    x = torch.ones(K, P, dtype=torch.float32, device=dev)
    nbytes = K * P * 4
    for seg in (64, 128, 256, 512, 1024):
        for xcd in (0, 1):
            times = []
            for i in range(25):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                assert lib.segbw(x.data_ptr(), P * 4, K, P * 4, seg, 1024, xcd, sink.data_ptr(), stream) == 0
                e.record()
                e.synchronize()
                if i >= 5:
                    times.append(s.elapsed_time(e))
            ms = float(np.median(times))
            print(json.dumps({"K": K, "P": P, "segment_bytes": seg, "xcd_contiguous": xcd,
                              "GBs": round(nbytes / ms / 1e6, 1), "ms": round(ms, 4)}), flush=True)
    del x
