"""Row-walk read bandwidth by load cache policy (tools/readbw.hip readbw_policy): the
fold's access pattern at configs[2]'s footprint (1024 rows x 16 MiB), aux 0..3 and with sc1.
Prints one JSON line: GB/s per aux and grid, median of 5 launches, interleaved."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "_build", "libreadbw_policy.so")
os.makedirs(os.path.dirname(so), exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-mcode-object-version=5", "-O3", "-std=c++17",
                "-fPIC", "-shared", os.path.join(HERE, "readbw.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
lib.readbw_policy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
sink = torch.zeros(4, dtype=torch.int32, device=dev)
K, row = 1024, 16 << 20
x = torch.empty(K * row, dtype=torch.uint8, device=dev)
x.fill_(1)
stream = torch.cuda.current_stream().cuda_stream
res = {}
for rep in range(5):
    for aux in (0, 1, 2, 3, 16, 17, 18, 19):
        for g in (256, 768):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            rc = lib.readbw_policy(aux, x.data_ptr(), row, K, row, g, sink.data_ptr(), stream)
            e.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            res.setdefault(f"aux{aux}_grid{g}", []).append(K * row / (s.elapsed_time(e) * 1e-3) / 1e9)
print(json.dumps({k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}))
