"""Read-bandwidth ceilings: contiguous stream vs the fold's row walk (tools/readbw.hip)."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "_build", "libreadbw.so")
if not os.path.exists(so):
    os.makedirs(os.path.dirname(so), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-mcode-object-version=5", "-O3",
                    "-std=c++17", "-fPIC", "-shared", os.path.join(HERE, "readbw.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
lib.readbw.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
sink = torch.zeros(4, dtype=torch.int32, device=dev)
res = {}
for K, row_mb in [(1024, 16), (1024, 64), (1024, 128), (1024, 250)]:
    row = row_mb << 20
    x = torch.empty(K * row, dtype=torch.uint8, device=dev)
    x.fill_(1)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream().cuda_stream
    for mode, grids in [(0, [2048, 4096, 8192]), (1, [256, 512, 768, 1024])]:
        for g in grids:
            lib.readbw(mode, x.data_ptr(), row, K, row, g, sink.data_ptr(), stream)
            s.record()
            for _ in range(3):
                lib.readbw(mode, x.data_ptr(), row, K, row, g, sink.data_ptr(), stream)
            e.record()
            e.synchronize()
            res[f"{K}x{row_mb}MB_mode{mode}_grid{g}"] = round(K * row / (s.elapsed_time(e) / 3 / 1e3) / 1e9, 1)
    del x
    torch.cuda.empty_cache()
print(json.dumps({"probe": "readbw", "GBs": res}))
