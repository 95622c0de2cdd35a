"""Does a hipMemsetAsync recorded in a HIP graph take effect before the next kernel node on
replay? Captures [memset(buf, 0) ; out = buf + 0 (a kernel)] and, for comparison,
[buf.zero_() (a fill kernel) ; out = buf + 0], sets buf to 7 before each replay and prints
whether out reads zeros. Sizes 16 bytes and 64 KiB. Exploration only."""
import ctypes
import json

import torch

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
res = {}
for nbytes in (16, 65536):
    for how in ("hipMemsetAsync", "fill_kernel"):
        buf = torch.full((nbytes // 4,), 7, dtype=torch.int32, device=dev)
        out = torch.empty_like(buf)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                if how == "hipMemsetAsync":
                    rc = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, ctypes.c_size_t(nbytes),
                                            ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0, rc
                else:
                    buf.zero_()
                torch.add(buf, 0, out=out)
        ok = []
        for _ in range(5):
            buf.fill_(7)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            ok.append(bool((out == 0).all().item()))
        res[f"{how}_{nbytes}B"] = ok
print(json.dumps(res))
