"""What does a dependency between parameter buckets cost on MI355X? (informs the
bucketed fold + reduce pipeline of include/fjcomm.h)

One step = the fold of a 128-client x 4 Mi f32 shard (one rank of configs[3]),
either as one launch or as 4 / 8 bucket launches, with nothing, a HIP event, or an
event plus a second stream waiting on it after every bucket. Prints one JSON line
per variant: ms per step (wall, 40 steps, after warmup).

usage (GPU box): python tools/probe_events.py
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fedjax_amd import _lib, distributed as fd, kernels  # noqa: E402


def hip_runtime():
    path = _lib.hip_runtimes_mapped()[0]
    hip = ctypes.CDLL(path)
    hip.hipEventCreateWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    return hip


def main(K=128, P=4 * 1024 * 1024, steps=40):
    dev = torch.device("cuda:0")
    x = torch.empty(K, P, device=dev)
    kernels.fill_synth(x, seed=0)
    w = torch.full((K,), 0.5, device=dev)
    out = torch.empty(P, device=dev)
    s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    hip = hip_runtime()
    flags = {"default": 0x0, "no_timing": 0x2, "release_to_device": 0x2 | 0x40000000,
             "no_system_fence": 0x20000000}
    evs = {}
    for name, f in flags.items():
        lst = []
        for _ in range(8):
            e = ctypes.c_void_p()
            rc = hip.hipEventCreateWithFlags(ctypes.byref(e), f)
            lst.append(e if rc == 0 else None)
        evs[name] = lst

    def step(nb, ev=None, wait=False):
        for b, (p0, p1) in enumerate(fd.bucket_edges(P, nb)):
            kernels.weighted_sum_dense(x[:, p0:p1], w, scale=0.25, out=out[p0:p1], nontemporal=True)
            if ev is not None:
                hip.hipEventRecord(ev[b], ctypes.c_void_p(s.cuda_stream))
                if wait:
                    hip.hipStreamWaitEvent(ctypes.c_void_p(side.cuda_stream), ev[b], 0)
        if wait:  # the caller's stream waits for the side stream at the end of the step
            e = torch.cuda.Event()
            e.record(side)
            s.wait_event(e)

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    res = {"one launch": timed(lambda: step(1))}
    for nb in (4, 8):
        res[f"{nb} buckets"] = timed(lambda: step(nb))
        for name, lst in evs.items():
            if any(e is None for e in lst):
                res[f"{nb} buckets + {name} event"] = "unsupported"
                continue
            res[f"{nb} buckets + {name} event"] = timed(lambda: step(nb, lst))
            res[f"{nb} buckets + {name} event + side-stream wait"] = timed(lambda: step(nb, lst, True))
    for k, v in res.items():
        print(json.dumps({"variant": k, "ms_per_step": round(v, 4) if isinstance(v, float) else v}), flush=True)


if __name__ == "__main__":
    main()
