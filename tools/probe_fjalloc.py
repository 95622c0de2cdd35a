"""fjalloc_alloc / fjalloc_free called directly (after torch has initialised the device), one
fresh process per (reserve, align) configuration: a sequence of segment sizes, each step's
result and fjalloc_stats (last failure decoded as [step, hipError_t]: 1 reserve, 2 create,
3 map, 4 access, 5 range full). usage: python tools/probe_fjalloc.py [RESERVE_GiB ALIGN_KiB MODE]"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(reserve_gib, align_kib, mode):
    import torch

    from fedjax_amd import _lib, memory
    torch.zeros(1, device="cuda")
    lib = _lib.load()
    assert lib.fjalloc_configure(reserve_gib << 30, align_kib << 10, mode, 68 << 10) == 0
    ptrs, steps = [], []
    for mib in (2, 2, 20, 20, 20, 64, 2, 20, 256):
        p = lib.fjalloc_alloc(mib << 20, 0, None)
        st = memory.stats(0)
        steps.append({"MiB": mib, "ok": bool(p), "last_failure": [st["last_failure"] >> 16, st["last_failure"] & 0xFFFF]})
        if p:
            ptrs.append((p, mib << 20))
    st = memory.stats(0)
    for p, n in ptrs:
        lib.fjalloc_free(p, n, 0, None)
    print(json.dumps({"mode": mode, "reserve_GiB": reserve_gib, "align_KiB": align_kib,
                      "granularity": st["granularity"], "at_hint": st["at_hint"], "off_hint": st["off_hint"],
                      "steps": steps, "failures": st["failures"], "live_after_free": memory.stats(0)["live_segments"]}),
          flush=True)


if __name__ == "__main__":
    if len(sys.argv) == 4:
        one(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))
    else:
        for reserve, align, mode in ((1, 2048, 2), (512, 2048, 1), (512, 2048, 0)):
            subprocess.run([sys.executable, os.path.abspath(__file__), str(reserve), str(align), str(mode)],
                           check=False, timeout=120)
