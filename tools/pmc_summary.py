"""Per-launch HBM traffic of the fold kernel from rocprofv3 --pmc CSVs.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports exactly half
the bytes of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.

usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [kernel-substring]
"""
import csv
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_tag(path=os.path.join(ROOT, "fedjax_amd", "_build", "libfjagg.so")) -> str:
    """The identity of the kernel build the counters describe: sha256 of libfjagg.so."""
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def per_dispatch(d, counter, pat):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter and pat in r.get("Kernel_Name", ""):
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    agg = {}
    for did, v in rows:
        agg[did] = agg.get(did, 0.0) + v
    return [agg[k] for k in sorted(agg)]


def main():
    fdir, wdir, out = sys.argv[1:4]
    pat = sys.argv[4] if len(sys.argv) > 4 else "k_dense"
    fetch = per_dispatch(fdir, "FETCH_SIZE", pat)
    write = per_dispatch(wdir, "WRITE_SIZE", pat)
    if not fetch or not write:
        raise SystemExit(f"no counters found (fetch={len(fetch)}, write={len(write)})")
    f_med = sorted(fetch)[len(fetch) // 2]
    w_med = sorted(write)[len(write) // 2]
    read_b = 2 * f_med * 1024
    write_b = w_med * 1024
    res = {"kernel": pat, "dispatches": {"fetch": len(fetch), "write": len(write)},
           "fetch_size_kib_median": f_med, "write_size_kib_median": w_med,
           "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": read_b + write_b,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024",
           "build": build_tag(), "collected": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, one pass each, median per dispatch"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
