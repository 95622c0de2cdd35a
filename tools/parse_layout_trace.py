"""Per-placement k_ptrs / k_dense durations from a rocprofv3 kernel trace of
tools/probe_ptrs_layout.py (each mode: WARM + REPS calls, then one extra call)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "k_ptrs" in r["Kernel_Name"] or "k_dense" in r["Kernel_Name"]]
n = 56  # 5 warm + 50 timed + 1 checked call per pytree mode
names = ["views", "clones", "packed", "slab"]
if len(ks) >= 2 * 55 + 4 * n - 1:  # probes with the linear/w-only modes first (55 calls each)
    for i, name in enumerate(["views_linear_w_only", "clones_linear_w_only"]):
        seg = ks[i * 55:(i + 1) * 55]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg[5:55]]
        print(f"{name:21s} median {statistics.median(d):7.2f} us")
    ks = ks[110:]
for i, name in enumerate(names):
    seg = ks[i * n:(i + 1) * n]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg[5:55]]
    print(f"{name:7s} {seg[0]['Kernel_Name'].split('(')[0][-40:]:40s} median {statistics.median(d):7.2f} us "
          f"mean {statistics.mean(d):7.2f} us  ({len(d)} calls)")
