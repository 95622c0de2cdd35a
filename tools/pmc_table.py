"""Median per-dispatch counter values of one kernel from rocprofv3 --pmc / --kernel-trace
output directories. usage: python tools/pmc_table.py KERNEL_SUBSTRING OUT.json DIR [DIR ...]

Counters with an instance dimension (e.g. TCC_EA0_RDREQ per channel) are summed per
dispatch and also reported as max/min over instances (channel balance). Kernel-trace
directories give the median duration in us."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    pat, out, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {}
    for d in dirs:
        name = os.path.basename(d.rstrip("/"))
        per = {}
        inst = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if pat not in r.get("Kernel_Name", ""):
                        continue
                    key = (r["Counter_Name"], int(r["Dispatch_Id"]))
                    per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
                    inst.setdefault(key, []).append(float(r["Counter_Value"]))
        entry = {}
        for c in sorted({k[0] for k in per}):
            vals = [v for (cn, _), v in per.items() if cn == c]
            entry[c] = statistics.median(vals)
            spreads = [(max(v), min(v)) for (cn, _), v in inst.items() if cn == c and len(v) > 1]
            if spreads:
                entry[c + "@max_instance"] = statistics.median([a for a, _ in spreads])
                entry[c + "@min_instance"] = statistics.median([b for _, b in spreads])
                entry[c + "@instances"] = len([v for (cn, _), v in inst.items() if cn == c][0])
        durs = []
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if pat in r.get("Kernel_Name", ""):
                        durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if durs:
            entry["duration_us_median"] = statistics.median(durs)
            entry["dispatches"] = len(durs)
        res[name] = entry
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
