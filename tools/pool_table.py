"""Per-mode medians of the k_ptrs dispatches of tools/probe_delta_pool.py runs (modes run one
after another in one process, the same number of dispatches each): kernel-trace duration and
the UTCL1 translation counters. usage: python tools/pool_table.py TRACE_DIR PMC_DIR OUT.json"""
import collections
import csv
import glob
import json
import statistics
import sys


def split(ids, n=3):
    k = len(ids) // n
    return [ids[i * k:(i + 1) * k] for i in range(n)]


def main(trace_dir, pmc_dir, out, modes=("clones", "pool", "views")):
    durs = {}
    for f in glob.glob(f"{trace_dir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_ptrs" in r["Kernel_Name"]:
                durs[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per = collections.defaultdict(dict)
    for f in glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_ptrs" in r["Kernel_Name"]:
                d, c = int(r["Dispatch_Id"]), r["Counter_Name"]
                per[d][c] = per[d].get(c, 0.0) + float(r["Counter_Value"])
    res = {}
    for m, g in zip(modes, split(sorted(durs))):
        res.setdefault(m, {})["k_ptrs_us_median"] = round(statistics.median(durs[d] for d in g), 2)
    for m, g in zip(modes, split(sorted(per))):
        for c in sorted({c for d in g for c in per[d]}):
            res[m][c] = statistics.median(per[d][c] for d in g)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
