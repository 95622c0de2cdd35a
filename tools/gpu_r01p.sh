#!/bin/bash
# Full GPU suite + pytree timings (tree_mean / +l2 / +server Adam) under rocprof.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu-tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r01p_gpu_tests.log 2>&1"
tail -1 $OUT/r01p_gpu_tests.log
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/r01p_prof -o run --output-format csv -- python tools/time_pytree.py
python - <<'PY'
import csv, statistics as st
rows=list(csv.DictReader(open('gpurun_out/r01p_prof/run_kernel_trace.csv')))
for key in ("k_ptrs<0, (anonymous namespace)::AccF, 0, 4, true, false>", "k_ptrs<0, (anonymous namespace)::AccF, 0, 4, true, true>", "k_ptrs_opt<0, 4, true>"):
    d=[int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in rows if key in r['Kernel_Name']]
    small=[x for x in d if x < 1e6]
    print(key[-30:], len(small), 'median us', st.median(small)/1e3 if small else None)
PY
