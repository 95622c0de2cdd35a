#!/bin/bash
# Per-leaf element units on the pytree path: full GPU suite, layout probe (+ rocprof kernel trace).
set -u
T=${1:-r01zb}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu-tests 600 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${T}_gpu_tests.log 2>&1"
tail -1 $OUT/${T}_gpu_tests.log
run layout 120 bash -c "python tools/probe_ptrs_layout.py > $OUT/${T}_layout.json 2> $OUT/${T}_layout.err"
cat $OUT/${T}_layout.json
run layout-prof 150 rocprofv3 --kernel-trace --stats -d $OUT/${T}_layout_prof -o run --output-format csv -- python tools/probe_ptrs_layout.py
python tools/parse_layout_trace.py $OUT/${T}_layout_prof/run_kernel_trace.csv
