#!/bin/bash
# Native host helper (fjhost) on the pytree path: full GPU suite + tree_mean / compression timings.
set -u
T=${1:-r01q}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu-tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${T}_gpu_tests.log 2>&1"
tail -1 $OUT/${T}_gpu_tests.log
run pytree 300 bash -c "python tools/time_pytree.py > $OUT/${T}_pytree.json 2> $OUT/${T}_pytree.err"
cat $OUT/${T}_pytree.json
run comp-bench 600 bash -c "python tools/bench_compression.py --cpu-sample 0 > $OUT/${T}_comp_bench.jsonl 2> $OUT/${T}_comp_bench.err"
cat $OUT/${T}_comp_bench.jsonl
