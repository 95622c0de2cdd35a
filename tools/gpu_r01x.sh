#!/bin/bash
# Native tree_mean tail (fjhost.fold_table): full GPU suite, host profile, pytree timing.
set -u
T=${1:-r01x}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu-tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${T}_gpu_tests.log 2>&1"
tail -1 $OUT/${T}_gpu_tests.log
run prof-host 200 bash -c "python tools/prof_host.py > $OUT/${T}_prof_host.txt 2>&1"
grep "host issue" $OUT/${T}_prof_host.txt
run time-pytree 300 bash -c "python tools/time_pytree.py > $OUT/${T}_time_pytree.jsonl 2> $OUT/${T}_time_pytree.err"
cat $OUT/${T}_time_pytree.jsonl
