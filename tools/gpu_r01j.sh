#!/bin/bash
# Full GPU test suite + pytree-path timing (configs[1] through tree_mean) + compression rounds.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu-tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r01j_gpu_tests.log 2>&1"
tail -2 $OUT/r01j_gpu_tests.log
run pytree 300 bash -c "python tools/time_pytree.py > $OUT/r01j_pytree.json 2> $OUT/r01j_pytree.err"
cat $OUT/r01j_pytree.json
run comp-bench 600 bash -c "python tools/bench_compression.py --cpu-sample 0 > $OUT/r01j_comp_bench.jsonl 2> $OUT/r01j_comp_bench.err"
cat $OUT/r01j_comp_bench.jsonl
