#!/bin/bash
# Compression kernels after the segment-search change: parity tests, round timings, kernel stats.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run comp-tests 600 bash -c "python -u -m pytest tests/test_gpu_compression.py -x -q --timeout 200 --timeout-method thread > $OUT/r01l_comp_tests.log 2>&1"
tail -1 $OUT/r01l_comp_tests.log
run comp-bench 600 bash -c "python tools/bench_compression.py --cpu-sample 0 > $OUT/r01l_comp_bench.jsonl 2> $OUT/r01l_comp_bench.err"
cat $OUT/r01l_comp_bench.jsonl
run comp-prof 600 rocprofv3 --kernel-trace --stats -d $OUT/r01l_comp_prof -o run --output-format csv -- python tools/bench_compression.py --rounds 3 --warmup 1 --cpu-sample 0
