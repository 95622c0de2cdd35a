#!/bin/bash
# Compression path: GPU tests, round timings, kernel breakdown after the host/stats rework.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run comp-tests 600 bash -c "python -u -m pytest tests/test_gpu_compression.py -x -q --timeout 120 --timeout-method thread > $OUT/r01e_comp_tests.log 2>&1"
tail -2 $OUT/r01e_comp_tests.log
run comp-bench 600 bash -c "python tools/bench_compression.py --cpu-sample 0 > $OUT/r01e_comp_bench.jsonl 2> $OUT/r01e_comp_bench.err"
cat $OUT/r01e_comp_bench.jsonl
run comp-prof 600 rocprofv3 --kernel-trace --stats -d $OUT/r01e_comp_prof -o run --output-format csv -- python tools/bench_compression.py --rounds 3 --warmup 1 --cpu-sample 0
run cprofile 300 bash -c "python -c \"
import cProfile, pstats, sys
sys.argv=['x','--rounds','20','--warmup','2','--cpu-sample','0','--only','uniform']
sys.path.insert(0,'tools')
import bench_compression as b
cProfile.run('b.main()','/tmp/cp')
pstats.Stats('/tmp/cp').sort_stats('cumtime').print_stats(35)
\" > $OUT/r01e_cprofile.txt 2>&1"
