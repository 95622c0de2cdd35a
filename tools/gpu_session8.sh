#!/bin/bash
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2 a1=$3; shift 3; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; if [ $rc -eq 0 ] || { [ $a1 = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi; exit $rc; }
run gpu-tests 900 1 bash -c "python -m pytest tests -q -m gpu -rf -x > $OUT/r01_gpu_tests_s8.log 2>&1"
tail -15 $OUT/r01_gpu_tests_s8.log
run bench-norms 600 0 bash -c "python bench.py --no-cpu-baseline --with-norms > $OUT/r01_bench_norms.json 2>&1 && python bench.py --no-cpu-baseline > $OUT/r01_bench_nonorms.json 2>&1 && python bench.py --no-cpu-baseline --workload c2 --with-norms > $OUT/r01_bench_c2_norms.json 2>&1 && python bench.py --no-cpu-baseline --workload c2 > $OUT/r01_bench_c2c.json 2>&1 && python bench.py --workload c5s --steps 5 --warmup 2 > $OUT/r01_bench_c5s_b.json 2>&1"
for f in r01_bench_norms r01_bench_nonorms r01_bench_c2_norms r01_bench_c2c r01_bench_c5s_b; do tail -1 $OUT/$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['config']['workload'][:40])"; done
