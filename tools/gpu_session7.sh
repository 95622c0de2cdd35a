#!/bin/bash
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2 a1=$3; shift 3; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; if [ $rc -eq 0 ] || { [ $a1 = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi; exit $rc; }
run gpu-tests 900 1 bash -c "python -m pytest tests -q -m gpu -rf > $OUT/r01_gpu_tests_s7.log 2>&1"
tail -3 $OUT/r01_gpu_tests_s7.log
export SWEEP_VARIANTS=1,2,4,5,6,11,12,13
run sweep 1500 0 bash -c "python tools/sweep.py 1024 4194304 f32 3 5 > $OUT/r01_sweep4.jsonl && python tools/sweep.py 128 4194304 f32 3 10 >> $OUT/r01_sweep4.jsonl && python tools/sweep.py 128 1048576 f32 3 10 >> $OUT/r01_sweep4.jsonl && python tools/sweep.py 1024 16777216 bf16 2 3 >> $OUT/r01_sweep4.jsonl && python tools/sweep.py 128 1206590 f32 3 10 >> $OUT/r01_sweep4.jsonl && python tools/sweep.py 10 1206590 f32 3 20 >> $OUT/r01_sweep4.jsonl && python tools/sweep.py 1024 65536 f32 3 20 >> $OUT/r01_sweep4.jsonl"
cat $OUT/r01_sweep4.jsonl
run bench 600 0 bash -c "python bench.py --no-cpu-baseline > $OUT/r01_bench_s7.json 2>&1"
tail -1 $OUT/r01_bench_s7.json
