#!/bin/bash
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2 a1=$3; shift 3; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; if [ $rc -eq 0 ] || { [ $a1 = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi; exit $rc; }
run gpu-tests 900 1 bash -c "python -m pytest tests -q -m gpu -rf -x -k fused > $OUT/r01_gpu_tests_s9.log 2>&1"
tail -2 $OUT/r01_gpu_tests_s9.log
run prof-c2 600 0 rocprofv3 --kernel-trace --stats -d $OUT/r01_prof_c2n -o run --output-format csv -- python bench.py --no-cpu-baseline --workload c2 --with-norms
cat $OUT/r01_prof_c2n/run_kernel_stats.csv | cut -c1-60,200-
run prof-c3 600 0 rocprofv3 --kernel-trace --stats -d $OUT/r01_prof_c3n -o run --output-format csv -- python bench.py --no-cpu-baseline --with-norms
cat $OUT/r01_prof_c3n/run_kernel_stats.csv | cut -c1-60,200-
run bfsweep 900 0 bash -c "SWEEP_VARIANTS=12 python tools/sweep.py 1024 33554432 bf16 2 3 > $OUT/r01_bfsize.jsonl && SWEEP_VARIANTS=12 python tools/sweep.py 1024 67108864 bf16 2 3 >> $OUT/r01_bfsize.jsonl && SWEEP_VARIANTS=12 python tools/sweep.py 512 125000000 bf16 2 3 >> $OUT/r01_bfsize.jsonl && SWEEP_VARIANTS=12 python tools/sweep.py 1024 125000000 bf16 2 2 >> $OUT/r01_bfsize.jsonl && SWEEP_VARIANTS=12 python tools/sweep.py 2048 16777216 f32 2 3 >> $OUT/r01_bfsize.jsonl"
cat $OUT/r01_bfsize.jsonl
