#!/bin/bash
# Fused l2 norms on the pytree path: GPU parity tests + kernel timing under rocprof.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 bash -c "python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/r01k_parity.log 2>&1"
tail -2 $OUT/r01k_parity.log
run prof 300 rocprofv3 --kernel-trace --stats -d $OUT/r01k_prof -o run --output-format csv -- python tools/time_pytree.py
cat $OUT/r01k_prof/run_kernel_stats.csv | cut -c1-150
