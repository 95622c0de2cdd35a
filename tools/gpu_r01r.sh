#!/bin/bash
# New native-table GPU tests, then the full GPU suite.
set -u
T=${1:-r01r}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run native-tests 300 bash -c "python -u -m pytest tests/test_gpu_parity.py -k native -x -v --timeout 120 --timeout-method thread > $OUT/${T}_native.log 2>&1"
tail -4 $OUT/${T}_native.log
run gpu-tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${T}_gpu_tests.log 2>&1"
tail -1 $OUT/${T}_gpu_tests.log
