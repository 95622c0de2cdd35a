#!/bin/bash
# Pytree fold schedule per plan: parity, A/B vs the previous build, rocprof of both.
set -u
T=${1:-r01v}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 bash -c "python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $OUT/${T}_parity.log 2>&1"
tail -1 $OUT/${T}_parity.log
: > $OUT/${T}_ab.jsonl
for r in 1 2; do
  run ab-prev-$r 300 bash -c "FJAGG_LIB=tools/_ab/libfjagg_prev.so python tools/ab_kernels.py prev >> $OUT/${T}_ab.jsonl 2>> $OUT/${T}_ab.err"
  run ab-new-$r 300 bash -c "python tools/ab_kernels.py new >> $OUT/${T}_ab.jsonl 2>> $OUT/${T}_ab.err"
done
cat $OUT/${T}_ab.jsonl
run rocprof-prev 300 env FJAGG_LIB=tools/_ab/libfjagg_prev.so rocprofv3 --kernel-trace --stats -d $OUT/${T}_prof_prev -o run --output-format csv -- python tools/ab_kernels.py prev
run rocprof-new 300 rocprofv3 --kernel-trace --stats -d $OUT/${T}_prof_new -o run --output-format csv -- python tools/ab_kernels.py new
