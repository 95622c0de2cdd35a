#!/bin/bash
# Fused-norm fold A/B on one GPU box: the tests that pin the norms' bits, then the norms
# loop (tools/time_norms_loop.py) and the dense fused-norm bench under rocprofv3 kernel trace,
# once with the in-tree libfjagg.so and once with the library at FJAGG_LIB_OLD.
# usage (repo root, on the box): FJAGG_LIB_OLD=scratch/oldlib/libfjagg.so bash tools/gpu_l2_ab.sh TAG
set -u
TAG=${1:-l2ab}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree_ops.py tests/test_gpu_parity.py tests/test_gpu_running_sum_fuzz.py \
  tests/test_gpu_fuzz.py tests/test_gpu_algorithms.py tests/test_gpu_pipeline.py -q -rfs -x --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in new old; do
  mkdir -p "$O/$v"
  if [ $v = old ]; then export FJAGG_LIB=$FJAGG_LIB_OLD; fi
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$O/$v/loop" -o run --output-format csv -- \
    python tools/time_norms_loop.py 10 > "$O/$v/loop.json" 2> "$O/$v/loop.err" || exit $?
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$O/$v/dense" -o run --output-format csv -- \
    python bench.py --with-norms --no-cpu-baseline --no-dropin > "$O/$v/dense.json" 2> "$O/$v/dense.err" || exit $?
  rm -f "$O"/$v/*/run_kernel_trace.csv
  unset FJAGG_LIB
done
echo done
