#!/bin/bash
# Round-4 check on one GPU box: the GPU test files the round changed, the drop-in host timings
# (tools/time_dropin_host.py), the early-flush sweep on a GPU-bound model
# (tools/time_flush_large.py) and the delta-pool placement probe (tools/probe_delta_pool.py).
# Every GPU step runs under its own limit; the script stops at the first failing step.
# usage (repo root, on the box): bash tools/gpu_r04_check.sh TAG
set -u
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_tree_ops.py tests/test_gpu_fuzz.py \
  tests/test_gpu_host_tables.py tests/test_gpu_parity.py tests/test_gpu_algorithms.py tests/test_gpu_inference_tensors.py \
  tests/test_gpu_memory.py tests/test_gpu_running_sum_fuzz.py -q -rfs -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_dropin_host.py > "$O/host.json" 2> "$O/host.err" || exit $?
cat "$O/host.json"
timeout -k 10 300 python tools/time_norms_loop.py > "$O/norms_loop.json" 2> "$O/norms_loop.err" || exit $?
cat "$O/norms_loop.json"
timeout -k 10 300 python tools/time_flush_large.py > "$O/flush_large.json" 2> "$O/flush_large.err" || exit $?
cat "$O/flush_large.json"
timeout -k 10 300 python tools/probe_delta_pool.py > "$O/pool.jsonl" 2> "$O/pool.err" || exit $?
cat "$O/pool.jsonl"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/pool_trace" -o run --output-format csv -- \
  python tools/probe_delta_pool.py clones,pool,views 20 > "$O/pool_trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -d "$O/pool_pmc" \
  -o run --output-format csv -- python tools/probe_delta_pool.py clones,pool,views 10 > "$O/pool_pmc.log" 2>&1 || exit $?
rm -f "$O"/pool_trace/*/run_kernel_trace.csv.bak
echo done
