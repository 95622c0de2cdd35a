#!/bin/bash
# Host-path A/B timings + delta-pool (fjalloc) placement study on one GPU box.
# usage (repo root, on the box): bash tools/gpu_r04_pool.sh TAG
set -u
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python tools/time_dropin_host.py > "$O/host.json" 2> "$O/host.err" || exit $?
cat "$O/host.json"
timeout -k 10 400 python tools/probe_fjalloc.py > "$O/fjalloc.jsonl" 2> "$O/fjalloc.err"; rc=$?
cat "$O/fjalloc.jsonl"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/probe_delta_pool.py > "$O/pool.jsonl" 2> "$O/pool.err"; rc=$?
cat "$O/pool.jsonl"; tail -2 "$O/pool.err"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/pool_trace" -o run --output-format csv -- \
  python tools/probe_delta_pool.py clones,pool,views 20 > "$O/pool_trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -d "$O/pool_pmc" \
  -o run --output-format csv -- python tools/probe_delta_pool.py clones,pool,views 10 > "$O/pool_pmc.log" 2>&1 || exit $?
echo done
