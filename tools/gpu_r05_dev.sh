#!/bin/bash
# Round-5 development run on one GPU box: the GPU suite, the fused-norm A/B (probe_l2_ab),
# the host cost of the per-client norm call (prof_norm_call), the default bench line (with
# its oracle check, e2e sample and drop-in record) and the bare N=2 launcher (gloo exchange,
# both ranks on the box's GPU: its tolerance check). Each step has its own limit; the script
# stops at the first failing step.
# usage (repo root, on the box): bash tools/gpu_r05_dev.sh TAG [skip-tests]
set -u
TAG=${1:-r05}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rfs --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
  tail -3 "$O/gpu_tests.log"
fi
timeout -k 10 300 python tools/probe_l2_ab.py 50 5 > "$O/l2_ab.jsonl" 2> "$O/l2_ab.err" || { tail -20 "$O/l2_ab.err"; exit 1; }
cat "$O/l2_ab.jsonl"
timeout -k 10 300 python tools/prof_norm_call.py 40 > "$O/norm_call.json" 2> "$O/norm_call.err" || { tail -20 "$O/norm_call.err"; exit 1; }
cat "$O/norm_call.json"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > "$O/bench_n2_gloo.json" \
  2> "$O/bench_n2_gloo.err" || { tail -20 "$O/bench_n2_gloo.err"; exit 1; }
cat "$O/bench_n2_gloo.json"
echo done
