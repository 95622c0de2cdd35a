#!/bin/bash
# Evidence run on one GPU box: full GPU suite (-rs: skip reasons), smoke, the default bench
# line, the FETCH/WRITE traffic passes of this build (bench.py --measure-traffic), the bare
# N=2 launcher (gloo exchange, both ranks on the box's GPU, e2e leg), the rocprofv3
# kernel-trace summary of the bench (its timed kernels: no e2e leg), and the examples/fed_avg.py
# round with lazy norms: its timing and its PMC read traffic per mode. Each step has its own limit; the script stops
# at the first failing step (test failures included).
# usage (repo root, on the box): bash tools/gpu_r06_final.sh TAG
set -u
TAG=${1:-r06}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfs --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1 || exit $?
tail -1 "$O/smoke.log"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit $?
cat "$O/bench.json"
timeout -k 10 900 python bench.py --measure-traffic --traffic-out "$O/traffic_c3.json" --no-cpu-baseline --no-dropin --no-e2e \
  > "$O/bench_traffic.json" 2> "$O/bench_traffic.err" || exit $?
cat "$O/bench_traffic.json"
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > "$O/bench_n2_gloo.json" \
  2> "$O/bench_n2_gloo.err" || exit $?
cat "$O/bench_n2_gloo.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-dropin --no-e2e > "$O/prof.log" 2>&1 || exit $?
cat "$O"/prof/run_kernel_stats.csv | head -8
rm -f "$O"/prof/run_kernel_trace.csv
# the examples/fed_avg.py round: timing (lazy / eager norms / mean only) and its PMC traffic per mode
timeout -k 10 300 python tools/time_example_round.py > "$O/example_round.json" 2> "$O/example_round.err" || exit $?
cat "$O/example_round.json"
bash tools/gpu_pmc_example.sh "$TAG/pmc_example" > "$O/pmc_example.log" 2>&1 || exit $?
cat "$O/pmc_example.log"
echo done
