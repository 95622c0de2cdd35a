#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench at N=1, the bare N=2 launcher (gloo
# exchange, both ranks on the box's one GPU), rocprofv3 kernel-trace summary of the bench.
# Every GPU step has its own time limit; the session ends at the first step that fails
# with anything but ordinary test failures (faults, aborts, time limits end it).
# usage (on the box, from the repo root): bash tools/gpu_session.sh TAG [pytest -k expr]
# (tools/gpu_full.sh TAG adds the FETCH_SIZE / WRITE_SIZE PMC passes behind profiles/traffic_c3.json;
#  tools/gpu_study.sh STUDY runs the studies behind DESIGN.md's other numbers)
set -u
TAG=${1:-r02}
KEXPR=${2:-}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit allow_rc1 cmd...
  local name=$1 lim=$2 allow1=$3; shift 3
  timeout -k 10 "$lim" "$@"; local rc=$?
  echo "[$name] rc=$rc" >&2
  if [ $rc -eq 0 ] || { [ "$allow1" = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi
  exit $rc
}
if [ -n "$KEXPR" ]; then
  step gpu-tests 900 1 python -u -m pytest tests -x -v -m gpu -k "$KEXPR" --timeout 300 --timeout-method thread -rs \
    -p no:cacheprovider > "$OUT/${TAG}_gpu_tests.log" 2>&1
else
  step gpu-tests 1100 1 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rfs \
    -p no:cacheprovider > "$OUT/${TAG}_gpu_tests.log" 2>&1
fi
tail -5 "$OUT/${TAG}_gpu_tests.log"
step smoke 300 1 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/${TAG}_smoke.log" 2>&1
tail -2 "$OUT/${TAG}_smoke.log"
step bench 600 0 python bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
cat "$OUT/${TAG}_bench.json"
step bench-n2-gloo 600 0 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 \
  > "$OUT/${TAG}_bench_n2_gloo.json" 2> "$OUT/${TAG}_bench_n2_gloo.err"
cat "$OUT/${TAG}_bench_n2_gloo.json"
step rocprof 600 0 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- \
  python bench.py --no-cpu-baseline
find "$OUT/${TAG}_prof" -name '*kernel_stats.csv' -exec cat {} \;
