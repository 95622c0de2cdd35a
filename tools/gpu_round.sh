#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Stops at the first step that ends in anything but success or ordinary test
# failures (faults, aborts, time limits end the session).
# usage (on the box, from the repo root): bash tools/gpu_round.sh TAG [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit allow_rc1 cmd...
  local name=$1 lim=$2 allow1=$3; shift 3
  timeout -k 10 "$lim" "$@"; local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -eq 0 ] || { [ "$allow1" = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi
  exit $rc
}
step gpu-tests 900 1 bash -c "python -m pytest tests -q -m gpu -rf > $OUT/${TAG}_gpu_tests.log 2>&1"
tail -5 "$OUT/${TAG}_gpu_tests.log"
step smoke 300 1 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/${TAG}_smoke.log 2>&1"
tail -2 "$OUT/${TAG}_smoke.log"
step bench 600 0 bash -c "python bench.py $* > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err"
cat "$OUT/${TAG}_bench.json"
step rocprof 600 0 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python bench.py --no-cpu-baseline "$@"
find "$OUT/${TAG}_prof" -name '*kernel_stats.csv' -exec cat {} \;
