#!/bin/bash
# Full evidence run: GPU tests, smoke, bench (+cpu baseline), rocprofv3 kernel
# trace summary, FETCH_SIZE and WRITE_SIZE PMC passes (separate runs), traffic json.
# usage (on the box, repo root): bash tools/gpu_full.sh TAG
set -u
TAG=${1:-r01}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2 a1=$3; shift 3; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; if [ $rc -eq 0 ] || { [ $a1 = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi; exit $rc; }
run gpu-tests 900 1 bash -c "python -u -m pytest tests -q -m gpu -rfs --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1"
tail -2 $OUT/${TAG}_gpu_tests.log
run smoke 300 0 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/${TAG}_smoke.log 2>&1"
tail -1 $OUT/${TAG}_smoke.log
run bench 600 0 bash -c "python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err"
cat $OUT/${TAG}_bench.json
run rocprof 600 0 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline
cat $OUT/${TAG}_prof/run_kernel_stats.csv
run pmc-fetch 600 0 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run pmc-write 600 0 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run traffic 60 0 python tools/pmc_summary.py $OUT/${TAG}_pmc_fetch $OUT/${TAG}_pmc_write $OUT/${TAG}_traffic_c3.json
