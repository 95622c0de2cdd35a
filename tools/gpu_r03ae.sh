mkdir -p gpurun_out/r03ae
PT="python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests > gpurun_out/r03ae/suite.log 2>&1; rc=$?; tail -1 gpurun_out/r03ae/suite.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do CPROF=0 timeout -k 10 120 python tools/cprof_library_loop.py 2>/dev/null | grep round_ms || exit 1; done
timeout -k 10 300 python tools/prof_literal_loop.py 2>/dev/null
timeout -k 10 300 python tools/time_tree_mean_latency.py 2>/dev/null
