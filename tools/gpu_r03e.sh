mkdir -p gpurun_out/r03e
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_pipeline.py > gpurun_out/r03e/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03e/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_tree_mean_latency.py 0 0.25 -0.25 0.15 > gpurun_out/r03e/latency3.jsonl 2> gpurun_out/r03e/latency.err; rc=$?; cat gpurun_out/r03e/latency3.jsonl; exit $rc
