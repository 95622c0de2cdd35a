mkdir -p gpurun_out/r03z
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_pipeline.py tests/test_gpu_host_tables.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/r03z/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03z/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_tree_mean_latency.py 0.25 0 0.25 > gpurun_out/r03z/latency.jsonl 2>&1; cat gpurun_out/r03z/latency.jsonl
