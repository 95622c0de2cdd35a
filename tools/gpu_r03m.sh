mkdir -p gpurun_out/r03m
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_fullsize.py tests/test_gpu_host_tables.py tests/test_native_host.py tests/test_gpu_inference_tensors.py > gpurun_out/r03m/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03m/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_tree_mean_latency.py > gpurun_out/r03m/latency_native.jsonl 2>&1 || exit 1
FJAGG_NATIVE_MEAN=0 timeout -k 10 300 python tools/time_tree_mean_latency.py > gpurun_out/r03m/latency_python.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/time_tree_mean_latency.py > gpurun_out/r03m/latency_native2.jsonl 2>&1 || exit 1
FJAGG_NATIVE_MEAN=0 timeout -k 10 300 python tools/time_tree_mean_latency.py > gpurun_out/r03m/latency_python2.jsonl 2>&1 || exit 1
grep -h single gpurun_out/r03m/latency_*.jsonl
