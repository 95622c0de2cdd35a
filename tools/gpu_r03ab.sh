mkdir -p gpurun_out/r03ab
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_tree_ops.py tests/test_gpu_fuzz.py tests/test_gpu_inference_tensors.py tests/test_gpu_graphs.py tests/test_gpu_parity.py > gpurun_out/r03ab/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03ab/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do CPROF=0 timeout -k 10 120 python tools/cprof_library_loop.py 2>/dev/null | grep round_ms || exit 1; done
