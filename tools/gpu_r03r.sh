mkdir -p gpurun_out/r03r
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_tree_ops.py tests/test_gpu_fuzz.py tests/test_gpu_inference_tensors.py tests/test_gpu_pipeline.py > gpurun_out/r03r/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03r/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/cprof_library_loop.py > gpurun_out/r03r/cprof2.txt 2>&1; rc=$?; head -30 gpurun_out/r03r/cprof2.txt; exit $rc
