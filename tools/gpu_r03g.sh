mkdir -p gpurun_out/r03g
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -k "pipeline or pipelined or busy or chunked or configs1 or configs2" > gpurun_out/r03g/tests3.log 2>&1; rc=$?; tail -3 gpurun_out/r03g/tests3.log; exit $rc
