mkdir -p gpurun_out/r03w
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_pipeline.py tests/test_gpu_host_tables.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py > gpurun_out/r03w/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03w/tests.log; exit $rc
