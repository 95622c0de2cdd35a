mkdir -p gpurun_out/r03i
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_fuzz.py > gpurun_out/r03i/fuzz.log 2>&1; rc=$?; tail -3 gpurun_out/r03i/fuzz.log; exit $rc
