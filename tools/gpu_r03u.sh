mkdir -p gpurun_out/r03u
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_server_ext.py > gpurun_out/r03u/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03u/tests.log; [ $rc -eq 0 ] || exit $rc
true
