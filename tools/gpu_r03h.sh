mkdir -p gpurun_out/r03h
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_gpu_server_ext.py tests/test_gpu_adafactor.py -k "server or opt or rmsprop or haiku or schedule or adafactor or fedavg" > gpurun_out/r03h/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03h/tests.log; exit $rc
