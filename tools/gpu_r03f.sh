mkdir -p gpurun_out/r03f
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_adafactor.py > gpurun_out/r03f/tests.log 2>&1; rc=$?; tail -15 gpurun_out/r03f/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/valu_latency.bin > gpurun_out/r03f/valu_latency.jsonl 2>&1 || exit 1
cat gpurun_out/r03f/valu_latency.jsonl
timeout -k 10 300 python tools/time_adafactor.py > gpurun_out/r03f/time.json 2> gpurun_out/r03f/time.err || exit 1
cat gpurun_out/r03f/time.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03f/prof -o run --output-format csv -- python tools/time_adafactor.py > gpurun_out/r03f/prof.log 2>&1 || exit 1
rm -f gpurun_out/r03f/prof/run_kernel_trace.csv
