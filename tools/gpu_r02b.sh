set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree_ops.py tests/test_gpu_distributed.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02b_tests.log; echo "[tests] rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/time_running_mean.py > gpurun_out/r02b_time.json 2>gpurun_out/r02b_time.err || exit $?
cat gpurun_out/r02b_time.json
timeout -k 10 300 python bench.py --single-process --gpus 1 --steps 10 --warmup 3 > gpurun_out/r02b_single.json 2>gpurun_out/r02b_single.err || exit $?
cat gpurun_out/r02b_single.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02b_prof -o run --output-format csv -- python tools/time_running_mean.py > gpurun_out/r02b_prof.log 2>&1 || exit $?
cat gpurun_out/r02b_prof/run_kernel_stats.csv
