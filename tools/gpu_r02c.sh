set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree_ops.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02c_tests.log; echo "[tests] rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/prof_literal_loop.py > gpurun_out/r02c_loop.json 2>gpurun_out/r02c_loop.err || exit $?
cat gpurun_out/r02c_loop.json
timeout -k 10 300 python tools/time_running_mean.py > gpurun_out/r02c_time.json 2>gpurun_out/r02c_time.err || exit $?
cat gpurun_out/r02c_time.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02c_prof -o run --output-format csv -- python tools/prof_literal_loop.py > gpurun_out/r02c_prof.log 2>&1 || exit $?
head -6 gpurun_out/r02c_prof/run_kernel_stats.csv
