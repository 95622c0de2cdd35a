set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02k_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02k_tests.log; [ $rc -le 1 ] || exit $rc
for m in 524288 0; do
  FJAGG_NARROW_MAX_BYTES=$m timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02k_narrow_$m -o run --output-format csv -- python tools/time_narrow_pytree.py > gpurun_out/r02k_narrow_$m.jsonl 2>&1 || exit 1
  grep '^{' gpurun_out/r02k_narrow_$m.jsonl
  grep -h "k_ptrs" gpurun_out/r02k_narrow_$m/run_kernel_stats.csv | cut -c1-60,200-400
done
