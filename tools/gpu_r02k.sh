set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02k_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02k_tests.log; [ $rc -le 1 ] || exit $rc
for m in 524288 0; do
  FJAGG_NARROW_MAX_BYTES=$m timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02k_narrow_$m -o run --output-format csv -- python tools/time_narrow_pytree.py > gpurun_out/r02k_narrow_$m.jsonl 2>&1 || exit 1
  rm -f gpurun_out/r02k_narrow_$m/run_kernel_trace.csv
  grep '^{' gpurun_out/r02k_narrow_$m.jsonl
  python -c "
import csv
for r in csv.DictReader(open('gpurun_out/r02k_narrow_$m/run_kernel_stats.csv')):
    if 'k_ptrs' in r['Name']: print(r['Name'][:90], r['Calls'], r['AverageNs'])
"
done
