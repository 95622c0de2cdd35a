# narrow-P exact fold (variant 18) parity + sweep vs the 16-byte variants
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "variants_bitwise or narrow_fold" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02i_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02i_tests.log; [ $rc -le 1 ] || exit $rc
for s in "1024 65536" "4096 16384" "512 131072" "256 262144" "128 524288" "2048 32768" "64 65536"; do
  SWEEP_VARIANTS=2,7,12,18 timeout -k 10 120 python tools/sweep.py $s f32 3 5 || exit 1
done > gpurun_out/r02i_sweep.jsonl
cat gpurun_out/r02i_sweep.jsonl
