# narrow-P exact fold (variant 18) parity + sweep vs the 16-byte variants (v0 = the default pick)
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "variants_bitwise or narrow_fold or golden or split or bf16" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02i_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02i_tests.log; [ $rc -le 1 ] || exit $rc
for s in "1024 65536 f32" "4096 16384 f32" "512 131072 f32" "256 262144 f32" "2048 32768 f32" "64 65536 f32" "16384 4096 f32" "1024 131072 bf16" "4096 32768 bf16" "1024 4194304 f32"; do
  SWEEP_VARIANTS=0,2,18 timeout -k 10 120 python tools/sweep.py $s 3 5 || exit 1
done > gpurun_out/r02i_sweep.jsonl
cat gpurun_out/r02i_sweep.jsonl
