mkdir -p gpurun_out/r03ad
PT="python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider"
for r in 1 2; do
timeout -k 10 600 $PT tests > gpurun_out/r03ad/suite_$r.log 2>&1; rc=$?; tail -1 gpurun_out/r03ad/suite_$r.log; [ $rc -le 1 ] || exit $rc
done
