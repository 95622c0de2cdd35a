mkdir -p gpurun_out/r03o
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
FJAGG_PTRS_PF=8 timeout -k 10 300 $PT tests/test_gpu_fullsize.py -k "configs1 or configs2" tests/test_gpu_host_tables.py > gpurun_out/r03o/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03o/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do for pf in 0 4 8 16; do
  FJAGG_PTRS_PF=$pf timeout -k 10 200 python tools/time_tree_mean_latency.py 0.25 > gpurun_out/r03o/lat_pf$pf.r$round.json 2>/dev/null || exit 1
  echo "pf=$pf r=$round $(cat gpurun_out/r03o/lat_pf$pf.r$round.json)"
done; done
