mkdir -p gpurun_out/r04d && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_algorithms.py tests/test_gpu_tree_ops.py tests/test_gpu_inference_tensors.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_fuzz.py tests/test_gpu_host_tables.py tests/test_gpu_adafactor.py tests/test_gpu_server_ext.py -q -rfs --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d/tests.log 2>&1
rc=$?; tail -8 gpurun_out/r04d/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/time_dropin_host.py > gpurun_out/r04d/host.json 2> gpurun_out/r04d/host.err; rc2=$?
cat gpurun_out/r04d/host.json; tail -3 gpurun_out/r04d/host.err
exit $(( rc > rc2 ? rc : rc2 ))
