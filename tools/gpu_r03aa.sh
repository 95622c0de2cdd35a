mkdir -p gpurun_out/r03aa
timeout -k 10 300 python tools/bench_compression.py --cpu-sample 0 > gpurun_out/r03aa/comp.jsonl 2> gpurun_out/r03aa/comp.err; rc=$?; cat gpurun_out/r03aa/comp.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03aa/prof -o run --output-format csv -- python tools/bench_compression.py --cpu-sample 0 --only uniform --rounds 5 > gpurun_out/r03aa/prof.log 2>&1 || exit 1
rm -f gpurun_out/r03aa/prof/run_kernel_trace.csv
