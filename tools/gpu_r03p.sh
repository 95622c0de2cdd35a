mkdir -p gpurun_out/r03p
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
true
timeout -k 10 300 python tools/time_aggregator_latency.py > gpurun_out/r03p/agg.jsonl 2>&1; cat gpurun_out/r03p/agg.jsonl
