mkdir -p gpurun_out/r03n
timeout -k 10 300 python tools/time_tree_mean_latency.py 0 0.1 0.15 0.25 0.35 > gpurun_out/r03n/latency_fracs.jsonl 2>&1; cat gpurun_out/r03n/latency_fracs.jsonl
