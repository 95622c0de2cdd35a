mkdir -p gpurun_out/r03y
timeout -k 10 600 python tools/dropin_flush_ab.py > gpurun_out/r03y/flush_ab.jsonl 2> gpurun_out/r03y/err.txt; rc=$?; cat gpurun_out/r03y/flush_ab.jsonl; exit $rc
