mkdir -p gpurun_out/r03j
timeout -k 10 300 python tools/segbw.py > gpurun_out/r03j/segbw.jsonl 2> gpurun_out/r03j/segbw.err; rc=$?; cat gpurun_out/r03j/segbw.jsonl; exit $rc
