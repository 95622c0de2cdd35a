mkdir -p gpurun_out/r03v
timeout -k 10 300 python tools/prof_literal_loop.py > gpurun_out/r03v/loop.json 2>/dev/null; cat gpurun_out/r03v/loop.json
