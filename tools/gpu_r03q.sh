mkdir -p gpurun_out/r03q
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r03q/bench.json 2> gpurun_out/r03q/bench.err; rc=$?; python -c "import json; d=json.load(open('gpurun_out/r03q/bench.json')); print(d['value'], d['roofline']['frac']); print(json.dumps(d['drop_in'], indent=0))"; exit $rc
