mkdir -p gpurun_out/r03ac
B="python bench.py --no-cpu-baseline --no-dropin"
timeout -k 10 300 $B --workload c2 > gpurun_out/r03ac/bench_c2.json 2> gpurun_out/r03ac/c2.err || exit 1
timeout -k 10 300 $B --rehearse-shard 8 > gpurun_out/r03ac/bench_c3_shard8.json 2> gpurun_out/r03ac/shard.err || exit 1
timeout -k 10 600 $B --workload c5s --steps 5 --warmup 2 > gpurun_out/r03ac/bench_c5s.json 2> gpurun_out/r03ac/c5s.err || exit 1
timeout -k 10 600 $B --workload c5 --rehearse-shard 8 --steps 5 --warmup 2 > gpurun_out/r03ac/bench_c5_shard8.json 2> gpurun_out/r03ac/c5.err || exit 1
for f in gpurun_out/r03ac/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['config'].get('buckets'), d['config'].get('exchange_engine'))"; done
