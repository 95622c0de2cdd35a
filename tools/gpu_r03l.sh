mkdir -p gpurun_out/r03l
for f in 0 0.25 0 0.25; do
FJAGG_PIPELINE_FRAC=$f timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03l/bench_f$f.json 2> gpurun_out/r03l/bench.err || exit 1
python -c "import json,sys; d=json.load(open('gpurun_out/r03l/bench_f$f.json')); print('$f', d['value'], d['drop_in'])"
done
