#!/bin/bash
# Native RCCL pipeline: GPU distributed tests, shard rehearsals (auto-tuned engine), N=1 bench.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run dist-tests 300 bash -c "python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread > $OUT/r01h_dist_tests.log 2>&1"
tail -4 $OUT/r01h_dist_tests.log
: > $OUT/r01h_rehearse.jsonl
for n in 8 4 2; do
  run "rehearse-$n" 300 bash -c "python bench.py --rehearse-shard $n --steps 50 --warmup 10 >> $OUT/r01h_rehearse.jsonl 2>> $OUT/r01h_rehearse.err"
done
run bench 300 bash -c "python bench.py --no-cpu-baseline > $OUT/r01h_bench.json 2> $OUT/r01h_bench.err"
python - <<'PY'
import json
for l in open('gpurun_out/r01h_rehearse.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); c=d['config']
    print(c['clients_per_gpu'], c['exchange_engine'], 'buckets', c['buckets'], 'ms/step', d['ms_per_step'], 'host', d['host_issue_ms_per_step'], 'kernel ms', d['roofline']['mean_launch_ms'], 'proj', d.get('rehearsal_projected_whole_job_GBs'), c.get('exchange_autotune_ms'))
d=json.load(open('gpurun_out/r01h_bench.json'))
print('N=1', d['value'], d['ms_per_step'], d['roofline'])
PY
