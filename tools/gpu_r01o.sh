#!/bin/bash
# After the variant change: GPU parity, shard rehearsals (auto-tuned), bucket/event probe.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 bash -c "python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > $OUT/r01o_parity.log 2>&1"
tail -1 $OUT/r01o_parity.log
: > $OUT/r01o_rehearse.jsonl
for n in 8 4 2; do
  run "rehearse-$n" 300 bash -c "python bench.py --rehearse-shard $n --steps 50 --warmup 10 >> $OUT/r01o_rehearse.jsonl 2>> $OUT/r01o_rehearse.err"
done
run probe 300 bash -c "python tools/probe_events.py > $OUT/r01o_probe_events.jsonl 2> $OUT/r01o_probe.err"
python - <<'PY'
import json
for l in open('gpurun_out/r01o_rehearse.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); c=d['config']
    print(c['clients_per_gpu'], c.get('exchange_engine'), 'buckets', c['buckets'], 'ms/step', d['ms_per_step'], 'proj', d.get('rehearsal_projected_whole_job_GBs'), c.get('exchange_autotune_ms'))
for l in open('gpurun_out/r01o_probe_events.jsonl'):
    print(l.strip())
PY
