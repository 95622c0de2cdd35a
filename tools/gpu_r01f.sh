#!/bin/bash
# Shard rehearsals (one GPU runs rank 0's share of an N-way shard, RCCL world 1) for N = 2, 4, 8,
# each bucket count, plus the default N=1 bench line.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
: > $OUT/r01f_rehearse.jsonl
for n in 8 4 2; do
  run "rehearse-$n-auto" 300 bash -c "python bench.py --rehearse-shard $n --steps 50 --warmup 10 >> $OUT/r01f_rehearse.jsonl 2>> $OUT/r01f_rehearse.err"
  for b in 1 4 16; do
    run "rehearse-$n-b$b" 300 bash -c "python bench.py --rehearse-shard $n --buckets $b --steps 50 --warmup 10 >> $OUT/r01f_rehearse.jsonl 2>> $OUT/r01f_rehearse.err"
  done
done
python -c "
import json
for l in open('$OUT/r01f_rehearse.jsonl'):
    d=json.loads(l); c=d['config']
    print(c['clients_per_gpu'], 'buckets', c['buckets'], 'ms/step', d['ms_per_step'], 'host', d['host_issue_ms_per_step'], 'kernel ms', d['roofline']['mean_launch_ms'], 'proj GB/s', d.get('rehearsal_projected_whole_job_GBs'), c.get('bucket_autotune_ms'))
"
