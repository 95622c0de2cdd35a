#!/bin/bash
# Dense fold variant sweep at the per-bucket shapes of the sharded pipeline (K = 1024/N, P = 4 Mi / buckets).
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
export SWEEP_VARIANTS=2,4,5,6,7,12,13
: > $OUT/r01n_sweep.jsonl
for kp in "128 524288" "128 1048576" "128 2097152" "256 524288" "256 1048576" "512 524288" "512 1048576" "1024 1048576"; do
  timeout -k 10 120 python tools/sweep.py $kp f32 3 5 >> $OUT/r01n_sweep.jsonl 2>> $OUT/r01n_sweep.err || exit $?
done
python - <<'PY'
import json
for l in open('gpurun_out/r01n_sweep.jsonl'):
    d=json.loads(l); g=d['GBs_median']
    best=max(g, key=g.get)
    print(d['sweep'], 'best', best, g[best], ' v12_bal1', g.get('v12_bal1'), ' v6_bal1', g.get('v6_bal1'), ' v4_bal1', g.get('v4_bal1'), ' v5_bal1', g.get('v5_bal1'), ' v7_bal1', g.get('v7_bal1'))
PY
