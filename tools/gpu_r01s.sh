#!/bin/bash
# Row-pointer prefetch in the fold, group-ahead loads in k_quant_fold, tapered buckets:
# parity on the changed paths, A/B against the previous library, rocprof, bench, rehearsal.
set -u
T=${1:-r01s}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
: parity done in r01s

: > $OUT/${T}_ab.jsonl
for r in 1 2; do
  run ab-base-$r 300 bash -c "FJAGG_LIB=tools/_ab/libfjagg_base.so python tools/ab_kernels.py base >> $OUT/${T}_ab.jsonl 2>> $OUT/${T}_ab.err"
  run ab-new-$r 300 bash -c "python tools/ab_kernels.py new >> $OUT/${T}_ab.jsonl 2>> $OUT/${T}_ab.err"
done
cat $OUT/${T}_ab.jsonl
run rocprof-ab 300 rocprofv3 --kernel-trace --stats -d $OUT/${T}_prof_ab -o run --output-format csv -- python tools/ab_kernels.py new
run bench 300 bash -c "python bench.py > $OUT/${T}_bench.json 2> $OUT/${T}_bench.err"
cat $OUT/${T}_bench.json
: > $OUT/${T}_rehearse.jsonl
for n in 8 4; do
  run "rehearse-$n" 300 bash -c "python bench.py --rehearse-shard $n --steps 50 --warmup 10 >> $OUT/${T}_rehearse.jsonl 2>> $OUT/${T}_rehearse.err"
done
grep '^{' $OUT/${T}_rehearse.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); c=d['config']; print(c['clients_per_gpu'], c['exchange_engine'], c['buckets'], d['ms_per_step'], c['exchange_autotune_ms'])"
