#!/bin/bash
# Burst/interleaved fold schedules: full GPU suite, bucket probe vs the previous library,
# pytree/compression A/B, rocprof of the bench, bench, shard rehearsal.
set -u
T=${1:-r01t}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu-tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${T}_gpu_tests.log 2>&1"
tail -1 $OUT/${T}_gpu_tests.log
F=$OUT/${T}_probe_bucket.jsonl; : > $F
for K in 128 1024; do
  run pb-base-$K 200 bash -c "FJAGG_LIB=tools/_ab/libfjagg_base.so python tools/probe_bucket.py base $K >> $F"
  run pb-new-$K 200 bash -c "python tools/probe_bucket.py new $K >> $F"
done
: > $OUT/${T}_ab.jsonl
for r in 1 2; do
  run ab-base-$r 300 bash -c "FJAGG_LIB=tools/_ab/libfjagg_base.so python tools/ab_kernels.py base >> $OUT/${T}_ab.jsonl 2>> $OUT/${T}_ab.err"
  run ab-new-$r 300 bash -c "python tools/ab_kernels.py new >> $OUT/${T}_ab.jsonl 2>> $OUT/${T}_ab.err"
done
run rocprof-ab-base 300 env FJAGG_LIB=tools/_ab/libfjagg_base.so rocprofv3 --kernel-trace --stats -d $OUT/${T}_prof_ab_base -o run --output-format csv -- python tools/ab_kernels.py base
run rocprof-ab-new 300 rocprofv3 --kernel-trace --stats -d $OUT/${T}_prof_ab_new -o run --output-format csv -- python tools/ab_kernels.py new
run bench 300 bash -c "python bench.py > $OUT/${T}_bench.json 2> $OUT/${T}_bench.err"
cat $OUT/${T}_bench.json
run rocprof-bench 300 rocprofv3 --kernel-trace --stats -d $OUT/${T}_prof_bench -o run --output-format csv -- python bench.py --no-cpu-baseline
: > $OUT/${T}_rehearse.jsonl
for n in 8 4 2; do
  run "rehearse-$n" 300 bash -c "python bench.py --rehearse-shard $n --steps 50 --warmup 10 >> $OUT/${T}_rehearse.jsonl 2>> $OUT/${T}_rehearse.err"
done
