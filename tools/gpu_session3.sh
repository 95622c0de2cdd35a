#!/bin/bash
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run probe2 900 bash -c "python tools/probe2.py > $OUT/r01_probe2.jsonl 2> $OUT/r01_probe2.err"
cat $OUT/r01_probe2.jsonl
run pytree-c2 300 bash -c "python tools/time_pytree.py > $OUT/r01_pytree_c2b.json 2> $OUT/r01_pytree_c2b.err"
cat $OUT/r01_pytree_c2b.json
