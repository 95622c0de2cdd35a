#!/bin/bash
# Bucket-width probe of the dense fold for several library builds (tools/probe_bucket.py).
set -u
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
F=$OUT/${1:-r01s}_probe_bucket.jsonl
: > $F
for K in 128 1024; do
  for r in 1 2; do
    run pb-base 200 bash -c "FJAGG_LIB=tools/_ab/libfjagg_base.so python tools/probe_bucket.py base $K >> $F"
    run pb-new 200 bash -c "python tools/probe_bucket.py new $K >> $F"
    run pb-sb 200 bash -c "FJAGG_LIB=tools/_ab/libfjagg_sb.so python tools/probe_bucket.py sb $K >> $F"
  done
done
cat $F
