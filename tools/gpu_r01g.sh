#!/bin/bash
# Kernel timeline of the 8-way shard rehearsal at 1 and 4 buckets.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for b in 1 4; do
run "prof-b$b" 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/r01g_b$b -o run --output-format csv -- python bench.py --rehearse-shard 8 --buckets $b --steps 10 --warmup 3 --no-cpu-baseline
done
