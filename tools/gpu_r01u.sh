#!/bin/bash
# Current build: PMC HBM traffic of the configs[2] fold, configs[1] slab bench, configs[4] per-GPU shard.
set -u
T=${1:-r01u}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run pmc-fetch 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/${T}_pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run pmc-write 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/${T}_pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run traffic 60 python tools/pmc_summary.py $OUT/${T}_pmc_fetch $OUT/${T}_pmc_write $OUT/${T}_traffic_c3.json
cat $OUT/${T}_traffic_c3.json
run bench-c2 300 bash -c "python bench.py --workload c2 --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${T}_bench_c2.json 2> $OUT/${T}_bench_c2.err"
cat $OUT/${T}_bench_c2.json
run bench-c5s 600 bash -c "python bench.py --workload c5s --steps 5 --warmup 2 > $OUT/${T}_bench_c5s.json 2> $OUT/${T}_bench_c5s.err"
cat $OUT/${T}_bench_c5s.json
