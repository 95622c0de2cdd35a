#!/bin/bash
# PMC traffic passes + N=2 gloo rehearsal + config-2 pytree timing + E2E rate.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run pmc-fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/r01_pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run pmc-write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/r01_pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
python tools/pmc_summary.py $OUT/r01_pmc_fetch $OUT/r01_pmc_write $OUT/traffic_c3.json
run pytree-c2 300 bash -c "python tools/time_pytree.py > $OUT/r01_pytree_c2.json 2> $OUT/r01_pytree_c2.err"
cat $OUT/r01_pytree_c2.json
run bench-c2 300 bash -c "python bench.py --workload c2 --no-cpu-baseline > $OUT/r01_bench_c2.json 2> $OUT/r01_bench_c2.err"
cat $OUT/r01_bench_c2.json
run rehearse-n2 600 bash -c "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --all-ranks --steps 5 --warmup 2 > $OUT/r01_rehearse_n2.json 2> $OUT/r01_rehearse_n2.err"
cat $OUT/r01_rehearse_n2.json
run e2e 900 bash -c "python bench.py --e2e --steps 5 --warmup 2 --no-cpu-baseline > $OUT/r01_bench_e2e.json 2> $OUT/r01_bench_e2e.err"
cat $OUT/r01_bench_e2e.json
