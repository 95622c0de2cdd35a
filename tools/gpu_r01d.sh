#!/bin/bash
# N=2 gloo rehearsal of the bucket auto-tune + compression round timings and kernel breakdown.
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run rehearse-n2 300 bash -c "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --all-ranks --steps 5 --warmup 2 > $OUT/r01d_rehearse_n2.json 2> $OUT/r01d_rehearse_n2.err"
cat $OUT/r01d_rehearse_n2.json; grep -h auto-tune $OUT/r01d_rehearse_n2.err || true
run comp-bench 600 bash -c "python tools/bench_compression.py > $OUT/r01d_comp_bench.jsonl 2> $OUT/r01d_comp_bench.err"
cat $OUT/r01d_comp_bench.jsonl
run comp-prof 600 rocprofv3 --kernel-trace --stats -d $OUT/r01d_comp_prof -o run --output-format csv -- python tools/bench_compression.py --rounds 3 --warmup 1 --cpu-sample 0
cut -c1-160 $OUT/r01d_comp_prof/run_kernel_stats.csv
