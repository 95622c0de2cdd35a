#!/bin/bash
# Exchange auto-tune over reduce and all_reduce: N=2 gloo rehearsal (two ranks on one GPU)
# and the one-GPU N=8 shard rehearsal on the native RCCL engine (world 1).
set -u
T=${1:-r01zf}
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run rehearse-n2 300 bash -c "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $OUT/${T}_rehearse_n2_gloo.json 2> $OUT/${T}_rehearse_n2_gloo.err"
cat $OUT/${T}_rehearse_n2_gloo.json; grep -h auto-tune $OUT/${T}_rehearse_n2_gloo.err || true
run shard-n8 300 bash -c "python bench.py --rehearse-shard 8 --steps 50 --warmup 10 > $OUT/${T}_shard_rehearsal_n8.json 2> $OUT/${T}_shard_rehearsal_n8.err"
cat $OUT/${T}_shard_rehearsal_n8.json
