#!/bin/bash
# A/B of two libfjagg.so builds on tools/probe_l2_ab.py (pytree K=128/64 and dense, plain and
# fused-norm folds), alternating builds pass by pass on one box.
# usage (repo root, on the box): bash tools/ab_lib_l2.sh OUT BASE_SO [PASSES]
O=$1; BASE=$2; N=${3:-3}
mkdir -p "$O"
for p in $(seq 1 "$N"); do
  for lib in "$BASE" fedjax_amd/_build/libfjagg.so; do
    FJAGG_LIB=$lib timeout -k 10 200 python tools/probe_l2_ab.py 200 5 > "$O/tmp.jsonl" || exit $?
    sed "s|^|lib=$lib pass=$p |" "$O/tmp.jsonl" >> "$O/ab.jsonl"
  done
done
rm -f "$O/tmp.jsonl"
