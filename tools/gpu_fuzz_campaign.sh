#!/bin/bash
# A longer fuzz campaign on one GPU box over seeds the suite does not run: tree_mean /
# mean_aggregator cases (tests/test_gpu_fuzz.py) and running-sum programs in both modes
# (tests/test_gpu_running_sum_fuzz.py), every case against the oracle, and standalone lazy-norm
# programs (tests/test_gpu_lazy_norms_fuzz.py).
# usage (repo root, on the box): bash tools/gpu_fuzz_campaign.sh TAG SEED0 CASES_MEAN CASES_SUM [CASES_NORM]
set -u
TAG=${1:-fuzz}; SEED0=${2:-50000}; CM=${3:-2000}; CS=${4:-1500}; CN=${5:-1000}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
FJ_FUZZ_SEED0=$SEED0 FJ_FUZZ_CASES=$CM timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -q -rf \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k random_case > "$O/mean.log" 2>&1
rc1=$?; tail -5 "$O/mean.log"; [ $rc1 -le 1 ] || exit $rc1
FJ_FUZZ_SEED0=$SEED0 FJ_FUZZ_CASES=$CS timeout -k 10 500 python -u -m pytest tests/test_gpu_running_sum_fuzz.py -q -rf \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/sum.log" 2>&1
rc2=$?; tail -5 "$O/sum.log"; [ $rc2 -le 1 ] || exit $rc2
FJ_FUZZ_SEED0=$SEED0 FJ_FUZZ_CASES=$CN timeout -k 10 500 python -u -m pytest tests/test_gpu_lazy_norms_fuzz.py -q -rf \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/norms.log" 2>&1
rc3=$?; tail -5 "$O/norms.log"
m=$(( rc1 > rc2 ? rc1 : rc2 ))
exit $(( m > rc3 ? m : rc3 ))
