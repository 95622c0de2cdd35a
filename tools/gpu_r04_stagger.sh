#!/bin/bash
# fjalloc mode-2 segment stagger A/B: k_ptrs kernel trace + UTCL1 counters per stagger.
# usage (repo root, on the box): bash tools/gpu_r04_stagger.sh TAG
set -u
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for st in 0 68 4 260; do
  FJALLOC_STAGGER_KIB=$st timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/s$st/trace" -o run \
    --output-format csv -- python tools/probe_delta_pool.py clones,pool,views 20 > "$O/s$st.log" 2>&1 || exit $?
  grep '"mode"' "$O/s$st.log"
  python tools/pool_table.py "$O/s$st/trace" "$O/s$st/trace" "$O/s$st/table.json" || exit $?
  rm -f "$O"/s$st/trace/*/run_kernel_trace.csv.gz
done
FJALLOC_STAGGER_KIB=68 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCC_TAG_STALL_sum \
  -d "$O/s68/pmc" -o run --output-format csv -- python tools/probe_delta_pool.py clones,pool,views 10 \
  > "$O/s68_pmc.log" 2>&1 || exit $?
python tools/pool_table.py "$O/s68/trace" "$O/s68/pmc" "$O/s68/table_pmc.json"
echo done
