# A/B of the translation warm-up in k_ptrs (FJAGG_PTRS_PREFETCH) over leaf placements
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r02f
for r in 1 0; do
  for m in views clones rows2m bigseg; do
    FJAGG_PTRS_PREFETCH=$r timeout -s KILL 90 rocprofv3 --kernel-trace -d $O/r${r}_${m}/trace -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 30 > $O.log 2>&1 || { echo "trace $r $m failed"; exit 1; }
    FJAGG_PTRS_PREFETCH=$r timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_THRASHING_STALL_sum -d $O/r${r}_${m}/pmcA -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O.log 2>&1 || { echo "pmcA $r $m failed"; exit 1; }
    FJAGG_PTRS_PREFETCH=$r timeout -s KILL 90 rocprofv3 --pmc TCC_TAG_STALL_sum GRBM_UTCL2_BUSY -d $O/r${r}_${m}/pmcC -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O.log 2>&1 || { echo "pmcC $r $m failed"; exit 1; }
  done
done
python tools/pmc_table.py k_ptrs $O/table.json $O/r1_views $O/r1_clones $O/r1_rows2m $O/r1_bigseg $O/r0_views $O/r0_clones $O/r0_rows2m $O/r0_bigseg | python -c "
import json,sys
d=json.load(open('$O/table.json'))
for k,v in d.items(): print(k, round(v.get('duration_us_median',0),2), v.get('TCP_UTCL1_TRANSLATION_MISS_sum'), v.get('TCC_TAG_STALL_sum'), v.get('GRBM_UTCL2_BUSY'))
"
