# k_ptrs placement counter study (tools/probe_ptrs_pmc.py): kernel trace + 3 PMC passes per mode
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r02e
for m in views clones rows2m bigseg; do
  timeout -s KILL 90 rocprofv3 --kernel-trace -d $O/${m}_trace -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 20 > $O.$m.log 2>&1 || { echo "trace $m failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d $O/${m}_pmcA -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O.$m.log 2>&1 || { echo "pmcA $m failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d $O/${m}_pmcB -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O.$m.log 2>&1 || { echo "pmcB $m failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum -d $O/${m}_pmcC -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O.$m.log 2>&1 || { echo "pmcC $m failed"; exit 1; }
  echo "$m done"
done
for m in views clones rows2m bigseg; do mkdir -p $O/$m; for p in trace pmcA pmcB pmcC; do mv $O/${m}_$p $O/$m/$p; done; done
python tools/pmc_table.py k_ptrs $O/table.json $O/views $O/clones $O/rows2m $O/bigseg
