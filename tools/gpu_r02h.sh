# k_quant_fold counters: kernel trace + 3 PMC passes over the compression bench
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r02h
B="python tools/bench_compression.py --only uniform,terngrad --rounds 3 --warmup 1 --cpu-sample 0"
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/comp/trace -o run --output-format csv -- $B > $O.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc VALUBusy VALUUtilization -d $O/comp/pmc1 -o run --output-format csv -- $B >> $O.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $O/comp/pmc2 -o run --output-format csv -- $B >> $O.log 2>&1 || { echo pmc2 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $O/comp/pmc3 -o run --output-format csv -- $B >> $O.log 2>&1 || { echo pmc3 failed; exit 1; }
python tools/pmc_table.py k_quant_fold $O/table.json $O/comp > /dev/null && cat $O/table.json
