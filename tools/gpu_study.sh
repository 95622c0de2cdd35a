#!/bin/bash
# GPU-box studies behind DESIGN.md's numbers (run from the repo root on the box):
#   bash tools/gpu_study.sh STUDY
# STUDY:
#   tree_ops      per-call tree-op tests, literal running-sum loop host costs and timing,
#                 rocprofv3 kernel stats of the loop                   (profiles/r02c_*)
#   placement     k_ptrs by leaf placement: kernel trace + UTCL1 / UTCL2 / TCC PMC passes
#                                                                      (profiles/r02e_ptrs_placement)
#   quant         k_quant_fold VALU counters                           (profiles/r02h_*)
#   narrow        k_dense_narrow parity + variant sweep on narrow shapes (profiles/r02i_*)
#   narrow_tree   k_ptrs_narrow vs k_ptrs on small models (FJAGG_NARROW_MAX_BYTES A/B, profiles/r02k_*)
#   ptrs_u        k_ptrs at configs[1] with 4 / 8 / 16 clients in flight (FJAGG_PTRS_U, an experiment build
#                 of k_ptrs not kept in the tree; profiles/r02n_ptrs_u)
#   karg          FJAGG_HOST_TABLES: parity tests, tree_mean wall at configs[1], bench c2 / c3 / N=8 shard
#                 rehearsal with kernel-argument weights vs uploaded weights, kernel trace of the
#                 tree_mean loop                                       (profiles/r02r_*)
#   delta_pool    fjalloc modes, k_ptrs per segment stagger with UTCL1 / TCC tag-stall counters
#                                                                      (profiles/r04m_delta_pool)
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -u
STUDY=${1:?study name}
O=gpurun_out/study_$STUDY
mkdir -p "$O"
export TMPDIR=/tmp
die() { echo "$1 failed"; exit 1; }
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
case "$STUDY" in
  tree_ops)
    timeout -k 10 300 $PT tests/test_gpu_tree_ops.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
    timeout -k 10 300 python tools/prof_literal_loop.py > $O/loop.json 2> $O/loop.err || die loop
    timeout -k 10 300 python tools/time_running_mean.py > $O/time.json 2> $O/time.err || die time
    cat $O/loop.json $O/time.json
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
      python tools/prof_literal_loop.py > $O/prof.log 2>&1 || die rocprof
    rm -f $O/prof/run_kernel_trace.csv
    ;;
  placement)
    for m in ${MODES:-views clones rows2m bigseg expseg}; do
      timeout -s KILL 90 rocprofv3 --kernel-trace -d $O/$m/trace -o run --output-format csv -- \
        python tools/probe_ptrs_pmc.py $m 20 > $O/$m.log 2>&1 || die "trace $m"
      timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
        TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d $O/$m/pmcA -o run --output-format csv -- \
        python tools/probe_ptrs_pmc.py $m 10 >> $O/$m.log 2>&1 || die "pmcA $m"
      timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum \
        TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE \
        -d $O/$m/pmcB -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O/$m.log 2>&1 || die "pmcB $m"
      timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum \
        -d $O/$m/pmcC -o run --output-format csv -- python tools/probe_ptrs_pmc.py $m 10 >> $O/$m.log 2>&1 || die "pmcC $m"
    done
    python tools/pmc_table.py k_ptrs $O/table.json $(for m in ${MODES:-views clones rows2m bigseg expseg}; do echo $O/$m; done)
    ;;
  quant)
    B="python tools/bench_compression.py --only uniform,terngrad --rounds 3 --warmup 1 --cpu-sample 0"
    timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/comp/trace -o run --output-format csv -- $B > $O.log 2>&1 || die trace
    timeout -s KILL 120 rocprofv3 --pmc VALUBusy VALUUtilization -d $O/comp/pmc1 -o run --output-format csv -- $B >> $O.log 2>&1 || die pmc1
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
      GRBM_GUI_ACTIVE -d $O/comp/pmc2 -o run --output-format csv -- $B >> $O.log 2>&1 || die pmc2
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_ACTIVE_INST_VALU -d $O/comp/pmc3 -o run --output-format csv -- $B >> $O.log 2>&1 || die pmc3
    python tools/pmc_table.py k_quant_fold $O/table.json $O/comp
    ;;
  narrow)
    timeout -k 10 300 $PT tests/test_gpu_parity.py -k "variants_bitwise or narrow_fold or golden or split or bf16" \
      > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
    for s in "1024 65536 f32" "4096 16384 f32" "512 131072 f32" "256 262144 f32" "2048 32768 f32" "64 65536 f32" \
             "16384 4096 f32" "1024 131072 bf16" "4096 32768 bf16" "1024 4194304 f32"; do
      SWEEP_VARIANTS=0,2,18 timeout -k 10 120 python tools/sweep.py $s 3 5 || die "sweep $s"
    done > $O/sweep.jsonl
    cat $O/sweep.jsonl
    ;;
  narrow_tree)
    for m in 262144 0; do
      FJAGG_NARROW_MAX_BYTES=$m timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/max_$m -o run \
        --output-format csv -- python tools/time_narrow_pytree.py > $O/max_$m.jsonl 2>&1 || die "narrow $m"
      rm -f $O/max_$m/run_kernel_trace.csv
      grep '^{' $O/max_$m.jsonl
    done
    ;;
  ptrs_u)
    for u in 4 8 16; do
      for m in views clones; do
        FJAGG_PTRS_U=$u timeout -s KILL 90 rocprofv3 --kernel-trace -d $O/u${u}_$m -o run --output-format csv -- \
          python tools/probe_ptrs_pmc.py $m 30 > $O/u${u}_$m.log 2>&1 || die "trace u$u $m"
      done
    done
    python tools/pmc_table.py k_ptrs $O/table.json $O/u4_views $O/u4_clones $O/u8_views $O/u8_clones \
      $O/u16_views $O/u16_clones | grep -E '"u|duration'
    ;;
  karg)
    timeout -k 10 600 $PT tests/test_gpu_host_tables.py tests/test_gpu_distributed.py tests/test_boundary.py \
      > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python tools/time_pytree.py > $O/time_pytree.jsonl 2> $O/time_pytree.err || die time_pytree
    cat $O/time_pytree.jsonl
    for wl in c2 c3; do
      for dw in "" "--device-weights"; do
        timeout -k 10 300 python bench.py --workload $wl --steps 50 --warmup 10 --no-cpu-baseline $dw \
          > $O/bench_${wl}${dw:+_dw}.json 2> $O/bench_${wl}${dw:+_dw}.err || die "bench $wl $dw"
      done
    done
    for dw in "" "--device-weights"; do
      timeout -k 10 300 python bench.py --rehearse-shard 8 --steps 50 --warmup 10 --buckets 1 $dw \
        > $O/shard8${dw:+_dw}.json 2> $O/shard8${dw:+_dw}.err || die "shard8 $dw"
    done
    grep -h -o '"ms_per_step": [0-9.]*\|"workload": "[^"]*"\|"weights_path": [^}]*}\|"mean_launch_ms": [0-9.]*' \
      $O/bench_*.json $O/shard8*.json
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- \
      python tools/time_pytree.py > $O/trace.log 2>&1 || die trace
    ;;
  c5_rehearse)
    # configs[4]: rank 0's share (1024 of 8192 clients x 125 M bf16) through the full sharded
    # step on a world-1 RCCL communicator: fold -> f32 partial -> reduce -> bf16 cast
    timeout -k 10 900 python bench.py --workload c5 --rehearse-shard 8 --steps ${STEPS:-10} --warmup 3 \
      > $O/c5_rehearse.json 2> $O/c5_rehearse.err || die c5_rehearse
    cat $O/c5_rehearse.json
    ;;
  narrow_pmc)
    # k_dense_narrow (variant 18) counters at the two verdict shapes; SQ / GRBM / TCC in separate passes
    for s in "16384 4096" "4096 16384"; do
      n=$(echo $s | tr ' ' x)
      B="python tools/sweep.py $s f32 1 5"
      SWEEP_VARIANTS=${NARROW_VARIANTS:-18} timeout -s KILL 90 rocprofv3 --kernel-trace -d $O/$n/trace -o run \
        --output-format csv -- $B > $O/$n.log 2>&1 || die "trace $n"
      SWEEP_VARIANTS=${NARROW_VARIANTS:-18} timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
        SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY \
        -d $O/$n/pmcA -o run --output-format csv -- $B >> $O/$n.log 2>&1 || die "pmcA $n"
      SWEEP_VARIANTS=${NARROW_VARIANTS:-18} timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE \
        -d $O/$n/pmcB -o run --output-format csv -- $B >> $O/$n.log 2>&1 || die "pmcB $n"
      SWEEP_VARIANTS=${NARROW_VARIANTS:-18} timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS \
        SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU \
        -d $O/$n/pmcC -o run --output-format csv -- $B >> $O/$n.log 2>&1 || die "pmcC $n"
      python tools/pmc_table.py ${NARROW_KERNEL:-k_dense_narrow} $O/table_$n.json $O/$n/trace $O/$n/pmcA \
        $O/$n/pmcB $O/$n/pmcC > /dev/null
    done
    cat $O/table_*.json
    ;;
  stripe)
    # k_dense_stripe (variants 19-22) parity, then the narrow-shape sweep against k_dense_narrow (18)
    timeout -k 10 600 $PT tests/test_gpu_parity.py -k "stripe or variants_bitwise or narrow_fold" \
      > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
    for s in "16384 4096 f32" "4096 16384 f32" "2048 32768 f32" "1024 65536 f32" "512 131072 f32" \
             "256 262144 f32" "4096 32768 bf16" "1024 4096 f32" "128 16384 f32" "65536 1024 f32" \
             "64 65536 f32" "16 65536 f32" "32 16384 f32" "8192 8192 f32" "1024 131072 bf16" "256 32768 f32"; do
      SWEEP_BALANCED_ONLY=1 SWEEP_VARIANTS=${SWEEP_VARIANTS:-2,18,19,20,21,22} timeout -k 10 120 \
        python tools/sweep.py $s 3 5 || die "sweep $s"
    done > $O/sweep.jsonl
    cat $O/sweep.jsonl
    ;;
  r03tests)
    # round-3 GPU tests: inference tensors, server ignore/schedules, norm combine orders, configs[4] share
    timeout -k 10 900 $PT tests/test_gpu_inference_tensors.py tests/test_gpu_server_ext.py \
      tests/test_gpu_tree_ops.py -k "norm_combine or data_writes or chain_budget or f32_in_bf16 or inference \
      or ignore or schedule or frozen or configs4_rank0" tests/test_gpu_parity.py \
      "tests/test_gpu_fullsize.py::test_configs4_rank0_share_native_pipeline" > $O/tests.log 2>&1
    rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit 1
    ;;
  stripe_tree)
    # k_ptrs_stripe parity, then tree_mean over small models with many clients: stripe vs narrow
    timeout -k 10 900 $PT tests/test_gpu_parity.py -k "ptrs_stripe or narrow or golden" tests/test_gpu_fuzz.py \
      > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
    for sp in 0 1; do
      for mx in 262144 524288; do
        FJAGG_STRIPE_PYTREE=$sp FJAGG_NARROW_MAX_BYTES=$mx timeout -k 10 300 python tools/time_narrow_pytree.py \
          > $O/time_sp${sp}_max${mx}.jsonl 2> $O/time_sp${sp}_max${mx}.err || die "time sp=$sp max=$mx"
      done
    done
    grep -H . $O/time_*.jsonl
    ;;
  delta_pool)
    # fjalloc placement (DESIGN §3 "Caller-side placement", profiles/r04m_delta_pool): k_ptrs on
    # default / pooled / slab-view leaves per segment stagger (FJALLOC_STAGGER_KIB), kernel trace +
    # UTCL1 and TCC tag-stall counters, and the allocator modes (tools/probe_fjalloc.py)
    timeout -k 10 300 python tools/probe_fjalloc.py > $O/fjalloc.jsonl 2> $O/fjalloc.err || die fjalloc
    for st in ${STAGGERS:-0 4 68 260}; do
      FJALLOC_STAGGER_KIB=$st timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/s$st/trace -o run \
        --output-format csv -- python tools/probe_delta_pool.py clones,pool,views 20 > $O/s$st.log 2>&1 || die "trace $st"
      python tools/pool_table.py $O/s$st/trace $O/s$st/trace $O/s$st/table.json || die "table $st"
      rm -f $O/s$st/trace/run_kernel_trace.csv
    done
    FJALLOC_STAGGER_KIB=68 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCC_TAG_STALL_sum \
      -d $O/s68/pmc -o run --output-format csv -- python tools/probe_delta_pool.py clones,pool,views 10 \
      > $O/s68_pmc.log 2>&1 || die pmc
    python tools/pool_table.py $O/s68/trace $O/s68/pmc $O/s68/table_pmc.json
    ;;
  *) echo "unknown study $STUDY"; exit 2 ;;
esac
