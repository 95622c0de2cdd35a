#!/bin/bash
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 lim=$2 a1=$3; shift 3; timeout -k 10 "$lim" "$@"; local rc=$?; echo "[$name] rc=$rc"; if [ $rc -eq 0 ] || { [ $a1 = 1 ] && [ $rc -eq 1 ]; }; then return 0; fi; exit $rc; }
run gpu-tests 900 1 bash -c "python -m pytest tests -q -m gpu -rf -x > $OUT/r01_gpu_tests_s10.log 2>&1"
tail -4 $OUT/r01_gpu_tests_s10.log
run prof-pytree 600 0 rocprofv3 --kernel-trace --stats -d $OUT/r01_prof_pytree -o run --output-format csv -- python tools/time_pytree.py
cut -c1-80,220- $OUT/r01_prof_pytree/run_kernel_stats.csv
grep -h "k_ptrs" $OUT/r01_prof_pytree/run_kernel_trace.csv | awk -F'","' '{print $0}' | python3 -c "
import sys,csv
rows=list(csv.reader(open('$OUT/r01_prof_pytree/run_kernel_trace.csv')))
h=rows[0]; i=h.index('Kernel_Name'); s=h.index('Start_Timestamp'); e=h.index('End_Timestamp'); g=h.index('Grid_Size_X')
d=[(int(r[e])-int(r[s]), int(r[g])) for r in rows[1:] if 'k_ptrs' in r[i]]
small=[x for x in d if x[0]<1e6]; big=[x for x in d if x[0]>=1e6]
import statistics as st
print('ptrs c2 launches', len(small), 'median us', st.median([x[0] for x in small])/1e3 if small else None, 'grid', small[0][1] if small else None)
print('ptrs c3 launches', len(big), 'median ms', st.median([x[0] for x in big])/1e6 if big else None, 'grid', big[0][1] if big else None)
"
