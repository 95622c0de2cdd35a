mkdir -p gpurun_out/r03s
for r in 1 2 3; do for fb in 268435456 1073741824 134217728; do
CPROF=0 timeout -k 10 120 python tools/cprof_library_loop.py $fb 2>/dev/null | grep round_ms || exit 1
done; done
