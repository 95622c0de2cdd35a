#!/bin/bash
# PMC traffic of the examples/fed_avg.py round per mode (tools/pmc_example_round.py), one
# counter per rocprofv3 pass. usage (repo root, on the box): bash tools/gpu_pmc_example.sh TAG
set -u
O=gpurun_out/${1:-r06_pmc_example}
mkdir -p "$O"
export TMPDIR=/tmp
for m in norms eager mean_only; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/$m/fetch" -o run --output-format csv -- \
    python tools/pmc_example_round.py $m > "$O/$m.fetch.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/$m/write" -o run --output-format csv -- \
    python tools/pmc_example_round.py $m > "$O/$m.write.log" 2>&1 || exit 1
  python tools/pmc_example_round.py --summarize "$O/$m/fetch" "$O/$m/write" 10 > "$O/$m.json" || exit 1
  echo "$m $(cat $O/$m.json)"
done
