"""A/B of k_ptrs' XCD-aware plan order (fjagg.hip xcd_plan_index,
FJAGG_XCD_REMAP): run tools/probe_l2_ab.py's pytree case in two processes, with and without
the reservation, interleaved, and print both JSON lines per pass."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for p in range(passes):
    for on in ("1", "0"):
        env = dict(os.environ, FJAGG_XCD_REMAP=on)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_l2_ab.py"), "200", "5"],
                             env=env, capture_output=True, text=True, timeout=600)
        for line in out.stdout.splitlines():
            if "pytree" in line:
                print(f"xcd_remap={on} pass={p} {line}", flush=True)
        if out.returncode:
            print(out.stderr[-2000:], flush=True)
            sys.exit(out.returncode)
