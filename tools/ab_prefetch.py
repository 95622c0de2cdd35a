"""A/B of fjhost's leaf prefetch in tree_weight's capture (FJHOST_PREFETCH): the capture parts
over 128 clients and the library loop's per-client tree_weight cost, in two processes per pass."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for on in ("1", "0"):
        env = dict(os.environ, FJHOST_PREFETCH=on)
        for tool in ("prof_capture_parts.py", "prof_library_loop.py"):
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool)], env=env, capture_output=True,
                                 text=True, timeout=600)
            print(f"prefetch={on} pass={p} {tool} {out.stdout.strip()}", flush=True)
            if out.returncode:
                print(out.stderr[-2000:])
                sys.exit(1)
