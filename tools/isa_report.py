"""Summarise kernels in a hipcc -S device assembly file: loads, VGPR/SGPR, spills.

usage: python tools/isa_report.py fjagg.s [substring-of-demangled-name ...]
"""
import re
import subprocess
import sys


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    s = open(path).read()
    names = re.findall(r"^(_Z\S+):\s*;", s, re.M)
    dem = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True).stdout.split("\n")
    for n, d in zip(names, dem):
        if pats and not all(p in d for p in pats):
            continue
        start = s.index(n + ":")
        body = s[start:s.index(".Lfunc_end", start)]
        lines = body.splitlines()
        meta_i = s.find(".amdhsa_kernel " + n)
        meta = s[meta_i:s.find(".end_amdhsa_kernel", meta_i)]
        get = lambda k: (re.search(r"\." + k + r"\s+(\d+)", meta) or [None, "?"])[1]
        gl = [l.strip() for l in lines if "global_load" in l or "buffer_load" in l]
        print(d)
        print("  vgpr(next_free)=%s sgpr=%s scratch=%s  global/buffer loads=%d  s_load=%d  waitcnt=%d" % (
            get("amdhsa_next_free_vgpr"), get("amdhsa_next_free_sgpr"),
            get("amdhsa_private_segment_fixed_size"), len(gl),
            sum("s_load" in l for l in lines), sum("s_waitcnt" in l for l in lines)))
        for l in gl[:3]:
            print("   ", l)


if __name__ == "__main__":
    main()
