"""The per-call fused norm's cross-workgroup combine in the compiled ISA (VERDICT r2 next #6,
DESIGN.md §3d). fjtree.hip's k_leaves<.., NORM> hands each workgroup's partial to the last
workgroup in one of two forms (include/fjtree.h):

* default, the gfx950 hand-off (MI355X guide, Guideline 16 R1): the partial is an sc1
  (write-through) store, the storing wave drains it (``s_waitcnt vmcnt(0)``) before the
  relaxed counter add, and the last workgroup reads the partials with sc1 loads;
* FJTREE_ORDERED: the counter add is an acquire-release RMW (``buffer_wbl2`` before,
  ``buffer_inv`` after): ordered by the HIP memory model.

The default form is ordered by the hardware, not by the language, so a compiler change
could break it silently; this test reads the .s the build produces and checks the order
of those instructions on every norm kernel. CPU only (hipcc cross-compiles gfx950)."""
import os
import re
import shutil
import subprocess

import pytest

from fedjax_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def fjtree_asm(tmp_path_factory):
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "fjtree.s"
    import __graft_entry__ as g
    flags = [f for f in g.HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
    subprocess.run([HIPCC, *flags, "--cuda-device-only", "-S", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "fedjax_amd", "csrc", "fjtree.hip"), "-o", str(out)],
                   check=True, capture_output=True, timeout=300)
    return out.read_text()


def kernels_with_norm(asm):
    """{mangled name: body} of every k_leaves<K, OUT, NORM = true> kernel."""
    out = {}
    for m in re.finditer(r"^(_ZN\S*k_leavesILi(\d)ELb(\d)ELb1E\S*):", asm, re.M):
        start = m.end()
        out[m.group(1)] = asm[start:asm.index(".Lfunc_end", start)]
    return out


def code_lines(body):
    return [ln.strip() for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", "."))]


def test_default_handoff_order_in_isa(fjtree_asm):
    ks = kernels_with_norm(fjtree_asm)
    assert len(ks) >= 3, list(ks)
    for name, body in ks.items():
        lines = code_lines(body)
        adds = [i for i, ln in enumerate(lines) if ln.startswith("global_atomic_add")]
        assert len(adds) == 2, (name, "one counter add per combine form")
        stores = [i for i, ln in enumerate(lines)
                  if ln.startswith("global_store_dword") and ln.endswith("sc1") and i < adds[0]]
        assert stores, (name, "the partial is an sc1 (write-through) store before the count")
        st = stores[-1]

        def window(i):  # the instructions since the previous store / add, up to add i
            j = max([st] + [a for a in adds if a < i])
            return lines[j + 1:i]

        ordered_add = [i for i in adds if any(ln.startswith("buffer_wbl2") for ln in window(i))]
        handoff_add = [i for i in adds if i not in ordered_add]
        assert len(ordered_add) == 1 and len(handoff_add) == 1, name
        # the handoff path: no release fence between the partial and its count, but a drain
        h = handoff_add[0]
        assert any(re.match(r"s_waitcnt vmcnt\(0\)", ln) for ln in window(h)), (
            name, "partial drained (s_waitcnt vmcnt(0)) before the counter add")
        # the ordered path: release before its add, acquire invalidate after it
        o = ordered_add[0]
        assert any(ln.startswith("buffer_inv") for ln in lines[o:o + 6]), (name, "acquire after the ordered add")
        # the last workgroup reads the partials with sc1 loads only, after both adds
        loads = [ln for ln in lines[max(adds):] if ln.startswith("global_load")]
        assert loads and all(ln.endswith("sc1") for ln in loads), (name, loads)


def test_ordered_flag_matches_header():
    text = open(os.path.join(ROOT, "include", "fjtree.h")).read()
    defines = dict(re.findall(r"#define (FJTREE_\w+) \(1 << (\d+)\)", text))
    assert 1 << int(defines["FJTREE_ORDERED"]) == _lib.TREE_ORDERED
    assert 1 << int(defines["FJTREE_NORM"]) == _lib.TREE_NORM
