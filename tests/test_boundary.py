"""The C-ABI boundary: library loads, exports exactly what include/fjagg.h declares,
binds to torch's HIP runtime, validates arguments on the host; the product
package never touches the oracle. No GPU needed."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

from fedjax_amd import _lib, kernels

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("fjagg.h", "fjcomp.h", "fjcomm.h", "fjtree.h", "fjopt.h",
                                                           "fjalloc.h")]


def header_symbols():
    syms = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        syms |= set(re.findall(r"\b(fj(?:agg|comp|comm|tree|opt|alloc)_\w+)\s*\(", src))
    return syms


def test_header_and_binding_agree():
    assert header_symbols() == set(_lib.SYMBOLS)


def test_flag_values_match_the_header():
    """The ctypes layer's flag constants are fjagg.h's `enum fjagg_flags` values."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADERS[0]).read(), flags=re.S)
    enum = re.search(r"enum fjagg_flags \{(.*?)\};", src, re.S).group(1)
    values = {name: 1 << int(bit) for name, bit in re.findall(r"FJAGG_(\w+)\s*=\s*1\s*<<\s*(\d+)", enum)}
    assert values == {n: getattr(_lib, n) for n in values}
    assert set(values) == {"SCALE", "ACCUMULATE", "NONTEMPORAL", "UNALIGNED", "UNBALANCED", "NARROW", "HOST_TABLES",
                           "ZEROED_WS"}


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (fj(?:agg|comp|comm|tree|opt|alloc)_\w+)", out))
    assert header_symbols() <= exported, header_symbols() - exported


def test_hip_imports_resolve_in_torch_runtime():
    und = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    need = {m.split("@")[0] for m in re.findall(r"U (\S*hip\S*)", und)}
    torch_hip = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    have = subprocess.run(["nm", "-D", "--defined-only", torch_hip], capture_output=True, text=True,
                          check=True).stdout
    defined = {m.split("@")[0] for m in re.findall(r"\bT (\S+)", have)}
    assert need and need <= defined, need - defined


def test_loads_with_one_hip_runtime():
    lib = _lib.load()
    assert lib.fjagg_abi_version() == _lib.ABI_VERSION
    assert len(_lib.hip_runtimes_mapped()) == 1


def test_host_side_validation_without_gpu():
    lib = _lib.load()
    # bad dtype combination is rejected before any HIP call
    rc = lib.fjagg_wsum_dense(_lib.F32, _lib.I32, _lib.F32, 16, 4, 1, 4, 16, 1.0, 16, 0, 0, None, 0, None)
    assert rc == -3 and b"unsupported" in lib.fjagg_last_error()
    rc = lib.fjagg_wsum_dense(_lib.F32, _lib.F32, _lib.F32, 16, 4, 0, 4, 16, 1.0, 16, 0, 0, None, 0, None)
    assert rc == -1 and b"K must be" in lib.fjagg_last_error()
    rc = lib.fjagg_wsum_dense(_lib.I32, _lib.I32, _lib.I32, 16, 4, 2, 4, 16, 1.0, 16, _lib.SCALE, 0, None, 0, None)
    assert rc == -1
    rc = lib.fjagg_wsum_dense(_lib.F32, _lib.F32, _lib.F32, 16, 4, 2, 8, 16, 1.0, 16, 0, 0, None, 0, None)
    assert rc == -1 and b"ld" in lib.fjagg_last_error()
    with pytest.raises(_lib.FjaggError):
        _lib.call("fjagg_wsum_ptrs", _lib.F32, _lib.F32, _lib.F32, None, 1, 1, 5, None, 1.0, 0, None)


def test_host_tables_refused_before_any_launch():
    """FJAGG_HOST_TABLES launches the library does not build are refused on the host with
    FJAGG_EUNSUPPORTED (the callers then upload the tables); no GPU call happens first."""
    lib = _lib.load()
    w = np.ones(2000, np.float32)
    dense = [  # (in, acc, out, K, P, mode, flags)
        (_lib.F32, _lib.F32, _lib.F32, 2000, 200_000, 0, 0),           # K > FJAGG_KARG_MAX_WEIGHTS
        (_lib.F32, _lib.F32, _lib.F32, 64, 20_000, 0, 0),              # the narrow kernel's shape
        (_lib.F32, _lib.F32, _lib.F32, 64, 200_000, 1, 0),             # split mode
        (_lib.F32, _lib.F32, _lib.F32, 64, 200_000, 0, 1 << 8),        # a tuning variant
        (_lib.I32, _lib.I32, _lib.I32, 64, 200_000, 0, 0),             # integer fold
        (_lib.BF16, _lib.BF16, _lib.BF16, 64, 200_000, 0, 0),          # bf16 reference fold
        (_lib.F32, _lib.F32, _lib.BF16, 64, 200_000, 0, 0),
    ]
    for in_c, acc, out_c, K, P, mode, fl in dense:
        rc = lib.fjagg_wsum_dense(in_c, acc, out_c, 16, P, K, P, w.ctypes.data, 1.0, 16, fl | _lib.HOST_TABLES, mode,
                                  None, 0, None)
        assert rc == -3 and b"HOST_TABLES" in lib.fjagg_last_error(), (in_c, acc, out_c, K, P, mode, fl)
    img = np.zeros(64, np.int64)
    for in_c, out_c, fl in ((_lib.BF16, _lib.BF16, 0), (_lib.F32, _lib.F32, _lib.NARROW),
                            (_lib.F32, _lib.F32, _lib.UNALIGNED)):
        rc = lib.fjagg_wsum_ptrs(in_c, _lib.F32, out_c, img.ctypes.data, 2, 4, 3, w.ctypes.data, 1.0,
                                 fl | _lib.HOST_TABLES, None)
        assert rc == -3, (in_c, fl)
    assert lib.fjagg_karg_image_words(128, 8, 256) == 128 * 8 + 16 + 512 + 64
    assert lib.fjagg_karg_image_words(4000, 1, 10) > _lib.KARG_MAX_WORDS
    rc = lib.fjagg_wsum_ptrs(_lib.F32, _lib.F32, _lib.F32, img.ctypes.data, 1, 4000, 10, w.ctypes.data, 1.0,
                             _lib.HOST_TABLES, None)
    assert rc == -3 and b"words" in lib.fjagg_last_error()


def test_split_workspace_sizing():
    assert kernels.split_workspace_bytes(1024, 4 * 1024 * 1024) == 0  # exact path fills the chip
    ws = kernels.split_workspace_bytes(1024, 16384)
    assert ws > 0 and ws % 256 == 0


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "fedjax_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
    code = "import sys; sys.path.insert(0, %r); import fedjax_amd, fedjax_amd.distributed; " \
           "print(any(m == 'oracle' or m.startswith('oracle.') for m in sys.modules))" % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout
    assert out.strip() == "False"


def test_reference_api_surface():
    import fedjax_amd
    # fedjax/core/tree_util.py:29-133 public functions
    for name in ["tree_weight", "tree_inverse_weight", "tree_zeros_like", "tree_add", "tree_sum",
                 "tree_mean", "tree_size", "tree_l2_squared", "tree_l2_norm", "tree_clip_by_global_norm"]:
        assert callable(getattr(fedjax_amd.tree_util, name)), name
    # fedjax/aggregators/aggregator.py:26-75
    for name in ["Aggregator", "MeanAggregatorState", "mean_aggregator"]:
        assert hasattr(fedjax_amd.aggregators, name), name
    assert callable(fedjax_amd.dataclass)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_fails_loudly_without_gpu():
    import fedjax_amd
    with pytest.raises(_lib.FjaggError):
        fedjax_amd.tree_util.tree_mean([({"w": np.ones(3, np.float32)}, 1)])
    with pytest.raises(_lib.FjaggError):
        fedjax_amd.aggregators.mean_aggregator().apply([("a", {"w": np.ones(3, np.float32)}, 2.)], None)


def test_comm_host_side_validation_without_gpu():
    lib = _lib.load()
    assert lib.fjcomm_abi_version() == _lib.COMM_ABI_VERSION
    rc = lib.fjcomm_sharded_wsum_dense(None, _lib.F32, 16, 4, 1, 4, 16, 1.0, 16, 1, 0, 0, None, None)
    assert rc == -1  # FJAGG_EINVAL
    assert b"communicator" in lib.fjagg_last_error()
    assert lib.fjcomm_init(None, None, 1, 0) in (-1, -3)  # null handle / RCCL absent
    assert lib.fjcomm_destroy(None) == 0


def test_tree_table_layout_and_validation():
    """include/fjtree.h: the ctypes mirror has the C layout (static_assert in fjtree.hip), and
    bad tables are refused before any HIP call."""
    import ctypes
    assert ctypes.sizeof(_lib.TreeLeaves) == 2104
    lib = _lib.load()
    t = _lib.TreeLeaves()
    t.K, t.L = 3, 1
    assert lib.fjtree_fold_leaves(ctypes.byref(t), None) == -1 and b"K must be" in lib.fjagg_last_error()
    t.K, t.L = 1, 65
    assert lib.fjtree_fold_leaves(ctypes.byref(t), None) == -1
    t.L, t.n[0] = 1, 10
    assert lib.fjtree_fold_leaves(ctypes.byref(t), None) == -1 and b"null operand" in lib.fjagg_last_error()
    t.flags = _lib.TREE_NORM
    assert lib.fjtree_workspace_bytes(ctypes.byref(t)) == 256 + 4
    t.n[0] = 4097
    assert lib.fjtree_workspace_bytes(ctypes.byref(t)) == 256 + 8


def test_multi_device_entry_points_validate_without_gpu():
    """include/fjcomm.h single-process entry points refuse bad arguments before any HIP or
    RCCL work (no GPU here)."""
    import ctypes
    lib = _lib.load()
    h = (ctypes.c_void_p * 2)()
    assert lib.fjcomm_init_all(h, 0, (ctypes.c_int * 1)(0)) != 0
    assert lib.fjcomm_init_all(h, 2, (ctypes.c_int * 2)(0, 0)) != 0  # a device listed twice
    assert lib.fjcomm_init_all(None, 1, (ctypes.c_int * 1)(0)) != 0
    vp = ctypes.c_void_p * 1
    i64 = ctypes.c_int64 * 1
    rc = lib.fjcomm_multi_wsum_dense(None, 1, _lib.F32, vp(16), i64(4), i64(1), 4, vp(16), 1.0, vp(16),
                                     None, 1, 0, 0, vp(0))
    assert rc == -1 and b"null argument" in lib.fjagg_last_error()
    rc = lib.fjcomm_multi_wsum_dense(h, 1, _lib.F32, vp(16), i64(4), i64(1), 4, vp(16), 1.0, vp(16),
                                     None, 1, 0, 0, vp(0))
    assert rc == -1 and b"not an initialised communicator" in lib.fjagg_last_error()
    rc = lib.fjcomm_multi_wsum_dense(h, 0, _lib.F32, vp(16), i64(4), i64(1), 4, vp(16), 1.0, vp(16),
                                     None, 1, 0, 0, vp(0))
    assert rc == -1 and b"ndev" in lib.fjagg_last_error()


def test_host_constants_match_headers():
    """Constants the Python host shares with the C ABI are the headers' values."""
    from fedjax_amd import _compress as C

    text = open(os.path.join(ROOT, "include", "fjcomp.h")).read()
    defines = dict(re.findall(r"#define (FJCOMP_\w+) (\d+)", text))
    assert int(defines["FJCOMP_SIGN_BLOCK_PAIRS"]) == C.SIGN_BLOCK
