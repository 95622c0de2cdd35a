"""Host side of the compression path (no GPU): the key schedule in libfjagg.so
against the oracle restatement and the Random123 KATs, the Walsh-Hadamard tiling
mirror, table layouts and the arithmetic-coding bit count."""

import ctypes

import numpy as np
import numpy.testing as npt
import pytest

from fedjax_amd import _compress as C
from fedjax_amd import _lib, random
from oracle import compression_ref as cref
from oracle import jax_random_ref as jr


@pytest.mark.parametrize("key,ctr,expect", [
    ((0, 0), (0, 0), (0x6b200159, 0x99ba4efe)),
    ((0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff), (0x1cb996fc, 0xbb002be7)),
    ((0x13198a2e, 0x03707344), (0x243f6a88, 0x85a308d3), (0xc4923a9c, 0x483df7a0)),
])
def test_library_threefry_kat(key, ctr, expect):
    k = np.array(key, np.uint32)
    x0, x1 = np.array([ctr[0]], np.uint32), np.array([ctr[1]], np.uint32)
    y0, y1 = np.empty(1, np.uint32), np.empty(1, np.uint32)
    _lib.call("fjcomp_threefry2x32", k.ctypes.data, x0.ctypes.data, x1.ctypes.data, 1, y0.ctypes.data,
              y1.ctypes.data)
    assert (int(y0[0]), int(y1[0])) == expect


def test_library_threefry_matches_oracle_bulk():
    rs = np.random.RandomState(0)
    k = rs.randint(0, 2 ** 32, 2, dtype=np.uint64).astype(np.uint32)
    x0 = rs.randint(0, 2 ** 32, 1000, dtype=np.uint64).astype(np.uint32)
    x1 = rs.randint(0, 2 ** 32, 1000, dtype=np.uint64).astype(np.uint32)
    y0, y1 = np.empty_like(x0), np.empty_like(x1)
    _lib.call("fjcomp_threefry2x32", k.ctypes.data, x0.ctypes.data, x1.ctypes.data, 1000, y0.ctypes.data,
              y1.ctypes.data)
    e0, e1 = jr.threefry2x32(k, x0, x1)
    npt.assert_array_equal(y0, e0)
    npt.assert_array_equal(y1, e1)


@pytest.mark.parametrize("seed", [0, 1, 42, (3 << 32) | 7])
@pytest.mark.parametrize("num", [1, 2, 3, 8, 17])
def test_split_matches_oracle(seed, num):
    npt.assert_array_equal(random.split(random.PRNGKey(seed), num), jr.split(jr.prng_key(seed), num))


def test_split_many_and_sequence():
    keys = jr.split(jr.prng_key(5), 6)
    got = random.split_many(keys, 4)
    for i in range(6):
        npt.assert_array_equal(got[i], jr.split(keys[i], 4))
    seq, ref = random.PRNGSequence(random.PRNGKey(11)), jr.PRNGSequence(jr.prng_key(11))
    batch = seq.take(5)
    for i in range(5):
        npt.assert_array_equal(batch[i], next(ref))
    npt.assert_array_equal(next(seq), next(ref))  # state carried across calls
    assert random.PRNGSequence(11).take(1).tolist() == random.PRNGSequence(random.PRNGKey(11)).take(1).tolist()


def test_bad_key_shape():
    with pytest.raises(ValueError):
        random.split(np.zeros(3, np.uint32))


@pytest.mark.parametrize("m", list(range(0, 35)))
def test_wht_tiling_mirror(m):
    lib = _lib.load()
    passes = C.wht_passes(m)
    assert passes == (1 if m <= 13 else 1 + -(-(m - 13) // 8))
    covered = 0
    for p in range(passes + 1):
        assert C.wht_tiles(m, p) == lib.fjcomp_wht_tiles(m, p), (m, p)
    for p in range(passes):
        lo, nb = C.wht_pass_bits(m, p)
        assert lo == covered  # passes take the butterfly bits in increasing order
        covered += nb
        c = min(1 << lo, 8192 >> nb)
        assert C.wht_tiles(m, p) * (c << nb) == 1 << m  # each pass covers the vector once
        assert p == 0 or c >= 32 or (1 << lo) == c  # later passes read >= 128-byte segments
    assert covered == m


def test_padded_size_and_sqrt():
    assert [C.padded_size(n) for n in (1, 2, 3, 5, 18432, 1179648)] == [1, 2, 4, 8, 32768, 2097152]
    assert [C.padded_size(n) for n in (1, 2, 3, 5, 18432, 1179648)] == [cref.padded_size(n) for n in
                                                                         (1, 2, 3, 5, 18432, 1179648)]
    with pytest.raises(ValueError):
        C.padded_size(0)
    assert C.sqrt_f32(2) == float(np.sqrt(np.float32(2)))
    with pytest.raises(ValueError):
        C.log2_exact(12)


def test_table_layouts_match_header():
    assert C.WHT_JOB.itemsize == 72 and C.SIGN_JOB.itemsize == 24 and C.ROW.itemsize == 16
    assert C.QPARAMS.itemsize == 24 and C.STATS.itemsize == 48
    assert C.WHT_JOB.fields["kind"][1] == 60 and C.WHT_JOB.fields["sqrt_d"][1] == 64


@pytest.mark.parametrize("vals", [[1., 2., 3., 4., 5.], [1., 1., 2.], [0.5] * 7, [3., -1., 3., 3., 0., -1.]])
def test_arithmetic_bits_from_counts_matches_oracle(vals):
    v = np.array(vals, np.float32)
    _, counts = np.unique(v, return_counts=True)
    assert C.arithmetic_bits_from_counts(counts, v.size) == cref.arithmetic_encoding_num_bits(v)


def test_qparams_host():
    q = C.qparams_host(-1.0, 3.0)[0]
    assert q["vmin"] == -1 and q["vmax"] == 3 and q["range"] == 4 and q["rcp_range"] == 0.25


def test_host_argument_validation():
    lib = _lib.load()
    assert lib.fjcomp_random_split(None, -1, 2, None) == -1
    assert lib.fjcomp_quant_fold(9, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 1.0, 0, 1, None, None) == -1
    assert b"unknown method" in lib.fjagg_last_error()
    assert lib.fjcomp_quant_fold(1, 1, 1, 1, 1, 0, 1, 1, 1, 1, 2, 1.0, 0, 1, None, None) == -1
    assert lib.fjcomp_row_stats(1, 1, 2, 1, 0, 1, None, None, 0, None) == -1  # nchunks < R
    assert lib.fjcomp_random_bits(0, 0, 1 << 33, None, None) == -1
    tiles = (ctypes.c_int64 * 1)(0)
    assert lib.fjcomp_wht(None, None, 1, 1, tiles, None) == -1


def _arith_bits_rowwise(H, Q, K, leaf_n, num_levels):
    """Per-(client, leaf) restatement: level values -> np.unique merge -> oracle bit count."""
    f32 = np.float32
    L = len(leaf_n)
    qv = (np.arange(num_levels, dtype=f32) / f32(num_levels - 1)).astype(f32)
    out = []
    for k in range(K):
        bits = 0
        for l in range(L):
            q = Q[k * L + l]
            with np.errstate(all="ignore"):
                vals = (q["vmin"] + (qv * q["range"]).astype(f32)).astype(f32)
            vals = cref.nan_to_num(np.concatenate([vals, [f32(np.nan)]]).astype(f32))
            cnt = H[k * L + l]
            nz = cnt > 0
            uniq, inv = np.unique(vals[nz], return_inverse=True)
            merged = np.zeros(uniq.size, dtype=np.int64)
            np.add.at(merged, inv.reshape(-1), cnt[nz])
            bits = bits + cref.arithmetic_bits_from_counts(merged, int(leaf_n[l]))
        out.append(f32(bits))
    return out


@pytest.mark.parametrize("num_levels", [2, 3, 16])
def test_arithmetic_bits_vectorised_matches_rowwise(num_levels):
    rs = np.random.RandomState(num_levels)
    K, leaf_n = 37, [32, 288, 64, 18432, 128, 1179648, 62, 7936]
    L = len(leaf_n)
    R = K * L
    Q = np.zeros(R, dtype=C.QPARAMS)
    Q["vmin"] = rs.standard_normal(R).astype(np.float32)
    Q["range"] = np.abs(rs.standard_normal(R)).astype(np.float32)
    Q["range"][::7] = 0.0  # constant rows: every level collapses onto vmin
    Q["vmin"][::11] = np.inf  # NaN level values after the range product
    Q["vmin"][::13] = 0.0  # a level equal to the NaN bin's 0
    H = rs.randint(0, 50, size=(R, num_levels + 1)).astype(np.int64)
    H[rs.rand(R, num_levels + 1) < 0.3] = 0
    H[::5, :] = 0
    H[::5, 0] = 9  # single occupied bin
    got = C.arithmetic_bits_host(H, Q, K, leaf_n, num_levels)
    want = _arith_bits_rowwise(H, Q, K, leaf_n, num_levels)
    assert np.array_equal(np.array(got, np.float32).view(np.uint32), np.array(want, np.float32).view(np.uint32))


@pytest.mark.parametrize("num_levels", [2, 16])
def test_arithmetic_bits_fast_path_matches_rowwise(num_levels):
    """No NaN-bin counts and strictly increasing levels: the compaction fast path."""
    rs = np.random.RandomState(100 + num_levels)
    K, leaf_n = 29, [32, 288, 64, 18432, 128, 1179648, 62, 7936]
    R = K * len(leaf_n)
    Q = np.zeros(R, dtype=C.QPARAMS)
    Q["vmin"] = rs.standard_normal(R).astype(np.float32)
    Q["range"] = (np.abs(rs.standard_normal(R)) + 0.1).astype(np.float32)
    H = rs.randint(0, 50, size=(R, num_levels + 1)).astype(np.int64)
    H[rs.rand(R, num_levels + 1) < 0.3] = 0
    H[:, -1] = 0
    H[::5, :] = 0
    H[::5, 0] = 9
    got = C.arithmetic_bits_host(H, Q, K, leaf_n, num_levels)
    want = _arith_bits_rowwise(H, Q, K, leaf_n, num_levels)
    assert np.array_equal(np.array(got, np.float32).view(np.uint32), np.array(want, np.float32).view(np.uint32))


def test_wht_jobs_vectorised_matches_single():
    d = np.array([32, 512, 2 ** 21], dtype=np.int64)
    j = C.wht_jobs(np.array([[1, 2, 3]], np.uint64) * 16, 64, [5 * 16, 6 * 16, 7 * 16], d[None, :],
                   kind=2, n_in=[30, 300, 2 ** 20 + 1], signs=np.array([[8, 9, 10]], np.uint64) * 16)
    for i in range(3):
        one = C.wht_job(16 * (i + 1), 64, 16 * (5 + i), int(d[i]), kind=2, n_in=[30, 300, 2 ** 20 + 1][i],
                        signs=16 * (8 + i))
        assert j[i].tobytes() == one[0].tobytes()
    assert list(j["log2d"]) == [5, 9, 21] and j["sqrt_d"][2] == np.float32(np.sqrt(np.float32(2 ** 21)))
