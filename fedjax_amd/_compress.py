"""Launch engine of the compression-aggregator kernels (include/fjcomp.h).

Builds the (client, leaf) tables the kernels walk, uploads them in one pinned H2D
copy per launch group, and strings the launches together for the three round
shapes of ``fedjax/aggregators/compression.py``:

* ``quantized_mean``   stats -> quantize + fold          (uniform, binary, terngrad)
* ``rotated_quantized_mean``  shared rotation per leaf: signs -> WHT -> stats ->
                       quantize + fold in the rotated domain -> ONE inverse WHT of
                       the mean (the rotation is linear and identical for every
                       client, compression.py:241-251, so the per-client inverses of
                       the reference commute with the weighted mean)
* ``drive_mean``       per-client rotation: signs -> WHT -> sums -> DRIVE + inverse
                       WHT -> dense fold (compression.py:298-308)

Everything is asynchronous on torch's current stream; only the arithmetic-coding
bit count (``hist=True``) reads results back. Device work is batched over clients
to a workspace budget so HBM holds K rotated deltas only when it fits.
"""

from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from fedjax_amd import _lib, tree_util

ROW = np.dtype([("ptr", "<u8"), ("n", "<i8")])
SIGN_JOB = np.dtype([("k0", "<u4"), ("k1", "<u4"), ("d", "<i8"), ("words", "<u8")])
WHT_JOB = np.dtype([("src", "<u8"), ("mid", "<u8"), ("dst", "<u8"), ("signs", "<u8"), ("stats", "<u8"),
                    ("n_in", "<i8"), ("n_out", "<i8"), ("log2d", "<i4"), ("kind", "<i4"),
                    ("sqrt_d", "<f4"), ("flags", "<i4")])
WHT_F_SUMS = 1  # FJCOMP_WHT_F_SUMS (include/fjcomp.h)
QPARAMS = np.dtype([("vmin", "<f4"), ("vmax", "<f4"), ("range", "<f4"), ("thr", "<f4"), ("rcp_range", "<f8")])
STATS = np.dtype([("min", "<f8"), ("max", "<f8"), ("absmax", "<f8"), ("sum", "<f8"), ("sumsq", "<f8"),
                  ("sumabs", "<f8")])
assert ROW.itemsize == 16 and SIGN_JOB.itemsize == 24 and WHT_JOB.itemsize == 72
assert QPARAMS.itemsize == 24 and STATS.itemsize == 48

WHT_BITS = 13       # butterfly bits of pass 0
WHT_HIGH_BITS = 8   # butterfly bits of each later pass
WHT_MAX_LOG2 = 34
QBLOCK = 256  # k_quant_fold threads (element pairs) per workgroup
SIGN_BLOCK = 8192  # FJCOMP_SIGN_BLOCK_PAIRS (include/fjcomp.h): the largest share
SIGN_MIN_BLOCKS = 2048  # k_rademacher workgroups wanted before the share grows (8 per CU)
DEFAULT_WORKSPACE_BYTES = 4 << 30


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class Upload:
    """Host tables packed 16-byte aligned into one pinned buffer, copied once."""

    def __init__(self):
        self._parts: List[Tuple[int, np.ndarray]] = []
        self._size = 0
        self.dev: Optional[torch.Tensor] = None

    def add(self, arr: np.ndarray) -> int:
        off = (self._size + 15) & ~15
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        self._parts.append((off, b))
        self._size = off + b.size
        return off

    def commit(self, device: torch.device) -> int:
        host = np.zeros(max(self._size, 16), dtype=np.uint8)
        for off, b in self._parts:
            host[off:off + b.size] = b
        self.dev = _lib.upload(torch.from_numpy(host), device)
        return self.dev.data_ptr()


# ----------------------------------------------------------------------------- tiling
def log2_exact(d: int) -> int:
    m = int(d).bit_length() - 1
    if d < 1 or (1 << m) != d:
        raise ValueError(f"Walsh-Hadamard length must be a power of two, got {d}")
    return m


def padded_size(n: int) -> int:
    """walsh_hadamard.py:142: ``2 ** ceil(log2(n))``."""
    if n < 1:
        raise ValueError("cannot rotate an empty leaf (the reference fails on log2(0))")
    return 1 << (int(n) - 1).bit_length()


def wht_passes(m: int) -> int:
    return 1 if m <= WHT_BITS else 1 + -(-(m - WHT_BITS) // WHT_HIGH_BITS)


def wht_pass_bits(m: int, p: int) -> Tuple[int, int]:
    """(lo, nb): pass p does butterfly bits [lo, lo + nb)."""
    lo = 0 if p == 0 else WHT_BITS + WHT_HIGH_BITS * (p - 1)
    return lo, max(0, min(WHT_BITS if p == 0 else WHT_HIGH_BITS, m - lo))


def wht_tiles(m: int, p: int) -> int:
    """Tiles of pass p of a 2^m job (mirror of wht_tiling in fjcomp.hip)."""
    if p >= wht_passes(m):
        return 0
    lo, nb = wht_pass_bits(m, p)
    c = min(1 << lo, (1 << WHT_BITS) >> nb)
    return (1 << m) // (c << nb)


def sqrt_f32(d: int) -> float:
    """``jnp.sqrt(d)`` for a Python int d: f32(sqrt(f32(d))), correctly rounded."""
    return float(np.sqrt(np.float32(d)))


# ----------------------------------------------------------------------------- launches
def row_stats(rows: Sequence[Tuple[int, int]], method: int, device: torch.device,
              want_qparams: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Stats (and quantizer parameters) of rows given as (device pointer, n)."""
    return row_stats_table([p for p, _ in rows], [n for _, n in rows], method, device, want_qparams)


def row_stats_table(ptrs, ns, method: int, device: torch.device,
                    want_qparams: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """:func:`row_stats` with the row pointers and lengths as arrays."""
    ns = np.asarray(ns, dtype=np.int64).reshape(-1)
    R = ns.size
    tab = np.empty(R, dtype=ROW)
    tab["ptr"] = np.asarray(ptrs, dtype=np.uint64).reshape(-1)
    tab["n"] = ns
    if (ns < 1).any():
        raise ValueError("quantizing an empty leaf: the reference fails on amin/amax of an empty array")
    chunks = np.maximum(1, (ns + _lib.STATS_CHUNK - 1) // _lib.STATS_CHUNK)
    prefix = np.zeros(R + 1, dtype=np.int64)
    np.cumsum(chunks, out=prefix[1:])
    nchunks = int(prefix[-1])
    up = Upload()
    o_rows, o_pre = up.add(tab), up.add(prefix)
    base = up.commit(device)
    stats = torch.empty(R * STATS.itemsize, dtype=torch.uint8, device=device)
    qp = torch.empty(R * QPARAMS.itemsize, dtype=torch.uint8, device=device) if want_qparams else None
    ws_bytes = int(_lib.load().fjcomp_row_stats_workspace_bytes(nchunks))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=device)
    _lib.call("fjcomp_row_stats", base + o_rows, base + o_pre, R, nchunks, method, stats.data_ptr(),
              None if qp is None else qp.data_ptr(), ws.data_ptr(), ws_bytes, _stream(device))
    return stats, qp


def stats_from_partials(ptrs, ns, part_prefix: np.ndarray, part: torch.Tensor, method: int,
                        device: torch.device, want_qparams: bool = True):
    """Min / max stats and qparams of rows whose per-tile partials a ROTATE WHT wrote into
    ``part`` (row r: partials part_prefix[r] .. part_prefix[r+1]-1)."""
    ns = np.asarray(ns, dtype=np.int64).reshape(-1)
    R = ns.size
    tab = np.empty(R, dtype=ROW)
    tab["ptr"] = np.asarray(ptrs, dtype=np.uint64).reshape(-1)
    tab["n"] = ns
    up = Upload()
    o_rows, o_pre = up.add(tab), up.add(np.ascontiguousarray(part_prefix, dtype=np.int64))
    base = up.commit(device)
    stats = torch.empty(R * STATS.itemsize, dtype=torch.uint8, device=device)
    qp = torch.empty(R * QPARAMS.itemsize, dtype=torch.uint8, device=device) if want_qparams else None
    _lib.call("fjcomp_stats_combine", base + o_rows, base + o_pre, R, method, part.data_ptr(), stats.data_ptr(),
              None if qp is None else qp.data_ptr(), _stream(device))
    return stats, qp, up


def _last_pass_tiles(leaf_d: np.ndarray) -> np.ndarray:
    """Tiles of each power-of-two job's last WHT pass (its partials slots)."""
    return np.array([wht_tiles(int(d).bit_length() - 1, wht_passes(int(d).bit_length() - 1) - 1) for d in leaf_d],
                    dtype=np.int64)


def qparams_host(vmin: float, vmax: float) -> np.ndarray:
    """Quantizer parameters for explicitly given v_min / v_max (compression.py:58-61)."""
    q = np.zeros(1, dtype=QPARAMS)
    lo, hi = np.float32(vmin), np.float32(vmax)
    rng = np.float32(hi - lo)
    q["vmin"], q["vmax"], q["range"] = lo, hi, rng
    with np.errstate(divide="ignore"):
        q["rcp_range"] = np.float64(1.0) / np.float64(rng)
    return q


def quant_fold(method: int, in_ptrs: np.ndarray, keys: np.ndarray, qparams_ptr: int, w: np.ndarray,
               leaf_n: np.ndarray, out_ptrs: np.ndarray, device: torch.device, *, num_levels: int = 2,
               scale: Optional[float] = None, accumulate: bool = False,
               hist: Optional[torch.Tensor] = None) -> None:
    """k_quant_fold over in_ptrs [K, L] with keys [K, L, 2] and weights w [K]."""
    K, L = in_ptrs.shape
    leaf_n = np.ascontiguousarray(leaf_n, dtype=np.int64)
    blocks = ((leaf_n + 1) // 2 + QBLOCK - 1) // QBLOCK
    prefix = np.concatenate([[0], np.cumsum(blocks)]).astype(np.int64)
    up = Upload()
    o_in = up.add(np.ascontiguousarray(in_ptrs, dtype=np.uint64))
    o_keys = up.add(np.ascontiguousarray(keys, dtype=np.uint32))
    o_w = up.add(np.ascontiguousarray(w, dtype=np.float32))
    o_n = up.add(leaf_n)
    o_pre = up.add(prefix)
    o_out = up.add(np.ascontiguousarray(out_ptrs, dtype=np.uint64))
    base = up.commit(device)
    flags = (_lib.SCALE if scale is not None else 0) | (_lib.ACCUMULATE if accumulate else 0)
    _lib.call("fjcomp_quant_fold", method, base + o_in, base + o_keys, qparams_ptr, base + o_w, K, L, base + o_n,
              base + o_pre, int(prefix[-1]), int(num_levels), float(np.float32(scale if scale is not None else 1.0)),
              flags, base + o_out, None if hist is None else hist.data_ptr(), _stream(device))
    return up


def rademacher_words(keys: np.ndarray, ds: Sequence[int], device: torch.device,
                     block_pairs: int = 0) -> Tuple[torch.Tensor, np.ndarray]:
    """Sign bits for jobs (keys [J, 2], lengths ds): one word buffer, per-job word offsets.
    ``block_pairs`` (tests) forces the kernel's workgroup share instead of the sized one."""
    J = len(ds)
    ds = np.asarray(ds, dtype=np.int64)
    nwords = (ds + 31) // 32
    woff = np.concatenate([[0], np.cumsum(nwords)]).astype(np.int64)
    words = torch.empty(max(int(woff[-1]), 1), dtype=torch.int32, device=device)
    jobs = np.empty(J, dtype=SIGN_JOB)
    keys = np.asarray(keys, dtype=np.uint32).reshape(J, 2)
    jobs["k0"], jobs["k1"], jobs["d"] = keys[:, 0], keys[:, 1], ds
    jobs["words"] = words.data_ptr() + 4 * woff[:-1]
    # the largest workgroup share (power of two pairs, 256 .. SIGN_BLOCK) that still gives
    # every CU a few workgroups
    pairs = int(((ds + 1) // 2).sum())
    bp = SIGN_BLOCK
    while bp > 256 and pairs < bp * SIGN_MIN_BLOCKS:
        bp //= 2
    bp = block_pairs or bp
    blocks = ((ds + 1) // 2 + bp - 1) // bp
    prefix = np.concatenate([[0], np.cumsum(blocks)]).astype(np.int64)
    up = Upload()
    o_jobs, o_pre = up.add(jobs), up.add(prefix)
    base = up.commit(device)
    _lib.call("fjcomp_rademacher", base + o_jobs, base + o_pre, J, int(prefix[-1]), bp, _stream(device))
    return words, woff


def _tiles_by_pass(ms: np.ndarray) -> np.ndarray:
    """[npass, J] tile counts of every pass of 2^m jobs (evaluated once per distinct m)."""
    uniq, inv = np.unique(ms, return_inverse=True)
    npass = max(wht_passes(int(m)) for m in uniq)
    per_m = np.array([[wht_tiles(int(m), p) for m in uniq] for p in range(npass)], dtype=np.int64)
    return per_m[:, inv.reshape(-1)]


def run_wht(jobs: np.ndarray, device: torch.device) -> Upload:
    """Launch every pass of the WHT jobs (structured WHT_JOB array)."""
    J = len(jobs)
    if J == 0:
        return Upload()
    ms = jobs["log2d"].astype(np.int64)
    if (ms < 0).any() or (ms > WHT_MAX_LOG2).any():
        raise ValueError("Walsh-Hadamard length out of range")
    tiles = _tiles_by_pass(ms)
    npass = tiles.shape[0]
    pre = np.zeros((npass, J + 1), dtype=np.int64)
    np.cumsum(tiles, axis=1, out=pre[:, 1:])
    totals = np.ascontiguousarray(pre[:, -1])
    up = Upload()
    o_jobs, o_pre = up.add(jobs), up.add(pre)
    base = up.commit(device)
    _lib.call("fjcomp_wht", base + o_jobs, base + o_pre, J, npass, totals.ctypes.data, _stream(device))
    return up


def wht_jobs(src, mid, dst, d, *, kind: int, n_in=None, n_out=None, signs=0, stats=0, flags: int = 0) -> np.ndarray:
    """WHT_JOB table; every argument is a scalar or an array broadcast to the job count.
    d are the (power-of-two) transform lengths; n_in / n_out default to d."""
    cols = np.broadcast_arrays(*(np.asarray(a, dtype=np.uint64 if i < 3 or i > 5 else np.int64)
                                 for i, a in enumerate((src, mid, dst, d,
                                                        d if n_in is None else n_in,
                                                        d if n_out is None else n_out,
                                                        signs, stats))))
    src, mid, dst, d, n_in, n_out, signs, stats = (c.reshape(-1) for c in cols)
    ud, inv = np.unique(d, return_inverse=True)
    log2 = np.array([log2_exact(int(x)) for x in ud], dtype=np.int32)[inv.reshape(-1)]
    j = np.zeros(d.size, dtype=WHT_JOB)
    j["src"], j["mid"], j["dst"], j["signs"], j["stats"] = src, mid, dst, signs, stats
    j["n_in"], j["n_out"] = n_in, n_out
    j["log2d"], j["kind"], j["flags"] = log2, kind, flags
    j["sqrt_d"] = np.sqrt(d.astype(np.float32))  # jnp.sqrt(d): correctly rounded f32
    return j


def wht_job(src: int, mid: int, dst: int, d: int, *, kind: int, n_in: Optional[int] = None,
            n_out: Optional[int] = None, signs: int = 0, stats: int = 0) -> np.ndarray:
    return wht_jobs(src, mid, dst, d, kind=kind, n_in=n_in, n_out=n_out, signs=signs, stats=stats)


# ----------------------------------------------------------------------------- rounds
def _leaf_layout(leaf_n: Sequence[int]):
    ds = [padded_size(n) for n in leaf_n]
    offs = np.concatenate([[0], np.cumsum(ds)]).astype(np.int64)
    return ds, offs


def _batch_size(K: int, per_client_bytes: int, budget: int) -> int:
    return max(1, min(K, budget // max(per_client_bytes, 1)))


def quantized_mean(method: int, rows: List[List[torch.Tensor]], keys: np.ndarray, w: np.ndarray,
                   scale: Optional[float], outs: List[torch.Tensor], *, num_levels: int = 2,
                   hist: bool = False, qparams: Optional[torch.Tensor] = None):
    """outs[l] = [scale *] sum_k fl(Q(rows[k][l]) * w_k) (tree_mean over quantized
    deltas). Returns (hist tensor or None, qparams tensor)."""
    device = outs[0].device
    K, L = len(rows), len(rows[0])
    in_ptrs = tree_util._ptr_table(rows, np.uint64)
    leaf_n = np.array([x.numel() for x in rows[0]], dtype=np.int64)
    if qparams is None:
        _, qparams = row_stats_table(in_ptrs.reshape(-1), np.tile(leaf_n, K), method, device)
    h = None
    if hist:
        if K * L * (num_levels + 1) > (1 << 28):
            raise ValueError("arithmetic-coding histogram too large (K * leaves * (num_levels + 1) > 2^28)")
        h = torch.zeros(K * L * (num_levels + 1), dtype=torch.int32, device=device)
    out_ptrs = np.array([o.data_ptr() for o in outs], dtype=np.uint64)
    quant_fold(method, in_ptrs, keys, qparams.data_ptr(), w, leaf_n, out_ptrs, device, num_levels=num_levels,
               scale=scale, hist=h)
    return h, qparams


def rotated_quantized_mean(rows: List[List[torch.Tensor]], rot_keys: np.ndarray, client_keys: np.ndarray,
                           w: np.ndarray, scale: Optional[float], outs: List[torch.Tensor], *, num_levels: int,
                           workspace_bytes: int = DEFAULT_WORKSPACE_BYTES) -> None:
    """rotated_uniform_stochastic_quantizer's round (compression.py:238-256), inverse
    rotation applied once to the mean."""
    device = outs[0].device
    K, L = len(rows), len(rows[0])
    leaf_n = [x.numel() for x in rows[0]]
    ds, offs = _leaf_layout(leaf_n)
    D = int(offs[-1])
    signs, woff = rademacher_words(rot_keys, ds, device)
    sptr = [signs.data_ptr() + 4 * int(o) for o in woff[:-1]]
    acc = torch.empty(D, dtype=torch.float32, device=device)
    B = _batch_size(K, 4 * D, workspace_bytes)
    Y = torch.empty((B, D), dtype=torch.float32, device=device)
    leaf_d = np.array(ds, dtype=np.int64)
    leaf_n = np.asarray(leaf_n, dtype=np.int64)
    loff = 4 * offs[:-1].astype(np.uint64)
    sptr = np.asarray(sptr, dtype=np.uint64)
    src_all = tree_util._ptr_table(rows, np.uint64)
    # the rotation's last pass writes every tile's min / max (fjcomp_wht ROTATE partials), so
    # the quantizer constants need no separate pass over the rotated deltas
    last_tiles = _last_pass_tiles(leaf_d)
    part_slot = int(_lib.load().fjcomp_row_stats_workspace_bytes(1))
    part = torch.empty(max(B * int(last_tiles.sum()) * part_slot, 16), dtype=torch.uint8, device=device)
    keep = []
    for k0 in range(0, K, B):
        kb = min(B, K - k0)
        ybase = np.uint64(Y.data_ptr()) + np.uint64(4 * D) * np.arange(kb, dtype=np.uint64)[:, None]
        ydst = ybase + loff[None, :]  # [kb, L]
        pre = np.zeros(kb * L + 1, dtype=np.int64)
        np.cumsum(np.tile(last_tiles, kb), out=pre[1:])
        pptr = (np.uint64(part.data_ptr()) + np.uint64(part_slot) * pre[:-1].astype(np.uint64)).reshape(kb, L)
        keep.append(run_wht(wht_jobs(src_all[k0:k0 + kb], ydst, ydst, leaf_d[None, :], kind=_lib.WHT_ROTATE,
                                     n_in=leaf_n[None, :], signs=sptr[None, :], stats=pptr), device))
        _, qp, up = stats_from_partials(ydst.reshape(-1), np.broadcast_to(leaf_d, (kb, L)).reshape(-1), pre, part,
                                        _lib.COMP_UNIFORM, device)
        keep.append(up)
        out_ptrs = np.uint64(acc.data_ptr()) + loff
        last = k0 + kb == K
        keep.append(quant_fold(_lib.COMP_UNIFORM, ydst, client_keys[k0:k0 + kb], qp.data_ptr(), w[k0:k0 + kb],
                               leaf_d, out_ptrs, device, num_levels=num_levels,
                               scale=scale if last else None, accumulate=k0 > 0))
        keep.append(qp)
    accp = np.uint64(acc.data_ptr()) + loff
    keep.append(run_wht(wht_jobs(accp, accp, [o.data_ptr() for o in outs], leaf_d, kind=_lib.WHT_UNROTATE,
                                 n_out=leaf_n, signs=sptr), device))
    # keep the tables alive until the stream has consumed them (the caching allocator
    # reuses freed blocks only in stream order, so dropping them afterwards is safe)
    del keep


def drive_mean(rows: List[List[torch.Tensor]], client_keys: np.ndarray, w: np.ndarray, scale: Optional[float],
               out_flat: torch.Tensor, *, workspace_bytes: int = DEFAULT_WORKSPACE_BYTES) -> None:
    """structured_drive_quantizer's round (compression.py:292-308) into out_flat [P]
    (leaves concatenated in flatten order)."""
    from fedjax_amd import kernels  # local: kernels imports nothing from here

    device = out_flat.device
    K, L = len(rows), len(rows[0])
    leaf_n = [x.numel() for x in rows[0]]
    ds, offs = _leaf_layout(leaf_n)
    D = int(offs[-1])
    P = int(sum(leaf_n))
    loff = np.concatenate([[0], np.cumsum(leaf_n)]).astype(np.int64)
    Pp = (P + 3) // 4 * 4
    B = _batch_size(K, 4 * (D + Pp), workspace_bytes)
    Y = torch.empty((B, D), dtype=torch.float32, device=device)
    Z = torch.empty((B, Pp), dtype=torch.float32, device=device)
    # pinned + non_blocking: a pageable copy would make the host wait for the previous
    # round to drain and then leave the GPU idle while this round's tables are built
    w_dev = _lib.upload(torch.from_numpy(np.ascontiguousarray(w, dtype=np.float32)), device)
    leaf_n = np.asarray(leaf_n, dtype=np.int64)
    leaf_d = np.asarray(ds, dtype=np.int64)
    yoff = 4 * offs[:-1].astype(np.uint64)
    zoff = 4 * loff[:-1].astype(np.uint64)
    src_all = tree_util._ptr_table(rows, np.uint64)
    # the rotation's last pass writes every tile's sumsq / sumabs (f64) partials, so DRIVE's
    # scale needs no separate pass over the rotated deltas
    last_tiles = _last_pass_tiles(leaf_d)
    part_slot = int(_lib.load().fjcomp_row_stats_workspace_bytes(1))
    part = torch.empty(max(B * int(last_tiles.sum()) * part_slot, 16), dtype=torch.uint8, device=device)
    for k0 in range(0, K, B):
        kb = min(B, K - k0)
        signs, woff = rademacher_words(client_keys[k0:k0 + kb].reshape(-1, 2), ds * kb, device)
        sptr = (np.uint64(signs.data_ptr()) + 4 * woff[:-1].astype(np.uint64)).reshape(kb, L)
        bidx = np.arange(kb, dtype=np.uint64)[:, None]
        ydst = np.uint64(Y.data_ptr()) + np.uint64(4 * D) * bidx + yoff[None, :]
        zdst = np.uint64(Z.data_ptr()) + np.uint64(4 * Pp) * bidx + zoff[None, :]
        pre = np.zeros(kb * L + 1, dtype=np.int64)
        np.cumsum(np.tile(last_tiles, kb), out=pre[1:])
        pptr = (np.uint64(part.data_ptr()) + np.uint64(part_slot) * pre[:-1].astype(np.uint64)).reshape(kb, L)
        t1 = run_wht(wht_jobs(src_all[k0:k0 + kb], ydst, ydst, leaf_d[None, :], kind=_lib.WHT_ROTATE,
                              n_in=leaf_n[None, :], signs=sptr, stats=pptr, flags=WHT_F_SUMS), device)
        stats, _, t0 = stats_from_partials(ydst.reshape(-1), np.broadcast_to(leaf_d, (kb, L)).reshape(-1), pre,
                                           part, 0, device, want_qparams=False)
        sts = np.uint64(stats.data_ptr()) + np.uint64(STATS.itemsize) * np.arange(kb * L, dtype=np.uint64)
        t2 = run_wht(wht_jobs(ydst, ydst, zdst, leaf_d[None, :], kind=_lib.WHT_UNROTATE_DRIVE,
                              n_out=leaf_n[None, :], signs=sptr, stats=sts.reshape(kb, L)), device)
        last = k0 + kb == K
        kernels.weighted_sum_dense(Z[:kb, :P], w_dev[k0:k0 + kb], scale=scale if last else None, out=out_flat,
                                   accumulate=k0 > 0)
        del t0, t1, t2, signs, stats


# ----------------------------------------------------------------------------- bits
def _log2_f32(x: np.ndarray) -> np.ndarray:
    with np.errstate(divide="ignore", invalid="ignore"):
        return (np.log(x.astype(np.float32)) / np.log(np.float32(2))).astype(np.float32)


def arithmetic_bits_from_counts(counts: np.ndarray, d: int) -> np.float32:
    """compression.py:125-149 given the histogram of the d values' distinct values."""
    f32 = np.float32
    hist = np.asarray(counts, dtype=np.int64)
    k = hist.size
    p = (hist.astype(f32) / f32(hist.sum())).astype(f32)
    with np.errstate(divide="ignore", invalid="ignore"):
        ent = f32(-np.sum((p * _log2_f32(p)).astype(f32), dtype=f32))
        e = f32(np.exp(f32(1)))
        hist_bits = f32(f32(k) * _log2_f32(np.array([f32(f32(e * f32(d + k)) / f32(k))]))[0])
    return f32(f32(f32(hist_bits + f32(f32(d) * ent)) + f32(64)) + f32(2))


def arithmetic_bits(hist: torch.Tensor, qparams: torch.Tensor, K: int, leaf_n: Sequence[int],
                    num_levels: int) -> List[np.float32]:
    """Per-client bit counts (sum over leaves) from the level histograms: the level
    values are recomputed with the kernel's f32 op sequence and equal values merged,
    which is jnp.unique + jnp.histogram of the quantized leaf (compression.py:143-149).
    Vectorised over the K x L (client, leaf) rows; rows with the same number of
    distinct values share one array pass (numpy's row reductions are the 1-D ones)."""
    L = len(leaf_n)
    nb = num_levels + 1
    H = hist.cpu().numpy().reshape(K * L, nb).astype(np.int64)
    Q = np.frombuffer(qparams.cpu().numpy().tobytes(), dtype=QPARAMS).reshape(K * L)
    return arithmetic_bits_host(H, Q, K, leaf_n, num_levels)


def arithmetic_bits_host(H: np.ndarray, Q: np.ndarray, K: int, leaf_n: Sequence[int],
                         num_levels: int) -> List[np.float32]:
    """:func:`arithmetic_bits` on host arrays H [K*L, num_levels + 1], Q [K*L]."""
    f32 = np.float32
    L = len(leaf_n)
    R = K * L
    nb = num_levels + 1
    lm1 = f32(num_levels - 1)
    fmax = np.finfo(f32).max
    with np.errstate(all="ignore"):
        qv = (np.arange(num_levels, dtype=f32) / lm1).astype(f32)
        vals = (Q["vmin"][:, None] + (qv[None, :] * Q["range"][:, None]).astype(f32)).astype(f32)
    if not H[:, -1].any() and np.isfinite(vals).all() and (vals[:, 1:] > vals[:, :-1]).all():
        # common case: no NaN-bin counts and strictly increasing finite levels, so the
        # occupied bins ARE the distinct values in ascending (np.unique) order
        occupied = H[:, :num_levels] > 0
        u = occupied.sum(axis=1)
        merged = np.zeros((R, nb), dtype=np.int64)
        merged[np.arange(nb)[None, :] < u[:, None]] = H[:, :num_levels][occupied]
    else:
        vals = np.concatenate([vals, np.zeros((R, 1), f32)], axis=1)  # the NaN bin: nan_to_num(NaN) = 0
        vals = np.nan_to_num(vals, nan=0.0, posinf=fmax, neginf=-fmax).astype(f32)
        # distinct values of the occupied bins, ascending (np.unique order), counts merged
        big = np.where(H > 0, vals, np.inf)
        order = np.argsort(big, axis=1, kind="stable")
        sv = np.take_along_axis(big, order, axis=1)
        sc = np.take_along_axis(H, order, axis=1)
        occupied = sc > 0
        new = occupied.copy()
        new[:, 1:] &= sv[:, 1:] != sv[:, :-1]
        grp = np.cumsum(new, axis=1) - 1  # group index of each occupied sorted bin
        u = new.sum(axis=1)  # distinct values per row
        flat = (np.arange(R)[:, None] * nb + grp)[occupied]
        merged = np.bincount(flat, weights=sc[occupied], minlength=R * nb).astype(np.int64).reshape(R, nb)
    d = np.asarray(leaf_n, dtype=np.int64)[np.arange(R) % L]
    e = f32(np.exp(f32(1)))
    per_row = np.zeros(R, dtype=f32)
    # rows with 1..7 distinct values at once: numpy sums fewer than 8 terms left to right,
    # so zero terms appended to a row leave its entropy sum's bits unchanged
    small = np.nonzero((u >= 1) & (u < 8))[0]
    if small.size:
        kk = u[small]
        hist = np.ascontiguousarray(merged[small, :7])
        with np.errstate(divide="ignore", invalid="ignore"):
            p = (hist.astype(f32) / hist.sum(axis=1).astype(f32)[:, None]).astype(f32)
            term = np.where(hist > 0, (p * _log2_f32(p)).astype(f32), f32(0))
            ent = (-np.sum(term, axis=1, dtype=f32)).astype(f32)
            dk, kf = d[small], kk.astype(f32)
            hist_bits = (kf * _log2_f32(((e * (dk + kk).astype(f32)).astype(f32) / kf).astype(f32))).astype(f32)
            per_row[small] = (((hist_bits + (dk.astype(f32) * ent).astype(f32)).astype(f32) + f32(64)).astype(f32)
                              + f32(2)).astype(f32)
    for k in np.unique(u[(u < 1) | (u >= 8)]):
        sel = np.nonzero(u == k)[0]
        hist = np.ascontiguousarray(merged[sel, :k])
        with np.errstate(divide="ignore", invalid="ignore"):
            p = (hist.astype(f32) / hist.sum(axis=1).astype(f32)[:, None]).astype(f32)
            ent = (-np.sum((p * _log2_f32(p)).astype(f32), axis=1, dtype=f32)).astype(f32)
            dk = d[sel]
            hist_bits = (f32(k) * _log2_f32(((e * (dk + k).astype(f32)).astype(f32) / f32(k)).astype(f32))).astype(f32)
            per_row[sel] = (((hist_bits + (dk.astype(f32) * ent).astype(f32)).astype(f32) + f32(64)).astype(f32)
                            + f32(2)).astype(f32)
    per_row = per_row.reshape(K, L)
    bits = per_row[:, 0].copy()
    for l in range(1, L):
        bits = (bits + per_row[:, l]).astype(f32)
    return [f32(b) for b in bits]
