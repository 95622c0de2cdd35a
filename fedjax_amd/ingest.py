"""Host-resident client deltas: FedJAX's msgpack wire format and pipelined ingestion.

In deployment the client deltas start in host memory (simulated clients feed the
server from host RAM, or deltas arrive serialized). This module covers that edge
of the path:

* :func:`msgpack_serialize` / :func:`msgpack_deserialize` — byte-compatible with
  fedjax/core/serialization.py:79-192 for numeric arrays (ext type 1 = ndarray
  ``(shape, dtype name, C-order bytes)``, 2 = complex, 3 = numpy scalar,
  4 = bytes ndarray). ``bfloat16`` arrays (dtype name ``b'bfloat16'``,
  serialization.py:91-96) decode to :class:`BF16Array`, a uint16 view, since
  numpy has no bfloat16.
* :class:`DeltaIngestor` — copies host deltas (pytrees or msgpack payloads) into
  the rows of a :class:`~fedjax_amd.slab.ClientDeltaSlab` through a ring of pinned
  staging buffers on a dedicated copy stream. Host decode of client k+1 overlaps
  the DMA of client k, and :meth:`DeltaIngestor.ready` makes the compute stream
  wait for the copies, so ``slab.mean`` can be enqueued right away.

The host path is PCIe-bound (≈57 GB/s measured on MI355X, profiles/r01_bench_e2e.json).
The device-resident fold is ~120× faster, so the ingestion rate is the E2E rate.
"""

from __future__ import annotations

import enum
import warnings
from typing import Any, List, Optional, Union

import msgpack
import numpy as np
import torch

from fedjax_amd import pytree
from fedjax_amd.slab import ClientDeltaSlab


class _Ext(enum.IntEnum):  # serialization.py:136-141
    ndarray = 1
    native_complex = 2
    npscalar = 3
    bytes_ndarray = 4


class BF16Array(np.ndarray):
    """uint16 storage of a bfloat16 array decoded from the wire (numpy lacks bf16)."""

    def __new__(cls, u16: np.ndarray):
        return np.asarray(u16, dtype=np.uint16).view(cls)

    @property
    def wire_dtype(self) -> str:
        return "bfloat16"


def _ndarray_to_bytes(arr) -> bytes:  # serialization.py:79-87
    if isinstance(arr, torch.Tensor):
        t = arr.detach().cpu().contiguous()
        if t.dtype == torch.bfloat16:
            arr = BF16Array(t.view(torch.int16).numpy().view(np.uint16))
        else:
            arr = t.numpy()
    if isinstance(arr, BF16Array):
        return msgpack.packb((arr.shape, "bfloat16", np.asarray(arr, np.uint16).tobytes("C")),
                             use_bin_type=True)
    if arr.dtype.hasobject or arr.dtype.isalignedstruct:
        raise ValueError("Object and structured dtypes not supported for serialization of ndarrays.")
    return msgpack.packb((arr.shape, arr.dtype.name, arr.tobytes("C")), use_bin_type=True)


def _ndarray_from_bytes(data: bytes):  # serialization.py:99-103
    shape, dtype_name, buffer = msgpack.unpackb(data, raw=True)
    if dtype_name == b"bfloat16":
        return BF16Array(np.frombuffer(buffer, dtype=np.uint16).reshape(shape, order="C"))
    return np.frombuffer(buffer, dtype=np.dtype(dtype_name.decode()), count=-1, offset=0).reshape(
        shape, order="C")


def _bytes_ndarray_to_bytes(x) -> bytes:  # serialization.py:106-112
    flat = list(x.flatten())
    if flat and not isinstance(flat[0], bytes):
        raise ValueError("Only ndarrays holding bytes objects can be serialized.")
    return msgpack.packb((x.shape, flat), use_bin_type=True)


def _ext_pack(x):  # serialization.py:144-161
    if isinstance(x, np.ndarray) and x.dtype.hasobject:
        return msgpack.ExtType(_Ext.bytes_ndarray, _bytes_ndarray_to_bytes(x))
    if isinstance(x, (np.ndarray, torch.Tensor)):
        return msgpack.ExtType(_Ext.ndarray, _ndarray_to_bytes(x))
    if isinstance(x, np.generic):
        return msgpack.ExtType(_Ext.npscalar, _ndarray_to_bytes(np.asarray(x)))
    if isinstance(x, complex):
        return msgpack.ExtType(_Ext.native_complex, msgpack.packb((x.real, x.imag)))
    return x


def _ext_unpack(code, data):  # serialization.py:164-176
    if code == _Ext.ndarray:
        return _ndarray_from_bytes(data)
    if code == _Ext.native_complex:
        c = msgpack.unpackb(data)
        return complex(c[0], c[1])
    if code == _Ext.npscalar:
        return _ndarray_from_bytes(data)[()]
    if code == _Ext.bytes_ndarray:
        shape, flat = msgpack.unpackb(data, raw=True)
        return np.array(flat, dtype=object).reshape(shape)
    return msgpack.ExtType(code, data)


def msgpack_serialize(tree) -> bytes:
    """serialization.py:179-192 (dicts and lists of arrays; tuples become lists)."""
    return msgpack.packb(tree, default=_ext_pack, strict_types=True)


def msgpack_deserialize(encoded: bytes):
    """serialization.py:195-208; arrays are zero-copy views of ``encoded``."""
    return msgpack.unpackb(encoded, ext_hook=_ext_unpack, raw=False)


# ------------------------------------------------------------- zero-copy decoding
import struct as _struct

_U8, _U16, _U32, _U64 = (_struct.Struct(f) for f in (">B", ">H", ">I", ">Q"))
_I8, _I16, _I32, _I64 = (_struct.Struct(f) for f in (">b", ">h", ">i", ">q"))
_F32, _F64 = _struct.Struct(">f"), _struct.Struct(">d")


def _read(buf: memoryview, i: int):
    """One msgpack object at buf[i:] -> (value, next index). bin / ext payloads stay
    memoryviews into ``buf``; ndarray ext payloads decode to numpy views (no copy)."""
    b = buf[i]
    i += 1
    if b <= 0x7F:
        return b, i
    if b >= 0xE0:
        return b - 0x100, i
    if 0x80 <= b <= 0x8F:
        return _read_map(buf, i, b & 0x0F)
    if 0x90 <= b <= 0x9F:
        return _read_array(buf, i, b & 0x0F)
    if 0xA0 <= b <= 0xBF:
        n = b & 0x1F
        return bytes(buf[i:i + n]).decode(), i + n
    if b == 0xC0:
        return None, i
    if b in (0xC2, 0xC3):
        return b == 0xC3, i
    if b in (0xC4, 0xC5, 0xC6):  # bin 8/16/32
        st = (_U8, _U16, _U32)[b - 0xC4]
        n = st.unpack_from(buf, i)[0]
        i += st.size
        return buf[i:i + n], i + n
    if b in (0xC7, 0xC8, 0xC9):  # ext 8/16/32
        st = (_U8, _U16, _U32)[b - 0xC7]
        n = st.unpack_from(buf, i)[0]
        i += st.size
        code = _I8.unpack_from(buf, i)[0]
        i += 1
        return _ext(code, buf[i:i + n]), i + n
    if b in (0xD4, 0xD5, 0xD6, 0xD7, 0xD8):  # fixext 1..16
        n = 1 << (b - 0xD4)
        code = _I8.unpack_from(buf, i)[0]
        i += 1
        return _ext(code, buf[i:i + n]), i + n
    if b == 0xCA:
        return _F32.unpack_from(buf, i)[0], i + 4
    if b == 0xCB:
        return _F64.unpack_from(buf, i)[0], i + 8
    if 0xCC <= b <= 0xD3:
        st = (_U8, _U16, _U32, _U64, _I8, _I16, _I32, _I64)[b - 0xCC]
        return st.unpack_from(buf, i)[0], i + st.size
    if b in (0xD9, 0xDA, 0xDB):  # str 8/16/32
        st = (_U8, _U16, _U32)[b - 0xD9]
        n = st.unpack_from(buf, i)[0]
        i += st.size
        return bytes(buf[i:i + n]).decode(), i + n
    if b in (0xDC, 0xDD):
        st = _U16 if b == 0xDC else _U32
        return _read_array(buf, i + st.size, st.unpack_from(buf, i)[0])
    if b in (0xDE, 0xDF):
        st = _U16 if b == 0xDE else _U32
        return _read_map(buf, i + st.size, st.unpack_from(buf, i)[0])
    raise ValueError(f"unsupported msgpack byte 0x{b:02x}")


def _read_array(buf, i, n):
    out = []
    for _ in range(n):
        v, i = _read(buf, i)
        out.append(v)
    return out, i


def _read_map(buf, i, n):
    out = {}
    for _ in range(n):
        k, i = _read(buf, i)
        v, i = _read(buf, i)
        out[bytes(k).decode() if isinstance(k, memoryview) else k] = v
    return out, i


def _ext(code: int, payload: memoryview):
    if code in (_Ext.ndarray, _Ext.npscalar):
        (shape, name, data), _ = _read(payload, 0)
        name = bytes(name).decode() if isinstance(name, memoryview) else name
        if name == "bfloat16":
            a = BF16Array(np.frombuffer(data, dtype=np.uint16).reshape(shape))
        else:
            a = np.frombuffer(data, dtype=np.dtype(name)).reshape(shape)
        return a[()] if code == _Ext.npscalar else a
    return _ext_unpack(code, bytes(payload))


def msgpack_deserialize_view(encoded) -> Any:
    """msgpack_deserialize without copying array payloads: ndarray leaves are
    read-only numpy views into ``encoded`` (keep it alive while they are used)."""
    buf = memoryview(encoded).cast("B")
    v, i = _read(buf, 0)
    if i != len(buf):
        raise ValueError("trailing bytes after the msgpack object")
    return v


# ------------------------------------------------------------------------ ingestion
def _f32_to_bf16_bits(a: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even float32 -> bfloat16 bits (NaN stays NaN)."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    nan = (u & np.uint32(0x7FFFFFFF)) > np.uint32(0x7F800000)
    r = ((u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)).astype(np.uint16)
    return np.where(nan, ((u >> np.uint32(16)) | np.uint32(0x40)).astype(np.uint16), r)


def _host_view(x, slab_dtype: torch.dtype) -> np.ndarray:
    """Flat uint8 view of a host leaf in the slab's dtype (f32 or bf16 bits)."""
    if isinstance(x, torch.Tensor):
        if x.is_cuda:
            raise ValueError("DeltaIngestor takes host deltas; device deltas go to slab.set_client")
        t = x.detach().contiguous()
        if t.dtype != slab_dtype:
            t = t.to(slab_dtype)
        return t.view(torch.uint8).numpy().reshape(-1) if t.numel() else np.empty(0, np.uint8)
    if slab_dtype == torch.bfloat16:
        a = np.asarray(x, np.uint16) if isinstance(x, BF16Array) else _f32_to_bf16_bits(np.asarray(x))
    else:
        a = np.asarray(x)
        if isinstance(x, BF16Array):
            a = (np.asarray(x, np.uint32) << np.uint32(16)).view(np.float32)
        elif a.dtype != np.float32:
            a = a.astype(np.float32)  # jnp canonicalisation (float64 -> float32)
    return np.ascontiguousarray(a).view(np.uint8).reshape(-1)


class DeltaIngestor:
    """Pipelined host -> slab copies through ``depth`` pinned staging rows.

    ``put(k, delta)`` takes a host pytree (numpy / host tensors / BF16Array
    leaves, in the slab's dtype) or msgpack bytes; it packs the leaves into a
    pinned row (one host memcpy per leaf) and enqueues the H2D copy into slab row
    k on the copy stream. ``ready()`` makes the current stream wait for every copy
    enqueued so far.
    """

    def __init__(self, slab: ClientDeltaSlab, depth: Optional[int] = None, copy_threads: int = 4):
        self.slab = slab
        # host threads of the staging copy: the DMA engine reads host memory at the same
        # time, and a copy on every OpenMP thread slows it (128 x 16 MiB rows on MI355X:
        # 46 GB/s end to end with 16 threads, 53 GB/s with 4 = 98 % of the 54 GB/s of
        # back-to-back pinned row copies; profiles/r01zi_ingest_stages.jsonl)
        self.copy_threads = max(1, int(copy_threads))
        self.device = slab.device
        self.stream = torch.cuda.Stream(self.device)
        self.row_bytes = slab.num_params * slab.storage.element_size()
        if depth is None:  # 8 rows in flight (51-52 GB/s vs 46-47 with 4), at most ~1 GiB pinned
            depth = max(2, min(8, (1 << 30) // max(1, self.row_bytes)))
        self.staging = [torch.empty(max(1, self.row_bytes), dtype=torch.uint8).pin_memory()
                        for _ in range(max(1, depth))]
        self.events: List[Optional[torch.cuda.Event]] = [None] * len(self.staging)
        self.n = 0
        self._after_compute = False  # copy stream ordered after prior slab readers?

    def put(self, k: int, delta: Union[bytes, bytearray, memoryview, Any]) -> None:
        if isinstance(delta, (bytes, bytearray, memoryview)):
            delta = msgpack_deserialize_view(delta)
        leaves = pytree.flatten_as(self.slab.treedef, _tuples_as_lists(delta, self.slab.treedef))
        i = self.n % len(self.staging)
        if self.events[i] is not None:
            self.events[i].synchronize()  # the DMA that last used this row has finished
        prev_threads = torch.get_num_threads()
        if prev_threads != self.copy_threads:
            torch.set_num_threads(self.copy_threads)
        try:
            self._stage(k, leaves, self.staging[i])
        finally:
            if prev_threads != self.copy_threads:
                torch.set_num_threads(prev_threads)
        dst = self.slab.storage[k].view(torch.uint8)[: self.row_bytes]
        if not self._after_compute:  # earlier kernels may still read the slab rows
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            self._after_compute = True
        with torch.cuda.stream(self.stream):
            dst.copy_(self.staging[i][: self.row_bytes], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.events[i] = ev
        self.n += 1

    def _stage(self, k: int, leaves, row: torch.Tensor) -> None:
        """Pack client k's leaves back to back into the pinned staging row."""
        off = 0
        for x, size in zip(leaves, self.slab.sizes):
            a = _host_view(x, self.slab.dtype)
            if a.size != size * self.slab.storage.element_size():
                raise ValueError(f"client {k}: leaf of {a.size} bytes, slab expects "
                                 f"{size * self.slab.storage.element_size()}")
            if a.size:  # torch's host copy runs on copy_threads threads for large buffers
                if a.flags.writeable:
                    src = torch.from_numpy(a)
                else:  # a read-only view into the payload: only ever read here
                    with warnings.catch_warnings():
                        warnings.simplefilter("ignore", UserWarning)
                        src = torch.frombuffer(a, dtype=torch.uint8)
                row[off:off + a.size].copy_(src)
            off += a.size

    def ready(self) -> None:
        """Order the current stream after every enqueued copy (call before the fold)."""
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        self._after_compute = False


def _tuples_as_lists(tree, treedef: pytree.TreeDef):
    """msgpack turns tuples into lists (serialization.py:17-19): restore the slab's
    container types where the structure says tuple."""
    k = treedef.kind
    if k == "tuple" and isinstance(tree, list):
        return tuple(_tuples_as_lists(t, c) for t, c in zip(tree, treedef.children))
    if k == "list" and isinstance(tree, list):
        return [_tuples_as_lists(t, c) for t, c in zip(tree, treedef.children)]
    if k == "dict" and isinstance(tree, dict):
        child = dict(zip(treedef.aux, treedef.children))
        return {key: (_tuples_as_lists(v, child[key]) if key in child else v) for key, v in tree.items()}
    return tree


__all__ = ["BF16Array", "DeltaIngestor", "msgpack_deserialize", "msgpack_deserialize_view",
           "msgpack_serialize"]
