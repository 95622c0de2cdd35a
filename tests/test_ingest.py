"""Wire format of fedjax/core/serialization.py (CPU) and pipelined ingestion (GPU)."""
import msgpack
import numpy as np
import numpy.testing as npt
import pytest
import torch

from fedjax_amd import ingest


def _ref_ndarray_to_bytes(arr):
    # restatement of fedjax/core/serialization.py:79-87 (the encoder under test must match it)
    return msgpack.packb((arr.shape, arr.dtype.name, arr.tobytes("C")), use_bin_type=True)


def _ref_serialize(tree):
    def ext(x):
        if isinstance(x, np.ndarray) and x.dtype.hasobject:
            return msgpack.ExtType(4, msgpack.packb((x.shape, list(x.flatten())), use_bin_type=True))
        if isinstance(x, np.ndarray):
            return msgpack.ExtType(1, _ref_ndarray_to_bytes(x))
        if isinstance(x, np.generic):
            return msgpack.ExtType(3, _ref_ndarray_to_bytes(np.asarray(x)))
        return x
    return msgpack.packb(tree, default=ext, strict_types=True)


def test_reference_dict_case():
    # fedjax/core/serialization_test.py:23-41
    original = {"int32": np.arange(4, dtype=np.int32).reshape([2, 2]),
                "float64": -np.arange(4, dtype=np.float64).reshape([1, 4]),
                "bytes": np.array([b"a", b"bc", b"def"], dtype=object).reshape([3, 1])}
    enc = ingest.msgpack_serialize(original)
    assert enc == _ref_serialize(original)
    out = ingest.msgpack_deserialize(enc)
    assert out["int32"].dtype == np.int32 and out["float64"].dtype == np.float64
    npt.assert_array_equal(out["int32"], original["int32"])
    npt.assert_array_equal(out["float64"], original["float64"])
    assert out["bytes"].dtype == object
    npt.assert_array_equal(out["bytes"], original["bytes"])


def test_reference_nested_list_case():
    # fedjax/core/serialization_test.py:43-63
    original = [np.arange(4, dtype=np.int32).reshape([2, 2]),
                [-np.arange(4, dtype=np.float64).reshape([1, 4]),
                 [np.array([b"a", b"bc", b"def"], dtype=object).reshape([3, 1]), []]]]
    out = ingest.msgpack_deserialize(ingest.msgpack_serialize(original))
    int32_array, rest = out
    npt.assert_array_equal(int32_array, original[0])
    float64_array, rest = rest
    npt.assert_array_equal(float64_array, original[1][0])
    bytes_array, rest = rest
    npt.assert_array_equal(bytes_array, original[1][1][0])
    assert rest == []


def test_scalars_bf16_and_float32_deltas():
    d = {"w": np.linspace(-1, 1, 12, dtype=np.float32).reshape(3, 4), "s": np.float32(2.5)}
    out = ingest.msgpack_deserialize(ingest.msgpack_serialize(d))
    npt.assert_array_equal(out["w"], d["w"])
    assert out["s"] == np.float32(2.5) and isinstance(out["s"], np.float32)
    bits = np.array([0x3F80, 0xC000, 0x7FC0], np.uint16)
    enc = ingest.msgpack_serialize({"b": ingest.BF16Array(bits)})
    shape, name, buf = msgpack.unpackb(msgpack.unpackb(enc, raw=True)[b"b"].data, raw=True)
    assert name == b"bfloat16" and list(shape) == [3]
    back = ingest.msgpack_deserialize(enc)["b"]
    assert isinstance(back, ingest.BF16Array) and np.array_equal(np.asarray(back, np.uint16), bits)


def test_zero_copy_decoder_matches_msgpack():
    d = {"w": np.arange(12, dtype=np.float32).reshape(3, 4), "n": [np.int32(7), 1.5, -3, "x", None, True],
         "big": np.arange(70000, dtype=np.float32), "bf": ingest.BF16Array(np.array([1, 2, 3], np.uint16)),
         "i64": np.int64(-(2 ** 40)), "u": 2 ** 40, "neg": -200, "s16": "y" * 300}
    enc = ingest.msgpack_serialize(d)
    a = ingest.msgpack_deserialize(enc)
    b = ingest.msgpack_deserialize_view(enc)
    assert set(a) == set(b)
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k
    assert not b["big"].flags.writeable  # a view into the payload, not a copy
    assert np.shares_memory(b["big"], np.frombuffer(enc, np.uint8))


def test_f32_to_bf16_rounding():
    x = np.array([1.0, 1.00390625, 1.01171875, -2.0, np.inf, np.nan, 3.0e38], np.float32)
    b = ingest._f32_to_bf16_bits(x)
    back = (b.astype(np.uint32) << 16).view(np.float32)
    assert back[0] == 1.0 and back[1] == 1.0 and back[2] == 1.015625  # ties to even
    assert back[3] == -2.0 and np.isinf(back[4]) and np.isnan(back[5])


@pytest.mark.gpu
def test_ingest_msgpack_into_slab_then_mean(cuda, coracle):
    import fedjax_amd
    from oracle import tree_util_ref as ref
    K, P = 24, 3000
    xh = coracle.synth_f32(K, P, seed=41)
    template = {"a": np.zeros(1000, np.float32), "b": (np.zeros((10, 100), np.float32), np.zeros(1000, np.float32))}
    slab = fedjax_amd.ClientDeltaSlab(template, K, device=cuda)
    ing = ingest.DeltaIngestor(slab, depth=3)
    for k in range(K):
        d = {"a": xh[k, :1000], "b": [xh[k, 1000:2000].reshape(10, 100), xh[k, 2000:]]}
        # the wire format has no tuples (serialization.py:17-19): lists become the slab's tuple
        ing.put(k, ingest.msgpack_serialize(d) if k % 2 else d)
    ing.ready()
    wi = [int(v) for v in ref.fedavg_weights(K, seed=42)]
    m = slab.mean(wi)
    got = np.concatenate([m["a"].cpu().numpy(), m["b"][0].cpu().numpy().ravel(), m["b"][1].cpu().numpy()])
    want = coracle.wsum_f32(xh, np.float32(wi), scale=ref.mean_scale(wi))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
