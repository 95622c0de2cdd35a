"""ctypes view of oracle/fold_ref.c (test infrastructure)."""
import ctypes

import numpy as np

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i64, _u64, _f32, _f64, _int = ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_double, ctypes.c_int


class COracle:
    def __init__(self, path):
        lib = ctypes.CDLL(path)
        lib.oracle_fill_synth_f32.argtypes = [_f32p, _i64, _i64, _i64, _i64, _u64, _f32]
        lib.oracle_fill_synth_bf16.argtypes = [_u16p, _i64, _i64, _i64, _i64, _u64, _f32]
        lib.oracle_wsum_f32.argtypes = [_f32p, _i64, _i64, _i64, _f32p, _f32, _int, _int, _f32p]
        lib.oracle_wsum_bf16_f64.argtypes = [_u16p, _i64, _i64, _i64, _f64p, _f64, _f64p]
        lib.oracle_wsum_bf16_refsem.argtypes = [_u16p, _i64, _i64, _i64, _f32p, _f32, _u16p]
        lib.oracle_wsum_bound_f32.argtypes = [_f32p, _i64, _i64, _i64, _f32p, _f32, _f32p, _f64p]
        lib.oracle_tree_mean_refseq_f32.argtypes = [_f32p, _i64, _i64, _i64, _f32p, _f32, _f32p, _int]
        lib.oracle_tree_mean_refseq_f32.restype = _int
        lib.oracle_synth_cols_f32.argtypes = [_f32p, _i64, _i64, np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS"),
                                              _i64, _u64, _f32, _int]
        self.lib = lib

    def synth_cols_f32(self, K, cols, seed=0, amp=0.01, k0=0, bf16=False):
        """Clients k0..k0+K-1 of the synthetic slab at columns ``cols`` only: [K, len(cols)]
        float32 (bf16: the bf16-rounded values, widened)."""
        cols = np.ascontiguousarray(cols, dtype=np.int64)
        x = np.empty((K, cols.size), np.float32)
        self.lib.oracle_synth_cols_f32(x, K, k0, cols, cols.size, seed, amp, int(bool(bf16)))
        return x

    def synth_f32(self, K, P, seed=0, amp=0.01, k0=0):
        x = np.empty((K, P), np.float32)
        self.lib.oracle_fill_synth_f32(x, P, K, P, k0, seed, amp)
        return x

    def synth_bf16(self, K, P, seed=0, amp=0.01, k0=0):
        x = np.empty((K, P), np.uint16)
        self.lib.oracle_fill_synth_bf16(x, P, K, P, k0, seed, amp)
        return x

    def wsum_f32(self, x, w, scale=None, init=None):
        K, P = x.shape
        y = np.zeros(P, np.float32) if init is None else np.array(init, np.float32)
        self.lib.oracle_wsum_f32(np.ascontiguousarray(x), P, K, P, np.asarray(w, np.float32),
                                 np.float32(1 if scale is None else scale), scale is not None,
                                 init is not None, y)
        return y

    def refseq_f32(self, x, w, scale, nthreads=1):
        K, P = x.shape
        y = np.empty(P, np.float32)
        rc = self.lib.oracle_tree_mean_refseq_f32(np.ascontiguousarray(x), P, K, P,
                                                  np.asarray(w, np.float32), np.float32(scale), y, nthreads)
        assert rc == 0
        return y

    def wsum_bf16_f64(self, x_u16, w, scale):
        K, P = x_u16.shape
        y = np.empty(P, np.float64)
        self.lib.oracle_wsum_bf16_f64(np.ascontiguousarray(x_u16), P, K, P, np.asarray(w, np.float64), scale, y)
        return y

    def wsum_bf16_refsem(self, x_u16, w, scale):
        K, P = x_u16.shape
        y = np.empty(P, np.uint16)
        self.lib.oracle_wsum_bf16_refsem(np.ascontiguousarray(x_u16), P, K, P, np.asarray(w, np.float32),
                                         np.float32(scale), y)
        return y

    def bound_f32(self, x, w, scale, y_ref):
        K, P = x.shape
        b = np.empty(P, np.float64)
        self.lib.oracle_wsum_bound_f32(np.ascontiguousarray(x), P, K, P, np.asarray(w, np.float32),
                                       np.float32(scale), np.asarray(y_ref, np.float32), b)
        return b


def load(path):
    return COracle(path)


def bf16_to_f32(u16):
    return (np.asarray(u16, np.uint32) << 16).view(np.float32)
