"""TEST INFRASTRUCTURE ONLY -- ctypes binding to the C restatement (oracle/kmer_oracle.c).

Built by ``make -C oracle`` (called from __graft_entry__.build()) into
oracle/build/liboracle.so.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline may import this.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run make -C oracle)")
        L = ctypes.CDLL(LIB_PATH)
        L.orc_count_dense.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.orc_count_dense.restype = ctypes.c_int64
        L.orc_count_sparse.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p]
        L.orc_count_sparse.restype = ctypes.c_int64
        L.orc_synth.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_uint64]
        L.orc_synth.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def _as_u8(seq):
    if isinstance(seq, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(seq), np.uint8)
    return np.ascontiguousarray(seq, dtype=np.uint8)


def count_dense(seq, k, with_first=False):
    """seq: uint8 numpy array / bytes.  Returns counts (u32[4^k]) [, first (u32[4^k])]."""
    seq = _as_u8(seq)
    counts = np.zeros(1 << (2 * k), dtype=np.uint32)
    first = np.zeros(1 << (2 * k), dtype=np.uint32) if with_first else None
    r = lib().orc_count_dense(_ptr(seq), seq.size, k, _ptr(counts),
                              _ptr(first) if with_first else None)
    if r < 0:
        raise ValueError("orc_count_dense failed")
    return (counts, first) if with_first else counts


def count_sparse(seq, k, canonical=False):
    """Returns (codes u64, counts u32, first u64) in ascending code order."""
    seq = _as_u8(seq)
    nwin = max(seq.size - k + 1, 1)
    codes = np.zeros(nwin, np.uint64)
    counts = np.zeros(nwin, np.uint32)
    first = np.zeros(nwin, np.uint64)
    d = lib().orc_count_sparse(_ptr(seq), seq.size, k, int(bool(canonical)), _ptr(codes),
                               _ptr(counts), _ptr(first))
    if d < 0:
        raise ValueError("orc_count_sparse failed")
    return codes[:d].copy(), counts[:d].copy(), first[:d].copy()


def synth(length, seed, start=0):
    out = np.empty(length, np.uint8)
    lib().orc_synth(_ptr(out), start, length, seed)
    return out
