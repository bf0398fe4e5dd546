"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front end for ``oracle/build/librs_oracle.so`` (the C restatement of
usebeforefree/reed-solomon-cc in ``rs_oracle.c``). Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product package never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "librs_oracle.so")

CORRECTED = 0
Q_D1 = 1
Q_D2 = 2
REF_LITERAL = Q_D1 | Q_D2

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u8p, u16p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint16)
        pp = C.POINTER(C.c_void_p)
        L.rso_init.restype = None
        for name in ("rso_exp", "rso_log", "rso_skew", "rso_log_walsh"):
            getattr(L, name).restype = u16p
        L.rso_mul128.restype = u8p
        L.rso_mul16.restype = C.c_uint16
        L.rso_mul16.argtypes = [C.c_uint16, C.c_uint16]
        L.rso_mul_chunk.argtypes = [C.c_void_p, C.c_void_p, C.c_uint16, C.c_int]
        for name in ("rso_fft", "rso_ifft"):
            getattr(L, name).argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_uint64,
                                         C.c_uint64, C.c_int]
        for name in ("rso_fft_partial", "rso_ifft_partial"):
            getattr(L, name).argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint16, C.c_int]
        L.rso_mul_scalar.argtypes = [C.c_void_p, C.c_size_t, C.c_uint16, C.c_int]
        L.rso_fwht.argtypes = [C.c_void_p, C.c_uint64]
        L.rso_eval_poly.argtypes = [C.c_void_p, C.c_uint64]
        L.rso_use_high_rate.argtypes = [C.c_uint64, C.c_uint64]
        L.rso_encode.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, pp, pp, C.c_int]
        L.rso_encode_low.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, pp, pp, C.c_int]
        L.rso_decode.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, pp, pp, pp, C.c_int]
        L.rso_encode_batch.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, C.c_size_t, C.c_void_p,
                                       C.c_void_p, C.c_int, C.c_int]
        L.rso_reconstruct_batch.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, C.c_size_t, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.rso_force_scalar.argtypes = [C.c_int]
        L.rso_bench_encode.restype = C.c_double
        L.rso_bench_encode.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, C.c_uint64, C.c_int]
        L.rso_init()
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def table(name: str) -> np.ndarray:
    L = lib()
    n = {"exp": 65536, "log": 65536, "skew": 65535, "log_walsh": 65536}[name]
    p = getattr(L, "rso_" + name)()
    return np.ctypeslib.as_array(p, shape=(n,)).copy()


def mul128() -> np.ndarray:
    p = lib().rso_mul128()
    return np.ctypeslib.as_array(p, shape=(65536, 2, 4, 16)).copy()


def mul16(x: int, log_m: int) -> int:
    return int(lib().rso_mul16(x, log_m))


def mul_chunk(chunk: np.ndarray, log_m: int, quirks: int = CORRECTED) -> np.ndarray:
    src = np.ascontiguousarray(chunk, dtype=np.uint8).reshape(64)
    out = np.zeros(64, np.uint8)
    lib().rso_mul_chunk(_ptr(src), _ptr(out), log_m, quirks)
    return out


def fft(work: np.ndarray, pos, size, trunc, skew_delta, quirks=CORRECTED):
    """In-place engine FFT on a [shard_count, shard_bytes] uint8 buffer."""
    L = work.shape[1] // 64
    lib().rso_fft(_ptr(work), L, pos, size, trunc, skew_delta, quirks)


def ifft(work: np.ndarray, pos, size, trunc, skew_delta, quirks=CORRECTED):
    L = work.shape[1] // 64
    lib().rso_ifft(_ptr(work), L, pos, size, trunc, skew_delta, quirks)


def ifft_partial(x: np.ndarray, y: np.ndarray, log_m: int, quirks=CORRECTED):
    lib().rso_ifft_partial(_ptr(x), _ptr(y), x.size // 64, log_m, quirks)


def fft_partial(x: np.ndarray, y: np.ndarray, log_m: int, quirks=CORRECTED):
    lib().rso_fft_partial(_ptr(x), _ptr(y), x.size // 64, log_m, quirks)


def mul_scalar(x: np.ndarray, log_m: int, quirks=CORRECTED):
    lib().rso_mul_scalar(_ptr(x), x.size // 64, log_m, quirks)


def fwht(data: np.ndarray, m: int):
    assert data.dtype == np.uint16 and data.size == 65536
    lib().rso_fwht(_ptr(data), m)


def eval_poly(erasures: np.ndarray, trunc: int):
    assert erasures.dtype == np.uint16 and erasures.size == 65536
    lib().rso_eval_poly(_ptr(erasures), trunc)


def use_high_rate(k: int, m: int) -> int:
    return int(lib().rso_use_high_rate(k, m))


def _ptr_array(arrs):
    arr = (C.c_void_p * len(arrs))()
    for i, a in enumerate(arrs):
        arr[i] = None if a is None else a.ctypes.data
    return arr


def encode(k: int, m: int, original: np.ndarray, quirks: int = CORRECTED):
    """original: [k, shard_bytes] uint8 -> (status, recovery [m, shard_bytes])."""
    original = np.ascontiguousarray(original, dtype=np.uint8)
    sb = original.shape[1]
    rec = np.zeros((m, sb), np.uint8)
    ins = _ptr_array([original[i] for i in range(k)])
    outs = _ptr_array([rec[i] for i in range(m)])
    st = lib().rso_encode(k, m, sb, ins, outs, quirks)
    return st, rec


def encode_low(k: int, m: int, original: np.ndarray, quirks: int = CORRECTED):
    """Low-rate encode (absent from the reference: PARITY UNPINNED, restated from
    reed-solomon-simd's low-rate encoder). original [k, sb] -> (status, recovery [m, sb])."""
    original = np.ascontiguousarray(original, dtype=np.uint8)
    sb = original.shape[1]
    rec = np.zeros((m, sb), np.uint8)
    ins = _ptr_array([original[i] for i in range(k)])
    outs = _ptr_array([rec[i] for i in range(m)])
    st = lib().rso_encode_low(k, m, sb, ins, outs, quirks)
    return st, rec


def decode(k: int, m: int, original, recovery, shard_bytes: int, quirks: int = CORRECTED):
    """original / recovery: lists with None for missing shards -> (status, restored [k, sb])."""
    orig = [None if o is None else np.ascontiguousarray(o, dtype=np.uint8) for o in original]
    rec = [None if r is None else np.ascontiguousarray(r, dtype=np.uint8) for r in recovery]
    out = np.zeros((k, shard_bytes), np.uint8)
    st = lib().rso_decode(k, m, shard_bytes, _ptr_array(orig), _ptr_array(rec),
                          _ptr_array([out[i] for i in range(k)]), quirks)
    return st, out


def encode_batch(k, m, data: np.ndarray, quirks=CORRECTED, threads=1):
    """data: [n, k, sb] -> parity [n, m, sb]."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n, kk, sb = data.shape
    assert kk == k
    par = np.zeros((n, m, sb), np.uint8)
    st = lib().rso_encode_batch(k, m, sb, n, _ptr(data), _ptr(par), quirks, threads)
    if st:
        raise RuntimeError(f"rso_encode_batch status {st}")
    return par


def reconstruct_batch(k, m, present: np.ndarray, shards: np.ndarray, quirks=CORRECTED, threads=1):
    """shards: [n, k+m, sb]; present: k+m bools -> restored [n, e, sb]."""
    shards = np.ascontiguousarray(shards, dtype=np.uint8)
    present = np.ascontiguousarray(present, dtype=np.uint8)
    n, km, sb = shards.shape
    e = int(k - present[:k].sum())
    out = np.zeros((n, e, sb), np.uint8)
    st = lib().rso_reconstruct_batch(k, m, sb, n, _ptr(present), _ptr(shards), _ptr(out), quirks, threads)
    if st:
        raise RuntimeError(f"rso_reconstruct_batch status {st}")
    return out


def force_scalar(on: bool):
    lib().rso_force_scalar(1 if on else 0)


def bench_encode_ns(k, m, shard_bytes, iters, quirks=CORRECTED) -> float:
    """benchmarks.zig:14-61 protocol timed natively: mean ns per insert + encode."""
    return lib().rso_bench_encode(k, m, shard_bytes, iters, quirks)
