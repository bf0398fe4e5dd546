"""reedsol_amd — Python mirror of the usebeforefree/reed-solomon-cc codec API.

Same names, argument meaning and error behaviour as the reference's module
``reedsol`` (src/root.zig): ``encode``, ``decode``, ``Encoder``, ``Decoder``,
``use_high_rate``; errors are raised as ``ReedSolomonError`` subclasses named
after the Zig error set. Everything is computed by the gfx950 HIP kernels of
``librs_amd.so`` through its C ABI (include/reedsol.h); there is no CPU
fallback — without the library or a gfx950 device every call raises.

Device batch API (``encode_batch_dev`` / ``reconstruct_batch_dev``) takes
torch tensors that already live in HBM (PyTorch is only the allocator and
stream provider here).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RS_AMD_LIB", os.path.join(PKG_DIR, "build", "librs_amd.so"))

FLAG_CORRECTED = 0
FLAG_QUIRK_D1 = 1
FLAG_QUIRK_D2 = 2
FLAG_REF_LITERAL = 3

_STATUS_NAMES = [
    "Ok", "TooFewOriginalShards", "NotEnoughShards", "InvalidShardSize", "UnsupportedShardCount",
    "TooManyOriginalShards", "DifferentShardSize", "InvalidShardIndex", "DuplicateShardIndex",
    "TooManyShards", "OutOfMemory", "Overflow", "LowRateUnsupported", "ShardTailUnsupported",
    "InvalidArgument", "DeviceError", "NoDevice",
]


class ReedSolomonError(Exception):
    status = -1


_ERRORS = {}
for _i, _n in enumerate(_STATUS_NAMES[1:], start=1):
    _cls = type(_n, (ReedSolomonError,), {"status": _i})
    globals()[_n] = _cls
    _ERRORS[_i] = _cls

_lib = None


def lib():
    """Load librs_amd.so (import torch first when mixing with torch tensors so
    both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"librs_amd.so not built: {LIB_PATH} (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, u8p, u16p, sz, u64, u32 = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint16), C.c_size_t, \
        C.c_uint64, C.c_uint32
    pp = C.POINTER(C.c_void_p)
    sig = {
        "rs_version": (C.c_char_p, []),
        "rs_status_name": (C.c_char_p, [C.c_int]),
        "rs_last_error": (C.c_char_p, []),
        "rs_use_high_rate": (C.c_int, [u64, u64]),
        "rs_encode": (C.c_int, [u64, u64, sz, pp, pp]),
        "rs_decode": (C.c_int, [u64, u64, sz, pp, pp, pp]),
        "rs_encoder_new": (C.c_int, [u64, u64, sz, C.POINTER(vp)]),
        "rs_encoder_add_original_shard": (C.c_int, [vp, vp, sz]),
        "rs_encoder_encode": (C.c_int, [vp, pp]),
        "rs_encoder_reset": (C.c_int, [vp]),
        "rs_encoder_free": (None, [vp]),
        "rs_decoder_new": (C.c_int, [u64, u64, sz, C.POINTER(vp)]),
        "rs_decoder_add_original_shard": (C.c_int, [vp, u64, vp, sz]),
        "rs_decoder_add_recovery_shard": (C.c_int, [vp, u64, vp, sz]),
        "rs_decoder_decode": (C.c_int, [vp, pp]),
        "rs_decoder_free": (None, [vp]),
        "rs_encode_batch_dev": (C.c_int, [u64, u64, sz, u64, vp, u64, vp, u64, u32, vp]),
        "rs_reconstruct_batch_dev": (C.c_int, [u64, u64, sz, u64, vp, vp, u64, vp, u64, vp, u64, u32, vp]),
        "rs_reconstruct_batch_dev_patterns": (C.c_int, [u64, u64, sz, u64, vp, u64, u32, vp, u64, vp, u64, vp, u64,
                                                        vp, u32, vp]),
        "rs_encode_batch_host": (C.c_int, [u64, u64, sz, u64, vp, u64, vp, u64, u32]),
        "rs_reconstruct_batch_host": (C.c_int, [u64, u64, sz, u64, vp, vp, u64, vp, u64, vp, u64, u32]),
        "rs_encode_batch_host_multi": (C.c_int, [u64, u64, sz, u64, vp, u64, vp, u64, u32, vp, C.c_int]),
        "rs_reconstruct_batch_host_multi": (C.c_int, [u64, u64, sz, u64, vp, vp, u64, vp, u64, vp, u64, u32, vp,
                                                      C.c_int]),
        "rs_encode_kernel_name": (C.c_char_p, [u64, u64, sz]),
        "rs_reconstruct_kernel_name": (C.c_char_p, [u64, u64, sz, vp]),
        "rs_net_compile_check": (C.c_int, [u64, u64, vp, u32, vp]),
        "rs_net_wait": (C.c_int, []),
        "rs_reconstruct_warm": (C.c_int, [u64, u64, sz, vp, u32]),
        "rs_last_kernels": (C.c_char_p, []),
        "rs_debug_fail_alloc": (C.c_int64, [C.c_int64]),
        "rs_debug_release_caches": (C.c_int, [vp]),
        "rs_debug_erasure_logs_check": (C.c_int64, [C.c_uint64, C.c_uint64, vp, C.c_int]),
        "rs_debug_fft_stamps": (C.c_int, [vp, u64]),
        "rs_jit_stats": (C.c_int, [vp, vp, vp]),
        "rs_fft_compile_check": (C.c_int, [u64, u64, u32, vp, vp, vp]),
        "rs_psyn_compile_check": (C.c_int, [u64, u64, u32, vp, vp]),
        "rs_patterns_kernel_name": (C.c_char_p, [u64, u64, sz, u32, u32]),
        "rs_fft_selftest": (C.c_int, [u64, u64, u32, vp, C.c_int, vp]),
        "rs_fft_decode_compile_check": (C.c_int, [u64, u64, vp, vp]),
        "rs_fft_pdecode_compile_check": (C.c_int, [u64, u64, vp, vp, vp]),
        "rs_fft_decode_selftest": (C.c_int, [u64, u64, u32, C.c_int, vp]),
        "rs_lowrate_selftest": (C.c_int, [u64, u64, C.c_int, u64, vp]),
        "rs_engine_fft": (C.c_int, [vp, u64, sz, u64, u64, u64, u64, u32]),
        "rs_engine_ifft": (C.c_int, [vp, u64, sz, u64, u64, u64, u64, u32]),
        "rs_engine_mul_scalar": (C.c_int, [vp, sz, C.c_uint16, u32]),
        "rs_engine_eval_poly": (C.c_int, [vp, u64]),
        "rs_table_exp": (u16p, []),
        "rs_table_log": (u16p, []),
        "rs_table_skew": (u16p, []),
        "rs_table_log_walsh": (u16p, []),
        "rs_table_mul_128": (C.POINTER(C.c_uint8), []),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(status: int):
    if status:
        detail = lib().rs_last_error().decode(errors="replace")
        raise _ERRORS.get(status, ReedSolomonError)(detail)


def _buf(b) -> C.Array:
    if isinstance(b, (bytes, bytearray, memoryview)):
        return (C.c_uint8 * len(b)).from_buffer_copy(bytes(b))
    import numpy as np
    a = np.ascontiguousarray(b, dtype=np.uint8)
    return (C.c_uint8 * a.size).from_buffer_copy(a.tobytes())


def use_high_rate(original_count: int, recovery_count: int) -> bool:
    """root.zig:397-415."""
    r = lib().rs_use_high_rate(original_count, recovery_count)
    if r < 0:
        _check(-r)
    return bool(r)


def encode(original_count: int, recovery_count: int, original: Sequence[bytes]) -> list:
    """root.zig:14-30 (Encoder.init -> addOriginalShard x n -> encode): the recovery shards."""
    if len(original) == 0:
        raise TooFewOriginalShards("no original shards")  # noqa: F821 (generated class), root.zig:20
    enc = Encoder(original_count, recovery_count, len(original[0]))
    try:
        for o in original:
            enc.add_original_shard(o)
        return enc.encode()
    finally:
        enc.deinit()


def decode(original_count: int, recovery_count: int, original: Sequence[Optional[bytes]],
           recovery: Sequence[Optional[bytes]]) -> list:
    """root.zig:32-84: all original shards (present ones copied through)."""
    sb = next((len(r) for r in recovery[:recovery_count] if r is not None), None)
    if sb is None:  # root.zig:42-58
        if all(original[i] is not None for i in range(original_count)):
            return [bytes(original[i]) for i in range(original_count)]
        raise NotEnoughShards("no recovery shards and originals incomplete")  # noqa: F821
    dec = Decoder(original_count, recovery_count, sb)
    try:
        for i in range(original_count):
            if original[i] is not None:
                dec.add_original_shard(i, original[i])
        for i in range(recovery_count):
            if recovery[i] is not None:
                dec.add_recovery_shard(i, recovery[i])
        return dec.decode()
    finally:
        dec.deinit()


class Encoder:
    """root.zig:86-174 Encoder{init, addOriginalShard, encode, deinit}."""

    def __init__(self, original_count: int, recovery_count: int, shard_bytes: int):
        self._h = C.c_void_p()
        _check(lib().rs_encoder_new(original_count, recovery_count, shard_bytes, C.byref(self._h)))
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    def add_original_shard(self, shard: bytes):
        b = _buf(shard)
        _check(lib().rs_encoder_add_original_shard(self._h, C.addressof(b), len(shard)))

    def encode(self) -> list:
        out = (C.c_void_p * self.recovery_count)()
        _check(lib().rs_encoder_encode(self._h, out))
        return [C.string_at(p, self.shard_bytes) for p in out]

    def reset(self):
        _check(lib().rs_encoder_reset(self._h))

    def deinit(self):
        if self._h:
            lib().rs_encoder_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.deinit()
        except Exception:
            pass


class Decoder:
    """root.zig:176-336 Decoder (private in the reference; same checks)."""

    def __init__(self, original_count: int, recovery_count: int, shard_bytes: int):
        self._h = C.c_void_p()
        _check(lib().rs_decoder_new(original_count, recovery_count, shard_bytes, C.byref(self._h)))
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    def add_original_shard(self, index: int, shard: bytes):
        b = _buf(shard)
        _check(lib().rs_decoder_add_original_shard(self._h, index, C.addressof(b), len(shard)))

    def add_recovery_shard(self, index: int, shard: bytes):
        b = _buf(shard)
        _check(lib().rs_decoder_add_recovery_shard(self._h, index, C.addressof(b), len(shard)))

    def decode(self) -> list:
        out = (C.c_void_p * self.original_count)()
        _check(lib().rs_decoder_decode(self._h, out))
        return [C.string_at(p, self.shard_bytes) for p in out]

    def deinit(self):
        if self._h:
            lib().rs_decoder_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.deinit()
        except Exception:
            pass


# ------------------------------------------------------------ device batch API
def _stream_handle(stream):
    if stream is None:
        import torch
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


def encode_batch_dev(original_count: int, recovery_count: int, data, parity, flags: int = FLAG_CORRECTED,
                     stream=None):
    """data: uint8 CUDA tensor [n, k, shard_bytes] -> parity [n, m, shard_bytes] (in place).

    Asynchronous on `stream` (default: torch's current stream)."""
    n, k, sb = data.shape
    assert k == original_count and parity.shape == (n, recovery_count, sb)
    assert data.is_cuda and parity.is_cuda and data.is_contiguous() and parity.is_contiguous()
    _check(lib().rs_encode_batch_dev(original_count, recovery_count, sb, n, C.c_void_p(data.data_ptr()), 0,
                                     C.c_void_p(parity.data_ptr()), 0, flags, _stream_handle(stream)))


def reconstruct_batch_dev(original_count: int, recovery_count: int, present: Sequence[bool], original,
                          recovery, restored, flags: int = FLAG_CORRECTED, stream=None):
    """original [n, k, sb], recovery [n, m, sb] (missing slots unread) -> restored [n, e, sb]."""
    n, k, sb = original.shape
    pres = (C.c_uint8 * (original_count + recovery_count))(*[1 if p else 0 for p in present])
    _check(lib().rs_reconstruct_batch_dev(
        original_count, recovery_count, sb, n, pres, C.c_void_p(original.data_ptr()), original.stride(0),
        C.c_void_p(recovery.data_ptr()), recovery.stride(0), C.c_void_p(restored.data_ptr()), restored.stride(0),
        flags, _stream_handle(stream)))


def encode_batch_host(original_count: int, recovery_count: int, data, parity, flags: int = FLAG_CORRECTED):
    """Host-resident batch (numpy arrays or CPU tensors, ideally pinned): data [n, k, sb] -> parity [n, m, sb]."""
    n, k, sb = data.shape
    _check(lib().rs_encode_batch_host(original_count, recovery_count, sb, n, C.c_void_p(_host_ptr(data)), 0,
                                      C.c_void_p(_host_ptr(parity)), 0, flags))


def reconstruct_batch_host(original_count: int, recovery_count: int, present, original, recovery, restored,
                           flags: int = FLAG_CORRECTED):
    n, k, sb = original.shape
    pres = (C.c_uint8 * (original_count + recovery_count))(*[1 if p else 0 for p in present])
    _check(lib().rs_reconstruct_batch_host(original_count, recovery_count, sb, n, pres,
                                           C.c_void_p(_host_ptr(original)), 0, C.c_void_p(_host_ptr(recovery)), 0,
                                           C.c_void_p(_host_ptr(restored)), 0, flags))


def _devices(devices):
    if devices is None:
        return None, 0
    arr = (C.c_int * len(devices))(*devices)
    return arr, len(devices)


def encode_batch_host_multi(original_count: int, recovery_count: int, data, parity, devices=None,
                            flags: int = FLAG_CORRECTED):
    """Host batch split over several GPUs (contiguous stripe ranges, one worker per device)."""
    n, k, sb = data.shape
    dv, nd = _devices(devices)
    _check(lib().rs_encode_batch_host_multi(original_count, recovery_count, sb, n, C.c_void_p(_host_ptr(data)), 0,
                                            C.c_void_p(_host_ptr(parity)), 0, flags, dv, nd))


def reconstruct_batch_host_multi(original_count: int, recovery_count: int, present, original, recovery, restored,
                                 devices=None, flags: int = FLAG_CORRECTED):
    n, k, sb = original.shape
    pres = (C.c_uint8 * (original_count + recovery_count))(*[1 if p else 0 for p in present])
    dv, nd = _devices(devices)
    _check(lib().rs_reconstruct_batch_host_multi(original_count, recovery_count, sb, n, pres,
                                                 C.c_void_p(_host_ptr(original)), 0, C.c_void_p(_host_ptr(recovery)),
                                                 0, C.c_void_p(_host_ptr(restored)), 0, flags, dv, nd))


def _host_ptr(a) -> int:
    if hasattr(a, "data_ptr"):
        assert not a.is_cuda and a.is_contiguous()
        return a.data_ptr()
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def reconstruct_batch_dev_patterns(original_count: int, recovery_count: int, present, original, recovery,
                                   restored, status=None, flags: int = FLAG_CORRECTED, stream=None):
    """Per-stripe erasure patterns. present: uint8 CUDA tensor [n, k+m]; restored [n, max_e, sb];
    status: optional int32 CUDA tensor [n] (0 ok, 2 NotEnoughShards, 14 too many erasures for max_e)."""
    n, k, sb = original.shape
    max_e = restored.shape[1]
    _check(lib().rs_reconstruct_batch_dev_patterns(
        original_count, recovery_count, sb, n, C.c_void_p(present.data_ptr()), present.stride(0), max_e,
        C.c_void_p(original.data_ptr()), original.stride(0), C.c_void_p(recovery.data_ptr()), recovery.stride(0),
        C.c_void_p(restored.data_ptr()), restored.stride(0),
        C.c_void_p(status.data_ptr()) if status is not None else None, flags, _stream_handle(stream)))


def encode_kernel_name(k, m, shard_bytes) -> str:
    return lib().rs_encode_kernel_name(k, m, shard_bytes).decode()


def patterns_kernel_name(k, m, shard_bytes, max_e, flags=0) -> str:
    """Path of reconstruct_batch_dev_patterns for these arguments (include/reedsol.h)."""
    return lib().rs_patterns_kernel_name(k, m, shard_bytes, max_e, flags).decode()


def reconstruct_kernel_name(k, m, shard_bytes, present=None) -> str:
    if present is None:
        return lib().rs_reconstruct_kernel_name(k, m, shard_bytes, None).decode()
    pres = (C.c_uint8 * (k + m))(*[1 if p else 0 for p in present])
    return lib().rs_reconstruct_kernel_name(k, m, shard_bytes, pres).decode()


def net_compile_check(k, m, present=None, flags=0) -> float:
    """Generate + hipRTC-compile the bit-sliced network of an encode (present None)
    or of one reconstruct pattern, for gfx950, without a device. Returns ms."""
    ms = C.c_double(0)
    pres = None if present is None else (C.c_uint8 * (k + m))(*[1 if p else 0 for p in present])
    _check(lib().rs_net_compile_check(k, m, pres, flags, C.byref(ms)))
    return ms.value


def jit_stats() -> dict:
    """hipRTC compiles, on-disk code-object cache hits and modules loaded by this process."""
    c, h, mo = C.c_uint64(), C.c_uint64(), C.c_uint64()
    _check(lib().rs_jit_stats(C.byref(c), C.byref(h), C.byref(mo)))
    return {"compiles": c.value, "cache_hits": h.value, "modules": mo.value}


def fft_compile_check(k, m, flags=0) -> dict:
    """Generate + hipRTC-compile the bit-sliced FFT encode kernel of a wide code (no device)."""
    ms, b, ops = C.c_double(), C.c_uint64(), C.c_uint64()
    _check(lib().rs_fft_compile_check(k, m, flags, C.byref(ms), C.byref(b), C.byref(ops)))
    return {"compile_ms": ms.value, "code_bytes": b.value, "valu_ops_per_unit": ops.value}


def psyn_compile_check(k, m, flags=0) -> dict:
    """Generate + hipRTC-compile the per-stripe syndrome-network reconstruct kernel (no device)."""
    ms, b = C.c_double(), C.c_uint64()
    _check(lib().rs_psyn_compile_check(k, m, flags, C.byref(ms), C.byref(b)))
    return {"compile_ms": ms.value, "code_bytes": b.value}


def lowrate_selftest(k, m, trials=8, seed=1) -> int:
    """Host check of the low-rate reconstruct's algebra: wrong restored symbols."""
    bad = C.c_uint64()
    _check(lib().rs_lowrate_selftest(k, m, trials, seed, C.byref(bad)))
    return bad.value


def fft_selftest(k, m, flags=0, skip=None, trials=8) -> int:
    """Host check of the FFT kernel's arithmetic vs the scalar encode: mismatching symbols."""
    bad = C.c_uint64()
    sk = None if skip is None else (C.c_uint8 * k)(*[1 if x else 0 for x in skip])
    _check(lib().rs_fft_selftest(k, m, flags, sk, trials, C.byref(bad)))
    return bad.value


def fft_decode_compile_check(k, m) -> dict:
    """Generate + hipRTC-compile the fused FFT reconstruct kernel (no device)."""
    ms, b = C.c_double(0), C.c_uint64(0)
    _check(lib().rs_fft_decode_compile_check(k, m, C.byref(ms), C.byref(b)))
    return {"compile_ms": ms.value, "code_bytes": b.value}


def fft_pdecode_compile_check(k, m, present) -> dict:
    """Generate + hipRTC-compile the fused FFT reconstruct with one pattern compiled in (no device)."""
    ms, b = C.c_double(0), C.c_uint64(0)
    pres = (C.c_uint8 * (k + m))(*[1 if p else 0 for p in present])
    _check(lib().rs_fft_pdecode_compile_check(k, m, pres, C.byref(ms), C.byref(b)))
    return {"compile_ms": ms.value, "code_bytes": b.value}


def fft_decode_selftest(k, m, erased, trials=8) -> int:
    """Host check of the fused FFT reconstruct's schedule: wrong restored symbols."""
    bad = C.c_uint64(0)
    _check(lib().rs_fft_decode_selftest(k, m, erased, trials, C.byref(bad)))
    return bad.value


def net_wait() -> None:
    """Block until no background plan build or network compile is queued or running
    (include/reedsol.h)."""
    _check(lib().rs_net_wait())


def reconstruct_warm(k, m, shard_bytes, present, flags: int = FLAG_CORRECTED) -> None:
    """Drive one erasure pattern to its steady state (full plan, every kernel its calls
    launch compiled and loaded), blocking; include/reedsol.h rs_reconstruct_warm."""
    pres = (C.c_uint8 * (k + m))(*[1 if p else 0 for p in present])
    _check(lib().rs_reconstruct_warm(k, m, shard_bytes, pres, flags))


def debug_erasure_logs_check(k: int, m: int, received, low: bool = False) -> int:
    """Positions where the library's point-by-point erasure locators differ (mod 65535) from
    evalPoly's two transforms for one received pattern (host only; include/reedsol.h)."""
    buf = (C.c_uint8 * len(received))(*[1 if r else 0 for r in received])
    return int(lib().rs_debug_erasure_logs_check(k, m, buf, 1 if low else 0))


def debug_fail_alloc(n: int) -> int:
    """Arm allocation-failure injection (the n-th allocation fails; n < 0 disarms);
    returns the allocations counted since the previous call (include/reedsol.h)."""
    return int(lib().rs_debug_fail_alloc(n))


def debug_release_caches() -> int:
    """Drop every plan / table / staging cache holding device or pinned memory; returns the
    one-shot contexts left pooled."""
    n = C.c_uint64()
    _check(lib().rs_debug_release_caches(C.byref(n)))
    return n.value


def debug_fft_stamps():
    """Phase stamps of an FFT measurement build (RS_AMD_FFT_DEBUG bit 6): numpy uint64 [8, 64]."""
    import numpy as np
    a = np.zeros(8 * 64, np.uint64)
    _check(lib().rs_debug_fft_stamps(a.ctypes.data_as(C.c_void_p), a.size))
    return a.reshape(8, 64)


def last_kernels() -> list:
    """Kernels the calling thread's most recent compute call launched, in order
    (hipRTC kernels by their symbol, as rocprofv3 names them)."""
    t = lib().rs_last_kernels().decode()
    return t.split(";") if t else []


# ------------------------------------------------------------ engine test shims
def engine_fft(shards: bytearray, shard_count, shard_bytes, pos, size, trunc, skew_delta, flags=0, inverse=False):
    buf = (C.c_uint8 * len(shards)).from_buffer(shards)
    f = lib().rs_engine_ifft if inverse else lib().rs_engine_fft
    _check(f(C.addressof(buf), shard_count, shard_bytes, pos, size, trunc, skew_delta, flags))


def engine_mul_scalar(chunks: bytearray, log_m: int, flags=0):
    buf = (C.c_uint8 * len(chunks)).from_buffer(chunks)
    _check(lib().rs_engine_mul_scalar(C.addressof(buf), len(chunks), log_m, flags))


def engine_eval_poly(erasures, truncated_size: int):
    """erasures: numpy uint16[65536], in place (host FWHT, Generic.zig:200-215)."""
    _check(lib().rs_engine_eval_poly(erasures.ctypes.data_as(C.c_void_p), truncated_size))


def table(name: str):
    """tables.zig: exp / log / skew / log_walsh (u16), or mul_128 ([65536][2][4][16] u8)."""
    import numpy as np
    if name == "mul_128":
        p = lib().rs_table_mul_128()
        if not p:
            raise MemoryError("rs_table_mul_128")
        return np.ctypeslib.as_array(p, shape=(65536, 2, 4, 16)).copy()
    n = {"exp": 65536, "log": 65536, "skew": 65535, "log_walsh": 65536}[name]
    p = getattr(lib(), "rs_table_" + name)()
    return np.ctypeslib.as_array(p, shape=(n,)).copy()
