"""CPU-side checks of librs_amd.so: it loads, exports every symbol include/reedsol.h
declares, and its host logic (tables, rate selection, evalPoly, argument
validation) matches the oracle — no device compute here."""
import re

import numpy as np
import pytest

from rs_amd import HEADER, reedsol_amd as R


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(rs_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    L = R.lib()
    names = header_functions()
    assert len(names) >= 28
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_symbols_match_ctypes_signatures():
    L = R.lib()
    # every declared function is bound with a signature in the Python mirror
    for n in header_functions():
        assert getattr(L, n).argtypes is not None, n


def test_tables_match_oracle(oracle):
    for name in ("exp", "log", "skew", "log_walsh"):
        assert (R.table(name) == oracle.table(name)).all(), name


def test_mul_128_matches_oracle(oracle):
    """tables.zig:94-118 mul_128 (the Lut seam) through the C ABI == the oracle's table."""
    got = R.table("mul_128")
    assert got.shape == (65536, 2, 4, 16)
    assert (got.reshape(-1) == oracle.mul128().reshape(-1)).all()


@pytest.mark.parametrize("k,m", [(10, 4), (5, 5), (3, 4), (4, 3), (2, 4), (0, 4), (4, 0), (65537, 1),
                                 (32768, 32768), (32769, 32768), (200, 55), (1, 1), (65536, 1)])
def test_use_high_rate_matches_oracle(oracle, k, m):
    assert R.lib().rs_use_high_rate(k, m) == oracle.use_high_rate(k, m)


@pytest.mark.parametrize("trunc", [1, 6, 14, 20, 255, 4096])
def test_eval_poly_matches_oracle(oracle, trunc):
    rng = np.random.default_rng(trunc)
    e = np.zeros(65536, np.uint16)
    e[:trunc] = rng.integers(0, 2, trunc)
    a, b = e.copy(), e.copy()
    R.engine_eval_poly(a, trunc)
    oracle.eval_poly(b, trunc)
    assert (a == b).all()


def test_status_names_mirror_zig_errors():
    L = R.lib()
    assert L.rs_status_name(2) == b"NotEnoughShards"
    assert L.rs_status_name(1) == b"TooFewOriginalShards"
    assert L.rs_status_name(8) == b"DuplicateShardIndex"
    for i, n in enumerate(R._STATUS_NAMES):
        assert L.rs_status_name(i).decode() == n


def test_validation_precedes_device():
    """Argument errors are reported with the reference's precedence, before any device use."""
    with pytest.raises(R.UnsupportedShardCount):
        R.Encoder(0, 4, 64)
    with pytest.raises(R.InvalidShardSize):
        R.Encoder(10, 4, 63)
    with pytest.raises(R.InvalidShardSize):
        R.Encoder(10, 4, 0)
    R.Encoder(200, 400, 64).deinit()  # low rate: accepted (the reference panics on any low rate)
    R.Encoder(10, 4, 66).deinit()  # tails accepted (root.zig:338-348 layout; the reference panics)
    with pytest.raises(R.TooFewOriginalShards):
        R.encode(10, 4, [])
    enc = R.Encoder(2, 1, 64)
    enc.add_original_shard(bytes(64))
    with pytest.raises(R.DifferentShardSize):
        enc.add_original_shard(bytes(128))
    with pytest.raises(R.TooFewOriginalShards):
        enc.encode()
    enc.add_original_shard(bytes(64))
    with pytest.raises(R.TooManyOriginalShards):
        enc.add_original_shard(bytes(64))
    dec = R.Decoder(3, 2, 64)
    with pytest.raises(R.InvalidShardIndex):
        dec.add_original_shard(3, bytes(64))
    dec.add_original_shard(0, bytes(64))
    with pytest.raises(R.DuplicateShardIndex):
        dec.add_original_shard(0, bytes(64))
    with pytest.raises(R.InvalidShardIndex):
        dec.add_recovery_shard(2, bytes(64))
    with pytest.raises(R.NotEnoughShards):
        dec.decode()
    # root.zig:42-58: no recovery shards + complete originals -> copy-through, no device
    out = R.decode(2, 2, [b"a" * 64, b"b" * 64], [None, None])
    assert out == [b"a" * 64, b"b" * 64]
    with pytest.raises(R.NotEnoughShards):
        R.decode(2, 2, [b"a" * 64, None], [None, None])


def test_device_entry_points_fail_loudly_without_gpu():
    """No CPU fallback: with no gfx950 device the compute entry points raise NoDevice."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(R.NoDevice):
        R.encode(4, 2, [bytes(64)] * 4)
    with pytest.raises(R.NoDevice):
        R.engine_mul_scalar(bytearray(64), 7)
    with pytest.raises(R.NoDevice):
        R.reconstruct_warm(10, 4, 4096, [0] + [1] * 13)
    assert R.last_kernels() == []  # nothing launched by the failed call
    with pytest.raises(R.NotEnoughShards):  # validation first
        R.reconstruct_warm(10, 4, 4096, [0] * 5 + [1] * 9)
    R.debug_fail_alloc(-1)  # injection arms / disarms without a device
    assert R.debug_fail_alloc(-1) == 0
    assert R.debug_release_caches() == 0


def test_kernel_selection_network(monkeypatch):
    """Bit-sliced network kernels (rs_jit.hpp) for shards in whole 4 KiB units and <= 16 outputs."""
    assert R.encode_kernel_name(10, 4, 1 << 20) == "net_encode_i10_o4"
    assert R.reconstruct_kernel_name(10, 4, 1 << 20) == "net_reconstruct_i10_o4"
    assert R.encode_kernel_name(16, 16, 4096) == "net_encode_i16_o16"
    present = [1] * 20
    present[3] = 0
    assert R.reconstruct_kernel_name(16, 4, 8192, present) == "net_reconstruct_i16_o1"
    # 1 / 2 KiB shards: reconstructs on the networks, encodes on the table kernels unless forced
    present4 = [0, 0, 0, 0] + [1] * 10
    assert R.reconstruct_kernel_name(10, 4, 2048, present4) == "net_reconstruct_i10_o4"  # 2 stripes per wave unit
    assert R.reconstruct_kernel_name(10, 4, 1024, present4) == "net_reconstruct_i10_o4"  # 4 stripes per wave unit
    assert R.encode_kernel_name(10, 4, 2048).startswith("encode_reg_w4")
    assert R.encode_kernel_name(10, 4, 3072) == "encode_reg_w4_nv2"  # not a whole 4 KiB unit
    # wide codes (chunk 32 / 64): the bit-sliced FFT kernel (rs_fftnet.hpp)
    assert R.encode_kernel_name(200, 55, 1 << 18) == "net_fft_encode_i200_o55"
    assert R.encode_kernel_name(100, 20, 1 << 18) == "net_fft_encode_i100_o20"
    # wide code, 55 / 20 erasures: the first calls run the fused FFT reconstruct with the
    # pattern as data (round 3), the steady state the same kernel with the pattern compiled
    # in (round 4, background-compiled); RS_AMD_FDEC=1 the pattern as data for good,
    # RS_AMD_FDEC=0 syndromes on the FFT kernel + the 55 x 55 map as a network
    assert R.reconstruct_kernel_name(200, 55, 1 << 18) == "net_fft_pdecode_i200_o55"
    p20 = [0] * 20 + [1] * 235
    assert R.reconstruct_kernel_name(200, 55, 1 << 18, p20) == "net_fft_pdecode_i200_o55"
    monkeypatch.setenv("RS_AMD_FDEC", "1")
    assert R.reconstruct_kernel_name(200, 55, 1 << 18) == "net_fft_decode_i200_o55"
    monkeypatch.setenv("RS_AMD_FDEC", "0")
    assert R.reconstruct_kernel_name(200, 55, 1 << 18) == "syndrome+net_fft_encode_i200_o55+net_syndrome_i55_o55"


def test_kernel_selection_async_cap(monkeypatch):
    """RS_AMD_NET_ASYNC_BLOCKS=0 keeps large maps on the table kernels."""
    monkeypatch.setenv("RS_AMD_NET_ASYNC_BLOCKS", "0")
    monkeypatch.setenv("RS_AMD_FDEC", "0")
    assert R.reconstruct_kernel_name(200, 55, 1 << 18) == "syndrome+net_fft_encode_i200_o55+decode_mtile16_nv1"
    monkeypatch.setenv("RS_AMD_FFT", "0")
    assert R.encode_kernel_name(100, 20, 1 << 18) == "encode_reg_w32_nv1"
    assert R.encode_kernel_name(200, 55, 1 << 18) == "encode_ws64_nv1"


def test_kernel_selection(monkeypatch):
    monkeypatch.setenv("RS_AMD_JIT", "0")
    assert R.encode_kernel_name(10, 4, 1 << 20) == "encode_reg_w4_nv4"
    assert R.reconstruct_kernel_name(10, 4, 1 << 20) == "decode_matrix_e4_nv4"
    # wide code, 55 erasures: encode the received data, then the 55 x 55 syndrome solve
    assert R.reconstruct_kernel_name(200, 55, 1 << 18) == "syndrome+encode_ws64_nv1+decode_mtile16_nv1"
    present = [1] * 255
    for i in (3, 77, 150, 199):
        present[i] = 0
    assert R.reconstruct_kernel_name(200, 55, 1 << 18, present) == "decode_matrix_e4_nv4"  # 4 x 200 MACs cheaper
    monkeypatch.setenv("RS_AMD_DECODE", "matrix")
    assert R.reconstruct_kernel_name(200, 55, 1 << 18) == "decode_mtile16_nv1"
    monkeypatch.delenv("RS_AMD_DECODE")
    assert R.reconstruct_kernel_name(200, 55, 320).startswith("decode_generic")
    assert R.encode_kernel_name(200, 55, 1 << 18) == "encode_ws64_nv1"
    assert R.encode_kernel_name(100, 20, 1 << 18) == "encode_reg_w32_nv1"


def test_net_kernels_compile_for_gfx950():
    """The generated bit-sliced network kernels (encode and one reconstruct pattern of
    the bench shape, plus a quirk-mode encode) compile with hipRTC for gfx950 on a host
    without a GPU: what a plan does before its first launch."""
    assert R.net_compile_check(10, 4) > 0
    assert R.net_compile_check(10, 4, [0, 0, 0, 0] + [1] * 10) > 0
    assert R.net_compile_check(4, 2, None, 3) > 0
    with pytest.raises(R.InvalidArgument):
        R.net_compile_check(200, 55)  # 55 outputs: no network form
    # 32 of 200 data shards lost: the direct map (1,600 blocks) is past the background
    # cap, so the plan's network is the 32 x 32 syndrome map (256 blocks)
    present = [1] * 255
    for i in range(0, 64, 2):
        present[i] = 0
    assert R.net_compile_check(200, 55, present) > 0


@pytest.mark.parametrize("pieces", ["2", "4"])
def test_small_shard_net_kernels_compile_for_gfx950(monkeypatch, pieces):
    """The 2 KiB / 1 KiB-shard network variants (wave units spanning 2 / 4 stripes)
    compile with hipRTC for gfx950 without a GPU (RS_AMD_NET_CHECK_PIECES)."""
    monkeypatch.setenv("RS_AMD_NET_CHECK_PIECES", pieces)
    assert R.net_compile_check(10, 4) > 0
    assert R.net_compile_check(10, 4, [0, 0, 0, 0] + [1] * 10) > 0


@pytest.mark.parametrize("k,m,flags", [(200, 55, 0), (200, 55, 3), (100, 20, 0), (64, 64, 1), (40, 50, 0),
                                       (1000, 64, 0), (33, 17, 2),
                                       # chunk 16 (the per-stripe pattern path's syndromes)
                                       (16, 16, 0), (40, 12, 3), (100, 16, 0), (9, 9, 0), (64, 10, 2)])
def test_fft_kernel_arithmetic(k, m, flags):
    """The bit-sliced FFT encode kernel's schedule with its (u, v)-coordinate matrices
    (Cantor-basis subfield split) reproduces the codec's scalar encode, both quirk
    modes, with and without erased (skipped) shards — host only."""
    assert R.fft_selftest(k, m, flags, trials=6) == 0
    skip = [1 if (i * 7) % 5 == 0 else 0 for i in range(k)]
    assert R.fft_selftest(k, m, flags, skip=skip, trials=4) == 0


def test_fft_kernel_compiles_for_gfx950(monkeypatch):
    info = R.fft_compile_check(200, 55)
    assert info["code_bytes"] > 10000 and info["valu_ops_per_unit"] > 0
    monkeypatch.setenv("RS_AMD_FFT_CHECK_PIECES", "2")  # 1 KiB shards: units of two stripes
    assert R.fft_compile_check(32, 32)["code_bytes"] > 10000


def test_shared_network_compiles_for_gfx950(monkeypatch):
    """Two output tiles: the shared-input form (one workgroup of tile waves per unit,
    inputs staged through LDS) is generated and compiles; so does the classic form."""
    assert R.net_compile_check(16, 16) > 0
    # 24 outputs = 3 tiles of 8: four balanced waves of 6 (RS_AMD_NET_BALANCE), or three
    assert R.net_compile_check(24, 24) > 0
    monkeypatch.setenv("RS_AMD_NET_BALANCE", "0")
    assert R.net_compile_check(24, 24) > 0
    monkeypatch.setenv("RS_AMD_NET_SHARED", "0")
    assert R.net_compile_check(16, 16) > 0


def test_patterns_path_selection(monkeypatch):
    """rs_reconstruct_batch_dev_patterns' path per code (include/reedsol.h)."""
    assert R.patterns_kernel_name(10, 4, 1 << 20, 4) == "psyn_k10_m4"
    assert R.patterns_kernel_name(64, 4, 4096, 4) == "psyn_k64_m4"
    # wide codes (round 3): the fused FFT reconstruct with per-stripe decode blocks for
    # max_e >= 0.6 m, FFT syndromes + the generic solve below that
    assert R.patterns_kernel_name(200, 55, 1 << 18, 8) == "fft_syndromes+psyn_solve"
    assert R.patterns_kernel_name(200, 55, 1 << 18, 55) == "fft_decode"
    assert R.patterns_kernel_name(200, 55, 1 << 18, 33) == "fft_decode"
    assert R.patterns_kernel_name(200, 55, 1 << 18, 32) == "fft_syndromes+psyn_solve"
    assert R.patterns_kernel_name(200, 55, 6144, 8) == "fft_decode"  # whole 2 KiB units
    assert R.patterns_kernel_name(200, 55, 5120, 8) == "pattern_fft"  # no whole 2 KiB units
    assert R.patterns_kernel_name(10, 4, 1 << 20, 4, 1) == "pattern_matrix" or \
        R.patterns_kernel_name(10, 4, 1 << 20, 4, 1) == "pattern_fft"  # D1: no syndrome network
    assert R.patterns_kernel_name(10, 4, 2048, 4) == "pattern_matrix"  # below the 4 KiB unit
    assert R.patterns_kernel_name(5, 5, 4096, 5) == "psyn_k5_m5"
    # mid-band codes (round 3): the fused syndrome network for k <= 256, m <= 8; the
    # chunk-16 fused FFT reconstruct for 9 <= m <= 16
    assert R.patterns_kernel_name(100, 4, 1 << 20, 4) == "psyn_k100_m4"
    assert R.patterns_kernel_name(32, 8, 1 << 20, 8) == "psyn_k32_m8"
    assert R.patterns_kernel_name(40, 12, 1 << 20, 12) == "fft_decode"
    assert R.patterns_kernel_name(16, 16, 1 << 20, 16) == "fft_decode"
    assert R.patterns_kernel_name(64, 16, 1 << 20, 16) == "fft_decode"
    # RS_AMD_FDEC=0: FFT syndromes + the generic e x e solve (max_e > 8: output groups of 8)
    monkeypatch.setenv("RS_AMD_FDEC", "0")
    assert R.patterns_kernel_name(200, 55, 1 << 18, 9) == "fft_syndromes+psyn_solve"
    assert R.patterns_kernel_name(16, 16, 1 << 20, 16) == "fft_syndromes+psyn_solve"
    monkeypatch.delenv("RS_AMD_FDEC")
    assert R.patterns_kernel_name(300, 8, 1 << 20, 8) in ("pattern_matrix", "pattern_fft")  # k > 256
    monkeypatch.setenv("RS_AMD_PATTERNS", "fft")
    assert R.patterns_kernel_name(10, 4, 1 << 20, 4) == "pattern_fft"


def test_psyn_kernel_compiles_for_gfx950():
    """Per-stripe syndrome network (rs_psyn.hpp): generated and compiled per code; codes
    outside its range (k > 256 with m <= 8, D1 multiply, low rate) have none."""
    assert R.psyn_compile_check(10, 4)["code_bytes"] > 10000
    assert R.psyn_compile_check(4, 2, 2)["code_bytes"] > 1000
    assert R.psyn_compile_check(5, 5)["code_bytes"] > 10000  # m in 5..8: one output at a time
    assert R.psyn_compile_check(100, 20)["code_bytes"] > 10000  # wide: FFT with per-stripe masks + solve
    assert R.psyn_compile_check(40, 12)["code_bytes"] > 10000  # chunk 16: the same, two waves per workgroup
    for k, m, flags in ((300, 8, 0), (10, 4, 1), (2, 4, 0)):
        with pytest.raises(R.InvalidArgument):
            R.psyn_compile_check(k, m, flags)


@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("flags", [0, 3])
def test_fft_inverse_arithmetic(monkeypatch, k, flags):
    """Every original lost, RS(k,k) with k = chunk: the inverse FFT kernel's schedule
    (IFFT at skew 0, FFT at skew chunk) yields data whose scalar encode is the input."""
    monkeypatch.setenv("RS_AMD_FFT_CHECK_INVERSE", "1")
    assert R.fft_selftest(k, k, flags, trials=6) == 0
    present = np.ones(2 * k, np.uint8)
    present[:k] = 0
    assert R.reconstruct_kernel_name(k, k, 1024, present) == f"net_fft_inverse_i{k}_o{k}"
    assert R.reconstruct_kernel_name(k, k, 1 << 20, present) == f"net_fft_inverse_i{k}_o{k}"
    present[k] = 0  # a recovery shard lost too: not enough shards, no inverse form
    assert R.reconstruct_kernel_name(k, k, 1024, present) != f"net_fft_inverse_i{k}_o{k}"


def test_disk_code_object_cache(tmp_path):
    """A second process compiling the same network finds the code object on disk."""
    import os
    import subprocess
    import sys
    import json
    code = ("import sys, json; sys.path.insert(0, %r); import reedsol_amd as R; "
            "R.net_compile_check(10, 4); print(json.dumps(R.jit_stats()))") % os.path.dirname(os.path.dirname(R.__file__))
    env = dict(os.environ, RS_AMD_CACHE_DIR=str(tmp_path))
    first = json.loads(subprocess.run([sys.executable, "-c", code], env=env, check=True, capture_output=True,
                                      text=True).stdout.strip().splitlines()[-1])
    second = json.loads(subprocess.run([sys.executable, "-c", code], env=env, check=True, capture_output=True,
                                       text=True).stdout.strip().splitlines()[-1])
    assert first["compiles"] >= 1 and first["cache_hits"] == 0
    assert second["compiles"] == 0 and second["cache_hits"] >= 1
    assert any(p.suffix == ".co" for p in tmp_path.iterdir())
