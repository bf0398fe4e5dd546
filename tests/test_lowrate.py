"""Low-rate codec: pow2(k) < pow2(m), or equal with k > m.

The reference panics here (root.zig:119-121, 226-228), so there is no reference
output to pin: PARITY UNPINNED. The encode follows reed-solomon-simd's low-rate
encoder (the crate the reference ports, benchmarks.zig:1-2), restated in the
oracle (rso_encode_low) and in the library (rs_gf.cpp scalar_encode_low); the
GPU encode is checked against that restatement, and reconstruct — unique for an
MDS code — by round trips. The CPU tests pin the restatement's MDS property:
every k-subset of a codeword determines the data (GF(2) rank of the 16k x 16k
generator block), and the erasure-locator decode's algebra in the low-rate layout
(rs_lowrate_selftest) for every size class up to 65,536-point transforms."""
import itertools

import numpy as np
import pytest

from rs_amd import reedsol_amd as R

LOW_KM = [(1, 2), (2, 4), (3, 5), (3, 6), (5, 9), (4, 16), (10, 20), (7, 40), (16, 64)]
# past 64 recovery shards: FFT-form kernels (rs_lowrate.cpp), register (C <= 32) or generic
LOW_KM_WIDE = [(2, 100), (10, 200), (3, 1000), (17, 130), (100, 600), (40, 100)]
# the verdict's shapes past the old k * m <= 65536 map limit, and size-class extremes
LOW_KM_LARGE = [(300, 1000), (200, 1000), (1000, 4000)]
SELFTEST_KM = LOW_KM + LOW_KM_WIDE + LOW_KM_LARGE + [
    (1, 65535), (2, 65534), (64, 65472), (16384, 40000), (30000, 20000), (32, 33), (60, 40), (33, 65), (255, 257)]


def gf2_rank(rows):
    rows = [int(r) for r in rows]
    rank = 0
    for bit in range(max((r.bit_length() for r in rows), default=0) - 1, -1, -1):
        piv = next((i for i in range(rank, len(rows)) if rows[i] >> bit & 1), None)
        if piv is None:
            continue
        rows[rank], rows[piv] = rows[piv], rows[rank]
        for i in range(len(rows)):
            if i != rank and rows[i] >> bit & 1:
                rows[i] ^= rows[rank]
        rank += 1
    return rank


def generator_columns(oracle, k, m):
    """cols[s][b] = bit vector (16 (k+m) bits) of the codeword of basis symbol b at data shard s."""
    cols = []
    for s in range(k):
        for b in range(16):
            data = np.zeros((k, 64), np.uint8)
            data[s, 0] = (1 << b) & 0xFF  # symbol 0: lo byte at [0], hi byte at [32]
            data[s, 32] = (1 << b) >> 8
            st, rec = oracle.encode_low(k, m, data)
            assert st == 0
            word = [int(data[i, 0]) | int(data[i, 32]) << 8 for i in range(k)]
            word += [int(rec[r, 0]) | int(rec[r, 32]) << 8 for r in range(m)]
            cols.append(word)
    return cols


@pytest.mark.parametrize("k,m", [(1, 2), (2, 4), (3, 5), (3, 6), (4, 7)])
def test_low_rate_restatement_is_mds(oracle, k, m):
    assert R.use_high_rate(k, m) is False
    cols = generator_columns(oracle, k, m)
    for keep in itertools.combinations(range(k + m), k):
        # rows of the 16k x 16k block: for each basis input, its symbols on the kept shards
        rows = []
        for word in cols:
            v = 0
            for idx, sh in enumerate(keep):
                v |= word[sh] << (16 * idx)
            rows.append(v)
        assert gf2_rank(rows) == 16 * k, keep


@pytest.mark.parametrize("k,m", LOW_KM)
def test_low_rate_network_compiles(k, m):
    if k * ((m + 3) // 4) > 64:  # beyond the network size cap: table kernels only
        pytest.skip("no network form")
    assert R.net_compile_check(k, m) > 0


@pytest.mark.parametrize("k,m", SELFTEST_KM)
def test_low_rate_decode_algebra(k, m):
    """scalar_reconstruct_low restores every lost original (host, one symbol per shard)."""
    assert R.use_high_rate(k, m) is False
    assert R.lowrate_selftest(k, m, trials=4, seed=k * 7 + m) == 0


def test_low_rate_limits(monkeypatch):
    R.Encoder(2, 100, 64)
    R.Encoder(100, 600, 64)
    R.Encoder(200, 400, 64)  # past the round-2 map limit k * m <= 65536
    R.Encoder(16, 4097, 64)
    R.Encoder(30000, 20000, 64)
    with pytest.raises(R.UnsupportedShardCount):  # pow2(min) + max > 65536 (root.zig:407)
        R.Encoder(32769, 40000, 64)
    assert R.encode_kernel_name(2, 60, 1 << 16) == "net_encode_low_i2_o60"
    assert R.encode_kernel_name(2, 100, 1 << 16) == "encode_low_reg_w2_nv4"  # > 64 outputs: FFT form
    assert R.encode_kernel_name(100, 600, 1 << 16) == "encode_low_generic_nv1"
    assert R.encode_kernel_name(10, 20, 1 << 16) == "net_encode_low_i10_o20"
    # 256 blocks: a background-compiled network (the FFT-form kernel until it is ready)
    assert R.encode_kernel_name(16, 64, 1 << 16) == "net_encode_low_i16_o64"
    # C >= 128: the block form (C-point transforms); RS_AMD_LOW_BLOCK=0 or C < 128: W points
    assert R.reconstruct_kernel_name(1000, 4000, 4096, [0] * 10 + [1] * 4990) == "low_blocks"
    assert R.reconstruct_kernel_name(100, 600, 4096, [0] * 100 + [1] * 600) == "low_blocks"
    monkeypatch.setenv("RS_AMD_LOW_BLOCK", "0")
    assert R.reconstruct_kernel_name(1000, 4000, 4096, [0] * 10 + [1] * 4990) == "decode_generic_nv1"
    monkeypatch.delenv("RS_AMD_LOW_BLOCK")
    assert R.reconstruct_kernel_name(3, 5, 4096, [0, 1, 1] + [1] * 5).startswith("net_reconstruct_low")
    assert R.patterns_kernel_name(300, 1000, 4096, 300) == "pattern_fft_low"  # per-stripe patterns too
    monkeypatch.setenv("RS_AMD_NET_ASYNC_BLOCKS", "0")
    assert R.encode_kernel_name(16, 64, 1 << 16) == "encode_low_reg_w16_nv1"
    monkeypatch.setenv("RS_AMD_JIT", "0")
    assert R.encode_kernel_name(10, 20, 1 << 16) == "encode_low_reg_w16_nv1"
    assert R.reconstruct_kernel_name(3, 5, 4096, [0, 1, 1] + [1] * 5) == "decode_reg_w16_nv4"
    assert R.reconstruct_kernel_name(40, 100, 4096, [0] * 10 + [1] * 130) == "decode_generic_nv1"  # C = 64


# ----------------------------------------------------------------- GPU
torch = pytest.importorskip("torch")
gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("k,m", LOW_KM + LOW_KM_WIDE)
@pytest.mark.parametrize("jit", ["1", "0"])
@pytest.mark.parametrize("sb", [192, 8192])
def test_low_rate_gpu_vs_oracle_and_roundtrip(oracle, monkeypatch, k, m, jit, sb):
    """jit 1: networks where the map fits one kernel (else FFT form); jit 0: FFT form only."""
    monkeypatch.setenv("RS_AMD_JIT", jit)
    monkeypatch.setenv("RS_AMD_JIT_SYNC", "1")  # every pass's network, not the table kernels of a pending compile
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(k * 97 + m + sb)
    n = 3
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    d = torch.from_numpy(data).to(dev)
    R.encode_batch_dev(k, m, d, par)
    torch.cuda.synchronize()
    got = par.cpu().numpy()
    for s in range(n):
        st, exp = oracle.encode_low(k, m, data[s])
        assert st == 0
        assert (got[s] == exp).all(), (k, m, s)
    for trial in range(3):
        e = int(rng.integers(1, k + 1))
        lost = list(rng.choice(k, size=e, replace=False))
        extra = int(rng.integers(0, m - e + 1))
        lost += [k + int(i) for i in rng.choice(m, size=extra, replace=False)]
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        missing = [i for i in range(k) if not present[i]]
        out = torch.zeros((n, len(missing), sb), dtype=torch.uint8, device=dev)
        R.reconstruct_batch_dev(k, m, present, d, par, out)
        torch.cuda.synchronize()
        assert (out.cpu().numpy() == data[:, missing]).all(), (k, m, sorted(lost))


@pytest.mark.gpu
@gpu
def test_low_rate_exhaustive_rs3_5_one_shot():
    """tests.zig:61-102's protocol on a low-rate code: every presence mask of RS(3,5)."""
    k, m = 3, 5
    orig = [bytes((i * 7 + j) % 256 for j in range(64)) for i in range(k)]
    rec = R.encode(k, m, orig)
    ok = 0
    for mask in range(1 << (k + m)):
        o = [None if mask >> i & 1 else orig[i] for i in range(k)]
        r = [None if mask >> (k + i) & 1 else rec[i] for i in range(m)]
        if bin(mask).count("1") <= m:
            assert R.decode(k, m, o, r) == orig, mask
            ok += 1
        else:
            with pytest.raises(R.NotEnoughShards):
                R.decode(k, m, o, r)
    assert ok == sum(1 for mask in range(1 << 8) if bin(mask).count("1") <= 5)


@pytest.mark.gpu
@gpu
def test_low_rate_background_network(oracle, monkeypatch):
    """RS(16,64) low rate: the 16 x 64 encode map (256 blocks) compiles in the
    background; table-kernel calls before, network calls after, all == oracle."""
    monkeypatch.delenv("RS_AMD_JIT", raising=False)
    monkeypatch.delenv("RS_AMD_JIT_SYNC", raising=False)
    k, m, sb, n = 16, 64, 8192, 2
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(1664)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    exp = np.stack([oracle.encode_low(k, m, data[s])[1] for s in range(n)])
    d = torch.from_numpy(data).to(dev)

    def enc():
        p = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
        R.encode_batch_dev(k, m, d, p)
        torch.cuda.synchronize()
        return p.cpu().numpy()

    for _ in range(2):
        assert (enc() == exp).all()
    R.net_wait()
    assert (enc() == exp).all()


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("k,m", LOW_KM_LARGE)
@pytest.mark.parametrize("sb,n", [(4096, 2), (65536, 1)])
def test_low_rate_large_codes(oracle, k, m, sb, n):
    """Codes past the round-2 limit (k * m > 65536; chunk C = 256 / 512 / 1024, decode
    transforms of W = 2048 / 8192 points): the generic FFT-form encode bit-exact against
    the oracle's rso_encode_low, and the erasure-locator reconstruct restoring random
    erasures (originals and recovery shards) bit-exact. Parity unpinned."""
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(k + m + sb)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    par = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, d, par)
    torch.cuda.synchronize()
    got = par.cpu().numpy()
    for s in range(n):
        st, exp = oracle.encode_low(k, m, data[s])
        assert st == 0
        assert np.array_equal(got[s], exp), s
    for e in (1, min(k, 97), k):
        present = np.ones(k + m, np.uint8)
        present[rng.choice(k, size=e, replace=False)] = 0
        present[k + rng.choice(m, size=int(rng.integers(0, m - e + 1)), replace=False)] = 0
        missing = [i for i in range(k) if not present[i]]
        out = torch.zeros((n, len(missing), sb), dtype=torch.uint8, device=dev)
        R.reconstruct_batch_dev(k, m, present, d, par, out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), data[:, missing]), e


def _low_roundtrip(oracle, k, m, sb, n, present, seed, check_encode=True):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    par = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, d, par)
    torch.cuda.synchronize()
    if check_encode:
        st, exp = oracle.encode_low(k, m, data[0])
        assert st == 0 and np.array_equal(par[0].cpu().numpy(), exp)
    missing = [i for i in range(k) if not present[i]]
    out = torch.zeros((n, len(missing), sb), dtype=torch.uint8, device=dev)
    R.reconstruct_batch_dev(k, m, present, d, par, out)
    torch.cuda.synchronize()
    return np.array_equal(out.cpu().numpy(), data[:, missing])


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("form", ["1", "0"])
@pytest.mark.parametrize("k,m,sb,n,case", [
    (300, 1000, 4096, 2, "first"),      # C = 512: the rows used all in block 1
    (300, 1000, 4096, 2, "spread"),     # the first 450 recovery rows lost: rows used in blocks 1 and 2
    (100, 600, 2048, 3, "tail"),        # C = 128 (2-point last phases), rows used in the last block
    (128, 1000, 192 * 4, 2, "all"),     # every original lost
    (1000, 4000, 4096, 2, "one"),       # C = 1024, one original lost
    (5000, 9000, 64, 1, "spread"),      # C = 8192: three-phase transforms (LSUM, then SCATTER)
    (16384, 40000, 64, 1, "all"),       # C = 16384, W = 65536
])
def test_low_rate_block_form(oracle, monkeypatch, form, k, m, sb, n, case):
    """The low-rate reconstruct in block form (rs_lowrate.cpp, C-point transforms: the
    residual's syndromes, per-block IFFTs, the derivative split as k_dphase's) against the
    W-point decode (form 0) on the same losses: the restored originals are the lost data
    either way (an MDS code's reconstruct is unique). Parity unpinned, as every low-rate path."""
    monkeypatch.setenv("RS_AMD_LOW_BLOCK", form)
    monkeypatch.setenv("RS_AMD_JIT", "0")  # no reconstruct network for the small losses
    rng = np.random.default_rng(k + m + len(case))
    C = 1 << (k - 1).bit_length()
    present = np.ones(k + m, np.uint8)
    if case == "all":
        present[:k] = 0
        present[k:k + m // 3] = 0
    elif case == "one":
        present[int(rng.integers(0, k))] = 0
    else:
        e = min(k, 97)
        present[rng.choice(k, size=e, replace=False)] = 0
        if case == "spread":
            present[k:k + C - e // 2] = 0
        elif case == "tail":
            present[k:k + m - e - 3] = 0
    assert int(present.sum()) >= k
    name = R.reconstruct_kernel_name(k, m, sb, list(present))
    assert name == ("low_blocks" if form == "1" else "decode_generic_nv1"), name
    assert _low_roundtrip(oracle, k, m, sb, n, present, seed=k * 3 + m, check_encode=k <= 1000)


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("form", ["1", "0"])
@pytest.mark.parametrize("cap_mb", ["1", "64"])
def test_low_rate_reconstruct_scratch_cap(oracle, monkeypatch, form, cap_mb):
    """The generic low-rate reconstructs under the scratch cap: a stripe's scratch (block form
    3C + ylen rows with the whole derivative (two IFFT phases, C <= 4096), 2C + 2 ylen with the
    split one (low_block_rows); W-point decode W + ylen rows; several MiB each for RS(300,1000)
    4 KiB) above a 1 MiB cap still runs, one stripe per slice; 64 MiB takes all three
    at once."""
    monkeypatch.setenv("RS_AMD_LOW_BLOCK", form)
    monkeypatch.setenv("RS_AMD_SCRATCH_CAP_MB", cap_mb)
    monkeypatch.setenv("RS_AMD_JIT", "0")
    k, m, sb, n = 300, 1000, 4096, 3
    present = np.ones(k + m, np.uint8)
    present[np.arange(0, 300, 3)] = 0
    present[k:k + 50] = 0
    assert _low_roundtrip(oracle, k, m, sb, n, present, seed=int(cap_mb) + 7 * int(form), check_encode=True)


@pytest.mark.gpu
@gpu
def test_low_rate_block_form_many_blocks(oracle):
    """C = 128, W = 65536 (512 blocks): every original lost and the first 60,000 recovery rows
    too, so the rows used sit in blocks 469 and 470 (the launch walks 470 blocks)."""
    k, m, sb = 128, 65408, 64
    present = np.ones(k + m, np.uint8)
    present[:k] = 0
    present[k:k + 60000] = 0
    assert R.reconstruct_kernel_name(k, m, sb, list(present)) == "low_blocks"
    assert _low_roundtrip(oracle, k, m, sb, 1, present, seed=128, check_encode=False)


@pytest.mark.gpu
@gpu
def test_low_rate_block_form_skips_empty_blocks(oracle, monkeypatch):
    """the block form launches only the blocks holding a recovery row read (an empty
    block's syndromes are zero and so is what it adds): C = 128, rows read in blocks 3 and 9 only
    (1-2 and 4-8 skipped; the first block run stores A', the second accumulates). With
    RS_AMD_LOW_TRIM=0 (every present row read) the kernel name and the plan agree on the W-point
    decode."""
    monkeypatch.setenv("RS_AMD_JIT", "0")
    k, m, sb = 128, 1900, 256
    present = np.zeros(k + m, np.uint8)
    present[k // 2:k] = 1                            # 64 originals lost
    present[k + 2 * 128 + 5:k + 2 * 128 + 37] = 1    # 32 rows in block 3
    present[k + 8 * 128 + 1:k + 8 * 128 + 33] = 1    # 32 rows in block 9
    assert R.reconstruct_kernel_name(k, m, sb, list(present)) == "low_blocks"
    assert _low_roundtrip(oracle, k, m, sb, 2, present, seed=5, check_encode=False)
    monkeypatch.setenv("RS_AMD_LOW_TRIM", "0")
    assert R.reconstruct_kernel_name(k, m, sb, list(present)) != "low_blocks"
    assert _low_roundtrip(oracle, k, m, sb, 2, present, seed=6, check_encode=False)


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("k,m", [(1, 65535), (64, 65472), (2, 40000)])
def test_low_rate_widest_transforms(oracle, k, m):
    """65,536-point decode transforms (W = ceilPow2(C + m) = 65536) on 64-byte shards."""
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(k + m)
    sb = 64
    data = rng.integers(0, 256, (1, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    par = torch.zeros((1, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, d, par)
    torch.cuda.synchronize()
    st, exp = oracle.encode_low(k, m, data[0])
    assert st == 0 and np.array_equal(par.cpu().numpy()[0], exp)
    present = np.zeros(k + m, np.uint8)  # every original lost, the last k recovery shards kept
    present[k + m - k:] = 1
    out = torch.zeros((1, k, sb), dtype=torch.uint8, device=dev)
    R.reconstruct_batch_dev(k, m, present, d, par, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), data)


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("cap_mb", ["1", "3", "64"])
def test_low_rate_encode_scratch_cap(oracle, monkeypatch, cap_mb):
    """The generic low-rate encode keeps a stripe's scratch within the cap: its recovery chunks
    run in groups of G with (1 + G) C shard-regions per stripe (G = 1 when even two regions
    exceed the cap). RS(300,1000) 4 KiB: C = 512, region 2 MiB, 2 chunks; cap 1 MiB (below
    one stripe's two regions), 3 MiB (one chunk per launch), 64 MiB (both chunks at once)."""
    monkeypatch.setenv("RS_AMD_SCRATCH_CAP_MB", cap_mb)
    k, m, sb, n = 300, 1000, 4096, 3
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(300 + int(cap_mb))
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, torch.from_numpy(data).to(dev), par)
    torch.cuda.synchronize()
    got = par.cpu().numpy()
    for s in range(n):
        st, exp = oracle.encode_low(k, m, data[s])
        assert st == 0 and np.array_equal(got[s], exp), s


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("k,m,sb", [(3, 5, 64), (5, 9, 100), (10, 20, 4096), (17, 130, 192), (100, 600, 2048), (300, 1000, 4096)])
def test_low_rate_per_stripe_patterns(oracle, k, m, sb):
    """rs_reconstruct_batch_dev_patterns on low-rate codes (round 3 rejected them): one
    erasure pattern per stripe, originals and recovery shards lost, stripe 0 with exactly k
    present, one stripe with too few (NotEnoughShards, nothing written), and restored slots
    past each stripe's losses left alone. Encode checked against rso_encode_low; the
    reconstruct of an MDS code is unique, so the lost data is the expectation."""
    n = 6
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(k * 31 + m + sb)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    par = torch.zeros((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, d, par)
    torch.cuda.synchronize()
    st, exp0 = oracle.encode_low(k, m, data[0])
    assert st == 0 and np.array_equal(par[0].cpu().numpy(), exp0)
    present = np.ones((n, k + m), np.uint8)
    for s in range(n):
        e = k if s == 0 else int(rng.integers(1, k + 1))
        present[s, rng.choice(k, size=e, replace=False)] = 0
        extra = m - e if s == 0 else int(rng.integers(0, m - e + 1))
        present[s, k + rng.choice(m, size=extra, replace=False)] = 0
    present[n - 1, :] = 0
    present[n - 1, k + m - (k - 1):] = 1  # k - 1 present
    max_e = k
    out = torch.full((n, max_e, sb), 0xAB, dtype=torch.uint8, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    assert R.patterns_kernel_name(k, m, sb, max_e) == "pattern_fft_low"
    R.reconstruct_batch_dev_patterns(k, m, torch.from_numpy(present).to(dev), d, par, out, status)
    torch.cuda.synchronize()
    out, status = out.cpu().numpy(), status.cpu().numpy()
    for s in range(n - 1):
        missing = [i for i in range(k) if not present[s, i]]
        assert status[s] == 0, s
        assert np.array_equal(out[s, :len(missing)], data[s, missing]), (s, missing)
        assert (out[s, len(missing):] == 0xAB).all(), s
    assert status[n - 1] == 2  # RS_ERR_NOT_ENOUGH_SHARDS
