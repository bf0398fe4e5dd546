"""GPU parity of the fused FFT reconstruct (fftnet::Spec::decode): the
syndromes of e recovery rows and the reference's erasure-locator decode
(root.zig:268-335) restricted to the residual codeword, in one kernel with the pattern
as data. RS_AMD_FDEC=1 makes the batch syndrome path run it (and fail loudly if it
cannot). Restored originals are unique (MDS), so they are compared with the erased data
bit for bit, and a few cases also with the oracle's reconstruct."""
import os

import numpy as np
import pytest

from helpers import splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402

DEV = torch.device("cuda:0")


def reconstruct(k, m, present, data, par, flags=0):
    n, _, sb = data.shape
    e = int(k - np.sum(present[:k]))
    out = torch.zeros((n, max(e, 1), sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, torch.from_numpy(data).to(DEV), torch.from_numpy(par).to(DEV), out,
                            flags)
    torch.cuda.synchronize()
    return out.cpu().numpy()[:, :e]


@pytest.fixture
def fdec(monkeypatch):
    monkeypatch.setenv("RS_AMD_FDEC", "1")
    monkeypatch.setenv("RS_AMD_DECODE", "syndrome")


# chunk 16 / 32 / 64, one to sixteen data blocks, last block partial or full
# RS(1000,64) (16 data blocks; its fused kernel compiles for ~100 s with hipRTC) runs when
# RS_AMD_SLOW_TESTS=1
SLOW = pytest.mark.skipif(os.environ.get("RS_AMD_SLOW_TESTS") != "1", reason="~100 s compile: RS_AMD_SLOW_TESTS=1")
FDEC_KM = [(200, 55), (33, 17), (64, 64), (100, 20), (16, 16), (30, 9), (128, 32), pytest.param(1000, 64, marks=SLOW),
           (65, 33)]
# pattern-compiled kernels (k <= 256): one hipRTC compile per pattern, 1-16 s each
PDEC_KM = [(200, 55), (33, 17), (100, 20), (16, 16), (65, 33)]


@pytest.mark.parametrize("k,m", FDEC_KM)
def test_fdec_random_patterns(oracle, fdec, k, m):
    rng = np.random.default_rng(k * 7919 + m)
    sb, n = 4096, 3
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=4)
    for trial in range(4):
        e = int(rng.integers(1, min(k, m) + 1)) if trial else min(k, m)
        lost = list(rng.choice(k, size=e, replace=False))
        extra = int(rng.integers(0, m - e + 1))
        lost += [k + int(i) for i in rng.choice(m, size=extra, replace=False)]
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        got = reconstruct(k, m, present, data, par)
        assert (got == data[:, present[:k] == 0]).all(), (k, m, sorted(lost))


@pytest.mark.parametrize("k,m", PDEC_KM)
def test_pdec_pattern_compiled(oracle, monkeypatch, k, m):
    """The fused reconstruct with the pattern compiled in (fftnet::Spec::present: constant
    locator multiplies, static rows / blocks / outputs, pruned butterflies), reached through
    rs_reconstruct_warm; random losses incl. surplus recovery rows, against the data."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    rng = np.random.default_rng(k * 7907 + m)
    sb, n = 4096, 3
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=4)
    for trial in range(2):
        e = int(rng.integers(max(1, min(k, m) // 2), min(k, m) + 1)) if trial else min(k, m)
        lost = list(rng.choice(k, size=e, replace=False))
        lost += [k + int(i) for i in rng.choice(m, size=int(rng.integers(0, m - e + 1)), replace=False)]
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        R.reconstruct_warm(k, m, sb, present)
        got = reconstruct(k, m, present, data, par)
        ran = R.last_kernels()
        assert (got == data[:, present[:k] == 0]).all(), (k, m, sorted(lost), ran)
        assert any(x.startswith(("rs_fft_pdecode", "rs_net_reconstruct", "rs_fft_inverse")) for x in ran), ran


def test_fdec_vs_oracle_reconstruct(oracle, fdec):
    k, m, sb, n = 100, 20, 2048, 2
    rng = np.random.default_rng(100020)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data)
    present = np.ones(k + m, np.uint8)
    present[[0, 5, 63, 64, 99]] = 0
    present[[k + 1, k + 19]] = 0
    got = reconstruct(k, m, present, data, par)
    ref = oracle.reconstruct_batch(k, m, present, np.concatenate([data, par], axis=1))
    assert (got == ref).all()


def test_fdec_edge_blocks(oracle, fdec):
    """Erasures only in the last (partial) data block, only in the first, in one block."""
    k, m, sb, n = 200, 55, 2048, 2
    data = splitmix_bytes(0xFDEC, n * k * sb).reshape(n, k, sb)
    par = oracle.encode_batch(k, m, data, threads=4)
    for lost in ([192, 193, 199], [0], [63, 64], list(range(128, 183)), [199]):
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        got = reconstruct(k, m, present, data, par)
        assert (got == data[:, lost]).all(), lost


def test_fdec_c4_full_size():
    """configs[4] shape: RS(200,55) 256 KiB shards, 55 erased (every third from 1), the
    default selection (auto): the fused kernel runs while no network is loaded."""
    k, m, sb, n = 200, 55, 256 << 10, 2
    data = splitmix_bytes(0x200C4, n * k * sb).reshape(n, k, sb)
    d = torch.from_numpy(data).to(DEV)
    p = torch.zeros((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p)
    present = np.ones(k + m, np.uint8)
    lost = list(range(1, 165, 3))
    present[lost] = 0
    out = torch.zeros((n, 55, sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, d, p, out)
    torch.cuda.synchronize()
    assert torch.equal(out, d[:, lost])


@pytest.mark.parametrize("k,m,sb,n,max_e", [(200, 55, 4096, 9, 55), (200, 55, 8192, 7, 8), (64, 64, 4096, 6, 40),
                                            (40, 12, 8192, 6, 12), (16, 16, 4096, 9, 16), (100, 20, 2048, 11, 20)])
def test_fdec_per_stripe_patterns(oracle, monkeypatch, k, m, sb, n, max_e):
    """rs_reconstruct_batch_dev_patterns on wide codes: per-stripe decode blocks built on
    the GPU (trimmed rows R, erasure locator by FWHT, masks), then the fused kernel. Stripes
    lose 0..max_e + 3 originals and random recovery shards; more than max_e restore the
    first max_e (status 14); too few present report 2 and write nothing."""
    monkeypatch.setenv("RS_AMD_FDEC", "1")
    assert R.patterns_kernel_name(k, m, sb, max_e) == "fft_decode"
    rng = np.random.default_rng(k * 13 + m + max_e)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=8)
    present = np.ones((n, k + m), np.uint8)
    for s in range(n - 1):
        e = int(rng.integers(0, min(max_e + 3, m, k) + 1))
        present[s, rng.choice(k, size=e, replace=False)] = 0
        present[s, k + rng.choice(m, size=int(rng.integers(0, m - e + 1)), replace=False)] = 0
    present[n - 1, :] = 1
    present[n - 1, : m + 1] = 0
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    out = torch.full((n, max_e, sb), 0xAB, dtype=torch.uint8, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    R.reconstruct_batch_dev_patterns(k, m, dev(present), dev(data), dev(par), out, status)
    torch.cuda.synchronize()
    out, status = out.cpu().numpy(), status.cpu().numpy()
    assert status[n - 1] == 2 and (out[n - 1] == 0xAB).all()
    for s in range(n - 1):
        missing = [i for i in range(k) if not present[s, i]]
        assert status[s] == (14 if len(missing) > max_e else 0), s
        got = missing[:max_e]
        assert (out[s, :len(got)] == data[s, got]).all(), (s, missing)
        assert (out[s, len(got):] == 0xAB).all(), s


def _random_code(rng):
    c = int(rng.choice([16, 32, 64]))
    m = int(rng.integers(c // 2 + 1, c + 1))
    while True:
        k = int(rng.integers(1, min(16 * c, 300) + 1))
        pk = 1 << (k - 1).bit_length()
        if pk > c or (pk == c and k <= m):
            return k, m


@pytest.mark.parametrize("seed", range(12))
def test_fdec_fuzz(oracle, monkeypatch, seed):
    """Seeded fuzz of the forced fused FFT reconstruct: random high-rate codes of chunk
    16 / 32 / 64, shards of 1-6 whole 2 KiB units, 1-4 stripes, one batch pattern and one
    pattern per stripe (random data and recovery losses), against the data (MDS)."""
    monkeypatch.setenv("RS_AMD_FDEC", "1")
    rng = np.random.default_rng(0xFDEC + seed)
    k, m = _random_code(rng)
    sb, n = 2048 * int(rng.integers(1, 7)), int(rng.integers(1, 5))
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=4)
    e = int(rng.integers(1, min(k, m) + 1))
    present = np.ones(k + m, np.uint8)
    present[rng.choice(k, size=e, replace=False)] = 0
    present[k + rng.choice(m, size=int(rng.integers(0, m - e + 1)), replace=False)] = 0
    got = reconstruct(k, m, present, data, par)
    assert (got == data[:, present[:k] == 0]).all(), (k, m, sb, n, e)
    pres = np.ones((n, k + m), np.uint8)
    for s in range(n):
        es = int(rng.integers(0, min(k, m) + 1))
        pres[s, rng.choice(k, size=es, replace=False)] = 0
        pres[s, k + rng.choice(m, size=int(rng.integers(0, m - es + 1)), replace=False)] = 0
    max_e = int((pres[:, :k] == 0).sum(1).max()) or 1
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    out = torch.full((n, max_e, sb), 0xAB, dtype=torch.uint8, device=DEV)
    status = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    R.reconstruct_batch_dev_patterns(k, m, dev(pres), dev(data), dev(par), out, status)
    torch.cuda.synchronize()
    out, status = out.cpu().numpy(), status.cpu().numpy()
    for s in range(n):
        missing = [i for i in range(k) if not pres[s, i]]
        assert status[s] == 0, (s, k, m)
        assert (out[s, :len(missing)] == data[s, missing]).all(), (seed, s, k, m, sb, missing)


def test_fdec_pattern_across_shard_sizes(oracle):
    """One pattern used with 2 KiB-unit shards (fused kernel) and then with 1 KiB shards
    (no fused form: two stripes per unit) in the same process: each call takes a form that
    fits its shard size (the plan cache keys on it)."""
    k, m = 100, 20
    lost = list(range(0, 100, 6))[:15]
    present = np.ones(k + m, np.uint8)
    present[lost] = 0
    rng = np.random.default_rng(1024)
    for sb in (2048, 1024, 6144):
        data = rng.integers(0, 256, (3, k, sb), dtype=np.uint8)
        par = oracle.encode_batch(k, m, data, threads=4)
        for _ in range(2):
            assert (reconstruct(k, m, present, data, par) == data[:, lost]).all(), sb
