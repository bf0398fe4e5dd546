"""Shared-input network form (rs_jit.cpp generate_shared, RS_AMD_NET_SHARED=1): one
workgroup of n_tiles waves per 4 KiB unit, every input transformed once and shared
through LDS. Bit-exact against the oracle / the erased data on multi-tile maps: encode,
direct reconstruct and the syndrome map of a wide code."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.fixture
def shared(monkeypatch):
    monkeypatch.setenv("RS_AMD_NET_SHARED", "1")
    monkeypatch.setenv("RS_AMD_JIT_SYNC", "1")
    monkeypatch.setenv("RS_AMD_FFT", "0")  # keep the wide encodes off the FFT kernel: maps only


@pytest.mark.parametrize("k,m,sb,n", [(16, 16, 8192, 3), (12, 10, 4096, 5), (6, 20, 4096, 2)])
def test_shared_encode_vs_oracle(oracle, shared, k, m, sb, n):
    rng = np.random.default_rng(k * 13 + m)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    d = torch.from_numpy(data).to(DEV)
    p = torch.zeros((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p)
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    if R.use_high_rate(k, m):
        exp = oracle.encode_batch(k, m, data)
    else:
        exp = np.stack([oracle.encode_low(k, m, data[s])[1] for s in range(n)])
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("k,m,lost", [(16, 16, list(range(0, 16, 1))[:12]), (200, 55, list(range(1, 200, 9))[:20]),
                                      (100, 20, list(range(0, 100, 7))[:13])])
def test_shared_reconstruct(oracle, shared, k, m, lost):
    sb, n = 8192, 3
    rng = np.random.default_rng(k + len(lost))
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=8)
    present = np.ones(k + m, np.uint8)
    present[lost] = 0
    d = torch.from_numpy(data).to(DEV)
    d[:, lost] = 0
    out = torch.zeros((n, len(lost), sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, d, torch.from_numpy(par).to(DEV), out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), data[:, lost]), R.reconstruct_kernel_name(k, m, sb, present)


@pytest.mark.parametrize("k,m", [(40, 12), (200, 10)])
def test_encode_background_shared_network(oracle, monkeypatch, k, m):
    """Encode maps past the synchronous cap (m > 8, no FFT form): table kernels until the
    background compile of the shared-input network lands, the network after; all equal
    the oracle."""
    monkeypatch.delenv("RS_AMD_JIT_SYNC", raising=False)
    sb, n = 8192, 2
    assert R.encode_kernel_name(k, m, sb) == f"net_encode_i{k}_o{m}"
    rng = np.random.default_rng(k * 3 + m)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    exp = oracle.encode_batch(k, m, data)
    d = torch.from_numpy(data).to(DEV)

    def enc():
        p = torch.zeros((n, m, sb), dtype=torch.uint8, device=DEV)
        R.encode_batch_dev(k, m, d, p)
        torch.cuda.synchronize()
        return p.cpu().numpy()

    for _ in range(3):
        assert np.array_equal(enc(), exp)
    R.net_wait()
    assert np.array_equal(enc(), exp)


@pytest.mark.parametrize("balance", ["1", "0"])
@pytest.mark.parametrize("k,m,lost", [(64, 64, sorted(list(range(0, 64, 3))[:20] + list(range(1, 64, 3))[:20])),
                                      (40, 24, sorted(list(range(0, 32, 2)) + [1, 3, 5]))])
def test_shared_reconstruct_balanced_waves(oracle, shared, monkeypatch, balance, k, m, lost):
    """Maps of 3 and 5..7 output tiles: with RS_AMD_NET_BALANCE the workgroup runs 4 / 8
    waves over evenly split outputs (40 outputs: 8 x 5; 19: 3 x 5 + 4), else 3 / 5 waves
    of 8; both restore the erased data (rows in ascending shard order)."""
    monkeypatch.setenv("RS_AMD_NET_BALANCE", balance)
    sb, n = 8192, 2
    rng = np.random.default_rng(k + len(lost) + int(balance))
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=8)
    present = np.ones(k + m, np.uint8)
    present[lost] = 0
    d = torch.from_numpy(data).to(DEV)
    d[:, lost] = 0
    out = torch.zeros((n, len(lost), sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, d, torch.from_numpy(par).to(DEV), out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), data[:, lost]), R.reconstruct_kernel_name(k, m, sb, present)
