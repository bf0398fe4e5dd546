"""GPU parity of the bit-sliced FFT encode kernels (rs_fftnet.hpp):
wide codes (chunk 32 / 64) against the CPU oracle, bit-exact, in both quirk modes,
with strided stripes, and at the BASELINE c4 size (RS(200,55) 256 KiB) in full."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402

DEV = torch.device("cuda:0")

SHAPES = [(200, 55), (100, 20), (64, 64), (32, 32), (40, 50), (300, 40), (128, 33), (33, 17), (256, 64),
          (1000, 64), (65, 64)]



def enc(k, m, data, flags=0):
    d = torch.from_numpy(data).to(DEV)
    p = torch.zeros((data.shape[0], m, data.shape[2]), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p, flags)
    torch.cuda.synchronize()
    return p.cpu().numpy()


@pytest.mark.parametrize("k,m", SHAPES)
@pytest.mark.parametrize("flags", [0, 3])
def test_fft_encode_vs_oracle(oracle, k, m, flags):
    sb, n = 4096, 3
    rng = np.random.default_rng(k * 1000 + m + flags)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    assert "fft_encode" in R.encode_kernel_name(k, m, sb)
    got = enc(k, m, data, flags)
    exp = oracle.encode_batch(k, m, data, quirks=flags, threads=8)
    assert np.array_equal(got, exp)


def test_fft_encode_strided(oracle):
    k, m, sb, n = 200, 55, 2048, 5
    rng = np.random.default_rng(5)
    big = rng.integers(0, 256, (n, k + 3, sb), dtype=np.uint8)
    d = torch.from_numpy(big).to(DEV)
    p = torch.full((n, m + 2, sb), 7, dtype=torch.uint8, device=DEV)
    # stripe strides (k+3)*sb and (m+2)*sb through the C ABI
    st = R.lib().rs_encode_batch_dev(k, m, sb, n, d.data_ptr(), d.stride(0), p.data_ptr(), p.stride(0), 0, None)
    assert st == 0, R.lib().rs_last_error()
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    exp = oracle.encode_batch(k, m, np.ascontiguousarray(big[:, :k]), threads=8)
    assert np.array_equal(got[:, :m], exp)
    assert (got[:, m:] == 7).all()  # rows past the parity untouched


def test_fft_encode_c4_full(oracle):
    """BASELINE configs[4] shape, RS(200,55) 256 KiB shards: full parity of 4 stripes."""
    k, m, sb, n = 200, 55, 256 << 10, 4
    rng = np.random.default_rng(44)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    got = enc(k, m, data)
    exp = oracle.encode_batch(k, m, data, threads=16)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("k,m", [(32, 32), (64, 64), (200, 55), (33, 17), (100, 20)])
@pytest.mark.parametrize("n", [1, 2, 7])
def test_fft_encode_1k_shards(oracle, k, m, n):
    """1 KiB shards (the reference harness size, benchmarks.zig:11): a unit spans two
    stripes; an odd batch's last unit has no second stripe (zero-record resource:
    nothing read or written past the batch — a guard stripe stays untouched)."""
    sb = 1024
    rng = np.random.default_rng(k * 31 + m + n)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    assert "fft_encode" in R.encode_kernel_name(k, m, sb)
    d = torch.from_numpy(data).to(DEV)
    p = torch.full((n + 1, m, sb), 7, dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p[:n])
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    assert np.array_equal(got[:n], oracle.encode_batch(k, m, data, threads=8))
    assert (got[n] == 7).all()


def test_fft_syndrome_1k_shards(oracle, monkeypatch):
    """RS(200,55) losing 40 data shards at 1 KiB: syndromes on the two-stripe FFT variant."""
    monkeypatch.setenv("RS_AMD_JIT_SYNC", "1")
    k, m, sb, n = 200, 55, 1024, 5
    rng = np.random.default_rng(2055)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=8)
    present = np.ones(k + m, np.uint8)
    lost = list(range(3, 200, 5))[:40]
    present[lost] = 0
    assert "syndrome+net_fft_encode" in R.reconstruct_kernel_name(k, m, sb, present)
    d = torch.from_numpy(data).to(DEV)
    d[:, lost] = 0
    pr = torch.from_numpy(par).to(DEV)
    out = torch.zeros((n, len(lost), sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, d, pr, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), data[:, lost])


@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("sb,n", [(1024, 7), (4096, 3), (1 << 20, 2)])
def test_fft_inverse_reconstruct_all_originals(oracle, k, sb, n):
    """RS(k,k), every original lost: the data restored from the k recovery shards by the
    inverted encode (IFFT at skew 0, FFT at skew k) equal the originals; odd batches at
    1 KiB leave a guard stripe untouched."""
    rng = np.random.default_rng(k + sb + n)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, k, data, threads=8)
    present = np.ones(2 * k, np.uint8)
    present[:k] = 0
    assert R.reconstruct_kernel_name(k, k, sb, present) == f"net_fft_inverse_i{k}_o{k}"
    d = torch.zeros((n, k, sb), dtype=torch.uint8, device=DEV)
    pr = torch.from_numpy(par).to(DEV)
    out = torch.full((n + 1, k, sb), 7, dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, k, present, d, pr, out[:n])
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got[:n], data)
    assert (got[n] == 7).all()


@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("flags", [1, 3])
def test_fft_inverse_not_taken_under_d1(oracle, k, flags):
    """Under D1 the literal reconstruct (root.zig:268-335 with Generic.zig:283's multiply)
    is not the inverse of the encode, so every-original-lost must follow the reference's
    decode as written, not the inverted encode: compare with the oracle's reconstruct."""
    sb, n = 4096, 2
    rng = np.random.default_rng(k + flags)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, k, data, quirks=flags, threads=8)
    present = np.ones(2 * k, np.uint8)
    present[:k] = 0
    d = torch.zeros((n, k, sb), dtype=torch.uint8, device=DEV)
    pr = torch.from_numpy(par).to(DEV)
    out = torch.zeros((n, k, sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, k, present, d, pr, out, flags)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for s in range(n):
        exp = oracle.reconstruct_batch(k, k, present, np.concatenate([data[s:s + 1], par[s:s + 1]], axis=1),
                                       quirks=flags)
        assert np.array_equal(got[s], exp[0]), s
