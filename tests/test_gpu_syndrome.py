"""GPU parity of the reconstruct-by-syndromes path (wide codes): the restored
originals x solve A x = p_R ^ Enc_R(d') where d' is the received data with the
erased shards read as zeros (encode kernels with a skip mask) and A is the e x e
block of the encode map on (first e received recovery rows, erased columns); the
e x e inverse runs on the table-driven matrix kernels with XOR-fused inputs.
Bit-exact against the erased data (restored originals are unique)."""
import numpy as np
import pytest

from helpers import splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _syndrome_forms(monkeypatch):
    """These tests cover the syndrome path's own forms (FFT syndromes + e x e map / solve /
    table kernels); the fused FFT reconstruct has tests/test_gpu_fdec.py."""
    monkeypatch.setenv("RS_AMD_FDEC", "0")


def reconstruct(k, m, present, data, par, flags=0):
    n, _, sb = data.shape
    e = int(k - np.sum(present[:k]))
    out = torch.zeros((n, max(e, 1), sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, torch.from_numpy(data).to(DEV), torch.from_numpy(par).to(DEV), out,
                            flags)
    torch.cuda.synchronize()
    return out.cpu().numpy()[:, :e]


# encode kernels the syndrome path runs on: register (chunk <= 16) and wave-split (chunk 64)
SYN_KM = [(4, 2), (10, 4), (8, 4), (16, 16), (30, 2), (20, 16), (70, 33), (64, 64), (100, 60), (200, 55)]


@pytest.mark.parametrize("k,m", SYN_KM)
@pytest.mark.parametrize("flags", [0, 2])  # D2 changes the encode only; the decode is the same
def test_syndrome_reconstruct_vs_oracle(oracle, monkeypatch, k, m, flags):
    monkeypatch.setenv("RS_AMD_DECODE", "syndrome")
    monkeypatch.setenv("RS_AMD_JIT", "0")
    rng = np.random.default_rng(k * 1009 + m)
    sb, n = 1024, 2
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data)
    for trial in range(3):
        e = int(rng.integers(1, min(k, m) + 1))
        lost = list(rng.choice(k, size=e, replace=False))
        extra = int(rng.integers(0, m - e + 1))
        lost += [k + int(i) for i in rng.choice(m, size=extra, replace=False)]
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        missing = [i for i in range(k) if not present[i]]
        name = R.reconstruct_kernel_name(k, m, sb, present)
        assert name.startswith("syndrome"), name
        got = reconstruct(k, m, present, data, par, flags)
        assert (got == data[:, missing]).all(), (k, m, sorted(lost), name)


def test_syndrome_matches_matrix_kernel(oracle, monkeypatch):
    """Same bytes as the direct k x e matrix kernel (strided output, many stripes)."""
    k, m, sb, n = 70, 40, 4096, 5
    rng = np.random.default_rng(7040)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=4)
    present = np.ones(k + m, np.uint8)
    present[rng.choice(k, size=20, replace=False)] = 0
    present[k + 3] = 0
    outs = {}
    for mode in ("syndrome", "matrix"):
        monkeypatch.setenv("RS_AMD_DECODE", mode)
        outs[mode] = reconstruct(k, m, present, data, par)
    assert (outs["syndrome"] == outs["matrix"]).all()
    assert (outs["syndrome"] == data[:, present[:k] == 0]).all()


def test_syndrome_rs200_55_full_size_all_erasures():
    """configs[4] shape, 55 erased data shards: auto mode picks the syndrome path."""
    k, m, sb, n = 200, 55, 256 << 10, 2
    data = splitmix_bytes(0x200, n * k * sb).reshape(n, k, sb)
    par = torch.zeros((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, torch.from_numpy(data).to(DEV), par)
    torch.cuda.synchronize()
    present = np.ones(k + m, np.uint8)
    erase = list(range(1, 200, 3))[:55]
    present[erase] = 0
    assert R.reconstruct_kernel_name(k, m, sb, present).startswith("syndrome")
    got = reconstruct(k, m, present, data, par.cpu().numpy())
    assert (got == data[:, erase]).all()


def test_syndrome_network_background_compile(oracle, monkeypatch):
    """RS(200,55) losing 55 data shards: the 55 x 55 syndrome map (770 network blocks)
    compiles in the background; the calls before it is ready run the table kernel,
    the calls after it the network — both restore the erased shards bit-exactly."""
    monkeypatch.delenv("RS_AMD_JIT", raising=False)
    monkeypatch.delenv("RS_AMD_JIT_SYNC", raising=False)
    monkeypatch.setenv("RS_AMD_FDEC", "0")  # the syndrome path (round 2's steady state)
    k, m, sb, n = 200, 55, 8192, 2
    rng = np.random.default_rng(2055)
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data)
    lost = sorted(int(i) for i in rng.choice(k, size=55, replace=False))
    present = np.ones(k + m, np.uint8)
    present[lost] = 0
    assert R.reconstruct_kernel_name(k, m, sb, present) == "syndrome+net_fft_encode_i200_o55+net_syndrome_i55_o55"
    for _ in range(2):  # 2nd use queues the compile (RS_AMD_NET_ASYNC_AFTER)
        assert (reconstruct(k, m, present, data, par) == data[:, lost]).all()
    R.net_wait()
    assert (reconstruct(k, m, present, data, par) == data[:, lost]).all()



@pytest.mark.parametrize("k,m", [(200, 55), (70, 33), (64, 64), (100, 20), (300, 40)])
def test_syndrome_fft_encode_vs_oracle(oracle, monkeypatch, k, m):
    """The syndromes' encode on the bit-sliced FFT kernel (erased shards skipped, only
    the rows R stored), compiled synchronously, then the e x e map."""
    monkeypatch.setenv("RS_AMD_DECODE", "syndrome")
    monkeypatch.setenv("RS_AMD_JIT_SYNC", "1")
    rng = np.random.default_rng(k * 31 + m)
    sb, n = 4096, 3
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=8)
    for trial in range(2):
        e = int(rng.integers(1, min(k, m) + 1))
        lost = list(rng.choice(k, size=e, replace=False))
        extra = int(rng.integers(0, m - e + 1))
        lost += [k + int(i) for i in rng.choice(m, size=extra, replace=False)]
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        missing = [i for i in range(k) if not present[i]]
        name = R.reconstruct_kernel_name(k, m, sb, present)
        assert "fft_encode" in name, name
        assert (reconstruct(k, m, present, data, par) == data[:, missing]).all(), (k, m, sorted(lost), name)


@pytest.mark.parametrize("k,m,e", [(200, 55, 55), (200, 55, 20), (100, 20, 12), (64, 64, 40), (40, 50, 33)])
@pytest.mark.parametrize("net", ["async", "off"])
def test_syndrome_cold_pattern_form(oracle, monkeypatch, k, m, e, net):
    """A pattern whose own kernels are not loaded runs the pattern-agnostic form (the
    code's FFT kernel with the batch's erasure mask + the generic e x e solve) instead of
    the table kernels: first calls of fresh patterns, with the background network compile
    pending (async) or disabled (off: the solve serves every call). Recovery shards are
    lost too, so R is not a prefix of the rows."""
    monkeypatch.delenv("RS_AMD_JIT_SYNC", raising=False)
    monkeypatch.setenv("RS_AMD_DECODE", "syndrome")
    if net == "off":
        monkeypatch.setenv("RS_AMD_NET_ASYNC_BLOCKS", "0")
    rng = np.random.default_rng(k * 3 + m + e + (net == "off"))
    sb, n = 8192, 3
    data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
    par = oracle.encode_batch(k, m, data, threads=8)
    for trial in range(2):
        lost = list(rng.choice(k, size=e, replace=False))
        lost += [k + int(i) for i in rng.choice(m, size=min(m - e, 3), replace=False)]
        present = np.ones(k + m, np.uint8)
        present[lost] = 0
        missing = [i for i in range(k) if not present[i]]
        for call in range(2):
            got = reconstruct(k, m, present, data, par)
            assert (got == data[:, missing]).all(), (k, m, e, trial, call)
