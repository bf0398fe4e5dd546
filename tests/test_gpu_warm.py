"""Which kernel a reconstruct actually launches (rs_last_kernels) and the warm-up recipes of
include/reedsol.h / INTEGRATION.md: a wide-code pattern's first calls run the fused FFT
reconstruct with the pattern as data (rs_fft_decode_*); its RS_AMD_PDEC_AFTER-th call (default
2) queues the same kernel with the pattern compiled in (rs_fft_pdecode_*), and two calls +
rs_net_wait, or one rs_reconstruct_warm, bring the pattern to it: the next call launches it.
Per-pattern compiles are bounded (RS_AMD_PDEC_MAX per code) and a pattern whose steady state
is a direct network compiles only that network. RS_AMD_FDEC=0 keeps
the round-2 form (syndromes + the pattern's e x e network), RS_AMD_FDEC=1 the pattern as
data. Restored shards are checked against the data every time (MDS: restored originals are
unique). Reference: root.zig:268-335 (Decoder.decode)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402

DEV = torch.device("cuda:0")
K, M, SB, N = 200, 55, 4096, 4


@pytest.fixture(scope="module")
def c4_batch(oracle):
    rng = np.random.default_rng(0xC4C4)
    data = rng.integers(0, 256, (N, K, SB), dtype=np.uint8)
    par = oracle.encode_batch(K, M, data, threads=4)
    return torch.from_numpy(data).to(DEV), torch.from_numpy(par).to(DEV)


def pattern(seed, e=M):
    lost = sorted(int(i) for i in np.random.default_rng(seed).choice(K, size=e, replace=False))
    present = [0 if i in lost else 1 for i in range(K)] + [1] * M
    return lost, present


def run(present, lost, batch):
    d, p = batch
    out = torch.zeros((N, len(lost), SB), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(K, M, present, d, p, out)
    ran = R.last_kernels()
    torch.cuda.synchronize()
    assert torch.equal(out, d[:, lost])
    return ran


def has(ran, prefix):
    return any(k.startswith(prefix) for k in ran)


def test_last_kernels_headline_shapes():
    """RS(10,4) encode and reconstruct report the networks rocprofv3 shows (bench labels)."""
    k, m, sb, n = 10, 4, 4096, 8
    d = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=DEV)
    p = torch.empty((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p)
    assert R.last_kernels() and R.last_kernels()[0].startswith("rs_net_encode_i10_o4")
    present = [0, 0, 0, 0] + [1] * (k + m - 4)
    out = torch.empty((n, 4, sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, d, p, out)
    assert R.last_kernels()[0].startswith("rs_net_reconstruct_i10_o4")
    torch.cuda.synchronize()
    assert torch.equal(out, d[:, :4])


def test_first_call_runs_fused(c4_batch, monkeypatch):
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    lost, present = pattern(401)
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_fft_decode_k200_m55"), ran


def test_warm_reaches_pattern_kernel(c4_batch, monkeypatch):
    """rs_reconstruct_warm: the next call launches the pattern-compiled fused kernel."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    lost, present = pattern(402)
    R.reconstruct_warm(K, M, SB, present)
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_fft_pdecode_k200_m55"), ran
    assert not has(ran, "rs_fft_decode"), ran


def test_reuse_threshold_then_pattern_kernel(c4_batch, monkeypatch):
    """The INTEGRATION.md recipe without the warm call, call for call: a pattern used once is not
    compiled in (RS_AMD_PDEC_AFTER, default 2: a one-off pattern costs no hipRTC); its second
    call (still the pattern as data) queues the compile, rs_net_wait, then the third call runs
    the pattern-compiled kernel."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    monkeypatch.delenv("RS_AMD_PDEC_AFTER", raising=False)
    lost, present = pattern(403)
    assert has(run(present, lost, c4_batch), "rs_fft_decode")
    R.net_wait()
    ran = run(present, lost, c4_batch)  # second use: still the pattern as data, queues the compile
    assert has(ran, "rs_fft_decode_k200_m55") and not has(ran, "rs_fft_pdecode"), ran
    R.net_wait()
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_fft_pdecode_k200_m55"), ran


def test_pdec_after_three(c4_batch, monkeypatch):
    """RS_AMD_PDEC_AFTER=3 (round 5's default): two calls compile nothing, the third queues."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    monkeypatch.setenv("RS_AMD_PDEC_AFTER", "3")
    lost, present = pattern(413)
    run(present, lost, c4_batch)
    run(present, lost, c4_batch)
    R.net_wait()
    assert not has(run(present, lost, c4_batch), "rs_fft_pdecode")  # third call queues
    R.net_wait()
    assert has(run(present, lost, c4_batch), "rs_fft_pdecode_k200_m55")


def test_pdec_budget_per_code(monkeypatch):
    """RS_AMD_PDEC_MAX bounds the pattern-compiled kernels per code: past it a warmed pattern
    keeps the fused kernel with the pattern as data (correct bytes, no hipRTC). RS(100,32) 4 KiB
    losing 30 (chunk 32; too many losses for a direct network): its own budget, untouched by the
    RS(200,55) tests."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    monkeypatch.setenv("RS_AMD_PDEC_MAX", "1")
    k, m, sb, n = 100, 32, 4096, 3
    rng = np.random.default_rng(77)
    d = torch.from_numpy(rng.integers(0, 256, (n, k, sb), dtype=np.uint8)).to(DEV)
    p = torch.empty((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p)
    ran_by = []
    for seed in (1, 2):
        lost = sorted(int(i) for i in np.random.default_rng(seed).choice(k, size=30, replace=False))
        present = [0 if i in lost else 1 for i in range(k)] + [1] * m
        R.reconstruct_warm(k, m, sb, present)
        out = torch.zeros((n, len(lost), sb), dtype=torch.uint8, device=DEV)
        R.reconstruct_batch_dev(k, m, present, d, p, out)
        ran_by.append(R.last_kernels())
        torch.cuda.synchronize()
        assert torch.equal(out, d[:, lost])
    assert has(ran_by[0], "rs_fft_pdecode_k100_m32"), ran_by
    assert has(ran_by[1], "rs_fft_decode_k100_m32") and not has(ran_by[1], "rs_fft_pdecode"), ran_by


def test_few_losses_compile_only_the_network(monkeypatch):
    """a few-loss wide-code pattern whose steady state is its direct network
    compiles that network only (no pattern-compiled fused kernel nobody launches). RS(100,20)
    losing 4: the 100 -> 4 map (100 blocks, background); the warm-up adds exactly one module."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    k, m, sb, n = 100, 20, 4096, 3
    rng = np.random.default_rng(78)
    d = torch.from_numpy(rng.integers(0, 256, (n, k, sb), dtype=np.uint8)).to(DEV)
    p = torch.empty((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p)
    other = [0 if i in (5, 6, 7, 8) else 1 for i in range(k)] + [1] * m
    out = torch.zeros((n, 4, sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, other, d, p, out)  # loads the code's fused kernel
    assert has(R.last_kernels(), "rs_fft_decode_k100_m20")
    R.net_wait()
    lost = [1, 30, 61, 99]
    present = [0 if i in lost else 1 for i in range(k)] + [1] * m
    before = R.jit_stats()["modules"]
    R.reconstruct_warm(k, m, sb, present)
    assert R.jit_stats()["modules"] - before == 1
    R.reconstruct_batch_dev(k, m, present, d, p, out)
    ran = R.last_kernels()
    torch.cuda.synchronize()
    assert has(ran, "rs_net_reconstruct_i100_o4"), ran
    assert torch.equal(out, d[:, lost])


def test_pdecode_c4_shape():
    """The pattern-compiled kernel at the c4 shape (RS(200,55), 256 KiB shards, 2 stripes: 128
    units each), after rs_reconstruct_warm, against the data."""
    k, m, sb, n = 200, 55, 256 << 10, 2
    g = torch.Generator(device=DEV)
    g.manual_seed(0xC45)
    d = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=DEV, generator=g)
    p = torch.empty((n, m, sb), dtype=torch.uint8, device=DEV)
    R.encode_batch_dev(k, m, d, p)
    lost = list(range(1, k, 3))[:m]
    present = [0 if i in lost else 1 for i in range(k)] + [1] * m
    R.reconstruct_warm(k, m, sb, present)
    out = torch.zeros((n, m, sb), dtype=torch.uint8, device=DEV)
    R.reconstruct_batch_dev(k, m, present, d, p, out)
    ran = R.last_kernels()
    torch.cuda.synchronize()
    assert has(ran, "rs_fft_pdecode_k200_m55"), ran
    assert torch.equal(out, d[:, lost])


def test_module_cap_falls_back_to_pattern_as_data(c4_batch, monkeypatch):
    """RS_AMD_JIT_CACHE_MAX reached: a warmed wide pattern's pattern-compiled kernel is refused
    and the call runs the code's loaded fused kernel with the pattern as data, bytes right."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    lost0, present0 = pattern(420)
    assert has(run(present0, lost0, c4_batch), "rs_fft_decode_k200_m55")  # the code's fused kernel loaded
    R.net_wait()
    monkeypatch.setenv("RS_AMD_JIT_CACHE_MAX", str(R.jit_stats()["modules"]))
    lost, present = pattern(421)
    R.reconstruct_warm(K, M, SB, present)
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_fft_decode_k200_m55") and not has(ran, "rs_fft_pdecode"), ran


def test_warm_network_form(c4_batch, monkeypatch):
    """RS_AMD_FDEC=0: the round-2 steady state, syndromes + the pattern's 55 x 55 network."""
    monkeypatch.setenv("RS_AMD_FDEC", "0")
    lost, present = pattern(406)
    R.reconstruct_warm(K, M, SB, present)
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_net_syndrome_i55_o55"), ran


def test_forced_fused_after_warm(c4_batch, monkeypatch):
    monkeypatch.setenv("RS_AMD_FDEC", "1")
    lost, present = pattern(404)
    R.reconstruct_warm(K, M, SB, present)
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_fft_decode_k200_m55") and not has(ran, "rs_net_syndrome"), ran


@pytest.mark.parametrize("e", [1, 8, 20, 40])
def test_pattern_kernel_loss_counts(c4_batch, monkeypatch, e):
    """Any loss count: after the warm-up the pattern-compiled kernel (or, for few losses, the
    pattern's direct network) restores the data."""
    monkeypatch.delenv("RS_AMD_FDEC", raising=False)
    lost, present = pattern(405 + e, e=e)
    R.reconstruct_warm(K, M, SB, present)
    ran = run(present, lost, c4_batch)
    assert has(ran, "rs_fft_pdecode_k200_m55") or has(ran, "rs_net_reconstruct_i200"), ran
