"""Allocation-failure injection: the reference's "encode leaks" test (tests.zig:131-156)
runs an RS(5,5) encode under std.testing.checkAllAllocationFailures, which fails every
allocation of the call in turn and requires error.OutOfMemory with nothing leaked. Here
rs_debug_fail_alloc(n) fails the n-th allocation the library makes (plan objects, device,
stream-ordered and pinned buffers); the test walks n over every allocation of a cold RS(5,5)
Encoder + Decoder cycle (tests.zig:8-59 encodeDecodeCycle, input byte i % 256) and checks:
the cycle either raises OutOfMemory or returns the right bytes, nothing crashes, and after
the caches are dropped the device's free memory and the pooled one-shot contexts are back
where they started."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402


def cycle(k, m, sb, lost):
    """Encoder.encode, then Decoder.decode with the originals in `lost` missing."""
    data = [bytes((i * sb + j) % 256 for j in range(sb)) for i in range(k)]  # tests.zig:66-67
    enc = R.Encoder(k, m, sb)
    try:
        for d in data:
            enc.add_original_shard(d)
        rec = enc.encode()
    finally:
        enc.deinit()
    dec = R.Decoder(k, m, sb)
    try:
        for i in range(k):
            if i not in lost:
                dec.add_original_shard(i, data[i])
        for i in range(m):
            dec.add_recovery_shard(i, rec[i])
        out = dec.decode()
    finally:
        dec.deinit()
    assert out == data


def free_bytes():
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info()[0]


@pytest.mark.parametrize("k,m,sb,lost", [(5, 5, 64, (0, 1)), (10, 4, 4096, (0, 1, 2, 3)), (200, 55, 2048, (1, 4, 7))])
def test_every_allocation_fails_cleanly(k, m, sb, lost):
    cycle(k, m, sb, lost)  # kernels compiled and loaded (they stay across the cache drops)
    R.net_wait()
    R.debug_release_caches()
    R.debug_fail_alloc(-1)
    cycle(k, m, sb, lost)  # a cold cycle: count its allocations
    n = R.debug_fail_alloc(-1)
    assert n >= 4, n
    assert R.debug_release_caches() == 0

    def walk(check):
        free0, ooms = free_bytes(), 0
        for i in range(n):
            R.debug_fail_alloc(i)
            try:
                cycle(k, m, sb, lost)
            except R.OutOfMemory:  # noqa: F821 (generated from the Zig error set)
                ooms += 1
            finally:
                R.debug_fail_alloc(-1)
            R.net_wait()
            assert R.debug_release_caches() == 0, i
            if check:
                assert free_bytes() == free0, (i, free0 - free_bytes())
        return ooms

    # the first walk may take one-time runtime allocations (a fallback kernel's first
    # launch, its scratch); the second must leave the device exactly as it found it
    walk(False)
    assert walk(True) >= 1
    cycle(k, m, sb, lost)  # and the library still works
