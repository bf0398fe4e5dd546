"""GPU: the C ABI called from several host threads at once (SURVEY.md §8b:
"calls are thread-safe across devices and stateless apart from a per-(k,m)
plan cache"). ctypes releases the GIL, so the threads really overlap inside
the library: first-use plan builds and network compiles race on the plan
cache, device batches run on per-thread streams, and host-batch calls share
the per-device staging ring. Every result is compared bit-exactly with the
oracle (encode) or with the data that was erased (reconstruct)."""
import threading

import numpy as np
import pytest

from helpers import splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rs_amd import reedsol_amd as R  # noqa: E402

DEV = torch.device("cuda:0")

# (k, m, shard_bytes): repeated shapes race on one plan, distinct ones build side by side
SHAPES = [(10, 4, 65536), (10, 4, 65536), (6, 3, 8192), (12, 5, 16384), (20, 7, 4096), (4, 2, 65536),
          (40, 8, 4096), (6, 3, 8192)]


def _run_threads(fn, n):
    errors = []

    def wrap(i):
        try:
            fn(i)
        except BaseException as e:  # noqa: BLE001  (re-raised on the main thread)
            errors.append((i, e))

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a worker thread did not finish"
    if errors:
        raise errors[0][1]


def test_device_batches_from_threads(oracle):
    n_stripes = 3
    results = {}

    def work(i):
        k, m, sb = SHAPES[i]
        data = splitmix_bytes(0x7000 + i, n_stripes * k * sb).reshape(n_stripes, k, sb)
        rng = np.random.default_rng(i)
        lost = sorted(rng.choice(k, size=min(m, k), replace=False).tolist())
        present = [0 if j in lost else 1 for j in range(k)] + [1] * m
        stream = torch.cuda.Stream(device=DEV)
        with torch.cuda.stream(stream):
            d = torch.from_numpy(data).to(DEV, non_blocking=False)
            p = torch.zeros((n_stripes, m, sb), dtype=torch.uint8, device=DEV)
            out = torch.zeros((n_stripes, len(lost), sb), dtype=torch.uint8, device=DEV)
            for _ in range(3):  # repeated calls on the same plan
                R.encode_batch_dev(k, m, d, p, stream=stream)
                R.reconstruct_batch_dev(k, m, present, d, p, out, stream=stream)
            stream.synchronize()
            results[i] = (data, lost, p.cpu().numpy(), out.cpu().numpy())

    _run_threads(work, len(SHAPES))
    for i, (k, m, sb) in enumerate(SHAPES):
        data, lost, par, rest = results[i]
        np.testing.assert_array_equal(par, oracle.encode_batch(k, m, data, threads=2), err_msg=f"thread {i}")
        np.testing.assert_array_equal(rest, data[:, lost], err_msg=f"thread {i}")


def test_one_shot_and_host_batches_from_threads(oracle):
    def work(i):
        k, m, sb = SHAPES[i % 4 + 2]
        data = splitmix_bytes(0x9000 + i, k * sb).reshape(k, sb)
        if i % 2:  # one-shot API (root.zig:14-84)
            par = R.encode(k, m, [bytes(r) for r in data])
            exp = oracle.encode_batch(k, m, data[None], threads=1)[0]
            assert [bytes(r) for r in exp] == [bytes(p) for p in par], f"thread {i}"
            orig = [bytes(r) for r in data]
            orig[0] = None
            rest = R.decode(k, m, orig, [bytes(p) for p in par])
            assert bytes(rest[0]) == bytes(data[0]), f"thread {i}"
        else:  # host-resident batch through the shared per-device staging ring
            batch = splitmix_bytes(0xA000 + i, 4 * k * sb).reshape(4, k, sb)
            par = np.zeros((4, m, sb), np.uint8)
            R.encode_batch_host(k, m, batch, par)
            np.testing.assert_array_equal(par, oracle.encode_batch(k, m, batch, threads=1), err_msg=f"thread {i}")

    _run_threads(work, 8)
