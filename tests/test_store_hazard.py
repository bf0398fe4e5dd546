"""No generated kernel may rewrite a 128-bit store's data registers in the very next
instruction (profiles/r03/spill_root_cause.md): LLVM leaves out that wait state for
buffer stores with a register soffset, and on gfx950 such a store then sometimes wrote
the overwritten value. The FFT kernels' stores carry their own wait state (rs_fftnet.cpp
STB); these tests disassemble the code objects the library compiles and check every
wide store (tools/store_hazard_scan.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import store_hazard_scan as S  # noqa: E402

OBJDUMP = S.OBJDUMP


def _scan_dir(d):
    objs = [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(".co")]
    assert objs, "no code objects were compiled"
    bad = {}
    for p in objs:
        n, sites = S.scan(p)
        if sites:
            bad[os.path.basename(p)] = sites[:3]
    return len(objs), bad


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not in the image")
def test_fft_kernels_store_wait_state(tmp_path):
    """hipRTC builds of FFT encode kernels (incl. a spilling one) here, no device."""
    code = ("import reedsol_amd as R\n"
            "for k, m in [(33, 17), (100, 20), (64, 64)]: R.fft_compile_check(k, m)\n")
    env = dict(os.environ, RS_AMD_CACHE_DIR=str(tmp_path), PYTHONPATH=os.path.join(ROOT, "reed-solomon-cc_amd"))
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=600)
    n, bad = _scan_dir(tmp_path)
    assert n >= 3 and not bad, bad


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not in the image")
def test_box_built_kernels_store_wait_state(tmp_path):
    """The kernels a GPU process actually compiles (the box's hipRTC output can differ
    from this container's for the same source): encode, syndrome reconstruct, per-stripe
    patterns and the networks, through the library, then every code object scanned."""
    code = r"""
import numpy as np, torch, reedsol_amd as R
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(3)
def run(k, m, sb, n, lost):
    d = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, generator=g).to(dev)
    p = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, d, p)
    present = np.ones(k + m, dtype=np.uint8); present[list(lost)] = 0
    out = torch.empty((n, len([i for i in lost if i < k]), sb), dtype=torch.uint8, device=dev)
    R.reconstruct_batch_dev(k, m, present, d, p, out)
    pres = torch.ones((n, k + m), dtype=torch.uint8, device=dev); pres[:, :min(m, 4)] = 0
    rest = torch.empty((n, min(m, 4), sb), dtype=torch.uint8, device=dev)
    R.reconstruct_batch_dev_patterns(k, m, pres, d, p, rest)  # per-stripe pattern kernels
    torch.cuda.synchronize()
for k, m, sb, n, lost in [(200, 55, 4096, 4, range(55)), (100, 20, 4096, 4, range(20)),
                          (10, 4, 65536, 4, range(4)), (64, 64, 4096, 2, range(64))]:
    run(k, m, sb, n, lost)
R.net_wait()
"""
    env = dict(os.environ, RS_AMD_CACHE_DIR=str(tmp_path), RS_AMD_JIT_SYNC="1",
               PYTHONPATH=os.path.join(ROOT, "reed-solomon-cc_amd"))
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=900)
    n, bad = _scan_dir(tmp_path)
    assert n >= 4 and not bad, bad
