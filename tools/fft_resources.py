#!/usr/bin/env python3
"""Register / scratch / LDS use of generated FFT kernels (no device): the kernel is
compiled through the library's hipRTC path into a private code-object cache and its
AMDGPU metadata note is read with llvm-readelf.
  python tools/fft_resources.py K M [encode|decode|pdecode] [RS_AMD_X=v ...]
(pdecode: the pattern compiled in; m erased data shards, every third from 1)"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))


def main():
    k, m = int(sys.argv[1]), int(sys.argv[2])
    kind = sys.argv[3] if len(sys.argv) > 3 else "encode"
    for kv in sys.argv[4:]:
        n, v = kv.split("=", 1)
        os.environ[n] = v
    d = tempfile.mkdtemp(prefix="fftres")
    os.environ["RS_AMD_CACHE_DIR"] = d
    import reedsol_amd as R
    if kind == "pdecode":
        lost = list(range(1, k, 3))[:min(m, k)]
        r = R.fft_pdecode_compile_check(k, m, [0 if i in lost else 1 for i in range(k)] + [1] * m)
    else:
        r = (R.fft_decode_compile_check if kind == "decode" else R.fft_compile_check)(k, m)
    for co in glob.glob(os.path.join(d, "**", "*"), recursive=True):
        if not os.path.isfile(co):
            continue
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True,
                             text=True).stdout
        got = {}
        for key in (".vgpr_count", ".agpr_count", ".sgpr_count", ".private_segment_fixed_size",
                    ".group_segment_fixed_size", ".vgpr_spill_count", ".sgpr_spill_count"):
            mm = re.search(re.escape(key) + r":\s+(\d+)", out)
            if mm:
                got[key.strip(".")] = int(mm.group(1))
        print(os.path.basename(co)[:24], got, {"compile_ms": round(r["compile_ms"])})


if __name__ == "__main__":
    main()
