#!/usr/bin/env python3
"""Spill investigation, step 2 (profiles/r03/spill_root_cause.md): launch hand-assembled
variants of the FFT encode kernel's ISA on the repro's batch (RS(1000,64), 4 KiB shards,
96 stripes) and compare with the oracle (and run the library's own build first, same buffers).

Variants are code objects assembled from `hipcc -S` output of the generated source
(clang -x assembler + ld.lld) and given as NAME=PATH:KERNEL; each is launched `reps`
times exactly as fftnet::launch does (grid = min(units, CUs), 512 threads, same args).
NAME=library runs the library's own build instead.
  python tools/spill_asm_check.py reps NAME=file.co:kernel|library [...]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

reps = int(sys.argv[1])
variants = [a.split("=", 1) for a in sys.argv[2:]]
k, m, sb, n = 1000, 64, 4096, 96
dev = torch.device("cuda:0")
rng = np.random.default_rng(1000)
data = rng.integers(0, 256, (n, k, sb), dtype=np.uint8)
exp = torch.from_numpy(O.encode_batch(k, m, data, threads=16)).to(dev)  # the oracle's parity
d = torch.from_numpy(data).to(dev)
out = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)  # one output buffer for every variant
hip = C.CDLL("libamdhip64.so")
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def report(name, kname, bad):
    print(json.dumps({"variant": name, "kernel": kname, "reps": reps, "bad_launches": len(bad), "detail": bad[:4]}),
          flush=True)


def check(r, bad):
    diff = out != exp
    if bool(diff.any()):
        nz = diff.nonzero()
        bad.append({"rep": r, "bytes": int(diff.sum()), "shards": sorted(set(nz[:, 1].tolist()))[:8]})


for name, spec in variants:
    if spec == "library":  # the library's own build (RS_AMD_FFT_PREFETCH / RS_AMD_FFT_ALLOW_SPILL)
        bad = []
        for r in range(reps):
            out.fill_(0)
            R.encode_batch_dev(k, m, d, out)
            torch.cuda.synchronize()
            check(r, bad)
        report(name, R.encode_kernel_name(k, m, sb), bad)
        continue
    path, kname = spec.split(":")
    if os.path.isdir(path):  # a code-object cache directory: its one entry
        path = os.path.join(path, sorted(os.listdir(path))[0])
    mod, fn = C.c_void_p(), C.c_void_p()
    assert hip.hipModuleLoad(C.byref(mod), path.encode()) == 0, path
    assert hip.hipModuleGetFunction(C.byref(fn), mod, kname.encode()) == 0, kname
    ups = sb // 2048
    n_units = n * ups
    args = [C.c_uint64(d.data_ptr()), C.c_uint64(k * sb), C.c_uint64(d.data_ptr()), C.c_uint64(0),
            C.c_uint64(out.data_ptr()), C.c_uint64(m * sb), C.c_uint32(sb), C.c_uint32(ups),
            C.c_uint64(n_units), C.c_uint64(n), C.c_uint64(0), C.c_uint32(0)]
    params = (C.c_void_p * len(args))(*[C.cast(C.byref(a), C.c_void_p) for a in args])
    grid = min(n_units, n_cu)
    bad = []
    for r in range(reps):
        out.fill_(0)
        torch.cuda.synchronize()
        st = hip.hipModuleLaunchKernel(fn, grid, 1, 1, 512, 1, 1, 0, stream, params, None)
        assert st == 0, st
        torch.cuda.synchronize()
        check(r, bad)
    report(name, kname, bad)
