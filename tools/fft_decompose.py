#!/usr/bin/env python3
"""Where the FFT kernels' time goes: interleaved A/B rounds in one process over build
variants selected by env vars the generator reads (RS_AMD_FFT_DEBUG bits: 1 no loads,
2 no stores, 4 decode without its tail, 8 decode without runtime multiplies, 16 round-3
decode load order; RS_AMD_FFT_PREFETCH). Times the encode and the fused reconstruct
(RS_AMD_FDEC=1) of one code with HIP events, reports median ms, the kernels launched and
whether the bytes are right (measurement builds are not).
  python tools/fft_decompose.py K M SB STRIPES LOSSES 'VAR=a,b' ['VAR2=c,d' ...]"""
import itertools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402


def main():
    k, m, sb, n, e = (int(x) for x in sys.argv[1:6])
    axes = [(kv.split("=", 1)[0], kv.split("=", 1)[1].split(",")) for kv in sys.argv[6:]]
    variants = [tuple(zip([a[0] for a in axes], v)) for v in itertools.product(*[a[1] for a in axes])]
    rounds, reps = int(os.environ.get("ROUNDS", "4")), int(os.environ.get("REPS", "3"))
    form = os.environ.get("FORM", "dyn")  # dyn: the pattern as data; pattern: compiled in (warmed)
    if form == "dyn":
        os.environ["RS_AMD_FDEC"] = "1"
    dev = torch.device("cuda:0")
    lost = list(range(1, k, 3))[:e] if 3 * e <= k else list(range(e))
    present = [0 if i in lost else 1 for i in range(k)] + [1] * m
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev)
    par = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    out = torch.empty((n, e, sb), dtype=torch.uint8, device=dev)
    for kk in list(os.environ):
        if kk.startswith("RS_AMD_FFT_"):
            os.environ.pop(kk)
    R.encode_batch_dev(k, m, data, par)
    torch.cuda.synchronize()
    ref = par.clone()
    s = torch.cuda.current_stream()

    def timed(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    res = {v: {"enc": [], "rec": [], "ok_enc": True, "ok_rec": True, "kern": ""} for v in variants}
    for r in range(rounds + 1):
        for v in variants:
            for name, val in v:
                os.environ[name] = val
            if form == "pattern" and r == 0:
                R.reconstruct_warm(k, m, sb, present)
            te = timed(lambda: R.encode_batch_dev(k, m, data, par, stream=s))
            ke = R.last_kernels()
            res[v]["ok_enc"] &= bool(torch.equal(par, ref))
            par.copy_(ref)
            out.zero_()
            tr = timed(lambda: R.reconstruct_batch_dev(k, m, present, data, par, out, stream=s))
            kr = R.last_kernels()
            res[v]["ok_rec"] &= bool(torch.equal(out, data[:, lost]))
            res[v]["kern"] = ";".join(ke + kr)
            print(f"round {r} {dict(v)} enc {te:.3f} rec {tr:.3f}", file=sys.stderr, flush=True)
            if r > 0:
                res[v]["enc"].append(te)
                res[v]["rec"].append(tr)
            for name, _ in v:
                os.environ.pop(name)
    alg_e, alg_r = (k + m) * sb * n, (k + e) * sb * n
    for v in variants:
        te, tr = float(np.median(res[v]["enc"])), float(np.median(res[v]["rec"]))
        print(json.dumps({"code": f"RS({k},{m}) {sb} B x {n}, {e} lost", **dict(v),
                          "enc_ms": round(te, 3), "enc_frac": round(alg_e / te / 8e9, 4),
                          "rec_ms": round(tr, 3), "rec_frac": round(alg_r / tr / 8e9, 4),
                          "ok_enc": res[v]["ok_enc"], "ok_rec": res[v]["ok_rec"], "kernels": res[v]["kern"]}),
              flush=True)


if __name__ == "__main__":
    main()
