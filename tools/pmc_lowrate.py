#!/usr/bin/env python3
"""HBM traffic of the low-rate kernels against the algorithmic bytes, from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE) over tools/kernel_sweep.py on one low-rate code. Each call's
launches are split into encode and reconstruct by their kernels (the encode's phases end with the
recovery store k_ephase<..., kEpFft | kEpOut>; the block-form reconstruct runs SYN / DLO / k_lbfin1 /
k_dphase). gfx950 corrections (MI355X_MICROARCH.md §HBM): counters in KiB, FETCH_SIZE doubled
(exact for 16-B-per-lane streaming reads; these kernels load 4-B lanes, so treat the read figure
as an estimate; the ratios between kernels hold).
  python tools/pmc_lowrate.py FETCH.csv WRITE.csv --k 300 --m 1000 --sb 1048576 --stripes 16 --erased 100"""
import argparse
import collections
import csv
import json
import re

ENC = {"k_ephase<64, 1, 0>", "k_ephase<64, 4, 8>", "k_ephase<8, 6, 0>"}


def per_kernel(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        kn = r["Kernel_Name"]
        if r["Counter_Name"] != counter or not kn.startswith("void rs::"):
            continue
        m = re.match(r"void rs::(?:dev::)?(?:\(anonymous namespace\)::)?(\w+)(<[^()]*>)?", kn)
        out.append((m.group(1) + (m.group(2) or ""), float(r["Counter_Value"]) * 1024,
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--k", type=int, default=300)
    ap.add_argument("--m", type=int, default=1000)
    ap.add_argument("--sb", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=16)
    ap.add_argument("--erased", type=int, default=100)
    a = ap.parse_args()
    f, w = per_kernel(a.fetch, "FETCH_SIZE"), per_kernel(a.write, "WRITE_SIZE")
    assert [x[0] for x in f] == [x[0] for x in w], "the two passes launched different kernels"
    # a scratch slice opens with the gather phase k_ephase<64, 1, 0> (the encode's and the
    # block-form reconstruct's alike); a slice holding k_lbfin1 / k_dphase is a reconstruct's
    starts = [i for i, x in enumerate(f) if x[0] == "k_ephase<64, 1, 0>"] + [len(f)]
    kinds = ["enc"] * len(f)
    for s0, s1 in zip(starts, starts[1:]):
        if any(x[0].startswith(("k_lbfin", "k_dphase")) for x in f[s0:s1]):
            kinds[s0:s1] = ["rec"] * (s1 - s0)
    tot = {"enc": collections.Counter(), "rec": collections.Counter()}
    for (n, fb, ms), (_, wb, _), kd in zip(f, w, kinds):
        tot[kd]["fetch"] += 2 * fb
        tot[kd]["write"] += wb
        tot[kd]["ms"] += ms
        tot[kd]["dispatches"] += 1
        tot[kd]["k:" + n] += 2 * fb + wb
    # calls: every slice (one stripe) opens with one gather phase
    res = {}
    alg = {"enc": (a.k + a.m) * a.sb * a.stripes, "rec": (a.k + a.erased) * a.sb * a.stripes}
    for kd in ("enc", "rec"):
        t = tot[kd]
        if not t["dispatches"]:
            continue
        first = "k_ephase<64, 1, 0>"
        n_first = sum(1 for (n, _, _), k2 in zip(f, kinds) if k2 == kd and n == first)
        calls = max(1, n_first // a.stripes)  # one stripe per scratch slice at 1 MiB shards (2 GiB cap)
        res[kd] = {"calls": calls, "algorithmic_GB": round(alg[kd] / 1e9, 3),
                   "fetch_GB": round(t["fetch"] / calls / 1e9, 3), "write_GB": round(t["write"] / calls / 1e9, 3),
                   "traffic_over_algorithmic": round((t["fetch"] + t["write"]) / calls / alg[kd], 2),
                   "kernel_ms_per_call": round(t["ms"] / calls, 3),
                   "traffic_TBps": round((t["fetch"] + t["write"]) / (t["ms"] * 1e-3) / 1e12, 3),
                   "per_kernel_GB": {k[2:]: round(v / calls / 1e9, 3) for k, v in t.items() if k.startswith("k:")}}
    print(json.dumps({"code": f"RS({a.k},{a.m}) {a.sb} B x {a.stripes}, {a.erased} erased", **res}, indent=1))


if __name__ == "__main__":
    main()
