#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json.

gfx950 corrections (MI355X_MICROARCH.md §HBM): counters are in KiB; FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores. Values are per launch, divided by
the stripes of that launch (--stripes), so bench.py can scale them to its batch.

  python tools/pmc_traffic.py gpurun_out/pmc --stripes 1024 --out profiles/traffic.json
"""
import argparse
import csv
import json
import os
import re
import statistics


def short_name(full):
    m = re.search(r"rs_net_(encode|reconstruct|syndrome)_i(\d+)_o(\d+)_[0-9a-f]+", full)
    if m:
        return f"net_{m.group(1)}_i{m.group(2)}_o{m.group(3)}"
    m = re.search(r"rs_fft_(encode|decode|pdecode|inverse)_k(\d+)_m(\d+)_[0-9a-f]+", full)
    if m:
        return f"net_fft_{m.group(1)}_i{m.group(2)}_o{m.group(3)}"
    m = re.search(r"k_(encode_reg|decode_reg|decode_matrix)<(\d+), (\d+)>", full)
    if m:
        kind, size, nv = m.groups()
        tag = {"encode_reg": "encode_reg_w", "decode_reg": "decode_reg_w", "decode_matrix": "decode_matrix_e"}[kind]
        return f"{tag}{size}_nv{nv}"
    m = re.search(r"k_(encode_generic|decode_generic)<(\d+)>", full)
    if m:
        return f"{m.group(1)}_nv{m.group(2)}"
    m = re.search(r"k_(encode_lds|decode_lds)\w*<([^>]*)>", full)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    return None


def read(path, counter):
    vals = {}
    with open(os.path.join(path, counter, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            n = short_name(r["Kernel_Name"])
            if n and r["Counter_Name"] == counter:
                vals.setdefault(n, []).append(float(r["Counter_Value"]) * 1024.0)
    return {n: statistics.median(v) for n, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--stripes", type=int, required=True)
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--e", type=int, default=4)
    ap.add_argument("--shard-bytes", type=int, default=1 << 20)
    ap.add_argument("--only", default="", help="comma list of kernel short names to record (default all)")
    ap.add_argument("--alg-shards", type=int, default=0, help="algorithmic shard passes per stripe (override)")
    a = ap.parse_args()
    fetch, write = read(a.pmc_dir, "FETCH_SIZE"), read(a.pmc_dir, "WRITE_SIZE")
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    only = {x for x in a.only.split(",") if x}
    for n in sorted(set(fetch) & set(write)):
        if only and n not in only:
            continue
        f, w = 2.0 * fetch[n], write[n]
        alg = ((a.k + a.m) if n.startswith(("encode", "net_encode", "net_fft_encode")) else (a.k + a.e)) * a.shard_bytes
        if a.alg_shards:
            alg = a.alg_shards * a.shard_bytes
        out[n] = {"fetch_bytes_per_stripe": f / a.stripes, "write_bytes_per_stripe": w / a.stripes,
                  "hbm_bytes_per_stripe": (f + w) / a.stripes, "algorithmic_bytes_per_stripe": alg,
                  "traffic_over_algorithmic": round((f + w) / a.stripes / alg, 4),
                  "hbm_bytes_per_launch": f + w, "stripes_per_launch": a.stripes,
                  "workload": f"RS({a.k},{a.m}) {a.shard_bytes} B shards, {a.stripes} stripes per launch",
                  "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950)"}
        print(n, json.dumps(out[n]))
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
