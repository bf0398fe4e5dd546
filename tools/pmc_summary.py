#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs: per kernel, the mean of each counter over
its dispatches (values summed over the dimension instances of one dispatch).
  python tools/pmc_summary.py gpurun_out/pmcw/c4_g1 [more dirs...]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            key = (row["Kernel_Name"], row.get("Dispatch_Id", row.get("Correlation_Id", "")))
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (kn, _), ctr in per.items():
        for c, v in ctr.items():
            out[kn][c].append(v)
    return out


def main():
    agg = collections.defaultdict(dict)
    for d in sys.argv[1:]:
        for kn, ctr in load(d).items():
            for c, vs in ctr.items():
                agg[kn][c] = (sum(vs) / len(vs), len(vs))
    for kn in sorted(agg):
        if kn.startswith("__amd"):
            continue
        print(kn[:90])
        for c in sorted(agg[kn]):
            v, n = agg[kn][c]
            print(f"   {c:24s} {v:12.5g}  (n={n})")


if __name__ == "__main__":
    main()
