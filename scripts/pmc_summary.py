#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one directory of pN/ passes) per kernel."""
import collections
import csv
import glob
import sys


def summarise(d, match="rt_trace"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if match not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


if __name__ == "__main__":
    for d in sys.argv[1:]:
        for k, v in summarise(d).items():
            print(d, k[:70])
            for c, x in sorted(v.items()):
                print(f"   {c:28s} {x:.4g}")
            if "SQ_INSTS_VALU" in v and "SQ_THREAD_CYCLES_VALU" in v:
                print(f"   lane util (THREAD_CYCLES_VALU / 64 INSTS_VALU) = {v['SQ_THREAD_CYCLES_VALU'] / (64 * v['SQ_INSTS_VALU']):.3f}")
