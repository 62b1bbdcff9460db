#!/usr/bin/env python3
"""Sums FETCH_SIZE / WRITE_SIZE (KiB) per kernel name over the LAST dispatch of each kernel in
rocprofv3 --pmc output directories. Usage: pmc_traffic.py DIR [DIR...]"""
import csv
import glob
import sys

for d in sys.argv[1:]:
    last = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"][:60], r["Counter_Name"])
            did = int(r["Dispatch_Id"])
            if k not in last or did >= last[k][0]:
                prev = last.get(k, (did, 0.0))
                last[k] = (did, (prev[1] if prev[0] == did else 0.0) + float(r["Counter_Value"]))
    for (kn, cn), (did, v) in sorted(last.items()):
        print(f"{d}: {kn:<60} {cn:<11} {v * 1024 / 1e6:12.1f} MB (dispatch {did})")
