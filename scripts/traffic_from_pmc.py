#!/usr/bin/env python3
"""HBM traffic per launch of the trace kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads (MI355X_MICROARCH.md §HBM), so it is doubled. Writes here are the
16-B-per-lane accumulator and 4-B rgba8 stores. Usage:
  traffic_from_pmc.py KEY FETCH_DIR WRITE_DIR [OUT_JSON]"""
import csv
import glob
import json
import re
import statistics
import sys
from pathlib import Path


def is_production(kernel_name: str) -> bool:
    """A trace-kernel launch of the shipped build: rt_trace_lbvh_kernel<LDS, COUNT, ...> or
    rt_trace_top_kernel<COUNT> with COUNT = false (the instrumented counting pass is excluded)."""
    m = re.search(r"rt_trace_(lbvh|top)_kernel<([^>]*)>", kernel_name)
    if not m:
        return False
    args = [a.strip() for a in m.group(2).split(",")]
    return (args[1] if m.group(1) == "lbvh" else args[0]) == "false"


def per_dispatch(d, counter):
    """Production launches only (is_production)."""
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and is_production(r["Kernel_Name"]):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    key, fdir, wdir = sys.argv[1:4]
    out = Path(sys.argv[4]) if len(sys.argv) > 4 else Path("profiles/pmc_traffic.json")
    f = per_dispatch(fdir, "FETCH_SIZE")
    w = per_dispatch(wdir, "WRITE_SIZE")
    if not f or not w:
        sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for the trace kernel in {fdir} / {wdir}")
    fk, wk = statistics.median(f), statistics.median(w)
    rec = {"fetch_size_kib_raw": fk, "write_size_kib": wk,
           "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
           "dispatches": [len(f), len(w)],
           "note": "hbm = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide reads)"}
    data = json.loads(out.read_text()) if out.exists() else {}
    data[key] = rec
    out.write_text(json.dumps(data, indent=1) + "\n")
    print(key, rec)


if __name__ == "__main__":
    main()
