#!/usr/bin/env python3
"""VALU issue utilisation of the trace kernel from a rocprofv3 --pmc pass holding SQ_INSTS_VALU
and SQ_THREAD_CYCLES_VALU (scripts/pmc_quick.txt, first line), recorded per bench workload in
profiles/pmc_valu.json (bench.py copies it into the roofline object).

  valu_issue_busy = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction issues over 2 cycles on a
                    32-lane SIMD, MI355X_MICROARCH.md) / (1024 SIMDs x 2.4 GHz x kernel duration)
  lane_util       = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU): active lanes per VALU issue
Usage: pmc_to_json.py KEY PASS_DIR [OUT_JSON]"""
import csv
import glob
import json
import re
import statistics
import sys
from pathlib import Path

SIMDS, CLOCK_HZ = 1024, 2.4e9


def is_production(kernel_name: str) -> bool:
    """A trace-kernel launch of the shipped build: rt_trace_lbvh_kernel<LDS, COUNT, ...> or
    rt_trace_top_kernel<COUNT> with COUNT = false (the instrumented counting pass is excluded)."""
    m = re.search(r"rt_trace_(lbvh|top)_kernel<([^>]*)>", kernel_name)
    if not m:
        return False
    args = [a.strip() for a in m.group(2).split(",")]
    return (args[1] if m.group(1) == "lbvh" else args[0]) == "false"


def main():
    key, d = sys.argv[1:3]
    out = Path(sys.argv[3]) if len(sys.argv) > 3 else Path("profiles/pmc_valu.json")
    per = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not is_production(k):
                continue
            e = per.setdefault(r["Dispatch_Id"], {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = [e for e in per.values() if "SQ_INSTS_VALU" in e and "SQ_THREAD_CYCLES_VALU" in e]
    if not rows:
        sys.exit(f"no SQ_INSTS_VALU / SQ_THREAD_CYCLES_VALU rows for the trace kernel in {d}")
    busy = [e["SQ_INSTS_VALU"] * 2 / (SIMDS * CLOCK_HZ * e["dur_ns"] * 1e-9) for e in rows]
    util = [e["SQ_THREAD_CYCLES_VALU"] / (64 * e["SQ_INSTS_VALU"]) for e in rows]
    rec = {"valu_issue_busy": round(statistics.median(busy), 3), "lane_util": round(statistics.median(util), 3),
           "valu_insts_per_launch": statistics.median(e["SQ_INSTS_VALU"] for e in rows),
           "kernel_ms": round(statistics.median(e["dur_ns"] for e in rows) * 1e-6, 3), "dispatches": len(rows),
           "note": "busy = SQ_INSTS_VALU x 2 cyc / (1024 SIMD x 2.4 GHz x duration); "
                   "lane_util = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)"}
    data = json.loads(out.read_text()) if out.exists() else {}
    data[key] = rec
    out.write_text(json.dumps(data, indent=1) + "\n")
    print(key, rec)


if __name__ == "__main__":
    main()
