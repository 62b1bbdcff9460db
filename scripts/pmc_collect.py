#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of one bench workload into profiles/pmc.json (read by bench.py
only when the library build matches, by its sha256 prefix).

For the production trace kernel (rt_trace_<form>_kernel<false, ...>: the instrumented counting
build is excluded), per dispatch, median over dispatches:
  valu_issue_busy = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction issues over 2 cycles on a
                    32-lane SIMD, MI355X_MICROARCH.md) / (1024 SIMDs x 2.4 GHz x kernel duration)
  lane_util       = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU): active lanes per VALU issue
  hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; gfx950 FETCH_SIZE reports half
                    of wide coalesced reads, MI355X_MICROARCH.md §HBM: doubled)
  l2_hit_rate     = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum) (MI355X_MICROARCH.md §L2), from --tcc DIR
Usage: pmc_collect.py KEY LIB_SO VALU_DIR FETCH_DIR WRITE_DIR [SQ_DIR] [--tcc TCC_DIR] [OUT_JSON]"""
import csv
import glob
import hashlib
import json
import re
import statistics
import sys
from pathlib import Path

SIMDS, CLOCK_HZ = 1024, 2.4e9


def is_production(kernel_name: str) -> bool:
    m = re.search(r"rt_trace_(lds|top|grid|global|brute)_kernel<([^>]*)>", kernel_name)
    return bool(m) and m.group(2).split(",")[0].strip() == "false"


def dispatches(d):
    per = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if not is_production(r["Kernel_Name"]):
                continue
            e = per.setdefault((f, r["Dispatch_Id"]), {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                        "kernel": r["Kernel_Name"]})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(per.values())


def main():
    tcc = None
    if "--tcc" in sys.argv:
        i = sys.argv.index("--tcc")
        tcc = sys.argv[i + 1]
        del sys.argv[i:i + 2]
    key, lib, vdir, fdir, wdir = sys.argv[1:6]
    sqdir = sys.argv[6] if len(sys.argv) > 6 and not sys.argv[6].endswith(".json") else None
    out = Path(sys.argv[-1]) if sys.argv[-1].endswith(".json") else Path("profiles/pmc.json")
    v = [e for e in dispatches(vdir) if "SQ_INSTS_VALU" in e and "SQ_THREAD_CYCLES_VALU" in e]
    f = [e["FETCH_SIZE"] for e in dispatches(fdir) if "FETCH_SIZE" in e]
    w = [e["WRITE_SIZE"] for e in dispatches(wdir) if "WRITE_SIZE" in e]
    if not v or not f or not w:
        sys.exit(f"missing production-kernel rows: valu {len(v)} fetch {len(f)} write {len(w)}")
    busy = [e["SQ_INSTS_VALU"] * 2 / (SIMDS * CLOCK_HZ * e["dur_ns"] * 1e-9) for e in v]
    util = [e["SQ_THREAD_CYCLES_VALU"] / (64 * e["SQ_INSTS_VALU"]) for e in v]
    fk, wk = statistics.median(f), statistics.median(w)
    rec = {"lib_sha256": hashlib.sha256(Path(lib).read_bytes()).hexdigest()[:16],
           "kernel": v[0]["kernel"][:120],
           "valu_issue_busy": round(statistics.median(busy), 3), "lane_util": round(statistics.median(util), 3),
           "valu_insts_per_launch": statistics.median(e["SQ_INSTS_VALU"] for e in v),
           "kernel_ms": round(statistics.median(e["dur_ns"] for e in v) * 1e-6, 3),
           "fetch_size_kib_raw": fk, "write_size_kib": wk,
           "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
           "dispatches": [len(v), len(f), len(w)]}
    if sqdir:
        s = [e for e in dispatches(sqdir)]
        if s:
            for c in ("SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
                      "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
                vals = [e[c] for e in s if c in e]
                if vals:
                    rec[c] = statistics.median(vals)
    if tcc:
        t = [e for e in dispatches(tcc) if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e]
        if t:
            hits = statistics.median(e["TCC_HIT_sum"] for e in t)
            miss = statistics.median(e["TCC_MISS_sum"] for e in t)
            rec["l2_hit_rate"] = round(hits / max(1.0, hits + miss), 4)
            rec["tcc_hit"], rec["tcc_miss"] = hits, miss
    rec["note"] = ("busy = SQ_INSTS_VALU x 2 cyc / (1024 SIMD x 2.4 GHz x duration); lane_util = "
                   "SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU); hbm = 2 x FETCH_SIZE + WRITE_SIZE; "
                   "l2_hit_rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)")
    data = json.loads(out.read_text()) if out.exists() else {}
    data[key] = rec
    out.write_text(json.dumps(data, indent=1) + "\n")
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
