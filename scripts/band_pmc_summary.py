"""Summary of rocprofv3 --pmc passes over config 4's rank-0 band (scripts/band_probe.py --ranks 0
--reps 1, one counter per pass): per trace-kernel launch, the counter value and the launch's
duration. The first launch has no LPT history; the second is the LPT-ordered launch the bench times.

usage: python scripts/band_pmc_summary.py OUT.json DIR [DIR ...]   (each DIR holds run_counter_collection.csv)"""
import csv
import json
import sys
from pathlib import Path

out, dirs = sys.argv[1], sys.argv[2:]
launches = []
for d in dirs:
    rows = list(csv.DictReader(open(Path(d) / "run_counter_collection.csv")))
    for r in rows:
        if "rt_trace_" not in r["Kernel_Name"]:
            continue
        launches.append({"kernel": r["Kernel_Name"][:100], "dispatch": int(r["Dispatch_Id"]),
                         "counter": r["Counter_Name"], "value_kb": float(r["Counter_Value"]),
                         "duration_ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
rec = {"what": "rocprofv3 --pmc of config 4's rank-0 band (136 rows of 1920x1080, 10000 spp) rendered alone on "
               "one MI355X (scripts/band_probe.py --ranks 0 --reps 1): first launch without LPT history, then "
               "the LPT-ordered launch; FETCH_SIZE / WRITE_SIZE in KiB as the counters report them",
       "launches": launches}
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec, indent=1))
