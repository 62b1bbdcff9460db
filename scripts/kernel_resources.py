#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of a HIP source for gfx950 (compiler remarks).

usage: python scripts/kernel_resources.py [file.hip] [extra hipcc flags...]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
src = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "ray-tracing-gpu-vulkan_amd/csrc/rt_kernels.hip")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
       f"-I{ROOT / 'include'}", "--offload-arch=gfx950", "-fno-gpu-rdc", "-fno-slp-vectorize",
       "--cuda-device-only", "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
print(f"{'kernel':<70} {'VGPR':>5} {'AGPR':>5} {'SGPR':>5} {'sSpill':>6} {'vSpill':>6} {'occ':>4}")
for r in rows:
    if "trace" not in r["name"] and "resolve" not in r["name"]:
        continue
    print(f"{r['name'][:70]:<70} {r.get('VGPRs', -1):>5} {r.get('AGPRs', -1):>5} {r.get('SGPRs', -1):>5} "
          f"{r.get('SGPRs Spill', -1):>6} {r.get('VGPRs Spill', -1):>6} {r.get('Occupancy [waves/SIMD]', -1):>4}")
