"""Static ISA instruction counts per phase of one trace kernel (DESIGN.md §4.4's phase split).

The kernels mark their phases with STAMP(k) (rt_kernels.hip); an -DRT_ASM_MARKS device-only
listing turns each into an `; RT_PHASE k` comment where the phase begins in program order (0 loop
head / refill, 4 sample start, 1 ray setup with the exhaustive big spheres, 2 walk, 3 shading,
5 refill: block hand-out, 6 refill: block fetch). Instructions are attributed to the most recent
marker above them, so code the compiler sinks or hoists across a marker counts where it lands.
Counts are static (each instruction once), not dynamic: a loop body counts once.

usage: python scripts/isa_phases.py LISTING.s [KERNEL_SUBSTRING] [--json out]
       (listing: make -C ray-tracing-gpu-vulkan_amd asm DEVFLAGS="--offload-arch=gfx950 -fno-gpu-rdc -fno-slp-vectorize -DRT_ASM_MARKS")
default kernel: the headline form rt_trace_grid_kernel<false, MODE_HASH, IN_LDS, !COOP, REC, !CQ, FLAT>."""
import json
import re
import sys
from collections import Counter, OrderedDict

PHASES = {0: "loop head", 4: "sample start", 5: "refill: hand-out", 6: "refill: block fetch", 1: "ray setup (big spheres)",
          2: "walk", 3: "shading", 7: "exit", -1: "prologue"}
HEADLINE = "_ZN12_GLOBAL__N_120rt_trace_grid_kernelILb0ELi1ELb1ELb0ELb1ELb0ELb1EEEvN2rt11TraceParamsE"


def classify(op: str) -> list:
    c = []
    if op.startswith("v_"):
        c.append("valu")
        if op.startswith(("v_sqrt", "v_rcp", "v_rsq", "v_sin", "v_cos", "v_exp", "v_log")):
            c.append("valu_trans")
        if op.startswith("v_cndmask"):
            c.append("v_cndmask")
        if op.startswith(("v_mul_lo_u32", "v_mul_hi", "v_mad_u64", "v_mad_i64")):
            c.append("valu_int_mul")
        if op.startswith(("v_cmp", "v_cmpx")):
            c.append("v_cmp")
        if "f64" in op:
            c.append("valu_f64")
        if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            c.append("lane_xfer")
    elif op.startswith("s_"):
        if op.startswith(("s_load", "s_buffer_load")):
            c.append("smem")
        elif op.startswith("s_waitcnt"):
            c.append("waitcnt")
        elif op.startswith(("s_cbranch", "s_branch")):
            c.append("branch")
        elif op.startswith(("s_nop", "s_endpgm", "s_barrier", "s_sleep", "s_setprio")):
            c.append("other_s")
        else:
            c.append("salu")
            if "exec" in op:
                c.append("exec_op")
    elif op.startswith("ds_"):
        c.append("lds")
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        c.append("vmem")
        if op.startswith("scratch_") or "offen" in op:
            pass
    return c


def count(path: str, kernel: str = HEADLINE) -> OrderedDict:
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        if ln.startswith(kernel) and ln.rstrip().endswith(tuple([":", "TraceParamsE"])) or ln.startswith(kernel + ":"):
            start = i
            break
    if start is None:
        raise SystemExit(f"kernel {kernel} not found")
    phase = -1
    per = OrderedDict()
    scratch = Counter()
    for ln in lines[start + 1:]:
        s = ln.strip()
        if s.startswith(".Lfunc_end") or s.startswith("; -- End function"):
            break
        m = re.search(r"RT_PHASE (\d+)", s)
        if m:
            phase = int(m.group(1))
            continue
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c = per.setdefault(phase, Counter())
        c["total"] += 1
        for k in classify(op):
            c[k] += 1
        if op.startswith("scratch_") or ("buffer_" in op and "off" in s and "s[0:3]" in s):
            scratch[phase] += 1
    out = OrderedDict()
    for ph, c in per.items():
        out[PHASES.get(ph, str(ph))] = dict(c, **({"scratch": scratch[ph]} if scratch[ph] else {}))
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if js in args:
        args.remove(js)
    path = args[0]
    kernel = args[1] if len(args) > 1 else HEADLINE
    res = count(path, kernel)
    cols = ["total", "valu", "valu_trans", "v_cndmask", "v_cmp", "valu_int_mul", "salu", "exec_op", "branch",
            "lds", "vmem", "smem", "waitcnt", "scratch"]
    print(f"{'phase':26s}" + "".join(f"{c:>10s}" for c in cols))
    tot = Counter()
    for ph, c in res.items():
        print(f"{ph:26s}" + "".join(f"{c.get(k, 0):>10d}" for k in cols))
        tot.update(c)
    print(f"{'all':26s}" + "".join(f"{tot.get(k, 0):>10d}" for k in cols))
    if js:
        with open(js, "w") as f:
            json.dump({"kernel": kernel, "phases": res}, f, indent=1)


if __name__ == "__main__":
    main()
