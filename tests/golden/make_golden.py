"""Generates the golden fixtures in this directory from the CPU oracle (oracle/rt_oracle.cpp).

The reference has no test data for the hot path: these fixtures pin the oracle
against regressions and are the shared expected outputs of the GPU parity tests. Re-run only on a
deliberate contract change:  python tests/golden/make_golden.py
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle  # noqa: E402

CASES = {
    # name: W, H, band (offset_y, band_h), spp, max_depth, seed_mode, rng_mode
    "g64x36_spp4": dict(W=64, H=36, offset=[0, 0], band_w=64, band_h=36, spp=4, max_depth=50,
                        seed_mode=0, rng_mode=0, t=0.0, K=11),
    "g48x32_spp3_depth3_local": dict(W=48, H=64, offset=[0, 32], band_w=48, band_h=32, spp=3,
                                     max_depth=3, seed_mode=1, rng_mode=0, t=0.0, K=11),
    "g40x24_spp2_counter": dict(W=40, H=24, offset=[0, 0], band_w=40, band_h=24, spp=2, max_depth=50,
                                seed_mode=0, rng_mode=1, t=0.5, K=11),
    # RT_RNG_SAMPLE_HASH (counter-based per-sample streams, fixed-point sums), a band with offset
    "g56x40_spp7_hash": dict(W=56, H=48, offset=[0, 8], band_w=56, band_h=40, spp=7, max_depth=50,
                             seed_mode=0, rng_mode=2, t=0.0, K=11),
}


def main(only=None):
    oracle.build()
    for name, m in CASES.items():
        if only and name not in only:
            continue
        sc = oracle.generate_scene(m["t"], m["K"])
        rci = oracle.render_call_info(m["spp"], m["W"], m["H"], tuple(m["offset"]))
        op = oracle.options(max_depth=m["max_depth"], seed_mode=m["seed_mode"], rng_mode=m["rng_mode"])
        acc, out, st = oracle.render(sc, rci, m["band_w"], m["band_h"], opts=op, threads=4)
        np.savez_compressed(HERE / f"{name}.npz", accum=acc, rgba8=out, stats=np.array(st, np.uint64))
        (HERE / f"{name}.json").write_text(json.dumps(m, indent=1) + "\n")
        print(name, st)


if __name__ == "__main__":
    main(sys.argv[1:])
