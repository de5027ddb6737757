#!/usr/bin/env python
"""Summarise one rocprofv3 SQ pass (tools/pmc_valu.sh) into per-kernel f64 VALU work.

A CDNA4 SIMD is 16 lanes wide, so every non-packed wave64 VALU instruction (f64, f32, int, DPP
move) occupies it for 4 cycles: the issue peak is 256 CUs x 4 SIMDs x 2.4 GHz / 4 = 614.4 G
wave-instructions/s (x 64 = 39.3 T lane-ops/s, the f64 vector peak: 78.6 TFLOP/s with an FMA
counted as two flops).  bench.py divides SQ_INSTS_VALU per launch by the kernel's live mean launch
time and prices it against that peak.  The f64 share (ADD+MUL+FMA+TRANS_F64) is kept beside it,
with the per-kernel totals of every counter.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import read_counter, source_sha  # noqa: E402

COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
            "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU", "SQ_WAVES")
F64 = COUNTERS[1:5]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    per = {c: read_counter(a.csv, c) for c in COUNTERS}
    kernels = {}
    for name in sorted(set().union(*[set(v) for v in per.values()])):
        launches = max(per[c].get(name, [0, 0.0])[0] for c in COUNTERS)
        tot = {c: per[c].get(name, [0, 0.0])[1] for c in COUNTERS}
        f64 = sum(tot[c] for c in F64)
        kernels[name] = {
            "launches": launches,
            "counters": {c: int(v) for c, v in tot.items()},
            "f64_lane_ops_per_launch": int(64 * f64 / max(1, launches)),
            "valu_insts_per_launch": int(tot["SQ_INSTS_VALU"] / max(1, launches)),
            "f64_share_of_valu": round(f64 / tot["SQ_INSTS_VALU"], 3) if tot["SQ_INSTS_VALU"] else None,
        }
    rec = {"workload": a.workload, "source_sha": source_sha(),
           "command": "bench.py --workload %s --steps 1 --warmup 0 --no-cpu-baseline" % a.workload,
           "definition": "valu_insts = SQ_INSTS_VALU (wave64 instructions, 4 SIMD cycles each); "
                         "f64 lane-ops = 64 x (ADD+MUL+FMA+TRANS)_F64",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v["f64_lane_ops_per_launch"] for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
