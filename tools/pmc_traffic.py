#!/usr/bin/env python
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM traffic.

Usage (after two separate ``rocprofv3 --pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE``
runs of ``bench.py --steps 1 --warmup 0 --no-cpu-baseline``):

    python tools/pmc_traffic.py --fetch gpurun_out/pmcF/pmc_counter_collection.csv \
        --write gpurun_out/pmcW/pmc_counter_collection.csv --workload C2 \
        --out profiles/r01_c2_pmc_traffic.json

Corrections (MI355X_MICROARCH.md § HBM): counters are in KiB; on gfx950
FETCH_SIZE tallies a wide coalesced 128-B request as 64 B, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  The raw values are kept beside
the corrected ones.  ``source_sha`` fingerprints the HIP sources so bench.py
only quotes traffic measured on the code it is timing.
"""
from __future__ import annotations

import argparse
import collections
import csv
import hashlib
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ("iterative_cleaner_amd/csrc/ic_kernels.hip", "iterative_cleaner_amd/csrc/ic_session.hip",
           "iterative_cleaner_amd/csrc/ic_internal.h", "iterative_cleaner_amd/csrc/ic_comm.hip",
           "iterative_cleaner_amd/csrc/ic_comm.h")


def source_sha() -> str:
    h = hashlib.sha256()
    for rel in SOURCES:
        with open(os.path.join(REPO, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def short_name(kernel_name: str) -> str:
    """'void icgpu::k_diag_p2<1024>(...)' -> 'k_diag' (the bench's kernel ids)."""
    n = kernel_name.split("(")[0].split("::")[-1]
    n = n.split("<")[0]
    return "k_diag" if n.startswith("k_diag") else n


def read_counter(path: str, counter: str):
    per = collections.defaultdict(lambda: [0, 0.0])
    seen = set()
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = short_name(r["Kernel_Name"])
            if not name.startswith("k_"):
                continue
            key = (r["Dispatch_Id"], name)
            if key not in seen:
                seen.add(key)
                per[name][0] += 1
            per[name][1] += float(r["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = read_counter(a.fetch, "FETCH_SIZE")
    write = read_counter(a.write, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        nf, fkib = fetch.get(name, [0, 0.0])
        nw, wkib = write.get(name, [0, 0.0])
        launches = max(nf, nw)
        fetch_b = 2.0 * fkib * 1024.0          # gfx950 FETCH_SIZE reads 1/2 on wide streams
        write_b = wkib * 1024.0
        kernels[name] = {
            "launches": launches,
            "fetch_kib_raw": round(fkib, 1),
            "write_kib_raw": round(wkib, 1),
            "traffic_bytes": int(fetch_b + write_b),
            "traffic_bytes_per_launch": int((fetch_b + write_b) / max(1, launches)),
        }
    rec = {"workload": a.workload, "source_sha": source_sha(),
           "command": "bench.py --workload %s --steps 1 --warmup 0 --no-cpu-baseline" % a.workload,
           "correction": "FETCH_SIZE x2 (gfx950 wide-stream tally), KiB -> bytes",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: v["traffic_bytes_per_launch"] for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
