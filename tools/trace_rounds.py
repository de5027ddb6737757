#!/usr/bin/env python
"""Per-dispatch view of one cleaning run from a rocprofv3 --kernel-trace CSV:
kernel, grid size (workgroups), duration and the gap before it, for the
dispatches of the LAST ic_run in the trace (from its last k_chan_partials<0>,
the first pass of a run, on)."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("icgpu::", "") for r in rows]
    first = max(i for i, n in enumerate(names) if n.startswith("k_chan_partials<0>"))
    prev_end = None
    tot = {}
    for r, n in zip(rows[first - 4:], names[first - 4:]):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) // max(1, int(r.get("Workgroup_Size_X", 1) or 1))
        print("%-28s grid %8d  %9.1f us  gap %7.1f us" % (n[:28], grid, (e - s) / 1e3, gap))
        tot[n] = tot.get(n, 0.0) + (e - s) / 1e3
    print(sorted(((round(v, 1), k) for k, v in tot.items()), reverse=True))


if __name__ == "__main__":
    main(sys.argv[1])
