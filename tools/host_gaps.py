"""Where the host spends the GPU's idle time between two cleans: from a
rocprofv3 --hip-trace --kernel-trace run (CSV), the HIP API calls made while
no kernel was running, for the largest idle intervals of the trace.

    python tools/host_gaps.py DIR [--top N]   (DIR: the rocprofv3 -d directory)"""
import argparse
import csv
import glob
import os


def load(d, pat):
    f = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=4)
    ap.add_argument("--max-us", type=float, default=5000.0, help="ignore longer idle intervals (setup, code loads)")
    ap.add_argument("--tail", type=float, default=0.5, help="only the last fraction of the trace's kernels")
    a = ap.parse_args()
    kern = load(a.dir, "*kernel_trace.csv") + load(a.dir, "*memory_copy_trace.csv")
    api = load(a.dir, "*hip_api_trace.csv")
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kern)
    iv = iv[int(len(iv) * (1.0 - a.tail)):]
    gaps = []
    for (s0, e0), (s1, e1) in zip(iv, iv[1:]):
        if s1 > e0 and s1 - e0 <= a.max_us * 1e3:
            gaps.append((s1 - e0, e0, s1))
    gaps.sort(reverse=True)
    calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", r.get("Operation", "?")))
                   for r in api)
    print("kernels/copies %d, idle intervals %d, idle total %.1f us" % (len(iv), len(gaps), sum(g[0] for g in gaps) / 1e3))
    for g, e0, s1 in gaps[:a.top]:
        print("\nidle %.1f us" % (g / 1e3))
        agg = {}
        for s, e, f in calls:
            lo, hi = max(s, e0), min(e, s1)
            if hi > lo:
                t, n = agg.get(f, (0, 0))
                agg[f] = (t + hi - lo, n + 1)
        covered = 0
        for f, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
            print("  %-40s %4d calls %8.1f us" % (f[:40], n, t / 1e3))
            covered += t
        print("  (time inside HIP calls %.1f us of %.1f; the rest is the caller's own code)" % (covered / 1e3, g / 1e3))
        print("  in order (start offset from the idle start, duration):")
        for s, e, f in calls:
            if e > e0 and s < s1:
                print("    %+9.1f  %8.1f  %s" % ((s - e0) / 1e3, (e - s) / 1e3, f))


if __name__ == "__main__":
    main()
