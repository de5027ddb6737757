"""Copy one round's evidence from gpurun_out/ into profiles/ under the round's names.

    python tools/collect_evidence.py TAG ROUND [SESSION]      (e.g. v55 r04 ev14)

Reads what tools/evidence.sh left in gpurun_out/evidence_TAG/ (bench lines,
kernel stats, VALU summaries) and gpurun_out/{prof,valu}_TAG_<wl>/ (PMC
summaries), including the FFT-mode runs of tools/profile_c2.sh / tools/pmc_valu.sh under the tag
TAG_c2fft plus the bench line of that session (gpurun_out/SESSION/c2fft.json)."""
from __future__ import annotations

import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json_line(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit("no JSON line in %s" % path)


def main():
    tag = sys.argv[1]
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r04"
    prof = os.path.join(REPO, "profiles")
    ev = os.path.join(REPO, "gpurun_out", "evidence_" + tag)
    copied = []
    for f in sorted(glob.glob(os.path.join(ev, "*.json"))):
        wl = os.path.basename(f)[:-5]
        d = last_json_line(f)
        dst = os.path.join(prof, "%s_bench_%s_%s.json" % (rnd, wl, tag))
        open(dst, "w").write(json.dumps(d) + "\n")
        copied.append((dst, d["ms_per_step"]))
    for f in sorted(glob.glob(os.path.join(ev, "kernel_stats_*.csv"))):
        wl = os.path.basename(f)[len("kernel_stats_"):-4]
        shutil.copy(f, os.path.join(prof, "%s_%s_kernel_stats_%s.csv" % (rnd, wl, tag)))
    for f in sorted(glob.glob(os.path.join(ev, "pmc_valu_summary_*.txt"))):
        wl = os.path.basename(f)[len("pmc_valu_summary_"):-4]
        shutil.copy(f, os.path.join(prof, "%s_%s_pmc_valu_summary_%s.txt" % (rnd, wl, tag)))
    # the PMC summaries (evidence.sh copies them into profiles/ on the box,
    # but only gpurun_out/ comes back) and the FFT mode's kernel stats
    for d in sorted(glob.glob(os.path.join(REPO, "gpurun_out", "prof_%s_*" % tag))):
        wl = os.path.basename(d)[len("prof_%s_" % tag):]
        shutil.copy(os.path.join(d, "pmc_traffic.json"), os.path.join(prof, "%s_%s_pmc_traffic_%s.json" % (rnd, wl, tag)))
        if wl == "c2fft":
            shutil.copy(os.path.join(d, "kernel_stats.csv"), os.path.join(prof, "%s_c2fft_kernel_stats_%s.csv" % (rnd, tag)))
    for d in sorted(glob.glob(os.path.join(REPO, "gpurun_out", "valu_%s_*" % tag))):
        wl = os.path.basename(d)[len("valu_%s_" % tag):]
        shutil.copy(os.path.join(d, "pmc_valu.json"), os.path.join(prof, "%s_%s_pmc_valu_%s.json" % (rnd, wl, tag)))
        if wl == "c2fft":
            shutil.copy(os.path.join(d, "summary.txt"), os.path.join(prof, "%s_c2fft_pmc_valu_summary_%s.txt" % (rnd, tag)))
    if len(sys.argv) > 3:
        d = last_json_line(os.path.join(REPO, "gpurun_out", sys.argv[3], "c2fft.json"))
        dst = os.path.join(prof, "%s_bench_c2fft_%s.json" % (rnd, tag))
        open(dst, "w").write(json.dumps(d) + "\n")
        copied.append((dst, d["ms_per_step"]))
    for dst, ms in copied:
        print("%-60s %8.3f ms" % (os.path.relpath(dst, REPO), ms))


if __name__ == "__main__":
    main()
