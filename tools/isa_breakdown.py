"""Per-category instruction counts of one kernel in the gfx950 assembly
(`make -C iterative_cleaner_amd/csrc asm` -> ic_kernels.s).

    python tools/isa_breakdown.py KERNEL_SUBSTRING [--asm PATH] [--blocks]

Counts are static (instructions in the text).  For the straight-line parts of
a persistent kernel (k_diag_p2's per-profile body) the static count of the
blocks one profile runs is its dynamic count; --blocks prints every basic block
with its counts so those blocks can be picked out, and --path L1,L2,... sums
the listed blocks (by label suffix) as one profile's path."""
from __future__ import annotations

import argparse
import collections
import re
import sys

CATS = [
    ("lds", re.compile(r"^ds_")),
    ("vmem", re.compile(r"^(global_|buffer_|flat_|scratch_)")),
    ("smem", re.compile(r"^s_(load|buffer_load|store|dcache)")),
    ("salu", re.compile(r"^s_")),
    ("dpp/lane", re.compile(r"(_dpp\b|^v_readlane|^v_readfirstlane|^v_writelane|^v_permlane|^v_mov_b64_dpp)")),
    ("cvt", re.compile(r"^v_cvt_")),
    ("f64 add", re.compile(r"^v_add_f64")),
    ("f64 mul", re.compile(r"^v_mul_f64")),
    ("f64 fma", re.compile(r"^v_fmac?_f64")),
    ("f64 other", re.compile(r"^v_\w+_f64")),
    ("f32 packed", re.compile(r"^v_pk_\w+_f32")),
    ("f32", re.compile(r"^v_\w+_f32")),
    ("cmp/cndmask", re.compile(r"^v_(cmp|cndmask)")),
    ("mov", re.compile(r"^v_mov_")),
    ("int/addr", re.compile(r"^v_")),
]


def cat_of(op: str, line: str) -> str:
    if "row_" in line or "quad_perm" in line or "row_mirror" in line or "row_half_mirror" in line:
        if op.startswith("v_"):
            return "dpp/lane"
    for name, rx in CATS:
        if rx.search(op):
            return name
    return "other"


def parse(asm: str, kernel: str):
    lines = asm.splitlines()
    start = None
    for i, l in enumerate(lines):
        if l.startswith("_Z") and l.split(":")[0].find(kernel) >= 0 and l.rstrip().endswith(
                (":", "E")) or (l.startswith("_Z") and kernel in l.split(":")[0] and ":" in l):
            start = i
            break
    if start is None:
        sys.exit("kernel %r not found" % kernel)
    name = lines[start].split(":")[0]
    blocks = collections.OrderedDict()
    cur = "entry"
    blocks[cur] = collections.Counter()
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB\w+):", s)
            if m:
                cur = m.group(1)
                blocks[cur] = collections.Counter()
            continue
        m = re.match(r"^([a-z_0-9]+)", s)
        if not m:
            continue
        op = m.group(1)
        if op in ("s_waitcnt", "s_nop", "s_setprio", "s_barrier", "s_sleep") or op.startswith("s_waitcnt"):
            blocks[cur]["(wait/nop/barrier)"] += 1
            continue
        blocks[cur][cat_of(op, s)] += 1
    return name, blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--asm", default="iterative_cleaner_amd/csrc/ic_kernels.s")
    ap.add_argument("--blocks", action="store_true")
    ap.add_argument("--path", default="", help="comma-separated block label suffixes to sum")
    a = ap.parse_args()
    name, blocks = parse(open(a.asm).read(), a.kernel)
    print(name)
    order = [c for c, _ in CATS] + ["other", "(wait/nop/barrier)"]
    if a.blocks:
        for lab, c in blocks.items():
            vt = sum(v for k, v in c.items() if k.startswith(("f", "cvt", "cmp", "mov", "int", "dpp")))
            print("%-16s valu=%4d  %s" % (lab, vt, " ".join("%s=%d" % (k, c[k]) for k in order if c[k])))
    sel = blocks.values()
    if a.path:
        want = a.path.split(",")
        sel = [c for lab, c in blocks.items() if any(lab.endswith("_" + w) or lab == w for w in want)]
    tot = collections.Counter()
    for c in sel:
        tot.update(c)
    valu = sum(tot[k] for k in order if k not in ("lds", "vmem", "smem", "salu", "other", "(wait/nop/barrier)"))
    print("VALU total %d" % valu)
    for k in order:
        if tot[k]:
            print("  %-20s %5d" % (k, tot[k]))


if __name__ == "__main__":
    main()
