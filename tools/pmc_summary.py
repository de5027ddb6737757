#!/usr/bin/env python
"""Sum each counter per kernel (short name) from a rocprofv3 counter_collection.csv."""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import short_name  # noqa: E402

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    n = short_name(r["Kernel_Name"])
    if not n.startswith("k_"):
        continue
    tot[n][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[n].add(r["Dispatch_Id"])
for n in sorted(tot):
    print(n, len(disp[n]), " ".join("%s=%.4g" % kv for kv in sorted(tot[n].items())))
