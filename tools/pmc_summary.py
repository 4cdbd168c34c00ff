"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        import re
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
for k, v in acc.items():
    if not any(x in k for x in ("encode", "decode", "idx", "compact", "scan")):
        continue
    print("==", k, "dispatches", len(disp[k]))
    for c in sorted(v):
        print("   %-24s %16.4g" % (c, v[c]))
