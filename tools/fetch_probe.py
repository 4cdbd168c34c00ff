"""Summarise the FETCH_SIZE / WRITE_SIZE calibration (tools/fetch_probe.hip).
Usage: python tools/fetch_probe.py gpurun_out/<tag> known.json [out.json]
<tag>/p1 holds the FETCH_SIZE pass, <tag>/p2 the WRITE_SIZE pass (rocprofv3
csv).  Prints, per probe kernel, counter bytes / known bytes: the factor a
counter must be multiplied by to read the bytes that kernel moved."""
import collections
import csv
import glob
import json
import os
import re
import sys

d, known_f = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else None
known = json.load(open(known_f))
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if m:
            vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {"_method": "FETCH_SIZE / WRITE_SIZE (KB x 1024) of each probe launch over its known "
                  "bytes (1 GiB streams, past the 256 MiB Infinity Cache); read kernels also "
                  "store a 4 MiB sink, subtracted from their WRITE_SIZE",
       "_source": d}
for k, c in sorted(vals.items()):
    if k not in known:
        continue
    fs = c.get("FETCH_SIZE", [])
    ws = c.get("WRITE_SIZE", [])
    f = fs[-1] * 1024 if fs else None  # last launch (k_wr16 runs twice: first is the flush)
    w = ws[-1] * 1024 if ws else None
    row = {"known_bytes": known[k], "FETCH_bytes": f, "WRITE_bytes": w}
    if k.startswith("k_rd"):
        row["fetch_over_known"] = round(f / known[k], 4) if f else None
        row["correction"] = round(known[k] / f, 4) if f else None
    else:
        row["write_over_known"] = round(w / known[k], 4) if w else None
        row["fetch_over_known"] = round(f / known[k], 4) if f is not None else None
    res[k] = row
if out:
    json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
