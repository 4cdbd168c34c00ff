"""HBM traffic per launch from rocprofv3 --pmc passes (tools/pmc.sh with
tools/pmc_traffic_sets.txt), corrected as /opt/skills/guides/MI355X_MICROARCH.md
prescribes for gfx950: FETCH_SIZE (KB) reads exactly 1/2 of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE (KB) is taken as is.
Writes profiles/pmc_traffic.json: {kernel: bytes per launch}, which bench.py
reports as roofline.traffic for the dominant kernel.
Usage: python tools/pmc_traffic.py gpurun_out/<tag> [out.json]"""
import collections
import csv
import glob
import json
import os
import re
import sys

d = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if not m:
            continue
        vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {"_method": "per launch: 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 bytes (gfx950 FETCH_SIZE "
                  "halving corrected); from rocprofv3 --pmc passes over tools/run_codec_once.py",
       "_source": d}
for k, c in vals.items():
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        res[k] = round(2 * f * 1024 + w * 1024)
        res[k + "_raw_KB"] = {"FETCH_SIZE": f, "WRITE_SIZE": w}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
