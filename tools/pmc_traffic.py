"""HBM traffic per launch from rocprofv3 --pmc passes (tools/pmc.sh with
tools/pmc_traffic_sets.txt).  FETCH_SIZE (KB) is corrected per access shape
with the factors measured by tools/fetch_probe.hip on gfx950
(profiles/r03/fetch_probe/calibration.json): coalesced 4/8/16-byte-per-lane
loads and 16-byte loads of unaligned records all read 1/2 of their bytes
(x2, the guide's rule); k_seq_scan's lane-divergent 32-byte window loads
read 1/1.63 (x1.63).  WRITE_SIZE (KB) is taken as is (exact for coalesced and
64-byte-per-lane stores; lane-divergent 16-byte stores, k_seq_scan's token
positions, count ~3.4x their bytes).
Writes profiles/pmc_traffic.json: {kernel: bytes per launch}, which bench.py
reports as roofline.traffic for the dominant kernel.
Usage: python tools/pmc_traffic.py gpurun_out/<tag> [out.json] [GiB gen elem_size block_size]
The workload (default: 4 GiB G1, element size 2, default blocks -- config 2)
is recorded as "_workload"; bench.py attaches the traffic only to a line of
that same workload."""
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
# FETCH_SIZE correction per kernel (access shape), from the probe calibration
FETCH_CORR = {"k_seq_scan": 1.6295}
res = {"_method": "per launch: c*FETCH_SIZE*1024 + WRITE_SIZE*1024 bytes, c = 2 for coalesced "
                  "and record loads, 1.63 for k_seq_scan's lane-divergent 32-B windows (measured: "
                  "profiles/r03/fetch_probe/calibration.json); from rocprofv3 --pmc passes over "
                  "tools/run_codec_once.py",
       "_source": d}
wl = sys.argv[3:7] if len(sys.argv) > 6 else ["4", "1", "2", "0"]
res["_workload"] = {"gen": int(wl[1]), "bytes_per_call": int(float(wl[0]) * (1 << 30)),
                    "elem_size": int(wl[2]), "block_size": int(wl[3]),
                    "what": "tools/run_codec_once.py %s both %s (elem_size %s, block_size %s)" % (
                        wl[0], wl[1], wl[2], wl[3])}
for k, c in vals.items():
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        res[k] = round(FETCH_CORR.get(k, 2.0) * f * 1024 + w * 1024)
        res[k + "_raw_KB"] = {"FETCH_SIZE": f, "WRITE_SIZE": w}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
