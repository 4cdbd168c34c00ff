#!/bin/bash
# A/B of whole library builds: ROUNDS x (each lib in its own fresh process),
# G1 and G2 (GENS="1 2"; AB_ELEM=E reads them as E-byte elements).
# Usage: bash tools/ab_libs.sh TAG GiB ROUNDS lib1.so lib2.so ...
set -o pipefail
TAG=$1; GIB=$2; ROUNDS=$3; shift 3
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/${TAG}_ab.jsonl
: > $out
for r in $(seq $ROUNDS); do
  for gen in ${GENS:-1 2}; do
    for L in "$@"; do
      BSHUF_LIB=$PWD/$L timeout -k 10 200 python -u tools/ab_one.py $GIB $gen 3 | sed "s/^/{\"gen\": $gen, \"r\": $r, \"d\": /; s/$/}/" >> $out || exit 1
    done
  done
done
python3 - "$out" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
shas = collections.defaultdict(set)
for r in rows:
    d = r["d"]
    shas[(r["gen"])].add(d["sha"])
    for k, v in d.items():
        if k not in ("sha", "lib"):
            agg[(r["gen"], d["lib"], k)].append(v)
for (g, lib, k), v in sorted(agg.items()):
    if k in ("k_lz4_encode", "k_lz4_decode", "k_seq_scan", "k_compact", "k_emit",
             "k_seq_scan_big", "k_lz4_exec_big", "k_lz4_encode_big"):
        print("gen %d %-12s %-14s %8.3f ms  %s" % (g, lib, k, sum(v) / len(v), " ".join("%.3f" % x for x in v)))
for g, s in shas.items():
    print("gen %d stream digests %s" % (g, "IDENTICAL" if len(s) == 1 else "DIFFER: %s" % s))
PY
