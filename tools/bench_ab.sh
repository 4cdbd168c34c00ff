#!/bin/bash
# Whole-step A/B of library builds through bench.py (config 2 unless
# BENCH_ARGS says otherwise), alternating libraries ROUNDS times, each run in a
# fresh process.  Usage: bash tools/bench_ab.sh TAG ROUNDS lib1.so lib2.so ...
TAG=$1; ROUNDS=$2; shift 2
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/${TAG}_bench_ab.jsonl
: > $out
for r in $(seq $ROUNDS); do
  for L in "$@"; do
    BSHUF_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_tmp.json || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_tmp.json')); print(json.dumps({'lib': sys.argv[1], 'r': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernels': d.get('kernels_ms_per_step'), 'parity': d['parity']['kind']}))" $(basename $L) >> $out
  done
done
cat $out
