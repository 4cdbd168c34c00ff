#!/bin/bash
# Element-size / block-size modes of bench.py: default
# blocks for E = 2, 3, 12; 256 KiB blocks for E = 2.  Each step time-limited.
set -o pipefail
TAG=${1:-bm}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A="--no-cpu-baseline --gib ${GIB:-1} --steps ${STEPS:-3} --warmup 1"
timeout -k 10 300 python -u bench.py $A > gpurun_out/${TAG}_e2.json 2> gpurun_out/${TAG}_e2.err && \
timeout -k 10 300 python -u bench.py $A --elem-size 3 > gpurun_out/${TAG}_e3.json 2> gpurun_out/${TAG}_e3.err && \
timeout -k 10 300 python -u bench.py $A --elem-size 12 > gpurun_out/${TAG}_e12.json 2> gpurun_out/${TAG}_e12.err && \
timeout -k 10 600 python -u bench.py $A --block-size ${BIGBS:-131072} > gpurun_out/${TAG}_big.json 2> gpurun_out/${TAG}_big.err
rc=$?
for c in e2 e3 e12 big; do python3 -c "
import json,sys
try:
    d=json.load(open('gpurun_out/${TAG}_$c.json'))
    print('$c', d['value'], 'GiB/s', d['ms_per_step'], 'ms', d['kernels_avg_ms'])
except Exception as e: print('$c', 'n/a', e)
"; tail -1 gpurun_out/${TAG}_$c.err; done
exit $rc
