#!/bin/bash
# Every BASELINE config through bench.py on one GPU (each step time-limited,
# chained with &&).  Config 1 twice: its 64 MiB BASELINE size (Infinity-Cache
# resident across steps) and a 4 GiB ramp that streams from HBM.
# Usage: bash tools/bench_all.sh TAG
set -o pipefail
TAG=${1:-ball}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_cfg2.json 2> gpurun_out/${TAG}_cfg2.err && \
timeout -k 10 300 python -u bench.py --config 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_cfg1.json 2> gpurun_out/${TAG}_cfg1.err && \
timeout -k 10 300 python -u bench.py --config 1 --gib 4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_cfg1hbm.json 2> gpurun_out/${TAG}_cfg1hbm.err && \
timeout -k 10 500 python -u bench.py --config 3 --steps 3 --warmup 1 > gpurun_out/${TAG}_cfg3.json 2> gpurun_out/${TAG}_cfg3.err && \
timeout -k 10 400 python -u bench.py --config 4 > gpurun_out/${TAG}_cfg4.json 2> gpurun_out/${TAG}_cfg4.err
rc=$?
for c in 2 1 1hbm 3 4; do cat gpurun_out/${TAG}_cfg$c.json 2>/dev/null; tail -2 gpurun_out/${TAG}_cfg$c.err 2>/dev/null; done
exit $rc
