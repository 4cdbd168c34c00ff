#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (one counter set per rocprofv3
# run, each under its own time limit).  Usage: bash tools/fetch_probe.sh TAG
set -o pipefail
TAG=${1:-fprobe}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 120 ./tools/fetch_probe > gpurun_out/$TAG/known.json || exit $?
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/$TAG/p$i -o run -- ./tools/fetch_probe > gpurun_out/$TAG/p$i.log 2>&1 || exit $?
done
python3 tools/fetch_probe.py gpurun_out/$TAG gpurun_out/$TAG/known.json gpurun_out/$TAG/calibration.json
