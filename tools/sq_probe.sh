#!/bin/bash
# SQ instruction-counter calibration: one rocprofv3 --pmc pass over
# tools/sq_probe (known instruction counts per wave).  Usage: bash tools/sq_probe.sh TAG
set -o pipefail
TAG=${1:-sqprobe}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 60 ./tools/sq_probe > gpurun_out/$TAG/known.json || exit $?
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d gpurun_out/$TAG/p1 -o run -- ./tools/sq_probe > gpurun_out/$TAG/p1.log 2>&1 || exit $?
cat gpurun_out/$TAG/known.json
find gpurun_out/$TAG/p1 -name "*counter_collection.csv" | head -1 | xargs -r cat | head -20
