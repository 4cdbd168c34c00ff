#!/bin/bash
# Quick GPU iteration: parity tests (optionally -k filter), A/B of encoder
# variants, one bench line.  Each GPU step has its own time limit; steps are
# chained with && so a failure stops the call.
set -o pipefail
TAG=${1:-it}
K=${2:-}
AB=${3:-0,2}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider "${KARG[@]}" > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/ab.py $AB 2 1 3 > gpurun_out/${TAG}_ab.log 2>&1 && \
timeout -k 10 300 python -u tools/ab.py $AB 2 2 2 > gpurun_out/${TAG}_ab_g2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
tail -4 gpurun_out/${TAG}_pytest.log
cat gpurun_out/${TAG}_ab.log gpurun_out/${TAG}_ab_g2.log gpurun_out/${TAG}_bench.json 2>/dev/null
exit $rc
