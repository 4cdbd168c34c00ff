#!/bin/bash
# GPU run for the host-path work: the -m gpu suite (optionally -k filter), then
# the stale-result experiment over transport modes.  The experiment runs only
# when the suite ended normally (passed, or failed without a fault/timeout).
set -o pipefail
TAG=${1:-h}
K=${2:-}
MODES=${3:-"kernel dma dma_fenced"}
PROCS=${4:-10}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider "${KARG[@]}" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
[ "$MODES" = "none" ] && exit $rc
timeout -k 10 900 python -u tools/stale_repro.py --procs $PROCS --passes 3 $MODES \
    > gpurun_out/${TAG}_repro.log 2>&1
rc2=$?
grep SUMMARY gpurun_out/${TAG}_repro.log
exit $(( rc > rc2 ? rc : rc2 ))
