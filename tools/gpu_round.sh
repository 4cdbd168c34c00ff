#!/bin/bash
# One GPU round: parity tests, bench, rocprofv3 kernel stats.  Each GPU step
# has its own time limit; steps are chained with && so a failure stops it.
set -o pipefail
TAG=${1:-r}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
cat gpurun_out/${TAG}_bench.json 2>/dev/null
exit $rc
