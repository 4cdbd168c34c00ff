#!/bin/bash
# Closing measurements without the counter passes: parity suite, rocprofv3
# kernel stats of bench.py, every config, the element-size / block-size modes.
set -o pipefail
TAG=${1:-cs}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err && \
bash tools/bench_all.sh ${TAG}_ball > gpurun_out/${TAG}_ball.txt 2>&1 && \
GIB=4 timeout -k 10 400 bash tools/bench_modes.sh ${TAG}_modes > gpurun_out/${TAG}_modes.txt 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
exit $rc
