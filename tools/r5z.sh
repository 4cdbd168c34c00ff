#!/bin/bash
# Round-5 last call: the driver's round-end tiers on the final tree -- the full
# -m gpu suite, smoke(), the default bench line and its rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5z_pytest.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5z_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5z_bench.json 2> gpurun_out/r5z_bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5z_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5z_prof_bench.json 2> gpurun_out/r5z_prof.err
rc=$?
tail -2 gpurun_out/r5z_pytest.log; tail -1 gpurun_out/r5z_smoke.log; cat gpurun_out/r5z_bench.json
exit $rc
