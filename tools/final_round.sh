#!/bin/bash
# The round's closing measurements at HEAD, one GPU call: parity suite,
# rocprofv3 kernel stats of bench.py, SQ counter passes (G1 and G2, 2 GiB),
# FETCH_SIZE / WRITE_SIZE passes (4 GiB G1) for profiles/pmc_traffic.json, and
# every config through bench.py.  Each GPU step has its own time limit; steps
# are chained with &&.  Usage: bash tools/final_round.sh TAG
set -o pipefail
TAG=${1:-fin}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err && \
bash tools/pmc.sh ${TAG}_sq_g1 2 tools/pmc_sets_sq.txt 1 && \
bash tools/pmc.sh ${TAG}_sq_g2 2 tools/pmc_sets_sq.txt 2 && \
bash tools/pmc.sh ${TAG}_traffic 4 tools/pmc_traffic_sets.txt 1 && \
python tools/pmc_summary.py gpurun_out/${TAG}_sq_g1 > gpurun_out/${TAG}_sq_g1/summary.txt && \
python tools/pmc_summary.py gpurun_out/${TAG}_sq_g2 > gpurun_out/${TAG}_sq_g2/summary.txt && \
python tools/pmc_traffic.py gpurun_out/${TAG}_traffic gpurun_out/${TAG}_pmc_traffic.json && \
bash tools/bench_all.sh ${TAG}_ball > gpurun_out/${TAG}_ball.txt 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
exit $rc
