#!/bin/bash
# The round's profiles at HEAD: rocprofv3 kernel stats of bench.py (the
# program directly after --), then PMC passes (SQ instruction/wait counters,
# FETCH_SIZE, WRITE_SIZE) over the config-2 data (4 GiB int16 G1, the bench's
# seed) and over 4 GiB of config 3's float32 G2.  Every GPU step has its own
# time limit; steps are chained with &&.  Usage: bash tools/prof_round.sh TAG
set -o pipefail
TAG=${1:-r}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err && \
bash tools/pmc.sh ${TAG}_pmc_g1 4 tools/pmc_sets.txt 1 && \
bash tools/pmc.sh ${TAG}_pmc_g2 4 tools/pmc_sets.txt 2
rc=$?
cat gpurun_out/${TAG}_prof_bench.json 2>/dev/null
exit $rc
