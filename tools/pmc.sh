#!/bin/bash
# PMC passes over one codec run (each rocprofv3 call: --pmc + --kernel-trace
# only, one counter set per pass, each under its own time limit).
# Usage: bash tools/pmc.sh TAG [GiB] [sets file] [gen] [enc|dec|both]
set -o pipefail
TAG=${1:-pmc}; GIB=${2:-1}; SETS=${3:-tools/pmc_sets.txt}; GEN=${4:-1}; WHAT=${5:-both}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d gpurun_out/$TAG/p$i -o run -- python tools/run_codec_once.py $GIB $WHAT $GEN > gpurun_out/$TAG/p$i.log 2>&1 || exit $?
done < "$SETS"
