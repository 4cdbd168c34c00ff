#!/bin/bash
# Runs GPU steps in order, each under its own time limit; a step that ends
# with a test failure (rc 1) does not stop the next one, anything else (a
# fault, abort, time limit: rc >= 2) does.  Usage:
#   bash tools/gpu_step.sh TAG 'cmd1' 'cmd2' ...   (each cmd: "SECONDS:command")
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1))
  lim=${spec%%:*}; cmd=${spec#*:}
  echo "== step $i ($lim s): $cmd" | tee -a gpurun_out/${TAG}_steps.txt
  timeout -k 10 $lim bash -c "$cmd" > gpurun_out/${TAG}_s$i.log 2>&1
  rc=$?
  echo "== step $i rc=$rc" | tee -a gpurun_out/${TAG}_steps.txt
  tail -4 gpurun_out/${TAG}_s$i.log
  if [ $rc -ge 2 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
