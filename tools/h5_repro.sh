#!/bin/bash
# HDF5 stale-result experiment: N fresh h5_harness processes
# per host transport mode, each writing and reading the reference's 42 LZ4
# regression datasets through the plugin P times (HDF5 hands the filter fresh
# malloc'ed chunk buffers on every call).  Counts processes with a wrong byte.
# Usage: bash tools/h5_repro.sh N P "mode ..."
set -o pipefail
N=${1:-20}; P=${2:-3}; MODES=${3:-"kernel dma dma_staged"}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
gcc -O2 -I/opt/conda/include tests/h5_harness.c -L/opt/conda/lib -lhdf5 -Wl,-rpath,/opt/conda/lib \
    -o /tmp/h5h || exit 1
# the transport / pool switches exist in the DIAGNOSTIC library only (make -C
# bitshuffle_amd diag): the plugin (rpath $ORIGIN) is run beside a copy of it
if [ -z "$PLUGIN_DIR" ]; then
  PLUGIN_DIR=/tmp/h5diag_plugin; mkdir -p $PLUGIN_DIR
  cp bitshuffle_amd/libh5bshuf_mi355x.so $PLUGIN_DIR/ &&
  cp bitshuffle_amd/libbitshuffle_mi355x_diag.so $PLUGIN_DIR/libbitshuffle_mi355x.so || exit 1
fi
export HDF5_PLUGIN_PATH=$PLUGIN_DIR H5H_DUMP=1 H5H_PASSES=$P
out=gpurun_out/h5_repro.log
for mode in $MODES; do
  # mode = transport[+allocws][+defaultpool]: the round-2 per-call
  # stream-ordered workspace, and the device's default (trimming) pool for it
  export BSHUF_HOST_XFER=${mode%%+*}
  unset BSHUF_DIAG_WS BSHUF_DIAG_POOL
  case $mode in *+allocws*) export BSHUF_DIAG_WS=alloc;; esac
  case $mode in *+defaultpool*) export BSHUF_DIAG_POOL=default;; esac
  bad=0
  for i in $(seq $N); do
    timeout -k 10 120 /tmp/h5h regress tests/golden/regression /tmp/r_x.h5 > /tmp/h5o.txt 2>&1
    rc=$?
    [ $rc -ge 124 ] && { echo "mode=$mode run $i rc=$rc: stopping" >> $out; exit 1; }
    if [ $rc -ne 0 ]; then bad=$((bad+1)); sed "s/^/$mode run $i: /" /tmp/h5o.txt | tail -20 >> $out; fi
  done
  echo "SUMMARY mode=$mode: $bad of $N processes wrong ($P passes x 42 datasets each)" | tee -a $out
done
exit 0
