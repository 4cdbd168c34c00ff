# Repeat the HDF5 regression harness N times with the current plugin, with the
# default host staging and with BSHUF_HOST_STAGING=0, counting failures.
# Usage: bash tools/h5rep.sh N
set -o pipefail
N=${1:-10}
export H5H_DUMP=1
mkdir -p gpurun_out
gcc -O2 -I/opt/conda/include tests/h5_harness.c -L/opt/conda/lib -lhdf5 -Wl,-rpath,/opt/conda/lib -o /tmp/h5h || exit 1
export HDF5_PLUGIN_PATH=$PWD/bitshuffle_amd
for stage in default 0; do
  bad=0
  for i in $(seq $N); do
    if [ $stage = default ]; then unset BSHUF_HOST_STAGING; else export BSHUF_HOST_STAGING=$stage; fi
    timeout -k 10 60 /tmp/h5h regress tests/golden/regression /tmp/r.h5 > /tmp/h5o.txt 2>&1
    rc=$?
    [ $rc -ge 124 ] && { echo "staging=$stage run $i rc=$rc" >> gpurun_out/h5rep.log; exit 1; }
    [ $rc -ne 0 ] && { bad=$((bad+1)); cat /tmp/h5o.txt >> gpurun_out/h5rep.log; }
  done
  echo "staging=$stage: $bad of $N runs failed" >> gpurun_out/h5rep.log
done
exit 0
