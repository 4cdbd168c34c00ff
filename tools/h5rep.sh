# Repeat the HDF5 regression harness N times with the current plugin and
# (if present) tools/oldlib, counting failures.  Usage: bash tools/h5rep.sh N
set -o pipefail
N=${1:-10}
export H5H_DUMP=1
mkdir -p gpurun_out
gcc -O2 -I/opt/conda/include tests/h5_harness.c -L/opt/conda/lib -lhdf5 -Wl,-rpath,/opt/conda/lib -o /tmp/h5h || exit 1
for lib in bitshuffle_amd tools/oldlib; do
  [ -d $lib ] || continue
  bad=0
  for i in $(seq $N); do
    HDF5_PLUGIN_PATH=$PWD/$lib timeout -k 10 60 /tmp/h5h regress tests/golden/regression /tmp/r.h5 > /tmp/h5o.txt 2>&1
    rc=$?
    [ $rc -ge 124 ] && { echo "$lib run $i rc=$rc" >> gpurun_out/h5rep.log; exit 1; }
    [ $rc -ne 0 ] && { bad=$((bad+1)); cat /tmp/h5o.txt >> gpurun_out/h5rep.log; }
  done
  echo "$lib: $bad of $N runs failed" >> gpurun_out/h5rep.log
done
exit 0
