# Fresh-process first-use check: N harness processes, each running the 42
# regression datasets PASSES times; prints which pass every failure was in.
set -o pipefail
N=${1:-10}; P=${2:-3}
export H5H_DUMP=1 H5H_PASSES=$P
mkdir -p gpurun_out
gcc -O2 -I/opt/conda/include tests/h5_harness.c -L/opt/conda/lib -lhdf5 -Wl,-rpath,/opt/conda/lib -o /tmp/h5h || exit 1
export HDF5_PLUGIN_PATH=$PWD/bitshuffle_amd
for i in $(seq $N); do
  timeout -k 10 60 /tmp/h5h regress tests/golden/regression /tmp/r.h5 > /tmp/h5o.txt 2>&1
  rc=$?
  [ $rc -ge 124 ] && { echo "run $i rc=$rc" >> gpurun_out/h5pass.log; exit 1; }
  [ $rc -ne 0 ] && grep -E "pass|mismatch|regress" /tmp/h5o.txt | sed "s/^/run $i: /" >> gpurun_out/h5pass.log
done
echo "done $N x $P" >> gpurun_out/h5pass.log
exit 0
