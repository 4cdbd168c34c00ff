#!/bin/bash
# BASELINE config 5 end to end (host memory, PCIe included, never the
# headline): 8 GiB uint16 written and read back through an HDF5 plugin by
# tests/h5_harness.c, three times on the same box:
#   ours  -- bitshuffle_amd/libh5bshuf_mi355x.so (this codec on the GPU)
#   ref   -- oracle/_ref/plugin/libh5bshuf_ref.so (the reference's own plugin,
#            AVX2 + OpenMP on the job's CPU share)
#   null  -- tools/h5_null_filter.c (pass-through: HDF5's filtered-I/O floor)
# plus the host C-ABI at 4 GiB and at one 32 MiB chunk.
# Output: gpurun_out/${TAG}_h5_{ours,ref,null}.json, gpurun_out/${TAG}_host*.json
set -o pipefail
TAG=${1:-h5}
N=${N:-4294967296}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out /tmp/h5null
H=/opt/conda
gcc -O2 -I$H/include tests/h5_harness.c -L$H/lib -lhdf5 -Wl,-rpath,$H/lib -o /tmp/h5_harness_bench && \
gcc -O2 -shared -fPIC -I$H/include tools/h5_null_filter.c -o /tmp/h5null/libh5null.so && \
BSHUF_H5_TIMING=1 BSHUF_H5_IO_FLOOR=1 HDF5_PLUGIN_PATH=$PWD/bitshuffle_amd timeout -k 10 600 \
  /tmp/h5_harness_bench roundtrip /tmp/cfg5_bench.h5 $N 16777216 > gpurun_out/${TAG}_h5_ours.json 2> gpurun_out/${TAG}_h5_ours.err && \
HDF5_PLUGIN_PATH=$PWD/oracle/_ref/plugin OMP_NUM_THREADS=${OMP_NUM_THREADS:-16} timeout -k 10 900 \
  /tmp/h5_harness_bench roundtrip /tmp/cfg5_bench.h5 $N 16777216 > gpurun_out/${TAG}_h5_ref.json 2> gpurun_out/${TAG}_h5_ref.err && \
HDF5_PLUGIN_PATH=/tmp/h5null timeout -k 10 600 \
  /tmp/h5_harness_bench roundtrip /tmp/cfg5_bench.h5 $N 16777216 > gpurun_out/${TAG}_h5_null.json 2> gpurun_out/${TAG}_h5_null.err && \
timeout -k 10 300 python tools/host_bench.py 4 3 > gpurun_out/${TAG}_host4g.json && \
timeout -k 10 300 python tools/host_bench.py 0.03125 20 > gpurun_out/${TAG}_host32m.json
rc=$?
rm -f /tmp/cfg5_bench.h5 /tmp/cfg5_bench.h5.raw
for f in ours ref null; do echo "== $f"; cat gpurun_out/${TAG}_h5_$f.json 2>/dev/null; tail -3 gpurun_out/${TAG}_h5_$f.err 2>/dev/null; done
cat gpurun_out/${TAG}_host4g.json gpurun_out/${TAG}_host32m.json 2>/dev/null
exit $rc
