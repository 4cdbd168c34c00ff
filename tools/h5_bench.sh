#!/bin/bash
# BASELINE config 5 end to end (host memory, PCIe included, never the
# headline): 8 GiB uint16 written and read back through the HDF5 plugin by
# tests/h5_harness.c, plus the drop-in host C-ABI at 4 GiB and at one 32 MiB
# chunk.  Output: gpurun_out/${TAG}_h5.json, gpurun_out/${TAG}_host*.json
set -o pipefail
TAG=${1:-h5}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
H=/opt/conda
gcc -O2 -I$H/include tests/h5_harness.c -L$H/lib -lhdf5 -Wl,-rpath,$H/lib -o /tmp/h5_harness_bench && \
BSHUF_H5_TIMING=1 BSHUF_H5_IO_FLOOR=1 HDF5_PLUGIN_PATH=$PWD/bitshuffle_amd timeout -k 10 600 /tmp/h5_harness_bench roundtrip /tmp/cfg5_bench.h5 4294967296 16777216 > gpurun_out/${TAG}_h5.json 2> gpurun_out/${TAG}_h5.err && \
timeout -k 10 300 python tools/host_bench.py 4 3 > gpurun_out/${TAG}_host4g.json && BSHUF_HOST_STAGING=0 timeout -k 10 300 python tools/host_bench.py 4 3 > gpurun_out/${TAG}_host4g_direct.json && \
timeout -k 10 300 python tools/host_bench.py 0.03125 20 > gpurun_out/${TAG}_host32m.json
rc=$?
rm -f /tmp/cfg5_bench.h5
cat gpurun_out/${TAG}_h5.err gpurun_out/${TAG}_h5.json gpurun_out/${TAG}_host4g.json gpurun_out/${TAG}_host32m.json 2>/dev/null
exit $rc
