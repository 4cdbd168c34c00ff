#!/bin/bash
# GPU tests at HEAD, then the odd-E deferral A/B (E = 3 and E = 12, 3 rounds)
# and the element-size / block-size modes at 4 GiB.  Each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=bitshuffle_amd/libbitshuffle_mi355x
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f_pytest.log 2>&1 && \
GENS=1 AB_ELEM=3 timeout -k 10 400 bash tools/ab_libs.sh r4f_e3 1 3 $L.so ${L}_nodef.so > gpurun_out/r4f_e3.txt 2>&1 && \
GENS=1 AB_ELEM=12 timeout -k 10 400 bash tools/ab_libs.sh r4f_e12 1 3 $L.so ${L}_nodef.so > gpurun_out/r4f_e12.txt 2>&1 && \
GIB=4 timeout -k 10 600 bash tools/bench_modes.sh r4f_modes > gpurun_out/r4f_modes.txt 2>&1
rc=$?
tail -3 gpurun_out/r4f_pytest.log
grep -v amdgpu.ids gpurun_out/r4f_e3.txt gpurun_out/r4f_e12.txt gpurun_out/r4f_modes.txt
exit $rc
