#!/bin/bash
# Round-4 A/B set: GPU tests, then E = 3, G1 E = 2 and 256 KiB-block library A/Bs
# (token-scan two-level loop, odd-E deferred copy-out / staged-transpose gathers,
# odd-E decoder occupancy).  Each step time-limited, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=bitshuffle_amd/libbitshuffle_mi355x
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4e_pytest.log 2>&1 && \
GENS=1 AB_ELEM=3 timeout -k 10 600 bash tools/ab_libs.sh r4e_e3 1 2 $L.so ${L}_s4.so ${L}_s5.so ${L}_unr.so ${L}_nodef.so ${L}_w5.so > gpurun_out/r4e_e3.txt 2>&1 && \
GENS=1 timeout -k 10 400 bash tools/ab_libs.sh r4e_g1 1 2 $L.so ${L}_s4.so ${L}_s5.so ${L}_unr.so > gpurun_out/r4e_g1.txt 2>&1 && \
GENS=1 AB_BS=131072 timeout -k 10 400 bash tools/ab_libs.sh r4e_big 1 2 $L.so ${L}_unr.so > gpurun_out/r4e_big.txt 2>&1
rc=$?
tail -3 gpurun_out/r4e_pytest.log
cat gpurun_out/r4e_e3.txt gpurun_out/r4e_g1.txt gpurun_out/r4e_big.txt 2>/dev/null
exit $rc
