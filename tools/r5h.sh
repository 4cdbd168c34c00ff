#!/bin/bash
# Round-5 call h: LDS bank-conflict attribution for k_lz4_encode -- one SQ
# pass each over 1 GiB of all-miss random int16 (search windows only), zeros
# (no search work) and config 2's G1, encode only.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/pmc.sh r5h_rand 1 tools/pmc_sets_lds.txt 8 enc && \
bash tools/pmc.sh r5h_zero 1 tools/pmc_sets_lds.txt 9 enc && \
bash tools/pmc.sh r5h_g1 1 tools/pmc_sets_lds.txt 1 enc && \
for t in rand zero g1; do python tools/pmc_summary.py gpurun_out/r5h_$t > gpurun_out/r5h_$t/summary.txt || exit 1; done
