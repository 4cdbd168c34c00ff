#!/bin/bash
# Round-5 call j: paired short wave matches in the decoder -- parity of the
# new library, then library A/B against the closing build (r5base), then the
# LDS conflict attribution passes (r5h.sh).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/gpu_step.sh r5j \
 "300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider" \
 "400:bash tools/ab_libs.sh r5j 1 2 bitshuffle_amd/libbitshuffle_mi355x_r5base.so bitshuffle_amd/libbitshuffle_mi355x.so" \
 "300:AB_ELEM=3 GENS=1 bash tools/ab_libs.sh r5j_e3 1 2 bitshuffle_amd/libbitshuffle_mi355x_r5base.so bitshuffle_amd/libbitshuffle_mi355x.so" \
 "300:bash tools/r5h.sh"
