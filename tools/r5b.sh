#!/bin/bash
# Round-5 A/B call: search_entry encoder variants + decoder batch-loop library A/B.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/gpu_step.sh r5b \
 "300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k 'variant or lz4_matches or golden or regression or corrupt or device or batch'" \
 "200:python -u tools/ab.py 319488,450560 2 1 3" \
 "200:python -u tools/ab.py 319488,450560 1 2 3" \
 "200:AB_ELEM=3 python -u tools/ab.py 40960,172032 1 1 3" \
 "200:AB_ELEM=12 python -u tools/ab.py 40960,172032 1 1 3" \
 "400:GENS='1 2' bash tools/ab_libs.sh r5b_dec 2 2 bitshuffle_amd/libbitshuffle_mi355x_base.so bitshuffle_amd/libbitshuffle_mi355x.so"
