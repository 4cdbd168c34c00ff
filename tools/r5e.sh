#!/bin/bash
# Round-5 call e: segmented match batches in the decoder (bshuf_set_variant
# bit 1 << 22) -- parity, A/B, phase split.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/gpu_step.sh r5e \
 "300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k 'crafted or (alternate and 4194304)'" \
 "200:python -u tools/ab.py 0,4194304 2 1 3" \
 "200:python -u tools/ab.py 0,4194304 1 2 3" \
 "200:AB_ELEM=3 python -u tools/ab.py 0,4194304 1 1 3" \
 "200:AB_ELEM=12 python -u tools/ab.py 0,4194304 1 1 3" \
 "200:python -u tools/diag_decode.py 1 1 4194304" \
 "200:python -u tools/diag_decode.py 1 2 4194304"
