#!/bin/bash
# Round-5 call d: the fused parse loop (parse_chain) and the emission's literal
# runs (lane_runs) -- parity, then A/B.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/gpu_step.sh r5d \
 "200:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k 'variant and (696320 or 974848 or 2793472 or 3072000)'" \
 "200:python -u tools/ab.py 450560,974848,3072000 2 1 3" \
 "200:python -u tools/ab.py 450560,974848,3072000 1 2 3" \
 "200:AB_ELEM=3 python -u tools/ab.py 172032,696320,2793472 1 1 3" \
 "200:AB_ELEM=12 python -u tools/ab.py 172032,696320,2793472 1 1 3"
