#!/bin/bash
# Round-5 call c: full GPU suite at the new defaults, bench config 2 + modes,
# encoder / decoder diag splits.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/gpu_step.sh r5c \
 "600:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "300:python -u bench.py > gpurun_out/r5c_cfg2.json" \
 "400:GIB=4 bash tools/bench_modes.sh r5c_m" \
 "200:python -u tools/diag_encode.py 1 1" \
 "200:python -u tools/diag_encode.py 1 1 3" \
 "200:python -u tools/diag_encode.py 1 2" \
 "200:python -u tools/diag_decode.py 1 1" \
 "200:python -u tools/diag_decode.py 1 2"
