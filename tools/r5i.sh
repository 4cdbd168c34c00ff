#!/bin/bash
# Round-5 call i: LDS conflict attribution (r5h.sh), then the host path at HEAD
# (config 5 through HDF5 + the host C-ABI, tools/h5_bench.sh).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
bash tools/r5h.sh && bash tools/h5_bench.sh r5i
