#!/bin/bash
# Round-5 call k: sanity of the rebuilt closing library, then the host path at
# HEAD (config 5 through HDF5 + the host C-ABI, tools/h5_bench.sh).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "golden or regression or full_size" > gpurun_out/r5k_pytest.log 2>&1 && \
bash tools/h5_bench.sh r5k
