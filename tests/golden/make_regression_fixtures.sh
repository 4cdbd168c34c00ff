#!/bin/bash
# Fixture generator, build container only (needs /root/reference and HDF5 1.10
# from /opt/conda).  Extracts the 42 LZ4 regression chunks + originals from the
# reference's tests/data/*.h5 into tests/golden/regression/ (committed).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REF=${REF:-/root/reference}
OUT=$HERE/regression
mkdir -p "$OUT"
rm -f "$OUT"/*.orig "$OUT"/*.chunk "$OUT"/MANIFEST
gcc -O1 -I/opt/conda/include "$HERE/extract_regression.c" -L/opt/conda/lib -lhdf5 \
    -Wl,-rpath,/opt/conda/lib -o /tmp/extract_regression
for v in 0.1.3 0.4.0; do
  /tmp/extract_regression "$REF/tests/data/regression_$v.h5" "$v" "$OUT" "$OUT/MANIFEST"
done
wc -l "$OUT/MANIFEST"
