#!/bin/bash
# Round-6 decoder A/B: GPU suite on the default library, then library A/B of
# the decoder variants over G1 / G2 (2 GiB, 2 rounds) and E = 3 (1 GiB).
# Usage: bash tools/r6_dec_ab.sh TAG lib1.so lib2.so ...
TAG=$1; shift
bash tools/gpu_step.sh $TAG \
  "400:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
  "500:GENS=\"1 2\" bash tools/ab_libs.sh ${TAG}g 1 2 $*" \
  "300:GENS=1 AB_ELEM=3 bash tools/ab_libs.sh ${TAG}e3 1 1 $*"
