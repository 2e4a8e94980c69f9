#!/bin/bash
# GPU box: the in-tree library's full GPU test suite, then (optional) a
# same-box c2 A/B with the cold-decode probe (AB="default x.so ...") and a
# single-shape A/B (SHAPES="..." SAB="default x.so ..."); each step under its
# own time limit, the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-rc}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
    || { echo "tests FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
if [ -n "$AB" ]; then
  NO_PARITY=1 PASSES=${PASSES:-2} timeout -k 10 600 bash tools/ab2.sh $AB || exit 1
fi
if [ -n "$SAB" ]; then
  PASSES=${SPASSES:-2} REPS=${REPS:-20} timeout -k 10 600 bash tools/shape_ab.sh $SAB || exit 1
fi
