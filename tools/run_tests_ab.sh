#!/bin/bash
# GPU box: the GPU test suite, then a same-box A/B of library variants on the
# c2 bench (tools/ab.sh).  usage: bash tools/run_tests_ab.sh [variant.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
  tail -15 gpurun_out/t1.log
  [ $rc -eq 0 ] || exit $rc
fi
AB_STEPS=${AB_STEPS:-50} bash tools/ab.sh "$@"
