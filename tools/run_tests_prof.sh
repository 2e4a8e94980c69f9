#!/bin/bash
# GPU box: the GPU test suite, then rocprofv3 kernel-trace stats of a
# profiling script (default: the sparse extras).  usage:
#   bash tools/run_tests_prof.sh <tag> [script.py]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sp}; SCRIPT=${2:-tools/prof/sparse_case.py}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
  tail -5 gpurun_out/t1.log
  [ $rc -eq 0 ] || exit $rc
fi
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- python3 $SCRIPT > gpurun_out/$TAG.log 2>&1 || exit $?
grep -v "^W\|^\[" gpurun_out/$TAG.log | tail -20
