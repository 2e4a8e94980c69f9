#!/bin/bash
# GPU box: the GPU test suite (in-tree library), then bench extras A/B of
# the given libraries (tools/debug/extras_ab.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
tail -3 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
bash tools/debug/extras_ab.sh "$@"
