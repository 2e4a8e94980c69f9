#!/bin/bash
# GPU box: the out-of-order-start tests against the test-only variant library
# tools/ablibs/pskew.so (python tools/variants.py pskew), which delays every
# k_pcompress workgroup by (63 - g % 64) us at its start.  The in-tree library
# is restored on exit, whatever happens.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/skew_default.so
trap 'cp /tmp/skew_default.so "$LIB"' EXIT
cp tools/ablibs/pskew.so "$LIB"
timeout -k 10 200 python -u -m pytest tests/test_gpu_progress.py tests/test_gpu_teams.py -x -v --timeout 120 \
  --timeout-method thread -k "out_of_order or team_layouts" > gpurun_out/${TAG:-skew}_skew_tests.log 2>&1
tail -3 gpurun_out/${TAG:-skew}_skew_tests.log
