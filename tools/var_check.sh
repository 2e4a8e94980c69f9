#!/bin/bash
# GPU box: for each variant library, swap it in, run the oracle/golden parity
# tests, then time it on the c2 bench; the in-tree library is restored after.
#   usage: bash tools/var_check.sh <variant.so>...   ("default" = in-tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/vc_default.so
trap 'cp /tmp/vc_default.so "$LIB"' EXIT
rc=0
for L in "$@"; do
  T=$(basename "$L" .so)
  if [ "$L" = default ]; then cp /tmp/vc_default.so "$LIB"; else cp "$L" "$LIB"; fi
  if [ "$L" != default ] && [ -z "$NO_PARITY" ]; then
    timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_compress_paths.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vc_$T.log 2>&1 || { echo "$T parity FAILED"; tail -30 gpurun_out/vc_$T.log; rc=1; break; }
    echo "$T parity $(tail -1 gpurun_out/vc_$T.log)"
  fi
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --no-verify --steps ${AB_STEPS:-50} > gpurun_out/ab_$T.log 2>&1 || { rc=1; break; }
  python3 -c "
import json
for l in open('gpurun_out/ab_$T.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$T', d['value'], d['ms_per_step'], d['kernels'])"
done
cp /tmp/vc_default.so "$LIB"
exit $rc
