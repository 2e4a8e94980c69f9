#!/bin/bash
# GPU box: A/B of kernel-variant libraries on the c2 bench (+ kernel-trace
# timeline of one step).  usage: bash tools/exp_ab.sh <lib.so|default>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in "$@"; do
  T=$(basename "$L" .so)
  if [ "$L" = default ]; then unset DIETGPU_AMD_LIB; else export DIETGPU_AMD_LIB=$PWD/$L; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/ab_$T.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/ab_$T.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$T', d['value'], d['ms_per_step'], d['kernels'])"
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/abkt_$T -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/abkt_$T.log 2>&1 || exit 1
  python3 tools/timeline_step.py gpurun_out/abkt_$T | tail -4
done
