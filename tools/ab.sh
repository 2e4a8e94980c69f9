#!/bin/bash
# GPU box: A/B of kernel-variant libraries on the c2 bench, one box, back to
# back.  Each variant .so is copied over the in-tree library of this scratch
# copy in turn (the product has no library override).
#   usage: bash tools/ab.sh <variant.so>...   (current in-tree lib = "default")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/ab_default.so
trap 'cp /tmp/ab_default.so "$LIB"' EXIT
for L in "$@"; do
  T=$(basename "$L" .so)
  if [ "$L" = default ]; then cp /tmp/ab_default.so "$LIB"; else cp "$L" "$LIB"; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --no-verify --steps ${AB_STEPS:-20} > gpurun_out/ab_$T.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/ab_$T.log'):
    if l.startswith('{'):
        d = json.loads(l); h = d.get('decode_hbm') or {}; print('$T', d['value'], d['ms_per_step'], d['kernels'], 'dec warm/cold', h.get('decode_warm_ms'), h.get('decode_cold_ms'))"
done
cp /tmp/ab_default.so "$LIB"
