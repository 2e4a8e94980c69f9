#!/bin/bash
# GPU box: bench.py's secondary configs (extras) for each library in turn
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/ab_default.so
trap 'cp /tmp/ab_default.so "$LIB"' EXIT
for L in "$@"; do
  T=$(basename "$L" .so)
  cp "$L" "$LIB"
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/xab_$T.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/xab_$T.log'):
    if l.startswith('{'):
        d = json.loads(l)
        for e in d['extras']:
            if 'compress_ms' in e: print('$T', e['config'][:40], e['compress_ms'], e['decompress_ms'])"
done
cp /tmp/ab_default.so "$LIB"
