#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of the c2 bench for each library
#   usage: bash tools/debug/trace_ab.sh default lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/tr_default.so
OUT=gpurun_out/trace_ab
mkdir -p "$OUT"
for L in "$@"; do
  T=$(basename "$L" .so)
  if [ "$L" = default ]; then cp /tmp/tr_default.so "$LIB"; else cp "$L" "$LIB"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$T" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extras --no-verify > "$OUT/$T.log" 2>&1 || { cp /tmp/tr_default.so "$LIB"; exit 1; }
  f=$(find "$OUT/$T" -name "*kernel_stats.csv" | head -1)
  echo "== $T"; head -8 "$f" | cut -d, -f1-5
done
cp /tmp/tr_default.so "$LIB"
