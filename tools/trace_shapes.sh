#!/bin/bash
# GPU box: kernel-trace timelines of single shapes (tools/debug/shape_prof.py),
# one rocprofv3 process per shape; prints the last ops of each (kernels,
# durations, idle gaps) via tools/timeline.py.
#   usage: SHOW=30 bash tools/trace_shapes.sh <shape>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for S in "$@"; do
  OUT=gpurun_out/tl_$S
  mkdir -p "$OUT"
  timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv -- python3 tools/debug/shape_prof.py $S ${REPS:-5} > "$OUT.log" 2>&1 || { echo "$S FAILED"; tail -5 "$OUT.log"; exit 1; }
  echo "=== $S: $(grep -E 'compress .* us' "$OUT.log")"
  python3 tools/timeline.py "$OUT" ${SHOW:-30}
done
