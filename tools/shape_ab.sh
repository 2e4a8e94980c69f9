#!/bin/bash
# GPU box: same-box A/B of kernel-variant libraries on single shapes
# (tools/debug/shape_prof.py), alternating libraries per pass.
#   usage: SHAPES="c5 c3" PASSES=2 bash tools/shape_ab.sh default tools/ablibs/x.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/sab_default.so
trap 'cp /tmp/sab_default.so "$LIB"' EXIT
for p in $(seq 1 ${PASSES:-2}); do
  for L in "$@"; do
    T=$(basename "$L" .so)
    if [ "$L" = default ]; then cp /tmp/sab_default.so "$LIB"; else cp "$L" "$LIB"; fi
    for S in $SHAPES; do
      r=$(timeout -k 10 240 python3 tools/debug/shape_prof.py $S ${REPS:-10} 2>&1 | tail -1) || { echo "$T $S FAILED: $r"; exit 1; }
      echo "pass $p $T $r"
    done
  done
done
