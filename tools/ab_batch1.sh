#!/bin/bash
# GPU box: tools/prof/batch1.py under each library variant, back to back.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/b1_default.so
trap 'cp /tmp/b1_default.so "$LIB"' EXIT
for L in "$@"; do
  T=$(basename "$L" .so)
  if [ "$L" = default ]; then cp /tmp/b1_default.so "$LIB"; else cp "$L" "$LIB"; fi
  timeout -k 10 200 python3 -u tools/prof/batch1.py $T || exit 1
done
cp /tmp/b1_default.so "$LIB"
