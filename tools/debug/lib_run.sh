#!/bin/bash
# GPU box: run one python script under each library in turn (swapped over the
# in-tree library; restored on exit).
#   usage: bash tools/debug/lib_run.sh "<script and args>" <lib.so|default>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/lr_default.so
trap 'cp /tmp/lr_default.so "$LIB"' EXIT
CMD=$1
shift
for L in "$@"; do
  if [ "$L" = default ]; then cp /tmp/lr_default.so "$LIB"; else cp "$L" "$LIB"; fi
  echo "== $(basename "$L" .so)"
  timeout -k 10 240 python3 -u $CMD || exit 1
done
