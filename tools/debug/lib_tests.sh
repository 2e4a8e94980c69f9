#!/bin/bash
# GPU box: the GPU tests given as arguments under one variant library
# (swapped over the in-tree library, restored on exit).
#   usage: bash tools/debug/lib_tests.sh <lib.so> <pytest args...>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/lt_default.so
trap 'cp /tmp/lt_default.so "$LIB"' EXIT
cp "$1" "$LIB"
shift
timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 200 --timeout-method thread
