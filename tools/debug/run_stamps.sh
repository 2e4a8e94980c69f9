#!/bin/bash
# GPU box: swap a stamp-instrumented library in, print the phase timeline.
#   usage: bash tools/debug/run_stamps.sh <stamp lib> <reader.py>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/stamps_default.so
trap 'cp /tmp/stamps_default.so "$LIB"' EXIT
cp "$1" "$LIB"
timeout -k 10 120 python3 -u "$2"
