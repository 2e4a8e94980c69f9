#!/bin/bash
# GPU box: sparse c4 timings of variant libraries, back to back.
#   usage: bash tools/debug/sp_ab.sh <a.so> <b.so> ...
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/sp_default.so
trap 'cp /tmp/sp_default.so "$LIB"' EXIT
for L in "$@"; do
  cp "$L" "$LIB"; echo -n "$(basename "$L" .so): "
  timeout -k 10 60 python tools/debug/sparse_bench.py 50 || { cp /tmp/sp_default.so "$LIB"; exit 1; }
done
cp /tmp/sp_default.so "$LIB"
