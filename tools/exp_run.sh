#!/bin/bash
# GPU box: time the bench under each experiment library (make exp EXP=k).
#   usage: bash tools/exp_run.sh <tag> k1 k2 ...
set -e
TAG=$1; shift
mkdir -p gpurun_out/exp_$TAG
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/exp_$TAG/base.json
for k in "$@"; do
  DIETGPU_AMD_LIB=$PWD/dietgpu_fork_amd/_lib/exp/libdietgpu_amd_exp$k.so \
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-verify > gpurun_out/exp_$TAG/exp$k.json
done
python3 - "$TAG" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(f"gpurun_out/exp_{sys.argv[1]}/*.json")):
    d = json.load(open(f)); print(os.path.basename(f), d["kernels"])
PY
