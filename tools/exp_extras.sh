#!/bin/bash
# GPU box: full bench (with the secondary configs) under the default library
# and under each experiment library.   usage: bash tools/exp_extras.sh <tag> k1 k2 ...
set -e
TAG=$1; shift
mkdir -p gpurun_out/ex_$TAG
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ex_$TAG/base.json
for k in "$@"; do
  DIETGPU_AMD_LIB=$PWD/dietgpu_fork_amd/_lib/exp/libdietgpu_amd_exp$k.so \
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ex_$TAG/exp$k.json
done
python3 - "$TAG" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(f"gpurun_out/ex_{sys.argv[1]}/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), d["ms_per_step"], d["kernels"])
    for e in d.get("extras", []):
        print("   ", e["config"][:44], e["compress_ms"], e["decompress_ms"], e["roundtrip_bit_exact"])
PY
