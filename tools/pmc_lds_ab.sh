#!/bin/bash
# GPU box: per library variant, the c2 bench's LDS PMC (bank conflicts /
# active cycles, one rocprofv3 pass) and its A/B timing (tools/ab.sh).
#   usage: bash tools/pmc_lds_ab.sh <variant.so>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/pl_default.so
trap 'cp /tmp/pl_default.so "$LIB"' EXIT
for L in "$@"; do
  T=$(basename "$L" .so)
  cp "$L" "$LIB"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    -d gpurun_out/pl_$T -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-verify > gpurun_out/pl_$T.log 2>&1 || exit 1
done
cp /tmp/pl_default.so "$LIB"
AB_STEPS=50 bash tools/ab.sh "$@"
