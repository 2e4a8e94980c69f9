#!/bin/bash
# GPU box: kernel-trace stats and HBM traffic (FETCH_SIZE / WRITE_SIZE, one
# rocprofv3 pass each) of the bench INCLUDING its secondary configs (c3,
# batch-1 large tensors, fp64, sparse), for the three-kernel path's kernels.
#   usage: bash tools/pmc_extras.sh <tag>; then python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
set -e
TAG=${1:-extras}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
A="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py $A > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 bench.py $A > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 bench.py $A > "$OUT/pmc_write.log" 2>&1
# VALU and SALU issue counters of every kernel (c3: the encode step chain)
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
  -d "$OUT/pmc_valu" -o run --output-format csv -- python3 bench.py $A > "$OUT/pmc_valu.log" 2>&1
echo "pmc_extras $TAG done"
