#!/bin/bash
# Runs on the GPU box (via gpurun): kernel-trace stats of the bench command,
# then PMC passes, each a separate rocprofv3 process (counters never combined
# with runtime/sys traces).  Output: gpurun_out/prof_<tag>/...
#   usage: bash tools/profile_gpu.sh <tag> [bench args...]
set -e
TAG=${1:-r01}; shift || true
ARGS=${*:-"--no-cpu-baseline --no-extras"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
PMC_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d "$OUT/pmc_sq1" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
  -d "$OUT/pmc_sq2" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE \
  -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_write.log" 2>&1
echo "profile $TAG done"
