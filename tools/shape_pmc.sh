#!/bin/bash
# GPU box: one shape in isolation (tools/debug/shape_prof.py): a kernel-trace
# --stats pass, then PMC passes (HBM traffic, VALU / LDS / wait counters),
# each its own rocprofv3 process.  Summarise with
#   python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
#   usage: bash tools/shape_pmc.sh <shape> [tag]
set -e
SHAPE=$1; TAG=${2:-shape_$1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
P="python3 tools/debug/shape_prof.py $SHAPE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $P 20 > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- $P 3 > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- $P 3 > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d "$OUT/pmc_sq1" -o run --output-format csv -- $P 3 > "$OUT/pmc_sq1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
  -d "$OUT/pmc_sq2" -o run --output-format csv -- $P 3 > "$OUT/pmc_sq2.log" 2>&1
echo "shape_pmc $SHAPE done"
