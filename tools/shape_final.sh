#!/bin/bash
# GPU box: kernel stats + PMC of single shapes (tools/shape_pmc.sh), summarised
# on the box into gpurun_out/final_shapes/ (the raw traces are too large to
# copy back).   usage: TAG=r06d bash tools/shape_final.sh <shape>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06d}
mkdir -p gpurun_out/final_shapes
for S in "$@"; do
  bash tools/shape_pmc.sh $S ${TAG}_shape_$S > /dev/null 2>&1 || { echo "$S FAILED"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_shape_$S ${TAG}_shape_$S > /dev/null || exit 1
  cp profiles/${TAG}_shape_${S}_* gpurun_out/final_shapes/
  grep -h "compress" gpurun_out/prof_${TAG}_shape_$S/trace.log | tail -1
  rm -rf gpurun_out/prof_${TAG}_shape_$S
done
