#!/bin/bash
# GPU box: the round's final evidence for the in-tree library -- the GPU test
# suite, the profile of the driver's exact bench command (kernel-trace stats
# + PMC passes), the extras' kernel trace + traffic, then the driver's bench
# command itself.  Each step under its own time limit; the first failure ends
# the call.   usage: bash tools/final_r06.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 \
  || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
bash tools/profile_gpu.sh ${TAG}_driver_cmd --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/pmc_extras.sh ${TAG}_extras || exit 1
# summaries on the box (the raw traces exceed what gpurun copies back)
mkdir -p gpurun_out/final_$TAG
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_driver_cmd ${TAG}_driver_cmd > /dev/null || exit 1
python3 tools/trace_headline.py gpurun_out/prof_${TAG}_driver_cmd profiles/${TAG}_driver_cmd_headline_kernel_stats.csv || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_extras ${TAG}_extras > /dev/null || exit 1
cp profiles/${TAG}_* gpurun_out/final_$TAG/
cp gpurun_out/prof_${TAG}_driver_cmd/trace.log gpurun_out/final_$TAG/${TAG}_driver_cmd_trace.log
rm -rf gpurun_out/prof_${TAG}_driver_cmd gpurun_out/prof_${TAG}_extras
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
head -c 400 gpurun_out/${TAG}_bench.json
echo "final $TAG done"
