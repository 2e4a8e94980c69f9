#!/bin/bash
# GPU box: the GPU test suite, then the profile of the driver's exact bench
# command (tools/profile_gpu.sh: kernel-trace stats + PMC passes) and the
# extras' kernel trace + traffic (tools/pmc_extras.sh).
#   usage: bash tools/run_final.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03b}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/t_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_gpu.sh ${TAG}_driver_cmd --gpus 1 --steps 20 --warmup 5 || exit 1
grep '^{"metric"' gpurun_out/prof_${TAG}_driver_cmd/trace.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'])"
[ -n "$NO_EXTRAS" ] || bash tools/pmc_extras.sh ${TAG}_extras || exit 1
echo final done
