#!/bin/bash
# GPU box: the round's standard check, in one call -- the GPU test suite, an
# optional same-box A/B of kernel-variant libraries (AB="lib.so ..."), then
# the default bench.  Each step under its own time limit; the first failure
# ends the call.  usage: TAG=r4a AB="default tools/ablibs/x.so" bash tools/gpu_round.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r4}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  tail -2 gpurun_out/${TAG}_tests.log
fi
if [ -n "$AB" ]; then
  AB_STEPS=${AB_STEPS:-100} timeout -k 10 500 bash tools/ab.sh $AB > gpurun_out/${TAG}_ab.txt 2>&1
  cat gpurun_out/${TAG}_ab.txt
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  head -c 600 gpurun_out/${TAG}_bench.json
fi
