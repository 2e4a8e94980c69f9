#!/bin/bash
# GPU box: c2 bench line at the driver's step counts with several settle
# phases, plus the hist-ahead memory-pattern microbenchmark.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-extras --no-cpu-baseline --steps 20 --warmup 5"
for st in 0 50 100 200 100; do
  timeout -k 10 120 python3 bench.py $A --settle-ms $st > gpurun_out/d1.log 2>&1 || { cat gpurun_out/d1.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/d1.log'):
    if l.startswith('{'):
        d=json.loads(l); print('settle $st', d['settle_steps'], d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'])"
done
if [ -x tools/microbench/hist_ahead ]; then timeout -k 10 120 tools/microbench/hist_ahead; fi
