#!/bin/bash
# GPU box: the decode's process-to-process spread -- several bench processes,
# each under a TCC hit/miss PMC pass; per process the bench line's decode time
# and k_decode's L2 hit/miss counts (tools/debug/decode_spread.py summarises).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/dsp/p$i -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-extras --steps 50 --warmup 5 > gpurun_out/dsp_$i.log 2>&1 || exit 1
done
echo done
