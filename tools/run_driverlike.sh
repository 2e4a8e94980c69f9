#!/bin/bash
# GPU box: what the driver runs at round end -- the GPU test suite, smoke(),
# then the bench command (default: --gpus 1 --steps 20 --warmup 5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dl_tests.log 2>&1 || { tail -30 gpurun_out/dl_tests.log; exit 1; }
tail -1 gpurun_out/dl_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/dl_smoke.log 2>&1 || { tail -20 gpurun_out/dl_smoke.log; exit 1; }
tail -1 gpurun_out/dl_smoke.log
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} > gpurun_out/dl_bench.log 2>&1 || { tail -20 gpurun_out/dl_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/dl_bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'], d['encode_plus_decode_algorithmic_GBps'])"
