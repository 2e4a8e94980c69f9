#!/bin/bash
# GPU box: VERDICT r5 #8 -- the exact multi-GPU step (RCCL process group, the
# size all-gather inside every timed step, barriers, max over ranks) run once
# on one GPU through torch.distributed.run, on BASELINE's c5 batch (8192 x 1
# MiB bf16); compare with the c5-at-G=1 extra of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --workload c5 --steps 10 --warmup 3 --no-extras --no-cpu-baseline \
  > gpurun_out/torchrun_c5.json 2> gpurun_out/torchrun_c5.err
rc=$?
tail -c 1500 gpurun_out/torchrun_c5.json
exit $rc
