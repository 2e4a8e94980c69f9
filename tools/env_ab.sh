#!/bin/bash
# GPU box: A/B of run-time knobs on the c2 bench, one bench run per setting.
# usage: bash tools/env_ab.sh "VAR=a VAR2=b" "VAR=c" ...   ("" = defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
i=0
for S in "$@"; do
  i=$((i + 1))
  env $S timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/envab_$i.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/envab_$i.log'):
    if l.startswith('{'):
        d = json.loads(l); print('[$S]', d['value'], d['ms_per_step'], d['kernels'])"
done
