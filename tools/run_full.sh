#!/bin/bash
# GPU box: the GPU test suite, then the default bench (headline + extras).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
  tail -2 gpurun_out/t1.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:---steps 100 --warmup 10} > gpurun_out/bench_full.log 2>&1 || exit $?
python3 - <<'PY'
import json
s = open("gpurun_out/bench_full.log").read()
d = json.JSONDecoder().raw_decode(s[s.rindex('{"metric"'):])[0]
print({k: d[k] for k in ("value", "ms_per_step", "kernels")}, d["roofline"]["frac"])
for e in d.get("extras", []):
    print(e.get("config")[:64], e.get("compress_ms"), e.get("decompress_ms"), e.get("algorithmic_GBps"))
PY
