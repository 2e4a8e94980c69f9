#!/bin/bash
# GPU box: instruction-fetch counters of the c2 bench (one rocprofv3 --pmc
# pass; counter names taken from this box's own list).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_icache
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
CTRS=$(python3 - "$OUT/avail.txt" <<'PY'
import re, sys
names = sorted(set(re.findall(r"\b(SQC?_[A-Z0-9_]*(?:ICACHE|IFETCH|INST_LEVEL|INSTS_SMEM)[A-Z0-9_]*)\b", open(sys.argv[1]).read())))
print(" ".join(names[:6]))
PY
)
echo "counters: $CTRS"
[ -n "$CTRS" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$OUT/pmc" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/pmc.log" 2>&1
echo "rc=$?"
