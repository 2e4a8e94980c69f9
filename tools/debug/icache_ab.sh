#!/bin/bash
# GPU box: instruction-cache counters of k_pcompress / k_decode for each
# library given (swapped over the in-tree one in turn), c2 bench.
#   usage: bash tools/debug/icache_ab.sh default lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/ic_default.so
OUT=gpurun_out/icache_ab
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
CTRS=$(python3 - "$OUT/avail.txt" <<'PY'
import re, sys
names = sorted(set(re.findall(r"\b(SQC_ICACHE_[A-Z0-9_]*)\b", open(sys.argv[1]).read())))
print(" ".join(names[:4]))
PY
)
echo "counters: $CTRS"
[ -n "$CTRS" ] || exit 1
for L in "$@"; do
  T=$(basename "$L" .so)
  if [ "$L" = default ]; then cp /tmp/ic_default.so "$LIB"; else cp "$L" "$LIB"; fi
  timeout -s KILL 120 rocprofv3 --pmc $CTRS GRBM_GUI_ACTIVE -d "$OUT/$T" -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-verify > "$OUT/$T.log" 2>&1 || { cp /tmp/ic_default.so "$LIB"; exit 1; }
  python3 - "$OUT/$T" "$T" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"]
    k = "pcompress" if "k_pcompress<2" in k else "decode" if "k_decode<2" in k else None
    if k: acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(sys.argv[2], k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
done
cp /tmp/ic_default.so "$LIB"
