#!/bin/bash
# GPU box: instruction counts of k_compress for kernel-variant libraries
# (make exp EXP=k).  usage: bash tools/exp_pmc_compress.sh <lib.so>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in "$@"; do
  T=$(basename "$L" .so)
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -d gpurun_out/pmc_$T -o run --output-format csv -- python3 tools/exp_trace_compress.py "$L" > gpurun_out/pmc_$T.log 2>&1 || exit 1
  python3 - "$T" <<'PY'
import csv, collections, glob, sys
t = sys.argv[1]
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"gpurun_out/pmc_{t}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_compress" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[(r["Counter_Name"], r["Dispatch_Id"])] = 1
d = len({k[1] for k in n}) or 1
w = acc["SQ_WAVES"] / d
print(t, "launches", d, "per wave:", {k: round(v / d / w, 1) for k, v in acc.items() if k != "SQ_WAVES"})
PY
done
