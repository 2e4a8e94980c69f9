#!/bin/bash
# GPU box: the default bench (extras included) once per library, alternating;
# prints every extra's compress / decompress ms side by side.
#   usage: PASSES=1 bash tools/extras_ab.sh default lib.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=dietgpu_fork_amd/_lib/libdietgpu_amd.so
cp "$LIB" /tmp/xab_default.so
trap 'cp /tmp/xab_default.so "$LIB"' EXIT
for p in $(seq 1 ${PASSES:-1}); do
  for L in "$@"; do
    T=$(basename "$L" .so)
    if [ "$L" = default ]; then cp /tmp/xab_default.so "$LIB"; else cp "$L" "$LIB"; fi
    timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/xab_${T}_$p.json 2>/dev/null || { echo "$T FAILED"; exit 1; }
  done
done
python3 - "$@" <<'PY'
import json, sys, glob, os
libs = [os.path.basename(a).replace('.so', '') for a in sys.argv[1:]]
rows = {}
for t in libs:
    for f in sorted(glob.glob(f"gpurun_out/xab_{t}_*.json")):
        d = json.loads(open(f).read().splitlines()[-1])
        rows.setdefault("c2 step", {}).setdefault(t, []).append(d["ms_per_step"])
        for e in d["extras"]:
            if "rows" in e:
                for r in e["rows"]:
                    k = f"{e['config'][:14]} {r.get('type')} b{r.get('batch')} n{r.get('words')}"
                    rows.setdefault(k, {}).setdefault(t, []).append((r.get("compress_ms"), r.get("decompress_ms")))
            else:
                rows.setdefault(e["config"][:60], {}).setdefault(t, []).append((e.get("compress_ms"), e.get("decompress_ms"), e.get("ms_per_step")))
for k, v in rows.items():
    print(k, " | ".join(f"{t}: {v.get(t)}" for t in libs))
PY
