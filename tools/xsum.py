"""Dev tool: compact table of a bench.py JSON line's extras (compress /
decompress ms, per-kernel ms), optionally against a second line.
    usage: python tools/xsum.py new.json [old.json]"""
import json
import sys


def load(p):
    for line in open(p):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {p}")


new = load(sys.argv[1])
old = load(sys.argv[2]) if len(sys.argv) > 2 else None
oc = {e["config"]: e for e in (old or {}).get("extras", [])}
print("headline", new["value"], new["ms_per_step"], new["kernels"], (old or {}).get("kernels"))
for e in new.get("extras", []):
    o = oc.get(e["config"], {})
    c, d = e.get("compress_ms", e.get("ms_per_step")), e.get("decompress_ms")
    oc_, od = o.get("compress_ms", o.get("ms_per_step")), o.get("decompress_ms")
    k = e.get("kernels_ms") or {}
    fb = e.get("barrier_fallbacks")
    print(f"{e['config'][:70]:70s} c {c} ({oc_})  d {d} ({od})  {k}" + (f" fb={fb}" if fb is not None else ""))
