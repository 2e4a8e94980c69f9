"""Summarise a tools/profile_gpu.sh run into profiles/<tag>_*.

  python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, the bench command)
and profiles/<tag>_pmc.json: per dietgpu kernel family the per-launch mean of
every collected counter plus hbm_bytes_per_launch =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024 — FETCH_SIZE / WRITE_SIZE are in KiB and
gfx950 FETCH_SIZE tallies half the bytes of a wide coalesced read
(MI355X_MICROARCH.md, HBM section).
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def family(name):
    """'void dietgpu::k_decode<2, 0>(...)' -> 'k_decode<2,0>': one entry per
    template instance, so the bf16 launches are not averaged with the byte
    (c3) or fp64 launches of the bench's secondary configs."""
    m = re.search(r"dietgpu::(?:\(anonymous namespace\)::)?(k_\w+)(<[^>(]*>)?", name)
    if not m:
        return None
    return m.group(1) + (m.group(2) or "").replace(" ", "")


def main(src, tag):
    outdir = os.path.join(ROOT, "profiles")
    os.makedirs(outdir, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(outdir, f"{tag}_kernel_stats.csv"))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        # one row per (dispatch, counter); sum over dimensions first
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            fam = family(r.get("Kernel_Name", ""))
            if fam:
                acc[(fam, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (fam, _, cname), v in acc.items():
            per[fam][cname].append(v)
    res = {}
    for fam, cs in per.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["launches_sampled"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        if d.get("SQ_WAVE_CYCLES"):
            w = d["SQ_WAVE_CYCLES"]
            d["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / w
            d["frac_wait_inst_any"] = d.get("SQ_WAIT_INST_ANY", 0) / w
            d["frac_active_inst"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
        res[fam] = d
    sys.path.insert(0, ROOT)
    from bench import library_sha256

    json.dump({"source": "rocprofv3 --pmc (separate passes), tools/profile_gpu.sh",
               "hbm_formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024",
               # the build the counters describe (bench.py takes traffic only
               # from a summary of the library it runs)
               "library_sha256": library_sha256(),
               "kernels": res}, open(os.path.join(outdir, f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
