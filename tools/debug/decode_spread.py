"""Summarise tools/debug/decode_spread_pmc.sh: per process, the bench line's
decode time and k_decode<2>'s mean TCC hit / miss counts per launch."""
import csv
import glob
import json

for i in range(1, 6):
    line = next((json.loads(l) for l in open(f"gpurun_out/dsp_{i}.log") if l.startswith('{"metric"')), None)
    hits, miss, n = 0.0, 0.0, 0
    for f in glob.glob(f"gpurun_out/dsp/p{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_decode<2" not in r["Kernel_Name"]:
                continue
            v = float(r["Counter_Value"])
            if r["Counter_Name"].startswith("TCC_HIT"):
                hits += v
                n += 1
            elif r["Counter_Name"].startswith("TCC_MISS"):
                miss += v
    if line and n:
        print(i, line["ms_per_step"], line["kernels"], f"hit {hits / n:.3e} miss {miss / n:.3e} rate {hits / (hits + miss):.3f}")
