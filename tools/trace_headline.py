"""Per-kernel duration stats of the HEADLINE phase of a profiled bench.py run:
the dispatches before the first k_hist dispatch (the c3 extra's first
kernel: the bench runs its c2 warm-up, settle, timed region, profiled pass
and cold-decode measurement first, then the CPU baseline, then the extras).
The whole-run rocprofv3 --stats summary averages k_pcompress<2,..> over the
extras too (small batches, c5 at G = 1, benchmark.py's shapes: the same
kernel instance at other sizes), so this is the summary that compares with
the bench line's roofline.
    usage: python tools/trace_headline.py gpurun_out/prof_<tag> profiles/<tag>_headline_kernel_stats.csv"""
import collections
import csv
import glob
import os
import statistics
import sys


def main(src, dst):
    trace = glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "dietgpu::k_hist" in name:
            break
        if "dietgpu::" not in name:
            continue
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs"])
        for name, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), round(sum(d) / len(d), 1), statistics.median(d), min(d), max(d)])
    for name, d in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:4]:
        print(f"{name[:70]:70s} calls {len(d):5d} avg {sum(d) / len(d) / 1e3:8.2f} us median "
              f"{statistics.median(d) / 1e3:8.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
