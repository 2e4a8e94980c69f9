"""Print kernel sequences (durations, gaps) from a rocprofv3 kernel trace:
the sequence starting at the k-th launch of a given kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2]
picks = [int(x) for x in sys.argv[3].split(",")]
cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 16
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
for k in picks:
    prev = None
    t0 = int(rows[idx[k]]["Start_Timestamp"])
    for r in rows[idx[k]: idx[k] + cnt]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev else 0.0
        print(f"{r['Kernel_Name'][:64]:64s} dur {(e - s) / 1000:7.1f} gap {gap:6.1f} end {(e - t0) / 1000:7.1f}")
        prev = e
    print("---")
