"""Timeline of the last steps of a rocprofv3 run (kernel + memory-copy
traces): every op with its start relative to the first op shown, its
duration and the idle gap before it.  Dev tool.
    usage: python3 tools/timeline.py <rocprofv3 output dir> [ops to show]"""
import csv
import glob
import sys


def rows(pattern, kind):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name") or r.get("Direction") or kind
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name[:60]))
    return out


def main():
    d = sys.argv[1]
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    ops = rows(f"{d}/**/*kernel_trace.csv", "K") + rows(f"{d}/**/*memory_copy_trace.csv", "M")
    ops.sort()
    ops = ops[-show:]
    t0 = ops[0][0]
    prev_end = ops[0][0]
    busy = 0
    for s, e, k, n in ops:
        gap = (s - prev_end) / 1e3
        print(f"{(s - t0) / 1e3:10.1f} us  {k} {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {n}")
        prev_end = max(prev_end, e)
        busy += e - s
    span = (ops[-1][1] - t0) / 1e3
    print(f"span {span:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / 1e3 / span:.1f} %)")


if __name__ == "__main__":
    main()
