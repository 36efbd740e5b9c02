"""Merge rocprofv3 kernel + memory-copy traces of several processes into one
timeline (used on gpurun_out/<dir>/p*/ from scripts/run_clock_bench.py).

    python scripts/trace_timeline.py DIR [last_ms]
"""
import csv
import glob
import os
import re
import sys

NAMES = {"0": "scatter_add", "1": "gather", "2": "assign_from", "3": "scatter_init"}


def short(n):
    m = re.search(r"row_op_kernel<[^,]*, 4, (\d)", n)
    if m:
        return NAMES[m.group(1)]
    if "bucket_sum" in n:
        return "bucket_sum"
    return n.split("(")[0][-30:]


def load(d):
    ev = []
    for pd in sorted(glob.glob(os.path.join(d, "p*"))):
        p = os.path.basename(pd)
        for f in glob.glob(os.path.join(pd, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), p,
                           short(r["Kernel_Name"]), r["Stream_Id"]))
        for f in glob.glob(os.path.join(pd, "**", "*memory_copy_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), p,
                           "copy " + r["Direction"].replace("MEMORY_COPY_", ""), r["Stream_Id"]))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
    ev = load(d)
    t0, end = ev[0][0], max(e[1] for e in ev)
    busy_until = None
    for s, e, p, n, st in ev:
        if s < end - last_ms * 1e6:
            continue
        gap = "" if busy_until is None or s <= busy_until else f"  <-- idle {(s - busy_until) / 1e6:.3f} ms"
        print(f"{(s - t0) / 1e6:10.3f} {(e - s) / 1e6:8.3f} {p} s{st:>2} {n}{gap}")
        busy_until = e if busy_until is None else max(busy_until, e)


if __name__ == "__main__":
    main()
