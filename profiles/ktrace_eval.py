"""Per-dispatch kernel durations of ONE evaluation from a rocprofv3 kernel trace (profiles/scripts/ktrace.sh):
the last complete evaluation (k_scatter ... the gradient gather) in dispatch order.
Usage: python profiles/ktrace_eval.py gpurun_out/<tag>_kt"""
import csv
import glob
import sys

rows = []
for p in glob.glob(sys.argv[1].rstrip("/") + "/*kernel_trace.csv"):
    with open(p) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if "k_scatter" in r[2]]
i0 = starts[-2]
i1 = starts[-1]
t0 = rows[i0][0]
tot = 0
for s, e, n in rows[i0:i1]:
    d = (e - s) / 1e3
    tot += d
    print(f"{(s - t0) / 1e3:9.1f} {d:8.1f} us  {n[:90]}")
print(f"sum {tot:.1f} us, span {(rows[i1][0] - t0) / 1e3:.1f} us")
