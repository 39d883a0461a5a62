#!/usr/bin/env python3
"""Per-dispatch durations (ms) of the last fit in a rocprofv3 kernel trace, in order."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last fit starts at the last k_poisson / k_bernoulli / k_fill before the end
starts = [i for i, r in enumerate(rows) if "k_poisson" in r["Kernel_Name"] or "k_bernoulli" in r["Kernel_Name"]]
for r in rows[starts[-1] if starts else 0:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if d >= 0.05:
        print(f"{r['Kernel_Name'].split('(')[0][:44]:44s} {d:8.3f}")
