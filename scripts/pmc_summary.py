#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run into profiles/<tag>/:

  kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied verbatim)
  summary.json       per kernel: calls, average duration (trace) and the average
                     per-dispatch PMC counters of the separate --pmc passes.
                     hbm_bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024: FETCH_SIZE is
                     in KiB and reports half of a wide streaming read on gfx950
                     (MI355X_MICROARCH.md, HBM section); k_transpose's known read size
                     (rows x row stride) is recorded as a calibration check.

usage: scripts/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def read_counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            out[short(r["Name"])] = {"calls": int(r["Calls"]),
                                     "avg_ms": float(r["AverageNs"]) / 1e6,
                                     "total_ms": float(r["TotalDurationNs"]) / 1e6}
    for sub in ("fetch", "write", "lds"):
        for k, cs in read_counters(os.path.join(src, sub)).items():
            d = out.setdefault(k, {})
            for cname, vals in cs.items():
                d[cname + "_avg"] = sum(vals) / len(vals)
    for k, d in out.items():
        if "FETCH_SIZE_avg" in d and "WRITE_SIZE_avg" in d:
            d["hbm_bytes_per_launch"] = 2 * d["FETCH_SIZE_avg"] * 1024 + d["WRITE_SIZE_avg"] * 1024
            if "avg_ms" in d and d["avg_ms"] > 0:
                d["hbm_GBs"] = d["hbm_bytes_per_launch"] / (d["avg_ms"] / 1e3) / 1e9
        if "SQ_LDS_IDX_ACTIVE_avg" in d and "SQ_LDS_BANK_CONFLICT_avg" in d:
            d["lds_conflict_frac"] = d["SQ_LDS_BANK_CONFLICT_avg"] / max(d["SQ_LDS_IDX_ACTIVE_avg"], 1)
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1, sort_keys=True)
    for k in sorted(out, key=lambda k: -out[k].get("total_ms", 0))[:8]:
        print(k, {a: round(b, 3) if isinstance(b, float) else b for a, b in out[k].items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
