"""Per-kernel sums of the counters in a PMC run directory (rocprofv3 --pmc csv passes).

usage: python3 scripts/pmc_kernels.py <dir> [kernel substring ...]
Prints, per kernel name (template arguments kept), launches, summed duration and every
counter summed over its launches.
"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    dur = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if keys and not any(s in k for s in keys):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = (f, r["Dispatch_Id"])
            if did not in seen:
                seen.add(did)
                n[(f, k)] += 1
                if "Start_Timestamp" in r:
                    dur[(f, k)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for k in sorted(acc):
        launches = max(v for (f, kk), v in n.items() if kk == k)
        ms = max(v for (f, kk), v in dur.items() if kk == k) if dur else 0.0
        print("%s: launches %d, %.2f ms" % (k, launches, ms))
        for c, v in sorted(acc[k].items()):
            print("   %-24s %.4g" % (c, v))


if __name__ == "__main__":
    main()
