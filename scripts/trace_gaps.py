"""GPU idle time per fit from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

A fit starts at its first sampler launch (the first of the two learner halves'); the GPU
is busy where any kernel or copy of either stream runs.  Prints per fit the time to the
next fit's start, the busy union, and the gaps longer than 0.2 ms (offset, length).

usage: python3 scripts/trace_gaps.py <kernel_trace.csv> [sampler kernel substring]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_bernoulli"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) + (r["Kernel_Name"],)
                for r in csv.DictReader(open(path)))
    starts = [k[0] for k in ks if mark in k[2]][0::2]
    for i, t0 in enumerate(starts):
        t1 = starts[i + 1] if i + 1 < len(starts) else ks[-1][1]
        end, busy, gaps = t0, 0, []
        for s, e, _ in (k for k in ks if t0 <= k[0] < t1):
            if s > end + 200_000:
                gaps.append((round((end - t0) / 1e6, 1), round((s - end) / 1e6, 2)))
            if e > end:
                busy += e - max(s, end)
                end = e
        print("fit %d: to next %.1f ms, busy %.1f ms, gaps %s" % (i, (t1 - t0) / 1e6, busy / 1e6, gaps))


if __name__ == "__main__":
    main()
