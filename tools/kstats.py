"""Summarize a rocprofv3 --kernel-trace --stats CSV directory: per kernel
calls and average duration, and (for a --pmc run) per-kernel counter means."""
import collections
import csv
import glob
import os
import sys


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
        print(f)
        for r in csv.DictReader(open(f)):
            print("  %-70s calls %6s avg %9.2f us  %5.1f%%" % (
                r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        print(f)
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            print("  %-60s %-22s n=%4d mean %.5g" % (k, c, len(v), sum(v) / len(v)))


if __name__ == "__main__":
    main(sys.argv[1])
