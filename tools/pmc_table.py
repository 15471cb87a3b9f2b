"""Per-kernel averages of the counters of a rocprofv3 --pmc run (the
*_counter_collection.csv files under a directory): one line per kernel with
its dispatch count and each counter's mean per dispatch.
    python tools/pmc_table.py gpurun_out/<tag>/c5pmc"""
import collections
import csv
import glob
import os
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")
                k = k if len(k) < 40 else k[:40]
                disp[k].add((f, row.get("Dispatch_Id")))
                acc[k][row.get("Counter_Name", "?")] += float(row.get("Counter_Value", 0) or 0)
    names = sorted({c for v in acc.values() for c in v})
    print("%-40s %6s " % ("kernel", "disp") + " ".join("%14s" % c for c in names))
    for k in sorted(acc, key=lambda k: -len(disp[k])):
        n = len(disp[k])
        print("%-40s %6d " % (k, n) + " ".join("%14.0f" % (acc[k][c] / n) for c in names))


if __name__ == "__main__":
    main(sys.argv[1])
