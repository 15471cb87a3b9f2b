"""Per-kernel means of the counters of a rocprofv3 --pmc run (the
run_results.db under a directory, view counters_collection): one line per
kernel with its dispatch count and each counter's mean per dispatch.
    python tools/pmc_table.py gpurun_out/<tag>/c5pmc"""
import collections
import glob
import os
import sqlite3
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for k, name, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
            acc[k.split("(")[0].strip()[:40]][name].append(float(v))
    names = sorted({n for v in acc.values() for n in v})
    print("%-40s %6s " % ("kernel", "disp") + " ".join("%14s" % n[:14] for n in names))
    for k in sorted(acc, key=lambda k: -max(len(x) for x in acc[k].values())):
        n = max(len(x) for x in acc[k].values())
        print("%-40s %6d " % (k, n) + " ".join("%14.0f" % (sum(acc[k][c]) / max(1, len(acc[k][c]))) for c in names))


if __name__ == "__main__":
    main(sys.argv[1])
