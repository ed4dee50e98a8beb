#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv passes: mean counter value per dispatch of
every kernel matching a filter, over all pass directories given.

    python tools/pmc_csv.py 'k_tb3d' gpurun_out/pmc_tb/mr2/p*/run_counter_collection.csv
"""
import csv
import sys
from collections import defaultdict


def main():
    filt = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[2:]:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if filt not in name:
                    continue
                short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print("  %-28s %16.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
