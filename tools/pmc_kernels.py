#!/usr/bin/env python3
"""Per-kernel means of every counter in rocprofv3 --pmc CSV directories (one directory
per pass), e.g. the output of tools/ubench/pmc_lat.sh.

usage: python tools/pmc_kernels.py DIR [DIR ...] [--match REGEX]
"""
import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="k_")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("mpas::", "")
                if re.search(a.match, n):
                    agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n in sorted(agg):
        print(n)
        for c, v in sorted(agg[n].items()):
            print(f"    {c:40s} {sum(v) / len(v):16.4g}")


if __name__ == "__main__":
    main()
