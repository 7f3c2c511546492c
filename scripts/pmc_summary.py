#!/usr/bin/env python3
"""Average of each PMC counter per kernel (by demangled-ish name) over all
dispatches, from one or more rocprofv3 counter_collection.csv directories.
usage: pmc_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            m = re.search(r"(gemm\w*_kernel)I(.*?)EEv", k)
            name = (m.group(1) + "<" + re.sub(r"Li|E", lambda x: "" if x.group(0) == "Li" else ",", m.group(2)) + ">") \
                if m else k.split("(")[0][:60]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(agg.items()):
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.0f}   (n={len(v)})")
