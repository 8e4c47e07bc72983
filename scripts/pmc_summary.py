#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + per-dispatch PMC means) into profiles/<tag>/."""
import collections
import csv
import glob
import os
import shutil
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
tag = sys.argv[2] if len(sys.argv) > 2 else "latest"
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
for f in glob.glob(os.path.join(src, "prof_*", "*kernel_stats.csv")):
    shutil.copy(f, os.path.join(dst, os.path.basename(f)))
    print(open(f).read())
for f in glob.glob(os.path.join(src, "prof_*", "*counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    name = os.path.basename(f).replace("_counter_collection.csv", "_summary.csv")
    with open(os.path.join(dst, name), "w") as o:
        o.write("kernel,counter,mean_per_dispatch,dispatches\n")
        for (k, c), v in sorted(agg.items()):
            o.write(f'"{k}",{c},{sum(v) / len(v):.1f},{len(v)}\n')
            if "kpe_" in k:
                print(f"{k:40s} {c:24s} {sum(v) / len(v):16.1f}")
