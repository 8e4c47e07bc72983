#!/usr/bin/env python3
"""Per-wave SQ counters of one kernel from a rocprofv3 --pmc pass (scripts/gpu_pass.sh pmc:...).

    pmc_waves.py <rocprofv3 -d dir> <kernel name prefix>

Sums each counter over a dispatch's rows, takes the median dispatch of the kernels whose name
starts with the prefix, and prints the totals and the per-wave figures (SQ_WAVE_CYCLES counts
quad-cycles on gfx950, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d, prefix = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").split("(")[0]
            if k.startswith(prefix):
                per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        sys.exit(f"no dispatch of {prefix} under {d}")
    counters = sorted({c for v in per.values() for c in v})
    med = {c: statistics.median(v.get(c, 0.0) for v in per.values()) for c in counters}
    waves = med.get("SQ_WAVES", 0.0) or 1.0
    print(f"{prefix}: {len(per)} dispatches (median)")
    for c in counters:
        print(f"  {c:20s} {med[c]:16.0f}  per wave {med[c] / waves:10.1f}")


if __name__ == "__main__":
    main()
