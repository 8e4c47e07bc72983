#!/usr/bin/env python3
"""HBM traffic of kpe_pattern_kernel per launch from FETCH_SIZE / WRITE_SIZE rocprofv3 passes
(gpurun_out/pt_<cfg>_fetch, _write): writes perf/pmc_traffic_<cfg>.json (bench.py reads it for the
pattern-dominated configurations). gfx950 correction as scripts/pmc_summary.py: FETCH_SIZE x 2."""
import csv
import glob
import json
import os
import sys

cfg = sys.argv[1]
KERNEL = sys.argv[2] if len(sys.argv) > 2 else "kpe_pattern_kernel"  # a kernel-name prefix


def mean(counter, tag):
    vals = []
    for f in glob.glob(f"gpurun_out/pt_{cfg}_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("void ", "")
            # the evaluation launches (the per-binding prologue instance, <..., true, ...>, is not one)
            if name.startswith(KERNEL) and ", true, false>" not in name.split("(")[0][-14:] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


fetch, write = mean("FETCH_SIZE", "fetch"), mean("WRITE_SIZE", "write")
if fetch is None or write is None:
    sys.exit(f"no {KERNEL} counters for {cfg}")
t = {"kernel": KERNEL, "fetch_kib_raw": fetch, "write_kib_raw": write,
     "fetch_bytes_corrected": fetch * 1024 * 2, "write_bytes": write * 1024,
     "scan_bytes_per_launch": fetch * 1024 * 2 + write * 1024,
     "correction": "FETCH_SIZE x2 (gfx950 half-count of wide coalesced reads), KiB -> bytes",
     "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over bench.py --config {cfg}"}
os.makedirs("gpurun_out/pt_json", exist_ok=True)
for out in (f"perf/pmc_traffic_{cfg}.json", f"gpurun_out/pt_json/pmc_traffic_{cfg}.json"):
    json.dump(t, open(out, "w"), indent=1)
print(cfg, t["scan_bytes_per_launch"])
