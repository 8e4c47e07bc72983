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

# HBM traffic of the scan kernel per launch from the FETCH_SIZE / WRITE_SIZE passes.
# Units: KiB. gfx950 correction (MI355X_MICROARCH.md § HBM): FETCH_SIZE reports half the
# bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.
SCAN_KERNELS = ("kpe_lean5_batch_kernel", "kpe_lean5_kernel", "kpe_scan_kernel<true, true, false",
                "kpe_scan_kernel<true, false, false")


def _mean(fname, counter):
    p = os.path.join(dst, fname)
    if not os.path.exists(p):
        return None
    rows = list(csv.DictReader(open(p)))
    for kernel in SCAN_KERNELS:  # the resource-scan instantiation the run used
        for r in rows:
            if kernel in r["kernel"] and r["counter"] == counter:
                return float(r["mean_per_dispatch"]), r["kernel"]
    return None


fm, wm = _mean("pmc_fetch_summary.csv", "FETCH_SIZE"), _mean("pmc_write_summary.csv", "WRITE_SIZE")
if fm is not None and wm is not None:
    import json

    (fetch, kname), (write, _) = fm, wm
    t = {"kernel": kname, "fetch_kib_raw": fetch, "write_kib_raw": write,
         "fetch_bytes_corrected": fetch * 1024 * 2, "write_bytes": write * 1024,
         "scan_bytes_per_launch": fetch * 1024 * 2 + write * 1024,
         "correction": "FETCH_SIZE x2 (gfx950 half-count of wide coalesced reads), KiB -> bytes",
         "source": f"profiles/{tag}/pmc_fetch_summary.csv, pmc_write_summary.csv"}
    cfg = os.environ.get("CFG", "c2")  # bench.py reads profiles/pmc_traffic_<config>.json
    for out in (os.path.join(dst, "pmc_traffic.json"), os.path.join("perf", f"pmc_traffic_{cfg}.json")):
        json.dump(t, open(out, "w"), indent=1)
    print("traffic", t["scan_bytes_per_launch"])
