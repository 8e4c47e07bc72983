#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    pmc_summary.py --dir <rocprofv3 -d dir> --kernel <name prefix> --out <json>

Reads every *counter_collection.csv under --dir (one pass per counter: a TCC block cannot hold both,
MI355X_MICROARCH.md), takes each counter's median over the dispatches of the kernels whose name
starts with --kernel (a pass's bench run also launches other legs of the same kernel, e.g. the
masks mode), and writes {fetch, write, bytes per launch}. Units: FETCH_SIZE / WRITE_SIZE are KiB;
gfx950 correction (MI355X_MICROARCH.md § HBM): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is. bench.py reports the result
as roofline.traffic when its kernel is the one measured (perf/pmc_traffic_<config>.json).
Also writes a per-kernel / per-counter mean table next to the json (<out>.csv)."""
import argparse
import collections
import csv
import glob
import json
import os


def norm(k):
    return k.split("(")[0].replace("void ", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--bench-log", default="", help="the pass's bench.py output: its roofline.alg_bytes_per_launch "
                                                     "(the same launches) gives traffic / algorithmic bytes")
    a = ap.parse_args()
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[(norm(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    with open(os.path.splitext(a.out)[0] + ".csv", "w") as o:
        o.write("kernel,counter,mean_per_dispatch,dispatches\n")
        for (k, c), v in sorted(agg.items()):
            o.write(f'"{k}",{c},{sum(v) / len(v):.1f},{len(v)}\n')

    def mean(counter):  # the median dispatch: a pass mixes leg kinds (e.g. masks-mode launches)
        vals, names = [], set()
        for (k, c), v in agg.items():
            if c == counter and k.startswith(a.kernel):
                vals += v
                names.add(k)
        return (sorted(vals)[len(vals) // 2], len(vals), sorted(names)) if vals else None

    fm, wm = mean("FETCH_SIZE"), mean("WRITE_SIZE")
    if fm is None or wm is None:
        raise SystemExit(f"no FETCH_SIZE / WRITE_SIZE dispatches of {a.kernel} under {a.dir}")
    t = {"kernel": fm[2][0], "fetch_kib_raw": fm[0], "write_kib_raw": wm[0], "dispatches": [fm[1], wm[1]],
         "fetch_bytes_corrected": fm[0] * 1024 * 2, "write_bytes": wm[0] * 1024,
         "scan_bytes_per_launch": fm[0] * 1024 * 2 + wm[0] * 1024,
         "correction": "FETCH_SIZE x2 (gfx950 half-count of wide coalesced reads), KiB -> bytes",
         "source": a.dir}
    if a.bench_log and os.path.exists(a.bench_log):
        for line in open(a.bench_log):
            if line.startswith("{"):
                alg = (json.loads(line).get("roofline") or {}).get("alg_bytes_per_launch")
                if alg:  # bench.py scales this ratio to its own launches' algorithmic bytes
                    t["alg_bytes_per_launch"] = alg
                    t["traffic_ratio"] = t["scan_bytes_per_launch"] / alg
    json.dump(t, open(a.out, "w"), indent=1)
    print("traffic", t["kernel"], t["scan_bytes_per_launch"])


if __name__ == "__main__":
    main()
