#!/usr/bin/env python3
"""Headline benchmark: resource-rule evals/s, 1M synthetic Pods x PSS restricted
(BASELINE.json metric/configs[1]) per GPU, weak-scaled over N GPUs (one process
per GPU, resources sharded, no data-path collective; the per-rule counters are
all-reduced once over RCCL after the timed region).

One step = one evaluation pass of the compiled program over one 1M-Pod shard
resident in HBM (dictionary predicate pass + resource-scan kernel + counters).
`--replicas` distinct shards are rotated so consecutive steps do not re-read a
corpus out of the 256 MiB Infinity Cache.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--resources", type=int, default=1_000_000, help="Pods per GPU")
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="Pods in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import kyverno_amd as K
    from kyverno_amd.shard import COUNT_FIELDS, allreduce_counts, max_over_ranks
    from tests.policies import restricted_latest

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    eng = K.Engine(ordinal=local)
    policy = restricted_latest()
    ps = K.PolicySet([policy])
    R = ps.num_rules
    n = args.resources
    corpora = []
    t_setup = time.time()
    for k in range(args.replicas):
        # shard k of rank r: rows [(r*replicas + k)*n, ...) of one logical corpus (seed 0xC2)
        first = (rank * args.replicas + k) * n
        nd = K.synth_resources(0xC2, n, mix=0, first_index=first)
        c = K.Corpus(nd, docs=False)  # PSS only: no document tapes
        del nd
        c.upload(eng.device)
        corpora.append(c)
    t_setup = time.time() - t_setup
    # correctness touch + counters from one synchronous evaluation per replica
    totals = [dict.fromkeys(COUNT_FIELDS, 0) for _ in range(R)]
    for c in corpora:
        _, _, cnt = eng.evaluate(ps, c)
        for r in range(R):
            for f in COUNT_FIELDS:
                totals[r][f] += cnt[r][f]

    for i in range(args.warmup):
        eng.evaluate_async(ps, corpora[i % len(corpora)])
    eng.device.sync()
    eng.device.set_timing(True)
    eng.device.kernel_stats(reset=True)
    eng.device.set_timing(False)

    # ---- timed region: exactly K steps ----
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        eng.evaluate_async(ps, corpora[i % len(corpora)])
    eng.device.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    elapsed = max_over_ranks(elapsed, device="cuda")
    # the one real exchange: per-rule totals (R x 6 u64, RCCL over xGMI)
    totals = allreduce_counts(totals, device="cuda")
    total_fail = totals[0]["fail"]

    # ---- per-kernel timing pass (HIP events on the evaluation stream) ----
    eng.device.set_timing(True)
    for i in range(args.steps):
        eng.evaluate_async(ps, corpora[i % len(corpora)])
    st = eng.device.kernel_stats(reset=True)
    eng.device.set_timing(False)
    scan_ms = st.pss_kernel_ms / max(st.launches, 1)
    dict_ms = st.dict_kernel_ms / max(st.launches, 1)
    achieved = st.scan_bytes / (scan_ms * 1e-3) / 1e9

    ms_per_step = elapsed / args.steps * 1e3
    evals = float(n) * R * world * args.steps
    value = evals / elapsed

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get("scan_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from tests.oracle_lib import load as load_oracle

        orc = load_oracle()
        nd = K.synth_resources(0xC2, args.cpu_sample, mix=0)
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        t1 = time.perf_counter()
        ref = orc.validate([policy], nd, nthreads=thr)
        dt = time.perf_counter() - t1
        cpu = {"value": ref.size / dt, "unit": "resource-rule evals/s", "cores": thr, "kind": "port",
               "sample": f"{args.cpu_sample} C2 Pods x {R} rules (NDJSON parse + typed decode + evaluate), "
                         f"oracle/ CPU restatement, {thr} threads, {dt:.2f}s"}

    if rank == 0:
        line = {
            "metric": "resource-rule evals/sec, 1M Pods × PSS restricted, 1/8 GPU; % HBM BW",
            "value": value,
            "unit": "resource-rule evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (kpe_synth C2 generator, seed 0xC2)",
            "config": {"workload": "C2: 1M synthetic Pods x PSS restricted:latest per GPU (R=3 rules after autogen)",
                       "resources_per_gpu": n, "rules": R, "global_resources": n * world,
                       "replicas_rotated": args.replicas, "parallelism": f"resource-sharded x{world}",
                       "fail_fraction": total_fail / float(n * args.replicas * world),
                       "counts_rule0": totals[0]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "kpe_scan_kernel", "kernel_ms": scan_ms, "dict_kernel_ms": dict_ms,
                         # the same bytes over the timed region's step time (launches of
                         # different shards overlap on two streams there)
                         "achieved_per_step": st.scan_bytes / (ms_per_step * 1e-3) / 1e9,
                         "alg_bytes_per_launch": st.scan_bytes},
            "cpu_baseline": cpu,
            "setup_s": t_setup,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
