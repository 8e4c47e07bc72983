#!/usr/bin/env python3
"""Headline benchmark: resource-rule evals/s (BASELINE.json metric) per GPU, weak-scaled over N
GPUs (one process per GPU, resources sharded, no data-path collective; the per-rule counters
are all-reduced once over RCCL after the timed region).

--config c2 (default, the metric's configuration, BASELINE.json configs[1]): 1M synthetic Pods
    x the PSS restricted:latest policy (R = 3 rules after autogen) per GPU.
--config c3: a 1/8 shard (1.25M rows) of 10M mixed resources x 200 wildcard ClusterPolicies
    per GPU (configs[2]; the full 10M is the 8-GPU job).
--config c4: 5M Deployments + Services x the selector policy set (matchLabels with wildcards,
    matchExpressions, namespaceSelector over a 10k-namespace label table) per GPU (configs[3]).
--config c5: 1M Pods / Deployments with 1-64 containers x the require-requests-limits /
    disallow-latest-tag / host-ports / anchor pattern set per GPU (configs[4]).

One step = one evaluation pass of the compiled program over one resident shard
(kpe_evaluate_async: resource-scan kernel, then the condition / exclusion / pattern kernels when
the program has such rules); the K timed steps are enqueued by one kpe_evaluate_batch_async call,
which sends a run of LEAN steps (C2) as ceil(K / 24) multi-shard launches of kpe_lean6_kernel (one
grid over the steps' shards) and every other step as its own launch. Every C2 step reads each
pod's 16-byte record, its tile header and its container / volume / sysctl / annotation list items
and decides the 17 PSA checks from them: nothing per pod is carried from one step to the next.
What a step does not rebuild is per corpus DICTIONARY: one code byte per distinct capability set,
sysctl name and annotation key / value (kpe_psa_codes_kernel), like the interned ids themselves,
and the binding's kind table; the cold leg rebuilds those too. Distinct shards are rotated so that
the bytes a step reads were last touched more than twice the 256 MiB Infinity Cache ago (the count
is derived from the algorithmic bytes of one step, `--replicas` overrides). Per-rule counters are
built once, after the timed region (kpe_fetch), not per step.
"""
import math
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
IC_BYTES = 256 << 20  # MI355X Infinity Cache (MALL)
# kpe_kernel_stats.scan_kernel -> kernel name (as rocprofv3 lists it)
SCAN_KERNELS = {1: "kpe_scan_kernel", 2: "kpe_scan_kernel", 7: "kpe_lean6_kernel", 9: "kpe_lean6_kernel"}


def scan_accounting(launches, kernel_ms_sum, bytes_sum, steps, ms_per_step, replicas):
    """Algorithmic-byte accounting of the timed steps' scan launches (pure arithmetic, tested on
    CPU in tests/test_bench_accounting.py). A multi-shard kpe_lean6_kernel launch carries a
    different number of steps than its neighbours (ceil(K / 24) launches over K steps), so the
    bytes are SUMMED over the launches and the time too: achieved = sum of bytes / sum of kernel
    time, the mean launch = sum / launches, and one step (one shard) = sum / K at any K."""
    L = max(int(launches), 1)
    per_step = bytes_sum / steps if steps else 0.0
    kernel_ms = kernel_ms_sum / L
    return {"launches": int(launches),
            "alg_bytes_per_launch": bytes_sum / L,  # the mean launch
            "alg_bytes_per_step": per_step,         # one shard's evaluation
            "kernel_ms": kernel_ms,
            "achieved_gbs": bytes_sum / (kernel_ms_sum * 1e-3) / 1e9 if kernel_ms_sum > 0 else 0.0,
            "achieved_per_step_gbs": per_step / (ms_per_step * 1e-3) / 1e9 if ms_per_step > 0 else 0.0,
            # the bytes read between two uses of one shard (each step evaluates one shard)
            "rotated_scan_bytes": per_step * replicas}


def cpu_budget():
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2 / v1 CPU quota
    (a GPU box grants each job a share of a larger machine: os.cpu_count() is the machine)."""
    machine = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = machine
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            quota = None
    usable = max(1, min(aff, math.floor(quota) if quota else aff))
    return {"machine": machine, "affinity": aff, "cgroup_quota": quota, "usable": usable}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _rank_main(rank, world, argv):
    """A rank started by launch_ranks: the torchrun environment, then the bench."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      GROUP_RANK="0")
    main(argv)


def spawn_check():
    """Each rank joins the process group and all-reduces its rank; rank 0 prints the result."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(os.environ.get("KPE_DIST_BACKEND", "gloo"))
    t = torch.tensor([rank], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"spawn_check": True, "n_gpus": world, "rank_sum": int(t.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def launch_ranks(world, argv):
    """`--gpus N` without an external launcher: N rank processes on this node, one per GPU, started
    with the spawn method before this process makes any GPU call (a child process each, never an
    exec of this one); rendezvous over 127.0.0.1. A failing rank fails the run."""
    import torch.multiprocessing as mp

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    mp.start_processes(_rank_main, args=(world, argv), nprocs=world, start_method="spawn", join=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); without an external launcher "
                                                        "(WORLD_SIZE unset) bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=("c2", "c3", "c4", "c5"), default="c2")
    ap.add_argument("--resources", type=int, default=0, help="rows per GPU (0 = the config's size)")
    ap.add_argument("--replicas", type=int, default=0, help="distinct shards rotated (0 = the config's default)")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="rows in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use (cpu_budget)")
    ap.add_argument("--traffic-json", default="")
    ap.add_argument("--total-resources", type=int, default=0,
                    help="strong scaling: this many rows in all, split over the ranks (C3 10M over 8 GPUs)")
    ap.add_argument("--spawn-check", action="store_true",
                    help="start the ranks, all-reduce their ids over the process group and exit (CPU check)")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:  # no external launcher: start the ranks here
        return launch_ranks(args.gpus, sys.argv[1:] if argv is None else argv)
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
    if args.spawn_check:
        return spawn_check()

    import numpy as np  # noqa: F401
    import torch
    import torch.distributed as dist

    import kyverno_amd as K
    from kyverno_amd.shard import COUNT_FIELDS, allreduce_counts, gather_packed, max_over_ranks, shard_range
    from tests.policies import c3_policy_set, c4_policy_set, c5_policy_set, restricted_latest

    cfg = args.config
    if cfg == "c2":
        policies, mix, seed, n_def, rep_def, docs = [restricted_latest()], K.SYNTH_PODS, 0xC2, 1_000_000, 0, False
        workload = "C2: 1M synthetic Pods x PSS restricted:latest per GPU (R=3 rules after autogen)"
    elif cfg == "c3":
        policies, mix, seed, n_def, rep_def, docs = c3_policy_set(), K.SYNTH_C3, 0xC3, 1_250_000, 1, True
        workload = ("C3: 1/8 shard (1.25M rows) of 10M mixed resources x 200 wildcard ClusterPolicies per GPU")
    elif cfg == "c4":
        policies, mix, seed, n_def, rep_def, docs = c4_policy_set(), K.SYNTH_SELECTORS, 0xC4, 5_000_000, 1, False
        workload = ("C4: 5M Deployments + Services x selector policies (namespaceSelector over 10k namespaces) "
                    "per GPU")
    else:
        policies, mix, seed, n_def, rep_def, docs = c5_policy_set(), K.SYNTH_FANOUT, 0xC5, 1_000_000, 1, True
        workload = "C5: 1M Pods/Deployments with 1-64 containers x requests-limits/latest-tag/host-ports/anchor patterns"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    n = args.resources or n_def
    first = None  # strong scaling: this rank's first row of the --total-resources corpus
    if args.total_resources:
        # (C2 keeps its derived replica count: copies of the rank's row range are rotated so the
        # steps stay HBM-bound; the others rotate one shard)
        first, n = shard_range(args.total_resources, rank, world)
        workload = (f"{cfg.upper()}: {args.total_resources} rows in all, split over {world} GPU(s) "
                    f"(contiguous row ranges); " + workload.split(": ", 1)[1].split(" per GPU")[0])
    n_all = args.total_resources or n * world
    if args.replicas:
        replicas = args.replicas
    elif rep_def:
        replicas = rep_def
    else:  # C2: enough shards that a shard's scan bytes leave the Infinity Cache before its next use
        alg = 43.0 * n  # LEAN6 on the C2 mix: ~40 B of pod record, header and list items read, R = 3 written
        replicas = max(2, math.ceil(2.25 * IC_BYTES / alg))
    # HBM bytes per scan launch from the FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_summary.py);
    # perf/ travels to the GPU box, profiles/ does not
    traffic_json = args.traffic_json or os.path.join(ROOT, "perf", f"pmc_traffic_{cfg}.json")

    # One rank per GPU over RCCL. KPE_DIST_BACKEND=gloo runs the collectives on host tensors: a
    # functional check of the N-rank path with several ranks sharing one device (RCCL refuses two
    # ranks on one GPU); ranks then take device LOCAL_RANK modulo the visible devices.
    backend = os.environ.get("KPE_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    coll_dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    def barrier():
        if world > 1:
            dist.barrier()

    eng = K.Engine(ordinal=local)
    ps = K.PolicySet(policies)
    R = ps.num_rules
    corpora = []
    t_flatten = t_upload = 0.0
    nsl = K.synth_ns_labels(seed, 10000, mix=mix) if cfg == "c4" else None
    from concurrent.futures import ThreadPoolExecutor

    # shard k of rank r: rows [(r*replicas + k)*n, ...) of one logical corpus; the synthetic NDJSON
    # of the next shards is generated on two threads while this one is flattened and uploaded
    with ThreadPoolExecutor(max_workers=2) as pool:
        futs = [pool.submit(K.synth_resources, seed, n, mix, first if first is not None else (rank * replicas + k) * n)
                for k in range(replicas)]
        for k in range(replicas):
            nd = futs[k].result()
            futs[k] = None
            t0 = time.perf_counter()
            c = K.Corpus(nd, namespace_labels=nsl, docs=docs)
            t1 = time.perf_counter()
            c.upload(eng.device)
            t2 = time.perf_counter()
            del nd  # (releasing the NDJSON's pages is not upload time)
            t_flatten += t1 - t0
            t_upload += t2 - t1
            corpora.append(c)
            if rank == 0 and (k % 4 == 3 or k == replicas - 1):
                print(f"[bench] {k + 1}/{replicas} shards of {n} rows flattened and uploaded", file=sys.stderr, flush=True)
    # the first binding of shard 0 (the end-to-end legs run after the timed region)
    eng.evaluate_async(ps, corpora[0])
    eng.device.sync()
    # correctness touch + counters from one synchronous evaluation per replica
    totals = [dict.fromkeys(COUNT_FIELDS, 0) for _ in range(R)]
    for c in corpora:
        _, _, cnt = eng.evaluate(ps, c)
        for r in range(R):
            for f in COUNT_FIELDS:
                totals[r][f] += cnt[r][f]

    # warm-up: every shard at least once (first binding: program upload, prologue image, PSA
    # summaries), then W more steps
    for i in range(len(corpora) + args.warmup):
        eng.evaluate_async(ps, corpora[i % len(corpora)])
    eng.device.sync()

    # ---- timed region: exactly K steps, enqueued by one call (kpe_evaluate_batch_async) ----
    steps_batch = eng.batch([corpora[i % len(corpora)] for i in range(args.steps)])
    # untimed: one rotation over every shard, in the timed region's order, so that each timed
    # step's shard was last read a whole rotation earlier (see the module docstring)
    rotation = eng.batch(corpora)
    eng.evaluate_batch_async(ps, rotation)
    eng.device.sync()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.evaluate_batch_async(ps, steps_batch)
    torch.cuda.synchronize()  # hipDeviceSynchronize: every stream of the device, the library's included
    elapsed = time.perf_counter() - t0
    barrier()
    elapsed = max_over_ranks(elapsed, device=coll_dev)
    # the exchanges, after the timed region: per-rule totals (R x 7 u64, one RCCL all-reduce over
    # xGMI) and the verdict matrix of each rank's first shard, packed on its GPU to 3-bit cells
    # and sent from HBM to rank 0 (grouped RCCL point-to-point: one send per rank, all receives
    # posted together on rank 0, unpacked there)
    totals = allreduce_counts(totals, device=coll_dev)
    eng.evaluate_async(ps, corpora[0])
    eng.device.sync()
    barrier()
    t1 = time.perf_counter()
    full = gather_packed(eng, ps, corpora[0], n_all, dst=0, device=coll_dev)
    torch.cuda.synchronize()
    gather_s = max_over_ranks(time.perf_counter() - t1, device=coll_dev)
    gather = {"rows": n_all, "bytes": sum(4 * K.packed_words(shard_range(n_all, r, world)[1] * R) for r in range(world)),
              "cell_bits": 3, "seconds": gather_s, "backend": backend if world > 1 else None,
              "rows_ok": bool(rank != 0 or (full is not None and full.shape == (n_all, R)))}

    # ---- per-kernel timing pass: the timed region's K steps again, with HIP events around every
    # launch on the library's stream (launches serialised there, so each duration is its own; a
    # multi-shard LEAN launch covers several steps) ----
    eng.evaluate_batch_async(ps, rotation)
    eng.device.sync()
    eng.device.set_timing(True)
    eng.device.kernel_stats(reset=True)
    t1 = time.perf_counter()
    eng.evaluate_batch_async(ps, steps_batch)
    st = eng.device.kernel_stats(reset=True)
    single_stream_ms = (time.perf_counter() - t1) / args.steps * 1e3
    L = max(st.launches, 1)
    ms_per_step = elapsed / args.steps * 1e3
    acct = scan_accounting(st.launches, st.pss_kernel_ms, st.scan_bytes_sum, args.steps, ms_per_step, replicas)
    step_bytes = acct["alg_bytes_per_step"]
    scan_ms = acct["kernel_ms"]
    dict_ms = st.dict_kernel_ms / L
    pat_ms = st.pattern_kernel_ms / L
    scan_achieved = acct["achieved_gbs"]
    # spread of the timed region's scan launches (HIP events, one stream): mean, std, min, max
    scan_std = math.sqrt(max(0.0, st.pss_kernel_ms_sq / L - scan_ms * scan_ms)) if st.launches else 0.0
    scan_spread = {"launches": st.launches, "mean_ms": scan_ms, "std_ms": scan_std, "min_ms": st.pss_kernel_ms_min,
                   "max_ms": st.pss_kernel_ms_max, "std_over_mean": scan_std / scan_ms if scan_ms > 0 else 0.0}

    # ---- the masks-producing instantiation (what a report needs for each FAIL cell's PSS
    # checks) and a cold step (per-corpus prologue re-run: dictionary predicate pass + prologue
    # image, as the first evaluation of a newly bound corpus), wall-clock and per kernel ----
    def leg(serial=False, batch=False, **kw):
        """serial: one evaluation at a time (enqueue, wait), i.e. one 1M-row shard's latency;
        batch: the K / 4 steps through kpe_evaluate_batch_async (multi-shard launches);
        otherwise per-evaluation launches enqueued back to back (two streams)."""
        for c in corpora:  # mode switch (argument block upload, masks buffer allocation) untimed
            eng.evaluate_async(ps, c, **kw)
        eng.device.sync()
        eng.device.set_timing(False)
        ks = max(1, args.steps // 4)
        sub = eng.batch([corpora[i % len(corpora)] for i in range(ks)]) if batch else None

        def run():
            if batch:
                eng.evaluate_batch_async(ps, sub, **kw)
                return
            for i in range(ks):
                eng.evaluate_async(ps, corpora[i % len(corpora)], **kw)
                if serial:
                    eng.device.sync()

        if batch:  # rotation first, as the timed region does
            eng.evaluate_batch_async(ps, rotation, **kw)
            eng.device.sync()
        t1 = time.perf_counter()
        run()
        eng.device.sync()
        wall = (time.perf_counter() - t1) / ks * 1e3
        eng.device.set_timing(True)
        eng.device.kernel_stats(reset=True)
        run()
        k = eng.device.kernel_stats(reset=True)
        a = scan_accounting(k.launches, k.pss_kernel_ms, k.scan_bytes_sum, ks, wall, replicas)
        kl = max(k.launches, 1)
        return {"ms_per_step": wall, "evals_per_s": float(n) * R / (wall * 1e-3), "steps": ks,
                "launches": k.launches, "scan_kernel_ms": a["kernel_ms"], "prologue_ms": k.dict_kernel_ms / kl,
                "later_kernels_ms": k.pattern_kernel_ms / kl, "scan_bytes_per_launch": a["alg_bytes_per_launch"],
                "scan_bytes_per_step": a["alg_bytes_per_step"], "scan_frac": a["achieved_gbs"] / HBM_PEAK_GBS}

    single_leg = leg(serial=True)               # one shard, no masks: the single-corpus latency
    masks_leg = leg(masks=True)                 # per-evaluation launches with check masks
    masks_batch_leg = leg(masks=True, batch=True)  # the same through the multi-shard launches
    cold_leg = leg(masks=True, cold=True)
    eng.device.set_timing(False)

    evals = float(n_all) * R * args.steps
    value = evals / elapsed

    traffic = None
    scan_kernel = SCAN_KERNELS.get(st.scan_kernel, "kpe_scan_kernel")
    if os.path.exists(traffic_json):
        try:
            tj = json.load(open(traffic_json))
            # only counters taken on the kernel this run launched (a stale file is not this kernel's)
            norm = lambda k: k.split("(")[0].replace("void ", "").replace(" ", "").split("<")[0]  # noqa: E731
            if norm(tj.get("kernel", "")) == norm(scan_kernel) or (
                    scan_kernel == "kpe_scan_kernel" and norm(tj.get("kernel", "")).startswith("kpe_scan_kernel")):
                # counter bytes over the algorithmic bytes of the same launches, applied to this run's
                # launches (a multi-shard launch's size follows K); else the pass's bytes as they are
                ratio = tj.get("traffic_ratio")
                traffic = ratio * acct["alg_bytes_per_launch"] if ratio else tj.get("scan_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    sample = args.cpu_sample if args.cpu_sample >= 0 else {"c2": 1_000_000, "c3": 200_000, "c4": 200_000,
                                                           "c5": 100_000}[cfg]
    if rank == 0 and world == 1 and sample > 0:
        from tests.oracle_lib import load as load_oracle

        orc = load_oracle()
        nd = K.synth_resources(seed, sample, mix=mix)
        nsl_s = K.synth_ns_labels(seed, 10000, mix=mix) if cfg == "c4" else None
        budget = cpu_budget()
        thr = args.cpu_threads or budget["usable"]
        t1 = time.perf_counter()
        ref = orc.validate(policies, nd, ns_labels=nsl_s, nthreads=thr)
        dt = time.perf_counter() - t1
        # single-thread leg on a 1/8 sub-sample (bounded run time)
        sub = b"\n".join(nd.split(b"\n")[: max(1, sample // 8)])
        t1 = time.perf_counter()
        ref1 = orc.validate(policies, sub, ns_labels=nsl_s, nthreads=1)
        dt1 = time.perf_counter() - t1
        cpu = {"value": ref.size / dt, "unit": "resource-rule evals/s", "cores": thr, "kind": "port",
               "single_thread_value": ref1.size / dt1, "cpu_model": cpu_model(), "cpu_budget": budget,
               "sample": f"{sample} {cfg.upper()} rows x {R} rules (NDJSON parse + typed decode + evaluate), "
                         f"oracle/ CPU restatement, {thr} threads {dt:.2f}s; single-thread leg "
                         f"{max(1, sample // 8)} rows {dt1:.2f}s"}

    if rank == 0:
        scan_roof = {"bound": "hbm", "achieved": scan_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": scan_achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": scan_kernel,
                     "kernel_ms": scan_ms, "alg_bytes_per_launch": acct["alg_bytes_per_launch"],
                     "kernel_spread": scan_spread, "dict_kernel_ms": dict_ms,
                     "pattern_kernel_ms": pat_ms,
                     # the same bytes over the timed region's step time (launches of different
                     # shards overlap on two streams there) and the isolated single-stream step
                     "launches": st.launches, "alg_bytes_per_step": step_bytes,
                     "achieved_per_step": acct["achieved_per_step_gbs"],
                     "single_stream_step_ms": single_stream_ms,
                     "note": ("kernel_ms: HIP events per launch, launches serialised on one stream "
                              "(kpe_lean6_kernel over several shards: one launch over up to 24 shards, i.e. "
                              "several steps, alg_bytes_per_launch the mean launch's shards' bytes (summed over "
                              "the launches / launches): pod records, tile headers, "
                              "container / volume / sysctl / annotation items, code bytes, verdicts); other kernels: "
                              "one launch per step, and consecutive shards' launches overlap on two streams in the "
                              "timed region; dict / pattern kernel ms are 0 when no such kernel ran")}
        if pat_ms > scan_ms and st.pattern_bytes > 0:
            # pattern-dominated configurations (C3, C5): the dominant kernel is the pattern VM;
            # its algorithmic bytes are every resource's document tape once plus the verdicts
            pat_sum = st.pattern_bytes_sum or st.pattern_bytes * L
            pat_achieved = pat_sum / (st.pattern_kernel_ms * 1e-3) / 1e9
            pat_traffic = None
            try:  # FETCH_SIZE / WRITE_SIZE of the pattern kernel (scripts/gpu_pass.sh traffic:<cfg>:kpe_pattern_kernel)
                tj = json.load(open(traffic_json))
                if tj.get("kernel", "").split("<")[0] == "kpe_pattern_kernel":  # either LT instance
                    pat_traffic = tj.get("scan_bytes_per_launch")
            except Exception:
                pat_traffic = None
            scan_roof = {"bound": "hbm", "achieved": pat_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": pat_achieved / HBM_PEAK_GBS, "traffic": pat_traffic, "kernel": "kpe_pattern_kernel",
                         "kernel_ms": pat_ms, "alg_bytes_per_launch": pat_sum / L,
                         "scan_kernel": {"kernel_ms": scan_ms, "alg_bytes_per_launch": acct["alg_bytes_per_launch"],
                                         "kernel_spread": scan_spread,
                                         "frac": scan_achieved / HBM_PEAK_GBS},
                         "single_stream_step_ms": single_stream_ms}
        # end-to-end ingestion of shard 0's NDJSON again (generated untimed, nothing else running):
        # serially (flatten the whole shard, H2D, one evaluation), then as a pipeline of row chunks
        nd0 = K.synth_resources(seed, n, mix, first if first is not None else 0)
        t0 = time.perf_counter()
        c0 = K.Corpus(nd0, namespace_labels=nsl, docs=docs)
        t1 = time.perf_counter()
        c0.upload(eng.device)
        t2 = time.perf_counter()
        eng.evaluate_async(ps, c0)
        eng.device.sync()
        t3 = time.perf_counter()
        del c0
        e2e_flat, e2e_up, t_eval1 = t1 - t0, t2 - t1, t3 - t2
        e2e_s = t3 - t0
        del nd0
        line = {
            "metric": "resource-rule evals/sec, 1M Pods × PSS restricted, 1/8 GPU; % HBM BW",
            "value": value,
            "unit": "resource-rule evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if args.total_resources else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic (kpe_synth {cfg.upper()} generator, seed {seed:#x})",
            "config": {"workload": workload, "resources_per_gpu": n, "rules": R, "global_resources": n_all,
                       "replicas_rotated": replicas, "parallelism": f"resource-sharded x{world}",
                       # scan bytes touched between two uses of one shard vs the Infinity Cache
                       "rotated_scan_bytes": acct["rotated_scan_bytes"], "infinity_cache_bytes": IC_BYTES,
                       "rotation_exceeds_infinity_cache": acct["rotated_scan_bytes"] >= 2 * IC_BYTES,
                       # cells where the rule matched the resource (a RuleResponse exists), per s
                       "matched_cell_evals_per_s": value * sum(n_all * replicas - totals[r]["na"]
                                                               for r in range(R)) / float(n_all * replicas * R),
                       "counts_rule0": totals[0]},
            "roofline": scan_roof,
            "cpu_baseline": cpu,
            "gather": gather,
            "single_shard_step": single_leg,
            "masks_step": masks_leg,
            "masks_batch_step": masks_batch_leg,
            "cold_masks_step": cold_leg,
            "e2e": {"e2e_evals_per_s": float(n) * R / e2e_s, "flatten_s": e2e_flat,
                    "upload_s": e2e_up, "first_eval_s": t_eval1,
                    "setup_flatten_s": t_flatten / replicas, "setup_upload_s": t_upload / replicas,
                    "note": "one shard, after the timed region: host flatten (NDJSON -> columns) + H2D + one evaluation (a new binding), not in value; setup_*: the setup's per-shard means (NDJSON generation ran beside them)",
                    # (round 6: the 8-chunk pipelined leg is gone: with the upload and the
                    # evaluation at ~6 ms of a ~0.25 s shard there is nothing for the flatten to hide
                    # behind, and it measured the same as this serial leg, profiles/r06_d)
                    },
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
