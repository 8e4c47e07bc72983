#!/usr/bin/env python3
"""Diagnostic: kernel times of the chart pattern policies (C1-style workload scaled to
N pods, seed 0xC1) for the library named by KPE_LIB. Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import kyverno_amd as K  # noqa: E402
from tests.test_gpu_pattern import chart_pattern_policies  # noqa: E402


def main():
    n = int(os.environ.get("N", "1000000"))
    steps = int(os.environ.get("STEPS", "20"))
    mix = int(os.environ.get("MIX", "0"))
    eng = K.Engine(ordinal=0)
    c = K.Corpus(K.synth_resources(0xC1, n, mix=mix))
    c.upload(eng.device)
    ps = K.PolicySet(chart_pattern_policies())
    for _ in range(3):
        eng.evaluate_async(ps, c)
    eng.device.sync()
    eng.device.set_timing(True)
    eng.device.kernel_stats(reset=True)
    for _ in range(steps):
        eng.evaluate_async(ps, c)
    st = eng.device.kernel_stats(reset=True)
    per = lambda ms: 1e3 * ms / st.launches  # noqa: E731
    pat_us = per(st.pattern_kernel_ms)
    print(json.dumps({"lib": os.path.basename(K._lib.lib_path()), "n": n, "rules": ps.num_rules, "mix": mix,
                      "pattern_us": pat_us, "scan_us": per(st.pss_kernel_ms), "dict_us": per(st.dict_kernel_ms),
                      "pattern_cells_per_s": n * ps.num_rules / (pat_us * 1e-6),
                      "doc_nodes": c.doc_nodes if hasattr(c, "doc_nodes") else None}))


if __name__ == "__main__":
    main()
