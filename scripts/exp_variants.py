#!/usr/bin/env python3
"""Scan-kernel cost breakdown on 1M C2 Pods under program variants (rule count,
PSS vs match-only), from HIP-event kernel timings. Diagnostic only."""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import kyverno_amd as K  # noqa: E402
from tests.policies import pss_policy, restricted_latest  # noqa: E402


def no_autogen(p):
    p = copy.deepcopy(p)
    p["metadata"].setdefault("annotations", {})["pod-policies.kyverno.io/autogen-controllers"] = "none"
    return p


def match_only(name, kinds):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"rules": [{"name": name, "match": {"any": [{"resources": {"kinds": kinds}}]},
                                "mutate": {"patchStrategicMerge": {"metadata": {"labels": {"x": "y"}}}}}]}}


def main():
    n = int(os.environ.get("N", "1000000"))
    eng = K.Engine(ordinal=0)
    corpora = []
    for k in range(2):
        c = K.Corpus(K.synth_resources(0xC2, n, mix=0, first_index=k * n))
        c.upload(eng.device)
        corpora.append(c)
    variants = {
        "restricted_latest_R3": [restricted_latest()],
        "restricted_latest_R1": [no_autogen(restricted_latest())],
        "baseline_latest_R3": [pss_policy("b", "baseline", "latest")],
        "restricted_v1.24_R3": [pss_policy("r", "restricted", "v1.24")],
        "match_only_R1": [match_only("m", ["Pod"])],
        "restricted_latest_x20_R60": [dict(restricted_latest(), metadata={"name": f"p{i}"}) for i in range(20)],
    }
    out = {}
    for name, pols in variants.items():
        ps = K.PolicySet(pols)
        for i in range(5):
            eng.evaluate_async(ps, corpora[i % 2])
        eng.device.sync()
        eng.device.set_timing(True)
        eng.device.kernel_stats(reset=True)
        for i in range(40):
            eng.evaluate_async(ps, corpora[i % 2])
        st = eng.device.kernel_stats(reset=True)
        eng.device.set_timing(False)
        out[name] = {"R": ps.num_rules, "scan_us": 1e3 * st.pss_kernel_ms / st.launches,
                     "pred_us": 1e3 * st.dict_kernel_ms / st.launches, "alg_MB": st.scan_bytes / 1e6}
        print(name, json.dumps(out[name]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "exp_variants.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
