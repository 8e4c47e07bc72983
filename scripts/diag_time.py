#!/usr/bin/env python3
"""Diagnostic: scan-kernel time on the C2 workload for the library named by KPE_LIB
(a normal or a -DKPE_DIAG=N build, scripts/diag_variants.sh). Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import kyverno_amd as K  # noqa: E402
from tests.policies import restricted_latest  # noqa: E402


def main():
    n = int(os.environ.get("N", "1000000"))
    steps = int(os.environ.get("STEPS", "50"))
    eng = K.Engine(ordinal=0)
    corpora = []
    for k in range(int(os.environ.get("REPLICAS", "8"))):  # 8 x 41 MB: past the 256 MB Infinity Cache
        c = K.Corpus(K.synth_resources(0xC2, n, mix=0, first_index=k * n), docs=False)
        c.upload(eng.device)
        corpora.append(c)
    ps = K.PolicySet([restricted_latest()])
    for i in range(8):
        eng.evaluate_async(ps, corpora[i % len(corpora)])
    eng.device.sync()
    eng.device.set_timing(True)
    eng.device.kernel_stats(reset=True)
    for i in range(steps):
        eng.evaluate_async(ps, corpora[i % len(corpora)])
    st = eng.device.kernel_stats(reset=True)
    print(json.dumps({"lib": os.path.basename(K._lib.lib_path()), "scan_us": 1e3 * st.pss_kernel_ms / st.launches,
                      "dict_us": 1e3 * st.dict_kernel_ms / st.launches}))


if __name__ == "__main__":
    main()
