#!/usr/bin/env python3
"""Diagnostic: chart pattern policies over N synthetic resources with the library named by
KPE_LIB (normally build/diag/libkpe_pvchk.so: bounds-flagged pattern VM); KPE_PATVM_ERR=1
makes the library print the VM's bounds flags after each launch. Compares with the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import kyverno_amd as K  # noqa: E402
from tests.oracle_lib import load  # noqa: E402
from tests.test_gpu_pattern import chart_pattern_policies  # noqa: E402


def main():
    n = int(os.environ.get("N", "20000"))
    mix = int(os.environ.get("MIX", "0"))
    seed = int(os.environ.get("SEED", str(0xC1)))
    pols = chart_pattern_policies()
    nd = K.synth_resources(seed, n, mix=mix)
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = load().validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    print(f"lib={os.path.basename(K._lib.lib_path())} n={n} mix={mix} mismatches={len(bad)} first={bad[:5].tolist()}",
          flush=True)


if __name__ == "__main__":
    main()
