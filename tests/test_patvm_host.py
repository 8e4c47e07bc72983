"""The pattern VM's device source (kyverno_amd/csrc/patvm.inl + strmatch.inl) compiled for
the host with AddressSanitizer/UBSan and bounds flags (scripts/patvm_check.cpp), run over
the chart policies, the validate_test.go trees, the test/cli/test scenarios and the edge
documents. Every cell the oracle applies must agree; no bounds flag may be raised. CPU only:
this keeps the exact kernel logic under test without a GPU."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K
from tests.test_gpu_pattern import CLI, PTREE, _policy_for, chart_pattern_policies, device_policies, edge_case_inputs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "scripts", "build", "patvm_check")


@pytest.fixture(scope="module")
def harness():
    from tests.conftest import build_host_tool

    build_host_tool("patvm_check")
    return BIN


def pattern_only(pols):  # the harness runs the pattern VM alone (no deny / foreach / preconditions)
    return [q for q in pols if not any((r.get("validate") or {}).get("deny") is not None or r.get("preconditions")
                                      or (r.get("validate") or {}).get("foreach") for r in q["spec"]["rules"])]


def _sets():
    out = [("chart-mix0", pattern_only(chart_pattern_policies()), K.synth_resources(0xC1, 1500, mix=0)),
           ("chart-mix2", pattern_only(chart_pattern_policies()), K.synth_resources(22, 1500, mix=2))]
    pols, nd = edge_case_inputs(1500)
    out.append(("edge", pols, nd))
    # C3's 200 policies share a handful of patterns: the memo slots (PR_MEMO_SH) carry verdicts
    from tests.policies import c3_policy_set
    c3p = [q for q in c3_policy_set(60) if "pattern" in q["spec"]["rules"][0]["validate"]]
    out.append(("c3-memo", c3p, K.synth_resources(0xC3, 1500, mix=5)))
    cases = [c for c in PTREE if isinstance(json.loads(c["resource"]), dict)]
    pols = pattern_only(device_policies([_policy_for(f"t{i}", json.loads(c["pattern"])) for i, c in enumerate(cases)]))
    out.append(("validate_test.go", pols, "\n".join(json.dumps(json.loads(c["resource"])) for c in cases).encode()))

    for c in CLI:
        p = pattern_only(device_policies(c["policies"]))
        if p and c["resources"]:
            out.append((c["name"], p, "\n".join(json.dumps(r) for r in c["resources"]).encode()))
    return out


SETS = _sets()


@pytest.mark.parametrize("name,pols,nd", SETS, ids=[s[0] for s in SETS])
def test_patvm_host_matches_oracle(harness, oracle, tmp_path, name, pols, nd):
    pj, rj, vb = tmp_path / "p.json", tmp_path / "r.ndjson", tmp_path / "v.bin"
    pj.write_text(json.dumps(pols))
    rj.write_bytes(nd)
    r = subprocess.run([harness, str(pj), str(rj), str(vb)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    ref = oracle.validate(pols, nd)
    v = np.fromfile(vb, dtype=np.uint8).reshape(ref.shape)
    # the harness resolves every pattern cell as if its rule matched; rows whose policy context
    # fails (images, KPE_ROW_CONTEXT_ERROR: every oracle cell 7) are not the pattern VM's
    applied = (ref != 0) & ~(ref == 7).all(axis=1, keepdims=True)
    bad = np.argwhere((v != ref) & applied)
    assert bad.size == 0, f"{len(bad)} cells differ, first {bad[:5].tolist()}"


def _nest(depth, leaf, side=None):
    v = leaf
    for _ in range(depth):
        v = {"a": v} if side is None else {"a": v, "b": side}
    return v


def test_caps_are_undecided_cells(harness, oracle, tmp_path):
    """Past the lane's frame stack (pattern and resource both nested deeper) or past the 32
    AnchorMap slots, a cell is KPE_UNDECIDED (7) instead of the policy being refused; every
    other cell stays bit-exact. A chain of one-member maps needs no frames (schema.h PNW_CHAIN):
    as deep, it is decided."""
    deep = _policy_for("deep", {"spec": _nest(16, {"x": "1"}, side="*")})
    many = _policy_for("many", {"spec": {**{f"(k{i})": "v*" for i in range(34)}, "x": "?*"}})
    chain = _policy_for("chain", {"spec": _nest(16, {"x": "1"})})
    docs = []
    for i in range(40):
        spec = _nest(16, {"x": str(i % 3)}, side="s") if i % 4 == 0 else ({"a": "flat"} if i % 4 == 1 else None)
        d = {"apiVersion": "v1", "kind": "Thing", "metadata": {"name": f"d{i}"}}
        if spec is not None:
            d["spec"] = dict(spec, **({f"k{j}": "v1" for j in range(i % 5)} if i % 4 == 1 else {}))
        docs.append(d)
    nd = "\n".join(json.dumps(d) for d in docs).encode()
    pols = [deep, many, chain]
    pj, rj, vb = tmp_path / "p.json", tmp_path / "r.ndjson", tmp_path / "v.bin"
    pj.write_text(json.dumps(pols))
    rj.write_bytes(nd)
    r = subprocess.run([harness, str(pj), str(rj), str(vb)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    ref = oracle.validate(pols, nd)
    v = np.fromfile(vb, dtype=np.uint8).reshape(ref.shape)
    und = v == 7
    assert (v[~und] == ref[~und]).all()
    deep_rows = np.array([i % 4 == 0 for i in range(len(docs))])
    assert und[:, 0].tolist() == deep_rows.tolist()  # only resources as deep as the pattern
    has_spec = np.array([d.get("spec") is not None for d in docs])
    assert und[:, 1].tolist() == has_spec.tolist()  # any resource whose spec map is visited
    assert not und[:, 2].any() and (ref[:, 2] == 2).sum() >= 10  # the chain walk: every cell decided
