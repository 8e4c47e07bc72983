"""The condition VM (kyverno_amd/csrc/condvm.inl, kpe_cond_kernel's lane body) compiled for the
host under ASan/UBSan (scripts/condvm_check.cpp) against the oracle, no GPU needed: the scan
kernel's part (which cells match) is seeded from the rules' kinds."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import cond_policy_set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "scripts", "build", "condvm_check")
PRE_ONLY = {"pre-ns", "pre-kind-pss"}  # other handlers behind per-resource preconditions


@pytest.fixture(scope="module")
def condvm_bin():
    from tests.conftest import build_host_tool

    build_host_tool("condvm_check")
    return BIN


@pytest.mark.parametrize("mix,seed", [(2, 0xB1), (1, 0xB2)])
def test_condvm_host_matches_oracle(condvm_bin, oracle, tmp_path, mix, seed):
    pols = cond_policy_set()
    rules = pols[0]["spec"]["rules"]
    keep = {"Pod", "Deployment", "Service", "ConfigMap"}
    lines = [l for l in K.synth_resources(seed, 2500, mix=mix).split(b"\n") if l and json.loads(l)["kind"] in keep]
    nd = b"\n".join(lines)
    kinds = [json.loads(l)["kind"] for l in lines]
    ref = oracle.validate(pols, nd, nthreads=8)
    N, R = ref.shape
    assert R == len(rules)
    seedm = np.zeros((N, R), dtype=np.uint8)
    for j, r in enumerate(rules):
        rk = set(r["match"]["any"][0]["resources"]["kinds"])
        for i, k in enumerate(kinds):
            if k in rk:
                seedm[i, j] = 3 if r["name"] in PRE_ONLY else 6  # 3: a handler verdict stand-in
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(nd)
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([condvm_bin, str(tmp_path / "p.json"), str(tmp_path / "r.ndjson"),
                           str(tmp_path / "seed.bin"), str(tmp_path / "out.bin")])
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(N, R)
    assert (out == 7).sum() == 0
    for j, r in enumerate(rules):
        if r["name"] in PRE_ONLY:
            held = out[:, j] == 3
            assert ((ref[:, j] == 5) == (out[:, j] == 5)).all(), r["name"]
            assert not (held & (ref[:, j] == 5)).any()
        else:
            bad = np.nonzero(out[:, j] != ref[:, j])[0]
            assert bad.size == 0, (r["name"], bad[:5].tolist(), out[bad[:5], j].tolist(), ref[bad[:5], j].tolist())


def test_condvm_host_chart(condvm_bin, oracle, tmp_path):
    """The chart's deny / foreach rules (with autogen: paths under spec.template / jobTemplate)."""
    chart = json.load(open(os.path.join(ROOT, "tests", "golden", "chart_policies.json")))
    pols = [p for p in chart["baseline"] + chart["restricted"]
            if any("deny" in r.get("validate", {}) or "foreach" in r.get("validate", {}) for r in p["spec"]["rules"])]
    assert len(pols) == 3
    names = oracle.rule_names(pols)
    nd = K.synth_resources(0xC1, 3000, mix=2)
    lines = [l for l in nd.split(b"\n") if l]
    kinds = [json.loads(l)["kind"] for l in lines]
    ref = oracle.validate(pols, nd, nthreads=8)
    N, R = ref.shape
    ctrl = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"}
    seedm = np.zeros((N, R), dtype=np.uint8)
    for j, n in enumerate(names):
        rule = n.split("/", 1)[1]
        ks = {"CronJob"} if rule.startswith("autogen-cronjob-") else ctrl if rule.startswith("autogen-") else {"Pod"}
        seedm[:, j] = [6 if k in ks else 0 for k in kinds]
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(b"\n".join(lines))
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([condvm_bin, str(tmp_path / "p.json"), str(tmp_path / "r.ndjson"),
                           str(tmp_path / "seed.bin"), str(tmp_path / "out.bin")])
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(N, R)
    bad = np.argwhere(out != ref)
    assert bad.size == 0, (bad[:5].tolist(), [int(out[i, j]) for i, j in bad[:5]], [int(ref[i, j]) for i, j in bad[:5]])
    assert {1, 2} <= set(np.unique(out).tolist())


def test_condvm_host_chart_on_c5(condvm_bin, oracle, tmp_path):
    """The chart's deny / foreach rules over the C5 fan-out corpus (Pods / Deployments with 1-64
    containers): lists longer than the VM's CV_LIST_CAP give KPE_UNDECIDED cells, handed back to
    the caller; every other cell is bit-exact. Prints the undecided fraction."""
    chart = json.load(open(os.path.join(ROOT, "tests", "golden", "chart_policies.json")))
    pols = [p for p in chart["baseline"] + chart["restricted"]
            if any("deny" in r.get("validate", {}) or "foreach" in r.get("validate", {}) for r in p["spec"]["rules"])]
    names = oracle.rule_names(pols)
    nd = K.synth_resources(0xC5, 4000, mix=K.SYNTH_FANOUT)
    lines = [l for l in nd.split(b"\n") if l]
    kinds = [json.loads(l)["kind"] for l in lines]
    ref = oracle.validate(pols, nd, nthreads=8)
    N, R = ref.shape
    ctrl = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"}
    seedm = np.zeros((N, R), dtype=np.uint8)
    for j, n in enumerate(names):
        rule = n.split("/", 1)[1]
        ks = {"CronJob"} if rule.startswith("autogen-cronjob-") else ctrl if rule.startswith("autogen-") else {"Pod"}
        seedm[:, j] = [6 if k in ks else 0 for k in kinds]
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(b"\n".join(lines))
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([condvm_bin, str(tmp_path / "p.json"), str(tmp_path / "r.ndjson"),
                           str(tmp_path / "seed.bin"), str(tmp_path / "out.bin")])
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(N, R)
    # rows whose policy context fails (an invalid image: every oracle cell 7, KPE_ROW_CONTEXT_ERROR
    # on the device) are not the condition VM's
    ctx = (ref == 7).all(axis=1, keepdims=True)
    und = (out == 7) & ~ctx
    applied = (ref != 0) & ~ctx
    bad = np.argwhere((out != ref) & ~und & ~ctx)
    assert bad.size == 0, (bad[:5].tolist(), [int(out[i, j]) for i, j in bad[:5]], [int(ref[i, j]) for i, j in bad[:5]])
    frac = und.sum() / max(1, applied.sum())
    print(f"C5 chart deny/foreach: {und.sum()} undecided of {applied.sum()} applicable cells ({frac:.4%})")
    assert frac < 0.01
