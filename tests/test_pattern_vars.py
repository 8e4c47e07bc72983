"""Pattern variables and foreach pattern entries.

- validate.pattern / anyPattern with {{ }} variables: substitutePatterns
  (pkg/engine/handlers/validation/validate_resource.go:456-476, variables/vars.go:311-420): a
  whole-string variable keeps the value's JSON type, other variables are spliced into the string;
  a substitution error is RuleError. The device resolves each variable per row in
  kpe_cond_kernel (the condition program's JMESPath subset) and kpe_pattern_kernel reads them.
- validate.foreach entries with pattern / anyPattern / nested foreach (validate_resource.go:
  186-254, newForEachValidator :92-119): kpe_cond_kernel<FEPAT> runs the pattern VM on the scoped
  element (or the resource) per element, with element<n> / elementIndex<n> per nesting level.

CPU: the oracle against the reference's validation_test.go foreach / variable cases
(test_oracle_golden.py), compile acceptance, and kpe_cond_kernel + kpe_pattern_kernel's lane
bodies compiled for the host (scripts/condvm_check.cpp) against the oracle.
GPU: bit-exact verdict matrices against the oracle on three synthetic mixes."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import VAR_UNDECIDED_OK, var_policy_set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CTRL = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"}
UNDECIDED = 7


def _rule_kinds(name):
    rule = name.split("/", 1)[1]
    return {"CronJob"} if rule.startswith("autogen-cronjob-") else CTRL if rule.startswith("autogen-") else {"Pod"}


def _check(v, ref, names):
    bad = []
    for j, n in enumerate(names):
        rule = n.split("/", 1)[1].replace("autogen-cronjob-", "").replace("autogen-", "")
        diff = v[:, j] != ref[:, j]
        if rule in VAR_UNDECIDED_OK:
            diff &= v[:, j] != UNDECIDED
        for i in np.nonzero(diff)[0][:3]:
            bad.append((n, int(i), int(v[i, j]), int(ref[i, j])))
    return bad


def test_var_policy_set_compiles(oracle):
    pols = var_policy_set()
    assert K.PolicySet(pols).rule_names == oracle.rule_names(pols)


@pytest.mark.parametrize("pattern", [
    {"metadata": {"labels": {"<({{request.object.metadata.name}})": "x"}}},  # a variable in a global anchor key
    {"metadata": {"labels": {"=({{request.object.metadata.name}})": "x", "{{request.object.kind}}": "y"}}},  # + another
    {"metadata": {"labels": {"a-{{request.object.metadata.name}}": "x", "{{request.object.kind}}": "y"}}},  # two, one partial
    {"metadata": {"name": "$(./namespace)"}},                              # a reference
    {"metadata": {"name": "{{ @ }}"}},                                     # {{@}}
    {"metadata": {"name": "{{ to_upper(request.object.metadata.name) }}"}},  # a function
])
def test_refused(pattern):
    pol = var_policy_set()[0]
    pol["spec"]["rules"] = [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                             "validate": {"pattern": pattern}}]
    with pytest.raises(K.KpeError):
        K.PolicySet([pol])


@pytest.mark.parametrize("mix,seed", [(2, 0xA1), (1, 0xA2)])
def test_host_pipeline_matches_oracle(oracle, tmp_path, mix, seed):
    """kpe_cond_kernel<true> then kpe_pattern_kernel lane bodies on the host (ASan/UBSan), the
    scan kernel's part seeded from the rules' kinds."""
    from tests.conftest import build_host_tool

    build_host_tool("condvm_check")
    pols = var_policy_set()
    names = oracle.rule_names(pols)
    lines = [l for l in K.synth_resources(seed, 2000, mix=mix).split(b"\n") if l]
    kinds = [json.loads(l)["kind"] for l in lines]
    nd = b"\n".join(lines)
    ref = oracle.validate(pols, nd, nthreads=8)
    N, R = ref.shape
    seedm = np.zeros((N, R), dtype=np.uint8)
    for j, n in enumerate(names):
        ks = _rule_kinds(n)
        seedm[:, j] = [6 if k in ks else 0 for k in kinds]
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(nd)
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([os.path.join(ROOT, "scripts", "build", "condvm_check"), str(tmp_path / "p.json"),
                           str(tmp_path / "r.ndjson"), str(tmp_path / "seed.bin"), str(tmp_path / "out.bin")],
                          stdout=subprocess.DEVNULL)
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(N, R)
    bad = _check(out, ref, names)
    assert not bad, bad[:12]


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 20000, 0xA3), (1, 20000, 0xA4), (2, 20000, 0xA5)])
def test_gpu_pattern_vars_bit_exact(oracle, mix, n, seed):
    pols = var_policy_set()
    eng = K.Engine(ordinal=0)
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=16)
    bad = _check(v, ref, oracle.rule_names(pols))
    assert not bad, bad[:12]
    assert {1, 2, 4} <= set(np.unique(v).tolist())


# pkg/engine/jsonutils/traverse_test.go's document (Test_TraverseLeafsCheckIfTheyHit: every leaf
# and every key is visited once), with the variables moved into keys as well
TRAVERSE_DOC = {
    "kind": "{{request.object.metadata.name1}}",
    "name": "ns-owner-{{request.object.metadata.name}}",
    "data": {"rules": [{"apiGroups": ["{{request.object.metadata.name}}"], "resources": ["namespaces"], "verbs": ["*"]}]},
    "{{request.object.metadata.name}}": {"ns-owner-{{request.object.metadata.name}}": "{{request.object.metadata.name}}"},
}


def test_oracle_substitutes_keys_and_leaves(oracle):
    """SubstituteAll (vars.go:311-313: OnlyForLeafsAndKeys) renames map keys with variables
    (traverse.go:90-117) and substitutes every leaf, nested ones included; a key variable that is
    not a string is an error; a missing member is the fork's NotFoundError."""
    res = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "web", "name1": "Kind1"}}
    st, doc = oracle.substitute_doc(TRAVERSE_DOC, res)
    assert st == 0
    assert doc == {"kind": "Kind1", "name": "ns-owner-web",
                   "data": {"rules": [{"apiGroups": ["web"], "resources": ["namespaces"], "verbs": ["*"]}]},
                   "web": {"ns-owner-web": "web"}}
    st, _ = oracle.substitute_doc({"{{request.object.metadata.labels.n}}": "x"},
                                  dict(res, metadata={"name": "a", "labels": {"n": 3}}))
    assert st == -1  # "expected string after substituting variables in key"
    st, _ = oracle.substitute_doc({"{{request.object.metadata.labels.n}}": "x"}, res)
    assert st == -1  # Unknown key "labels"
