"""kpe_lean6_kernel (the headline C2 evaluation) over full matrices at every PSS level and version.

Every kind-only podSecurity policy (baseline / restricted / privileged x latest and each version
a PSA check changes at) is forced through the LEAN6 evaluation, asserted by the kernel stats,
over 20k-row synthetic mixes with Deployments, CronJobs, nulls, type errors and windows pods.
Compared with the oracle: the whole verdict matrix, and with masks the whole versioned-check
matrix (kpe_fetch_cv_masks: a FAIL cell holds the failing versioned checks of its level /
version, evaluate.go:24-70; every other cell 0). Every evaluation reads each pod's record and its
container / volume / sysctl / annotation lists; only the PSA dictionary codes (per distinct
string, tests/test_psum.py) are kept per corpus."""
import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import pss_policy

pytestmark = pytest.mark.gpu

LEVELS = ("baseline", "restricted", "privileged")
VERSIONS = ("latest", "v1.0", "v1.8", "v1.19", "v1.22", "v1.23", "v1.24", "v1.25", "v1.27", "v1.29")
LEAN6 = 7  # kpe_kernel_stats.scan_kernel of a one-shard kpe_lean6_kernel launch


@pytest.fixture(scope="module")
def engine():
    return K.Engine(ordinal=0)


@pytest.fixture(scope="module", params=[(1, 20000, 0x51), (2, 20000, 0x52), (-1, 400, 0)], ids=["mixed", "edge", "seccomp"])
def corpus(request, engine):
    mix, n, seed = request.param
    if mix < 0:  # container / pod seccomp and AppArmor annotations (the v1.0 checks)
        from tests.golden.make_psum_digests import seccomp_ndjson
        nd = seccomp_ndjson(n)
    else:
        nd = K.synth_resources(seed, n, mix=mix)
    return nd, K.Corpus(nd, docs=False).upload(engine.device)


@pytest.mark.parametrize("level", LEVELS)
def test_lean6_full_matrix_every_version(engine, oracle, corpus, level):
    nd, c = corpus
    for ver in VERSIONS:
        pol = pss_policy(f"{level}-{ver.replace('.', '-')}", level, ver)
        ps = K.PolicySet([pol])
        assert ps.num_rules == 3  # Pod + the autogen controller and CronJob rules
        ref = oracle.validate([pol], nd, nthreads=8)
        # verdicts, no masks: the LEAN6 evaluation must be the one that ran
        engine.device.set_timing(True)
        engine.device.kernel_stats(reset=True)
        engine.evaluate_async(ps, c)
        st = engine.device.kernel_stats(reset=True)
        engine.device.set_timing(False)
        assert st.launches == 1 and st.scan_kernel == LEAN6, (level, ver, st.scan_kernel)
        v, _, _ = engine.evaluate(ps, c)
        bad = np.argwhere(v != ref)
        assert bad.size == 0, (level, ver, len(bad), bad[:5].tolist())
        # with masks: the same verdicts and the whole versioned-check matrix
        vm, _, _ = engine.evaluate(ps, c, check_masks=True)
        assert np.array_equal(vm, ref), (level, ver)
        cv = engine.cv_masks(ps, c)
        want_row = oracle.failing_cv_batch(level, ver, nd)
        assert want_row.shape[0] == c.n
        fail = vm == 2
        want = np.where(fail, np.maximum(want_row, 0)[:, None], 0).astype(np.int64)
        assert (want_row[fail.any(axis=1)] >= 0).all()  # a FAIL row always decodes
        got = cv.astype(np.int64)
        bad = np.argwhere(got != want)
        assert bad.size == 0, (level, ver, len(bad), bad[:5].tolist())
        if level != "privileged":
            assert fail.sum() > 0 and (got[fail] != 0).all()


def test_lean6_batch_launch(engine, oracle):
    """kpe_evaluate_batch_async over warm LEAN shards of different sizes (one pod, a partial
    tile, repeats in one launch): one multi-shard kpe_lean6_kernel launch, and every shard's verdict
    matrix (poisoned on the device beforehand) and check masks equal the oracle's."""
    import ctypes
    from tests.golden.make_psum_digests import seccomp_ndjson
    pols = [pss_policy("restricted-latest", "restricted", "latest")]
    ps = K.PolicySet(pols)
    nds = [K.synth_resources(0x61, 5000, mix=1), K.synth_resources(0x62, 1, mix=1),
           K.synth_resources(0x63, 64, mix=2), K.synth_resources(0x64, 20000, mix=2), seccomp_ndjson(777)]
    cs = [K.Corpus(nd, docs=False).upload(engine.device) for nd in nds]
    refs = [oracle.validate(pols, nd, nthreads=8) for nd in nds]
    hip = ctypes.CDLL("libamdhip64.so")
    for masks in (False, True):
        for c in cs:  # bind (prologue image, PSA dictionary codes), then poison the verdicts
            engine.evaluate(ps, c, check_masks=masks)
            ptr, nb = engine.device_verdicts(ps, c)
            assert hip.hipMemset(ctypes.c_void_p(ptr), 0xFF, ctypes.c_size_t(nb)) == 0
        assert hip.hipDeviceSynchronize() == 0
        order = [0, 1, 2, 3, 4, 3, 0]
        engine.device.set_timing(True)
        engine.device.kernel_stats(reset=True)
        engine.evaluate_batch_async(ps, [cs[i] for i in order], masks=masks)
        st = engine.device.kernel_stats(reset=True)
        engine.device.set_timing(False)
        assert st.launches == 1 and st.scan_kernel == 9, (st.launches, st.scan_kernel)
        engine.device.sync()
        for i, (c, ref) in enumerate(zip(cs, refs)):
            v, m, _ = engine.fetch(ps, c, check_masks=masks)
            bad = np.argwhere(v != ref)
            assert bad.size == 0, (masks, i, len(bad), bad[:5].tolist())
            if masks:
                want_row = oracle.failing_cv_batch("restricted", "latest", nds[i])
                fail = v == 2
                want = np.where(fail, np.maximum(want_row, 0)[:, None], 0).astype(np.int64)
                got = engine.cv_masks(ps, c).astype(np.int64)
                assert np.array_equal(got, want), (i, int((got != want).sum()))


def test_lean6_batch_many_shards(engine, oracle):
    """More than KPE_LEAN_BATCH (24) shards in one call: near-equal multi-shard launches, verdicts
    unchanged, and each launch's algorithmic bytes the sum of its shards' one-shard bytes."""
    pols = [pss_policy("baseline-latest", "baseline", "latest")]
    ps = K.PolicySet(pols)
    nd = K.synth_resources(0x65, 3000, mix=1)
    cs = [K.Corpus(nd, docs=False).upload(engine.device) for _ in range(3)]
    ref = oracle.validate(pols, nd, nthreads=8)
    for c in cs:
        engine.evaluate(ps, c)
    engine.device.set_timing(True)
    engine.device.kernel_stats(reset=True)
    engine.evaluate_async(ps, cs[0])
    one = engine.device.kernel_stats(reset=True)
    assert one.launches == 1 and one.scan_kernel == LEAN6
    engine.evaluate_batch_async(ps, [cs[i % 3] for i in range(130)])
    st = engine.device.kernel_stats(reset=True)
    engine.device.set_timing(False)
    assert st.launches == 6 and st.scan_kernel == 9
    assert abs(st.scan_bytes - 22 * one.scan_bytes) < 1  # 130 -> 21 + 21 + 22 + 22 + 22 + 22 shards (the last)
    engine.device.sync()
    for c in cs:
        v, _, _ = engine.fetch(ps, c)
        assert np.array_equal(v, ref)


def test_lean6_batch_tiles_per_wave(engine):
    """A batch large enough for 4 tiles per wave (one 1M + 37-pod shard nine times: 140k tiles;
    the last block of every shard partial): the same verdicts as the single-shard kernel, whose
    parity with the oracle the tests above pin."""
    import ctypes
    pols = [pss_policy("restricted-latest", "restricted", "latest")]
    ps = K.PolicySet(pols)
    c = K.Corpus(K.synth_resources(0x66, 1_000_037, mix=1), docs=False).upload(engine.device)
    want, _, _ = engine.evaluate(ps, c)
    ptr, nb = engine.device_verdicts(ps, c)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemset(ctypes.c_void_p(ptr), 0xFF, ctypes.c_size_t(nb)) == 0
    assert hip.hipDeviceSynchronize() == 0
    engine.device.set_timing(True)
    engine.device.kernel_stats(reset=True)
    engine.evaluate_batch_async(ps, [c] * 9)
    st = engine.device.kernel_stats(reset=True)
    engine.device.set_timing(False)
    assert st.launches == 1 and st.scan_kernel == 9
    engine.device.sync()
    got, _, _ = engine.fetch(ps, c)
    assert np.array_equal(got, want)


def lean_stress_ndjson(n, seed, unique_strings=True):
    """Pods that take every slow path of kpe_lean6_kernel: 1-12 containers (tiles past the 128
    staged containers, pods past the 4 clamped reads), 0-9 volumes, 0-4 sysctls and 1-7
    annotations per pod (past the 2 clamped reads and the 64 staged items), and, with
    unique_strings, a distinct annotation key / value and sysctl name per pod (code tables too large
    for the LDS: the global-code instantiation)."""
    import json
    import random

    rnd = random.Random(seed)
    caps = ["NET_BIND_SERVICE", "CHOWN", "SYS_ADMIN", "ALL", "NET_RAW", "KILL"]
    sec = [None, "RuntimeDefault", "Localhost", "Unconfined", "Bogus"]
    srcs = [("configMap", {"name": "c"}), ("emptyDir", {}), ("hostPath", {"path": "/x"}), ("nfs", {"server": "s", "path": "/"}),
            ("secret", {"secretName": "s"}), ("csi", {"driver": "d"}), ("gitRepo", {"repository": "r"}), ("projected", {"sources": []})]
    sysctls = ["kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range", "kernel.msgmax", "net.ipv4.tcp_keepalive_time",
               "net.ipv4.ip_local_reserved_ports", "vm.swappiness"]
    aa = ["runtime/default", "localhost/p", "unconfined"]
    sva = ["runtime/default", "docker/default", "localhost/p", "unconfined"]
    out = []
    for i in range(n):
        ctrs = []
        for k in range(1 + rnd.randrange(12)):
            sc = {}
            if rnd.random() < 0.8:
                if rnd.random() < 0.5:
                    sc["allowPrivilegeEscalation"] = rnd.random() < 0.2
                if rnd.random() < 0.1:
                    sc["privileged"] = True
                if rnd.random() < 0.6:
                    sc["capabilities"] = {"drop": rnd.sample(caps, rnd.randrange(3)), "add": rnd.sample(caps, rnd.randrange(2))}
                if rnd.random() < 0.5:
                    sc["runAsNonRoot"] = rnd.random() < 0.8
                s = rnd.choice(sec)
                if s:
                    sc["seccompProfile"] = {"type": s}
                if rnd.random() < 0.05:
                    sc["procMount"] = "Unmasked"
            c = {"name": f"c{k}", "image": "nginx:1.0", "securityContext": sc}
            if rnd.random() < 0.05:
                c["ports"] = [{"containerPort": 80, "hostPort": 8080}]
            ctrs.append(c)
        vols = [{"name": f"v{k}", src: dict(body)} for k, (src, body) in
                enumerate(rnd.choice(srcs) for _ in range(rnd.randrange(10)))]
        ann = {f"note-{i}" if unique_strings else "note": f"v-{i}" if unique_strings else "v"}
        for k in range(rnd.randrange(7)):
            r = rnd.random()
            if r < 0.3:
                ann[f"container.apparmor.security.beta.kubernetes.io/c{k}"] = rnd.choice(aa)
            elif r < 0.6:
                ann[f"container.seccomp.security.alpha.kubernetes.io/c{k}"] = rnd.choice(sva)
            elif r < 0.7:
                ann["seccomp.security.alpha.kubernetes.io/pod"] = rnd.choice(sva)
            else:
                ann[f"extra-{k}"] = f"x{rnd.randrange(5)}"
        spec = {"containers": ctrs, "volumes": vols}
        psc = {}
        if rnd.random() < 0.4:
            names = rnd.sample(sysctls, rnd.randrange(5))
            if unique_strings and rnd.random() < 0.5:
                names.append(f"net.custom.knob{i}")
            psc["sysctls"] = [{"name": nm, "value": "1"} for nm in names]
        if rnd.random() < 0.3:
            psc["runAsNonRoot"] = True
        if rnd.random() < 0.3:
            psc["seccompProfile"] = {"type": "RuntimeDefault"}
        if psc:
            spec["securityContext"] = psc
        out.append({"apiVersion": "v1", "kind": "Pod",
                    "metadata": {"name": f"st-{i}", "namespace": "default", "annotations": ann}, "spec": spec})
    return "\n".join(json.dumps(o, separators=(",", ":")) for o in out).encode()


@pytest.mark.parametrize("unique", [False, True], ids=["lds-codes", "global-codes"])
def test_lean6_slow_paths(engine, oracle, unique):
    """Long lists and large dictionaries: every overflow path of kpe_lean6_kernel, and the
    instantiation that reads the code bytes from global memory, bit-exact with the oracle (verdicts
    and check masks) at three level / version pairs, single-shard and multi-shard launches."""
    nd = lean_stress_ndjson(12000, 0x5E + unique, unique_strings=unique)
    c = K.Corpus(nd, docs=False).upload(engine.device)
    c2 = K.Corpus(nd, docs=False).upload(engine.device)
    for level, ver in (("restricted", "latest"), ("baseline", "v1.0"), ("restricted", "v1.25")):
        pol = pss_policy(f"{level}-{ver.replace('.', '-')}", level, ver)
        ps = K.PolicySet([pol])
        ref = oracle.validate([pol], nd, nthreads=8)
        engine.device.set_timing(True)
        engine.device.kernel_stats(reset=True)
        v, _, _ = engine.evaluate(ps, c, check_masks=True)
        st = engine.device.kernel_stats(reset=True)
        engine.device.set_timing(False)
        assert st.scan_kernel == LEAN6, st.scan_kernel
        bad = np.argwhere(v != ref)
        assert bad.size == 0, (level, ver, len(bad), bad[:5].tolist())
        want_row = oracle.failing_cv_batch(level, ver, nd)
        want = np.where(v == 2, np.maximum(want_row, 0)[:, None], 0).astype(np.int64)
        assert np.array_equal(engine.cv_masks(ps, c).astype(np.int64), want), (level, ver)
        engine.evaluate(ps, c2)
        engine.evaluate_batch_async(ps, [c, c2, c])
        engine.device.sync()
        for cc in (c, c2):
            vb, _, _ = engine.fetch(ps, cc)
            assert np.array_equal(vb, ref), (level, ver)
