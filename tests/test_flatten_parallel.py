"""The parallel flattener (flatten.cpp flatten_ndjson: line-aligned chunks flattened by
KPE_FLATTEN_THREADS threads, merged in document order) produces the exact encoding of a
one-thread flatten: every column, dictionary, scalar and capability-set id."""
import os

import pytest

import kyverno_amd as K


def _digest(nd, threads, docs):
    old = os.environ.get("KPE_FLATTEN_THREADS")
    os.environ["KPE_FLATTEN_THREADS"] = str(threads)
    try:
        c = K.Corpus(nd, docs=docs)
        return c.n, c.digest()
    finally:
        if old is None:
            os.environ.pop("KPE_FLATTEN_THREADS")
        else:
            os.environ["KPE_FLATTEN_THREADS"] = old


@pytest.mark.parametrize("mix,n", [(K.SYNTH_PODS, 30000), (2, 12000), (K.SYNTH_C3, 12000), (K.SYNTH_FANOUT, 6000)])
@pytest.mark.parametrize("docs", [False, True])
def test_parallel_flatten_is_sequential(mix, n, docs):
    nd = K.synth_resources(7, n, mix=mix)
    assert len(nd) > 3 << 20  # large enough to be cut into several chunks
    ref = _digest(nd, 1, docs)
    for t in (2, 5, 8):
        assert _digest(nd, t, docs) == ref, t


def test_parallel_flatten_errors_in_document_order():
    nd = K.synth_resources(3, 20000, mix=2)
    lines = nd.split(b"\n")
    lines[15000] = b'{"kind": "Pod", "metadata": '  # malformed, in a late chunk
    bad = b"\n".join(lines)
    for t in (1, 8):
        os.environ["KPE_FLATTEN_THREADS"] = str(t)
        try:
            with pytest.raises(K.KpeError) as e:
                K.Corpus(bad)
            assert e.value.status == 1
        finally:
            os.environ.pop("KPE_FLATTEN_THREADS")


@pytest.mark.parametrize("threads", [2, 5, 8, 16])
@pytest.mark.parametrize("docs", [False, True])
def test_parallel_dictionary_merge_is_sequential(threads, docs):
    """Dictionaries past 65536 strings are merged by hash buckets on several threads
    (flatten.cpp merge_dict_parallel) with the ids of a sequential merge: resource names repeating
    across chunks (first occurrence in an earlier chunk, or later in the same one), and strings
    that only some chunks hold."""
    import json

    rows = []
    for i in range(90000):
        name = f"res-{(i * 7919) % 70000}"
        rows.append(json.dumps({"apiVersion": "v1", "kind": "ConfigMap",
                                "metadata": {"name": name, "namespace": f"ns-{i % 13}",
                                             "labels": {"app": f"a-{i % 70001}"}}}))
    nd = "\n".join(rows).encode()
    assert _digest(nd, threads, docs) == _digest(nd, 1, docs)
