"""Host-side mirror of the reference engine interface, backed by libkpe.

Reference surface mirrored here (names and meaning kept):
  engineapi.Engine.Validate(ctx, PolicyContext) EngineResponse   pkg/engine/api/engine.go:17-23
  engineapi.EngineResponse / PolicyResponse.Rules                pkg/engine/api/engineresponse.go:14-60
  engineapi.RuleResponse (name, type, status)                    pkg/engine/api/ruleresponse.go:25-60
  engineapi.RuleStatus pass/fail/warning/error/skip              pkg/engine/api/rulestatus.go:4-21
  engine.NewPolicyContext(..., Create, ...).WithNewResource(r).WithPolicy(p).WithNamespaceLabels(l)
                                                                 pkg/controllers/report/utils/scanner.go:99-110
Single-resource Validate() is served by the same batch kernels (a batch of one);
batch callers (`kyverno apply`'s resource loop, the background scanner) use
Engine.validate_batch()/evaluate(), which evaluate the whole resource x rule
matrix on the GPU in one pass.
"""
import ctypes
import enum
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from ._lib import CliTotals, Counts, KernelStats, KpeError, check, load


class RuleStatus(str, enum.Enum):
    PASS = "pass"
    FAIL = "fail"
    WARN = "warning"
    ERROR = "error"
    SKIP = "skip"


# kpe_verdict cell codes -> RuleStatus (0 = no RuleResponse)
VERDICT = {1: RuleStatus.PASS, 2: RuleStatus.FAIL, 3: RuleStatus.WARN, 4: RuleStatus.ERROR, 5: RuleStatus.SKIP}
UNDECIDED = 7  # kpe_verdict KPE_UNDECIDED: a cell the device leaves to the reference engine


@dataclass
class RuleResponse:
    name: str
    status: RuleStatus
    rule_type: str = "Validation"
    pod_security_checks: List[str] = field(default_factory=list)  # failing PSA check IDs (PSS rules)


@dataclass
class EngineResponse:
    policy: str
    resource: Optional[dict]
    rules: List[RuleResponse]

    def is_successful(self):  # engineresponse.go IsSuccessful: no fail/error rule
        return not any(r.status in (RuleStatus.FAIL, RuleStatus.ERROR) for r in self.rules)


@dataclass
class PolicyContext:
    """engine.NewPolicyContext(..., kyvernov1.Create, ...) for background/CLI scans."""
    resource: dict
    policy: dict
    namespace_labels: Dict[str, str] = field(default_factory=dict)
    operation: str = "CREATE"

    def with_new_resource(self, r):
        self.resource = r
        return self

    def with_policy(self, p):
        self.policy = p
        return self

    def with_namespace_labels(self, l):
        self.namespace_labels = dict(l or {})
        return self


class Device:
    def __init__(self, ordinal: int = 0):
        L = load()
        h = ctypes.c_void_p()
        check(L.kpe_device_open(int(ordinal), ctypes.byref(h)))
        self.h, self.ordinal = h, ordinal

    def close(self):
        if self.h:
            load().kpe_device_close(self.h)
            self.h = None

    def sync(self):
        check(load().kpe_device_sync(self.h))

    def set_timing(self, on: bool):
        check(load().kpe_device_set_timing(self.h, 1 if on else 0))

    def kernel_stats(self, reset=False):
        st = KernelStats()
        check(load().kpe_device_kernel_stats(self.h, None, None, ctypes.byref(st), 1 if reset else 0))
        return st

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PolicySet:
    """Compiled policies (autogen applied once, autogen.ComputeRules)."""

    def __init__(self, policies, exceptions=None, background=False):
        """exceptions: PolicyException objects (kyverno.io/v2beta1) or their JSON; background:
        drop exceptions with spec.background false, as the background scanner does."""
        L = load()
        if isinstance(policies, (bytes, str)):
            raw = policies if isinstance(policies, bytes) else policies.encode()
            self.policies = None
        else:
            self.policies = list(policies) if isinstance(policies, (list, tuple)) else [policies]
            raw = json.dumps(self.policies).encode()
        if exceptions is None:
            xraw = b""
        elif isinstance(exceptions, (bytes, str)):
            xraw = exceptions if isinstance(exceptions, bytes) else exceptions.encode()
        else:
            xraw = json.dumps(list(exceptions) if isinstance(exceptions, (list, tuple)) else [exceptions]).encode()
        self.exceptions = exceptions
        h = ctypes.c_void_p()
        check(L.kpe_program_compile_ex(raw, len(raw), xraw or None, len(xraw), 1 if background else 0, ctypes.byref(h)))
        self.h = h
        n = L.kpe_program_num_rules(h)
        self.rule_names = [L.kpe_program_rule_name(h, i).decode() for i in range(n)]
        self.is_pss = [bool(L.kpe_program_rule_is_pss(h, i)) for i in range(n)]

    @property
    def num_rules(self):
        return len(self.rule_names)

    def __del__(self):
        try:
            if self.h:
                load().kpe_program_free(self.h)
                self.h = None
        except Exception:
            pass


class Corpus:
    """Flattened, string-interned resources (host columns, optionally on a device)."""

    DOCS = 1  # KPE_CORPUS_DOCS: keep document tapes (pattern / anyPattern rules)

    def __init__(self, resources, namespace_labels: Optional[Dict[str, Dict[str, str]]] = None, docs: bool = True):
        L = load()
        if isinstance(resources, (bytes, bytearray)):
            raw = bytes(resources)
        elif isinstance(resources, str):
            raw = resources.encode()
        else:
            raw = "\n".join(json.dumps(r, separators=(",", ":")) for r in resources).encode()
        if isinstance(namespace_labels, (bytes, bytearray)):
            nsl = bytes(namespace_labels)
        else:
            nsl = json.dumps(namespace_labels).encode() if namespace_labels else b""
        h = ctypes.c_void_p()
        check(L.kpe_corpus_flatten_ex(raw, len(raw), nsl if nsl else None, len(nsl), self.DOCS if docs else 0,
                                      ctypes.byref(h)))
        self.h = h
        self.n = int(L.kpe_corpus_num_resources(h))
        self.nbytes = int(L.kpe_corpus_bytes(h))
        self.device = None

    def row_flags(self) -> np.ndarray:
        """Per-row flatten status (kpe_corpus_row_flags): KPE_ROW_DECODE_ERROR = 1,
        KPE_ROW_LIMIT = 2, KPE_ROW_NO_SPEC = 4."""
        out = np.zeros(self.n, dtype=np.uint32)
        check(load().kpe_corpus_row_flags(self.h, out.ctypes.data))
        return out

    def digest(self) -> int:
        """64-bit digest of the columnar encoding (kpe_corpus_digest)."""
        return int(load().kpe_corpus_digest(self.h))

    def upload(self, dev: Device):
        check(load().kpe_corpus_upload(dev.h, self.h))
        self.device = dev
        return self

    def psa_summary(self) -> np.ndarray:
        """The per-pod PSA summary built on the corpus's device (kpe_corpus_psa_summary):
        n x 2 uint32 (schema.h PS_*)."""
        if self.device is None:
            raise KpeError(5, "corpus not uploaded")  # KPE_E_STATE
        out = np.zeros((self.n, 2), dtype=np.uint32)
        check(load().kpe_corpus_psa_summary(self.device.h, self.h, out.ctypes.data))
        return out

    def __del__(self):
        try:
            if self.h:
                load().kpe_corpus_free(self.h)
                self.h = None
        except Exception:
            pass


# kpe_synth_mix (include/kpe_synth.h)
SYNTH_PODS, SYNTH_MIXED, SYNTH_EDGE, SYNTH_SELECTORS, SYNTH_FANOUT, SYNTH_C3 = range(6)


def packed_words(cells: int) -> int:
    """32-bit words of a 3-bit packed verdict matrix of `cells` cells (10 cells per word)."""
    return int(load().kpe_packed_words(cells))


def unpack_verdicts(packed: np.ndarray, n: int, r: int) -> np.ndarray:
    """Host expansion of kpe_pack_verdicts output into an n x r uint8 verdict matrix."""
    packed = np.ascontiguousarray(packed, dtype=np.uint32)
    if packed.size < packed_words(n * r):
        raise ValueError("packed buffer too small")
    out = np.empty((n, r), dtype=np.uint8)
    check(load().kpe_unpack_verdicts(packed.ctypes.data, n * r, out.ctypes.data if n * r else None))
    return out


def evaluate_sharded(engines: Sequence["Engine"], ps: "PolicySet", shards: Sequence["Corpus"]):
    """One logical corpus over several devices of this process (kpe_evaluate_sharded): the
    shards' verdict rows in order and the summed per-rule counts."""
    L = load()
    k = len(shards)
    if len(engines) != k or k == 0:
        raise ValueError("one engine (device) per shard")
    for e, c in zip(engines, shards):
        if c.device is not e.device:
            c.upload(e.device)
    R = ps.num_rules
    N = sum(c.n for c in shards)
    v = np.zeros((N, R), dtype=np.uint8)
    counts = (Counts * max(R, 1))()
    devs = (ctypes.c_void_p * k)(*[e.device.h for e in engines])
    cps = (ctypes.c_void_p * k)(*[c.h for c in shards])
    check(L.kpe_evaluate_sharded(devs, cps, k, ps.h, v.ctypes.data if N * R else None, counts))
    cnt = [{"na": c.na, "pass": c.pass_, "fail": c.fail, "warn": c.warn, "error": c.error, "skip": c.skip,
            "undecided": c.undecided} for c in counts[:R]]
    return v, cnt


def synth_resources(seed: int, n: int, mix: int = 0, first_index: int = 0) -> bytes:
    """NDJSON from the synthetic generator (include/kpe_synth.h)."""
    L = load()
    p = ctypes.c_void_p()
    ln = ctypes.c_size_t()
    if L.kpe_synth_resources(seed, first_index, n, mix, ctypes.byref(p), ctypes.byref(ln)) != 0:
        raise KpeError(-1, "synth failed")
    try:
        # string_at's size is a C int in Python 3.10: corpora past 2 GiB are copied by array
        return bytes((ctypes.c_char * ln.value).from_address(p.value)) if ln.value else b""
    finally:
        L.kpe_synth_free(p)


def synth_ns_labels(seed: int, n_namespaces: int, mix: int = 0) -> bytes:
    """Namespace label table JSON from the synthetic generator (include/kpe_synth.h)."""
    L = load()
    p = ctypes.c_void_p()
    ln = ctypes.c_size_t()
    if L.kpe_synth_ns_labels(seed, n_namespaces, mix, ctypes.byref(p), ctypes.byref(ln)) != 0:
        raise KpeError(-1, "synth failed")
    try:
        # string_at's size is a C int in Python 3.10: corpora past 2 GiB are copied by array
        return bytes((ctypes.c_char * ln.value).from_address(p.value)) if ln.value else b""
    finally:
        L.kpe_synth_free(p)


class CorpusBatch:
    """Corpus handles packed once for kpe_evaluate_batch_async (keeps the corpora alive)."""

    def __init__(self, corpora: Sequence[Corpus]):
        self.corpora = list(corpora)
        self.n = len(self.corpora)
        self.arr = (ctypes.c_void_p * max(self.n, 1))(*[c.h for c in self.corpora])


class Engine:
    """engineapi.Engine (validate path) on one MI355X."""

    def __init__(self, device: Optional[Device] = None, ordinal: int = 0):
        self.device = device or Device(ordinal)

    # ---- columnar batch API ----
    def evaluate(self, ps: PolicySet, corpus: Corpus, check_masks=False):
        """Verdict matrix (N x R uint8, kpe_verdict), optional PSS check masks, per-rule counts."""
        L = load()
        if corpus.device is not self.device:
            corpus.upload(self.device)
        N, R = corpus.n, ps.num_rules
        v = np.zeros((N, R), dtype=np.uint8)
        m = np.zeros((N, R), dtype=np.uint32) if check_masks else None
        counts = (Counts * max(R, 1))()
        check(L.kpe_evaluate(self.device.h, ps.h, corpus.h, v.ctypes.data if N * R else None,
                             m.ctypes.data if (m is not None and N * R) else None, counts))
        cnt = [{"na": c.na, "pass": c.pass_, "fail": c.fail, "warn": c.warn, "error": c.error, "skip": c.skip,
                "undecided": c.undecided} for c in counts[:R]]
        return v, m, cnt

    def fetch(self, ps: PolicySet, corpus: Corpus, check_masks=False):
        """(verdicts, masks or None, counts) of the last enqueued evaluation of ps on corpus
        (kpe_fetch): the read-back half of evaluate_async / evaluate_batch_async."""
        N, R = corpus.n, ps.num_rules
        v = np.zeros((N, R), dtype=np.uint8)
        m = np.zeros((N, R), dtype=np.uint32) if check_masks else None
        counts = (Counts * max(R, 1))()
        check(load().kpe_fetch(self.device.h, ps.h, corpus.h, v.ctypes.data if N * R else None,
                               m.ctypes.data if (m is not None and N * R) else None, counts))
        cnt = [{"na": c.na, "pass": c.pass_, "fail": c.fail, "warn": c.warn, "error": c.error, "skip": c.skip,
                "undecided": c.undecided} for c in counts[:R]]
        return v, m, cnt

    CVM_XMATCH = 1 << 31  # KPE_CVM_XMATCH: a flag of FAIL cells, not a versioned check

    def cv_masks(self, ps: PolicySet, corpus: Corpus, raw=False):
        """Failing versioned PSS checks (N x R uint32, bit v = kpe_pss_cv_check(v)) of the last
        evaluation with check_masks=True (kpe_fetch_cv_masks). Bit 31 (KPE_CVM_XMATCH: the
        cell's podSecurity PolicyException matched) is cleared unless raw=True; the report
        functions take the raw words."""
        m = np.zeros((corpus.n, ps.num_rules), dtype=np.uint32)
        if m.size:
            check(load().kpe_fetch_cv_masks(self.device.h, ps.h, corpus.h, m.ctypes.data))
        return m if raw else m & np.uint32(0x7FFFFFFF)

    def evaluate_async(self, ps: PolicySet, corpus: Corpus, masks=False, cold=False):
        """Enqueue one evaluation (results stay on the device). masks: also write the check masks;
        cold: re-run the per-corpus prologue (dictionary pass, prologue image)."""
        if not masks and not cold:
            check(load().kpe_evaluate_async(self.device.h, ps.h, corpus.h))
        else:
            check(load().kpe_evaluate_async_ex(self.device.h, ps.h, corpus.h, (1 if masks else 0) | (2 if cold else 0)))

    def batch(self, corpora: Sequence[Corpus]) -> "CorpusBatch":
        """A reusable list of corpora on this engine's device for evaluate_batch_async."""
        for c in corpora:
            if c.device is not self.device:
                raise KpeError(5, "corpus not uploaded to this engine's device")  # KPE_E_STATE
        return CorpusBatch(corpora)

    def evaluate_batch_async(self, ps: PolicySet, batch, masks=False, cold=False):
        """Enqueue one evaluation per corpus of `batch` (a CorpusBatch or a list), in order, with
        one call (kpe_evaluate_batch_async)."""
        b = batch if isinstance(batch, CorpusBatch) else self.batch(batch)
        check(load().kpe_evaluate_batch_async(self.device.h, ps.h, b.arr, b.n, (1 if masks else 0) | (2 if cold else 0)))

    # ---- verdict exchange (device-resident) ----
    def device_verdicts(self, ps: PolicySet, corpus: Corpus):
        """(device address, bytes) of the corpus's verdict matrix after an evaluation of ps."""
        ptr, nb = ctypes.c_void_p(), ctypes.c_uint64()
        check(load().kpe_device_verdicts(self.device.h, ps.h, corpus.h, ctypes.byref(ptr), ctypes.byref(nb)))
        return ptr.value, nb.value

    def pack_verdicts(self, ps: PolicySet, corpus: Corpus, dst_ptr: int, words: int):
        """3-bit packing of the verdict matrix into device memory at dst_ptr (kpe_pack_verdicts)."""
        check(load().kpe_pack_verdicts(self.device.h, ps.h, corpus.h, ctypes.c_void_p(dst_ptr), words))

    def pattern_traces(self, ps: PolicySet, corpus: Corpus, cells) -> np.ndarray:
        """Failing-path records of pattern cells (kpe_pattern_traces) after an evaluation of ps on
        corpus: cells = flat indices row * R + column; returns (len(cells), KPE_TRACE_ROOTS,
        KPE_TRACE_WORDS) uint32."""
        c = np.ascontiguousarray(cells, dtype=np.uint64)
        out = np.zeros((c.size, TRACE_ROOTS, TRACE_WORDS), dtype=np.uint32)
        if c.size:
            check(load().kpe_pattern_traces(self.device.h, ps.h, corpus.h, c.ctypes.data, c.size, out.ctypes.data))
        return out

    def row_traces(self, ps: PolicySet, corpus: Corpus, row: int) -> np.ndarray:
        """Trace records of every cell of one row (the layout report_results(traces=) takes)."""
        R = ps.num_rules
        return self.pattern_traces(ps, corpus, np.arange(row * R, row * R + R, dtype=np.uint64))

    def cond_traces(self, ps: PolicySet, corpus: Corpus, row0: int = 0, nrows: Optional[int] = None,
                    ex: bool = False) -> np.ndarray:
        """Condition traces (kpe_fetch_cond_traces) of rows [row0, row0 + nrows) after an evaluation
        of ps on corpus: (nrows, R) uint32, the layout report_results(cond_traces=) takes per row.
        ex: kpe_fetch_cond_traces_ex, (nrows, R, KPE_CTRACE_WORDS) with the foreach and error
        records (foreach messages, RuleError texts)."""
        n = corpus.n - row0 if nrows is None else nrows
        out = np.zeros((n, ps.num_rules, CTRACE_WORDS) if ex else (n, ps.num_rules), dtype=np.uint32)
        if n:
            f = load().kpe_fetch_cond_traces_ex if ex else load().kpe_fetch_cond_traces
            check(f(self.device.h, ps.h, corpus.h, row0, n, out.ctypes.data))
        return out

    # ---- reference-shaped API ----
    def validate_batch(self, policies: Sequence[dict], resources: Sequence[dict],
                       namespace_labels: Optional[Dict[str, Dict[str, str]]] = None) -> List[List[EngineResponse]]:
        """EngineResponse per (resource, policy), rules in ComputeRules order, NA cells omitted."""
        ps = PolicySet(list(policies))
        corpus = Corpus(resources, namespace_labels)
        v, m, _ = self.evaluate(ps, corpus, check_masks=True)
        L = load()
        check_ids = [L.kpe_pss_check_id(k).decode() for k in range(17)]
        # policy boundaries by "<policy>/<rule>" prefix, in compile order
        spans, start = [], 0
        for p in policies:
            cnt = 0
            for x in ps.rule_names[start:]:
                if x.split("/", 1)[0] != p["metadata"]["name"]:
                    break
                cnt += 1
            spans.append((start, start + cnt))
            start += cnt
        out = []
        for i, res in enumerate(resources):
            row = []
            for (a, b), p in zip(spans, policies):
                rules = []
                for r in range(a, b):
                    cell = int(v[i, r])
                    if cell == 0:
                        continue
                    if cell == UNDECIDED:
                        raise KpeError(-1, f"cell ({i}, {ps.rule_names[r]}) is beyond the device's documented "
                                           "limits (KPE_UNDECIDED): evaluate it with the reference engine")
                    checks = [check_ids[k] for k in range(17) if (int(m[i, r]) >> k) & 1] if ps.is_pss[r] else []
                    rules.append(RuleResponse(ps.rule_names[r].split("/", 1)[1], VERDICT[cell],
                                              pod_security_checks=checks))
                row.append(EngineResponse(p["metadata"]["name"], res, rules))
            out.append(row)
        return out

    def validate(self, policy_context: PolicyContext) -> EngineResponse:
        """engineapi.Engine.Validate for one PolicyContext (a batch of one)."""
        nsl = None
        ns = (policy_context.resource.get("metadata") or {}).get("namespace")
        if ns and policy_context.namespace_labels:
            nsl = {ns: policy_context.namespace_labels}
        return self.validate_batch([policy_context.policy], [policy_context.resource], nsl)[0][0]


TRACE_WORDS, TRACE_ROOTS = 16, 4  # include/kpe.h KPE_TRACE_WORDS / KPE_TRACE_ROOTS
CTRACE_WORDS = 4  # include/kpe.h KPE_CTRACE_WORDS (kpe_fetch_cond_traces_ex)


class ReportArgs(ctypes.Structure):
    """include/kpe.h kpe_report_args"""
    _fields_ = [("prog", ctypes.c_void_p), ("corpus", ctypes.c_void_p), ("verdict_row", ctypes.c_void_p),
                ("cv_mask_row", ctypes.c_void_p), ("pattern_traces", ctypes.c_void_p),
                ("cond_traces", ctypes.c_void_p), ("resource_json", ctypes.c_char_p),
                ("resource_len", ctypes.c_size_t), ("cond_traces_ex", ctypes.c_void_p)]


def report_results(ps: PolicySet, verdict_row, cv_mask_row=None, resource=None, traces=None,
                   corpus: Optional[Corpus] = None, cond_traces=None) -> List[dict]:
    """EngineResponseToReportResults (pkg/utils/report/results.go:89-156) for one resource row,
    through kpe_report_results, or kpe_report_results_msg when the resource (a dict or its JSON
    bytes) is given: then results carry the RuleResponse message (podSecurity pass / fail,
    validate.pattern pass; no timestamp). With traces (Engine.row_traces of the row) and the
    corpus, kpe_report_results_msg_tr adds the pattern / anyPattern failure and anyPattern pass
    messages; with cond_traces (a row of Engine.cond_traces), kpe_report_results_ex adds the
    condition messages (preconditions skips, deny fails with condition messages)."""
    L = load()
    v = np.ascontiguousarray(verdict_row, dtype=np.uint8)
    m = None if cv_mask_row is None else np.ascontiguousarray(cv_mask_row, dtype=np.uint32)
    if v.size != ps.num_rules or (m is not None and m.size != ps.num_rules):
        raise ValueError("row length != number of rules")
    raw = None
    if resource is not None:
        raw = resource if isinstance(resource, (bytes, bytearray)) else json.dumps(resource).encode()
    cap = 4096
    while True:
        buf = ctypes.create_string_buffer(cap)
        mp = None if m is None else m.ctypes.data
        if raw is None:
            n = L.kpe_report_results(ps.h, v.ctypes.data, mp, buf, cap)
        elif cond_traces is not None:
            ct = np.ascontiguousarray(cond_traces, dtype=np.uint32)
            ex = ct.ndim == 2  # a row of Engine.cond_traces(ex=True): KPE_CTRACE_WORDS per rule
            if ct.size != ps.num_rules * (CTRACE_WORDS if ex else 1):
                raise ValueError("cond_traces: one word (or KPE_CTRACE_WORDS words) per rule of the row")
            t = None
            if traces is not None:
                t = np.ascontiguousarray(traces, dtype=np.uint32)
                if t.size != ps.num_rules * TRACE_ROOTS * TRACE_WORDS:
                    raise ValueError("traces: one record per rule of the row")
            a = ReportArgs(ps.h, corpus.h if corpus is not None else None, v.ctypes.data, mp,
                           None if t is None else t.ctypes.data, None if ex else ct.ctypes.data, raw, len(raw),
                           ct.ctypes.data if ex else None)
            n = L.kpe_report_results_ex(ctypes.byref(a), buf, cap)
        elif traces is not None:
            t = np.ascontiguousarray(traces, dtype=np.uint32)
            if t.size != ps.num_rules * TRACE_ROOTS * TRACE_WORDS:
                raise ValueError("traces: one record per rule of the row")
            n = L.kpe_report_results_msg_tr(ps.h, corpus.h if corpus is not None else None, v.ctypes.data, mp,
                                            t.ctypes.data, raw, len(raw), buf, cap)
        else:
            n = L.kpe_report_results_msg(ps.h, v.ctypes.data, mp, raw, len(raw), buf, cap)
        if n < 0:
            check(-n)
        if n < cap:
            return json.loads(buf.value.decode())
        cap = n + 1


def cli_summary(ps: PolicySet, counts: List[dict], audit_warn: bool = False) -> Dict[str, int]:
    """`kyverno apply` pass/fail/warn/error/skip totals (processor/result.go:34-68) from the
    per-rule counts Engine.evaluate returns, through kpe_cli_summary."""
    arr = (Counts * max(len(counts), 1))()
    for i, c in enumerate(counts):
        arr[i].na, arr[i].pass_, arr[i].fail = c["na"], c["pass"], c["fail"]
        arr[i].warn, arr[i].error, arr[i].skip = c["warn"], c["error"], c["skip"]
        arr[i].undecided = c.get("undecided", 0)
    out = CliTotals()
    check(load().kpe_cli_summary(ps.h, arr, 1 if audit_warn else 0, ctypes.byref(out)))
    return {"pass": out.pass_, "fail": out.fail, "warn": out.warn, "error": out.error, "skip": out.skip}
