"""ctypes binding to oracle/build/liboracle.so — the CPU restatement used as the
checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only."""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")

STATUS = {0: "na", 1: "pass", 2: "fail", 3: "warn", 4: "error", 5: "skip", 7: "unsupported"}


class Oracle:
    def __init__(self, path=LIB):
        self.lib = L = ctypes.CDLL(path)
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_wildcard_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_pss_evaluate.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_pss_failing_checks.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                                ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_pss_failing_cv.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_pss_failing_cv_batch.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_pss_failing_cv_batch.restype = ctypes.c_long
        L.oracle_pss_failing_cv.restype = ctypes.c_longlong
        L.oracle_substitute.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_substitute.restype = ctypes.c_int
        L.oracle_substitute_doc.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_substitute_doc.restype = ctypes.c_int
        L.oracle_pss_message_ex.argtypes = [ctypes.c_char_p] * 6 + [ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_pss_message_ex.restype = ctypes.c_int
        L.oracle_pss_message.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                          ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_rule_names.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_validate.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_validate.restype = ctypes.c_long
        L.oracle_validate_ex.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                         ctypes.c_size_t, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_int]
        L.oracle_validate_ex.restype = ctypes.c_long
        cp = ctypes.c_char_p
        L.oracle_pattern_validate.argtypes = [cp, cp]
        L.oracle_validate_string.argtypes = [cp, cp, cp]
        L.oracle_string_pattern.argtypes = [cp, cp, ctypes.c_int, cp]
        L.oracle_get_operator.argtypes = [cp]
        L.oracle_number_to_string.argtypes = [cp, cp, ctypes.c_size_t]
        L.oracle_validate_element.argtypes = [cp, cp, ctypes.c_int, ctypes.c_int, cp, ctypes.c_size_t]
        L.oracle_match_pattern.argtypes = [cp, cp, ctypes.c_int, cp, ctypes.c_size_t]
        L.oracle_condition.argtypes = [cp, cp, cp]
        L.oracle_image_info.argtypes = [cp, cp, ctypes.c_size_t]
        L.oracle_images_context.argtypes = [cp, cp, ctypes.c_size_t]
        L.oracle_pattern_messages.argtypes = [cp, cp, ctypes.c_size_t, cp, ctypes.c_size_t]
        L.oracle_pattern_messages.restype = ctypes.c_long

    def wildcard(self, pattern, text):
        return bool(self.lib.oracle_wildcard_match(pattern.encode(), text.encode()))

    def pss_evaluate(self, rule, pod):
        return self.lib.oracle_pss_evaluate(json.dumps(rule).encode(), json.dumps(pod).encode())

    def failing_checks(self, level, version, pod):
        buf = ctypes.create_string_buffer(4096)
        r = self.lib.oracle_pss_failing_checks(level.encode(), version.encode(), json.dumps(pod).encode(), buf, 4096)
        if r < 0:
            return None
        s = buf.value.decode()
        return s.split(",") if s else []

    def failing_cv(self, level, version, pod):
        """Failing versioned checks (bit = CV index) of a pod, no exclusions; None on error."""
        r = self.lib.oracle_pss_failing_cv(level.encode(), version.encode(), json.dumps(pod).encode())
        return None if r < 0 else int(r)

    def failing_cv_batch(self, level, version, ndjson: bytes, nthreads=8):
        """failing_cv for every NDJSON row, each decoded by its own kind (getSpec); -1 where
        getSpec rejects the row. int64 array of N."""
        n = ndjson.count(b"\n") + 2
        out = np.zeros(n, dtype=np.int64)
        r = self.lib.oracle_pss_failing_cv_batch(level.encode(), version.encode(), ndjson, len(ndjson),
                                                 out.ctypes.data, n, nthreads)
        if r < 0:
            raise RuntimeError("oracle_pss_failing_cv_batch failed")
        return out[:r]

    def pss_message(self, rule, level, version, resource):
        """RuleResponse message of a podSecurity rule without exclusions (None on error)."""
        buf = ctypes.create_string_buffer(1 << 16)
        r = self.lib.oracle_pss_message(rule.encode(), level.encode(), version.encode(),
                                        json.dumps(resource).encode(), buf, 1 << 16)
        return None if r < 0 else buf.value.decode()

    def pss_message_ex(self, rule, level, version, resource, excludes, xexcludes=None):
        """(status, message) of a podSecurity rule with exclusions and, when a podSecurity
        PolicyException matched, its exclusions: 1 pass, 0 fail, 2 skip, -1 error."""
        buf = ctypes.create_string_buffer(1 << 16)
        r = self.lib.oracle_pss_message_ex(rule.encode(), level.encode(), version.encode(),
                                           json.dumps(resource).encode(), json.dumps(excludes).encode(),
                                           json.dumps(xexcludes).encode(), buf, 1 << 16)
        return r, (buf.value.decode() if r >= 0 else None)

    def substitute(self, msg, resource):
        """variables.SubstituteAll of a message over the resource's context: (0, text) a string,
        (1, json) another value, (-1, None) an error, (-2, None) outside the restated subset."""
        buf = ctypes.create_string_buffer(1 << 16)
        r = self.lib.oracle_substitute(json.dumps(resource).encode(), msg.encode(), buf, 1 << 16)
        return (r, buf.value.decode() if r >= 0 else None)

    def substitute_doc(self, doc, resource):
        """variables.SubstituteAll of a JSON document (leaves and map keys) over the resource's
        context: (0, document) or (-1, None) an error, (-2, None) outside the restatement."""
        buf = ctypes.create_string_buffer(1 << 16)
        r = self.lib.oracle_substitute_doc(json.dumps(resource).encode(), json.dumps(doc).encode(), buf, 1 << 16)
        return (r, json.loads(buf.value.decode()) if r == 0 else None)

    def rule_names(self, policies):
        buf = ctypes.create_string_buffer(1 << 20)
        n = self.lib.oracle_rule_names(json.dumps(policies).encode(), buf, 1 << 20)
        if n < 0:
            raise RuntimeError(self.lib.oracle_last_error().decode())
        return buf.value.decode().splitlines()

    NEEDS_ERR_TEXT = "\x01"  # the reference's message embeds a Go error string (not restated)

    def pattern_messages(self, policies, ndjson: bytes):
        """Per row, per rule: the pattern / anyPattern RuleResponse message (validate_resource.go
        :316-454), "" for other rules / no response, NEEDS_ERR_TEXT where it embeds an error."""
        pj = json.dumps(policies).encode()
        cap = 1 << 20
        while True:
            buf = ctypes.create_string_buffer(cap)
            n = self.lib.oracle_pattern_messages(pj, ndjson, len(ndjson), buf, cap)
            if n < 0:
                raise RuntimeError(self.lib.oracle_last_error().decode())
            if n < cap:
                return json.loads(buf.value.decode())
            cap = n + 1

    def validate(self, policies, ndjson: bytes, ns_labels=None, nthreads=1, exceptions=None, background=False):
        """Verdict matrix (N x R uint8, oracle status codes) for NDJSON resources, with
        PolicyExceptions (kyverno.io/v2beta1 objects) when given."""
        R = len(self.rule_names(policies))
        N = ndjson.count(b"\n") + 1
        out = np.zeros(max(N * R, 1), dtype=np.uint8)
        pj = json.dumps(policies).encode()
        if isinstance(ns_labels, (bytes, bytearray)):
            nl = bytes(ns_labels)
        else:
            nl = json.dumps(ns_labels).encode() if ns_labels else None
        xj = json.dumps(list(exceptions)).encode() if exceptions else None
        n = self.lib.oracle_validate_ex(pj, xj, 1 if background else 0, ndjson, len(ndjson), nl, out.ctypes.data,
                                        out.size, nthreads)
        if n < 0:
            raise RuntimeError(self.lib.oracle_last_error().decode())
        return out[: n * R].reshape(n, R)


    # ---- pattern path (values are JSON texts; integer literals stay int64) ----
    def _chk(self, r):
        if r < 0:
            raise RuntimeError(self.lib.oracle_last_error().decode())
        return r

    def pattern_validate(self, value_json, pattern_json):
        return bool(self._chk(self.lib.oracle_pattern_validate(value_json.encode(), pattern_json.encode())))

    def validate_string(self, value_json, pattern, op):
        return bool(self._chk(self.lib.oracle_validate_string(value_json.encode(), pattern.encode(), op.encode())))

    def string_pattern(self, value_json, pattern, which, op=""):
        return bool(self._chk(self.lib.oracle_string_pattern(value_json.encode(), pattern.encode(), which,
                                                             op.encode())))

    OPS = ["", ">=", "<=", "!", ">", "<", "-", "!-"]

    def get_operator(self, pattern):
        return self.OPS[self.lib.oracle_get_operator(pattern.encode())]

    def number_to_string(self, value_json):
        buf = ctypes.create_string_buffer(512)
        r = self._chk(self.lib.oracle_number_to_string(value_json.encode(), buf, 512))
        return (None, True) if r == 1 else (buf.value.decode(), False)

    ERR_KINDS = ["none", "conditional", "global", "negation", "other", "skip"]

    def validate_element(self, resource_json, pattern_json, mode=0, all_float=True):
        buf = ctypes.create_string_buffer(4096)
        k = self._chk(self.lib.oracle_validate_element(resource_json.encode(), pattern_json.encode(), mode,
                                                       int(all_float), buf, 4096))
        return self.ERR_KINDS[k], buf.value.decode()

    def match_pattern(self, resource_json, pattern_json, all_float=True):
        """validate.MatchPattern -> ('pass'|'skip'|'fail', path)."""
        buf = ctypes.create_string_buffer(4096)
        k = self._chk(self.lib.oracle_match_pattern(resource_json.encode(), pattern_json.encode(), int(all_float),
                                                    buf, 4096))
        return ["pass", "skip", "fail"][k], buf.value.decode()


    def condition(self, key_json, op, value_json):
        """variables.Evaluate of one constant condition: True / False, 'error' or 'unsupported'."""
        r = self.lib.oracle_condition(key_json.encode(), op.encode(), value_json.encode())
        return {1: True, 0: False, -1: "error"}.get(r, "unsupported")


    def image_info(self, image):
        """GetImageInfo (default configuration): a dict, or None on a parse error."""
        buf = ctypes.create_string_buffer(8192)
        r = self.lib.oracle_image_info(image.encode(), buf, 8192)
        return json.loads(buf.value.decode()) if r == 0 else None

    def images_context(self, resource):
        """The `images` context map of a resource (None: absent); 'error' when extraction fails."""
        buf = ctypes.create_string_buffer(1 << 16)
        r = self.lib.oracle_images_context(json.dumps(resource).encode(), buf, 1 << 16)
        if r == 1:
            return "error"
        self._chk(r)
        return json.loads(buf.value.decode())


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_inst = None


def load():
    global _inst
    if _inst is None:
        if not os.path.exists(LIB):
            build()
        _inst = Oracle()
    return _inst
