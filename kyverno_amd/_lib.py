"""ctypes binding to the C-ABI in include/kpe.h (libkpe.so, built in-tree)."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class KpeError(RuntimeError):
    """A non-zero kpe_status; `status` carries the code (include/kpe.h)."""

    def __init__(self, status, msg):
        super().__init__(f"kpe status {status}: {msg}")
        self.status = status


class CliTotals(ctypes.Structure):
    _fields_ = [("pass_", ctypes.c_uint64), ("fail", ctypes.c_uint64), ("warn", ctypes.c_uint64),
                ("error", ctypes.c_uint64), ("skip", ctypes.c_uint64)]


class Counts(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("na", "pass_", "fail", "warn", "error", "skip", "undecided")]


class KernelStats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_uint64), ("pss_kernel_ms", ctypes.c_double),
                ("dict_kernel_ms", ctypes.c_double), ("scan_bytes", ctypes.c_double),
                ("pattern_kernel_ms", ctypes.c_double), ("pattern_bytes", ctypes.c_double),
                ("scan_kernel", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("scan_bytes_sum", ctypes.c_double), ("pattern_bytes_sum", ctypes.c_double),
                ("pss_kernel_ms_min", ctypes.c_double), ("pss_kernel_ms_max", ctypes.c_double),
                ("pss_kernel_ms_sq", ctypes.c_double)]


def lib_path():
    return os.environ.get("KPE_LIB", os.path.join(HERE, "libkpe.so"))


def load():
    """Load libkpe.so; raises if it is missing (no silent fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise KpeError(-1, f"{path} not built (run `make -C kyverno_amd` or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    vp, cp, sz, i32, i64 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64
    L.kpe_last_error.restype = cp
    L.kpe_version.restype = cp
    L.kpe_device_open.argtypes = [i32, ctypes.POINTER(vp)]
    L.kpe_device_close.argtypes = [vp]
    L.kpe_program_compile.argtypes = [cp, sz, ctypes.POINTER(vp)]
    L.kpe_program_compile_ex.argtypes = [cp, sz, cp, sz, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.kpe_resource_hash.argtypes = [cp, sz, ctypes.c_char_p]
    L.kpe_resource_hashes.argtypes = [cp, sz, ctypes.c_char_p, i64]
    L.kpe_resource_hashes.restype = i64
    L.kpe_program_num_rules.argtypes = [vp]
    L.kpe_program_rule_name.argtypes = [vp, i32]
    L.kpe_program_rule_name.restype = cp
    L.kpe_program_rule_is_pss.argtypes = [vp, i32]
    L.kpe_program_free.argtypes = [vp]
    L.kpe_corpus_flatten.argtypes = [cp, sz, cp, sz, ctypes.POINTER(vp)]
    L.kpe_corpus_flatten_ex.argtypes = [cp, sz, cp, sz, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.kpe_corpus_num_resources.argtypes = [vp]
    L.kpe_corpus_num_resources.restype = i64
    L.kpe_corpus_bytes.argtypes = [vp]
    L.kpe_corpus_bytes.restype = i64
    L.kpe_corpus_digest.argtypes = [vp]
    L.kpe_corpus_digest.restype = ctypes.c_uint64
    L.kpe_corpus_row_flags.argtypes = [vp, vp]
    L.kpe_corpus_upload.argtypes = [vp, vp]
    L.kpe_corpus_psa_summary.argtypes = [vp, vp, vp]
    L.kpe_corpus_free.argtypes = [vp]
    L.kpe_evaluate.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(Counts)]
    L.kpe_evaluate_async.argtypes = [vp, vp, vp]
    L.kpe_evaluate_async_ex.argtypes = [vp, vp, vp, ctypes.c_uint]
    L.kpe_evaluate_batch_async.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_uint]
    L.kpe_device_sync.argtypes = [vp]
    L.kpe_device_verdicts.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)]
    L.kpe_packed_words.argtypes = [ctypes.c_uint64]
    L.kpe_packed_words.restype = ctypes.c_uint64
    L.kpe_pack_verdicts.argtypes = [vp, vp, vp, vp, ctypes.c_uint64]
    L.kpe_unpack_verdicts.argtypes = [vp, ctypes.c_uint64, vp]
    L.kpe_evaluate_sharded.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i32, vp, vp, ctypes.POINTER(Counts)]
    L.kpe_fetch.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(Counts)]
    L.kpe_pss_check_id.argtypes = [i32]
    L.kpe_pss_check_id.restype = cp
    L.kpe_fetch_cv_masks.argtypes = [vp, vp, vp, vp]
    L.kpe_pss_cv_check.argtypes = [i32]
    L.kpe_report_results.argtypes = [vp, vp, vp, ctypes.c_char_p, sz]
    L.kpe_report_results.restype = ctypes.c_long
    L.kpe_report_results_msg.argtypes = [vp, vp, vp, ctypes.c_char_p, sz, ctypes.c_char_p, sz]
    L.kpe_report_results_msg.restype = ctypes.c_long
    L.kpe_report_results_msg_tr.argtypes = [vp, vp, vp, vp, vp, ctypes.c_char_p, sz, ctypes.c_char_p, sz]
    L.kpe_report_results_msg_tr.restype = ctypes.c_long
    L.kpe_pattern_traces.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, vp]
    L.kpe_pattern_traces.restype = ctypes.c_int
    L.kpe_fetch_cond_traces.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint64, vp]
    L.kpe_fetch_cond_traces.restype = ctypes.c_int
    L.kpe_report_results_ex.argtypes = [vp, ctypes.c_char_p, sz]
    L.kpe_fetch_cond_traces_ex.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_uint64, vp]
    L.kpe_report_results_ex.restype = ctypes.c_long
    L.kpe_cli_summary.argtypes = [vp, ctypes.POINTER(Counts), i32, ctypes.POINTER(CliTotals)]
    L.kpe_device_set_timing.argtypes = [vp, i32]
    L.kpe_device_kernel_stats.argtypes = [vp, vp, vp, ctypes.POINTER(KernelStats), i32]
    L.kpe_synth_resources.argtypes = [ctypes.c_uint64, i64, i64, i32, ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(sz)]
    L.kpe_synth_free.argtypes = [vp]
    L.kpe_debug_lean_kind.argtypes = [vp, ctypes.c_uint64]
    L.kpe_synth_ns_labels.argtypes = [ctypes.c_uint64, i64, i32, ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_size_t)]
    _LIB = L
    return L


def check(st):
    if st != 0:
        raise KpeError(st, load().kpe_last_error().decode(errors="replace"))
