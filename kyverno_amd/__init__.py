"""kyverno_amd — MI355X-native batch evaluation of Kyverno validate rules.

The product path is libkpe.so (include/kpe.h): a C++ flattener/compiler plus
CDNA4 HIP kernels. This package is the Python host binding over that C-ABI
(ctypes) and a thin mirror of the reference's engine interface
(pkg/engine/api/engine.go:17-56) for batch callers. There is no CPU fallback:
evaluation without a working gfx950 device raises KpeError.
"""
from ._lib import KpeError, lib_path, load  # noqa: F401
from .engine import (  # noqa: F401
    SYNTH_C3,
    SYNTH_EDGE,
    SYNTH_FANOUT,
    SYNTH_MIXED,
    SYNTH_PODS,
    SYNTH_SELECTORS,
    Corpus,
    Device,
    Engine,
    EngineResponse,
    evaluate_sharded,
    packed_words,
    unpack_verdicts,
    PolicyContext,
    PolicySet,
    RuleResponse,
    RuleStatus,
    cli_summary,
    report_results,
    synth_ns_labels,
    synth_resources,
)
from .scan import BackgroundScanner, resource_hash, resource_hashes  # noqa: F401

__all__ = [
    "BackgroundScanner",
    "Corpus",
    "Device",
    "Engine",
    "EngineResponse",
    "KpeError",
    "PolicyContext",
    "PolicySet",
    "RuleResponse",
    "RuleStatus",
    "report_results",
    "cli_summary",
    "synth_ns_labels",
    "synth_resources",
    "load",
    "lib_path",
    "resource_hash",
    "resource_hashes",
]
