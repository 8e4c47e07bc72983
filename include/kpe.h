/*
 * kpe — MI355X-native batch policy evaluation for Kyverno's validate path.
 *
 * C-ABI drop-in boundary (plain pointers and sizes; no C++/torch types).
 * The reference has no FFI: these entry points are what a cgo shim behind
 * Kyverno's engine interfaces binds:
 *
 *   engineapi.Engine.Validate(ctx, PolicyContext) EngineResponse
 *       pkg/engine/api/engine.go:17-23, implemented by engine.Validate
 *       pkg/engine/engine.go:87-101 (rule loop pkg/engine/validation.go:16-80)
 *     -> kpe_evaluate() answers every (resource, rule) cell of a batch at once;
 *        the Go shim slices one row per PolicyContext.
 *   handlers.Handler.Process (validatePssHandler)
 *       pkg/engine/handlers/handler.go:13-23,
 *       pkg/engine/handlers/validation/validate_pss.go:31-112
 *     -> PSS rules of the compiled program (kpe_check_masks gives the failing
 *        PSA check IDs that become PodSecurityChecks / report "controls").
 *   autogen.ComputeRules  pkg/autogen/autogen.go:236-270
 *     -> kpe_program_compile() runs autogen once, at compile time.
 *   callers: cmd/cli/kubectl-kyverno/processor/policy_processor.go:168-179
 *            (kyverno apply loop) and pkg/controllers/report/utils/scanner.go:99-110
 *            (background scan) build one PolicyContext per (resource, policy);
 *            kpe_corpus_flatten() + kpe_evaluate() replace that loop for a batch.
 *
 * Verdict cell alphabet (engineapi.RuleStatus, pkg/engine/api/rulestatus.go:4-21;
 * "no RuleResponse" = not applicable):
 */
#ifndef KPE_H_
#define KPE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum kpe_verdict {
  KPE_NA = 0,    /* rule did not match the resource: no RuleResponse      */
  KPE_PASS = 1,  /* RuleStatusPass                                         */
  KPE_FAIL = 2,  /* RuleStatusFail                                         */
  KPE_WARN = 3,  /* RuleStatusWarn (reserved; never produced by validate)  */
  KPE_ERROR = 4, /* RuleStatusError (e.g. typed decode failure in getSpec) */
  KPE_SKIP = 5,  /* RuleStatusSkip                                         */
  KPE_UNDECIDED = 7 /* the device could not decide this cell (a documented device limit,
                       e.g. a condition list longer than the VM's list capacity, a resource
                       string that may be JSON where an operator would decode it): the
                       caller evaluates this (resource, rule) with the reference engine */
};

/* Library status codes (0 = OK). Library-level failures set kpe_last_error(). */
typedef int kpe_status;
enum {
  KPE_OK = 0,
  KPE_E_INVALID = 1,     /* malformed input (policy / resource JSON)             */
  KPE_E_UNSUPPORTED = 2, /* policy uses a construct this engine does not evaluate */
  KPE_E_DEVICE = 3,      /* HIP runtime error / no device / kernel not loadable   */
  KPE_E_LIMIT = 4,       /* a corpus exceeds a documented encoding limit          */
  KPE_E_STATE = 5        /* wrong call order (e.g. corpus not uploaded)           */
};

typedef struct kpe_device kpe_device;   /* one HIP device + stream               */
typedef struct kpe_program kpe_program; /* compiled policy set (after autogen)    */
typedef struct kpe_corpus kpe_corpus;   /* flattened, string-interned resources   */

/* Per-rule totals over a batch (pkg/engine/api/policyresponse.go:10-21 counting,
 * cmd/cli/kubectl-kyverno/processor/result.go:34-68 summary line). */
typedef struct kpe_counts {
  uint64_t na, pass, fail, warn, error, skip, undecided;
} kpe_counts;

/* Thread-local message for the last failing call on this thread. */
const char* kpe_last_error(void);
const char* kpe_version(void);

/* ---- device ------------------------------------------------------------ */
kpe_status kpe_device_open(int ordinal, kpe_device** out);
void kpe_device_close(kpe_device* dev);

/* ---- policies ---------------------------------------------------------- */
/* policies_json: one ClusterPolicy/Policy object or a JSON array of them
 * (kyverno.io/v1 schema, api/kyverno/v1/spec_types.go:240-284). Autogen is
 * applied (autogen.ComputeRules). Rules are laid out policy-major, in
 * ComputeRules order: column r of the verdict matrix is rule r. */
kpe_status kpe_program_compile(const char* policies_json, size_t len, kpe_program** out);
/* kpe_program_compile with PolicyExceptions (kyverno.io/v2beta1, api/kyverno/v2beta1/
 * policy_exception_types.go; the exception lister of engine.NewEngine, pkg/engine/exceptions.go:12-35,
 * consulted per rule at engine.go:286-293): exceptions_json is one PolicyException or a JSON array
 * (NULL / 0: none). A matched cell of a rule an exception names (policyName = the policy key,
 * ruleNames = go-wildcard globs) becomes KPE_SKIP when the exception's match block holds for the
 * resource (pkg/engine/utils/exceptions.go:14-47, validate_resource.go:43-56, validate_pss.go:45-58).
 * KPE_COMPILE_BACKGROUND drops exceptions with spec.background: false, as the background scanner's
 * FetchPolicyExceptions does (pkg/controllers/report/utils/utils.go:113-124); kyverno apply uses
 * every exception it is given. An exception with podSecurity controls re-evaluates a failing pod
 * under them (validate_pss.go:88-104); `conditions` that read the resource, and exceptions on rules
 * whose preconditions read it, are applied after the preconditions (exceptions.go:33-41).
 * KPE_E_UNSUPPORTED: several exceptions on one rule when one has podSecurity controls or
 * conditions that do not fold to true (the first matching one decides). */
#define KPE_COMPILE_BACKGROUND 1u
kpe_status kpe_program_compile_ex(const char* policies_json, size_t len, const char* exceptions_json, size_t exc_len,
                                  uint32_t flags, kpe_program** out);
int kpe_program_num_rules(const kpe_program* prog);
/* "<policy-name>/<rule-name>" of rule r (owned by prog). */
const char* kpe_program_rule_name(const kpe_program* prog, int r);
/* 1 if rule r is a podSecurity rule (check masks are meaningful for it). */
int kpe_program_rule_is_pss(const kpe_program* prog, int r);
void kpe_program_free(kpe_program* prog);

/* ---- resources --------------------------------------------------------- */
/* ndjson: one resource JSON object per line. ns_labels_json: optional
 * {"<namespace>": {"k": "v", ...}, ...} (the namespace label table the
 * reference reads per resource: PolicyContext.NamespaceLabels). */
kpe_status kpe_corpus_flatten(const char* ndjson, size_t len, const char* ns_labels_json, size_t ns_len,
                              kpe_corpus** out);
/* Same with flags. KPE_CORPUS_DOCS keeps every resource's document tape (its JSON as the
 * reference's unstructured map, pkg/engine/validate/validate.go:31 walks it) for
 * pattern / anyPattern rules; kpe_corpus_flatten sets it. Without it the corpus only
 * serves podSecurity and match-only programs (KPE_E_STATE otherwise). */
#define KPE_CORPUS_DOCS 1u
kpe_status kpe_corpus_flatten_ex(const char* ndjson, size_t len, const char* ns_labels_json, size_t ns_len,
                                 uint32_t flags, kpe_corpus** out);
int64_t kpe_corpus_num_resources(const kpe_corpus* c);
/* Host bytes of the columnar encoding (what one evaluation may read). */
int64_t kpe_corpus_bytes(const kpe_corpus* c);
/* 64-bit digest of every column and dictionary of the encoding (identity of two flattens of
 * the same input, e.g. the parallel flattener against a one-thread flatten). */
uint64_t kpe_corpus_digest(const kpe_corpus* c);
/* Per-row status of the flatten (host only, no device call): out[i] for each of the
 * kpe_corpus_num_resources rows. KPE_ROW_DECODE_ERROR: the typed decode of getSpec
 * (validate_pss.go:137-188, encoding/json into corev1.Pod / appsv1.Deployment /
 * batchv1.CronJob) would fail, so every podSecurity cell of the row is a RuleError.
 * KPE_ROW_LIMIT: past a per-resource encoding limit, every cell is KPE_UNDECIDED.
 * KPE_ROW_NO_SPEC: a kind getSpec does not decode ("could not find correct resource type"). */
#define KPE_ROW_DECODE_ERROR 1u
#define KPE_ROW_LIMIT 2u
#define KPE_ROW_NO_SPEC 4u
/* KPE_ROW_CONTEXT_ERROR: NewPolicyContext fails for the resource (AddImageInfos: an invalid image
 * reference or container entry, policycontext/policy_context.go:230), so the reference engine
 * gives no response for any rule and the scanner records an error; every cell is KPE_UNDECIDED. */
#define KPE_ROW_CONTEXT_ERROR 8u
kpe_status kpe_corpus_row_flags(const kpe_corpus* c, uint32_t* out);
/* Resource hash of incremental background scans: CalculateResourceHash
 * (pkg/utils/report/metadata.go:137-155), md5 of json.Marshal([labels, annotations, the object
 * without metadata / status / scale / spec.nodeName]) as 32 lower-case hex digits + NUL in out33.
 * The background controller rescans a resource when it differs from the hash its report
 * recorded (pkg/controllers/report/background/controller.go:247-297). Host only. */
kpe_status kpe_resource_hash(const char* resource_json, size_t len, char* out33);
/* The hash of every NDJSON row (the rows kpe_corpus_flatten makes), 32 hex digits per row into
 * out (no NUL), on up to 16 threads. out == NULL: returns the row count. Returns the row count,
 * or -KPE_E_INVALID when cap_rows is too small. A row that is not a JSON object (which the
 * flattener keeps with KPE_ROW_DECODE_ERROR) has no hash: its 32 bytes are '-' (never a hex
 * digest), so an incremental scan always re-evaluates it. */
int64_t kpe_resource_hashes(const char* ndjson, size_t len, char* out, int64_t cap_rows);
/* Copy the columns to device memory (HBM). Evaluation requires this. */
kpe_status kpe_corpus_upload(kpe_device* dev, kpe_corpus* c);
/* The corpus's per-pod PSA summary, built on dev (waits for it; builds it first when no LEAN
 * evaluation has yet): 2 words per row (include-free layout of kyverno_amd/csrc/schema.h PS_*:
 * x = OR of the pod's container state bitmaps, y = the list codes under the PSA library's fixed
 * sets). Diagnostics and the summary's digest test; evaluation never needs it on the host. */
kpe_status kpe_corpus_psa_summary(kpe_device* dev, kpe_corpus* c, uint32_t* out);
void kpe_corpus_free(kpe_corpus* c);

/* ---- evaluation -------------------------------------------------------- */
/* Evaluate every (resource, rule) cell on the device and copy results back.
 *   verdicts    : N x R bytes (row-major, kpe_verdict), may be NULL
 *   check_masks : N x R uint32 (bit k = PSA check k failed, kpe_pss_check_id
 *                 order; 0 for non-PSS rules), may be NULL
 *   counts      : R entries, may be NULL
 * Synchronous. Safe to call from several OS threads on distinct devices; calls
 * on one device are serialised by a per-device mutex. */
kpe_status kpe_evaluate(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint8_t* verdicts,
                        uint32_t* check_masks, kpe_counts* counts);

/* Asynchronous form for pipelines/benchmarks: enqueue one evaluation on the
 * device stream; results stay in device buffers owned by the corpus. No host
 * synchronisation. Use kpe_device_sync() and kpe_fetch() afterwards. */
kpe_status kpe_evaluate_async(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c);
/* kpe_evaluate_async with options: KPE_EVAL_MASKS also writes the check masks (device
 * buffers read by kpe_fetch / kpe_fetch_cv_masks); KPE_EVAL_COLD re-runs the binding's
 * per-corpus prologue (dictionary predicate pass, prologue image and, for a LEAN program, the
 * per-pod PSA summaries) as the first evaluation of a newly bound corpus does. */
#define KPE_EVAL_MASKS 1u
#define KPE_EVAL_COLD 2u
kpe_status kpe_evaluate_async_ex(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, unsigned flags);
/* n evaluations enqueued by one call, corpora cs[0 .. n-1] in order (a corpus may repeat), each
 * with the results kpe_evaluate_async_ex(dev, prog, cs[i], flags) gives: the batch form a scanner
 * driving many resident shards (or a benchmark) uses instead of n foreign-function calls. A run of
 * consecutive warm shards whose evaluation is the LEAN evaluation alone (a bound kind-only
 * podSecurity program, no later kernels) goes out as ceil(m / 24) multi-shard launches of
 * kpe_lean6_kernel: one grid over the shards' tiles instead of one launch per shard. Every launch
 * evaluates each pod's PSA checks from its pod, container, volume, sysctl and annotation columns. */
kpe_status kpe_evaluate_batch_async(kpe_device* dev, const kpe_program* prog, const kpe_corpus* const* cs, int n,
                                    unsigned flags);
kpe_status kpe_device_sync(kpe_device* dev);
kpe_status kpe_fetch(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint8_t* verdicts,
                     uint32_t* check_masks, kpe_counts* counts);

/* ---- verdict exchange and several devices in one process ---------------- */
/* Device address and size of the corpus's N x R verdict matrix after an evaluation of prog on
 * dev (waits for it): valid until the next evaluation of the corpus. A collective can send it
 * straight from HBM (RCCL over xGMI); SURVEY.md 8(e)'s verdict gather. */
kpe_status kpe_device_verdicts(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, void** dptr,
                               uint64_t* bytes);
/* The verdict matrix packed on the device into 3-bit cells (the kpe_verdict alphabet fits),
 * 10 per 32-bit word, row-major: cell i is bits 3*(i % 10) .. +2 of word i / 10. dst_dev is
 * device memory of dev holding at least kpe_packed_words(N * R) words (e.g. a torch tensor
 * that RCCL then sends); synchronous. kpe_unpack_verdicts expands it on the host. */
uint64_t kpe_packed_words(uint64_t cells);
kpe_status kpe_pack_verdicts(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint32_t* dst_dev,
                             uint64_t words);
kpe_status kpe_unpack_verdicts(const uint32_t* packed, uint64_t cells, uint8_t* out);
/* One logical corpus sharded over several devices of this process: shards[i] uploaded to
 * devs[i] (distinct devices), evaluated concurrently; verdicts = the shards' rows in order
 * (sum of N_i x R bytes, may be NULL), counts = the per-rule sums (R entries, may be NULL). The
 * Go host's single-process multi-GPU entry. */
kpe_status kpe_evaluate_sharded(kpe_device* const* devs, kpe_corpus* const* shards, int nshards,
                                const kpe_program* prog, uint8_t* verdicts, kpe_counts* counts);

/* PSA check id k (bit k of a check mask), e.g. "capabilities_restricted". */
const char* kpe_pss_check_id(int k);
int kpe_pss_num_checks(void);

/* Versioned-check form of the check masks (after kpe_evaluate / kpe_evaluate_async with
 * masks): N x R uint32, bit v = PSA versioned check v failed (0 unless the cell is FAIL).
 * A rule pinned to a version runs every version of a check up to it
 * (pkg/pss/evaluate.go:51-66, evaluatePSS), so one check id can fail more than once;
 * kpe_pss_cv_check(v) is the check id index of versioned check v. Bit 31 (KPE_CVM_XMATCH)
 * of a FAIL cell of a rule with a podSecurity PolicyException: the exception matched the
 * resource, so its exclusions shape the cell's fail message (kpe_report_results_msg). */
#define KPE_CVM_XMATCH (1u << 31)
/* The versioned-check bits of a cv mask word (bits 0 .. kpe_pss_num_cv() - 1): mask with it
 * before walking set bits as versioned checks (bit 31 is a flag, not a check). */
#define KPE_CVM_CHECKS_ALL 0x7FFFFFFFu
kpe_status kpe_fetch_cv_masks(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint32_t* cv_masks);
int kpe_pss_num_cv(void);
int kpe_pss_cv_check(int v);

/* `kyverno apply` summary line (cmd/cli/kubectl-kyverno/processor/result.go:34-68) from the
 * per-rule counts of kpe_evaluate / kpe_fetch: unscored fails (policies.kyverno.io/scored:
 * "false") and, with audit_warn (--audit-warn), fails of Audit policies count as warn; a
 * response is counted once per validate rule of its policy with the same name (the
 * reference matches by name). KPE_E_UNSUPPORTED when audit_warn meets
 * validationFailureActionOverrides (the action then depends on each resource's namespace). */
typedef struct kpe_cli_totals {
  uint64_t pass, fail, warn, error, skip;
} kpe_cli_totals;
kpe_status kpe_cli_summary(const kpe_program* prog, const kpe_counts* counts, int audit_warn, kpe_cli_totals* out);

/* PolicyReport results of one resource (pkg/utils/report/results.go:89-156,
 * EngineResponseToReportResults), as the JSON array encoding/json writes for
 * []PolicyReportResult: one object per rule with a response, in rule order, with
 * source, policy (cache.MetaNamespaceKeyFunc key), rule, result (unscored fail => warn),
 * scored, properties {controls, standard, version} for failing podSecurity rules,
 * category and severity. No message (kpe_report_results_msg / _ex) and no timestamp.
 *   verdict_row : R verdict cells of the resource (kpe_evaluate row)
 *   cv_mask_row : R cells of kpe_fetch_cv_masks, or NULL (then no controls)
 * Writes at most cap-1 bytes plus NUL; returns the full length (call again with a larger
 * buffer when it is >= cap), or a negative kpe_status. Host only; no device call. */
long kpe_report_results(const kpe_program* prog, const uint8_t* verdict_row, const uint32_t* cv_mask_row, char* buf,
                        size_t cap);
/* kpe_report_results with the RuleResponse `message` of each result, rendered from the
 * resource's JSON (the EngineResponse resource, resource_len bytes): podSecurity pass
 * ("Validation rule '<rule>' passed.", validate_pss.go:85) and fail (validate_pss.go:108:
 * FormatChecksPrint of the failing checks after convertChecks; with podSecurity.exclude or a
 * podSecurity PolicyException, over the checks their exclusions leave), validate.pattern pass
 * ("validation rule '<rule>' passed.", validate_resource.go:339), validate.deny pass
 * ("validation rule '<rule>' passed.") and, when the deny block's condition message is known
 * without the resource (no condition `message`, or conditions folded at compile time), fail
 * (getDenyMessage, validate_resource.go:279-300: the rule message joined with the condition
 * message, or "validation error: rule <rule> failed" when both are empty); preconditions skips
 * of deny rules whose preconditions carry no `message` ("preconditions not met", engine.go:283)
 * and of preconditions folded at compile time; a PolicyException skip ("rule skipped due to
 * policy exception <key>") when it is the skip's only cause. A message with variables is
 * substituted over the resource (variables.SubstituteAll, vars.go:311-389) when every variable
 * is a `request.object` path of members and [N] indexes. A substitution error (a member missing
 * from an object) fails SubstituteAll: the pattern message is then not rendered (its reference
 * text embeds the Go error string), and getDenyMessage returns the condition message as is.
 * Messages with other variables are not rendered. Condition messages that depend on where a
 * block stopped need the condition traces (kpe_report_results_ex). Host only. */
long kpe_report_results_msg(const kpe_program* prog, const uint8_t* verdict_row, const uint32_t* cv_mask_row,
                            const char* resource_json, size_t resource_len, char* buf, size_t cap);

/* Failing paths of pattern cells, for their report messages (validate_resource.go:316-454;
 * validate.go MatchPattern PatternError.Path). After kpe_evaluate / kpe_evaluate_async of the
 * same program and corpus, for each listed cell (row * R + column) the device re-walks every root
 * of the cell's validate.pattern / anyPattern rule (at most KPE_TRACE_ROOTS; for a FAIL / ERROR
 * cell of a validate.foreach rule that a pattern entry decided, that entry's roots on the
 * element it validated, kpe_fetch_cond_traces_ex) and records the
 * path of the failure that decided it: out[i * KPE_TRACE_ROOTS * KPE_TRACE_WORDS + k *
 * KPE_TRACE_WORDS + w], w = 0: component count (bits 0-7) | KPE_TR_TRUNC | the root's verdict
 * << 16 | KPE_TR_VALID; w = 1..15: components (a pattern member, KPE_TC_KEY | key id, or
 * KPE_TC_IDX | array index). A cell of a rule without patterns gives a zero record. */
#define KPE_TRACE_WORDS 16u
#define KPE_TRACE_ROOTS 4u
#define KPE_TC_IDX 0x80000000u
#define KPE_TC_KEY 0x40000000u
#define KPE_TR_TRUNC 0x100u
#define KPE_TR_VALID 0x1000000u
kpe_status kpe_pattern_traces(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, const uint64_t* cells,
                              uint64_t ncells, uint32_t* out);
/* kpe_report_results_msg plus the pattern messages: `traces` holds the row's R cells in
 * kpe_pattern_traces layout (R * KPE_TRACE_ROOTS * KPE_TRACE_WORDS words; only pattern-rule
 * cells are read). Adds: validate.pattern fail ("validation error: <message>. rule <rule> failed
 * at path <path>", buildErrorMessage), anyPattern pass ("validation rule '<rule>' anyPattern[<i>]
 * passed.") and fail (buildAnyPatternErrorMessage over "rule <rule>[<i>] failed at path <path>").
 * The rule message is substituted as in kpe_report_results_msg. Not rendered (no message):
 * messages with other variables or a failed substitution, empty-path failures (their text is the
 * Go error string), skips, anyPattern fails with more than KPE_TRACE_ROOTS patterns. */
long kpe_report_results_msg_tr(const kpe_program* prog, const kpe_corpus* corpus, const uint8_t* verdict_row,
                               const uint32_t* cv_mask_row, const uint32_t* traces, const char* resource_json,
                               size_t resource_len, char* buf, size_t cap);

/* Condition traces, for the condition messages of validate rules (variables/evaluate.go:31-125):
 * after kpe_evaluate / kpe_evaluate_async of the same program and corpus, rows [row0, row0 +
 * nrows) into out (nrows x R words, row-major). A rule whose preconditions are evaluated per
 * resource, or whose validate.deny conditions carry a `message`, records where each block
 * stopped: the preconditions in bits 0-15, the deny block in bits 16-31, each as the index of
 * the first true `any` condition (bits 0-6), of the first false `all` condition (bits 7-13),
 * 0x4000 evaluated without an error, 0x8000 it held. Other cells (and blocks of more than 127
 * conditions) are 0. */
kpe_status kpe_fetch_cond_traces(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint64_t row0,
                                 uint64_t nrows, uint32_t* out);
/* Condition traces with the foreach and error records (report time): rows [row0, row0 + nrows)
 * into out, nrows x R x KPE_CTRACE_WORDS words. Word 0 of a cell is kpe_fetch_cond_traces' word,
 * where a block that raised an error records which condition raised it and on which side
 * (KPE_CT_ERR without the evaluated bit 0x4000: bits 0-6 the condition, any conditions first,
 * then all; bits 7-8 0 the key's substitution, 1 the value's, 2 the operator). For validate.foreach
 * rules (validateElements, validate_resource.go:206-254) the words describe the element that
 * decided a FAIL / ERROR cell: word 0 bits 16-31 its deny block (or its preconditions' error),
 * word 1 its path (nesting depth, what decided it, per level the entry and the element index),
 * words 2 and 3 the element's and the validated element's document nodes. The words of other cells
 * and of foreach cells that are not FAIL / ERROR are unspecified. */
#define KPE_CTRACE_WORDS 4u
#define KPE_CT_ERR 0x8000u
kpe_status kpe_fetch_cond_traces_ex(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint64_t row0,
                                    uint64_t nrows, uint32_t* out);
/* kpe_report_results_msg_tr plus the condition messages of kpe_fetch_cond_traces (cond_traces:
 * the row's R words, or NULL) or kpe_fetch_cond_traces_ex (cond_traces_ex, the row's R x
 * KPE_CTRACE_WORDS words; it takes precedence):
 *   - a preconditions skip (engine.go:282-284): "preconditions not met; <condition message>" of
 *     any validate rule, for preconditions evaluated per resource or folded at compile time;
 *   - validate.deny fail: getDenyMessage (validate_resource.go:279-300), the rule message joined
 *     with the deny block's condition message by "; " and substituted over the resource (on a
 *     substitution error the condition message as is);
 *   - a PolicyException skip of a rule whose preconditions read the resource, once the trace
 *     shows they held ("rule skipped due to policy exception <key>").
 * Preconditions and deny conditions are not substituted into condition messages before they join
 * (the reference substitutes only getDenyMessage's joined text).
 * With cond_traces_ex (and the corpus, for the element's document):
 *   - validate.foreach pass: "rule passed" (validate_resource.go:203); fail / error: the deciding
 *     element's response wrapped once per nesting level, "validation failure: <message>"
 *     (:239-247), where <message> is getDenyMessage over the element's context, the pattern /
 *     anyPattern message of the entry's walk on the element (kpe_pattern_traces records the
 *     foreach cell's element walk), or a RuleError text below; AddElementToContext's
 *     "failed to process foreach: cannot use elementScope=true ..." (:218-221);
 *   - RuleError texts: "failed to evaluate preconditions: <err>" (engine.go:279-281,
 *     validate_resource.go:125-128), "failed to check deny conditions: <err>" (:269-271),
 *     "variable substitution failed: <err>" (:139-141), "failed to deserialize anyPattern, expected
 *     type array: <err>" (:347-350), with <err> the substitution error the reference words itself:
 *     "failed to substitute variables in condition key|value: failed to resolve <var> at path <path>:
 *     JMESPath query failed: Unknown key \"<k>\" in path" (variables/evaluate.go:14-27, vars.go:
 *     311-389, context/evaluate.go:27-31), "invalid query (nil)", "expected string after
 *     substituting variables in key ...", "failed to create handler for condition operator".
 * Not rendered: pattern skips and empty-path pattern errors (their text is validate.go's chain of
 * anchor errors with Go %v renderings of resource and pattern values), errors whose text
 * go-jmespath words itself (a function's argument error), messages with variables outside the
 * restated paths, element<n> variables of an outer foreach level, and the RuleResponse timestamp. */
typedef struct kpe_report_args {
  const kpe_program* prog;
  const kpe_corpus* corpus;        /* pattern traces' key names; may be NULL without pattern traces */
  const uint8_t* verdict_row;      /* R verdict cells */
  const uint32_t* cv_mask_row;     /* R cells of kpe_fetch_cv_masks, or NULL */
  const uint32_t* pattern_traces;  /* kpe_pattern_traces layout for the row, or NULL */
  const uint32_t* cond_traces;     /* R words of kpe_fetch_cond_traces, or NULL */
  const char* resource_json;       /* the resource (NULL: no messages) */
  size_t resource_len;
  const uint32_t* cond_traces_ex;  /* R x KPE_CTRACE_WORDS words of kpe_fetch_cond_traces_ex, or NULL */
} kpe_report_args;
long kpe_report_results_ex(const kpe_report_args* args, char* buf, size_t cap);

/* ---- instrumentation (HIP events on the evaluation stream) ---------------- */
typedef struct kpe_kernel_stats {
  uint64_t launches;        /* timed launches since the last reset: one per evaluation, one per
                               multi-shard LEAN launch of kpe_evaluate_batch_async */
  double pss_kernel_ms;     /* summed duration of the resource-scan kernel      */
  double dict_kernel_ms;    /* summed duration of the dictionary predicate pass */
  double scan_bytes;        /* algorithmic bytes one scan-kernel launch reads+writes */
  double pattern_kernel_ms; /* summed duration of the kernels after the scan (condition, exclusion,
                               pattern-rule kernels; 0 without such rules) */
  double pattern_bytes;     /* algorithmic bytes of one pattern-kernel launch: every resource's
                               document tape (8 B per entry) and root offset once, plus the verdict
                               matrix read and written */
  int32_t scan_kernel;      /* the scan instantiation of the last timed launch: 1 kpe_scan_kernel
                               (general), 2 its LEAN instantiation (corpora past 4 GiB of pod
                               records), 7 kpe_lean6_kernel (one shard), 9 kpe_lean6_kernel (a multi-shard launch) */
  int32_t pad_;
  double scan_bytes_sum;    /* algorithmic bytes of every timed scan-kernel launch since the last reset,
                               summed (multi-shard launches differ in size: the mean launch carries
                               scan_bytes_sum / launches, not the last launch's scan_bytes) */
  double pattern_bytes_sum; /* the same for the pattern kernel's algorithmic bytes */
  double pss_kernel_ms_min, pss_kernel_ms_max, pss_kernel_ms_sq;  /* the scan launches' shortest and
                               longest duration and the sum of squared durations (spread) */
} kpe_kernel_stats;
kpe_status kpe_device_set_timing(kpe_device* dev, int enabled);
kpe_status kpe_device_kernel_stats(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c,
                                   kpe_kernel_stats* out, int reset);

#ifdef __cplusplus
}
#endif
#endif /* KPE_H_ */
