// Compiled policy set: rules after autogen, lowered to the device program
// (schema.h KpeRule/KpeFilter/KpeTerm tables) plus the string predicates the
// device evaluates over the corpus dictionaries.
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "pss_msg.hpp"
#include "schema.h"

namespace kpe {

struct Pred {
  uint32_t domain;
  std::vector<std::string> globs;  // OR of go-wildcard patterns
  uint32_t special = 0;            // PRED_SPECIAL_*: a validity test instead of globs
  bool global_only = false;        // read outside the scan kernel (kept in HBM, never LDS-only)
};

// Compiled validate.pattern / anyPattern trees (schema.h PN_* / PM_* / PL_* / PC_*).
// Member names and string operands are kept as text: a binding resolves names to corpus
// D_KEY ids and the device program turns operands into pattern records.
struct PatProgram {
  std::vector<KpePNode> nodes;
  std::vector<uint32_t> members;       // 4 words per member; y = index into keys
  std::vector<std::string> keys;       // member names
  std::vector<uint32_t> lists;         // node lists (PN_ARR_POS / PN_EXLIST)
  std::vector<KpeLeaf> leaves;
  std::vector<KpeCond> conds;          // KpeCond.pat / KpeLeaf.exact index operands
  std::vector<std::string> operands;   // glob operand text
  std::vector<uint8_t> operand_exact;  // 1: compare verbatim (the `value == pattern` check)
  std::vector<uint32_t> roots;         // 2 words per root: node, anchor slots used
  std::vector<KpePatRule> rules;
  std::vector<KpePVar> vars;           // pattern variable slots (PL_VAR / PT_VAR)
  std::vector<uint32_t> tpieces;       // 2 words per template piece (PT_*)
  std::vector<uint8_t> ttext;          // template texts
  uint32_t vkey_groups = 0;            // maps with several keys with variables (PVF_GROUP ids)
};
// Compiled preconditions / deny / foreach-deny programs (schema.h QO_* / KpeC*), evaluated per
// resource by kpe_cond_kernel. Field names are kept as text: a binding resolves them to corpus
// D_KEY ids.
struct CondProgram {
  std::vector<uint32_t> ops;  // 2 words per op
  std::vector<KpeCExpr> exprs;
  std::vector<KpeVTmpl> tmpls;
  std::vector<KpeCCond> conds;
  std::vector<KpeCBlock> blocks;
  std::vector<KpeCForeach> fes;
  std::vector<KpeCRule> rules;
  std::vector<KpeScalar> consts;  // constant table (SC_T_* types, SC_T_ARR lists in clist)
  std::vector<char> ctext;        // constant texts
  std::vector<uint32_t> clist;    // elements of constant lists
  std::vector<uint32_t> tpieces;  // VT_TMPL pieces, 2 words each: PT_TEXT | len << 1, ctext offset /
                                  // PT_VAR, expression
  std::vector<std::string> fields;
  uint32_t nmsg = 0;  // condition trace slots (KpeCRule::mslot)
};
// podSecurity rules with exclusions (schema.h KpeXRule / KpeXExcl), evaluated per pod by
// kpe_pssx_kernel after the scan. Predicate fields hold predicate ids (resolved per binding).
struct PssxProgram {
  std::vector<KpeXRule> rules;
  std::vector<KpeXExcl> excl;
  std::vector<std::string> rf_ann;  // XRF_ANN annotation keys K of restrictedField "metadata.annotations[K]"
};
#define PRED_SPECIAL_NONE 0u
#define PRED_SPECIAL_QNAME 1u   // validation.IsQualifiedName (label keys)
#define PRED_SPECIAL_LABVAL 2u  // validation.IsValidLabelValue

// Fixed predicate slots used by the PSS kernel (indices into Program::preds).
struct PssPreds {
  int32_t apparmor_key = -1, apparmor_val_ok = -1, seccomp_pod_key = -1, seccomp_ann_ok = -1;
  int32_t caps_baseline_ok = -1, cap_nbs = -1, cap_all = -1;
  int32_t sysctl[3] = {-1, -1, -1};  // 1.0, 1.27, 1.29 allow-lists
};

struct DeviceProgram;  // kpe_api.cpp

// What a PolicyReportResult carries for rule r besides its verdict
// (pkg/utils/report/results.go:89-156, EngineResponseToReportResults).
// The `message`s of one condition block (kyvernov1.Condition.Message) in evaluation order, and
// EvaluateConditions' message (variables/evaluate.go:31-125) from where the block stopped.
struct CondMsgs {
  bool present = false;  // a non-null block
  bool old = false;      // the deprecated list form (evaluateOldConditions)
  bool has_any = false;  // an `any` list (even empty: it then never holds)
  std::vector<std::string> any, all;  // the old form's list is `all`
  bool has_text() const;
  // as / ls: the first true `any` / first false `all` condition (schema.h CT_ANY / CT_ALL)
  std::string render(uint32_t as, uint32_t ls, bool held) const;
};
// stringutils.JoinNonEmpty
std::string join_non_empty(const std::vector<std::string>& v, const std::string& sep);

// A validate.foreach entry as the messages need it (parallel to CondProgram::fes): the raw blocks
// and pattern (document-order JSON, reparsed for a failing cell) and the deny block's messages
struct FeReport {
  uint32_t kind = FE_NONE;  // FE_*
  std::string pre_json, deny_json, pattern_json;
  CondMsgs deny_msgs;
  bool any = false;          // anyPattern
  std::string any_bad_type;  // an anyPattern that is not a list: its JSON type name
  uint32_t nested0 = 0, nnested = 0;  // FE_NEST: entries [nested0, + nnested)
  uint32_t root0 = 0, nroots = 0;     // FE_PAT: pattern roots
};

struct RuleReport {
  std::string policy_key;  // cache.MetaNamespaceKeyFunc: "<ns>/<name>" or "<name>"
  std::string rule;        // rule name after autogen
  std::string category;    // policies.kyverno.io/category
  std::string severity;    // SeverityFromString(policies.kyverno.io/severity)
  std::string pss_level, pss_version;  // podSecurity rules: PodSecurityChecks.Level / Version
  bool scored = true;      // policies.kyverno.io/scored != "false"
  bool has_validate = false;  // rule.HasValidate() (processor/result.go:42)
  bool audit = true;          // spec.validationFailureAction.Audit() (!Enforce, spec_types.go:31-37)
  bool overrides = false;     // spec.validationFailureActionOverrides non-empty (per-namespace action)
  uint32_t name_mult = 1;     // validate rules of the policy with this name (result.go:44 name match)
  bool pss = false;
  bool pss_excl = false;      // podSecurity.exclude or a podSecurity PolicyException (fail messages not rendered)
  bool msg_pattern = false;   // validate.pattern rule: pass message "validation rule '<rule>' passed."
  // validate.deny rule (`msg_deny`): pass "validation rule '<rule>' passed.", fail getDenyMessage
  // (validate_resource.go:279-300) of the rule message `deny_vmsg` and the deny block's condition
  // message: `deny_cm` when it is known at compile time (no condition `message`, or a block that
  // folds), else (`cond_deny`) rendered from the cell's condition trace. `msg_pre_skip`: its
  // preconditions carry no `message`, so a skip without a PolicyException is "preconditions not
  // met" (engine.go:283) even without condition traces.
  bool msg_deny = false, msg_pre_skip = false, cond_deny = false;
  std::string deny_vmsg, deny_cm;
  // Condition messages (variables/evaluate.go:31-125) of the preconditions and the deny block;
  // `cond_slot`: the rule has a condition trace slot (KpeCRule::mslot)
  CondMsgs pre_msgs, deny_msgs;
  bool cond_slot = false;
  // preconditions that fold to false at compile time: the skip message (engine.go:282-284)
  bool pre_const_skip = false;
  std::string pre_skip_msg;
  // validate.pattern / anyPattern rule (kpe_pattern_traces paths): failure messages are
  // buildErrorMessage / buildAnyPatternErrorMessage (validate_resource.go:418-454) of the rule's
  // validate.message; `vmsg_vars`: it holds variables (substituted per resource, substitute_message)
  // the rule's only PolicyException when its skips can only come from it: RuleSkip message
  // "rule skipped due to policy exception <key>" and report property exception: <name>
  std::string exc_key, exc_name;
  bool exc_after_pre = false;  // preconditions read the resource: only a skip after they held (trace)
  // podSecurity rules with exclusions: the rule's versioned checks and exclude entries, and a
  // podSecurity PolicyException's (fail messages after ApplyPodSecurityExclusion, pss_msg.cpp)
  uint32_t pss_cv = 0;
  std::vector<PssExcl> pss_excludes, pss_xexcludes;
  bool pss_has_xexcl = false;
  bool pat_rule = false, any_pattern = false, vmsg_vars = false;
  uint32_t pat_roots = 0;
  std::string vmsg;
  // RuleError texts (validate_resource.go:127,140,270,349; engine.go:279-281): the rule's raw
  // preconditions, deny conditions and pattern / anyPattern (document-order JSON), reparsed for an
  // erroring cell; `pat_vars`: the pattern has {{ }} variables (a substitution error is possible)
  std::string pre_json, deny_json, pattern_json, any_bad_type;
  bool pat_vars = false;
  // validate.foreach rules: the entries [fe0, fe0 + nfe) of Program::fe_reports and the four-word
  // condition trace slot (schema.h FT_*); the entries' messages use `vmsg` (the rule's message)
  bool foreach = false;
  uint32_t fe0 = 0, nfe = 0;
};

struct Program {
  std::vector<std::string> rule_names;  // "<policy>/<rule>"
  std::vector<RuleReport> reports;      // per rule, same order
  std::vector<KpeRule> rules;
  std::vector<KpeFilter> filters;
  std::vector<uint32_t> fterms;  // term indices of the filters
  std::vector<KpeTerm> terms;    // distinct terms (each evaluated once per resource)
  std::vector<KpeKindSel> kindsels;
  std::vector<KpeAnnPair> annpairs;
  std::vector<KpeSelector> selectors;
  std::vector<KpeSelReq> selreqs;
  std::vector<Pred> preds;
  PssPreds pss;
  uint32_t cv_union = 0;  // union of cv_mask over rules
  std::vector<uint32_t> cv_classes;  // distinct cv_masks of PSS rules
  bool any_apply_one = false;
  bool any_exc = false;    // some rule has PolicyExceptions (KpeRule::exc)
  bool any_const = false;  // some rule has a constant handler (H_CONST_*)
  bool any_pss = false;
  bool any_fe_pat = false;  // some foreach entry has a pattern / anyPattern (kpe_cond_kernel<true>)
  PatProgram pat;  // pattern rules (H_PATTERN)
  CondProgram cond;  // rules with preconditions / deny / foreach evaluated per resource
  std::vector<FeReport> fe_reports;  // per CondProgram::fes entry
  PssxProgram pssx;  // podSecurity.exclude
  int32_t pssx_preds[9] = {-1, -1, -1, -1, -1, -1, -1, -1, -1};  // PSA predicates of kpe_pssx_kernel
  DeviceProgram* devs[16] = {};  // per device ordinal: the program's tables on that device (kpe_api.cpp)
  std::mutex dev_mu;  // first-time creation of a devs[] slot (two device handles may share an ordinal)
  ~Program();
};

// Throws CompileError (unsupported construct) or std::invalid_argument (bad JSON).
struct CompileError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
std::unique_ptr<Program> compile_policies(const char* json, size_t len, const char* exceptions = nullptr,
                                          size_t exc_len = 0, bool background = false);

// variables.SubstituteAll of a rule message over one resource (program.cpp): false when the
// message holds variables outside the restated `request.object` path grammar; *nonstring: the
// message is one variable whose value is not a string (*out is its JSON).
// *subst_err (when given): false was returned for a substitution error (a member missing from
// an object, go-jmespath NotFound), not for an unrestated variable.
// MsgElem: the foreach element of the context (AddElement, context.go: element, element<depth>,
// elementIndex, elementIndex<depth>), as the JSON of its document node.
struct MsgElem {
  std::string json;
  int depth = 0;
  int64_t index = 0;
};
bool substitute_message(const std::string& msg, const char* json, size_t n, std::string* out, bool* nonstring,
                        bool* subst_err = nullptr, const MsgElem* el = nullptr);
// The error text of a condition block that raised one (`t`: its schema.h CT_ERR trace half), as
// variables/evaluate.go:14-27 and vars.go:311-389 word it: "failed to substitute variables in
// condition key: failed to resolve <var> at path <path>: JMESPath query failed: Unknown key \"<k>\"
// in path", the value's likewise, or the operator's. "" when the error is not one the host
// restates (an error go-jmespath words itself).
std::string block_error_text(const std::string& block_json, uint32_t t, const char* json, size_t n,
                             const MsgElem* el);
// SubstituteAll's error over a document (substitutePatterns, validate_resource.go:456-476): the
// first failing variable in traversal order (document order for maps, Go's is random), or "".
std::string doc_subst_error(const std::string& doc_json, const char* json, size_t n, const MsgElem* el);

}  // namespace kpe
