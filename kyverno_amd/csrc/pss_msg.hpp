// PodSecurity RuleResponse messages (pss_msg.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "podview.hpp"

namespace kpe {

// validate_pss.go:85 (allowed)
std::string pss_pass_message(const std::string& rule);
// validate_pss.go:108: the failing versioned checks `cv_fail` (bit v = CV_* v) of the pod
// decoded from a resource of `kind`, formatted by FormatChecksPrint after convertChecks.
std::string pss_fail_message(const std::string& rule, const std::string& level, const std::string& version,
                             const std::string& kind, const PodView& pod, uint32_t cv_fail);

// One podSecurity exclude entry (kyvernov1.PodSecurityStandard): controlName, images,
// restrictedField, values
struct PssExcl {
  std::string control;
  std::vector<std::string> images;
  std::string field;
  std::vector<std::string> values;
};
// validate_pss.go:76-110 for a rule with podSecurity.exclude and / or a podSecurity
// PolicyException: the fail message over the checks left by EvaluatePod's exclusions
// (pkg/pss/evaluate.go:242-317) and, when the exception applied (`exc` non-null), by its
// ApplyPodSecurityExclusion after convertChecks. `cv_mask`: the rule's versioned checks. The
// reference's result order after an exclusion pass is Go map order; this keeps evaluation order
// (first occurrence of each check id, its last failing version), as the oracle does.
std::string pss_fail_message_ex(const std::string& rule, const std::string& level, const std::string& version,
                                const std::string& kind, const PodView& pod, uint32_t cv_mask,
                                const std::vector<PssExcl>* rule_ex, const std::vector<PssExcl>* exc);

// go-wildcard v1.0.3 Match (program.cpp): ext/wildcard CheckPatterns' per-pattern test
bool go_wildcard(const std::string& pattern, const std::string& s);

}  // namespace kpe
