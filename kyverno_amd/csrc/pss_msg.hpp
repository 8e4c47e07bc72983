// PodSecurity RuleResponse messages (pss_msg.cpp).
#pragma once
#include <cstdint>
#include <string>

#include "podview.hpp"

namespace kpe {

// validate_pss.go:85 (allowed)
std::string pss_pass_message(const std::string& rule);
// validate_pss.go:108: the failing versioned checks `cv_fail` (bit v = CV_* v) of the pod
// decoded from a resource of `kind`, formatted by FormatChecksPrint after convertChecks.
std::string pss_fail_message(const std::string& rule, const std::string& level, const std::string& version,
                             const std::string& kind, const PodView& pod, uint32_t cv_fail);

}  // namespace kpe
