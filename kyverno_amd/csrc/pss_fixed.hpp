// The PSA library's fixed value sets (pod-security-admission v0.29 policy/check_*.go, restated in
// oracle/pss.hpp): shared by the compiler (program.cpp pss_preds: dictionary predicates the scan
// kernels read) and the device's per-pod summary (kpe_api.cpp psa_fixed_table -> lean.inl
// kpe_psa_dict_kernel). None of them depends on a policy: a podSecurity rule only picks the
// level / version (which checks run) and its exclusions.
#pragma once
#include <string>
#include <vector>

namespace kpe {
namespace pssfix {

inline const std::vector<std::string> kApparmorKey = {"container.apparmor.security.beta.kubernetes.io/*"};
inline const std::vector<std::string> kApparmorOk = {"runtime/default", "localhost/*"};
inline const std::vector<std::string> kSeccompPodKey = {"seccomp.security.alpha.kubernetes.io/pod"};
inline const std::vector<std::string> kSeccompAnnOk = {"runtime/default", "docker/default", "localhost/*"};
inline const std::vector<std::string> kCapsBaselineOk = {"AUDIT_WRITE", "CHOWN",  "DAC_OVERRIDE",     "FOWNER", "FSETID",
                                                         "KILL",        "MKNOD",  "NET_BIND_SERVICE", "SETFCAP",
                                                         "SETGID",      "SETPCAP", "SETUID",          "SYS_CHROOT"};
inline const std::vector<std::string> kCapNbs = {"NET_BIND_SERVICE"};
inline const std::vector<std::string> kCapAll = {"ALL"};
// allowed sysctls of check_sysctls.go v1.0, v1.27 and v1.29
inline std::vector<std::string> sysctls(int v) {
  std::vector<std::string> s = {"kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range",
                                "net.ipv4.ip_unprivileged_port_start", "net.ipv4.tcp_syncookies",
                                "net.ipv4.ping_group_range"};
  if (v >= 1) s.push_back("net.ipv4.ip_local_reserved_ports");
  if (v >= 2)
    for (auto n : {"net.ipv4.tcp_keepalive_time", "net.ipv4.tcp_fin_timeout", "net.ipv4.tcp_keepalive_intvl",
                   "net.ipv4.tcp_keepalive_probes"})
      s.push_back(n);
  return s;
}
// Every fixed glob above is a literal or a literal followed by one trailing '*' (go-wildcard:
// '*' matches any run of runes, so a trailing one is a byte-prefix match).
inline bool fixed_match(const std::vector<std::string>& globs, const std::string& s) {
  for (const auto& g : globs) {
    if (!g.empty() && g.back() == '*') {
      if (s.compare(0, g.size() - 1, g, 0, g.size() - 1) == 0 && s.size() >= g.size() - 1) return true;
    } else if (g == s) {
      return true;
    }
  }
  return false;
}

}  // namespace pssfix
}  // namespace kpe
