// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the Pod Security Standards path:
//   * kyverno adapter: pkg/pss/evaluate.go (evaluatePSS :24-70, exemptExclusions
//     :72-161, extractBadValues :163-182, remove :184-187, parseField :193-204,
//     getContainerInfo :206-219, ParseVersion :221-239, EvaluatePod :242-252,
//     ApplyPodSecurityExclusion :255-279, GetPodWithMatchingContainers :283-317),
//     control->check map pkg/pss/utils/mapping.go:45-107, exclude validation
//     api/kyverno/v1/common_types.go:472-478.
//   * third-party checks: k8s.io/pod-security-admission v0.29.1 replaced by
//     github.com/YTGhost/pod-security-admission v0.0.0-20231116105308-8b1daa0177f2
//     (go.mod:84,385). NOT present in /root/reference: restated from the published
//     PSA v0.29 policy/check_*.go algorithm plus the fork's WithFieldErrors field
//     paths, and pinned by pkg/pss/evaluate_test.go (227 cases), the chainsaw PSA
//     fixtures and test-report-background-mode (see tests/golden/).
#pragma once
#include <functional>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "k8s_typed.hpp"
#include "wildcard.hpp"

namespace oracle {

// --- field.Error -------------------------------------------------------------
enum class BVKind { None, Str, Bool, Int, StrList, Other };
struct FieldError {
  std::string type;   // "Required value" / "Forbidden"
  std::string field;  // field.Path.String()
  BVKind bk = BVKind::Str;  // field.Required/Forbidden default BadValue is ""
  std::string bs;
  bool bb = false;
  long long bi = 0;
  std::vector<std::string> bl;
};
inline FieldError required(const std::string& p) { return FieldError{"Required value", p}; }
inline FieldError forbidden(const std::string& p) { return FieldError{"Forbidden", p}; }
inline FieldError with_bool(FieldError e, bool v) {
  e.bk = BVKind::Bool;
  e.bb = v;
  return e;
}
inline FieldError with_str(FieldError e, const std::string& v) {
  e.bk = BVKind::Str;
  e.bs = v;
  return e;
}
inline FieldError with_int(FieldError e, long long v) {  // Go `int` bad value
  e.bk = BVKind::Int;
  e.bi = v;
  return e;
}
inline FieldError with_other(FieldError e, long long v) {  // int32 / int64 bad values
  e.bk = BVKind::Other;
  e.bi = v;
  return e;
}
inline FieldError with_list(FieldError e, std::vector<std::string> v) {
  e.bk = BVKind::StrList;
  e.bl = std::move(v);
  return e;
}

struct CheckResult {
  bool allowed = true;
  std::string reason;
  std::vector<FieldError> errs;
};

struct PSSCheckResult {
  std::string id;
  CheckResult result;
};

// --- api.Level / api.Version ---------------------------------------------------
enum class Level { Privileged, Baseline, Restricted };
struct Version {
  bool latest = false;
  int major = 0, minor = 0;
  bool older(const Version& o) const {  // PSA api.Version.Older
    if (latest) return false;
    if (o.latest) return true;
    if (major != o.major) return major < o.major;
    return minor < o.minor;
  }
};
inline Version V(int ma, int mi) { return Version{false, ma, mi}; }

// --- the 17 checks ---------------------------------------------------------------
using CheckFn = std::function<CheckResult(const ObjectMeta&, const PodSpec&)>;
struct VersionedCheck {
  Version min;
  CheckFn fn;
};
struct Check {
  std::string id;
  Level level;
  std::vector<VersionedCheck> versions;
};

// visitContainers: initContainers, containers, ephemeralContainers (PSA policy/visitor.go)
template <class F>
inline void visit_containers(const PodSpec& s, F fn) {
  for (size_t i = 0; i < s.initContainers.size(); ++i)
    fn(s.initContainers[i], "spec.initContainers[" + std::to_string(i) + "]");
  for (size_t i = 0; i < s.containers.size(); ++i) fn(s.containers[i], "spec.containers[" + std::to_string(i) + "]");
  for (size_t i = 0; i < s.ephemeralContainers.size(); ++i)
    fn(s.ephemeralContainers[i], "spec.ephemeralContainers[" + std::to_string(i) + "]");
}

inline CheckResult fail(const char* reason, std::vector<FieldError> errs) {
  CheckResult r;
  r.allowed = false;
  r.reason = reason;
  r.errs = std::move(errs);
  return r;
}
inline bool is_windows(const PodSpec& s) { return s.osName && *s.osName == "windows"; }

// check_allowPrivilegeEscalation.go
inline CheckResult ape_1_8(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    auto& sc = c.securityContext;
    // Unset is reported with a non-empty bad value that does not match "true"
    // (pinned by chainsaw psa/test-exclusion-privilege-escalation bad-pod.yaml).
    if (!sc || !sc->allowPrivilegeEscalation)
      e.push_back(with_bool(required(p + ".securityContext.allowPrivilegeEscalation"), false));
    else if (*sc->allowPrivilegeEscalation)
      e.push_back(with_bool(forbidden(p + ".securityContext.allowPrivilegeEscalation"), true));
  });
  if (!e.empty()) return fail("allowPrivilegeEscalation != false", e);
  return {};
}
inline CheckResult ape_1_25(const ObjectMeta& m, const PodSpec& s) {
  if (is_windows(s)) return {};
  return ape_1_8(m, s);
}

// check_appArmorProfile.go (v0.29: annotations only)
inline CheckResult apparmor_1_0(const ObjectMeta& m, const PodSpec&) {
  static const std::string pfx = "container.apparmor.security.beta.kubernetes.io/";
  std::vector<FieldError> e;
  for (auto& kv : m.annotations) {
    if (kv.first.compare(0, pfx.size(), pfx) == 0) {
      const std::string& v = kv.second;
      if (!(v == "runtime/default" || v.compare(0, 10, "localhost/") == 0))
        e.push_back(with_str(forbidden("metadata.annotations[" + kv.first + "]"), v));
    }
  }
  if (!e.empty()) return fail("forbidden AppArmor profile", e);
  return {};
}

inline const std::set<std::string>& caps_allowed_1_0() {
  static const std::set<std::string> s = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID",
                                          "KILL", "MKNOD", "NET_BIND_SERVICE", "SETFCAP", "SETGID",
                                          "SETPCAP", "SETUID", "SYS_CHROOT"};
  return s;
}
// check_capabilities_baseline.go
inline CheckResult caps_baseline_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (!c.securityContext || !c.securityContext->capabilities) return;
    std::vector<std::string> bad;
    for (auto& cap : c.securityContext->capabilities->add)
      if (!caps_allowed_1_0().count(cap)) bad.push_back(cap);
    if (!bad.empty()) e.push_back(with_list(forbidden(p + ".securityContext.capabilities.add"), bad));
  });
  if (!e.empty()) return fail("non-default capabilities", e);
  return {};
}
// check_capabilities_restricted.go
inline CheckResult caps_restricted_1_22(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (!c.securityContext || !c.securityContext->capabilities) {
      e.push_back(required(p + ".securityContext.capabilities.drop"));
      return;
    }
    auto& caps = *c.securityContext->capabilities;
    bool dropped = false;
    for (auto& d : caps.drop)
      if (d == "ALL") dropped = true;
    if (!dropped) e.push_back(required(p + ".securityContext.capabilities.drop"));
    std::vector<std::string> bad;
    for (auto& a : caps.add)
      if (a != "NET_BIND_SERVICE") bad.push_back(a);
    if (!bad.empty()) e.push_back(with_list(forbidden(p + ".securityContext.capabilities.add"), bad));
  });
  if (!e.empty()) return fail("unrestricted capabilities", e);
  return {};
}
inline CheckResult caps_restricted_1_25(const ObjectMeta& m, const PodSpec& s) {
  if (is_windows(s)) return {};
  return caps_restricted_1_22(m, s);
}
// check_hostNamespaces.go
inline CheckResult host_ns_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  if (s.hostNetwork) e.push_back(with_bool(forbidden("spec.hostNetwork"), true));
  if (s.hostPID) e.push_back(with_bool(forbidden("spec.hostPID"), true));
  if (s.hostIPC) e.push_back(with_bool(forbidden("spec.hostIPC"), true));
  if (!e.empty()) return fail("host namespaces", e);
  return {};
}
// check_hostPathVolumes.go
inline CheckResult host_path_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  for (size_t i = 0; i < s.volumes.size(); ++i)
    if (s.volumes[i].source("hostPath"))
      e.push_back(forbidden("spec.volumes[" + std::to_string(i) + "].hostPath"));
  if (!e.empty()) return fail("hostPath volumes", e);
  return {};
}
// check_hostPorts.go
inline CheckResult host_ports_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    for (size_t j = 0; j < c.ports.size(); ++j)
      if (c.ports[j].hostPort != 0)
        e.push_back(with_int(forbidden(p + ".ports[" + std::to_string(j) + "].hostPort"), c.ports[j].hostPort));
  });
  if (!e.empty()) return fail("hostPort", e);
  return {};
}
// check_privileged.go
inline CheckResult privileged_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->privileged && *c.securityContext->privileged)
      e.push_back(with_bool(forbidden(p + ".securityContext.privileged"), true));
  });
  if (!e.empty()) return fail("privileged", e);
  return {};
}
// check_procMount.go
inline CheckResult proc_mount_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->procMount && *c.securityContext->procMount != "Default")
      e.push_back(with_str(forbidden(p + ".securityContext.procMount"), *c.securityContext->procMount));
  });
  if (!e.empty()) return fail("procMount", e);
  return {};
}
// check_restrictedVolumes.go
inline CheckResult restricted_volumes_1_0(const ObjectMeta&, const PodSpec& s) {
  static const char* allowed[] = {"configMap", "csi", "downwardAPI", "emptyDir",
                                  "ephemeral", "persistentVolumeClaim", "projected", "secret"};
  static const char* bad_order[] = {"hostPath", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "nfs",
                                    "iscsi", "glusterfs", "rbd", "flexVolume", "cinder", "cephfs", "flocker",
                                    "fc", "azureFile", "vsphereVolume", "quobyte", "azureDisk",
                                    "photonPersistentDisk", "portworxVolume", "scaleIO", "storageos"};
  std::vector<FieldError> e;
  for (size_t i = 0; i < s.volumes.size(); ++i) {
    const Volume& v = s.volumes[i];
    bool ok = false;
    for (auto a : allowed)
      if (v.source(a)) ok = true;
    if (ok) continue;
    std::string t = "unknown";
    for (auto b : bad_order)
      if (v.source(b)) {
        t = b;
        break;
      }
    e.push_back(forbidden("spec.volumes[" + std::to_string(i) + "]." + t));
  }
  if (!e.empty()) return fail("restricted volume types", e);
  return {};
}
// check_runAsNonRoot.go
// Explicit bad setters (pod or container runAsNonRoot=false) are reported first
// and alone; implicitly-bad containers only when nothing was set explicitly.
inline CheckResult run_as_non_root_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> bad, implicit;
  bool pod_true = false;
  if (s.securityContext && s.securityContext->runAsNonRoot) {
    if (!*s.securityContext->runAsNonRoot)
      bad.push_back(with_bool(forbidden("spec.securityContext.runAsNonRoot"), false));
    else
      pod_true = true;
  }
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->runAsNonRoot) {
      if (!*c.securityContext->runAsNonRoot)
        bad.push_back(with_bool(forbidden(p + ".securityContext.runAsNonRoot"), false));
    } else if (!pod_true) {
      implicit.push_back(required(p + ".securityContext.runAsNonRoot"));
    }
  });
  if (!bad.empty()) return fail("runAsNonRoot != true", bad);
  if (!implicit.empty()) return fail("runAsNonRoot != true", implicit);
  return {};
}
// check_runAsUser.go
inline CheckResult run_as_user_1_23(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  if (s.securityContext && s.securityContext->runAsUser && *s.securityContext->runAsUser == 0)
    e.push_back(with_int(forbidden("spec.securityContext.runAsUser"), 0));
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->runAsUser && *c.securityContext->runAsUser == 0)
      e.push_back(with_int(forbidden(p + ".securityContext.runAsUser"), 0));
  });
  if (!e.empty()) return fail("runAsUser=0", e);
  return {};
}
// check_seLinuxOptions.go
inline CheckResult selinux_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  auto chk = [&](const SELinuxOptions& o, const std::string& p) {
    if (!(o.type.empty() || o.type == "container_t" || o.type == "container_init_t" || o.type == "container_kvm_t"))
      e.push_back(with_str(forbidden(p + ".type"), o.type));
    if (!o.user.empty()) e.push_back(with_str(forbidden(p + ".user"), o.user));
    if (!o.role.empty()) e.push_back(with_str(forbidden(p + ".role"), o.role));
  };
  if (s.securityContext && s.securityContext->seLinuxOptions)
    chk(*s.securityContext->seLinuxOptions, "spec.securityContext.seLinuxOptions");
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->seLinuxOptions)
      chk(*c.securityContext->seLinuxOptions, p + ".securityContext.seLinuxOptions");
  });
  if (!e.empty()) return fail("seLinuxOptions", e);
  return {};
}
// check_seccompProfile_baseline.go
inline bool valid_seccomp(const std::string& t) { return t == "RuntimeDefault" || t == "Localhost"; }
inline bool valid_seccomp_annotation(const std::string& v) {
  return v == "runtime/default" || v == "docker/default" || v.compare(0, 10, "localhost/") == 0;
}
inline CheckResult seccomp_baseline_1_0(const ObjectMeta& m, const PodSpec& s) {
  static const std::string podkey = "seccomp.security.alpha.kubernetes.io/pod";
  static const std::string cpfx = "container.seccomp.security.alpha.kubernetes.io/";
  std::vector<FieldError> e;
  if (auto v = m.annotation(podkey))
    if (!valid_seccomp_annotation(*v)) e.push_back(with_str(forbidden("metadata.annotations[" + podkey + "]"), *v));
  visit_containers(s, [&](const Container& c, const std::string&) {
    std::string k = cpfx + c.name;
    if (auto v = m.annotation(k))
      if (!valid_seccomp_annotation(*v)) e.push_back(with_str(forbidden("metadata.annotations[" + k + "]"), *v));
  });
  if (!e.empty()) return fail("seccompProfile", e);
  return {};
}
inline CheckResult seccomp_baseline_1_19(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  if (s.securityContext && s.securityContext->seccompProfile && !valid_seccomp(s.securityContext->seccompProfile->type))
    e.push_back(with_str(forbidden("spec.securityContext.seccompProfile.type"), s.securityContext->seccompProfile->type));
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->seccompProfile && !valid_seccomp(c.securityContext->seccompProfile->type))
      e.push_back(with_str(forbidden(p + ".securityContext.seccompProfile.type"), c.securityContext->seccompProfile->type));
  });
  if (!e.empty()) return fail("seccompProfile", e);
  return {};
}
// check_seccompProfile_restricted.go
// Same precedence as runAsNonRoot: explicit bad values first, implicit containers otherwise.
inline CheckResult seccomp_restricted_1_19(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> bad, implicit;
  bool pod_set = false;
  if (s.securityContext && s.securityContext->seccompProfile) {
    const std::string& t = s.securityContext->seccompProfile->type;
    if (!valid_seccomp(t))
      bad.push_back(with_str(forbidden("spec.securityContext.seccompProfile.type"), t));
    else
      pod_set = true;
  }
  visit_containers(s, [&](const Container& c, const std::string& p) {
    if (c.securityContext && c.securityContext->seccompProfile) {
      const std::string& t = c.securityContext->seccompProfile->type;
      if (!valid_seccomp(t)) bad.push_back(with_str(forbidden(p + ".securityContext.seccompProfile.type"), t));
    } else if (!pod_set) {
      implicit.push_back(required(p + ".securityContext.seccompProfile.type"));
    }
  });
  if (!bad.empty()) return fail("seccompProfile", bad);
  if (!implicit.empty()) return fail("seccompProfile", implicit);
  return {};
}
inline CheckResult seccomp_restricted_1_25(const ObjectMeta& m, const PodSpec& s) {
  if (is_windows(s)) return {};
  return seccomp_restricted_1_19(m, s);
}
// check_sysctls.go
inline CheckResult sysctls_with(const PodSpec& s, const std::set<std::string>& allowed) {
  std::vector<FieldError> e;
  if (s.securityContext)
    for (size_t i = 0; i < s.securityContext->sysctls.size(); ++i) {
      const std::string& n = s.securityContext->sysctls[i].name;
      if (!allowed.count(n))
        e.push_back(with_str(forbidden("spec.securityContext.sysctls[" + std::to_string(i) + "].name"), n));
    }
  if (!e.empty()) return fail("forbidden sysctls", e);
  return {};
}
inline const std::set<std::string>& sysctls_1_0() {
  static const std::set<std::string> s = {"kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range",
                                          "net.ipv4.ip_unprivileged_port_start", "net.ipv4.tcp_syncookies",
                                          "net.ipv4.ping_group_range"};
  return s;
}
inline const std::set<std::string>& sysctls_1_27() {
  static std::set<std::string> s = [] {
    auto x = sysctls_1_0();
    x.insert("net.ipv4.ip_local_reserved_ports");
    return x;
  }();
  return s;
}
inline const std::set<std::string>& sysctls_1_29() {
  static std::set<std::string> s = [] {
    auto x = sysctls_1_27();
    for (auto n : {"net.ipv4.tcp_keepalive_time", "net.ipv4.tcp_fin_timeout", "net.ipv4.tcp_keepalive_intvl",
                   "net.ipv4.tcp_keepalive_probes"})
      x.insert(n);
    return x;
  }();
  return s;
}
// check_windowsHostProcess.go
inline CheckResult win_host_process_1_0(const ObjectMeta&, const PodSpec& s) {
  std::vector<FieldError> e;
  visit_containers(s, [&](const Container& c, const std::string& p) {
    auto& sc = c.securityContext;
    if (sc && sc->windowsOptions && sc->windowsOptions->hostProcess && *sc->windowsOptions->hostProcess)
      e.push_back(with_bool(forbidden(p + ".securityContext.windowsOptions.hostProcess"), true));
  });
  auto& psc = s.securityContext;
  if (psc && psc->windowsOptions && psc->windowsOptions->hostProcess && *psc->windowsOptions->hostProcess)
    e.push_back(with_bool(forbidden("spec.securityContext.windowsOptions.hostProcess"), true));
  if (!e.empty()) return fail("hostProcess", e);
  return {};
}

// policy.DefaultChecks() in PSA registration (file-name) order.
inline const std::vector<Check>& default_checks() {
  static const std::vector<Check> checks = {
      {"allowPrivilegeEscalation", Level::Restricted, {{V(1, 8), ape_1_8}, {V(1, 25), ape_1_25}}},
      {"appArmorProfile", Level::Baseline, {{V(1, 0), apparmor_1_0}}},
      {"capabilities_baseline", Level::Baseline, {{V(1, 0), caps_baseline_1_0}}},
      {"capabilities_restricted", Level::Restricted,
       {{V(1, 22), caps_restricted_1_22}, {V(1, 25), caps_restricted_1_25}}},
      {"hostNamespaces", Level::Baseline, {{V(1, 0), host_ns_1_0}}},
      {"hostPathVolumes", Level::Baseline, {{V(1, 0), host_path_1_0}}},
      {"hostPorts", Level::Baseline, {{V(1, 0), host_ports_1_0}}},
      {"privileged", Level::Baseline, {{V(1, 0), privileged_1_0}}},
      {"procMount", Level::Baseline, {{V(1, 0), proc_mount_1_0}}},
      {"restrictedVolumes", Level::Restricted, {{V(1, 0), restricted_volumes_1_0}}},
      {"runAsNonRoot", Level::Restricted, {{V(1, 0), run_as_non_root_1_0}}},
      {"runAsUser", Level::Restricted, {{V(1, 23), run_as_user_1_23}}},
      {"seLinuxOptions", Level::Baseline, {{V(1, 0), selinux_1_0}}},
      {"seccompProfile_baseline", Level::Baseline,
       {{V(1, 0), seccomp_baseline_1_0}, {V(1, 19), seccomp_baseline_1_19}}},
      {"seccompProfile_restricted", Level::Restricted,
       {{V(1, 19), seccomp_restricted_1_19}, {V(1, 25), seccomp_restricted_1_25}}},
      {"sysctls", Level::Baseline,
       {{V(1, 0), [](const ObjectMeta&, const PodSpec& s) { return sysctls_with(s, sysctls_1_0()); }},
        {V(1, 27), [](const ObjectMeta&, const PodSpec& s) { return sysctls_with(s, sysctls_1_27()); }},
        {V(1, 29), [](const ObjectMeta&, const PodSpec& s) { return sysctls_with(s, sysctls_1_29()); }}}},
      {"windowsHostProcess", Level::Baseline, {{V(1, 0), win_host_process_1_0}}},
  };
  return checks;
}

// pkg/pss/utils/mapping.go:45-107
inline const std::map<std::string, std::vector<std::string>>& controls_to_check_id() {
  static const std::map<std::string, std::vector<std::string>> m = {
      {"Capabilities", {"capabilities_baseline", "capabilities_restricted"}},
      {"Seccomp", {"seccompProfile_baseline", "seccompProfile_restricted"}},
      {"Privileged Containers", {"privileged"}},
      {"Host Ports", {"hostPorts"}},
      {"/proc Mount Type", {"procMount"}},
      {"HostProcess", {"windowsHostProcess"}},
      {"SELinux", {"seLinuxOptions"}},
      {"Host Namespaces", {"hostNamespaces"}},
      {"HostPath Volumes", {"hostPathVolumes"}},
      {"Sysctls", {"sysctls"}},
      {"AppArmor", {"appArmorProfile"}},
      {"Privilege Escalation", {"allowPrivilegeEscalation"}},
      {"Running as Non-root", {"runAsNonRoot"}},
      {"Running as Non-root user", {"runAsUser"}},
      {"Volume Types", {"restrictedVolumes"}},
  };
  return m;
}

struct LevelVersion {
  Level level;
  Version version;
};

// evaluate.go:24-70
inline std::vector<PSSCheckResult> evaluate_pss(const LevelVersion& lv, const Pod& pod) {
  std::vector<PSSCheckResult> results;
  for (auto& check : default_checks()) {
    if (lv.level == Level::Baseline && check.level != lv.level) continue;
    const VersionedCheck* latest = &check.versions[0];
    for (size_t i = 1; i < check.versions.size(); ++i)
      if (!check.versions[i].min.older(latest->min)) latest = &check.versions[i];
    if (lv.version.latest) {
      CheckResult r = latest->fn(pod.meta, pod.spec);
      if (!r.allowed) results.push_back({check.id, r});
    }
    for (auto& vc : check.versions) {
      if (lv.version.latest) continue;
      if (lv.version.older(vc.min)) continue;
      CheckResult r = vc.fn(pod.meta, pod.spec);
      if (!r.allowed) results.push_back({check.id, r});
    }
  }
  return results;
}

struct PSSExclude {
  std::string controlName;
  std::vector<std::string> images;
  std::string restrictedField;
  std::vector<std::string> values;
};

// evaluate.go:163-182
inline std::vector<std::string> extract_bad_values(const FieldError& e) {
  switch (e.bk) {
    case BVKind::Str:
      if (e.bs.empty()) return {};
      return {e.bs};
    case BVKind::Bool: return {e.bb ? "true" : "false"};
    case BVKind::Int: return {std::to_string(e.bi)};
    case BVKind::StrList: return e.bl;
    default: return {};
  }
}

// regexIndex = `\d+` replaced by "*"
inline std::string replace_digits(const std::string& f) {
  std::string o;
  for (size_t i = 0; i < f.size();) {
    if (isdigit((unsigned char)f[i])) {
      while (i < f.size() && isdigit((unsigned char)f[i])) ++i;
      o += '*';
    } else {
      o += f[i++];
    }
  }
  return o;
}
// evaluate.go:193-204 parseField
struct ParsedField {
  std::string field;
  std::vector<long> idx;
  std::string ctype;
  bool container_level;
};
inline ParsedField parse_field(const std::string& f) {
  ParsedField p;
  p.field = replace_digits(f);
  std::vector<std::string> words;
  for (size_t i = 0; i < f.size();) {
    if (isdigit((unsigned char)f[i])) {
      size_t st = i;
      while (i < f.size() && isdigit((unsigned char)f[i])) ++i;
      p.idx.push_back(atol(f.substr(st, i - st).c_str()));
    } else if (isalpha((unsigned char)f[i])) {
      size_t st = i;
      while (i < f.size() && isalpha((unsigned char)f[i])) ++i;
      words.push_back(f.substr(st, i - st));
    } else {
      ++i;
    }
  }
  p.ctype = words.size() > 1 ? words[1] : "";
  p.container_level = p.ctype == "containers" || p.ctype == "initContainers" || p.ctype == "ephemeralContainers";
  return p;
}
// evaluate.go:206-219
inline const Container* container_info(const Pod& pod, long idx, const std::string& ctype) {
  const std::vector<Container>* v = nullptr;
  if (ctype == "containers") v = &pod.spec.containers;
  else if (ctype == "initContainers") v = &pod.spec.initContainers;
  else if (ctype == "ephemeralContainers") v = &pod.spec.ephemeralContainers;
  if (!v) return nullptr;
  if (idx < 0 || (size_t)idx >= v->size()) throw std::out_of_range("container index");  // Go would panic
  return &(*v)[idx];
}

struct ExemptError {};

// evaluate.go:72-161. The reference keeps a Go map keyed by check ID: duplicates
// of one ID collapse to the last result (map assignment), and the returned
// slice is in map order — order only affects messages, never the verdict.
inline std::vector<PSSCheckResult> exempt_exclusions(const std::vector<PSSCheckResult>& defaults,
                                                     const std::vector<PSSCheckResult>& excl_results,
                                                     const PSSExclude& ex, const Pod& pod, const Pod* matching,
                                                     bool container_level, bool* err) {
  *err = false;
  if ((!ex.restrictedField.empty() && ex.values.empty()) || (ex.restrictedField.empty() && !ex.values.empty())) {
    *err = true;
    return {};
  }
  std::map<std::string, PSSCheckResult> m;
  std::vector<std::string> order;
  for (auto& r : defaults) {
    if (!m.count(r.id)) order.push_back(r.id);
    m[r.id] = r;
  }
  auto it_ids = controls_to_check_id().find(ex.controlName);
  for (auto& xr : excl_results) {
    if (it_ids == controls_to_check_id().end()) continue;
    for (auto& check_id : it_ids->second) {
      if (xr.id != check_id) continue;
      for (auto& xe : xr.result.errs) {
        std::string xfield;
        const Container* xc = nullptr;
        bool xcl = false;
        if (container_level) {
          ParsedField pf = parse_field(xe.field);
          xfield = pf.field;
          xcl = pf.container_level;
          if (xcl) xc = container_info(*matching, pf.idx[0], pf.ctype);
        } else {
          xfield = replace_digits(xe.field);
        }
        auto bad = extract_bad_values(xe);
        if (!(xfield == ex.restrictedField || ex.restrictedField.empty())) continue;
        bool flag = true;
        if (!ex.values.empty())
          for (auto& b : bad)
            if (!check_patterns(ex.values, b)) {
              flag = false;
              break;
            }
        if (!flag) continue;
        auto dit = m.find(check_id);
        if (dit == m.end()) continue;  // zero-value result: nil ErrList
        auto& errs = dit->second.result.errs;
        for (size_t idx = 0; idx < errs.size(); ++idx) {
          std::string dfield;
          bool dcl = false;
          const Container* dc = nullptr;
          if (container_level) {
            ParsedField pf = parse_field(errs[idx].field);
            dfield = pf.field;
            dcl = pf.container_level;
            if (dcl) dc = container_info(pod, pf.idx[0], pf.ctype);
          } else {
            dfield = replace_digits(errs[idx].field);
          }
          bool hit = dcl ? (xfield == dfield && xc && dc && xc->name == dc->name) : (xfield == dfield);
          if (hit) {  // evaluate.go:184-187 remove(): swap with last, truncate
            errs[idx] = errs.back();
            errs.pop_back();
            break;
          }
        }
        if (errs.empty()) m.erase(dit);
      }
    }
  }
  std::vector<PSSCheckResult> out;
  for (auto& id : order)
    if (m.count(id)) out.push_back(m[id]);
  return out;
}

// evaluate.go:283-317
inline void pod_with_matching_containers(const PSSExclude& ex, const Pod& pod, Pod* spec_out, Pod* matching_out,
                                         bool* is_spec) {
  if (ex.images.empty()) {
    *spec_out = pod;
    spec_out->spec.containers = {Container{"fake", "", {}, std::nullopt}};
    spec_out->spec.initContainers.clear();
    spec_out->spec.ephemeralContainers.clear();
    *is_spec = true;
    return;
  }
  *is_spec = false;
  Pod m;
  m.meta.name = pod.meta.name;
  m.meta.ns = pod.meta.ns;
  for (auto& c : pod.spec.containers)
    if (check_patterns(ex.images, c.image)) m.spec.containers.push_back(c);
  for (auto& c : pod.spec.initContainers)
    if (check_patterns(ex.images, c.image)) m.spec.initContainers.push_back(c);
  for (auto& c : pod.spec.ephemeralContainers)
    if (check_patterns(ex.images, c.image)) m.spec.ephemeralContainers.push_back(c);
  *matching_out = m;
}

// evaluate.go:255-279
inline std::vector<PSSCheckResult> apply_exclusion(const LevelVersion& lv, const std::vector<PSSExclude>& excludes,
                                                   std::vector<PSSCheckResult> defaults, const Pod& pod,
                                                   bool* err) {
  *err = false;
  for (auto& ex : excludes) {
    Pod spec, matching;
    bool is_spec;
    pod_with_matching_containers(ex, pod, &spec, &matching, &is_spec);
    bool e = false;
    if (is_spec) {
      auto xr = evaluate_pss(lv, spec);
      defaults = exempt_exclusions(defaults, xr, ex, pod, nullptr, false, &e);
    } else {
      auto xr = evaluate_pss(lv, matching);
      defaults = exempt_exclusions(defaults, xr, ex, pod, &matching, true, &e);
    }
    *err = e;  // only the last exclude's error survives (reference quirk)
  }
  return defaults;
}

// evaluate.go:242-252
inline bool evaluate_pod(const LevelVersion& lv, const std::vector<PSSExclude>& excludes, const Pod& pod,
                         std::vector<PSSCheckResult>* out = nullptr) {
  auto res = evaluate_pss(lv, pod);
  bool err = false;
  if (!excludes.empty()) res = apply_exclusion(lv, excludes, res, pod, &err);
  if (out) *out = res;
  return res.empty() && !err;
}

// evaluate.go:331-362 FormatChecksPrint. A Forbidden error with a bad value (anything but the
// empty string) prints "<field> is forbidden, don't set the BadValue: %+v"; every other error
// prints field.Error.Error() = "<field>: <type>" (apimachinery v0.29.1 field/errors.go:
// Required and Forbidden bodies are the type string alone).
inline std::string format_checks_print(const std::vector<PSSCheckResult>& checks) {
  std::string s;
  for (auto& c : checks) {
    s += "\n(Forbidden reason: " + c.result.reason + ", field error list: [";
    for (size_t i = 0; i < c.result.errs.size(); ++i) {
      const FieldError& e = c.result.errs[i];
      const bool exist = !(e.bk == BVKind::Str && e.bs.empty());
      if (e.type == "Forbidden" && exist) {
        std::string v;  // %+v
        switch (e.bk) {
          case BVKind::Str: v = e.bs; break;
          case BVKind::Bool: v = e.bb ? "true" : "false"; break;
          case BVKind::Int:
          case BVKind::Other: v = std::to_string(e.bi); break;
          case BVKind::StrList:
            v = "[";
            for (size_t k = 0; k < e.bl.size(); ++k) v += (k ? " " : "") + e.bl[k];
            v += "]";
            break;
          default: break;
        }
        s += e.field + " is forbidden, don't set the BadValue: " + v;
      } else {
        s += e.field + ": " + e.type;
      }
      if (i + 1 != c.result.errs.size()) s += ", ";
    }
    s += "])";
  }
  return s;
}

inline std::string go_replace_all(const std::string& s, const std::string& a, const std::string& b) {
  std::string o;
  size_t i = 0, j;
  while ((j = s.find(a, i)) != std::string::npos) {
    o += s.substr(i, j - i) + b;
    i = j + a.size();
  }
  return o + s.substr(i);
}
// validate_pss.go:114-135 convertChecks: field paths of controllers / CronJobs, then every
// "metadata" -> "spec.template.metadata" (for every kind, Pods included)
inline void convert_checks(std::vector<PSSCheckResult>& checks, const std::string& kind) {
  const bool ctl = kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
                   kind == "ReplicaSet" || kind == "ReplicationController";
  for (auto& c : checks)
    for (auto& e : c.result.errs) {
      if (ctl) e.field = go_replace_all(e.field, "spec", "spec.template.spec");
      else if (kind == "CronJob") e.field = go_replace_all(e.field, "spec", "spec.jobTemplate.spec.template.spec");
      e.field = go_replace_all(e.field, "metadata", "spec.template.metadata");
    }
}

// evaluate.go:221-239 + PSA api.ParseVersion (`latest` or `v1.<minor>`)
inline bool parse_version(const std::string& v, Version* out) {
  if (v.empty() || v == "latest") {
    *out = Version{true, 0, 0};
    return true;
  }
  if (v.size() < 4 || v.compare(0, 3, "v1.") != 0) return false;
  std::string mi = v.substr(3);
  if (mi.empty() || mi.size() > 9) return false;
  for (char c : mi)
    if (!isdigit((unsigned char)c)) return false;
  if (mi.size() > 1 && mi[0] == '0') return false;
  *out = V(1, atoi(mi.c_str()));
  return true;
}

}  // namespace oracle
