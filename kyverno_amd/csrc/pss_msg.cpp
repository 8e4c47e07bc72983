// PodSecurity rule messages (host): the RuleResponse message text of a podSecurity cell whose
// verdict the GPU decided, rendered for one resource (kpe_report_results_msg).
//
//   pass: validate_pss.go:85  "Validation rule '<rule>' passed."
//   fail: validate_pss.go:108 "Validation rule '<rule>' failed. It violates PodSecurity
//         \"<level>:<version>\": " + pss.FormatChecksPrint(convertChecks(checks, kind))
//
// The failing versioned checks come from the scan kernel (kpe_fetch_cv_masks); this file only
// restates each failing check's field error list (the YTGhost/pod-security-admission fork's
// WithFieldErrors paths, go.mod:84,385) over the typed pod view, in evaluatePSS order
// (pkg/pss/evaluate.go:24-70: check registration order, then version order, one entry per
// failing versioned check), FormatChecksPrint (evaluate.go:331-362), convertChecks'
// strings.ReplaceAll field rewrites (validate_pss.go:114-135) and field.Error.Error()
// (apimachinery v0.29.1 field/errors.go: "<field>: <type>" for Required / Forbidden).
#include <cstdint>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#include "podview.hpp"
#include "pss_msg.hpp"
#include "schema.h"

namespace kpe {
namespace {

enum BV { BV_NONE, BV_STR, BV_BOOL, BV_INT, BV_LIST };
struct FieldErr {
  bool forbidden;
  std::string field;
  BV kind = BV_NONE;  // field.Required / field.Forbidden default BadValue is ""
  std::string val;    // %+v of the bad value
  std::vector<std::string> list;  // BV_LIST: the values
};
struct Failed {
  const char* reason;
  std::vector<FieldErr> errs;
};

FieldErr required(std::string f) { return FieldErr{false, std::move(f), BV_NONE, {}}; }
FieldErr forbidden(std::string f) { return FieldErr{true, std::move(f), BV_NONE, {}}; }
FieldErr forbidden(std::string f, bool b) { return FieldErr{true, std::move(f), BV_BOOL, b ? "true" : "false"}; }
FieldErr forbidden_str(std::string f, const std::string& v) {
  return FieldErr{true, std::move(f), v.empty() ? BV_NONE : BV_STR, v};
}
FieldErr forbidden_int(std::string f, long long v) { return FieldErr{true, std::move(f), BV_INT, std::to_string(v)}; }
FieldErr forbidden_list(std::string f, const std::vector<std::string>& v) {
  std::string s = "[";  // %+v of a []string
  for (size_t i = 0; i < v.size(); ++i) s += (i ? " " : "") + v[i];
  return FieldErr{true, std::move(f), BV_LIST, s + "]", v};
}

template <class F>
void visit(const PodView& p, F fn) {  // PSA visitContainers: init, regular, ephemeral
  static const char* const kList[3] = {"spec.initContainers[", "spec.containers[", "spec.ephemeralContainers["};
  for (int l = 0; l < 3; ++l)
    for (size_t i = 0; i < p.ctr[l].size(); ++i) fn(p.ctr[l][i], std::string(kList[l]) + std::to_string(i) + "]");
}
bool windows(const PodView& p) { return p.os && p.os_name == "windows"; }

// corev1.VolumeSource members in declaration order (VS_* bit order)
const char* const kVolNames[KPE_NUM_VOLUME_SOURCES] = {
    "hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "secret", "nfs", "iscsi",
    "glusterfs", "persistentVolumeClaim", "rbd", "flexVolume", "cinder", "cephfs", "flocker", "downwardAPI", "fc",
    "azureFile", "configMap", "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk", "projected",
    "portworxVolume", "scaleIO", "storageos", "csi", "ephemeral"};
constexpr uint32_t kAllowedVols = (1u << VS_CONFIGMAP) | (1u << VS_CSI) | (1u << VS_DOWNWARDAPI) |
                                  (1u << VS_EMPTYDIR) | (1u << VS_EPHEMERAL) | (1u << VS_PVC) |
                                  (1u << VS_PROJECTED) | (1u << VS_SECRET);

bool valid_seccomp_type(const std::string& t) { return t == "RuntimeDefault" || t == "Localhost"; }
bool valid_seccomp_ann(const std::string& v) {
  return v == "runtime/default" || v == "docker/default" || v.compare(0, 10, "localhost/") == 0;
}
const std::string* annotation(const PodView& p, const std::string& k) {
  for (auto& kv : p.ann)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

const std::set<std::string>& sysctl_allow(int v) {  // PSA check_sysctls.go at 1.0 / 1.27 / 1.29
  static const std::set<std::string> s0 = {"kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range",
                                           "net.ipv4.ip_unprivileged_port_start", "net.ipv4.tcp_syncookies",
                                           "net.ipv4.ping_group_range"};
  static const std::set<std::string> s1 = [] {
    auto x = s0;
    x.insert("net.ipv4.ip_local_reserved_ports");
    return x;
  }();
  static const std::set<std::string> s2 = [] {
    auto x = s1;
    for (auto n : {"net.ipv4.tcp_keepalive_time", "net.ipv4.tcp_fin_timeout", "net.ipv4.tcp_keepalive_intvl",
                   "net.ipv4.tcp_keepalive_probes"})
      x.insert(n);
    return x;
  }();
  return v == 0 ? s0 : v == 1 ? s1 : s2;
}

// The field errors of one failing versioned check (CV_* index).
Failed check_errors(uint32_t cv, const PodView& p) {
  std::vector<FieldErr> e;
  switch (cv) {
    case CV_APE_1_8:
    case CV_APE_1_25:
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (!c.sc || c.ape == TRI_UNSET) {
          FieldErr x = required(f + ".securityContext.allowPrivilegeEscalation");
          x.kind = BV_BOOL, x.val = "false";
          e.push_back(x);
        } else if (c.ape == TRI_TRUE) {
          e.push_back(forbidden(f + ".securityContext.allowPrivilegeEscalation", true));
        }
      });
      return {"allowPrivilegeEscalation != false", e};
    case CV_APPARMOR_1_0: {
      static const std::string pfx = "container.apparmor.security.beta.kubernetes.io/";
      for (auto& kv : p.ann)
        if (kv.first.compare(0, pfx.size(), pfx) == 0 &&
            !(kv.second == "runtime/default" || kv.second.compare(0, 10, "localhost/") == 0))
          e.push_back(forbidden_str("metadata.annotations[" + kv.first + "]", kv.second));
      return {"forbidden AppArmor profile", e};
    }
    case CV_CAPS_BASELINE_1_0: {
      static const std::set<std::string> ok = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID",
                                               "KILL", "MKNOD", "NET_BIND_SERVICE", "SETFCAP", "SETGID",
                                               "SETPCAP", "SETUID", "SYS_CHROOT"};
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (!c.sc || !c.caps) return;
        std::vector<std::string> bad;
        for (auto& a : c.add)
          if (!ok.count(a)) bad.push_back(a);
        if (!bad.empty()) e.push_back(forbidden_list(f + ".securityContext.capabilities.add", bad));
      });
      return {"non-default capabilities", e};
    }
    case CV_CAPS_RESTRICTED_1_22:
    case CV_CAPS_RESTRICTED_1_25:
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (!c.sc || !c.caps) {
          e.push_back(required(f + ".securityContext.capabilities.drop"));
          return;
        }
        bool all = false;
        for (auto& d : c.drop) all |= d == "ALL";
        if (!all) e.push_back(required(f + ".securityContext.capabilities.drop"));
        std::vector<std::string> bad;
        for (auto& a : c.add)
          if (a != "NET_BIND_SERVICE") bad.push_back(a);
        if (!bad.empty()) e.push_back(forbidden_list(f + ".securityContext.capabilities.add", bad));
      });
      return {"unrestricted capabilities", e};
    case CV_HOST_NS_1_0:
      if (p.hostnet) e.push_back(forbidden("spec.hostNetwork", true));
      if (p.hostpid) e.push_back(forbidden("spec.hostPID", true));
      if (p.hostipc) e.push_back(forbidden("spec.hostIPC", true));
      return {"host namespaces", e};
    case CV_HOST_PATH_1_0:
      for (size_t i = 0; i < p.vols.size(); ++i)
        if (p.vols[i] & (1u << VS_HOSTPATH)) e.push_back(forbidden("spec.volumes[" + std::to_string(i) + "].hostPath"));
      return {"hostPath volumes", e};
    case CV_HOST_PORTS_1_0:
      visit(p, [&](const CtrView& c, const std::string& f) {
        for (size_t j = 0; j < c.hostports.size(); ++j)
          if (c.hostports[j] != 0)
            e.push_back(forbidden_int(f + ".ports[" + std::to_string(j) + "].hostPort", c.hostports[j]));
      });
      return {"hostPort", e};
    case CV_PRIVILEGED_1_0:
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.priv == TRI_TRUE) e.push_back(forbidden(f + ".securityContext.privileged", true));
      });
      return {"privileged", e};
    case CV_PROC_MOUNT_1_0:
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.pm && c.pm_val != "Default") e.push_back(forbidden_str(f + ".securityContext.procMount", c.pm_val));
      });
      return {"procMount", e};
    case CV_RESTRICTED_VOLUMES_1_0:
      for (size_t i = 0; i < p.vols.size(); ++i) {
        const uint32_t m = p.vols[i];
        if (m & kAllowedVols) continue;
        std::string t = "unknown";
        for (int b = 0; b < KPE_NUM_VOLUME_SOURCES; ++b)
          if (m & (1u << b)) {
            t = kVolNames[b];
            break;
          }
        e.push_back(forbidden("spec.volumes[" + std::to_string(i) + "]." + t));
      }
      return {"restricted volume types", e};
    case CV_RUN_AS_NON_ROOT_1_0: {
      std::vector<FieldErr> bad, implicit;
      if (p.rnr == TRI_FALSE) bad.push_back(forbidden("spec.securityContext.runAsNonRoot", false));
      const bool pod_true = p.rnr == TRI_TRUE;
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.rnr == TRI_FALSE) bad.push_back(forbidden(f + ".securityContext.runAsNonRoot", false));
        else if (c.rnr == TRI_UNSET && !pod_true) implicit.push_back(required(f + ".securityContext.runAsNonRoot"));
      });
      return {"runAsNonRoot != true", bad.empty() ? implicit : bad};
    }
    case CV_RUN_AS_USER_1_23:
      if (p.rau == RAU_ZERO) e.push_back(forbidden_int("spec.securityContext.runAsUser", 0));
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.rau == RAU_ZERO) e.push_back(forbidden_int(f + ".securityContext.runAsUser", 0));
      });
      return {"runAsUser=0", e};
    case CV_SELINUX_1_0: {
      auto chk = [&](const std::string& type, const std::string& user, const std::string& role, const std::string& f) {
        if (!(type.empty() || type == "container_t" || type == "container_init_t" || type == "container_kvm_t"))
          e.push_back(forbidden_str(f + ".type", type));
        if (!user.empty()) e.push_back(forbidden_str(f + ".user", user));
        if (!role.empty()) e.push_back(forbidden_str(f + ".role", role));
      };
      if (p.sel) chk(p.sel_type, p.sel_user, p.sel_role, "spec.securityContext.seLinuxOptions");
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.sel) chk(c.sel_type, c.sel_user, c.sel_role, f + ".securityContext.seLinuxOptions");
      });
      return {"seLinuxOptions", e};
    }
    case CV_SECCOMP_BASELINE_1_0: {
      static const std::string podkey = "seccomp.security.alpha.kubernetes.io/pod";
      static const std::string cpfx = "container.seccomp.security.alpha.kubernetes.io/";
      if (const std::string* v = annotation(p, podkey))
        if (!valid_seccomp_ann(*v)) e.push_back(forbidden_str("metadata.annotations[" + podkey + "]", *v));
      visit(p, [&](const CtrView& c, const std::string&) {
        const std::string k = cpfx + c.name;
        if (const std::string* v = annotation(p, k))
          if (!valid_seccomp_ann(*v)) e.push_back(forbidden_str("metadata.annotations[" + k + "]", *v));
      });
      return {"seccompProfile", e};
    }
    case CV_SECCOMP_BASELINE_1_19:
      if (p.sec && !valid_seccomp_type(p.sec_type))
        e.push_back(forbidden_str("spec.securityContext.seccompProfile.type", p.sec_type));
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.sec && !valid_seccomp_type(c.sec_type))
          e.push_back(forbidden_str(f + ".securityContext.seccompProfile.type", c.sec_type));
      });
      return {"seccompProfile", e};
    case CV_SECCOMP_RESTRICTED_1_19:
    case CV_SECCOMP_RESTRICTED_1_25: {
      std::vector<FieldErr> bad, implicit;
      bool pod_set = false;
      if (p.sec) {
        if (!valid_seccomp_type(p.sec_type))
          bad.push_back(forbidden_str("spec.securityContext.seccompProfile.type", p.sec_type));
        else
          pod_set = true;
      }
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.sec) {
          if (!valid_seccomp_type(c.sec_type))
            bad.push_back(forbidden_str(f + ".securityContext.seccompProfile.type", c.sec_type));
        } else if (!pod_set) {
          implicit.push_back(required(f + ".securityContext.seccompProfile.type"));
        }
      });
      return {"seccompProfile", bad.empty() ? implicit : bad};
    }
    case CV_SYSCTLS_1_0:
    case CV_SYSCTLS_1_27:
    case CV_SYSCTLS_1_29: {
      const auto& ok = sysctl_allow((int)(cv - CV_SYSCTLS_1_0));
      for (size_t i = 0; i < p.sysctls.size(); ++i)
        if (!ok.count(p.sysctls[i]))
          e.push_back(forbidden_str("spec.securityContext.sysctls[" + std::to_string(i) + "].name", p.sysctls[i]));
      return {"forbidden sysctls", e};
    }
    case CV_WIN_HOST_PROCESS_1_0:
      visit(p, [&](const CtrView& c, const std::string& f) {
        if (c.whp == TRI_TRUE) e.push_back(forbidden(f + ".securityContext.windowsOptions.hostProcess", true));
      });
      if (p.whp == TRI_TRUE) e.push_back(forbidden("spec.securityContext.windowsOptions.hostProcess", true));
      return {"hostProcess", e};
  }
  return {"", e};
}

void replace_all(std::string& s, const std::string& from, const std::string& to) {  // strings.ReplaceAll
  std::string o;
  size_t i = 0;
  for (size_t j; (j = s.find(from, i)) != std::string::npos; i = j + from.size()) o += s.substr(i, j - i) + to;
  s = o + s.substr(i);
}

// ---- exclusions (pkg/pss/evaluate.go:72-317) ---------------------------------------------
static const uint8_t kCvCheckM[KPE_NUM_CV] = KPE_CV_CHECK_TABLE;
// one failing versioned check of evaluatePSS: its check id (CK_*) and field errors
struct PCheck {
  uint32_t ck;
  const char* reason;
  std::vector<FieldErr> errs;
};
// evaluatePSS (evaluate.go:24-70) of the rule's versioned checks over a pod view
std::vector<PCheck> evaluate_view(const PodView& p, uint32_t cv_mask) {
  std::vector<PCheck> out;
  for (uint32_t cv = 0; cv < KPE_NUM_CV; ++cv) {
    if (!((cv_mask >> cv) & 1u)) continue;
    // the 1.25 versions of these checks allow a pod whose spec.os.name is windows
    if ((cv == CV_APE_1_25 || cv == CV_CAPS_RESTRICTED_1_25 || cv == CV_SECCOMP_RESTRICTED_1_25) && windows(p)) continue;
    Failed f = check_errors(cv, p);
    if (!f.errs.empty()) out.push_back({kCvCheckM[cv], f.reason, std::move(f.errs)});
  }
  return out;
}
// PSS_controls_to_check_id (pkg/pss/utils/mapping.go:45-107): the check ids of a control, in order
const std::vector<uint32_t>& control_checks(const std::string& control) {
  static const std::vector<std::pair<std::string, std::vector<uint32_t>>> m = {
      {"Capabilities", {CK_CAPS_BASELINE, CK_CAPS_RESTRICTED}},
      {"Seccomp", {CK_SECCOMP_BASELINE, CK_SECCOMP_RESTRICTED}},
      {"Privileged Containers", {CK_PRIVILEGED}},
      {"Host Ports", {CK_HOST_PORTS}},
      {"/proc Mount Type", {CK_PROC_MOUNT}},
      {"HostProcess", {CK_WIN_HOST_PROCESS}},
      {"SELinux", {CK_SELINUX}},
      {"Host Namespaces", {CK_HOST_NS}},
      {"HostPath Volumes", {CK_HOST_PATH}},
      {"Sysctls", {CK_SYSCTLS}},
      {"AppArmor", {CK_APPARMOR}},
      {"Privilege Escalation", {CK_APE}},
      {"Running as Non-root", {CK_RUN_AS_NON_ROOT}},
      {"Running as Non-root user", {CK_RUN_AS_USER}},
      {"Volume Types", {CK_RESTRICTED_VOLUMES}},
  };
  static const std::vector<uint32_t> none;
  for (auto& kv : m)
    if (kv.first == control) return kv.second;
  return none;
}
// regexIndex `\d+` -> "*"
std::string star_digits(const std::string& f) {
  std::string o;
  for (size_t i = 0; i < f.size();) {
    if (f[i] >= '0' && f[i] <= '9') {
      while (i < f.size() && f[i] >= '0' && f[i] <= '9') ++i;
      o += '*';
    } else {
      o += f[i++];
    }
  }
  return o;
}
// parseField (evaluate.go:193-204): the starred field, the first index, the container list word
struct PField {
  std::string field, ctype;
  long idx = -1;
  bool ctr = false;
};
PField parse_field(const std::string& f) {
  PField p;
  p.field = star_digits(f);
  std::vector<std::string> words;
  for (size_t i = 0; i < f.size();) {
    const char c = f[i];
    if (c >= '0' && c <= '9') {
      const size_t b = i;
      while (i < f.size() && f[i] >= '0' && f[i] <= '9') ++i;
      if (p.idx < 0) p.idx = std::atol(f.substr(b, i - b).c_str());
    } else if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) {
      const size_t b = i;
      while (i < f.size() && ((f[i] >= 'a' && f[i] <= 'z') || (f[i] >= 'A' && f[i] <= 'Z'))) ++i;
      words.push_back(f.substr(b, i - b));
    } else {
      ++i;
    }
  }
  p.ctype = words.size() > 1 ? words[1] : "";
  p.ctr = p.ctype == "containers" || p.ctype == "initContainers" || p.ctype == "ephemeralContainers";
  return p;
}
// getContainerInfo (evaluate.go:206-219); null past the list (the reference would panic)
const CtrView* container_info(const PodView& p, long idx, const std::string& ctype) {
  const int l = ctype == "initContainers" ? 0 : ctype == "containers" ? 1 : ctype == "ephemeralContainers" ? 2 : -1;
  if (l < 0 || idx < 0 || (size_t)idx >= p.ctr[l].size()) return nullptr;
  return &p.ctr[l][(size_t)idx];
}
// extractBadValues (evaluate.go:163-182): a string (non-empty), bool, Go int or []string
std::vector<std::string> bad_values(const FieldErr& e) {
  switch (e.kind) {
    case BV_STR: return {e.val};
    case BV_BOOL:
    case BV_INT: return {e.val};
    case BV_LIST: return e.list;
    default: return {};
  }
}
bool check_patterns(const std::vector<std::string>& pats, const std::string& s) {  // wildcard.CheckPatterns
  for (auto& p : pats)
    if (go_wildcard(p, s)) return true;
  return false;
}
// exemptExclusions (evaluate.go:72-161): defaults keyed by check id (the last result of an id
// wins, as in the Go map), each exclude field error removing the first matching default error
// (remove: swap with the last); *err: an invalid exclude (Validate: restrictedField and values
// go together)
std::vector<PCheck> exempt(const std::vector<PCheck>& defaults, const std::vector<PCheck>& xres, const PssExcl& ex,
                           const PodView& pod, const PodView* matching, bool ctr_level, bool* err) {
  *err = false;
  if (ex.field.empty() != ex.values.empty()) {
    *err = true;
    return {};
  }
  std::vector<uint32_t> order;
  std::vector<PCheck> m(KPE_NUM_CHECKS);
  std::vector<bool> has(KPE_NUM_CHECKS, false);
  for (auto& r : defaults) {
    if (!has[r.ck]) order.push_back(r.ck);
    m[r.ck] = r, has[r.ck] = true;
  }
  const std::vector<uint32_t>& ids = control_checks(ex.control);
  for (auto& xr : xres)
    for (uint32_t id : ids) {
      if (xr.ck != id) continue;
      for (auto& xe : xr.errs) {
        std::string xfield;
        const CtrView* xc = nullptr;
        bool xcl = false;
        if (ctr_level) {
          const PField pf = parse_field(xe.field);
          xfield = pf.field, xcl = pf.ctr;
          if (xcl) xc = container_info(*matching, pf.idx, pf.ctype);
        } else {
          xfield = star_digits(xe.field);
        }
        if (!(xfield == ex.field || ex.field.empty())) continue;
        bool flag = true;
        if (!ex.values.empty())
          for (auto& b : bad_values(xe))
            if (!check_patterns(ex.values, b)) {
              flag = false;
              break;
            }
        if (!flag || !has[id]) continue;  // a missing id: the zero result, a nil ErrList
        auto& errs = m[id].errs;
        for (size_t i = 0; i < errs.size(); ++i) {
          std::string dfield;
          const CtrView* dc = nullptr;
          bool dcl = false;
          if (ctr_level) {
            const PField pf = parse_field(errs[i].field);
            dfield = pf.field, dcl = pf.ctr;
            if (dcl) dc = container_info(pod, pf.idx, pf.ctype);
          } else {
            dfield = star_digits(errs[i].field);
          }
          const bool hit = dcl ? (xfield == dfield && xc && dc && xc->name == dc->name) : xfield == dfield;
          if (hit) {
            errs[i] = errs.back();
            errs.pop_back();
            break;
          }
        }
        if (errs.empty()) has[id] = false;
      }
    }
  std::vector<PCheck> out;
  for (uint32_t id : order)
    if (has[id]) out.push_back(m[id]);
  return out;
}
// ApplyPodSecurityExclusion (evaluate.go:255-279) with GetPodWithMatchingContainers (:283-317):
// a pod-level exclude evaluates the pod with one empty "fake" container, an image exclude a pod of
// the matching containers only (name / namespace metadata, no other spec field); *err: the last
// exclude's error
std::vector<PCheck> apply_exclusion(const std::vector<PCheck>& defaults0, const std::vector<PssExcl>& excl,
                                    const PodView& pod, uint32_t cv_mask, bool* err) {
  std::vector<PCheck> defaults = defaults0;
  *err = false;
  for (auto& ex : excl) {
    bool e = false;
    if (ex.images.empty()) {
      PodView spec = pod;
      CtrView fake;
      fake.name = "fake";
      spec.ctr[0].clear(), spec.ctr[1].assign(1, fake), spec.ctr[2].clear();
      defaults = exempt(defaults, evaluate_view(spec, cv_mask), ex, pod, nullptr, false, &e);
    } else {
      PodView match;
      for (int l = 0; l < 3; ++l)
        for (auto& c : pod.ctr[l])
          if (check_patterns(ex.images, c.image)) match.ctr[l].push_back(c);
      defaults = exempt(defaults, evaluate_view(match, cv_mask), ex, pod, &match, true, &e);
    }
    *err = e;
  }
  return defaults;
}
// convertChecks (validate_pss.go:114-135) then FormatChecksPrint (evaluate.go:331-362)
std::string format_checks(std::vector<PCheck>& checks, const std::string& kind, bool convert) {
  const bool tmpl = kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
                    kind == "ReplicaSet" || kind == "ReplicationController";
  std::string out;
  for (auto& c : checks) {
    out += "\n(Forbidden reason: ";
    out += c.reason;
    out += ", field error list: [";
    for (size_t i = 0; i < c.errs.size(); ++i) {
      FieldErr& x = c.errs[i];
      if (convert) {
        if (tmpl) replace_all(x.field, "spec", "spec.template.spec");
        else if (kind == "CronJob") replace_all(x.field, "spec", "spec.jobTemplate.spec.template.spec");
        replace_all(x.field, "metadata", "spec.template.metadata");
      }
      if (x.forbidden && x.kind != BV_NONE) out += x.field + " is forbidden, don't set the BadValue: " + x.val;
      else out += x.field + (x.forbidden ? ": Forbidden" : ": Required value");
      if (i + 1 != c.errs.size()) out += ", ";
    }
    out += "])";
  }
  return out;
}

}  // namespace

std::string pss_fail_message_ex(const std::string& rule, const std::string& level, const std::string& version,
                                const std::string& kind, const PodView& pod, uint32_t cv_mask,
                                const std::vector<PssExcl>* rule_ex, const std::vector<PssExcl>* exc) {
  std::vector<PCheck> checks = evaluate_view(pod, cv_mask);  // EvaluatePod
  bool err = false;
  if (rule_ex && !rule_ex->empty()) checks = apply_exclusion(checks, *rule_ex, pod, cv_mask, &err);
  // convertChecks rewrites the fields in place; the exception's exclusions compare against them
  const bool tmpl = kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
                    kind == "ReplicaSet" || kind == "ReplicationController";
  for (auto& c : checks)
    for (auto& x : c.errs) {
      if (tmpl) replace_all(x.field, "spec", "spec.template.spec");
      else if (kind == "CronJob") replace_all(x.field, "spec", "spec.jobTemplate.spec.template.spec");
      replace_all(x.field, "metadata", "spec.template.metadata");
    }
  if (exc) checks = apply_exclusion(checks, *exc, pod, cv_mask, &err);
  return "Validation rule '" + rule + "' failed. It violates PodSecurity \"" + level + ":" + version + "\": " +
         format_checks(checks, kind, false);
}

std::string pss_pass_message(const std::string& rule) { return "Validation rule '" + rule + "' passed."; }

std::string pss_fail_message(const std::string& rule, const std::string& level, const std::string& version,
                             const std::string& kind, const PodView& pod, uint32_t cv_fail) {
  const bool tmpl = kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
                    kind == "ReplicaSet" || kind == "ReplicationController";
  std::string checks;
  for (uint32_t cv = 0; cv < KPE_NUM_CV; ++cv) {
    if (!((cv_fail >> cv) & 1u)) continue;
    Failed f = check_errors(cv, pod);
    checks += "\n(Forbidden reason: ";
    checks += f.reason;
    checks += ", field error list: [";
    for (size_t i = 0; i < f.errs.size(); ++i) {
      FieldErr& x = f.errs[i];
      // convertChecks (validate_pss.go:114-135)
      if (tmpl) replace_all(x.field, "spec", "spec.template.spec");
      else if (kind == "CronJob") replace_all(x.field, "spec", "spec.jobTemplate.spec.template.spec");
      replace_all(x.field, "metadata", "spec.template.metadata");
      // FormatChecksPrint: a Forbidden error with a non-empty bad value, else err.Error()
      if (x.forbidden && x.kind != BV_NONE) checks += x.field + " is forbidden, don't set the BadValue: " + x.val;
      else checks += x.field + (x.forbidden ? ": Forbidden" : ": Required value");
      if (i + 1 != f.errs.size()) checks += ", ";
    }
    checks += "])";
  }
  return "Validation rule '" + rule + "' failed. It violates PodSecurity \"" + level + ":" + version + "\": " + checks;
}

}  // namespace kpe
