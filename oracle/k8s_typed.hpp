// ORACLE — test infrastructure only. Never linked into the product path.
//
// Restatement of the typed decode the PSS handler performs before evaluating:
//   pkg/engine/handlers/validation/validate_pss.go:137-188 (getSpec):
//     resource.MarshalJSON() + encoding/json.Unmarshal into corev1.Pod /
//     appsv1.Deployment (for DaemonSet, Deployment, Job, StatefulSet, ReplicaSet,
//     ReplicationController) / batchv1.CronJob.
// Any JSON type mismatch in a decoded field makes the reference return a
// RuleError (validate_pss.go:66-68). encoding/json semantics restated here:
//   * object keys match struct fields case-insensitively, processed in order
//     (last occurrence wins);
//   * null leaves the field untouched (nil pointer / zero value);
//   * unknown keys are ignored;
//   * ints: a JSON number decodes into intN only if it is written as an
//     integer literal in range. The resource went through unstructured
//     (whole -> int64, else float64) and MarshalJSON first, so a float64 that is
//     integral and < 1e21 in magnitude is re-encoded as an integer literal.
// Typed-schema coverage: every member of the decode target is type-checked against
// k8s_schema.hpp (typecheck_struct, one pass over the whole document); the dec:: walkers
// below extract (and re-check) the fields the PSS checks read. See DESIGN.md §10.
#pragma once
#include <algorithm>
#include <cctype>
#include <optional>
#include <string>
#include <vector>

#include "json_dom.hpp"
#include "k8s_schema.hpp"
#include "pattern.hpp"

namespace oracle {

struct DecodeError {
  std::string msg;
};

struct SELinuxOptions {
  std::string user, role, type, level;
};
struct SeccompProfile {
  std::string type;
};
struct WindowsOptions {
  std::optional<bool> hostProcess;
};
struct Capabilities {
  std::vector<std::string> add, drop;
};
struct SecurityContext {
  std::optional<Capabilities> capabilities;
  std::optional<bool> privileged;
  std::optional<SELinuxOptions> seLinuxOptions;
  std::optional<WindowsOptions> windowsOptions;
  std::optional<int64_t> runAsUser;
  std::optional<bool> runAsNonRoot;
  std::optional<bool> allowPrivilegeEscalation;
  std::optional<std::string> procMount;
  std::optional<SeccompProfile> seccompProfile;
};
struct ContainerPort {
  int32_t hostPort = 0;
  int32_t containerPort = 0;
};
struct Container {
  std::string name, image;
  std::vector<ContainerPort> ports;
  std::optional<SecurityContext> securityContext;
};
struct Sysctl {
  std::string name, value;
};
struct PodSecurityContext {
  std::optional<SELinuxOptions> seLinuxOptions;
  std::optional<WindowsOptions> windowsOptions;
  std::optional<int64_t> runAsUser;
  std::optional<bool> runAsNonRoot;
  std::vector<Sysctl> sysctls;
  std::optional<SeccompProfile> seccompProfile;
};

// Volume source field names in corev1.VolumeSource declaration order.
static const char* const kVolumeSources[] = {
    "hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "secret", "nfs",
    "iscsi", "glusterfs", "persistentVolumeClaim", "rbd", "flexVolume", "cinder", "cephfs", "flocker",
    "downwardAPI", "fc", "azureFile", "configMap", "vsphereVolume", "quobyte", "azureDisk",
    "photonPersistentDisk", "projected", "portworxVolume", "scaleIO", "storageos", "csi", "ephemeral"};
constexpr int kNumVolumeSources = sizeof(kVolumeSources) / sizeof(kVolumeSources[0]);

struct Volume {
  std::string name;
  bool has[kNumVolumeSources] = {};
  bool source(const char* n) const {
    for (int i = 0; i < kNumVolumeSources; ++i)
      if (!strcmp(kVolumeSources[i], n)) return has[i];
    return false;
  }
};
struct PodSpec {
  std::vector<Volume> volumes;
  std::vector<Container> initContainers, containers, ephemeralContainers;
  bool hostNetwork = false, hostPID = false, hostIPC = false;
  std::optional<PodSecurityContext> securityContext;
  std::optional<std::string> osName;  // spec.os.name (nil os => nullopt)
};
struct ObjectMeta {
  std::string name, generateName, ns;
  std::vector<std::pair<std::string, std::string>> labels, annotations;
  const std::string* annotation(const std::string& k) const {
    for (auto& kv : annotations)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};
struct Pod {
  ObjectMeta meta;
  PodSpec spec;
};

// ---------------------------------------------------------------------------
namespace dec {

inline std::string fold(const std::string& s) {
  std::string o(s);
  for (auto& c : o) c = (char)tolower((unsigned char)c);
  return o;
}

[[noreturn]] inline void type_err(const char* want, const std::string& field) {
  throw DecodeError{std::string("json: cannot unmarshal into Go struct field ") + field + " of type " + want};
}

inline void want_obj(const JVal* v, const std::string& f) {
  if (v->t != JT::Obj) type_err("object", f);
}

inline bool integral_ok(const JVal* v, int64_t lo, int64_t hi, int64_t* out) {
  if (v->t == JT::Int) {
    if (v->i < lo || v->i > hi) return false;
    *out = v->i;
    return true;
  }
  if (v->t == JT::Float) {
    double d = v->f;
    if (!std::isfinite(d) || std::floor(d) != d || std::fabs(d) >= 1e21) return false;
    if (d < (double)lo || d > (double)hi) return false;
    *out = (int64_t)d;
    return true;
  }
  return false;
}

inline void i64(const JVal* v, std::optional<int64_t>& o, const std::string& f) {
  if (v->is_null()) return;
  int64_t x;
  if (!integral_ok(v, INT64_MIN, INT64_MAX, &x)) type_err("int64", f);
  o = x;
}
inline void i32(const JVal* v, int32_t& o, const std::string& f) {
  if (v->is_null()) return;
  int64_t x;
  if (!integral_ok(v, INT32_MIN, INT32_MAX, &x)) type_err("int32", f);
  o = (int32_t)x;
}
inline void i32p(const JVal* v, const std::string& f) {
  int32_t d = 0;
  i32(v, d, f);
}
inline void i64p(const JVal* v, const std::string& f) {
  std::optional<int64_t> d;
  i64(v, d, f);
}
inline void boolean(const JVal* v, bool& o, const std::string& f) {
  if (v->is_null()) return;
  if (v->t != JT::Bool) type_err("bool", f);
  o = v->b;
}
inline void boolp(const JVal* v, std::optional<bool>& o, const std::string& f) {
  if (v->is_null()) return;
  if (v->t != JT::Bool) type_err("bool", f);
  o = v->b;
}
inline void str(const JVal* v, std::string& o, const std::string& f) {
  if (v->is_null()) return;
  if (v->t != JT::Str) type_err("string", f);
  o = v->s;
}
inline void strp(const JVal* v, std::optional<std::string>& o, const std::string& f) {
  if (v->is_null()) return;
  if (v->t != JT::Str) type_err("string", f);
  o = v->s;
}
inline void strlist(const JVal* v, std::vector<std::string>& o, const std::string& f) {
  if (v->is_null()) {
    o.clear();
    return;
  }
  if (v->t != JT::Arr) type_err("[]string", f);
  o.clear();
  for (auto& e : v->a) {
    std::string s;
    str(e.get(), s, f);
    o.push_back(s);
  }
}
inline void i64list(const JVal* v, const std::string& f) {
  if (v->is_null()) return;
  if (v->t != JT::Arr) type_err("[]int64", f);
  for (auto& e : v->a) i64p(e.get(), f);
}
inline void strmap(const JVal* v, std::vector<std::pair<std::string, std::string>>& o, const std::string& f) {
  if (v->is_null()) {
    o.clear();
    return;
  }
  if (v->t != JT::Obj) type_err("map[string]string", f);
  o.clear();
  for (auto& kv : v->o) {
    std::string s;
    str(kv.second.get(), s, f);
    o.emplace_back(kv.first, s);
  }
}
// metav1.Time: null or an RFC3339 string.
inline bool rfc3339(const std::string& s) {
  // YYYY-MM-DDTHH:MM:SS[.frac](Z|+HH:MM|-HH:MM)
  auto d = [&](size_t i) { return i < s.size() && isdigit((unsigned char)s[i]); };
  if (s.size() < 20) return false;
  for (size_t i : {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18})
    if (!d(i)) return false;
  if (s[4] != '-' || s[7] != '-' || (s[10] != 'T' && s[10] != 't') || s[13] != ':' || s[16] != ':') return false;
  size_t i = 19;
  if (i < s.size() && s[i] == '.') {
    ++i;
    size_t st = i;
    while (d(i)) ++i;
    if (i == st) return false;
  }
  if (i < s.size() && (s[i] == 'Z' || s[i] == 'z')) return i + 1 == s.size();
  if (i < s.size() && (s[i] == '+' || s[i] == '-'))
    return i + 6 == s.size() && d(i + 1) && d(i + 2) && s[i + 3] == ':' && d(i + 4) && d(i + 5);
  return false;
}
inline void timev(const JVal* v, const std::string& f) {
  if (v->is_null()) return;
  if (v->t != JT::Str || !rfc3339(v->s)) type_err("Time", f);
}

template <class F>
inline void each_key(const JVal* v, const std::string& f, F fn) {
  want_obj(v, f);
  for (auto& kv : v->o) fn(fold(kv.first), kv.second.get());
}

inline void label_selector(const JVal* v, const std::string& f) {
  if (v->is_null()) return;
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    if (k == "matchlabels") {
      std::vector<std::pair<std::string, std::string>> m;
      strmap(x, m, f + ".matchLabels");
    } else if (k == "matchexpressions") {
      if (x->is_null()) return;
      if (x->t != JT::Arr) type_err("[]LabelSelectorRequirement", f);
      for (auto& e : x->a) {
        if (e->is_null()) continue;
        each_key(e.get(), f, [&](const std::string& k2, const JVal* y) {
          std::string s;
          std::vector<std::string> l;
          if (k2 == "key" || k2 == "operator") str(y, s, f);
          else if (k2 == "values") strlist(y, l, f);
        });
      }
    }
  });
}

inline void object_meta(const JVal* v, ObjectMeta& m, const std::string& f) {
  if (v->is_null()) return;
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::string tmp;
    std::vector<std::string> l;
    if (k == "name") str(x, m.name, f + ".name");
    else if (k == "generatename") str(x, m.generateName, f + ".generateName");
    else if (k == "namespace") str(x, m.ns, f + ".namespace");
    else if (k == "uid" || k == "resourceversion" || k == "selflink") str(x, tmp, f);
    else if (k == "generation") i64p(x, f + ".generation");
    else if (k == "creationtimestamp" || k == "deletiontimestamp") timev(x, f);
    else if (k == "labels") strmap(x, m.labels, f + ".labels");
    else if (k == "annotations") strmap(x, m.annotations, f + ".annotations");
    else if (k == "finalizers") strlist(x, l, f + ".finalizers");
  });
}

inline void selinux(const JVal* v, std::optional<SELinuxOptions>& o, const std::string& f) {
  if (v->is_null()) return;
  SELinuxOptions s = o ? *o : SELinuxOptions{};
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    if (k == "user") str(x, s.user, f);
    else if (k == "role") str(x, s.role, f);
    else if (k == "type") str(x, s.type, f);
    else if (k == "level") str(x, s.level, f);
  });
  o = s;
}
inline void seccomp(const JVal* v, std::optional<SeccompProfile>& o, const std::string& f) {
  if (v->is_null()) return;
  SeccompProfile s = o ? *o : SeccompProfile{};
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::optional<std::string> lp;
    if (k == "type") str(x, s.type, f);
    else if (k == "localhostprofile") strp(x, lp, f);
  });
  o = s;
}
inline void winopts(const JVal* v, std::optional<WindowsOptions>& o, const std::string& f) {
  if (v->is_null()) return;
  WindowsOptions w = o ? *o : WindowsOptions{};
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::optional<std::string> s;
    if (k == "hostprocess") boolp(x, w.hostProcess, f);
    else if (k == "gmsacredentialspecname" || k == "gmsacredentialspec" || k == "runasusername") strp(x, s, f);
  });
  o = w;
}
inline void security_context(const JVal* v, std::optional<SecurityContext>& o, const std::string& f) {
  if (v->is_null()) return;
  SecurityContext s = o ? *o : SecurityContext{};
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::optional<bool> b;
    if (k == "capabilities") {
      if (x->is_null()) return;
      Capabilities c = s.capabilities ? *s.capabilities : Capabilities{};
      each_key(x, f, [&](const std::string& k2, const JVal* y) {
        if (k2 == "add") strlist(y, c.add, f + ".capabilities.add");
        else if (k2 == "drop") strlist(y, c.drop, f + ".capabilities.drop");
      });
      s.capabilities = c;
    } else if (k == "privileged") boolp(x, s.privileged, f);
    else if (k == "selinuxoptions") selinux(x, s.seLinuxOptions, f);
    else if (k == "windowsoptions") winopts(x, s.windowsOptions, f);
    else if (k == "runasuser") i64(x, s.runAsUser, f);
    else if (k == "runasgroup") i64p(x, f);
    else if (k == "runasnonroot") boolp(x, s.runAsNonRoot, f);
    else if (k == "readonlyrootfilesystem") boolp(x, b, f);
    else if (k == "allowprivilegeescalation") boolp(x, s.allowPrivilegeEscalation, f);
    else if (k == "procmount") strp(x, s.procMount, f);
    else if (k == "seccompprofile") seccomp(x, s.seccompProfile, f);
  });
  o = s;
}
inline void pod_security_context(const JVal* v, std::optional<PodSecurityContext>& o, const std::string& f) {
  if (v->is_null()) return;
  PodSecurityContext s = o ? *o : PodSecurityContext{};
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::optional<std::string> sp;
    if (k == "selinuxoptions") selinux(x, s.seLinuxOptions, f);
    else if (k == "windowsoptions") winopts(x, s.windowsOptions, f);
    else if (k == "runasuser") i64(x, s.runAsUser, f);
    else if (k == "runasgroup" || k == "fsgroup") i64p(x, f);
    else if (k == "runasnonroot") boolp(x, s.runAsNonRoot, f);
    else if (k == "supplementalgroups") i64list(x, f);
    else if (k == "fsgroupchangepolicy") strp(x, sp, f);
    else if (k == "seccompprofile") seccomp(x, s.seccompProfile, f);
    else if (k == "sysctls") {
      if (x->is_null()) {
        s.sysctls.clear();
        return;
      }
      if (x->t != JT::Arr) type_err("[]Sysctl", f);
      s.sysctls.clear();
      for (auto& e : x->a) {
        Sysctl sy;
        if (!e->is_null())
          each_key(e.get(), f, [&](const std::string& k2, const JVal* y) {
            if (k2 == "name") str(y, sy.name, f);
            else if (k2 == "value") str(y, sy.value, f);
          });
        s.sysctls.push_back(sy);
      }
    }
  });
  o = s;
}
inline void container(const JVal* v, Container& c, const std::string& f) {
  if (v->is_null()) return;
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::string s;
    std::vector<std::string> l;
    bool b = false;
    if (k == "name") str(x, c.name, f);
    else if (k == "image") str(x, c.image, f);
    else if (k == "command" || k == "args") strlist(x, l, f);
    else if (k == "workingdir" || k == "imagepullpolicy" || k == "terminationmessagepath" ||
             k == "terminationmessagepolicy" || k == "targetcontainername")
      str(x, s, f);
    else if (k == "stdin" || k == "stdinonce" || k == "tty") boolean(x, b, f);
    else if (k == "ports") {
      if (x->is_null()) {
        c.ports.clear();
        return;
      }
      if (x->t != JT::Arr) type_err("[]ContainerPort", f);
      c.ports.clear();
      for (auto& e : x->a) {
        ContainerPort p;
        if (!e->is_null())
          each_key(e.get(), f, [&](const std::string& k2, const JVal* y) {
            std::string t;
            if (k2 == "hostport") i32(y, p.hostPort, f + ".ports.hostPort");
            else if (k2 == "containerport") i32(y, p.containerPort, f + ".ports.containerPort");
            else if (k2 == "name" || k2 == "protocol" || k2 == "hostip") str(y, t, f);
          });
        c.ports.push_back(p);
      }
    } else if (k == "env") {
      if (x->is_null()) return;
      if (x->t != JT::Arr) type_err("[]EnvVar", f);
      for (auto& e : x->a) {
        if (e->is_null()) continue;
        each_key(e.get(), f, [&](const std::string& k2, const JVal* y) {
          std::string t;
          if (k2 == "name" || k2 == "value") str(y, t, f);
          else if (k2 == "valuefrom" && !y->is_null()) want_obj(y, f);
        });
      }
    } else if (k == "resources") {
      if (!x->is_null()) want_obj(x, f);
    } else if (k == "securitycontext") security_context(x, c.securityContext, f + ".securityContext");
  });
}
inline void containers(const JVal* v, std::vector<Container>& o, const std::string& f) {
  if (v->is_null()) {
    o.clear();
    return;
  }
  if (v->t != JT::Arr) type_err("[]Container", f);
  o.clear();
  for (auto& e : v->a) {
    Container c;
    container(e.get(), c, f);
    o.push_back(c);
  }
}
inline void volumes(const JVal* v, std::vector<Volume>& o, const std::string& f) {
  if (v->is_null()) {
    o.clear();
    return;
  }
  if (v->t != JT::Arr) type_err("[]Volume", f);
  o.clear();
  for (auto& e : v->a) {
    Volume vol;
    if (!e->is_null())
      each_key(e.get(), f, [&](const std::string& k, const JVal* x) {
        if (k == "name") {
          str(x, vol.name, f);
          return;
        }
        for (int i = 0; i < kNumVolumeSources; ++i) {
          if (k == fold(kVolumeSources[i])) {
            if (x->is_null()) {
              vol.has[i] = false;
              return;
            }
            want_obj(x, f + "." + kVolumeSources[i]);
            vol.has[i] = true;
            // a few leaf types inside the common sources
            for (auto& kv : x->o) {
              std::string kk = fold(kv.first), t;
              const JVal* y = kv.second.get();
              if (kk == "path" || kk == "secretname" || kk == "claimname" || kk == "medium" || kk == "server")
                str(y, t, f);
              else if (kk == "defaultmode") i32p(y, f);
              else if (kk == "readonly") {
                bool b = false;
                boolean(y, b, f);
              }
            }
            return;
          }
        }
      });
    o.push_back(vol);
  }
}
inline void pod_spec(const JVal* v, PodSpec& s, const std::string& f) {
  if (v->is_null()) return;
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    std::string t;
    std::optional<bool> ob;
    std::optional<std::string> os;
    std::vector<std::pair<std::string, std::string>> m;
    if (k == "volumes") volumes(x, s.volumes, f + ".volumes");
    else if (k == "initcontainers") containers(x, s.initContainers, f + ".initContainers");
    else if (k == "containers") containers(x, s.containers, f + ".containers");
    else if (k == "ephemeralcontainers") containers(x, s.ephemeralContainers, f + ".ephemeralContainers");
    else if (k == "hostnetwork") boolean(x, s.hostNetwork, f);
    else if (k == "hostpid") boolean(x, s.hostPID, f);
    else if (k == "hostipc") boolean(x, s.hostIPC, f);
    else if (k == "securitycontext") pod_security_context(x, s.securityContext, f + ".securityContext");
    else if (k == "os") {
      if (x->is_null()) return;
      std::string name = s.osName ? *s.osName : std::string();
      each_key(x, f, [&](const std::string& k2, const JVal* y) {
        if (k2 == "name") str(y, name, f);
      });
      s.osName = name;
    } else if (k == "restartpolicy" || k == "dnspolicy" || k == "serviceaccountname" || k == "serviceaccount" ||
               k == "nodename" || k == "hostname" || k == "subdomain" || k == "priorityclassname" ||
               k == "schedulername")
      str(x, t, f);
    else if (k == "terminationgraceperiodseconds" || k == "activedeadlineseconds") i64p(x, f);
    else if (k == "priority") i32p(x, f);
    else if (k == "automountserviceaccounttoken" || k == "shareprocessnamespace" || k == "hostusers" ||
             k == "enableservicelinks")
      boolp(x, ob, f);
    else if (k == "runtimeclassname") strp(x, os, f);
    else if (k == "nodeselector") strmap(x, m, f);
  });
}
inline void pod_template(const JVal* v, Pod& p, const std::string& f) {
  if (v->is_null()) return;
  each_key(v, f, [&](const std::string& k, const JVal* x) {
    if (k == "metadata") object_meta(x, p.meta, f + ".metadata");
    else if (k == "spec") pod_spec(x, p.spec, f + ".spec");
  });
}

}  // namespace dec

// ---------------------------------------------------------------------------
// encoding/json.Unmarshal type checks over the Go struct table (k8s_schema.hpp).
namespace tc {

inline const GoStruct* find_struct(const std::string& n) {
  static const auto idx = [] {
    std::vector<std::pair<std::string, const GoStruct*>> v;
    for (auto& s : go_structs()) v.emplace_back(s.name, &s);
    return v;
  }();
  for (auto& e : idx)
    if (e.first == n) return e.second;
  return nullptr;
}

inline void value(const JVal* v, const std::string& ty, const std::string& f);

// a struct: keys match members exactly, else case-insensitively (encoding/json field
// matching); unknown members are ignored.
inline void struct_value(const JVal* v, const GoStruct* s, const std::string& f) {
  if (v->t != JT::Obj) dec::type_err(s->name, f);
  for (auto& kv : v->o) {
    const char* ty = nullptr;
    for (auto& fd : s->fields)
      if (kv.first == fd.first) {
        ty = fd.second;
        break;
      }
    if (!ty) {
      const std::string k = dec::fold(kv.first);
      for (auto& fd : s->fields)
        if (k == dec::fold(fd.first)) {
          ty = fd.second;
          break;
        }
    }
    if (ty) value(kv.second.get(), ty, f + "." + kv.first);
  }
}

inline void value(const JVal* v, const std::string& ty, const std::string& f) {
  if (v->is_null()) return;  // null leaves any Go value untouched
  int64_t x;
  if (ty == "string") {
    if (v->t != JT::Str) dec::type_err("string", f);
  } else if (ty == "bool") {
    if (v->t != JT::Bool) dec::type_err("bool", f);
  } else if (ty == "int32") {
    if (!dec::integral_ok(v, INT32_MIN, INT32_MAX, &x)) dec::type_err("int32", f);
  } else if (ty == "int64") {
    if (!dec::integral_ok(v, INT64_MIN, INT64_MAX, &x)) dec::type_err("int64", f);
  } else if (ty == "resource.Quantity") {
    // Quantity.UnmarshalJSON: ParseQuantity(strings.TrimSpace(...)) of the string, or of the
    // number's literal (any JSON number re-marshalled by Go parses as a quantity)
    if (v->t == JT::Str) {
      const std::string& s = v->s;
      size_t a = s.find_first_not_of(" \t\n\r"), b = s.find_last_not_of(" \t\n\r");
      pat::Qty q;
      if (a == std::string::npos || !pat::go_parse_quantity(s.substr(a, b - a + 1), &q))
        dec::type_err("Quantity", f);
    } else if (v->t != JT::Int && v->t != JT::Float) {
      dec::type_err("Quantity", f);
    }
  } else if (ty == "intstr.IntOrString") {  // a string, or an int32
    if (v->t != JT::Str && !dec::integral_ok(v, INT32_MIN, INT32_MAX, &x)) dec::type_err("IntOrString", f);
  } else if (ty == "metav1.Time") {
    dec::timev(v, f);
  } else if (ty == "metav1.FieldsV1") {
    // any JSON
  } else if (ty.rfind("[]", 0) == 0) {
    if (v->t != JT::Arr) dec::type_err(ty.c_str(), f);
    const std::string el = ty.substr(2);
    for (auto& e : v->a) value(e.get(), el, f);
  } else if (ty.rfind("map[string]", 0) == 0) {
    if (v->t != JT::Obj) dec::type_err(ty.c_str(), f);
    const std::string el = ty.substr(11);
    for (auto& kv : v->o) value(kv.second.get(), el, f);
  } else {
    const GoStruct* s = find_struct(ty);
    if (!s) throw std::logic_error("k8s_schema: unknown Go type " + ty);
    struct_value(v, s, f);
  }
}

}  // namespace tc

enum class SpecKind { Pod, Controller, CronJob, Other };

inline SpecKind spec_kind(const std::string& kind) {
  if (kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
      kind == "ReplicaSet" || kind == "ReplicationController")
    return SpecKind::Controller;
  if (kind == "CronJob") return SpecKind::CronJob;
  if (kind == "Pod") return SpecKind::Pod;
  return SpecKind::Other;
}

// validate_pss.go:137-188 getSpec. Throws DecodeError on type mismatch or an
// unsupported kind ("could not find correct resource type").
inline Pod get_spec(const JVal& res, const std::string& kind) {
  using namespace dec;
  SpecKind sk = spec_kind(kind);
  if (sk == SpecKind::Other) throw DecodeError{"could not find correct resource type"};
  tc::value(&res, sk == SpecKind::Pod ? "Pod" : sk == SpecKind::Controller ? "Deployment" : "CronJob", "");
  Pod out;
  ObjectMeta topmeta;
  each_key(&res, "", [&](const std::string& k, const JVal* x) {
    std::string t;
    if (k == "apiversion" || k == "kind") {
      str(x, t, k);
    } else if (k == "metadata") {
      object_meta(x, sk == SpecKind::Pod ? out.meta : topmeta, "metadata");
    } else if (k == "spec") {
      if (sk == SpecKind::Pod) {
        pod_spec(x, out.spec, "spec");
      } else if (sk == SpecKind::Controller) {
        if (x->is_null()) return;
        each_key(x, "spec", [&](const std::string& k2, const JVal* y) {
          std::optional<bool> b;
          if (k2 == "replicas" || k2 == "revisionhistorylimit" || k2 == "progressdeadlineseconds") i32p(y, "spec");
          else if (k2 == "minreadyseconds") i32p(y, "spec");
          else if (k2 == "paused") {
            bool bb = false;
            boolean(y, bb, "spec.paused");
          } else if (k2 == "selector") label_selector(y, "spec.selector");
          else if (k2 == "template") pod_template(y, out, "spec.template");
        });
      } else {  // CronJob
        if (x->is_null()) return;
        each_key(x, "spec", [&](const std::string& k2, const JVal* y) {
          std::string t2;
          std::optional<bool> b;
          std::optional<std::string> os;
          if (k2 == "schedule" || k2 == "concurrencypolicy") str(y, t2, "spec");
          else if (k2 == "timezone") strp(y, os, "spec");
          else if (k2 == "startingdeadlineseconds") i64p(y, "spec");
          else if (k2 == "suspend") boolp(y, b, "spec");
          else if (k2 == "successfuljobshistorylimit" || k2 == "failedjobshistorylimit") i32p(y, "spec");
          else if (k2 == "jobtemplate") {
            if (y->is_null()) return;
            each_key(y, "spec.jobTemplate", [&](const std::string& k3, const JVal* z) {
              // CronJob quirk (validate_pss.go:165-166): metadata comes from
              // spec.jobTemplate.metadata, not spec.jobTemplate.spec.template.metadata.
              if (k3 == "metadata") object_meta(z, out.meta, "spec.jobTemplate.metadata");
              else if (k3 == "spec") {
                if (z->is_null()) return;
                each_key(z, "spec.jobTemplate.spec", [&](const std::string& k4, const JVal* w) {
                  std::optional<bool> b4;
                  std::optional<std::string> s4;
                  if (k4 == "parallelism" || k4 == "completions" || k4 == "backofflimit" ||
                      k4 == "ttlsecondsafterfinished")
                    i32p(w, "spec.jobTemplate.spec");
                  else if (k4 == "activedeadlineseconds") i64p(w, "spec.jobTemplate.spec");
                  else if (k4 == "selector") label_selector(w, "spec.jobTemplate.spec.selector");
                  else if (k4 == "manualselector" || k4 == "suspend") boolp(w, b4, "spec.jobTemplate.spec");
                  else if (k4 == "completionmode") strp(w, s4, "spec.jobTemplate.spec");
                  else if (k4 == "template") {
                    Pod tmp;
                    pod_template(w, tmp, "spec.jobTemplate.spec.template");
                    out.spec = tmp.spec;  // template metadata is decoded (type-checked) but unused
                  }
                });
              }
            });
          }
        });
      }
    }
  });
  return out;
}

}  // namespace oracle
