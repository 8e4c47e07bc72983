// Corpus flattener: NDJSON resources -> columnar, string-interned tables.
//
// Two views of every resource are extracted in one walk:
//  * the unstructured view the match path reads (unstructured.GetKind/GetName/
//    GetNamespace/GetLabels/GetAnnotations; pkg/engine/utils/match.go:52-160);
//  * the typed pod view the PSS handler reads after
//    getSpec (pkg/engine/handlers/validation/validate_pss.go:137-188):
//    encoding/json.Unmarshal into corev1.Pod / appsv1.Deployment / batchv1.CronJob.
//    Keys match case-insensitively, null is a no-op, unknown keys are ignored and
//    any type mismatch in a modelled field marks the row R_DECODE_ERR (=> the
//    reference's RuleError). The modelled field set is listed in DESIGN.md.
// The flattener only ENCODES (dictionary ids, enum codes, presence bits); every
// predicate is evaluated on the device.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <memory>
#include <cstring>
#include <stdexcept>
#include <string>
#include <atomic>
#include <functional>
#include <thread>
#include <vector>

#include "corpus.hpp"
#include "goval.hpp"
#include "imageref.hpp"
#include "jscan.hpp"
#include "k8s_schema.hpp"
#include "podview.hpp"

namespace kpe {

namespace {

// c_sc enum word -> state bitmap (schema.h CX_*): one bit per state of each field.
uint32_t state_bitmap(uint32_t w) {
  auto tri = [&](uint32_t sh, uint32_t t, uint32_t f, uint32_t u) {
    const uint32_t v = FIELD(w, sh, 2);
    return v == TRI_TRUE ? t : v == TRI_FALSE ? f : u;
  };
  uint32_t x = tri(C_PRIV_SH, CX_PRIV_T, CX_PRIV_F, CX_PRIV_U) | tri(C_APE_SH, CX_APE_T, CX_APE_F, CX_APE_U) |
               tri(C_RNR_SH, CX_RNR_T, CX_RNR_F, CX_RNR_U);
  const uint32_t rau = FIELD(w, C_RAU_SH, 2);
  x |= rau == RAU_ZERO ? CX_RAU_Z : rau == RAU_NONZERO ? CX_RAU_NZ : CX_RAU_U;
  static const uint32_t sec[5] = {CX_SEC_NONE, CX_SEC_RD, CX_SEC_LH, CX_SEC_UNC, CX_SEC_OTHER};
  x |= sec[std::min(FIELD(w, C_SECCOMP_SH, 3), 4u)];
  const uint32_t pm = FIELD(w, C_PROCMOUNT_SH, 2);
  x |= pm == PROCMOUNT_OTHER ? CX_PM_OTHER : pm == PROCMOUNT_DEFAULT ? CX_PM_DEFAULT : CX_PM_U;
  const uint32_t sel = FIELD(w, C_SEL_SH, 3);
  x |= sel == SEL_NONE ? CX_SEL_NONE : sel == SEL_OTHER ? CX_SEL_OTHER : CX_SEL_OK;
  if (w & C_SEL_USER) x |= CX_SEL_USER;
  if (w & C_SEL_ROLE) x |= CX_SEL_ROLE;
  x |= FIELD(w, C_WHP_SH, 2) == TRI_TRUE ? CX_WHP_T : CX_WHP_NT;
  x |= (w & C_CAPS_PRESENT) ? CX_CAPS : CX_NOCAPS;
  x |= FIELD(w, C_HOSTPORT_SH, 4) ? CX_HOSTPORT : CX_NOHOSTPORT;
  if (w & C_SC_PRESENT) x |= CX_SC;
  return x;
}

struct UView {  // unstructured metadata view
  std::string kind, api_version, name, generate_name, ns;
  bool labels_ok = true, ann_ok = true;
  std::vector<std::pair<std::string, std::string>> labels, ann;
  void reset() {
    kind.clear();
    api_version.clear();
    name.clear();
    generate_name.clear();
    ns.clear();
    labels_ok = ann_ok = true;
    labels.clear();
    ann.clear();
  }
};

static const char* const kVolSrc[KPE_NUM_VOLUME_SOURCES] = {
    "hostpath", "emptydir", "gcepersistentdisk", "awselasticblockstore", "gitrepo", "secret", "nfs",
    "iscsi", "glusterfs", "persistentvolumeclaim", "rbd", "flexvolume", "cinder", "cephfs", "flocker",
    "downwardapi", "fc", "azurefile", "configmap", "vspherevolume", "quobyte", "azuredisk",
    "photonpersistentdisk", "projected", "portworxvolume", "scaleio", "storageos", "csi", "ephemeral"};

// Typed decoder: walks a JSON value with the schema of a K8s Go type. `err` is
// sticky (json.Unmarshal returns the first UnmarshalTypeError).
class Typed {
 public:
  explicit Typed(JCur& c) : c_(c) {}
  bool err = false;

  // ---- leaves ----
  void str(std::string* out) {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Str) {
      bad();
      return;
    }
    std::string_view v;
    c_.str(&v, vs_);
    if (out) out->assign(v.data(), v.size());
  }
  void strp(bool* set, std::string* out) {  // *string
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Str) {
      bad();
      return;
    }
    std::string_view v;
    c_.str(&v, vs_);
    if (set) *set = true;
    if (out) out->assign(v.data(), v.size());
  }
  void boolean(bool* out) {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Bool) {
      bad();
      return;
    }
    bool b = false;
    c_.boolean(&b);
    if (out) *out = b;
  }
  void tri(uint32_t* out) {  // *bool
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Bool) {
      bad();
      return;
    }
    bool b = false;
    c_.boolean(&b);
    if (out) *out = b ? TRI_TRUE : TRI_FALSE;
  }
  bool integer(int64_t lo, int64_t hi, int64_t* out) {  // returns true if a value was set
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return false;
    }
    if (k != JK::Num) {
      bad();
      return false;
    }
    JNum n;
    c_.number(&n);
    int64_t x;
    if (!n.integral(&x) || x < lo || x > hi) {
      err = true;  // the number is consumed already
      return false;
    }
    if (out) *out = x;
    return true;
  }
  void i32() { integer(INT32_MIN, INT32_MAX, nullptr); }
  void i64() { integer(INT64_MIN, INT64_MAX, nullptr); }
  void strlist(std::vector<std::string>* out) {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      if (out) out->clear();
      return;
    }
    if (k != JK::Arr) {
      bad();
      return;
    }
    if (out) out->clear();
    c_.arr_begin();
    bool f = true;
    while (c_.arr_next(f)) {
      std::string s;
      str(out ? &s : nullptr);
      if (out) out->push_back(std::move(s));
    }
  }
  void i64list() {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Arr) {
      bad();
      return;
    }
    c_.arr_begin();
    bool f = true;
    while (c_.arr_next(f)) i64();
  }
  void strmap(std::vector<std::pair<std::string, std::string>>* out) {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      if (out) out->clear();
      return;
    }
    if (k != JK::Obj) {
      bad();
      return;
    }
    if (out) out->clear();
    c_.obj_begin();
    bool f = true;
    std::string_view key;
    while (c_.obj_next(f, &key, ks_)) {
      std::string kk(key);
      std::string v;
      str(out ? &v : nullptr);
      if (out) {
        bool rep = false;
        for (auto& e : *out)
          if (e.first == kk) {
            e.second = v;
            rep = true;
          }
        if (!rep) out->emplace_back(std::move(kk), std::move(v));
      }
    }
  }
  void timev() {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Str) {
      bad();
      return;
    }
    std::string_view v;
    c_.str(&v, vs_);
    if (!rfc3339(v)) err = true;
  }
  // struct id of a k8s type (k8s_schema.hpp), looked up once per call site
#define sid(name) ([] { static const uint16_t id_ = k8s::schema().struct_id(name); return id_; }())
  // The value of member `key` of struct `s`: type-checked against the schema, or skipped when
  // `key` is not a member (encoding/json ignores unknown fields).
  void member(uint16_t s, std::string_view key) {
    const auto& S = k8s::schema();
    const int f = S.field(s, key);
    if (f < 0) {
      c_.skip();
      return;
    }
    check(S.structs[s].fields[f].type);
  }
  // Consume one value of schema type `ty` (encoding/json Unmarshal semantics; a mismatch is
  // sticky in `err`, decoding goes on).
  void check(uint16_t ty) {
    const auto& S = k8s::schema();
    const k8s::Type T = S.types[ty];
    const JK k = c_.peek();
    if (k == JK::Null) {  // null leaves any field unset
      c_.null();
      return;
    }
    switch (T.kind) {
      case k8s::K_STR:
        if (k == JK::Str) c_.skip();
        else bad();
        return;
      case k8s::K_BOOL:
        if (k == JK::Bool) c_.skip();
        else bad();
        return;
      case k8s::K_I32: i32(); return;
      case k8s::K_I64: i64(); return;
      case k8s::K_QTY: {  // resource.Quantity.UnmarshalJSON: a number, or a ParseQuantity string
        if (k == JK::Num) {
          c_.skip();
        } else if (k == JK::Str) {
          std::string_view v;
          c_.str(&v, vs_);
          std::string t(v);
          size_t a = t.find_first_not_of(" \t\n\r"), b = t.find_last_not_of(" \t\n\r");
          goval::Quantity q;
          if (a == std::string::npos || !goval::parse_quantity(std::string_view(t).substr(a, b - a + 1), &q))
            err = true;
        } else {
          bad();
        }
        return;
      }
      case k8s::K_IOS:  // intstr.IntOrString: a string, or an int32
        if (k == JK::Str) c_.skip();
        else if (k == JK::Num) i32();
        else bad();
        return;
      case k8s::K_TIME: timev(); return;
      case k8s::K_RAW: c_.skip(); return;
      case k8s::K_STRUCT: obj(T.sub, [](std::string_view) { return false; }); return;
      case k8s::K_LIST:
        if (k != JK::Arr) {
          bad();
          return;
        }
        {
          c_.arr_begin();
          bool f = true;
          while (c_.arr_next(f)) check(T.sub);
        }
        return;
      case k8s::K_MAP:
        if (k != JK::Obj) {
          bad();
          return;
        }
        {
          c_.obj_begin();
          bool f = true;
          std::string_view key;
          while (c_.obj_next(f, &key, ks_)) check(T.sub);
        }
        return;
    }
  }

  // Iterate the keys of an object of struct `s`; fn(key) consumes a modelled member's value
  // (return false: the member is type-checked against the schema instead).
  template <class F>
  void obj(uint16_t s, F fn) {
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return;
    }
    if (k != JK::Obj) {
      bad();
      return;
    }
    c_.obj_begin();
    bool f = true;
    std::string_view key;
    std::string kscratch;
    while (c_.obj_next(f, &key, kscratch)) {
      std::string kk(key);  // stable copy (nested parsing reuses scratch buffers)
      if (!fn(std::string_view(kk))) member(s, kk);
    }
  }
  template <class F>
  bool arr(F fn) {  // returns false if null (caller clears)
    JK k = c_.peek();
    if (k == JK::Null) {
      c_.null();
      return false;
    }
    if (k != JK::Arr) {
      bad();
      return true;
    }
    c_.arr_begin();
    bool f = true;
    while (c_.arr_next(f)) fn();
    return true;
  }

  // ---- K8s types ----
  void object_meta(std::vector<std::pair<std::string, std::string>>* ann) {
    obj(sid("ObjectMeta"), [&](std::string_view k) {
      if (keq(k, "name") || keq(k, "generatename") || keq(k, "namespace") || keq(k, "uid") ||
          keq(k, "resourceversion") || keq(k, "selflink"))
        str(nullptr);
      else if (keq(k, "generation")) i64();
      else if (keq(k, "creationtimestamp") || keq(k, "deletiontimestamp")) timev();
      else if (keq(k, "labels")) strmap(nullptr);
      else if (keq(k, "annotations")) strmap(ann);
      else if (keq(k, "finalizers")) strlist(nullptr);
      else return false;
      return true;
    });
  }
  void selinux(bool* set, std::string* type, std::string* user, std::string* role) {
    if (c_.peek() == JK::Null) {
      c_.null();
      return;
    }
    if (c_.peek() == JK::Obj) *set = true;
    obj(sid("SELinuxOptions"), [&](std::string_view k) {
      if (keq(k, "user")) str(user);
      else if (keq(k, "role")) str(role);
      else if (keq(k, "type")) str(type);
      else if (keq(k, "level")) str(nullptr);
      else return false;
      return true;
    });
  }
  void seccomp(bool* set, std::string* type) {
    if (c_.peek() == JK::Null) {
      c_.null();
      return;
    }
    if (c_.peek() == JK::Obj) *set = true;
    obj(sid("SeccompProfile"), [&](std::string_view k) {
      if (keq(k, "type")) str(type);
      else if (keq(k, "localhostprofile")) strp(nullptr, nullptr);
      else return false;
      return true;
    });
  }
  void winopts(uint32_t* hp) {
    obj(sid("WindowsSecurityContextOptions"), [&](std::string_view k) {
      if (keq(k, "hostprocess")) tri(hp);
      else if (keq(k, "gmsacredentialspecname") || keq(k, "gmsacredentialspec") || keq(k, "runasusername"))
        strp(nullptr, nullptr);
      else return false;
      return true;
    });
  }
  void security_context(CtrView& c) {
    if (c_.peek() == JK::Null) {
      c_.null();
      return;
    }
    if (c_.peek() == JK::Obj) c.sc = true;
    obj(sid("SecurityContext"), [&](std::string_view k) {
      if (keq(k, "capabilities")) {
        if (c_.peek() == JK::Null) {
          c_.null();
          return true;
        }
        if (c_.peek() == JK::Obj) c.caps = true;
        obj(sid("Capabilities"), [&](std::string_view k2) {
          if (keq(k2, "add")) strlist(&c.add);
          else if (keq(k2, "drop")) strlist(&c.drop);
          else return false;
          return true;
        });
      } else if (keq(k, "privileged")) tri(&c.priv);
      else if (keq(k, "selinuxoptions")) selinux(&c.sel, &c.sel_type, &c.sel_user, &c.sel_role);
      else if (keq(k, "windowsoptions")) winopts(&c.whp);
      else if (keq(k, "runasuser")) {
        int64_t v;
        if (integer(INT64_MIN, INT64_MAX, &v)) c.rau = v == 0 ? RAU_ZERO : RAU_NONZERO;
      } else if (keq(k, "runasgroup")) i64();
      else if (keq(k, "runasnonroot")) tri(&c.rnr);
      else if (keq(k, "readonlyrootfilesystem")) tri(nullptr);
      else if (keq(k, "allowprivilegeescalation")) tri(&c.ape);
      else if (keq(k, "procmount")) strp(&c.pm, &c.pm_val);
      else if (keq(k, "seccompprofile")) seccomp(&c.sec, &c.sec_type);
      else return false;
      return true;
    });
  }
  void pod_security_context(PodView& p) {
    if (c_.peek() == JK::Null) {
      c_.null();
      return;
    }
    if (c_.peek() == JK::Obj) p.sc = true;
    obj(sid("PodSecurityContext"), [&](std::string_view k) {
      if (keq(k, "selinuxoptions")) selinux(&p.sel, &p.sel_type, &p.sel_user, &p.sel_role);
      else if (keq(k, "windowsoptions")) winopts(&p.whp);
      else if (keq(k, "runasuser")) {
        int64_t v;
        if (integer(INT64_MIN, INT64_MAX, &v)) p.rau = v == 0 ? RAU_ZERO : RAU_NONZERO;
      } else if (keq(k, "runasgroup") || keq(k, "fsgroup")) i64();
      else if (keq(k, "runasnonroot")) tri(&p.rnr);
      else if (keq(k, "supplementalgroups")) i64list();
      else if (keq(k, "fsgroupchangepolicy")) strp(nullptr, nullptr);
      else if (keq(k, "seccompprofile")) seccomp(&p.sec, &p.sec_type);
      else if (keq(k, "sysctls")) {
        std::vector<std::string> names;
        bool notnull = arr([&]() {
          std::string nm;
          if (c_.peek() == JK::Null) c_.null();
          else
            obj(sid("Sysctl"), [&](std::string_view k2) {
              if (keq(k2, "name")) str(&nm);
              else if (keq(k2, "value")) str(nullptr);
              else return false;
              return true;
            });
          names.push_back(nm);
        });
        p.sysctls = notnull ? names : std::vector<std::string>();
      } else return false;
      return true;
    });
  }
  void container(CtrView& c, uint16_t s) {
    if (c_.peek() == JK::Null) {
      c_.null();
      return;
    }
    obj(s, [&](std::string_view k) {
      if (keq(k, "name")) str(&c.name);
      else if (keq(k, "image")) str(&c.image);
      else if (keq(k, "command") || keq(k, "args")) strlist(nullptr);
      else if (keq(k, "workingdir") || keq(k, "imagepullpolicy") || keq(k, "terminationmessagepath") ||
               keq(k, "terminationmessagepolicy") || keq(k, "targetcontainername"))
        str(nullptr);
      else if (keq(k, "stdin") || keq(k, "stdinonce") || keq(k, "tty")) boolean(nullptr);
      else if (keq(k, "ports")) {
        std::vector<int32_t> hp;
        bool notnull = arr([&]() {
          int64_t h = 0;
          if (c_.peek() == JK::Null) c_.null();
          else
            obj(sid("ContainerPort"), [&](std::string_view k2) {
              if (keq(k2, "hostport")) integer(INT32_MIN, INT32_MAX, &h);
              else if (keq(k2, "containerport")) i32();
              else if (keq(k2, "name") || keq(k2, "protocol") || keq(k2, "hostip")) str(nullptr);
              else return false;
              return true;
            });
          hp.push_back((int32_t)h);
        });
        c.hostports = notnull ? hp : std::vector<int32_t>();
      } else if (keq(k, "env")) {
        arr([&]() {
          if (c_.peek() == JK::Null) {
            c_.null();
            return;
          }
          obj(sid("EnvVar"), [&](std::string_view k2) {
            if (keq(k2, "name") || keq(k2, "value")) str(nullptr);
            else return false;
            return true;
          });
        });
      } else if (keq(k, "securitycontext")) security_context(c);
      else return false;
      return true;
    });
  }
  void containers(std::vector<CtrView>& out, const char* type) {
    const uint16_t s = k8s::schema().struct_id(type);
    std::vector<CtrView> v;
    bool notnull = arr([&]() {
      CtrView c;
      container(c, s);
      v.push_back(std::move(c));
    });
    out = notnull ? std::move(v) : std::vector<CtrView>();
  }
  void volumes(std::vector<uint32_t>& out) {
    std::vector<uint32_t> v;
    const uint16_t vsid = sid("Volume");
    bool notnull = arr([&]() {
      uint32_t src = 0;
      if (c_.peek() == JK::Null) c_.null();
      else
        obj(vsid, [&](std::string_view k) {
          if (keq(k, "name")) {
            str(nullptr);
            return true;
          }
          for (int i = 0; i < KPE_NUM_VOLUME_SOURCES; ++i) {
            if (keq_n(k, kVolSrc[i], strlen(kVolSrc[i]))) {
              JK t = c_.peek();
              if (t == JK::Null) {
                c_.null();
                src &= ~(1u << i);
                return true;
              }
              if (t != JK::Obj) {
                bad();
                return true;
              }
              src |= 1u << i;
              member(vsid, k);  // the source struct, type-checked against the schema
              return true;
            }
          }
          return false;
        });
      v.push_back(src);
    });
    out = notnull ? std::move(v) : std::vector<uint32_t>();
  }
  void pod_spec(PodView& p) {
    obj(sid("PodSpec"), [&](std::string_view k) {
      if (keq(k, "volumes")) volumes(p.vols);
      else if (keq(k, "initcontainers")) containers(p.ctr[0], "Container");
      else if (keq(k, "containers")) containers(p.ctr[1], "Container");
      else if (keq(k, "ephemeralcontainers")) containers(p.ctr[2], "EphemeralContainer");
      else if (keq(k, "hostnetwork")) boolean(&p.hostnet);
      else if (keq(k, "hostpid")) boolean(&p.hostpid);
      else if (keq(k, "hostipc")) boolean(&p.hostipc);
      else if (keq(k, "securitycontext")) pod_security_context(p);
      else if (keq(k, "os")) {
        if (c_.peek() == JK::Null) {
          c_.null();
          return true;
        }
        if (c_.peek() == JK::Obj) p.os = true;
        obj(sid("PodOS"), [&](std::string_view k2) {
          if (keq(k2, "name")) str(&p.os_name);
          else return false;
          return true;
        });
      } else if (keq(k, "restartpolicy") || keq(k, "dnspolicy") || keq(k, "serviceaccountname") ||
                 keq(k, "serviceaccount") || keq(k, "nodename") || keq(k, "hostname") || keq(k, "subdomain") ||
                 keq(k, "priorityclassname") || keq(k, "schedulername"))
        str(nullptr);
      else if (keq(k, "terminationgraceperiodseconds") || keq(k, "activedeadlineseconds")) i64();
      else if (keq(k, "priority")) i32();
      else if (keq(k, "automountserviceaccounttoken") || keq(k, "shareprocessnamespace") || keq(k, "hostusers") ||
               keq(k, "enableservicelinks"))
        tri(nullptr);
      else if (keq(k, "runtimeclassname")) strp(nullptr, nullptr);
      else if (keq(k, "nodeselector")) strmap(nullptr);
      else return false;
      return true;
    });
  }
  void label_selector() {
    obj(sid("LabelSelector"), [&](std::string_view k) {
      if (keq(k, "matchlabels")) strmap(nullptr);
      else if (keq(k, "matchexpressions")) {
        arr([&]() {
          if (c_.peek() == JK::Null) {
            c_.null();
            return;
          }
          obj(sid("LabelSelectorRequirement"), [&](std::string_view k2) {
            if (keq(k2, "key") || keq(k2, "operator")) str(nullptr);
            else if (keq(k2, "values")) strlist(nullptr);
            else return false;
            return true;
          });
        });
      } else return false;
      return true;
    });
  }
  // PodTemplateSpec; `meta_ann` receives template annotations when non-null.
  void pod_template(PodView& p, bool take_meta) {
    obj(sid("PodTemplateSpec"), [&](std::string_view k) {
      if (keq(k, "metadata")) object_meta(take_meta ? &p.ann : nullptr);
      else if (keq(k, "spec")) pod_spec(p);
      else return false;
      return true;
    });
  }

  static bool rfc3339(std::string_view s) {
    auto d = [&](size_t i) { return i < s.size() && s[i] >= '0' && s[i] <= '9'; };
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

 private:
  JCur& c_;
  std::string vs_, ks_;
  void bad() {
    err = true;
    c_.skip();
  }
};

uint32_t class_of(const std::string& kind) {
  if (kind == "DaemonSet" || kind == "Deployment" || kind == "Job" || kind == "StatefulSet" ||
      kind == "ReplicaSet" || kind == "ReplicationController")
    return R_CLASS_CONTROLLER;
  if (kind == "CronJob") return R_CLASS_CRONJOB;
  if (kind == "Pod") return R_CLASS_POD;
  return R_CLASS_OTHER;
}

// Pre-scan: top-level "kind" string (exact key, unstructured semantics).
std::string top_kind(const char* p, const char* e) {
  JCur c(p, e);
  std::string out;
  if (!c.obj_begin()) return out;
  bool f = true;
  std::string_view k;
  std::string ks, vs;
  while (c.obj_next(f, &k, ks)) {
    if (k == "kind" && c.peek() == JK::Str) {
      std::string_view v;
      c.str(&v, vs);
      out.assign(v);
    } else {
      c.skip();
    }
  }
  return out;
}

uint32_t seccomp_code(bool set, const std::string& t) {
  if (!set) return SECCOMP_NONE;
  if (t == "RuntimeDefault") return SECCOMP_RUNTIMEDEFAULT;
  if (t == "Localhost") return SECCOMP_LOCALHOST;
  if (t == "Unconfined") return SECCOMP_UNCONFINED;
  return SECCOMP_OTHER;
}
uint32_t sel_code(bool set, const std::string& t) {
  if (!set) return SEL_NONE;
  if (t.empty()) return SEL_EMPTY;
  if (t == "container_t") return SEL_CONTAINER_T;
  if (t == "container_init_t") return SEL_CONTAINER_INIT_T;
  if (t == "container_kvm_t") return SEL_CONTAINER_KVM_T;
  return SEL_OTHER;
}

struct LimitError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct DepthError : LimitError {  // per resource (DocBuilder)
  using LimitError::LimitError;
};
struct NeedSequential {};  // a corpus-wide dictionary limit was crossed by the merge of parallel parts

class Flattener {
 public:
  explicit Flattener(Corpus& c) : C(c) {}
  // typed_pod_view: walk one resource without emitting a row
  bool no_emit = false, last_err = false;
  // without document tapes the images context is checked from the typed container images only
  // (GetImageInfo validity per distinct image string); with tapes DocBuilder checks it exactly
  bool check_images = false, bad_image = false;
  std::vector<int8_t> img_ok_;  // per D_IMAGE id: -1 unknown, 0 invalid, 1 valid / blank
  bool image_ok(uint32_t id) {
    if (id >= img_ok_.size()) img_ok_.resize(id + 1, -1);
    if (img_ok_[id] < 0) {
      const std::string_view im = C.dict[D_IMAGE].at(id);
      size_t a = 0;
      while (a < im.size() && (im[a] == ' ' || (im[a] >= '\t' && im[a] <= '\r'))) ++a;
      imageref::Info info;
      img_ok_[id] = (a == im.size() || imageref::image_info(im, &info)) ? 1 : 0;
    }
    return img_ok_[id] == 1;
  }
  uint32_t last_cls = R_CLASS_OTHER;
  const PodView& view() const { return pod; }

  void add(const char* p, const char* e) {
    // The class (typed decode target) needs the resource's last top-level "kind". When "kind"
    // leads the object (after an optional "apiVersion"), the walk starts with its class and
    // checks at the end that no later "kind" changed it (else it walks again); otherwise a
    // pre-scan of the top-level members finds it first.
    std::string kind;
    if (!lead_kind(p, e, &kind)) kind = top_kind(p, e);
    uint32_t cls = class_of(kind);
    if (!walk(p, e, cls) && walk(p, e, class_of(u.kind))) throw std::logic_error("resource class changed twice");
  }

 private:
  // the leading "kind" string member of the object (at most one "apiVersion" string before it)
  static bool lead_kind(const char* p, const char* e, std::string* kind) {
    JCur c(p, e);
    if (!c.obj_begin()) return false;
    bool f = true;
    std::string_view k;
    std::string ks, vs;
    for (int i = 0; i < 2 && c.obj_next(f, &k, ks); ++i) {
      if (c.peek() != JK::Str || (k != "kind" && k != "apiVersion")) return false;
      std::string_view v;
      if (!c.str(&v, vs)) return false;
      if (k == "kind") {
        kind->assign(v);
        return true;
      }
    }
    return false;
  }
  // one walk of the resource with class `cls`; false: the last top-level "kind" is of another
  // class (nothing was emitted)
  bool walk(const char* p, const char* e, uint32_t cls) {
    u.reset();
    pod.reset();
    JCur cur(p, e);
    Typed t(cur);
    bool typed = cls != R_CLASS_OTHER;
    // top-level walk: unstructured keys are exact; typed keys fold case
    if (!cur.obj_begin()) throw std::invalid_argument("resource is not a JSON object");
    bool f = true;
    std::string_view key;
    std::string ks;
    while (cur.obj_next(f, &key, ks)) {
      const std::string_view k = key;  // valid until the next member
      if (k == "kind" || k == "apiVersion") {
        if (cur.peek() == JK::Str) {
          std::string_view v;
          std::string sc;
          cur.str(&v, sc);
          (k == "kind" ? u.kind : u.api_version).assign(v);
        } else if (typed && cur.peek() != JK::Null) {
          t.err = true;  // typed struct field is a string
          cur.skip();
        } else {
          cur.skip();
        }
      } else if (keq(k, "kind") || keq(k, "apiversion")) {
        if (typed) t.str(nullptr);
        else cur.skip();
      } else if (keq(k, "metadata")) {
        meta(cur, t, k == "metadata", typed, cls == R_CLASS_POD);
      } else if (keq(k, "spec") && typed) {
        spec(t, cls);
      } else if (typed) {  // status and the rest: type-checked against the decode target
        t.member(cls == R_CLASS_POD ? sid("Pod") : cls == R_CLASS_CONTROLLER ? sid("Deployment") : sid("CronJob"), k);
      } else {
        cur.skip();
      }
    }
    if (!cur.ok()) throw std::invalid_argument("malformed resource JSON");
    if (class_of(u.kind) != cls) return false;
    if (no_emit) {
      last_cls = cls;
      last_err = typed && t.err;
      return true;
    }
    emit(cls, typed && t.err);
    return true;
  }

  Corpus& C;
  UView u;
  PodView pod;

  // metadata: unstructured (exact key "metadata") and/or typed ObjectMeta
  void meta(JCur& cur, Typed& t, bool exact, bool typed, bool pod_meta) {
    if (!exact) {  // only the typed decoder sees a case-variant key
      if (typed) t.object_meta(pod_meta ? &pod.ann : nullptr);
      else cur.skip();
      return;
    }
    JK k0 = cur.peek();
    if (k0 != JK::Obj) {
      if (typed && k0 != JK::Null) t.err = true;
      cur.skip();
      return;
    }
    cur.obj_begin();
    bool f = true;
    std::string_view key;
    std::string ks;
    while (cur.obj_next(f, &key, ks)) {
      const std::string_view k = key;  // valid until the next member
      // unstructured accessors
      if (k == "name" || k == "generateName" || k == "namespace") {
        if (cur.peek() == JK::Str) {
          std::string_view v;
          std::string sc;
          cur.str(&v, sc);
          std::string& dst = k == "name" ? u.name : (k == "namespace" ? u.ns : u.generate_name);
          dst.assign(v);
        } else {
          if (typed && cur.peek() != JK::Null) t.err = true;
          cur.skip();
        }
        continue;
      }
      if (k == "labels" || k == "annotations") {
        bool is_lab = k == "labels";
        auto& dst = is_lab ? u.labels : u.ann;
        bool& ok = is_lab ? u.labels_ok : u.ann_ok;
        dst.clear();
        JK kk = cur.peek();
        if (kk == JK::Null) {
          cur.null();
          ok = false;  // nil map
          if (!is_lab && pod_meta) pod.ann.clear();
          continue;
        }
        if (kk != JK::Obj) {
          ok = false;
          if (typed) t.err = true;
          cur.skip();
          continue;
        }
        cur.obj_begin();
        bool f2 = true;
        std::string_view k2;
        std::string ks2;
        std::vector<std::pair<std::string, std::string>> typed_ann;
        std::string vsc;
        while (cur.obj_next(f2, &k2, ks2)) {  // k2 stays valid until the next member
          if (cur.peek() == JK::Str) {
            std::string_view v;
            cur.str(&v, vsc);
            upsert(dst, k2, v);
            if (!is_lab) upsert(typed_ann, k2, v);  // the typed view is kept for annotations only
          } else if (cur.peek() == JK::Null) {
            cur.null();
            ok = false;  // NestedStringMap: non-string value => error => nil
            if (!is_lab) upsert(typed_ann, k2, std::string_view());
          } else {
            ok = false;
            if (typed) t.err = true;
            cur.skip();
          }
        }
        if (!ok) dst.clear();
        if (!is_lab && pod_meta) pod.ann = typed_ann;
        continue;
      }
      // typed-only ObjectMeta fields (case-insensitive); unknown keys skipped
      if (!typed) {
        cur.skip();
        continue;
      }
      if (keq(k, "name") || keq(k, "generatename") || keq(k, "namespace") || keq(k, "uid") ||
          keq(k, "resourceversion") || keq(k, "selflink"))
        t.str(nullptr);
      else if (keq(k, "generation")) t.i64();
      else if (keq(k, "creationtimestamp") || keq(k, "deletiontimestamp")) t.timev();
      else if (keq(k, "labels")) t.strmap(nullptr);
      else if (keq(k, "annotations")) t.strmap(pod_meta ? &pod.ann : nullptr);
      else if (keq(k, "finalizers")) t.strlist(nullptr);
      else t.member(sid("ObjectMeta"), k);
    }
  }
  static void upsert(std::vector<std::pair<std::string, std::string>>& v, std::string_view k, std::string_view val) {
    for (auto& e : v)
      if (e.first == k) {
        e.second.assign(val);
        return;
      }
    v.emplace_back(std::string(k), std::string(val));
  }

  void spec(Typed& t, uint32_t cls) {
    if (cls == R_CLASS_POD) {
      t.pod_spec(pod);
    } else if (cls == R_CLASS_CONTROLLER) {
      t.obj(sid("DeploymentSpec"), [&](std::string_view k) {
        if (keq(k, "replicas") || keq(k, "revisionhistorylimit") || keq(k, "progressdeadlineseconds") ||
            keq(k, "minreadyseconds"))
          t.i32();
        else if (keq(k, "paused")) t.boolean(nullptr);
        else if (keq(k, "selector")) t.label_selector();
        else if (keq(k, "template")) t.pod_template(pod, true);
        else return false;
        return true;
      });
    } else {  // CronJob
      t.obj(sid("CronJobSpec"), [&](std::string_view k) {
        if (keq(k, "schedule") || keq(k, "concurrencypolicy")) t.str(nullptr);
        else if (keq(k, "timezone")) t.strp(nullptr, nullptr);
        else if (keq(k, "startingdeadlineseconds")) t.i64();
        else if (keq(k, "suspend")) t.tri(nullptr);
        else if (keq(k, "successfuljobshistorylimit") || keq(k, "failedjobshistorylimit")) t.i32();
        else if (keq(k, "jobtemplate")) {
          t.obj(sid("JobTemplateSpec"), [&](std::string_view k3) {
            // validate_pss.go:165-166: metadata from spec.jobTemplate.metadata
            if (keq(k3, "metadata")) t.object_meta(&pod.ann);
            else if (keq(k3, "spec")) {
              t.obj(sid("JobSpec"), [&](std::string_view k4) {
                if (keq(k4, "parallelism") || keq(k4, "completions") || keq(k4, "backofflimit") ||
                    keq(k4, "ttlsecondsafterfinished"))
                  t.i32();
                else if (keq(k4, "activedeadlineseconds")) t.i64();
                else if (keq(k4, "selector")) t.label_selector();
                else if (keq(k4, "manualselector") || keq(k4, "suspend")) t.tri(nullptr);
                else if (keq(k4, "completionmode")) t.strp(nullptr, nullptr);
                else if (keq(k4, "template")) {
                  PodView tmp;
                  t.pod_template(tmp, false);
                  // only the spec is taken from the job's pod template
                  for (int i = 0; i < 3; ++i) pod.ctr[i] = std::move(tmp.ctr[i]);
                  pod.vols = std::move(tmp.vols);
                  pod.sysctls = std::move(tmp.sysctls);
                  pod.hostnet = tmp.hostnet;
                  pod.hostpid = tmp.hostpid;
                  pod.hostipc = tmp.hostipc;
                  pod.sc = tmp.sc;
                  pod.rnr = tmp.rnr;
                  pod.rau = tmp.rau;
                  pod.whp = tmp.whp;
                  pod.sec = tmp.sec;
                  pod.sec_type = tmp.sec_type;
                  pod.sel = tmp.sel;
                  pod.sel_type = tmp.sel_type;
                  pod.sel_user = tmp.sel_user;
                  pod.sel_role = tmp.sel_role;
                  pod.os = tmp.os;
                  pod.os_name = tmp.os_name;
                } else return false;
                return true;
              });
            } else return false;
            return true;
          });
        } else return false;
        return true;
      });
    }
  }

  uint32_t capmask(const std::vector<std::string>& l) {  // names are interned (limits checked first)
    uint64_t m = 0;
    for (auto& s : l) m |= 1ull << C.dict[D_CAP].intern(s);
    last_mask_ = m;
    return 0;
  }
  // Per-resource limits of the encoding: would this pod's containers push the capability
  // dictionary past 64 names or the capability-set dictionary past KPE_MAX_CAPSETS?
  bool caps_over_limit() {
    std::vector<std::string> fresh;
    for (auto& ct : pod.ctr)
      for (auto& c : ct)
        for (auto* l : {&c.add, &c.drop})
          for (auto& n : *l)
            if (C.dict[D_CAP].find(n) < 0 && std::find(fresh.begin(), fresh.end(), n) == fresh.end()) fresh.push_back(n);
    if (C.dict[D_CAP].size() + fresh.size() > 64) return true;
    std::vector<std::string> keys;
    for (auto& ct : pod.ctr)
      for (auto& c : ct) {
        uint64_t ad = 0, dr = 0;
        for (auto& n : c.add) ad |= 1ull << C.dict[D_CAP].intern(n);
        for (auto& n : c.drop) dr |= 1ull << C.dict[D_CAP].intern(n);
        std::string key(16, '\0');
        memcpy(&key[0], &ad, 8);
        memcpy(&key[8], &dr, 8);
        if (!C.capset_index.count(key) && std::find(keys.begin(), keys.end(), key) == keys.end()) keys.push_back(key);
      }
    return C.capset_add.size() + keys.size() > KPE_MAX_CAPSETS;
  }
  uint64_t last_mask_ = 0;

  void emit(uint32_t cls, bool derr) {
    if (C.n >= 0x7FFFFFC0) throw LimitError("more than 2^31 - 64 resources in one corpus (32-bit row ids)");
    // ---- resource row (unstructured view) ----
    std::string_view group, version;  // views into u.api_version
    const std::string_view av = u.api_version;
    const size_t sl = av.find('/');
    if (sl == std::string_view::npos) version = av;
    else {
      group = av.substr(0, sl);
      version = av.substr(sl + 1);
    }
    bool limit = false;  // a per-resource limit: the row is kept, its cells are undecided
    auto small_id = [&](int d, std::string_view v, uint32_t cap) -> uint32_t {
      const int64_t id = C.dict[d].find(v);
      if (id >= 0) return (uint32_t)id;
      if (C.dict[d].size() >= cap) return limit = true, 0u;
      return C.dict[d].intern(v);
    };
    const uint32_t kid = small_id(D_KIND, u.kind, 4096), vid = small_id(D_VERSION, version, 1024),
                   gid = small_id(D_GROUP, group, 1024);
    C.r_gvk.push_back(kid | (vid << 12) | (gid << 22));
    bool is_ns = u.kind == "Namespace";
    // ---- per-resource limits of the pod view ----
    const size_t nctr0 = pod.ctr[0].size() + pod.ctr[1].size() + pod.ctr[2].size();
    if (nctr0 > KPE_MAX_LIST || pod.vols.size() > KPE_MAX_LIST || pod.sysctls.size() > KPE_MAX_LIST ||
        pod.ann.size() > KPE_MAX_LIST || caps_over_limit()) {
      limit = true;
      pod.reset();
    }
    uint32_t flags = cls | (derr ? R_DECODE_ERR : 0u) | (is_ns ? R_IS_NAMESPACE : 0u) |
                     (u.labels_ok ? 0u : R_LABELS_NIL) | (u.ann_ok ? 0u : R_ANNOT_NIL) | (limit ? R_LIMIT : 0u);
    if (limit) C.limit_rows.push_back((uint32_t)C.n);
    C.r_flags.push_back(flags);
    C.r_name.push_back(C.dict[D_NAME].intern(u.name.empty() ? u.generate_name : u.name));
    uint32_t nsa = C.dict[D_NS].intern(u.ns);
    C.r_nsa.push_back(nsa);
    C.r_mns.push_back(is_ns ? C.dict[D_NS].intern(u.name) : nsa);
    auto it = C.nsl_index.find(u.ns);
    C.r_nsl.push_back(it == C.nsl_index.end() ? KPE_NO_STR : it->second);
    for (auto& kv : u.labels) {
      C.lab_k.push_back(C.dict[D_LABK].intern(kv.first));
      C.lab_v.push_back(C.dict[D_LABV].intern(kv.second));
    }
    C.lab_off.push_back((uint32_t)C.lab_k.size());
    for (auto& kv : u.ann) {
      C.ann_k.push_back(C.dict[D_ANNK].intern(kv.first));
      C.ann_v.push_back(C.dict[D_ANNV].intern(kv.second));
    }
    C.ann_off.push_back((uint32_t)C.ann_k.size());

    // ---- pod view ----
    const size_t nctr = pod.ctr[0].size() + pod.ctr[1].size() + pod.ctr[2].size();
    uint32_t p = 0;
    if (pod.sc) p |= P_SC_PRESENT;
    if (pod.hostnet) p |= P_HOSTNET;
    if (pod.hostpid) p |= P_HOSTPID;
    if (pod.hostipc) p |= P_HOSTIPC;
    p |= pod.rnr << P_RNR_SH;
    p |= pod.rau << P_RAU_SH;
    p |= seccomp_code(pod.sec, pod.sec_type) << P_SECCOMP_SH;
    p |= sel_code(pod.sel, pod.sel_type) << P_SEL_SH;
    if (pod.sel && !pod.sel_user.empty()) p |= P_SEL_USER;
    if (pod.sel && !pod.sel_role.empty()) p |= P_SEL_ROLE;
    p |= pod.whp << P_WHP_SH;
    p |= (pod.os ? (pod.os_name == "windows" ? OS_WINDOWS : OS_OTHER) : OS_NONE) << P_OS_SH;
    C.p_sc.push_back(p);
    C.p_cold.push_back(pod.sec ? C.dict[D_MISC].intern(pod.sec_type) : KPE_NO_STR);
    C.p_cold.push_back(pod.sel ? C.dict[D_MISC].intern(pod.sel_type) : KPE_NO_STR);
    C.p_cold.push_back(pod.sel ? C.dict[D_MISC].intern(pod.sel_user) : KPE_NO_STR);
    C.p_cold.push_back(pod.sel ? C.dict[D_MISC].intern(pod.sel_role) : KPE_NO_STR);
    for (uint32_t v : pod.vols) C.vol_src.push_back(v);
    C.vol_off.push_back((uint32_t)C.vol_src.size());
    for (auto& s : pod.sysctls) C.sys_id.push_back(C.dict[D_SYSCTL].intern(s));
    C.sys_off.push_back((uint32_t)C.sys_id.size());
    for (auto& kv : pod.ann) {
      C.pann_k.push_back(C.dict[D_ANNK].intern(kv.first));
      C.pann_v.push_back(C.dict[D_ANNV].intern(kv.second));
      C.pann_kv.push_back(C.pann_k.back());
      C.pann_kv.push_back(C.pann_v.back());
    }
    C.pann_off.push_back((uint32_t)C.pann_k.size());
    static const std::string seccomp_ctr_prefix = "container.seccomp.security.alpha.kubernetes.io/";
    for (uint32_t ct = 0; ct < 3; ++ct) {
      for (auto& c : pod.ctr[ct]) {
        uint32_t w = 0;
        if (c.sc) w |= C_SC_PRESENT;
        w |= c.priv << C_PRIV_SH;
        w |= c.ape << C_APE_SH;
        w |= c.rnr << C_RNR_SH;
        w |= c.rau << C_RAU_SH;
        w |= seccomp_code(c.sec, c.sec_type) << C_SECCOMP_SH;
        w |= (c.pm ? (c.pm_val == "Default" ? PROCMOUNT_DEFAULT : PROCMOUNT_OTHER) : PROCMOUNT_UNSET)
             << C_PROCMOUNT_SH;
        w |= sel_code(c.sel, c.sel_type) << C_SEL_SH;
        if (c.sel && !c.sel_user.empty()) w |= C_SEL_USER;
        if (c.sel && !c.sel_role.empty()) w |= C_SEL_ROLE;
        w |= c.whp << C_WHP_SH;
        if (c.caps) w |= C_CAPS_PRESENT;
        w |= ct << C_TYPE_SH;
        uint32_t nz = 0;
        for (int32_t h : c.hostports)
          if (h != 0) ++nz;
        w |= std::min(nz, 15u) << C_HOSTPORT_SH;
        C.c_sc.push_back(w);
        capmask(c.add);
        C.c_add.push_back(last_mask_);
        capmask(c.drop);
        C.c_drop.push_back(last_mask_);
        {  // capability-set dictionary: distinct (add, drop) mask pairs
          std::string key(16, '\0');
          memcpy(&key[0], &C.c_add.back(), 8);
          memcpy(&key[8], &C.c_drop.back(), 8);
          auto it = C.capset_index.find(key);
          uint32_t cs;
          if (it == C.capset_index.end()) {
            cs = (uint32_t)C.capset_add.size();  // < KPE_MAX_CAPSETS (caps_over_limit)
            C.capset_index.emplace(key, cs);
            C.capset_add.push_back(C.c_add.back());
            C.capset_drop.push_back(C.c_drop.back());
          } else {
            cs = it->second;
          }
          C.crec.push_back(state_bitmap(w));
          C.crec.push_back(cs | (ct << 16));
        }
        C.c_name.push_back(C.dict[D_CNAME].intern(c.name));
        C.c_image.push_back(C.dict[D_IMAGE].intern(c.image));
        if (check_images && !image_ok(C.c_image.back())) bad_image = true;
        uint32_t sann = KPE_NO_STR, sann_key = KPE_NO_STR;  // join: "container.seccomp...kubernetes.io/<name>"
        if (!pod.ann.empty()) {
          std::string key = seccomp_ctr_prefix + c.name;
          for (auto& kv : pod.ann)
            if (kv.first == key) sann = C.dict[D_ANNV].intern(kv.second), sann_key = C.dict[D_ANNK].intern(kv.first);
        }
        C.c_sann.push_back(sann);
        C.c_sann_key.push_back(sann_key);
        C.c_sec_str.push_back(c.sec ? C.dict[D_MISC].intern(c.sec_type) : KPE_NO_STR);
        C.c_pm_str.push_back(c.pm ? C.dict[D_MISC].intern(c.pm_val) : KPE_NO_STR);
        C.c_selt_str.push_back(c.sel ? C.dict[D_MISC].intern(c.sel_type) : KPE_NO_STR);
        C.c_selu_str.push_back(c.sel ? C.dict[D_MISC].intern(c.sel_user) : KPE_NO_STR);
        C.c_selr_str.push_back(c.sel ? C.dict[D_MISC].intern(c.sel_role) : KPE_NO_STR);
        for (int32_t h : c.hostports) {
          C.cport_host.push_back(h);
          C.cport_str.push_back(h ? C.dict[D_MISC].intern(std::to_string(h)) : KPE_NO_STR);
        }
        C.cport_off.push_back((uint32_t)C.cport_host.size());
      }
    }
    C.ctr_off.push_back((uint32_t)C.c_sc.size());
    if (bad_image && !limit) {  // NewPolicyContext's AddImageInfos fails: no response at all
      C.r_flags.back() |= R_CTX_ERR;
      C.limit_rows.push_back((uint32_t)C.n);
    }
    bad_image = false;
    C.rec.push_back(p | ((flags & R_CLASS_MASK) << PR_CLASS_SH) | (derr ? PR_DECODE_ERR : 0u));
    C.rec.push_back(C.r_gvk.back());
    C.rec.push_back((uint32_t)nctr | ((uint32_t)pod.vols.size() << 8) | ((uint32_t)pod.sysctls.size() << 16) |
                    ((uint32_t)pod.ann.size() << 24));
    C.rec.push_back(nsa);
    C.n++;
  }
};

// ---- generic document tape (pattern rules) --------------------------------------------
// Scalar attributes (schema.h KpeScalar) from the value's text forms; see goval.hpp.
void scalar_attrs(KpeScalar& e, std::string_view numstr) {
  int64_t d;
  if (goval::parse_duration(numstr, &d)) e.flags |= SC_DUR, e.dur = d;
  goval::Quantity q;
  if (goval::parse_quantity(numstr, &q)) {
    e.flags |= SC_QTY | (q.neg ? SC_QNEG : 0u);
    goval::qty_key(q, &e.qexp, &e.qlo, &e.qhi);
  }
}

void spq(KpeScalar& e, const std::string& sprint) {
  if (goval::sprint_qty_same(sprint, e.flags & SC_QTY, e.flags & SC_QNEG, e.qexp, e.qlo, e.qhi)) e.flags |= SC_SPQ;
}

class DocBuilder {
 public:
  explicit DocBuilder(Corpus& c) : C(c) {
    if (C.scal.empty()) {  // fixed entries: null, false, true
      KpeScalar n{}, f{}, t{};
      n.flags = SC_T_NULL;
      scalar_attrs(n, "0");  // convertNumberToString(nil) == "0"
      f.flags = SC_T_BOOL | SC_TEXT;
      t.flags = SC_T_BOOL | SC_TEXT | SC_BTRUE;
      f.text_off = text("false"), f.text_len = 5;
      t.text_off = text("true"), t.text_len = 4;
      C.scal = {n, f, t};
    }
  }
  void add(const char* b, const char* e) {
    JCur c(b, e);
    uint64_t root;
    const size_t at = C.doc.size();
    try {
      root = value(c, 0, 0);
      if (!c.ok()) throw std::invalid_argument("malformed resource JSON");
    } catch (const DepthError&) {  // a per-resource limit: null document, the row's cells undecided
      C.doc.resize(at);  // drop the bodies of the partial walk
      root = entry(DN_SCALAR, 0, SC_NULL_ID);
      const uint32_t row = (uint32_t)(C.n - 1);
      C.r_flags[row] |= R_LIMIT;
      if (C.limit_rows.empty() || C.limit_rows.back() != row) C.limit_rows.push_back(row);
    }
    put(root);
    C.doc_off.push_back(C.doc.size() / 2 - 1);  // the resource's root entry
    C.img_off.push_back(KPE_NO_IMAGES);
    const uint32_t row = (uint32_t)(C.n - 1);
    if (!(C.r_flags[row] & R_LIMIT) && DN_KIND((uint32_t)root) == DN_MAP) {
      try {
        images((uint32_t)(C.doc.size() / 2 - 1));
      } catch (const ImageError&) {  // NewPolicyContext fails: no response for any rule
        if (!(C.r_flags[row] & R_CTX_ERR)) {  // the pod-column pass may have flagged the row already
          C.r_flags[row] |= R_CTX_ERR;
          if (C.limit_rows.empty() || C.limit_rows.back() != row) C.limit_rows.push_back(row);
        }
      }
    }
  }

 private:
  Corpus& C;
  std::string scratch;
  uint32_t text(std::string_view t) {
    const size_t off = C.scal_text.size();
    if (off + t.size() > 0xFFFFFFFFull) throw LimitError("scalar text pool exceeds 4 GiB");
    C.scal_text.insert(C.scal_text.end(), t.begin(), t.end());
    return (uint32_t)off;
  }
  uint32_t push_scalar(KpeScalar e) {
    if (C.scal.size() >= 0xFFFFFFFFull) throw LimitError("too many distinct scalars");
    C.scal.push_back(e);
    return (uint32_t)(C.scal.size() - 1);
  }
  uint32_t int_id(int64_t v) {
    auto it = C.scal_int.find(v);
    if (it != C.scal_int.end()) return it->second;
    KpeScalar e{};
    e.flags = SC_T_INT | SC_TEXT;
    e.ival = v;
    const std::string t = std::to_string(v);
    e.text_off = text(t), e.text_len = (uint32_t)t.size();
    const std::string sp = goval::sprint_float((double)v);  // condition context numbers are float64
    text(sp), e.sp_len = (uint32_t)sp.size();
    scalar_attrs(e, t);
    spq(e, sp);
    return C.scal_int[v] = push_scalar(e);
  }
  uint32_t float_id(double v) {
    uint64_t bits;
    memcpy(&bits, &v, 8);
    auto it = C.scal_float.find(bits);
    if (it != C.scal_float.end()) return it->second;
    KpeScalar e{};
    e.flags = SC_T_FLOAT | SC_TEXT;
    e.fval = v;
    const std::string t = goval::fmt_E(v);
    e.text_off = text(t), e.text_len = (uint32_t)t.size();
    const std::string sp = goval::sprint_float(v);
    text(sp), e.sp_len = (uint32_t)sp.size();
    scalar_attrs(e, goval::fmt_f(v));
    spq(e, sp);
    return C.scal_float[bits] = push_scalar(e);
  }
  uint32_t str_id(std::string_view v) {
    const uint64_t h = StrIndex::hash(v);
    const int64_t found = C.scal_str.find(v, h, [&](uint32_t id) { return C.scal_text_of(id); });
    if (found >= 0) return (uint32_t)found;
    KpeScalar e{};
    e.flags = SC_T_STR | SC_TEXT;
    e.text_off = text(v), e.text_len = (uint32_t)v.size();
    int64_t i;
    double f;
    if (goval::parse_int(v, &i)) e.flags |= SC_PINT, e.ival = i;
    if (goval::parse_float(v, &f)) e.flags |= SC_PFLOAT, e.fval = f;
    scalar_attrs(e, v);
    json_attrs(e, v);
    if (goval::pattern_simple(v)) e.flags |= SC_PSIMPLE;
    if (e.flags & SC_RANGE) {  // endpoints of the InRange form: their duration / quantity parses
      size_t at = 0;
      goval::range_split(v, "-", &at);
      if (v.find('|') != std::string_view::npos) {
        e.flags = (e.flags & ~SC_RANGE) | SC_RANGEU;  // validateStringPatterns splits on `|` first
      } else {
        const uint32_t lo = str_id(v.substr(0, at)), hi = str_id(v.substr(at + 1));
        e.ival = (int64_t)((uint64_t)lo | ((uint64_t)hi << 32));
      }
    }
    const uint32_t id = push_scalar(e);
    C.scal_str.insert(h, id);
    return id;
  }
  // What the condition set operators read from a string value (anyin.go:73-93): json.Valid
  // (and whether it is an array) and the InRange form
  static void json_attrs(KpeScalar& e, std::string_view v) {
    if (goval::in_range_form(v)) e.flags |= SC_RANGE;
    size_t i = 0;
    while (i < v.size() && (v[i] == ' ' || v[i] == '\t' || v[i] == '\n' || v[i] == '\r')) ++i;
    if (i == v.size()) return;
    const char c = v[i];
    if (!(c == '[' || c == '{' || c == '"' || c == '-' || (c >= '0' && c <= '9') || c == 't' || c == 'f' || c == 'n'))
      return;  // no JSON value starts here
    JCur jc(v.data(), v.data() + v.size());
    jc.ws();
    if (!jc.skip()) return;
    jc.ws();
    if (!jc.ok() || jc.pos() != v.data() + v.size()) return;
    e.flags |= SC_JVALID | (c == '[' ? SC_JARR : 0u);
  }
  // ---- the `images` context (context.go:306-348, pkg/utils/api/image.go:17-229) ----------
  struct ImageError {};
  uint32_t key1(const char* k) { return C.dict[D_KEY].intern(k) + 1u; }
  uint64_t at(uint32_t e) const { return (uint64_t)C.doc[(size_t)e * 2] | ((uint64_t)C.doc[(size_t)e * 2 + 1] << 32); }
  // member `k` of map entry e (the tape keeps the last of duplicate names), or ~0u
  uint32_t member(uint32_t e, uint32_t k1) const {
    const uint32_t b = C.doc[(size_t)e * 2 + 1], n = C.doc[(size_t)b * 2];
    for (uint32_t i = 0; i < n; ++i)
      if (DN_KEY(C.doc[(size_t)(b + 1 + i) * 2]) == k1) return b + 1 + i;
    return ~0u;
  }
  bool is_null(uint32_t e) const {
    const uint32_t x = C.doc[(size_t)e * 2];
    return DN_KIND(x) == DN_SCALAR && C.doc[(size_t)e * 2 + 1] == SC_NULL_ID;
  }
  // a string scalar's text, or false
  bool text(uint32_t e, std::string_view* out) const {
    const uint32_t x = C.doc[(size_t)e * 2];
    if (DN_KIND(x) != DN_SCALAR) return false;
    const KpeScalar& sc = C.scal[C.doc[(size_t)e * 2 + 1]];
    if (SC_TYPE(sc.flags) != SC_T_STR) return false;
    *out = std::string_view(C.scal_text.data() + sc.text_off, sc.text_len);
    return true;
  }
  void images(uint32_t root) {
    // ExtractImagesFromResource: the standard extractors of the resource's kind
    std::string_view kind;
    const uint32_t ke = member(root, key1("kind"));
    if (ke == ~0u || !text(ke, &kind)) return;
    std::vector<const char*> prefix;
    if (kind == "Pod") prefix = {"spec"};
    else if (kind == "DaemonSet" || kind == "Deployment" || kind == "ReplicaSet" || kind == "ReplicationController" ||
             kind == "StatefulSet" || kind == "Job")
      prefix = {"spec", "template", "spec"};
    else if (kind == "CronJob") prefix = {"spec", "jobTemplate", "spec", "template", "spec"};
    else return;
    uint32_t obj = root;
    std::string path;
    for (const char* f : prefix) {  // extract(): a nil value ends the walk, a non-map is an error
      if (DN_KIND(C.doc[(size_t)obj * 2]) != DN_MAP) throw ImageError{};
      const uint32_t c = member(obj, key1(f));
      path += "/";
      path += f;
      if (c == ~0u || is_null(c)) return;
      obj = c;
    }
    if (DN_KIND(C.doc[(size_t)obj * 2]) != DN_MAP) throw ImageError{};
    struct One {
      std::string name, pointer;
      imageref::Info info;
    };
    std::vector<std::pair<std::string, std::vector<One>>> types;
    for (const char* tag : {"containers", "ephemeralContainers", "initContainers"}) {  // JSON key order
      const uint32_t lst = member(obj, key1(tag));
      if (lst == ~0u || is_null(lst)) continue;
      const uint32_t lx = C.doc[(size_t)lst * 2];
      if (DN_KIND(lx) == DN_SCALAR) throw ImageError{};  // `*` over a scalar: "invalid type"
      const uint32_t b = C.doc[(size_t)lst * 2 + 1], n = C.doc[(size_t)b * 2];
      std::vector<One> got;
      std::vector<std::pair<std::string, uint32_t>> elems;  // (path element, entry)
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t e = b + 1 + i;
        if (DN_KIND(lx) == DN_ARR) elems.push_back({std::to_string(i), e});
        else elems.push_back({std::string(C.dict[D_KEY].at(DN_KEY(C.doc[(size_t)e * 2]) - 1)), e});
      }
      if (DN_KIND(lx) == DN_MAP) std::sort(elems.begin(), elems.end());  // Go map order: unpinned
      for (auto& el : elems) {
        const uint32_t e = el.second;
        if (is_null(e)) continue;
        if (DN_KIND(C.doc[(size_t)e * 2]) != DN_MAP) throw ImageError{};  // "invalid image config"
        std::string_view nm, im;
        const uint32_t ne = member(e, key1("name"));
        if (ne == ~0u || !text(ne, &nm)) throw ImageError{};  // "invalid key"
        const uint32_t ie = member(e, key1("image"));
        if (ie == ~0u || !text(ie, &im)) continue;
        size_t a = 0, z = im.size();
        while (a < z && (im[a] == ' ' || (im[a] >= '\t' && im[a] <= '\r'))) ++a;
        if (a == z) continue;  // strings.TrimSpace(value) == "": the image is not present
        One o;
        if (!imageref::image_info(im, &o.info)) throw ImageError{};  // "invalid image"
        o.name.assign(nm);
        o.pointer = path + "/" + tag + "/" + el.first + "/image";
        got.push_back(std::move(o));
      }
      if (got.empty()) continue;
      // a map keyed by container name (the last one wins), marshalled with sorted keys
      std::stable_sort(got.begin(), got.end(), [](const One& x, const One& y) { return x.name < y.name; });
      std::vector<One> uniq;
      for (size_t q = 0; q < got.size(); ++q)
        if (q + 1 == got.size() || got[q + 1].name != got[q].name) uniq.push_back(std::move(got[q]));
      types.push_back({tag, std::move(uniq)});
    }
    if (types.empty()) return;
    std::vector<uint64_t> tkids;
    for (auto& t : types) {
      std::vector<uint64_t> ckids;
      for (auto& o : t.second) {
        const imageref::Info& in = o.info;
        const std::string base = (in.registry.empty() ? "" : in.registry + "/") + in.path;
        const std::string reference = in.digest.empty() ? base + ":" + in.tag : base + "@" + in.digest;
        const std::string rwt = base + ":" + in.tag;
        std::vector<uint64_t> f;
        auto put_str = [&](const char* k, const std::string& v, bool omitempty) {
          if (omitempty && v.empty()) return;
          f.push_back(entry(DN_SCALAR, key1(k), str_id(v)));
        };
        put_str("digest", in.digest, true);
        put_str("jsonPointer", o.pointer, false);
        put_str("name", in.name, false);
        put_str("path", in.path, false);
        put_str("reference", reference, true);
        put_str("referenceWithTag", rwt, true);
        put_str("registry", in.registry, true);
        put_str("tag", in.tag, true);
        ckids.push_back(entry(DN_MAP, C.dict[D_KEY].intern(o.name) + 1u, body(f)));
      }
      tkids.push_back(entry(DN_MAP, key1(t.first.c_str()), body(ckids)));
    }
    put(entry(DN_MAP, 0, body(tkids)));
    C.img_off.back() = C.doc.size() / 2 - 1;
  }
  static uint64_t entry(uint32_t kind, uint32_t key1, uint32_t y) {
    return (uint64_t)(kind | (key1 << 2)) | ((uint64_t)y << 32);
  }
  void put(uint64_t en) {
    C.doc.push_back((uint32_t)en);
    C.doc.push_back((uint32_t)(en >> 32));
  }
  // A container's body: {count, 0} then its member / element entries, contiguous, so a
  // member lookup reads one short run of independent entries (schema.h DN_*).
  uint32_t body(std::vector<uint64_t>& kids) {
    const size_t at = C.doc.size() / 2;
    if (at + 1 + kids.size() > 0xFFFFFFFFull) throw LimitError("document tape exceeds 2^32 entries");
    put((uint64_t)kids.size());
    for (uint64_t en : kids) put(en);
    return (uint32_t)at;
  }
  uint64_t value(JCur& c, uint32_t key1, int depth) {
    if (depth > 256) throw DepthError("document nesting deeper than 256");
    switch (c.peek()) {
      case JK::Null: c.null(); return entry(DN_SCALAR, key1, SC_NULL_ID);
      case JK::Bool: {
        bool b = false;
        c.boolean(&b);
        return entry(DN_SCALAR, key1, b ? SC_TRUE_ID : SC_FALSE_ID);
      }
      case JK::Num: {
        JNum n;
        c.number(&n);
        return entry(DN_SCALAR, key1, n.is_int ? int_id(n.i) : float_id(n.f));
      }
      case JK::Str: {
        std::string_view v;
        c.str(&v, scratch);
        return entry(DN_SCALAR, key1, str_id(v));
      }
      case JK::Obj: {
        c.obj_begin();
        bool f = true;
        std::string_view k;
        std::string ks;
        std::vector<uint64_t> kids;
        bool dup = false;
        while (c.obj_next(f, &k, ks)) {
          const uint32_t kid = C.dict[D_KEY].intern(k);
          if (kid >= DN_MAX_KEYS) throw LimitError("too many distinct member names");
          const uint64_t en = value(c, kid + 1, depth + 1);
          for (size_t q = 0; q < kids.size() && !dup && kids.size() < 64; ++q)
            dup = DN_KEY((uint32_t)kids[q]) == kid + 1;
          kids.push_back(en);
        }
        if (kids.size() >= 64 && !dup) {
          std::vector<uint32_t> names;
          for (uint64_t en : kids) names.push_back(DN_KEY((uint32_t)en));
          std::sort(names.begin(), names.end());
          dup = std::adjacent_find(names.begin(), names.end()) != names.end();
        }
        if (dup) {  // duplicate names: a Go map decode keeps the last one
          std::unordered_map<uint32_t, size_t> last;
          for (size_t q = 0; q < kids.size(); ++q) last[DN_KEY((uint32_t)kids[q])] = q;
          std::vector<uint64_t> kept;
          for (size_t q = 0; q < kids.size(); ++q)
            if (last[DN_KEY((uint32_t)kids[q])] == q) kept.push_back(kids[q]);
          kids.swap(kept);
        }
        return entry(DN_MAP, key1, body(kids));
      }
      case JK::Arr: {
        c.arr_begin();
        bool f = true;
        std::vector<uint64_t> kids;
        while (c.arr_next(f)) kids.push_back(value(c, 0, depth + 1));
        return entry(DN_ARR, key1, body(kids));
      }
      default: throw std::invalid_argument("malformed resource JSON");
    }
  }
};

void load_ns_labels(Corpus& C, const char* js, size_t len) {
  if (!js || !len) return;
  JCur c(js, js + len);
  if (c.peek() == JK::Null) return;
  if (!c.obj_begin()) throw std::invalid_argument("ns_labels_json must be an object");
  bool f = true;
  std::string_view k;
  std::string ks, vs;
  while (c.obj_next(f, &k, ks)) {
    std::string ns(k);
    uint32_t idx = (uint32_t)(C.nsl_off.size() - 1);
    if (c.peek() == JK::Obj) {
      c.obj_begin();
      bool f2 = true;
      std::string_view k2;
      std::string ks2;
      while (c.obj_next(f2, &k2, ks2)) {
        std::string lk(k2);
        if (c.peek() == JK::Str) {
          std::string_view v;
          c.str(&v, vs);
          C.nsl_k.push_back(C.dict[D_LABK].intern(lk));
          C.nsl_v.push_back(C.dict[D_LABV].intern(v));
        } else {
          c.skip();
        }
      }
    } else {
      c.skip();
    }
    C.nsl_off.push_back((uint32_t)C.nsl_k.size());
    C.nsl_index[ns] = idx;
  }
  if (!c.ok()) throw std::invalid_argument("malformed ns_labels_json");
}

}  // namespace

bool typed_pod_view(const char* json, size_t len, PodView* out, std::string* kind) {
  Corpus scratch;
  Flattener f(scratch);
  f.no_emit = true;
  if (kind) *kind = top_kind(json, json + len);
  try {
    f.add(json, json + len);
  } catch (const std::exception&) {
    return false;
  }
  if (f.last_cls == R_CLASS_OTHER || f.last_err) return false;
  *out = f.view();
  return true;
}

int64_t Corpus::bytes() const {
  int64_t b = 0;
  auto add = [&](const auto& v) { b += (int64_t)(v.size() * sizeof(v[0])); };
  add(r_flags), add(r_gvk), add(r_name), add(r_mns), add(r_nsa), add(r_nsl);
  add(lab_off), add(lab_k), add(lab_v), add(ann_off), add(ann_k), add(ann_v);
  add(rec), add(hdr), add(crec), add(vol_src), add(sys_id), add(pann_kv), add(capset_add), add(capset_drop);
  add(c_sann);
  add(doc), add(doc_off), add(img_off), add(scal), add(scal_text);
  return b;
}

namespace {

void flatten_range(Corpus& C, const char* buf, size_t i, size_t len, bool docs) {
  // resource names are mostly distinct: size their dictionary for the range up front (one row per
  // ~400 bytes at most), so it does not rehash every name at each doubling
  if (C.dict[D_NAME].size() == 0) C.dict[D_NAME].reserve(std::min<size_t>((len - i) / 400 + 64, (size_t)1 << 24));
  Flattener fl(C);
  fl.check_images = !docs;
  std::unique_ptr<DocBuilder> db;
  if (docs) db = std::make_unique<DocBuilder>(C), C.has_docs = true;
  while (i < len) {
    const void* nl = memchr(buf + i, '\n', len - i);
    const size_t j = nl ? (size_t)(static_cast<const char*>(nl) - buf) : len;
    size_t a = i, b = j;
    while (a < b && (buf[a] == ' ' || buf[a] == '\t' || buf[a] == '\r')) ++a;
    while (b > a && (buf[b - 1] == ' ' || buf[b - 1] == '\t' || buf[b - 1] == '\r')) --b;
    if (b > a) {
      fl.add(buf + a, buf + b);
      if (db) db->add(buf + a, buf + b);
    }
    i = j + 1;
  }
}

// wave headers (schema.h): list bases of every 64-row tile, plus the sentinel
void rebuild_headers(Corpus& C) {
  C.hdr.clear();
  for (int64_t r = 0; r < C.n; r += 64) {
    C.hdr.push_back(C.ctr_off[r]), C.hdr.push_back(C.vol_off[r]);
    C.hdr.push_back(C.sys_off[r]), C.hdr.push_back(C.pann_off[r]);
  }
  C.hdr.push_back((uint32_t)C.c_sc.size());
  C.hdr.push_back((uint32_t)C.vol_src.size());
  C.hdr.push_back((uint32_t)C.sys_id.size());
  C.hdr.push_back((uint32_t)(C.pann_kv.size() / 2));
}

unsigned flatten_threads();

template <class T>
void grow(std::vector<T>& v, size_t n) {
  v.resize(v.size() + n);
}

// f(i) for i in [0, n) on up to nth threads (dynamic assignment)
template <class F>
void parallel_for(size_t n, unsigned nth, F f) {
  const unsigned T = (unsigned)std::min<size_t>(n, std::max(1u, nth));
  if (T <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> err(T);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      try {
        for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
      } catch (...) {
        err[t] = std::current_exception();
        next = n;  // the others stop at their next item
      }
    });
  for (auto& x : th) x.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// Dictionary domain d of every part merged into G in document order on up to nth threads, with
// the ids a sequential merge (G.intern of each part's strings in order) gives: a string's id is
// its first occurrence's rank. Strings are hash-partitioned into buckets, each bucket's thread
// finds every string's first occurrence (or its id in G) walking the parts in order; the parts
// then number their first occurrences in local order after G's size plus the earlier parts'
// counts, references take their first occurrence's id, the bytes are appended per part, and the
// index is rebuilt in parallel (Dict::reindex). dmap[t][d][i]: G id of part t's string i.
void merge_dict_parallel(Dict& G, std::vector<Corpus>& parts, int d,
                         std::vector<std::vector<std::vector<uint32_t>>>& dmap, unsigned nth) {
  const size_t T = parts.size();
  constexpr uint32_t kB = 64, kFirst = 0xFFFFFFFEu, kRef = 0xFFFFFFFDu;
  std::vector<std::vector<uint64_t>> hs(T), ref(T);
  std::vector<std::vector<std::vector<uint32_t>>> lists(T, std::vector<std::vector<uint32_t>>(kB));
  parallel_for(T, nth, [&](size_t t) {
    const Dict& D = parts[t].dict[d];
    hs[t].resize(D.size());
    ref[t].assign(D.size(), ~0ull);
    dmap[t][d].assign(D.size(), kFirst);
    for (uint32_t i = 0; i < D.size(); ++i) {
      const uint64_t h = Dict::hash(D.at(i));
      hs[t][i] = h;
      lists[t][h >> 58].push_back(i);
    }
  });
  const bool gempty = G.size() == 0;
  parallel_for(kB, nth, [&](size_t b) {
    size_t n = 0;
    for (size_t t = 0; t < T; ++t) n += lists[t][b].size();
    size_t cap = 16;
    while (cap < n * 2) cap *= 2;
    std::vector<uint64_t> tab(cap, ~0ull);  // first occurrences: t << 32 | i
    const size_t mask = cap - 1;
    for (size_t t = 0; t < T; ++t) {
      const Dict& D = parts[t].dict[d];
      for (uint32_t i : lists[t][b]) {
        const std::string_view sv = D.at(i);
        const uint64_t h = hs[t][i];
        if (!gempty) {
          const int64_t g = G.find_h(sv, h);
          if (g >= 0) {
            dmap[t][d][i] = (uint32_t)g;
            continue;
          }
        }
        for (size_t k = h & mask;; k = (k + 1) & mask) {
          const uint64_t e = tab[k];
          if (e == ~0ull) {
            tab[k] = (uint64_t)t << 32 | i;  // dmap stays kFirst
            break;
          }
          const size_t t0 = (size_t)(e >> 32);
          const uint32_t i0 = (uint32_t)e;
          if (hs[t0][i0] == h && parts[t0].dict[d].at(i0) == sv) {
            ref[t][i] = e;
            dmap[t][d][i] = kRef;
            break;
          }
        }
      }
    }
  });
  // first occurrences per part -> ids; their bytes
  std::vector<size_t> nf(T, 0), nb(T, 0);
  std::vector<std::vector<uint8_t>> first(T);
  parallel_for(T, nth, [&](size_t t) {
    const Dict& D = parts[t].dict[d];
    first[t].assign(D.size(), 0);
    for (uint32_t i = 0; i < D.size(); ++i)
      if (dmap[t][d][i] == kFirst) first[t][i] = 1, ++nf[t], nb[t] += D.at(i).size();
  });
  const uint32_t g0 = G.size();
  std::vector<size_t> idb(T + 1, g0), byb(T + 1, G.bytes.size());
  for (size_t t = 0; t < T; ++t) idb[t + 1] = idb[t] + nf[t], byb[t + 1] = byb[t] + nb[t];
  if (byb[T] > 0xFFFFFFFFull) throw LimitError("a dictionary's text exceeds 4 GiB");
  G.bytes.resize(byb[T]);
  G.off.resize(idb[T] + 1);
  parallel_for(T, nth, [&](size_t t) {
    const Dict& D = parts[t].dict[d];
    uint32_t id = (uint32_t)idb[t];
    size_t pos = byb[t];
    for (uint32_t i = 0; i < D.size(); ++i) {
      if (!first[t][i]) continue;
      const std::string_view sv = D.at(i);
      memcpy(G.bytes.data() + pos, sv.data(), sv.size());
      pos += sv.size();
      G.off[id + 1] = (uint32_t)pos;
      dmap[t][d][i] = id++;
    }
  });
  parallel_for(T, nth, [&](size_t t) {  // references: their first occurrence's id (an earlier part or index)
    for (uint32_t i = 0; i < dmap[t][d].size(); ++i)
      if (dmap[t][d][i] == kRef) {
        const uint64_t e = ref[t][i];
        dmap[t][d][i] = dmap[(size_t)(e >> 32)][d][(uint32_t)e];
      }
  });
  std::vector<uint64_t> gh(G.size());
  parallel_for((g0 + 4095) / 4096, nth, [&](size_t c) {
    for (uint32_t id = (uint32_t)(c * 4096); id < g0 && id < (c + 1) * 4096; ++id) gh[id] = Dict::hash(G.at(id));
  });
  parallel_for(T, nth, [&](size_t t) {
    for (uint32_t i = 0; i < first[t].size(); ++i)
      if (first[t][i]) gh[dmap[t][d][i]] = hs[t][i];
  });
  G.reindex(gh, nth);
}

}  // namespace

void Dict::reindex(const std::vector<uint64_t>& hs, unsigned nth) {
  const size_t n = size();
  size_t cap = 64;
  while (cap < (n + 1) * 2) cap *= 2;
  slots.assign(cap, Slot{0u, 0u});
  const size_t mask = cap - 1;
  unsigned P = 1;
  while (P * 2 <= std::max(1u, nth) && cap / (P * 2) >= 4096) P *= 2;
  const size_t span = cap / P;
  std::vector<size_t> cnt(P + 1, 0);
  for (size_t id = 0; id < n; ++id) ++cnt[(hs[id] & mask) / span + 1];
  for (unsigned p = 0; p < P; ++p) cnt[p + 1] += cnt[p];
  std::vector<uint32_t> order(n);
  {
    std::vector<size_t> at(cnt.begin(), cnt.end() - 1);
    for (size_t id = 0; id < n; ++id) order[at[(hs[id] & mask) / span]++] = (uint32_t)id;
  }
  std::vector<std::vector<uint32_t>> deferred(P);
  parallel_for(P, P, [&](size_t p) {
    const size_t end = (p + 1) * span;
    for (size_t q = cnt[p]; q < cnt[p + 1]; ++q) {
      const uint32_t id = order[q];
      size_t i = hs[id] & mask;
      while (i < end && slots[i].id1) ++i;
      if (i == end) {  // the probe leaves the range: placed after every range is done
        deferred[p].push_back(id);
        continue;
      }
      slots[i] = Slot{(uint32_t)(hs[id] >> 32), id + 1};
    }
  });
  for (auto& v : deferred)
    for (uint32_t id : v) put(hs[id], id);
}

namespace {

// Concatenate per-chunk corpora (flattened in parallel, each with its own dictionaries) into
// C. Parts are merged in document order, so every dictionary, scalar and capability-set id
// is the one a sequential flatten assigns (first occurrence order).
void merge_parts(Corpus& C, std::vector<Corpus>& parts, bool docs, unsigned nthreads) {
  const size_t T = parts.size();
  const auto tm0 = std::chrono::steady_clock::now();
  // ---- id maps (sequential, document order) ----
  std::vector<std::vector<std::vector<uint32_t>>> dmap(T, std::vector<std::vector<uint32_t>>(KPE_NUM_DOMAINS));
  std::vector<std::vector<uint32_t>> capmap(T), scmap(T);
  auto merge_scalars = [&] {  // scalar tables (document tapes), parts in document order
    for (size_t t = 0; t < T; ++t) {
      const Corpus& P = parts[t];
      if (C.scal.empty()) C.scal.assign(P.scal.begin(), P.scal.begin() + 3), C.scal_text.assign(P.scal_text.begin(), P.scal_text.begin() + 9);
      auto& sm = scmap[t];
      sm.resize(P.scal.size());
      for (uint32_t k = 0; k < 3 && k < P.scal.size(); ++k) sm[k] = k;  // null, false, true
      for (size_t k = 3; k < P.scal.size(); ++k) {
        const KpeScalar& e = P.scal[k];
        const uint32_t ty = SC_TYPE(e.flags);
        uint32_t* slot = nullptr;
        uint32_t str_slot = 0xFFFFFFFFu;  // string scalars: the index lookup's result
        uint64_t str_h = 0;
        if (ty == SC_T_INT) {
          slot = &C.scal_int.emplace(e.ival, 0xFFFFFFFFu).first->second;
        } else if (ty == SC_T_FLOAT) {
          uint64_t bits;
          memcpy(&bits, &e.fval, 8);
          slot = &C.scal_float.emplace(bits, 0xFFFFFFFFu).first->second;
        } else {
          const std::string_view sv(P.scal_text.data() + e.text_off, e.text_len);
          const uint64_t h = StrIndex::hash(sv);
          const int64_t found = C.scal_str.find(sv, h, [&](uint32_t id) { return C.scal_text_of(id); });
          str_slot = found >= 0 ? (uint32_t)found : 0xFFFFFFFFu;
          slot = &str_slot;
          str_h = h;
        }
        if (*slot == 0xFFFFFFFFu) {
          KpeScalar g = e;
          if ((g.flags & SC_RANGE) && SC_TYPE(g.flags) == SC_T_STR) {  // endpoint ids (lower indices: mapped)
            const uint64_t x = (uint64_t)e.ival;
            g.ival = (int64_t)((uint64_t)sm[(uint32_t)x] | ((uint64_t)sm[(uint32_t)(x >> 32)] << 32));
          }
          const size_t nb = (size_t)e.text_len + e.sp_len;
          if (C.scal_text.size() + nb > 0xFFFFFFFFull) throw LimitError("scalar text pool exceeds 4 GiB");
          g.text_off = (uint32_t)C.scal_text.size();
          C.scal_text.insert(C.scal_text.end(), P.scal_text.begin() + e.text_off, P.scal_text.begin() + e.text_off + nb);
          *slot = (uint32_t)C.scal.size();
          C.scal.push_back(g);
          if (slot == &str_slot) C.scal_str.insert(str_h, *slot);
        }
        sm[k] = *slot;
      }
  
    }
  };
  {  // one thread per domain and one for the scalars (all independent); parts in document order
    std::vector<std::thread> th;
    std::exception_ptr serr;
    if (docs)
      th.emplace_back([&] {
        try {
          merge_scalars();
        } catch (...) {
          serr = std::current_exception();
        }
      });
    std::vector<std::exception_ptr> derr(KPE_NUM_DOMAINS);
    for (int d = 0; d < KPE_NUM_DOMAINS; ++d)
      th.emplace_back([&, d] {
        size_t tot = C.dict[d].size();
        for (size_t t = 0; t < T; ++t) tot += parts[t].dict[d].size();
        if (tot >= (1u << 16) && nthreads > 1) {  // e.g. resource names (one per resource)
          try {
            merge_dict_parallel(C.dict[d], parts, d, dmap, nthreads);
          } catch (...) {
            derr[d] = std::current_exception();
          }
          return;
        }
        C.dict[d].reserve(tot);
        for (size_t t = 0; t < T; ++t) {
          const Dict& D = parts[t].dict[d];
          auto& m = dmap[t][d];
          m.resize(D.size());
          for (uint32_t i = 0; i < D.size(); ++i) m[i] = C.dict[d].intern(D.at(i));
        }
      });
    for (auto& x : th) x.join();
    if (serr) std::rethrow_exception(serr);
    for (auto& e : derr)
      if (e) std::rethrow_exception(e);
  }
  const auto tm1 = std::chrono::steady_clock::now();
  // per-resource limits decided against one part's dictionaries may differ from the merged
  // ones: such a corpus is flattened again on one thread
  if (C.dict[D_CAP].size() > 64 || C.dict[D_KIND].size() > 4096 || C.dict[D_VERSION].size() > 1024 ||
      C.dict[D_GROUP].size() > 1024)
    throw NeedSequential();
  if (docs && C.dict[D_KEY].size() >= DN_MAX_KEYS) throw LimitError("too many distinct member names");
  auto capbits = [](uint64_t m, const std::vector<uint32_t>& cm) {
    uint64_t o = 0;
    for (; m; m &= m - 1) o |= 1ull << cm[__builtin_ctzll(m)];
    return o;
  };
  for (size_t t = 0; t < T; ++t) {
    const Corpus& P = parts[t];
    for (size_t j = 0; j < P.capset_add.size(); ++j) {
      const uint64_t ad = capbits(P.capset_add[j], dmap[t][D_CAP]), dr = capbits(P.capset_drop[j], dmap[t][D_CAP]);
      std::string key(16, '\0');
      memcpy(&key[0], &ad, 8);
      memcpy(&key[8], &dr, 8);
      auto it = C.capset_index.find(key);
      uint32_t cs;
      if (it == C.capset_index.end()) {
        cs = (uint32_t)C.capset_add.size();
        if (cs >= KPE_MAX_CAPSETS) throw NeedSequential();
        C.capset_index.emplace(key, cs);
        C.capset_add.push_back(ad), C.capset_drop.push_back(dr);
      } else {
        cs = it->second;
      }
      capmap[t].push_back(cs);
    }
  }
  // ---- bases of every part in the merged columns ----
  struct Base {
    size_t n, lab, ann, ctr, vol, sys, pann, port, doc;
  };
  std::vector<Base> base(T + 1);
  base[0] = Base{(size_t)C.n, C.lab_k.size(), C.ann_k.size(), C.c_sc.size(), C.vol_src.size(), C.sys_id.size(),
                 C.pann_k.size(), C.cport_host.size(), C.doc.size() / 2};
  for (size_t t = 0; t < T; ++t) {
    const Corpus& P = parts[t];
    base[t + 1] = Base{base[t].n + (size_t)P.n, base[t].lab + P.lab_k.size(), base[t].ann + P.ann_k.size(),
                       base[t].ctr + P.c_sc.size(), base[t].vol + P.vol_src.size(), base[t].sys + P.sys_id.size(),
                       base[t].pann + P.pann_k.size(), base[t].port + P.cport_host.size(),
                       base[t].doc + P.doc.size() / 2};
  }
  const Base& e = base[T];
  if (e.n >= 0x7FFFFFC0ull) throw LimitError("more than 2^31 - 64 resources in one corpus (32-bit row ids)");
  if (e.doc > 0xFFFFFFFFull) throw LimitError("document tape exceeds 2^32 entries");
  const size_t n0 = C.n;
  // the merged columns, sized on several threads (their zero fill is the first touch of fresh
  // pages, which costs more than the placement itself)
  std::vector<std::function<void()>> sz;
  for (auto* v : {&C.r_flags, &C.r_gvk, &C.r_name, &C.r_mns, &C.r_nsa, &C.r_nsl, &C.p_sc})
    sz.push_back([v, &e] { v->resize(e.n); });
  sz.push_back([&] { C.p_cold.resize(e.n * 4); });
  sz.push_back([&] { C.rec.resize(e.n * 4); });
  for (auto* v : {&C.lab_off, &C.ann_off, &C.ctr_off, &C.vol_off, &C.sys_off, &C.pann_off})
    sz.push_back([v, &e] { v->resize(e.n + 1); });
  for (auto* v : {&C.lab_k, &C.lab_v}) sz.push_back([v, &e] { v->resize(e.lab); });
  for (auto* v : {&C.ann_k, &C.ann_v}) sz.push_back([v, &e] { v->resize(e.ann); });
  sz.push_back([&] { C.vol_src.resize(e.vol); });
  sz.push_back([&] { C.sys_id.resize(e.sys); });
  for (auto* v : {&C.pann_k, &C.pann_v}) sz.push_back([v, &e] { v->resize(e.pann); });
  sz.push_back([&] { C.pann_kv.resize(e.pann * 2); });
  for (auto* v : {&C.c_sc, &C.c_name, &C.c_image, &C.c_sann, &C.c_sann_key, &C.c_sec_str, &C.c_pm_str, &C.c_selt_str,
                  &C.c_selu_str, &C.c_selr_str})
    sz.push_back([v, &e] { v->resize(e.ctr); });
  sz.push_back([&] { C.c_add.resize(e.ctr); });
  sz.push_back([&] { C.c_drop.resize(e.ctr); });
  sz.push_back([&] { C.crec.resize(e.ctr * 2); });
  sz.push_back([&] { C.cport_off.resize(e.ctr + 1); });
  sz.push_back([&] { C.cport_host.resize(e.port); });
  sz.push_back([&] { C.cport_str.resize(e.port); });
  if (docs) {
    sz.push_back([&] { C.doc.resize(e.doc * 2); });
    sz.push_back([&] { C.doc_off.resize(e.n); });
    sz.push_back([&] { C.img_off.resize(e.n); });
    C.has_docs = true;
  }
  parallel_for(sz.size(), nthreads, [&](size_t i) { sz[i](); });
  // ---- remap and place every part (parallel) ----
  auto place = [&](size_t t) {
    const Corpus& P = parts[t];
    const Base& b = base[t];
    const auto& M = dmap[t];
    auto id = [&](int d, uint32_t x) { return x == KPE_NO_STR ? x : M[d][x]; };
    for (size_t r = 0; r < (size_t)P.n; ++r) {
      const size_t g = b.n + r;
      const uint32_t gv = P.r_gvk[r];
      const uint32_t gvk = M[D_KIND][GVK_KIND(gv)] | (M[D_VERSION][GVK_VER(gv)] << 12) | (M[D_GROUP][GVK_GRP(gv)] << 22);
      C.r_flags[g] = P.r_flags[r], C.r_gvk[g] = gvk, C.r_name[g] = id(D_NAME, P.r_name[r]);
      C.r_mns[g] = id(D_NS, P.r_mns[r]), C.r_nsa[g] = id(D_NS, P.r_nsa[r]), C.r_nsl[g] = P.r_nsl[r];
      C.p_sc[g] = P.p_sc[r];
      for (int k = 0; k < 4; ++k) C.p_cold[g * 4 + k] = id(D_MISC, P.p_cold[r * 4 + k]);
      C.rec[g * 4] = P.rec[r * 4], C.rec[g * 4 + 1] = gvk, C.rec[g * 4 + 2] = P.rec[r * 4 + 2];
      C.rec[g * 4 + 3] = id(D_NS, P.rec[r * 4 + 3]);
      C.lab_off[g + 1] = (uint32_t)(b.lab + P.lab_off[r + 1]), C.ann_off[g + 1] = (uint32_t)(b.ann + P.ann_off[r + 1]);
      C.ctr_off[g + 1] = (uint32_t)(b.ctr + P.ctr_off[r + 1]), C.vol_off[g + 1] = (uint32_t)(b.vol + P.vol_off[r + 1]);
      C.sys_off[g + 1] = (uint32_t)(b.sys + P.sys_off[r + 1]);
      C.pann_off[g + 1] = (uint32_t)(b.pann + P.pann_off[r + 1]);
    }
    for (size_t k = 0; k < P.lab_k.size(); ++k)
      C.lab_k[b.lab + k] = id(D_LABK, P.lab_k[k]), C.lab_v[b.lab + k] = id(D_LABV, P.lab_v[k]);
    for (size_t k = 0; k < P.ann_k.size(); ++k)
      C.ann_k[b.ann + k] = id(D_ANNK, P.ann_k[k]), C.ann_v[b.ann + k] = id(D_ANNV, P.ann_v[k]);
    for (size_t k = 0; k < P.vol_src.size(); ++k) C.vol_src[b.vol + k] = P.vol_src[k];
    for (size_t k = 0; k < P.sys_id.size(); ++k) C.sys_id[b.sys + k] = id(D_SYSCTL, P.sys_id[k]);
    for (size_t k = 0; k < P.pann_k.size(); ++k) {
      const uint32_t ak = id(D_ANNK, P.pann_k[k]), av = id(D_ANNV, P.pann_v[k]);
      C.pann_k[b.pann + k] = ak, C.pann_v[b.pann + k] = av;
      C.pann_kv[(b.pann + k) * 2] = ak, C.pann_kv[(b.pann + k) * 2 + 1] = av;
    }
    for (size_t k = 0; k < P.c_sc.size(); ++k) {
      const size_t g = b.ctr + k;
      C.c_sc[g] = P.c_sc[k];
      C.c_add[g] = capbits(P.c_add[k], M[D_CAP]), C.c_drop[g] = capbits(P.c_drop[k], M[D_CAP]);
      C.c_name[g] = id(D_CNAME, P.c_name[k]), C.c_image[g] = id(D_IMAGE, P.c_image[k]);
      C.c_sann[g] = id(D_ANNV, P.c_sann[k]), C.c_sann_key[g] = id(D_ANNK, P.c_sann_key[k]);
      C.c_sec_str[g] = id(D_MISC, P.c_sec_str[k]), C.c_pm_str[g] = id(D_MISC, P.c_pm_str[k]);
      C.c_selt_str[g] = id(D_MISC, P.c_selt_str[k]), C.c_selu_str[g] = id(D_MISC, P.c_selu_str[k]);
      C.c_selr_str[g] = id(D_MISC, P.c_selr_str[k]);
      const uint32_t y = P.crec[k * 2 + 1];
      C.crec[g * 2] = P.crec[k * 2], C.crec[g * 2 + 1] = capmap[t][CY_CAPSET(y)] | (y & 0xFFFF0000u);
      C.cport_off[g + 1] = (uint32_t)(b.port + P.cport_off[k + 1]);
    }
    for (size_t k = 0; k < P.cport_host.size(); ++k)
      C.cport_host[b.port + k] = P.cport_host[k], C.cport_str[b.port + k] = id(D_MISC, P.cport_str[k]);
    if (!docs) return;
    const auto& sm = scmap[t];
    const uint32_t tb = (uint32_t)b.doc;
    auto remap = [&](uint32_t x, uint32_t y, uint32_t* ox, uint32_t* oy) {
      const uint32_t key1 = DN_KEY(x);
      *ox = DN_KIND(x) | ((key1 ? M[D_KEY][key1 - 1] + 1u : 0u) << 2);
      *oy = DN_KIND(x) == DN_SCALAR ? sm[y] : y + tb;
    };
    std::vector<uint32_t> stack;
    for (size_t r = 0; r < (size_t)P.n; ++r) {  // walk every document (and images map) from its root entry
      const uint32_t root = (uint32_t)P.doc_off[r];
      C.doc_off[b.n + r] = tb + root;
      stack.assign(1, root);
      C.img_off[b.n + r] = P.img_off[r] == KPE_NO_IMAGES ? KPE_NO_IMAGES : tb + P.img_off[r];
      if (P.img_off[r] != KPE_NO_IMAGES) stack.push_back((uint32_t)P.img_off[r]);
      while (!stack.empty()) {
        const uint32_t en = stack.back();
        stack.pop_back();
        const uint32_t x = P.doc[en * 2], y = P.doc[en * 2 + 1];
        remap(x, y, &C.doc[(size_t)(tb + en) * 2], &C.doc[(size_t)(tb + en) * 2 + 1]);
        if (DN_KIND(x) != DN_SCALAR) {
          const uint32_t cnt = P.doc[y * 2];
          C.doc[(size_t)(tb + y) * 2] = cnt, C.doc[(size_t)(tb + y) * 2 + 1] = 0;
          for (uint32_t q = 0; q < cnt; ++q) stack.push_back(y + 1 + q);
        }
      }
    }
  };
  auto place_and_free = [&](size_t t) {
    place(t);
    parts[t] = Corpus();  // release the part's columns on this thread
  };
  if (T > 0) {
    C.lab_off[n0] = (uint32_t)base[0].lab, C.ann_off[n0] = (uint32_t)base[0].ann;
    C.ctr_off[n0] = (uint32_t)base[0].ctr, C.vol_off[n0] = (uint32_t)base[0].vol;
    C.sys_off[n0] = (uint32_t)base[0].sys, C.pann_off[n0] = (uint32_t)base[0].pann;
  }
  if (base[0].ctr < C.cport_off.size()) C.cport_off[base[0].ctr] = (uint32_t)base[0].port;
  for (size_t t = 0; t < T; ++t)
    for (uint32_t row : parts[t].limit_rows) C.limit_rows.push_back((uint32_t)(base[t].n + row));
  const auto tm2 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (size_t t = 0; t < T; ++t) {
    if (th.size() >= nthreads) th.front().join(), th.erase(th.begin());
    th.emplace_back(place_and_free, t);
  }
  for (auto& x : th) x.join();
  C.n = (int64_t)e.n;
  if (getenv("KPE_DEBUG")) {
    const auto tm3 = std::chrono::steady_clock::now();
    fprintf(stderr, "kpe merge: dictionaries %.3f s, capability sets + sizing %.3f s, placement %.3f s\n",
            std::chrono::duration<double>(tm1 - tm0).count(), std::chrono::duration<double>(tm2 - tm1).count(),
            std::chrono::duration<double>(tm3 - tm2).count());
  }
}

unsigned flatten_threads() {
  if (const char* ev = getenv("KPE_FLATTEN_THREADS")) return std::max(1, std::min(64, atoi(ev)));
  const unsigned hw = std::thread::hardware_concurrency();
  return std::max(1u, std::min(16u, hw ? hw : 1u));  // the GPU box's CPU share is 16
}

}  // namespace

// Entry used by kpe_corpus_flatten. Throws std::invalid_argument / LimitError. Large inputs are
// cut at line boundaries and flattened by up to flatten_threads() threads into per-chunk
// corpora, then merged in document order (ids equal to a sequential flatten). The first error
// in document order is the one thrown; corpus-wide limits are checked at the merge.
void flatten_ndjson(Corpus& C, const char* buf, size_t len, const char* nsl, size_t nsl_len, bool docs) {
  load_ns_labels(C, nsl, nsl_len);
  const unsigned T = std::min<unsigned>(flatten_threads(), (unsigned)(len / (1u << 20)));
  if (T <= 1 || C.n != 0) {
    flatten_range(C, buf, 0, len, docs);
    rebuild_headers(C);
    return;
  }
  std::vector<size_t> cut(T + 1, len);
  cut[0] = 0;
  for (unsigned t = 1; t < T; ++t) {
    size_t p = std::max(cut[t - 1], len * t / T);
    while (p < len && buf[p] != '\n') ++p;
    cut[t] = p < len ? p + 1 : len;
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<Corpus> parts(T);
  std::vector<std::exception_ptr> errs(T);
  for (auto& P : parts) P.nsl_index = C.nsl_index;
  {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        try {
          flatten_range(parts[t], buf + cut[t], 0, cut[t + 1] - cut[t], docs);
        } catch (...) {
          errs[t] = std::current_exception();
        }
      });
    for (auto& x : th) x.join();
  }
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  const auto t1 = std::chrono::steady_clock::now();
  try {
    merge_parts(C, parts, docs, T);
  } catch (const NeedSequential&) {
    parts.clear();
    C = Corpus();
    load_ns_labels(C, nsl, nsl_len);
    flatten_range(C, buf, 0, len, docs);
  }
  rebuild_headers(C);
  if (getenv("KPE_DEBUG")) {
    const auto t2 = std::chrono::steady_clock::now();
    fprintf(stderr, "kpe flatten: %u threads, chunks %.3f s, merge %.3f s\n", T,
            std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
  }
}

bool is_limit_error(const std::exception& e) { return dynamic_cast<const LimitError*>(&e) != nullptr; }

}  // namespace kpe
