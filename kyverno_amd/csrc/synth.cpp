// Synthetic corpus generator (see include/kpe_synth.h). Benchmark/test utility.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kpe_synth.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {
    for (int i = 0; i < 4; ++i) next();
  }
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double u() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  int below(int n) { return (int)(next() % (uint64_t)n); }
  bool p(double x) { return u() < x; }
};

const char* kImages[50] = {"nginx", "redis", "postgres", "mysql", "mongo", "busybox", "alpine", "ubuntu", "debian",
                           "httpd", "node", "python", "golang", "openjdk", "ruby", "php", "memcached", "rabbitmq",
                           "elasticsearch", "kibana", "logstash", "grafana", "prometheus", "consul", "vault",
                           "traefik", "haproxy", "envoy", "etcd", "zookeeper", "kafka", "cassandra", "influxdb",
                           "telegraf", "fluentd", "jenkins", "gitlab", "nextcloud", "wordpress", "ghost", "drupal",
                           "tomcat", "jetty", "caddy", "minio", "registry", "coredns", "calico", "cilium", "istio"};

struct Ctr {
  std::string name, image;
  int ape = 0;          // 0 false, 1 true, 2 absent
  int rnr = 0;          // 0 true, 1 false, 2 absent
  int caps = 0;         // 0 drop ALL, 1 no capabilities, 2 drop other, 3 drop ALL + add SYS_ADMIN, 4 drop ALL + add CHOWN, 5 drop ALL + add NET_BIND_SERVICE
  int seccomp = 0;      // 0 RuntimeDefault, 1 Localhost, 2 absent, 3 Unconfined, 4 bogus
  bool priv = false, privFalse = false;
  bool procUnmasked = false;
  bool runAsUser0 = false, runAsUser = false;
  int selinux = 0;      // 0 none, 1 container_t, 2 spc_t, 3 user set
  bool whp = false;
  int hostPort = 0;
  bool port = false;
  bool sc_null = false;
};

void emit_ctr(std::string& o, const Ctr& c) {
  o += "{\"name\":\"" + c.name + "\",\"image\":\"" + c.image + "\"";
  if (c.port) {
    o += ",\"ports\":[{\"containerPort\":8080";
    if (c.hostPort) o += ",\"hostPort\":" + std::to_string(c.hostPort);
    o += "}]";
  }
  if (c.sc_null) {
    o += ",\"securityContext\":null}";
    return;
  }
  o += ",\"securityContext\":{";
  bool first = true;
  auto f = [&](const std::string& s) {
    if (!first) o += ",";
    first = false;
    o += s;
  };
  if (c.ape == 0) f("\"allowPrivilegeEscalation\":false");
  else if (c.ape == 1) f("\"allowPrivilegeEscalation\":true");
  if (c.rnr == 0) f("\"runAsNonRoot\":true");
  else if (c.rnr == 1) f("\"runAsNonRoot\":false");
  switch (c.caps) {
    case 0: f("\"capabilities\":{\"drop\":[\"ALL\"]}"); break;
    case 1: break;
    case 2: f("\"capabilities\":{\"drop\":[\"NET_RAW\"]}"); break;
    case 3: f("\"capabilities\":{\"drop\":[\"ALL\"],\"add\":[\"SYS_ADMIN\"]}"); break;
    case 4: f("\"capabilities\":{\"drop\":[\"ALL\"],\"add\":[\"CHOWN\"]}"); break;
    case 5: f("\"capabilities\":{\"drop\":[\"ALL\"],\"add\":[\"NET_BIND_SERVICE\"]}"); break;
  }
  switch (c.seccomp) {
    case 0: f("\"seccompProfile\":{\"type\":\"RuntimeDefault\"}"); break;
    case 1: f("\"seccompProfile\":{\"type\":\"Localhost\",\"localhostProfile\":\"profiles/audit.json\"}"); break;
    case 2: break;
    case 3: f("\"seccompProfile\":{\"type\":\"Unconfined\"}"); break;
    case 4: f("\"seccompProfile\":{\"type\":\"bogus\"}"); break;
  }
  if (c.priv) f("\"privileged\":true");
  else if (c.privFalse) f("\"privileged\":false");
  if (c.procUnmasked) f("\"procMount\":\"Unmasked\"");
  if (c.runAsUser0) f("\"runAsUser\":0");
  else if (c.runAsUser) f("\"runAsUser\":1000");
  if (c.selinux == 1) f("\"seLinuxOptions\":{\"type\":\"container_t\"}");
  else if (c.selinux == 2) f("\"seLinuxOptions\":{\"type\":\"spc_t\"}");
  else if (c.selinux == 3) f("\"seLinuxOptions\":{\"user\":\"system_u\",\"level\":\"s0\"}");
  if (c.whp) f("\"windowsOptions\":{\"hostProcess\":true}");
  o += "}}";
}

// C4 label sets: 8 distinct keys from a 64-key vocabulary (some prefixed), values
// from small per-key vocabularies; ~1% carry a key or value that is not a valid
// label (selector parse errors when a wildcard resolves to it).
std::string label_key(int k) {
  static const char* kPre[4] = {"", "app.kubernetes.io/", "example.com/", "team.io/"};
  return std::string(kPre[k & 3]) + "k" + std::to_string(k);
}
std::string selector_labels(Rng& r) {
  uint64_t used = 0;
  std::string l = "{";
  for (int i = 0; i < 8; ++i) {
    int k;
    do k = r.below(64);
    while (used >> k & 1);
    used |= 1ull << k;
    std::string v = "v" + std::to_string(r.below(k < 8 ? 4 : 16));
    std::string key = label_key(k);
    if (r.p(0.005)) v = "bad value";
    if (r.p(0.005)) key = "Bad_/key/x";
    l += (i ? ",\"" : "\"") + key + "\":\"" + v + "\"";
  }
  return l + "}";
}

// C5: irregular fan-out pods for the require-pod-requests-limits /
// disallow-latest-tag / disallow-host-ports pattern set. Container counts follow a geometric
// law of mean ~6 truncated to [1, 64] (redrawn above 64).
// 64 lowercase hex digits derived from x (splitmix64 rounds): a valid sha256 digest string
// (go-digest), so the images context of the row builds (AddImageInfos, context.go:293-330)
std::string hex_digest(uint64_t x) {
  static const char* hx = "0123456789abcdef";
  std::string d;
  for (int k = 0; k < 4; ++k) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (int i = 0; i < 16; ++i) d += hx[(z >> (4 * i)) & 15u];
  }
  return d;
}

void gen_fanout(std::string& o, Rng& r, int64_t idx) {
  auto count = [&]() {
    for (;;) {
      const double u = r.u();
      const int k = 1 + (int)std::floor(std::log(1.0 - u) / std::log(1.0 - 1.0 / 6.0));
      if (k <= 64) return k;
    }
  };
  const int nc = count();
  const int ni = r.p(0.7) ? 0 : 1 + r.below(3);
  auto ctr = [&](std::string& s, const std::string& name) {
    s += "{\"name\":\"" + name + "\",\"image\":\"";
    const std::string img = kImages[r.below(50)];
    const double t = r.u();
    if (t < 0.45) s += img + ":1." + std::to_string(r.below(30)) + "." + std::to_string(r.below(10));
    else if (t < 0.65) s += img + ":latest";
    else if (t < 0.80) s += img;  // no tag
    else if (t < 0.90) s += img + "@sha256:" + hex_digest(1000000 + r.below(1000000));  // a well-formed digest
    else s += "ghcr.io/org-" + std::to_string(r.below(9)) + "/" + img + (r.p(0.5) ? ":2.0" : ":latest");
    s += "\"";
    const double pp = r.u();
    if (pp < 0.4) s += ",\"imagePullPolicy\":\"Always\"";
    else if (pp < 0.7) s += ",\"imagePullPolicy\":\"IfNotPresent\"";
    const double q = r.u();
    if (q < 0.75) {
      s += ",\"resources\":{\"limits\":{\"memory\":\"" + std::to_string(64 << r.below(5)) + "Mi\",\"cpu\":\"" +
           std::to_string(100 * (1 + r.below(8))) + "m\"},\"requests\":{\"cpu\":\"" +
           std::to_string(50 * (1 + r.below(8))) + "m\",\"memory\":\"" + std::to_string(32 << r.below(5)) + "Mi\"}}";
    } else if (q < 0.85) {
      s += ",\"resources\":{\"limits\":{\"memory\":\"256Mi\"},\"requests\":{\"memory\":\"128Mi\"}}";  // no cpu request
    } else if (q < 0.90) {
      s += ",\"resources\":{\"limits\":{\"memory\":\"\"},\"requests\":{\"cpu\":\"1\",\"memory\":\"1Gi\"}}";
    } else if (q < 0.95) {
      s += ",\"resources\":{\"requests\":{}}";
    }
    const double pt = r.u();
    if (pt < 0.30) s += ",\"ports\":[{\"containerPort\":8080}]";
    else if (pt < 0.33) s += ",\"ports\":[{\"containerPort\":80,\"hostPort\":0},{\"containerPort\":443}]";
    else if (pt < 0.36) s += ",\"ports\":[{\"containerPort\":9090,\"hostPort\":" + std::to_string(9000 + r.below(99)) + "}]";
    s += "}";
  };
  std::string spec = "{";
  if (ni) {
    spec += "\"initContainers\":[";
    for (int i = 0; i < ni; ++i) {
      if (i) spec += ",";
      ctr(spec, "init-" + std::to_string(i));
    }
    spec += "],";
  }
  spec += "\"containers\":[";
  for (int i = 0; i < nc; ++i) {
    if (i) spec += ",";
    ctr(spec, "c-" + std::to_string(i));
  }
  spec += "]";
  if (r.p(0.1)) spec += ",\"volumes\":[{\"name\":\"data\",\"hostPath\":{\"path\":\"/data\"}}]";
  spec += "}";
  char nsbuf[16];
  snprintf(nsbuf, sizeof nsbuf, "ns-%04d", r.below(1000));
  const std::string name = "res-" + std::to_string(idx);
  const std::string labels = "{\"app\":\"app-" + std::to_string(r.below(200)) + "\"}";
  if (r.p(0.85)) {
    o += "{\"apiVersion\":\"v1\",\"kind\":\"Pod\",\"metadata\":{\"name\":\"" + name + "\",\"namespace\":\"" + nsbuf +
         "\",\"labels\":" + labels + "},\"spec\":" + spec + "}";
  } else {
    o += "{\"apiVersion\":\"apps/v1\",\"kind\":\"Deployment\",\"metadata\":{\"name\":\"" + name + "\",\"namespace\":\"" +
         nsbuf + "\",\"labels\":" + labels + "},\"spec\":{\"replicas\":2,\"selector\":{\"matchLabels\":" + labels +
         "},\"template\":{\"metadata\":{\"labels\":" + labels + "},\"spec\":" + spec + "}}}";
  }
}

void gen_one(std::string& o, uint64_t seed, int64_t idx, int mix) {
  Rng r(seed ^ ((uint64_t)idx * 0xD1B54A32D192ED03ull));
  if (mix == KPE_SYNTH_FANOUT) {
    gen_fanout(o, r, idx);
    return;
  }
  // ---- kind ----
  int kind = 0;  // 0 Pod, 1 Deployment, 2 DaemonSet, 3 Job, 4 CronJob, 5 Service, 6 ConfigMap, 7 StatefulSet
  const bool sel_mix = mix == KPE_SYNTH_SELECTORS;
  const bool c3 = mix == KPE_SYNTH_C3;
  if (sel_mix) {
    kind = r.p(0.5) ? 1 : 5;
  } else if (c3) {  // SURVEY.md 8(d) C3 ratios
    double u = r.u();
    kind = u < 0.40 ? 0 : u < 0.60 ? 1 : u < 0.75 ? 5 : u < 0.90 ? 6 : u < 0.9333 ? 3 : u < 0.9667 ? 4 : 7;
  } else if (mix >= KPE_SYNTH_MIXED) {
    double u = r.u();
    kind = u < 0.40 ? 0 : u < 0.60 ? 1 : u < 0.64 ? 2 : u < 0.67 ? 3 : u < 0.70 ? 4 : u < 0.85 ? 5 : u < 0.97 ? 6 : 7;
  }
  bool edge = mix == KPE_SYNTH_EDGE;
  char nsbuf[32];
  if (sel_mix) snprintf(nsbuf, sizeof nsbuf, "ns-%05d", r.below(10000));
  else if (c3) {
    const double u = r.u();
    const int t = r.below(40);
    if (u < 0.35) snprintf(nsbuf, sizeof nsbuf, "team-%d-prod", t);
    else if (u < 0.60) snprintf(nsbuf, sizeof nsbuf, "team-%d-dev", t);
    else if (u < 0.75) snprintf(nsbuf, sizeof nsbuf, "team-%d", t);
    else if (u < 0.85) snprintf(nsbuf, sizeof nsbuf, "shop-%d-prod", t % 7);
    else if (u < 0.92) snprintf(nsbuf, sizeof nsbuf, "kube-system");
    else snprintf(nsbuf, sizeof nsbuf, "default");
  } else snprintf(nsbuf, sizeof nsbuf, "ns-%04d", r.below(1000));
  std::string ns = nsbuf;
  std::string name = "res-" + std::to_string(idx);
  if (c3) {
    static const char* kWords[12] = {"api", "web", "cart", "auth", "db", "cache", "queue", "search", "pay", "mail",
                                     "log", "ui"};
    const double u = r.u();
    const std::string w = kWords[r.below(12)];
    if (u < 0.40) name = "app-" + w + "-" + std::string(1, (char)('a' + r.below(26)));  // app-*-?
    else if (u < 0.55) name = "app-" + w + "-" + std::to_string(idx % 1000);
    else if (u < 0.70) name = "web-" + w + "-" + std::to_string(idx % 97);
    else if (u < 0.80) name = w + "-db-" + std::to_string(idx % 13);
    else if (u < 0.88) name = w + "-canary";
    else name = "res-" + std::to_string(idx);
  }
  static const char* kKinds[] = {"Pod", "Deployment", "DaemonSet", "Job", "CronJob", "Service", "ConfigMap", "StatefulSet"};
  static const char* kApi[] = {"v1", "apps/v1", "apps/v1", "batch/v1", "batch/v1", "v1", "v1", "apps/v1"};
  auto labels = [&]() {
    if (sel_mix) return selector_labels(r);
    std::string l = "{\"app\":\"app-" + std::to_string(r.below(200)) + "\",\"tier\":\"" +
                    (r.p(0.5) ? "frontend" : "backend") + "\"";
    if (r.p(0.3)) l += ",\"team\":\"team-" + std::to_string(r.below(20)) + "\"";
    return l + "}";
  };
  o += "{\"apiVersion\":\"" + std::string(kApi[kind]) + "\",\"kind\":\"" + kKinds[kind] + "\",\"metadata\":{\"name\":\"" +
       name + "\",\"namespace\":\"" + ns + "\",\"labels\":" + labels();
  if (kind == 5 || kind == 6) {  // non-pod kinds
    o += "}";
    if (kind == 5) o += ",\"spec\":{\"selector\":{\"app\":\"x\"},\"ports\":[{\"port\":80,\"targetPort\":8080}]}}";
    else o += ",\"data\":{\"key\":\"value-" + std::to_string(r.below(100)) + "\"}}";
    return;
  }
  // ---- pod spec (the same generator serves templates) ----
  int ncont;
  double u = r.u();
  ncont = u < 0.7 ? 1 : u < 0.9 ? 2 : u < 0.97 ? 3 : 4;
  int ninit = r.p(0.2) ? 1 : 0;
  std::vector<Ctr> ctrs(ncont + ninit);
  for (size_t i = 0; i < ctrs.size(); ++i) {
    ctrs[i].name = (i < (size_t)ninit ? "init-" : "c-") + std::to_string(i);
    ctrs[i].image = std::string(kImages[r.below(50)]) + (r.p(0.5) ? ":latest" : ":1." + std::to_string(r.below(30)) + ".0");
    if (r.p(0.3)) {
      ctrs[i].port = true;
    }
    if (r.p(0.25)) ctrs[i].seccomp = 1;
    if (r.p(0.2)) ctrs[i].runAsUser = true;
    if (r.p(0.1)) ctrs[i].privFalse = true;
    if (r.p(0.05)) ctrs[i].selinux = 1;
    if (r.p(0.05)) ctrs[i].caps = 5;
  }
  bool hostNetwork = false, hostPID = false, hostIPC = false, hostPath = false, nfs = false, sysctlBad = false,
       podRunAsUser0 = false, podWhp = false, podSeccompUnconfined = false, podRnrFalse = false;
  std::string apparmor;
  bool windows = edge && r.p(0.05);
  int podSeccomp = 0;  // 0 none, 1 RuntimeDefault
  if (r.p(0.3)) podSeccomp = 1;
  bool podRnr = r.p(0.3);
  if (r.p(0.4)) {  // violating resource: 1-3 violations among the 17 checks
    int nv = 1 + r.below(3);
    for (int k = 0; k < nv; ++k) {
      Ctr& c = ctrs[r.below((int)ctrs.size())];
      bool present = r.p(0.5);
      switch (r.below(17)) {
        case 0: c.ape = present ? 1 : 2; break;
        case 1: apparmor = c.name; break;
        case 2: c.caps = 3; break;
        case 3: c.caps = present ? 2 : (r.p(0.5) ? 1 : 4); break;
        case 4: (r.p(0.34) ? hostNetwork : r.p(0.5) ? hostPID : hostIPC) = true; break;
        case 5: hostPath = true; break;
        case 6: c.port = true, c.hostPort = 8000 + r.below(100); break;
        case 7: c.priv = true; break;
        case 8: c.procUnmasked = true; break;
        case 9: nfs = true; break;
        case 10:
          if (present) c.rnr = 1;
          else c.rnr = 2, podRnr = false;
          if (r.p(0.2)) podRnrFalse = true;
          break;
        case 11: (r.p(0.5) ? c.runAsUser0 : podRunAsUser0) = true; break;
        case 12: c.selinux = present ? 2 : 3; break;
        case 13: (r.p(0.5) ? c.seccomp : podSeccomp) = 3, podSeccompUnconfined = true; break;
        case 14:
          c.seccomp = present ? 4 : 2;
          podSeccomp = 0;
          break;
        case 15: sysctlBad = true; break;
        case 16: (r.p(0.5) ? c.whp : podWhp) = true; break;
      }
    }
  }
  if (edge && r.p(0.05)) ctrs[0].sc_null = true;
  std::string spec = "{";
  if (hostNetwork) spec += "\"hostNetwork\":true,";
  if (hostPID) spec += "\"hostPID\":true,";
  if (hostIPC) spec += "\"hostIPC\":true,";
  if (windows) spec += "\"os\":{\"name\":\"windows\"},";
  bool psc = podSeccomp || podRnr || podRnrFalse || podRunAsUser0 || podWhp || sysctlBad || podSeccompUnconfined;
  if (psc) {
    spec += "\"securityContext\":{";
    bool first = true;
    auto f = [&](const std::string& s) {
      if (!first) spec += ",";
      first = false;
      spec += s;
    };
    if (podSeccomp == 1) f("\"seccompProfile\":{\"type\":\"RuntimeDefault\"}");
    else if (podSeccomp == 3) f("\"seccompProfile\":{\"type\":\"Unconfined\"}");
    if (podRnrFalse) f("\"runAsNonRoot\":false");
    else if (podRnr) f("\"runAsNonRoot\":true");
    if (podRunAsUser0) f("\"runAsUser\":0");
    if (podWhp) f("\"windowsOptions\":{\"hostProcess\":true}");
    if (sysctlBad) f("\"sysctls\":[{\"name\":\"kernel.msgmax\",\"value\":\"65536\"}]");
    else if (edge && r.p(0.1)) f("\"sysctls\":[{\"name\":\"net.ipv4.ip_local_reserved_ports\",\"value\":\"1\"}]");
    spec += "},";
  }
  if (edge && r.p(0.03)) spec += "\"hostNetwork\":\"yes\",";  // typed decode error
  spec += "\"volumes\":[";
  spec += "{\"name\":\"cfg\",\"configMap\":{\"name\":\"cfg\"}}";
  if (r.p(0.3)) spec += ",{\"name\":\"tmp\",\"emptyDir\":{}}";
  if (hostPath) spec += ",{\"name\":\"host\",\"hostPath\":{\"path\":\"/var/run\"}}";
  if (nfs) spec += ",{\"name\":\"share\",\"nfs\":{\"server\":\"nfs.local\",\"path\":\"/x\"}}";
  spec += "],";
  auto list = [&](const char* key, int a, int b) {
    spec += std::string("\"") + key + "\":[";
    for (int i = a; i < b; ++i) {
      if (i > a) spec += ",";
      emit_ctr(spec, ctrs[i]);
    }
    spec += "]";
  };
  if (ninit) {
    list("initContainers", 0, ninit);
    spec += ",";
  }
  list("containers", ninit, (int)ctrs.size());
  spec += "}";
  std::string ann;
  if (!apparmor.empty() || r.p(0.2)) {
    ann = "\"annotations\":{\"owner\":\"team-" + std::to_string(r.below(20)) + "\"";
    if (!apparmor.empty())
      ann += ",\"container.apparmor.security.beta.kubernetes.io/" + apparmor + "\":\"unconfined\"";
    else if (r.p(0.3))
      ann += ",\"container.apparmor.security.beta.kubernetes.io/c-0\":\"runtime/default\"";
    ann += "}";
  }
  if (kind == 0) {
    if (!ann.empty()) o += "," + ann;
    o += "},\"spec\":" + spec + "}";
    return;
  }
  o += "}";
  std::string tmpl = "{\"metadata\":{\"labels\":" + labels() + (ann.empty() ? "" : "," + ann) + "},\"spec\":" + spec + "}";
  if (kind == 4) {
    o += ",\"spec\":{\"schedule\":\"*/5 * * * *\",\"jobTemplate\":{\"metadata\":{" +
         (ann.empty() ? std::string("\"labels\":{\"job\":\"x\"}") : ann) + "},\"spec\":{\"template\":" + tmpl + "}}}}";
  } else {
    o += ",\"spec\":{\"replicas\":" + std::to_string(1 + r.below(5)) +
         ",\"selector\":{\"matchLabels\":{\"app\":\"x\"}},\"template\":" + tmpl + "}}";
  }
}

}  // namespace

extern "C" int kpe_synth_resources(uint64_t seed, int64_t first, int64_t n, int mix, char** out, size_t* len) {
  if (n < 0 || !out || !len) return 1;
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 10000) nt = 1;
  std::vector<std::string> parts(nt);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) {
    th.emplace_back([&, t]() {
      int64_t a = n * t / nt, b = n * (t + 1) / nt;
      std::string& s = parts[t];
      s.reserve((size_t)(b - a) * 900);
      for (int64_t i = a; i < b; ++i) {
        gen_one(s, seed, first + i, mix);
        s += '\n';
      }
    });
  }
  for (auto& x : th) x.join();
  size_t tot = 0;
  for (auto& p : parts) tot += p.size();
  char* buf = (char*)malloc(tot + 1);
  if (!buf) return 2;
  size_t off = 0;
  for (auto& p : parts) {
    memcpy(buf + off, p.data(), p.size());
    off += p.size();
  }
  buf[tot] = 0;
  *out = buf;
  *len = tot;
  return 0;
}

extern "C" void kpe_synth_free(char* p) { free(p); }

extern "C" int kpe_synth_ns_labels(uint64_t seed, int64_t n_namespaces, int mix, char** out, size_t* len) {
  if (n_namespaces < 0 || !out || !len) return 1;
  std::string s = "{";
  static const char* kEnv[3] = {"prod", "staging", "dev"};
  for (int64_t i = 0; i < n_namespaces; ++i) {
    Rng r(seed ^ 0x5EEDull ^ ((uint64_t)i * 0xA24BAED4963EE407ull));
    char nsbuf[16];
    if (mix == KPE_SYNTH_SELECTORS) snprintf(nsbuf, sizeof nsbuf, "ns-%05d", (int)i);
    else snprintf(nsbuf, sizeof nsbuf, "ns-%04d", (int)i);
    if (i) s += ",";
    s += "\"" + std::string(nsbuf) + "\":{\"kubernetes.io/metadata.name\":\"" + nsbuf + "\",\"env\":\"" +
         kEnv[r.below(3)] + "\",\"team\":\"team-" + std::to_string(r.below(50)) + "\"";
    if (r.p(0.5)) s += ",\"pss\":\"" + std::string(r.p(0.5) ? "restricted" : "baseline") + "\"";
    if (r.p(0.1)) s += ",\"region\":\"r" + std::to_string(r.below(6)) + "\"";
    s += "}";
  }
  s += "}";
  char* buf = (char*)malloc(s.size() + 1);
  if (!buf) return 2;
  memcpy(buf, s.data(), s.size() + 1);
  *out = buf;
  *len = s.size();
  return 0;
}
