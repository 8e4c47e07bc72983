// ORACLE — test infrastructure only. Never linked into the product path.
//
// The `images` JSON context of a policy context (pkg/engine/context/context.go:293-348
// AddImageInfos / convertImagesToUnstructured), from:
//   pkg/utils/api/image.go:17-229  ExtractImagesFromResource, extract, BuildStandardExtractors
//   pkg/utils/image/infos.go:11-100 ImageInfo, GetImageInfo, addDefaultRegistry
//   github.com/distribution/reference v0.5.0 (go.mod:17; third-party, absent here) Parse and
//     its regexp grammar (regexp.go), restated with std::regex (ECMAScript backtracking is the
//     same leftmost-first preference Go's regexp gives FindStringSubmatch)
//   github.com/opencontainers/go-digest v1.0.0 (go.mod:40) Digest.Validate: sha256 / sha384 /
//     sha512 with lower-case hex of exactly 64 / 96 / 128 digits
// Configuration: defaultRegistry "docker.io", enableDefaultRegistryMutation true (the
// pkg/config defaults, config.go:243-245), no custom image extractors.
// A resource whose images fail to extract makes NewPolicyContext fail
// (policycontext/policy_context.go:230): no rule of any policy gives a response
// (ImageError).
#pragma once
#include <algorithm>
#include <map>
#include <regex>
#include <string>
#include <vector>

#include "json_dom.hpp"

namespace oracle {
namespace img {

struct ImageError {
  std::string msg;
};
struct Info {
  std::string registry, name, path, tag, digest, reference, reference_with_tag, pointer;
};

inline const std::regex& reference_re() {
  static const std::string alnum = "[a-z0-9]+", sep = "(?:[._]|__|[-]+)";
  static const std::string comp = "(?:[a-zA-Z0-9]|[a-zA-Z0-9][a-zA-Z0-9-]*[a-zA-Z0-9])";
  static const std::string domain_name = comp + "(?:\\." + comp + ")*";
  static const std::string ipv6 = "\\[(?:[a-fA-F0-9:]+)\\]";
  static const std::string host = "(?:" + domain_name + "|" + ipv6 + ")";
  static const std::string domain_port = host + "(?::[0-9]+)?";
  static const std::string path_comp = alnum + "(?:" + sep + alnum + ")*";
  static const std::string remote = path_comp + "(?:/" + path_comp + ")*";
  static const std::string name = "(?:" + domain_port + "/)?" + remote;
  static const std::string tag = "[\\w][\\w.-]{0,127}";
  static const std::string digest = "[A-Za-z][A-Za-z0-9]*(?:[-_+.][A-Za-z][A-Za-z0-9]*)*[:][0-9A-Fa-f]{32,}";
  static const std::regex re("^(" + name + ")(?::(" + tag + "))?(?:@(" + digest + "))?$");
  return re;
}
inline const std::regex& name_re() {
  static const std::string alnum = "[a-z0-9]+", sep = "(?:[._]|__|[-]+)";
  static const std::string comp = "(?:[a-zA-Z0-9]|[a-zA-Z0-9][a-zA-Z0-9-]*[a-zA-Z0-9])";
  static const std::string domain_name = comp + "(?:\\." + comp + ")*";
  static const std::string ipv6 = "\\[(?:[a-fA-F0-9:]+)\\]";
  static const std::string domain_port = "(?:" + domain_name + "|" + ipv6 + ")(?::[0-9]+)?";
  static const std::string path_comp = alnum + "(?:" + sep + alnum + ")*";
  static const std::string remote = path_comp + "(?:/" + path_comp + ")*";
  static const std::regex re("^(?:(" + domain_port + ")/)?(" + remote + ")$");
  return re;
}
// go-digest Digest.Validate
inline bool digest_ok(const std::string& d) {
  const size_t i = d.find(':');
  if (i == std::string::npos || i == 0 || i + 1 == d.size()) return false;
  const std::string alg = d.substr(0, i), enc = d.substr(i + 1);
  size_t want = alg == "sha256" ? 64 : alg == "sha384" ? 96 : alg == "sha512" ? 128 : 0;
  if (!want || enc.size() != want) return false;
  for (char c : enc)
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  return true;
}
// GetImageInfo (infos.go:48-100); throws ImageError
inline Info get_image_info(const std::string& image) {
  std::string full = image;
  const size_t i = image.find('/');
  if (i == std::string::npos) {
    full = "docker.io/" + image;
  } else {
    const std::string first = image.substr(0, i);
    std::string lower = first;
    for (auto& c : lower) c = (char)tolower((unsigned char)c);
    if (first.find_first_of(".:") == std::string::npos && first != "localhost" && lower == first)
      full = "docker.io/" + image;
  }
  std::smatch m;
  if (!std::regex_match(full, m, reference_re())) throw ImageError{"bad image: " + full};
  const std::string name = m[1].str();
  if (name.size() > 255) throw ImageError{"repository name must not be more than 255 characters"};
  Info o;
  std::smatch nm;
  if (std::regex_match(name, nm, name_re()) && nm[1].matched) o.registry = nm[1].str(), o.path = nm[2].str();
  else o.path = name;
  o.tag = m[2].matched ? m[2].str() : "";
  o.digest = m[3].matched ? m[3].str() : "";
  if (!o.digest.empty() && !digest_ok(o.digest)) throw ImageError{"invalid digest"};
  o.name = o.path.substr(o.path.rfind('/') == std::string::npos ? 0 : o.path.rfind('/') + 1);
  if (o.digest.empty() && o.tag.empty()) o.tag = "latest";
  o.reference_with_tag = (o.registry.empty() ? "" : o.registry + "/") + o.path + ":" + o.tag;
  const std::string base = (o.registry.empty() ? "" : o.registry + "/") + o.path;
  o.reference = o.digest.empty() ? base + ":" + o.tag : base + "@" + o.digest;
  return o;
}

// ExtractImagesFromResource (image.go:183-229) with the standard extractors of the resource's
// kind: (container type, [(container name, info)]) in extractor order; throws ImageError
struct Extracted {
  std::string type;
  std::map<std::string, Info> infos;  // keyed by container name (the last one wins); JSON key order
};
inline std::vector<Extracted> extract_images(const JVal& res) {
  const JVal* k = res.get("kind");
  const std::string kind = k && k->t == JT::Str ? k->s : "";
  std::vector<std::string> prefix;
  if (kind == "Pod") prefix = {"spec"};
  else if (kind == "DaemonSet" || kind == "Deployment" || kind == "ReplicaSet" || kind == "ReplicationController" ||
           kind == "StatefulSet" || kind == "Job")
    prefix = {"spec", "template", "spec"};
  else if (kind == "CronJob") prefix = {"spec", "jobTemplate", "spec", "template", "spec"};
  else return {};
  std::vector<Extracted> out;
  for (const char* tag : {"initContainers", "containers", "ephemeralContainers"}) {
    Extracted ex;
    ex.type = tag;
    // extract(obj, path, "name", "image", fields = prefix + [tag, "*"])
    const JVal* obj = &res;
    std::string path;
    bool done = false;
    for (auto& f : prefix) {  // a missing field is nil: nothing to extract; a non-map: error
      if (obj->t != JT::Obj) throw ImageError{"invalid image config"};
      obj = obj->get(f.c_str());
      path += "/" + f;
      if (!obj || obj->t == JT::Null) {
        done = true;
        break;
      }
    }
    if (!done) {
      if (obj->t != JT::Obj) throw ImageError{"invalid image config"};
      const JVal* lst = obj->get(tag);
      path += std::string("/") + tag;
      if (lst && lst->t != JT::Null) {
        if (lst->t == JT::Obj) {
          // `*` over a map: every value (Go map order; the keys are sorted here, parity unpinned)
          std::vector<std::pair<std::string, const JVal*>> kv;
          for (auto& e : lst->o) kv.push_back({e.first, e.second.get()});
          std::sort(kv.begin(), kv.end(), [](auto& a, auto& b) { return a.first < b.first; });
          for (auto& e : kv) {
            if (!e.second || e.second->t == JT::Null) continue;
            if (e.second->t != JT::Obj) throw ImageError{"invalid image config"};
            const JVal* nm = e.second->get("name");
            if (!nm || nm->t != JT::Str) throw ImageError{"invalid key"};
            const JVal* im = e.second->get("image");
            if (!im || im->t != JT::Str) continue;
            std::string t = im->s;
            size_t a = t.find_first_not_of(" \t\n\v\f\r"), b = t.find_last_not_of(" \t\n\v\f\r");
            if (a == std::string::npos) continue;
            (void)b;
            Info in = get_image_info(im->s);
            in.pointer = path + "/" + e.first + "/image";
            ex.infos[nm->s] = in;
          }
        } else if (lst->t == JT::Arr) {
          for (size_t i = 0; i < lst->a.size(); ++i) {
            const JVal* c = lst->a[i].get();
            if (!c || c->t == JT::Null) continue;
            if (c->t != JT::Obj) throw ImageError{"invalid image config"};
            const JVal* nm = c->get("name");
            if (!nm || nm->t != JT::Str) throw ImageError{"invalid key"};
            const JVal* im = c->get("image");
            if (!im || im->t != JT::Str) continue;
            if (im->s.find_first_not_of(" \t\n\v\f\r") == std::string::npos) continue;
            Info in = get_image_info(im->s);
            in.pointer = path + "/" + std::to_string(i) + "/image";
            ex.infos[nm->s] = in;
          }
        } else {
          throw ImageError{"invalid type"};
        }
      }
    }
    if (!ex.infos.empty()) out.push_back(std::move(ex));
  }
  return out;
}

}  // namespace img
}  // namespace oracle
