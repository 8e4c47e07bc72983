// The typed pod view of getSpec (validate_pss.go:137-188): the fields the PSA checks read, as
// the flattener's typed decode extracts them (flatten.cpp Typed). Shared by the flattener and
// the PodSecurity message renderer (pss_msg.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "schema.h"

namespace kpe {

struct CtrView {
  std::string name, image;
  bool sc = false;
  uint32_t priv = TRI_UNSET, ape = TRI_UNSET, rnr = TRI_UNSET, rau = RAU_UNSET, whp = TRI_UNSET;
  bool caps = false;
  std::vector<std::string> add, drop;
  bool sec = false;
  std::string sec_type;
  bool pm = false;
  std::string pm_val;
  bool sel = false;
  std::string sel_type, sel_user, sel_role;
  std::vector<int32_t> hostports;
  void reset() { *this = CtrView(); }
};

struct PodView {
  bool hostnet = false, hostpid = false, hostipc = false;
  bool sc = false;
  uint32_t rnr = TRI_UNSET, rau = RAU_UNSET, whp = TRI_UNSET;
  bool sec = false;
  std::string sec_type;
  bool sel = false;
  std::string sel_type, sel_user, sel_role;
  bool os = false;
  std::string os_name;
  std::vector<std::string> sysctls;
  std::vector<uint32_t> vols;
  std::vector<CtrView> ctr[3];  // init, containers, ephemeral
  std::vector<std::pair<std::string, std::string>> ann;  // typed metadata annotations (map: unique keys)
  void reset() {
    hostnet = hostpid = hostipc = sc = sec = sel = os = false;
    rnr = TRI_UNSET;
    rau = RAU_UNSET;
    whp = TRI_UNSET;
    sec_type.clear();
    sel_type.clear();
    sel_user.clear();
    sel_role.clear();
    os_name.clear();
    sysctls.clear();
    vols.clear();
    for (auto& c : ctr) c.clear();
    ann.clear();
  }
};

// Typed decode of one resource (host): false when getSpec fails for it (a kind without a pod
// spec, or a JSON type mismatch).
bool typed_pod_view(const char* json, size_t len, PodView* out, std::string* kind);

}  // namespace kpe
