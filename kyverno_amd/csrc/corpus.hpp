// Host-side columnar corpus: string dictionaries + SoA columns (see schema.h).
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "schema.h"

namespace kpe {

constexpr uint64_t KPE_NO_IMAGES = ~0ull;

// String dictionary: ids in first-intern order over one byte pool; the index is an
// open-addressing table of (hash, id + 1) slots keyed by the pool bytes (no per-string
// allocation, no std::string built for a lookup).
struct Dict {
  std::vector<char> bytes;
  std::vector<uint32_t> off{0};
  uint32_t intern(std::string_view s) {
    const uint64_t h = hash(s);
    if ((size() + 1) * 2 > slots.size()) grow(std::max<size_t>(64, slots.size() * 2));
    const size_t mask = slots.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& e = slots[i];
      if (e.id1 == 0) break;
      if (e.h == (uint32_t)(h >> 32) && at(e.id1 - 1) == s) return e.id1 - 1;
    }
    const uint32_t id = size();
    bytes.insert(bytes.end(), s.begin(), s.end());
    off.push_back((uint32_t)bytes.size());
    put(h, id);
    return id;
  }
  int64_t find(std::string_view s) const {
    if (slots.empty()) return -1;
    const uint64_t h = hash(s);
    const size_t mask = slots.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& e = slots[i];
      if (e.id1 == 0) return -1;
      if (e.h == (uint32_t)(h >> 32) && at(e.id1 - 1) == s) return (int64_t)(e.id1 - 1);
    }
  }
  void reserve(size_t n) {
    size_t cap = 64;
    while (cap < n * 2) cap *= 2;
    if (cap > slots.size()) grow(cap);
  }
  uint32_t size() const { return (uint32_t)(off.size() - 1); }
  std::string_view at(uint32_t i) const { return std::string_view(bytes.data() + off[i], off[i + 1] - off[i]); }
  // lookup with the string's hash already known (read-only: safe from several threads)
  int64_t find_h(std::string_view s, uint64_t h) const {
    if (slots.empty()) return -1;
    const size_t mask = slots.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& e = slots[i];
      if (e.id1 == 0) return -1;
      if (e.h == (uint32_t)(h >> 32) && at(e.id1 - 1) == s) return (int64_t)(e.id1 - 1);
    }
  }
  // Rebuild the index over every id from their hashes (hs[id]) on up to nth threads: the slot
  // table is cut into nth contiguous ranges, each thread places the ids whose home slot is in its
  // range and defers those whose probe would leave it; the deferred ones are placed afterwards.
  // The result is a valid linear-probing table (every id at or after its home slot, no empty slot
  // between), like inserting them one by one.
  void reindex(const std::vector<uint64_t>& hs, unsigned nth);  // flatten.cpp
  static uint64_t hash(std::string_view s) {  // 64-bit FNV-1a over 8-byte words, then a finalizer
    uint64_t h = 0xcbf29ce484222325ull ^ s.size();
    size_t i = 0;
    for (; i + 8 <= s.size(); i += 8) {
      uint64_t w;
      __builtin_memcpy(&w, s.data() + i, 8);
      h = (h ^ w) * 0x100000001b3ull;
    }
    for (; i < s.size(); ++i) h = (h ^ (unsigned char)s[i]) * 0x100000001b3ull;
    h ^= h >> 33, h *= 0xff51afd7ed558ccdull, h ^= h >> 33, h *= 0xc4ceb9fe1a85ec53ull, h ^= h >> 33;
    return h;
  }

 private:
  struct Slot {
    uint32_t h, id1;  // high hash bits, id + 1 (0: empty)
  };
  std::vector<Slot> slots;
  void put(uint64_t h, uint32_t id) {
    const size_t mask = slots.size() - 1;
    size_t i = h & mask;
    while (slots[i].id1) i = (i + 1) & mask;
    slots[i] = Slot{(uint32_t)(h >> 32), id + 1};
  }
  void grow(size_t cap) {
    slots.assign(cap, Slot{0u, 0u});
    for (uint32_t id = 0; id < size(); ++id) put(hash(at(id)), id);
  }
};

// String -> id index whose strings live elsewhere (the caller's text pool): open addressing over
// (hash, id + 1) slots like Dict, lookups by string_view with no allocation.
struct StrIndex {
  template <class Get>  // Get(id) -> std::string_view of that id's string
  int64_t find(std::string_view s, uint64_t h, Get get) const {
    if (slots.empty()) return -1;
    const size_t mask = slots.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& e = slots[i];
      if (e.id1 == 0) return -1;
      if (e.h == (uint32_t)(h >> 32) && get(e.id1 - 1) == s) return (int64_t)(e.id1 - 1);
    }
  }
  void insert(uint64_t h, uint32_t id) {
    if ((n + 1) * 2 > slots.size()) {  // grow: re-place every slot by its kept hash bits
      std::vector<Slot> old;
      old.swap(slots);
      slots.assign(std::max<size_t>(64, old.size() * 2), Slot{0u, 0u, 0u});
      for (const Slot& e : old)
        if (e.id1) place(e);
    }
    place(Slot{(uint32_t)(h >> 32), id + 1, (uint32_t)h});
    ++n;
  }
  static uint64_t hash(std::string_view s) {  // Dict's hash
    uint64_t h = 0xcbf29ce484222325ull ^ s.size();
    size_t i = 0;
    for (; i + 8 <= s.size(); i += 8) {
      uint64_t w;
      __builtin_memcpy(&w, s.data() + i, 8);
      h = (h ^ w) * 0x100000001b3ull;
    }
    for (; i < s.size(); ++i) h = (h ^ (unsigned char)s[i]) * 0x100000001b3ull;
    h ^= h >> 33, h *= 0xff51afd7ed558ccdull, h ^= h >> 33, h *= 0xc4ceb9fe1a85ec53ull, h ^= h >> 33;
    return h;
  }

 private:
  struct Slot {
    uint32_t h, id1, lo;  // high hash bits, id + 1 (0: empty), low hash bits (the slot index)
  };
  void place(const Slot& e) {
    const size_t mask = slots.size() - 1;
    size_t i = e.lo & mask;
    while (slots[i].id1) i = (i + 1) & mask;
    slots[i] = e;
  }
  std::vector<Slot> slots;
  size_t n = 0;
};

struct DeviceCorpus;  // defined in kpe_api.cpp

struct Corpus {
  int64_t n = 0;
  Dict dict[KPE_NUM_DOMAINS];
  // ---- resource rows (unstructured view, used by match/exclude) ----
  std::vector<uint32_t> r_flags, r_gvk, r_name, r_mns, r_nsa, r_nsl;
  std::vector<uint32_t> limit_rows;  // rows past a per-resource limit (R_LIMIT): all cells undecided
  std::vector<uint32_t> lab_off{0}, lab_k, lab_v;  // metadata.labels CSR
  std::vector<uint32_t> ann_off{0}, ann_k, ann_v;  // metadata.annotations CSR
  // ---- PSS pod view (typed decode of getSpec) ----
  std::vector<uint32_t> p_sc;
  std::vector<uint32_t> ctr_off{0};
  std::vector<uint32_t> vol_off{0}, vol_src;
  std::vector<uint32_t> sys_off{0}, sys_id;
  std::vector<uint32_t> pann_off{0}, pann_k, pann_v;  // pod-template metadata annotations
  std::vector<uint32_t> p_cold;  // cold (D_MISC), 4 per pod: seccomp type, seLinux type / user / role
  // ---- containers (visit order: initContainers, containers, ephemeralContainers) ----
  std::vector<uint32_t> c_sc;
  std::vector<uint64_t> c_add, c_drop;
  std::vector<uint32_t> c_name, c_image, c_sann;
  std::vector<uint32_t> c_sann_key;  // cold: D_ANNK id of the container's seccomp annotation key
  std::vector<uint32_t> c_sec_str, c_pm_str, c_selt_str, c_selu_str, c_selr_str;  // cold (D_MISC)
  std::vector<uint32_t> cport_off{0};
  std::vector<int32_t> cport_host;  // cold: hostPort of every port
  std::vector<uint32_t> cport_str;  // cold: D_MISC id of strconv.Itoa(hostPort), KPE_NO_STR for 0
  // ---- packed hot records for the PSS scan (schema.h) ----
  std::vector<uint32_t> rec;   // 4 words per pod
  std::vector<uint32_t> hdr;   // 4 words per 64 pods
  std::vector<uint32_t> crec;  // 2 words per container
  std::vector<uint32_t> pann_kv;  // (key, value) pairs of pod-template annotations
  std::vector<uint64_t> capset_add, capset_drop;
  std::unordered_map<std::string, uint32_t> capset_index;
  // ---- namespace label table (PolicyContext.NamespaceLabels) ----
  std::vector<uint32_t> nsl_off{0}, nsl_k, nsl_v;
  std::unordered_map<std::string, uint32_t> nsl_index;

  // ---- generic document tape + scalar table (pattern rules; schema.h DN_* / KpeScalar) ----
  bool has_docs = false;
  std::vector<uint32_t> doc;          // 2 words per entry (schema.h DN_*)
  std::vector<uint64_t> doc_off;      // root entry (absolute tape index) of each resource
  std::vector<uint64_t> img_off;      // root entry of each resource's `images` context map, or
                                      // KPE_NO_IMAGES (no images: the context has no `images`)
  std::vector<KpeScalar> scal;        // scalar table (ids 0/1/2 = null/false/true)
  std::vector<char> scal_text;        // compareString texts
  StrIndex scal_str;                  // string scalars by their text (scal_text)
  std::string_view scal_text_of(uint32_t id) const {
    return std::string_view(scal_text.data() + scal[id].text_off, scal[id].text_len);
  }
  std::unordered_map<int64_t, uint32_t> scal_int;
  std::unordered_map<uint64_t, uint32_t> scal_float;

  DeviceCorpus* dev = nullptr;
  int64_t bytes() const;
};

}  // namespace kpe
