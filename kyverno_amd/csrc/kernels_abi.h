// Kernel argument structs shared by kernels.hip (device) and kpe_api.cpp (host).
#pragma once
#include <stdint.h>

#include "schema.h"

#define PRED_LOCAL 0x80000000u  // pred_word flag: bitset lives in the scan block's LDS
#define KPE_SMALL_R 64          // rules counted via LDS ballots + per-block partials

// ScanArgs.need: which columns / lists the compiled program reads
#define NEED_FLAGS (1u << 0)
#define NEED_GVK (1u << 1)
#define NEED_CAPS (1u << 2)
#define NEED_SANN (1u << 3)
#define NEED_VOL (1u << 4)
#define NEED_SYS (1u << 5)
#define NEED_PANN (1u << 6)
#define NEED_NSA (1u << 7)
#define NEED_LAB (1u << 8)   // resource labels (CSR) for label selectors
#define NEED_NSL (1u << 9)   // namespace label table for namespaceSelector
#define NEED_NAME (1u << 10) // r_name (name / names terms)
#define NEED_MNS (1u << 11)  // r_mns (namespaces terms)

// Pattern classes (host-classified go-wildcard patterns; '?' or an inner '*' => PK_GLOB)
#define PK_ANY 0u       // "*"
#define PK_EXACT 1u     // no wildcard
#define PK_PREFIX 2u    // "lit*"
#define PK_SUFFIX 3u    // "*lit"
#define PK_CONTAINS 4u  // "*lit*"
#define PK_GLOB 5u      // general: full pattern text
#define PK_QNAME 6u     // validation.IsQualifiedName (apimachinery v0.29.1, label keys)
#define PK_LABVAL 7u    // validation.IsValidLabelValue
struct KpePat {
  uint32_t kind, off, len, pad;  // literal (or full pattern for PK_GLOB) = pat_bytes[off, off+len)
};

struct PredJob {
  uint32_t domain;
  uint32_t pat0, npat;  // patterns [pat0, pat0+npat) of the pattern table
  uint32_t out_word;    // first output word
  uint32_t blk0;        // first block of this job
};

struct PredArgs {
  const uint8_t* dict_bytes[KPE_NUM_DOMAINS];
  const uint32_t* dict_off[KPE_NUM_DOMAINS];
  uint32_t dict_n[KPE_NUM_DOMAINS];
  const uint8_t* pat_bytes;
  const KpePat* pats;
  const PredJob* jobs;
  uint32_t njobs;
  uint32_t* out;
};


struct ScanArgs {
  int64_t n;
  // resource rows (unstructured view) — read by match terms
  const uint32_t *r_gvk, *r_name, *r_mns, *r_nsa, *ann_off, *ann_k, *ann_v;
  const uint32_t *lab_off, *lab_k, *lab_v;           // metadata.labels CSR
  const uint32_t *r_nsl, *nsl_off, *nsl_k, *nsl_v;   // namespace label table row per resource
  // PSS hot records (schema.h): pod records, wave headers, container records
  const uint32_t* rec;        // 4 words per pod
  const uint32_t* hdr;        // 4 words per 64 pods
  const uint32_t* crec;       // 2 words per container
  const uint32_t* vol_src;    // per volume: VolumeSource presence mask
  const uint32_t* sys_id;     // per sysctl: D_SYSCTL id
  const uint32_t* pann_kv;    // per pod-template annotation: (D_ANNK id, D_ANNV id)
  const uint32_t* c_sann;     // per container: value id of its seccomp annotation (cold)
  const uint32_t* capsets;    // capability-set dictionary: 4 words (add lo/hi, drop lo/hi) per set
  uint32_t ncapsets;
  uint32_t nctr_total, nvol_total, nsys_total, npann_total;  // list lengths (load clamping)
  // program tables (wave-uniform: read with scalar loads)
  const KpeRule* rules;
  const KpeFilter* filters;
  const uint32_t* fterms;
  const KpeTerm* terms;
  const KpeKindSel* kindsels;
  const KpeAnnPair* annpairs;
  const KpeSelector* selectors;
  const KpeSelReq* selreqs;
  uint32_t nrules, nterms;
  // predicate bitsets: pbuf[0, npreds) = directory (PRED_LOCAL | LDS word index, or pbuf
  // word index); pbuf[npreds, blob_words) = small-domain bitsets, copied into LDS by every
  // block (same word indices); the rest = large-domain bitsets read from HBM/L2.
  const uint32_t* pbuf;
  uint32_t blob_words, npreds;
  uint32_t tm_lds;  // LDS word offset of the per-wave term-mask table (nterms x u64 per wave)
  int32_t pp_apparmor_key, pp_apparmor_ok, pp_seccomp_pod_key, pp_seccomp_ann_ok;
  int32_t pp_caps_ok, pp_cap_nbs, pp_cap_all, pp_sysctl0, pp_sysctl1, pp_sysctl2;
  uint32_t cv_union, need;
  // outputs
  uint8_t* verdicts;                 // n x nrules
  uint32_t* masks;                   // n x nrules or null
  uint32_t* counts_part;             // blocks x nrules x 6 (nrules <= KPE_SMALL_R)
  unsigned long long* counts_global; // nrules x 6 (nrules > KPE_SMALL_R)
};
