// Kernel argument structs shared by kernels.hip (device) and kpe_api.cpp (host).
#pragma once
#include <stdint.h>

#include "schema.h"

#define PRED_LOCAL 0x80000000u  // pred_word flag: bitset lives in the scan block's LDS

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
#define PK_NONEMPTY 8u  // '*'s around one '?' ("?*", "*?", "*?*"): one rune or more, i.e. non-empty
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
  uint32_t pat_len;
  const KpePat* pats;  // pattern records
  const PredJob* jobs;
  uint32_t njobs;
  uint32_t* out;
};


// Predicate references in the scan kernel's tables are resolved per binding to
// bitset locations: PRED_LOCAL | LDS word index, or a pbuf word index; PRED_NONE = absent.
#define PRED_NONE 0xFFFFFFFFu
#define KPE_RULE_CHUNK 32  // rules evaluated per transposed pass (one rule per lane)

// Rule lane record (uint4, one per rule, evaluated by one lane in the transposed pass):
//   x = handler | cv_class << 4 | match_mode << 16 | excl_mode << 18
//   y = match_f0 | match_nf << 24, z = excl_f0 | excl_nf << 24, w = pol_term (PRED_NONE: none)
#define RL_HANDLER(x) ((x) & 0xFu)
#define RL_CV(x) (((x) >> 4) & 0xFFFu)
#define RL_MATCH_MODE(x) (((x) >> 16) & 3u)
#define RL_EXCL_MODE(x) (((x) >> 18) & 3u)
#define RL_F0(y) ((y) & 0xFFFFFFu)
#define RL_NF(y) ((y) >> 24)

// NARROW programs (<= KPE_NARROW_TERMS distinct terms, <= KPE_NARROW_R rules): each
// lane evaluates every rule for its own resource from a term bit vector.
// Narrow rule record (uint4): x = handler | match_mode << 4 | excl_mode << 6 |
//   NR_APPLY_ONE | NR_NEW_POLICY | (pol_term + 1) << 16 (0: no namespaced-policy term),
//   y = cv_mask, z = match filters (RL_F0 / RL_NF), w = exclude filters;
//   fmask[f] = bit mask of the terms filter f ANDs.
#define KPE_NARROW_TERMS 32
#define KPE_NARROW_R 32
#define KPE_NARROW_FILTERS 64
#define KPE_TT_TERMS 8
#define NR_HANDLER(x) ((x) & 0xFu)
#define NR_MATCH_MODE(x) (((x) >> 4) & 3u)
#define NR_EXCL_MODE(x) (((x) >> 6) & 3u)
#define NR_APPLY_ONE (1u << 8)
#define NR_NEW_POLICY (1u << 9)
#define NR_POLTERM(x) ((x) >> 16)

// Per-wave PSS list staging (LDS): 128 container entries (uint2), 128 one-byte volume codes,
// 64 one-byte codes each for sysctls and pod annotations.
#define KPE_STAGE_CTR 128
#define KPE_STAGE_VOL 128  // pods average > 1 volume (C2: 1.4): two preloaded slots per lane
#define KPE_STAGE_SMALL 64
#define KPE_STAGE_WORDS ((KPE_STAGE_CTR * 8 + KPE_STAGE_VOL + 2 * KPE_STAGE_SMALL) / 4)

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
  uint32_t ntiles;            // ceil(n / 64); hdr has ntiles + 1 entries
  const uint32_t* zero_page;  // >= 64 zero bytes: source of the loads of unneeded columns
  const uint32_t* capsets;    // capability-set dictionary: 4 words (add lo/hi, drop lo/hi) per set
  uint32_t ncapsets;
  uint32_t nctr_total, nvol_total, nsys_total, npann_total;  // list lengths (load clamping)
  // program tables; predicate fields resolved to bitset locations (binding copies)
  const KpeRule* rules;
  const uint32_t* rule_lanes;  // packed rule lane records (RL_*)
  const uint32_t* narrow_rules;  // NARROW: 4 words per rule (NR_*)
  const uint32_t* rule_exc;      // KpeRule::exc per rule (XE_*), or null: no PolicyExceptions
  const uint32_t* fmask;         // NARROW: term mask per filter
  uint32_t nfilters;
  // NARROW truth-table fast path (tt_lds != PRED_NONE: <= KPE_TT_TERMS terms, no ApplyOne):
  // every block tabulates matched-rule masks for all 2^nterms term vectors in LDS at
  // tt_lds; narrow_cls holds (cv_mask, rule mask) per distinct PSS version set.
  uint32_t tt_lds, ncls, pss_rules, err_rules, pat_rules;
  const uint32_t* narrow_cls;
  const KpeFilter* filters;
  const uint32_t* fterms;
  const KpeTerm* terms;
  const KpeKindSel* kindsels;
  const KpeAnnPair* annpairs;
  const KpeSelector* selectors;
  const KpeSelReq* selreqs;
  const uint32_t* cv_classes;  // distinct PSS cv_masks (rule.cv_class indexes them)
  uint32_t filt_lds, fterm_lds, nfterms;  // filters / filter terms staged in LDS at these word
                                          // offsets (filt_lds == PRED_NONE: read from HBM)
  uint32_t nrules, nterms, ncv, any_apply_one;
  // predicate bitsets: pbuf[0, blob_words) = small-domain bitsets, copied into LDS by
  // every block (same word indices); the rest = large-domain bitsets (HBM/L2)
  const uint32_t* pbuf;
  uint32_t blob_words;
  // Fused dictionary pass (npairs > 0): every block evaluates the small-domain
  // predicates itself from the binding's fuse image, copied into LDS at fuse_lds:
  // [pair table (uint2 per (string, pattern))][KpePat table][pattern bytes][strings].
  // Pair: x = string LDS byte address | length << 20; y = pattern index |
  // bitset word << 12 | bit << 27 (OR-ed in with an LDS atomic).
  const uint32_t* fuse;
  uint32_t fuse_words, fuse_lds, npairs;
  uint32_t fuse_pats, fuse_patb;  // LDS word index of the pattern table / pattern bytes
  uint32_t wave_lds, wave_words;  // per-wave LDS regions: dyn[wave_lds + wv * wave_words ...]
  // fixed PSS predicates (resolved locations)
  uint32_t pp_apparmor_key, pp_apparmor_ok, pp_seccomp_pod_key, pp_seccomp_ann_ok;
  uint32_t pp_caps_ok, pp_cap_nbs, pp_cap_all, pp_sysctl0, pp_sysctl1, pp_sysctl2;
  uint32_t cv_union, need;
  // Prologue image (kpe_scan_kernel<..., PREP = true>, one block per binding, writes it): a
  // copy of the scan block's LDS words [0, pimg_words) = [predicate bitsets (blob_words)]
  // [truth table at tt_lds][kind table at kt_lds][capability-set bits (bytes) at capb_lds].
  // Every scan block copies it into LDS with straight 16-byte loads. Null: every scan block
  // computes its own prologue (the fuse area then sits at fuse_lds, after the wave regions).
  uint32_t* pimg;
  uint32_t pimg_words, capb_lds;
  // LEAN scans (kind-only match terms): kt[kind id] = matched-rule mask (PRED_NONE: no table)
  uint32_t kt_lds, nkinds;
  const uint32_t* psum;  // PSUM general scan: per-pod scan records (3 words per pod: pod word, failing versioned checks, kind << 16)
  // Selector requirement masks (selm bit 0: label selectors, bit 1: namespaceSelectors; built
  // per binding by kpe_selmask_kernel). Requirement q of a selector is bit qbit + q. Label
  // selectors: sel_km[key id] = {requirements whose key glob holds, wildcard requirements whose
  // key is a valid qualified name} and sel_vm[value id] = {requirements whose value set holds,
  // wildcard requirements whose value is a valid label value}, 64-bit each, folded per row over
  // its labels in order; sm_* = the requirements of each operator class. namespaceSelectors:
  // ns_q[namespace row] = the requirements that hold on that namespace's labels (row ns_none:
  // a resource without a namespace row).
  const uint4* sel_km;
  const uint4* sel_vm;
  const uint64_t* ns_q;
  uint32_t selm, ns_none, nlabk, nlabv;
  // sel_km then sel_vm staged in each scan block's LDS at this word offset (the label fold then
  // reads LDS, not L2), or PRED_NONE
  uint32_t selt_lds, selt_pad;
  // kind terms (T_KSLOT): LDS word offset of the corpus's distinct GVKs (ascending, nkslot_g of
  // them, padded to an even count) followed by each one's 64-bit kind-term mask; PRED_NONE: none
  uint32_t kslot_lds, nkslot_g;
  const uint32_t* kslot_tab;  // the table in HBM (copied by every scan block)
  uint64_t sm_pos, sm_wild, sm_notin, sm_exists, sm_dne;
  // outputs
  uint8_t* verdicts;  // n x nrules
  uint32_t* masks;    // n x nrules failing versioned checks (bit v = KpeCheckVersion v) or null
};

// The PSA dictionary codes of a corpus (lean.inl kpe_psa_codes_kernel): the four dictionaries it
// codes (PsaCodeArgs::dict_*[PSD_*]) and the fixed sets of the PSA library (pss_fixed.hpp) as bits
// of a string's set-hit word (the fixed table's set numbers).
#define PSD_CAP 0
#define PSD_SYSCTL 1
#define PSD_ANNK 2
#define PSD_ANNV 3
#define PSF_CAPS_OK 0
#define PSF_CAP_NBS 1
#define PSF_CAP_ALL 2
#define PSF_SYSCTL0 3
#define PSF_SYSCTL1 4
#define PSF_SYSCTL2 5
#define PSF_APPARMOR_KEY 6
#define PSF_SECCOMP_POD_KEY 7
#define PSF_APPARMOR_OK 8
#define PSF_SECCOMP_ANN_OK 9
// Fixed-set table (psa_fixed_table in kpe_api.cpp), 32-bit words:
//   [0] exact entries E, [1] prefix entries X, [2 + len] (first | end << 16) of the exact entries
//   of byte length len < KPE_PSF_MAXLEN (sorted by length), then E + X entries of 2 words
//   {set | prefix << 7 | len << 8, word index of the literal}, then the literals (4-byte padded).
// A prefix entry is a literal followed by one trailing '*' (go-wildcard: a byte-prefix match).
#define KPE_PSF_MAXLEN 64u
#define KPE_PSF_ENT0 (2u + KPE_PSF_MAXLEN)
// Code bytes of a corpus: [capability sets | sysctls | annotation keys | annotation values], each
// part 4-byte aligned (PsaCodes offsets). Capability set: CS_* bits (kernels.hip) | 8: the set
// holds a capability id >= 64 (never read: such a resource is a per-resource limit row); sysctl:
// bit v = outside version v's allowed set; annotation key: bit 0 AppArmor container key, bit 1
// pod seccomp key; annotation value: bit 0 allowed AppArmor profile, bit 1 allowed seccomp profile.
struct PsaCodes {
  uint32_t ncapsets, nsysd, nannk, nannv;  // entries of each part
  uint32_t o_sys, o_annk, o_annv, bytes;   // byte offsets of the parts, total bytes
};
struct PsaCodeArgs {
  const uint8_t* dict_bytes[4];
  const uint32_t* dict_off[4];
  uint32_t dict_n[4];
  const uint32_t* capsets;  // (add lo, add hi, drop lo, drop hi) capability-id masks per set
  const uint32_t* fixed;    // fixed-set table (above)
  uint32_t fixed_words, pad_;
  PsaCodes L;
  uint8_t* codes;           // out
};
// kpe_psum_kernel (the general scan's per-pod PSA records, rebuilt by every evaluation of a
// podSecurity program that is not LEAN, and kpe_corpus_psa_summary)
struct PsumArgs {
  int64_t n;
  uint32_t ntiles, pad_;
  const uint32_t *rec, *hdr, *crec, *vol_src, *sys_id, *pann_kv, *c_sann;
  const uint8_t* codes;  // PsaCodeArgs::codes
  PsaCodes L;
  uint32_t* psum;        // out: 3 words per pod (pod word, failing versioned checks, kind << 16)
  uint32_t* summ;        // out (or null): 2 words per pod (OR of container states, codes; schema.h PS_*)
};

// kpe_selmask_kernel: the selector requirement masks of a binding (ScanArgs::sel_km / sel_vm /
// ns_q) from the predicate bitsets (prologue image for local ones, pbuf for the rest).
struct SelMaskArgs {
  const uint32_t* pimg;      // prologue image: local bitsets at their LDS word index
  const uint32_t* pbuf;      // global bitsets
  const KpeSelReq* reqs;     // resolved requirement records (binding copy)
  const uint32_t* rq;        // label-selector requirement of bit b (selreqs index), nrq entries
  const uint32_t* nq;        // namespaceSelector requirement of bit b, nnq entries
  uint32_t nrq, nnq, nlabk, nlabv, nrows;  // nrows: namespace label table rows (ns_q has nrows + 1)
  uint32_t pad_;
  const uint32_t *nsl_off, *nsl_k, *nsl_v;
  uint4* km;                 // out: nlabk entries
  uint4* vm;                 // out: nlabv entries
  uint64_t* nsq;             // out: nrows + 1 entries
};

// kpe_lean6_kernel: the LEAN evaluation of one or more bound shards of one program in one launch
// (kpe_evaluate_async: one shard; kpe_evaluate_batch_async: up to KPE_LEAN_BATCH). Passed by
// value (< 4 KiB of kernel arguments): block b of the grid belongs to the shard s with
// blk0[s] <= b < blk0[s + 1]. Every launch reads each pod's record and its container, volume,
// sysctl and annotation lists: nothing per pod is carried over from an earlier evaluation.
#define KPE_LEAN_BATCH 24
struct LeanShard {
  const uint32_t *rec, *hdr, *crec, *vol, *sys, *pann, *sann;  // the corpus's PSS columns
  const uint8_t* codes;   // the corpus's PSA dictionary codes (PsaCodeArgs::codes)
  const uint32_t* kt;     // the binding's kind table: matched-rule mask per kind id (prologue image)
  uint8_t* verdicts;      // n x R
  uint32_t* masks;        // n x R failing versioned checks, or null
  uint32_t n, nkinds, nctr, nvol, nsys, npann;
  PsaCodes L;
};
struct LeanBatchArgs {
  uint32_t nshards, nrules, ncls, cv_union, pss_rules, err_rules, pat_rules, need;
  uint32_t kt_words, code_words, wave_words, tpw;  // LDS: kind table, codes (LC), per-wave stage
  const uint32_t* narrow_cls;  // (cv classes, rule mask) pairs of the program
  uint32_t blk0[KPE_LEAN_BATCH + 1];  // a block covers 4 * tpw tiles of 64 pods
  LeanShard sh[KPE_LEAN_BATCH];
};
// Per-wave LDS stage of kpe_lean6_kernel: a tile's staged list items (container codes as uint2,
// volume / sysctl / annotation codes as bytes); items past these counts are loaded again.
#define KPE_L6_CTR 128u
#define KPE_L6_VOL 128u
#define KPE_L6_SMALL 64u
#define KPE_L6_STAGE_BYTES (KPE_L6_CTR * 8u + KPE_L6_VOL + 2u * KPE_L6_SMALL)

// kpe_pattern_kernel arguments (device-resident, one copy per binding)
struct PatArgs {
  int64_t n;
  uint32_t R, npr;                 // rules per row, pattern rules
  const uint32_t* doc;             // document tape (2 words per node)
  const uint64_t* doc_off;         // first node of each resource
  const uint32_t* perm;            // lane -> row: rows by descending tape size (wave-uniform walk lengths)
  const KpeScalar* scal;
  const uint8_t* scal_text;
  const KpePNode* nodes;
  const uint4* members;            // resolved per binding (names -> D_KEY ids + 1)
  const uint32_t* lists;
  const KpeLeaf* leaves;
  const KpeCond* conds;
  const KpePat* pats;              // operand records
  const uint8_t* pat_bytes;
  const uint32_t* roots;           // (node, anchor slots) pairs
  const KpePatRule* rules;
  const uint32_t* col2pr;          // verdict column -> C2P_MAKE(pattern rule index + 1, memo slot), or null
  const uint32_t* pbuf;            // glob member-name bitsets (HBM)
  // pattern variables: per-row values written by kpe_cond_kernel (pvals[row * nvars + slot]),
  // template pieces / texts, and the condition-program constants a value may name
  const uint2* pvals;
  uint32_t nvars, pad_;
  const uint2* ptmpl;
  const uint8_t* ttext;
  const KpeScalar* ctab;
  const uint8_t* ctext;
  uint8_t* verdicts;
  // Leaf table (kpe_leaf_table_kernel, once per binding): a leaf whose result depends only on
  // the scalar (no variables) has a slot, lslot[leaf] (KPE_NO_LSLOT: none), and bit sid of
  // ltab[slot * ltab_words ...] is pattern.Validate of scalar sid against it. Null: no table.
  const uint32_t* lslot;
  uint32_t* ltab;
  uint32_t ltab_words, nkeyd;  // nkeyd: strings of the member-name dictionary (D_KEY)
  // the member-name dictionary (D_KEY): keys named by substituted key templates (PMF_VKEY) are
  // looked up by text
  const uint8_t* key_bytes;
  const uint32_t* key_off;
  // table sizes and an error word: read only by KPE_PATVM_CHECK builds (bounds flags)
  uint32_t nnodes, nmembers, nlists, nleaves, nconds, npats, nroots, npbuf;
  uint64_t nscal, ndoc;
  uint32_t* err;
  // memo slot s's representative pattern rule (any rule of the slot: they share the pattern), or
  // ~0u for an unused slot; kpe_pattern_kernel evaluates a row's slots in slot order
  uint32_t slot_rule[KPE_PAT_MEMO];
  // set to 1 by kpe_pattern_kernel when it marks a cell KPE_DEEP_ (cleared before every launch);
  // kpe_pattern_deep_kernel returns at once while it is 0 (no 1-byte-per-cell rescan); null: none
  uint32_t* deep_any;
};

// kpe_cond_kernel arguments (device-resident, one copy per binding)
struct CondArgs {
  int64_t n;
  uint32_t R, ncr;                 // rules per row, condition rules
  const uint32_t* doc;             // document tape (2 words per entry)
  const uint64_t* doc_off;         // root entry of each resource
  const uint64_t* img_off;         // root entry of each resource's images map (KPE_NO_IMAGES: none)
  const uint32_t* perm;            // lane -> row (PatArgs::perm)
  const KpeScalar* scal;
  const uint8_t* scal_text;
  const uint8_t* key_bytes;        // D_KEY dictionary (keys(@) results)
  const uint32_t* key_off;
  const uint2* ops;                // condition program (program.hpp CondProgram)
  const KpeCExpr* exprs;
  const KpeVTmpl* tmpls;
  const KpeCCond* conds;
  const KpeCBlock* blocks;
  const KpeCForeach* fes;
  const KpeCRule* rules;
  const KpeScalar* ctab;           // constants
  const uint8_t* ctext;
  const uint32_t* clist;
  const uint32_t* fkeys;           // field index -> D_KEY id + 1 (0: absent from the corpus)
  const KpeLeaf* leaves;           // InRange values of set operators (KpeCCond::aux): string-pattern
  const KpeCond* pconds;           // leaves of the pattern program's tables
  const KpePat* pats;
  const uint8_t* pat_bytes;
  const PatArgs* pat;              // the pattern program (foreach pattern / anyPattern entries)
  const uint2* tpieces;            // VT_TMPL pieces (CondProgram::tpieces)
  uint32_t txt, pad2_;             // 1: VT_TMPL templates exist (the kernel's LDS text slots)
  const KpePVar* pvars;            // pattern variable slots (query template, use flags)
  uint2* pvals;                    // their per-row values (PatArgs::pvals), or null
  uint32_t nvars, nmsg;             // pattern variable slots; condition trace slots per row
  uint8_t* verdicts;
  uint32_t* mtrace;                // N x nmsg condition traces (schema.h CT_*), or null
};

// kpe_pssx_kernel arguments (device-resident, one copy per binding): podSecurity rules with
// exclusions, after the scan wrote their plain PSS verdicts.
struct PssxArgs {
  int64_t n;
  uint32_t R, nxr;
  const KpeXRule* rules;
  const KpeXExcl* excl;            // predicate fields resolved to pbuf word indices
  const uint32_t* rec;             // pod records (x = pod word)
  const uint32_t *ctr_off, *vol_off, *sys_off, *pann_off;  // per-pod list offsets (n + 1)
  const uint32_t* crec;            // container records (state bitmap, capset | type << 16)
  const uint32_t* capsets;         // 4 words per capability set
  const uint32_t *c_name, *c_image, *c_sann, *c_sann_key;
  const uint32_t *c_sec_str, *c_pm_str, *c_selt_str, *c_selu_str, *c_selr_str;
  const uint32_t *cport_off, *cport_str;
  const uint32_t *vol_src, *sys_id, *pann_k, *pann_v;
  const uint32_t* p_cold;          // 4 words per pod (D_MISC ids)
  const uint32_t *misc_off, *annv_off, *sysd_off;  // dictionary offsets (empty-string tests)
  const uint32_t* ann_norm;        // D_ANNK id -> normalised-key id
  const uint32_t* rf_ann;          // XRF_ANN text index -> normalised-key id (KPE_NO_STR: none)
  uint32_t key_pod_sec, key_fake_sec;  // D_ANNK ids of the pod / "fake" container seccomp keys
  const uint32_t* pbuf;            // predicate bitsets (global locations)
  uint32_t pp_apparmor_key, pp_apparmor_ok, pp_seccomp_ok, pp_caps_ok, pp_nbs, pp_all;
  uint32_t pp_sysctl[3];
  uint8_t* verdicts;
  uint32_t* masks;                 // n x R failing versioned checks, or null
};
