// Columnar encoding shared by the host flattener and the CDNA4 kernels.
//
// One resource = one row. String fields are dictionary-encoded per domain
// (kpe::Dict); enum-typed K8s fields with a closed set of legal values are
// stored as small codes (+ an OTHER code) in packed words; free-form strings a
// rule may need verbatim stay as dictionary ids in "cold" columns that only the
// exclusion/message paths read. All evaluation (which values are allowed, per
// check and per PSS version, glob/prefix predicates, match/exclude) happens on
// the device; the host only encodes.
#pragma once
#include <stdint.h>

// ---- string domains ------------------------------------------------------------
enum KpeDomain {
  D_GROUP = 0,   // apiVersion group ("" for core)
  D_VERSION,     // apiVersion version
  D_KIND,        // kind
  D_NAME,        // metadata.name, or metadata.generateName when name is empty (utils/match.go:78-81)
  D_NS,          // metadata.namespace (and the name of Namespace objects, utils/match.go:18-22)
  D_LABK,        // metadata.labels keys
  D_LABV,        // metadata.labels values
  D_ANNK,        // annotation keys (resource metadata and pod-template metadata)
  D_ANNV,        // annotation values
  D_CAP,         // capability names (<= 64 distinct per corpus: masks are u64)
  D_SYSCTL,      // pod securityContext.sysctls[].name
  D_IMAGE,       // container images
  D_CNAME,       // container names
  D_MISC,        // seccomp type / procMount / seLinux strings (cold, exclusions)
  D_KEY,         // object member names of the generic document tape (pattern rules)
  KPE_NUM_DOMAINS
};

#define KPE_NO_STR 0xFFFFFFFFu

// ---- resource word r_flags -------------------------------------------------------
#define R_CLASS_MASK 0x3u      // PSS spec class: validate_pss.go:137-188
#define R_CLASS_POD 0u
#define R_CLASS_CONTROLLER 1u  // DaemonSet, Deployment, Job, StatefulSet, ReplicaSet, ReplicationController
#define R_CLASS_CRONJOB 2u
#define R_CLASS_OTHER 3u       // "could not find correct resource type" => RuleError
#define R_DECODE_ERR (1u << 2) // typed json.Unmarshal would fail => RuleError
#define R_IS_NAMESPACE (1u << 3)
#define R_LABELS_NIL (1u << 4)  // unstructured NestedStringMap failed => nil map
#define R_ANNOT_NIL (1u << 5)
#define R_LIMIT (1u << 6)       // a per-resource encoding limit (e.g. > 255 containers): every cell of
                                // the row is KPE_UNDECIDED_ (Corpus::limit_rows)
#define R_CTX_ERR (1u << 7)     // NewPolicyContext fails (AddImageInfos: an invalid image or container
                                // entry): the reference gives no response; every cell KPE_UNDECIDED_

// r_gvk = kind_id | version_id << 12 | group_id << 22
#define GVK_KIND(x) ((x) & 0xFFFu)
#define GVK_VER(x) (((x) >> 12) & 0x3FFu)
#define GVK_GRP(x) ((x) >> 22)

// ---- tri-state / enum codes ----------------------------------------------------
#define TRI_UNSET 0u
#define TRI_FALSE 1u
#define TRI_TRUE 2u
#define RAU_UNSET 0u
#define RAU_NONZERO 1u
#define RAU_ZERO 2u
#define SECCOMP_NONE 0u        // seccompProfile == nil
#define SECCOMP_RUNTIMEDEFAULT 1u
#define SECCOMP_LOCALHOST 2u
#define SECCOMP_UNCONFINED 3u
#define SECCOMP_OTHER 4u       // any other type string (incl. "")
#define PROCMOUNT_UNSET 0u
#define PROCMOUNT_DEFAULT 1u
#define PROCMOUNT_OTHER 2u
#define SEL_NONE 0u            // seLinuxOptions == nil
#define SEL_EMPTY 1u           // type ""
#define SEL_CONTAINER_T 2u
#define SEL_CONTAINER_INIT_T 3u
#define SEL_CONTAINER_KVM_T 4u
#define SEL_OTHER 5u
#define OS_NONE 0u
#define OS_WINDOWS 1u
#define OS_OTHER 2u

// ---- pod word p_sc (pod-level securityContext and spec flags) ---------------------
#define P_SC_PRESENT (1u << 0)
#define P_HOSTNET (1u << 1)
#define P_HOSTPID (1u << 2)
#define P_HOSTIPC (1u << 3)
#define P_RNR_SH 4      // tri
#define P_RAU_SH 6      // RAU_*
#define P_SECCOMP_SH 8  // 3 bits
#define P_SEL_SH 11     // 3 bits
#define P_SEL_USER (1u << 14)
#define P_SEL_ROLE (1u << 15)
#define P_WHP_SH 16     // tri
#define P_OS_SH 18      // OS_*
#define FIELD(w, sh, bits) (((w) >> (sh)) & ((1u << (bits)) - 1u))

// ---- packed hot records of the PSS scan ------------------------------------------------
// Pod record (uint4, one dwordx4 per lane):
//   x = pod word p_sc (bits 0..19) | R_CLASS << PR_CLASS_SH | PR_DECODE_ERR
//   y = r_gvk, z = list counts (PRC_*), w = r_nsa (namespace id)
// Wave header (uint4 per 64 pods, plus one sentinel): first container / volume / sysctl /
//   pod-annotation index of the tile; tile t's lists are [hdr[t], hdr[t+1]) and a lane's
//   own offsets are the exclusive wave scan of the counts.
// Container record (uint2): x = container state bitmap (CX_*), y = capability-set id
//   (dictionary of distinct (add, drop) capability masks) | type << 16.
#define PR_CLASS_SH 20
#define PR_DECODE_ERR (1u << 22)
#define PRC_CTR(z) ((z) & 0xFFu)
#define PRC_VOL(z) (((z) >> 8) & 0xFFu)
#define PRC_SYS(z) (((z) >> 16) & 0xFFu)
#define PRC_PANN(z) ((z) >> 24)
#define KPE_MAX_LIST 255u  // per-pod containers / volumes / sysctls / annotations (KPE_E_LIMIT beyond)
#define KPE_MAX_CAPSETS 2048u

// ---- container word c_sc -----------------------------------------------------------
#define C_SC_PRESENT (1u << 0)
#define C_PRIV_SH 1        // tri
#define C_APE_SH 3         // tri
#define C_RNR_SH 5         // tri
#define C_RAU_SH 7         // RAU_*
#define C_SECCOMP_SH 9     // 3 bits
#define C_PROCMOUNT_SH 12  // 2 bits
#define C_SEL_SH 14        // 3 bits
#define C_SEL_USER (1u << 17)
#define C_SEL_ROLE (1u << 18)
#define C_WHP_SH 19        // tri
#define C_CAPS_PRESENT (1u << 21)
#define C_TYPE_SH 22       // 0 initContainers, 1 containers, 2 ephemeralContainers
#define C_HOSTPORT_SH 24   // 4 bits: number of ports with hostPort != 0 (saturating at 15)

// ---- container state bitmap (crec.x of the scan's container record) ------------------
// One bit per STATE of each securityContext field the PSA checks read (a bitmap
// index of c_sc: exactly one bit of every group is set). The PSA container checks are
// all "some container is in state s", so a pod's OR of its containers' bitmaps is a
// sufficient statistic: the scan ORs 1..255 records and decides the checks once per pod.
#define CX_PRIV_T (1u << 0)
#define CX_PRIV_F (1u << 1)
#define CX_PRIV_U (1u << 2)
#define CX_APE_T (1u << 3)
#define CX_APE_F (1u << 4)
#define CX_APE_U (1u << 5)
#define CX_RNR_T (1u << 6)
#define CX_RNR_F (1u << 7)
#define CX_RNR_U (1u << 8)
#define CX_RAU_NZ (1u << 9)
#define CX_RAU_Z (1u << 10)
#define CX_RAU_U (1u << 11)
#define CX_SEC_NONE (1u << 12)    // seccompProfile == nil
#define CX_SEC_RD (1u << 13)      // RuntimeDefault
#define CX_SEC_LH (1u << 14)      // Localhost
#define CX_SEC_UNC (1u << 15)     // Unconfined
#define CX_SEC_OTHER (1u << 16)   // any other type string
#define CX_PM_U (1u << 17)        // procMount unset
#define CX_PM_DEFAULT (1u << 18)
#define CX_PM_OTHER (1u << 19)
#define CX_SEL_NONE (1u << 20)    // seLinuxOptions == nil
#define CX_SEL_OK (1u << 21)      // type "", container_t, container_init_t, container_kvm_t
#define CX_SEL_OTHER (1u << 22)   // any other type
#define CX_SEL_USER (1u << 23)    // user != "" (only with seLinuxOptions set)
#define CX_SEL_ROLE (1u << 24)    // role != ""
#define CX_WHP_T (1u << 25)       // windowsOptions.hostProcess == true
#define CX_WHP_NT (1u << 26)      // hostProcess unset or false
#define CX_CAPS (1u << 27)        // capabilities present
#define CX_NOCAPS (1u << 28)
#define CX_HOSTPORT (1u << 29)    // some port with hostPort != 0
#define CX_NOHOSTPORT (1u << 30)
#define CX_SC (1u << 31)          // securityContext present
// crec.y = capability-set id (bits 0..15) | container type (C_TYPE) << 16
#define CY_CAPSET(y) ((y) & 0xFFFFu)

// ---- volumes: vol_src bit i = corev1.VolumeSource field i present (declaration order) ----
#define KPE_NUM_VOLUME_SOURCES 29
#define VS_HOSTPATH 0
#define VS_EMPTYDIR 1
#define VS_GCEPD 2
#define VS_AWSEBS 3
#define VS_GITREPO 4
#define VS_SECRET 5
#define VS_NFS 6
#define VS_ISCSI 7
#define VS_GLUSTERFS 8
#define VS_PVC 9
#define VS_RBD 10
#define VS_FLEXVOLUME 11
#define VS_CINDER 12
#define VS_CEPHFS 13
#define VS_FLOCKER 14
#define VS_DOWNWARDAPI 15
#define VS_FC 16
#define VS_AZUREFILE 17
#define VS_CONFIGMAP 18
#define VS_VSPHERE 19
#define VS_QUOBYTE 20
#define VS_AZUREDISK 21
#define VS_PHOTONPD 22
#define VS_PROJECTED 23
#define VS_PORTWORX 24
#define VS_SCALEIO 25
#define VS_STORAGEOS 26
#define VS_CSI 27
#define VS_EPHEMERAL 28
// restrictedVolumes (check_restrictedVolumes.go): the volume sources a restricted pod may use
#define PSS_ALLOWED_VOLUMES                                                                                     \
  ((1u << VS_CONFIGMAP) | (1u << VS_CSI) | (1u << VS_DOWNWARDAPI) | (1u << VS_EMPTYDIR) | (1u << VS_EPHEMERAL) | \
   (1u << VS_PVC) | (1u << VS_PROJECTED) | (1u << VS_SECRET))
// Per-pod PSA summary (2 words per row, built on the device: lean.inl kpe_psum_kernel): x = OR of
// the container state bitmaps (CX_*), y = the OR-ed list codes under the PSA library's fixed
// sets: capability-set bits (CS_* of kernels.hip) | volume codes << 3 (bit 0 hostPath, bit 1 a
// source outside PSS_ALLOWED_VOLUMES) | sysctl codes << 5 (bit v: a sysctl outside version v's
// set) | annotation codes << 8 (bit 0 AppArmor, bit 1 pod seccomp annotation not allowed) | bit
// 10: a container's seccomp annotation (c_sann) outside the allowed profiles (check_seccompProfile
// v1.0)
#define PS_CAPS(y) ((y) & 7u)
#define PS_SECANN(y) (((y) >> 10) & 1u)
#define PS_VOL(y) (((y) >> 3) & 3u)
#define PS_SYS(y) (((y) >> 5) & 7u)
#define PS_ANN(y) (((y) >> 8) & 3u)

// ---- PSA checks (bit k of a check mask), policy.DefaultChecks() order ----------------------
enum KpeCheck {
  CK_APE = 0,            // allowPrivilegeEscalation
  CK_APPARMOR,           // appArmorProfile
  CK_CAPS_BASELINE,      // capabilities_baseline
  CK_CAPS_RESTRICTED,    // capabilities_restricted
  CK_HOST_NS,            // hostNamespaces
  CK_HOST_PATH,          // hostPathVolumes
  CK_HOST_PORTS,         // hostPorts
  CK_PRIVILEGED,         // privileged
  CK_PROC_MOUNT,         // procMount
  CK_RESTRICTED_VOLUMES, // restrictedVolumes
  CK_RUN_AS_NON_ROOT,    // runAsNonRoot
  CK_RUN_AS_USER,        // runAsUser
  CK_SELINUX,            // seLinuxOptions
  CK_SECCOMP_BASELINE,   // seccompProfile_baseline
  CK_SECCOMP_RESTRICTED, // seccompProfile_restricted
  CK_SYSCTLS,            // sysctls
  CK_WIN_HOST_PROCESS,   // windowsHostProcess
  KPE_NUM_CHECKS
};

// ---- versioned check functions (bit v of a rule's cv_mask) --------------------------------
enum KpeCheckVersion {
  CV_APE_1_8 = 0,
  CV_APE_1_25,
  CV_APPARMOR_1_0,
  CV_CAPS_BASELINE_1_0,
  CV_CAPS_RESTRICTED_1_22,
  CV_CAPS_RESTRICTED_1_25,
  CV_HOST_NS_1_0,
  CV_HOST_PATH_1_0,
  CV_HOST_PORTS_1_0,
  CV_PRIVILEGED_1_0,
  CV_PROC_MOUNT_1_0,
  CV_RESTRICTED_VOLUMES_1_0,
  CV_RUN_AS_NON_ROOT_1_0,
  CV_RUN_AS_USER_1_23,
  CV_SELINUX_1_0,
  CV_SECCOMP_BASELINE_1_0,
  CV_SECCOMP_BASELINE_1_19,
  CV_SECCOMP_RESTRICTED_1_19,
  CV_SECCOMP_RESTRICTED_1_25,
  CV_SYSCTLS_1_0,
  CV_SYSCTLS_1_27,
  CV_SYSCTLS_1_29,
  CV_WIN_HOST_PROCESS_1_0,
  KPE_NUM_CV
};

// A check-mask word (kpe_fetch_cv_masks) of a podSecurity cell with a PolicyException's
// podSecurity controls: bit 31 set when the exception matched the resource (its exclusions then
// shaped the fail message, validate_pss.go:88-110); the checks are bits [0, KPE_NUM_CV)
#define KPE_CVM_XMATCH (1u << 31)
#define KPE_CVM_CHECKS ((1u << KPE_NUM_CV) - 1u)
// PSA check of each versioned check (KpeCheckVersion -> KpeCheck); shared by the device
// (per-ID check masks) and the host (report `controls`, one entry per failing versioned check).
#define KPE_CV_CHECK_TABLE                                                                              \
  {CK_APE,           CK_APE,           CK_APPARMOR,          CK_CAPS_BASELINE,      CK_CAPS_RESTRICTED, \
   CK_CAPS_RESTRICTED, CK_HOST_NS,     CK_HOST_PATH,         CK_HOST_PORTS,         CK_PRIVILEGED,      \
   CK_PROC_MOUNT,    CK_RESTRICTED_VOLUMES, CK_RUN_AS_NON_ROOT, CK_RUN_AS_USER,     CK_SELINUX,         \
   CK_SECCOMP_BASELINE, CK_SECCOMP_BASELINE, CK_SECCOMP_RESTRICTED, CK_SECCOMP_RESTRICTED, CK_SYSCTLS,    \
   CK_SYSCTLS,       CK_SYSCTLS,       CK_WIN_HOST_PROCESS}

// ---- per-container derived violation bits (device-internal) ------------------------------------
#define CB_APE (1u << 0)            // sc nil || ape nil || ape true
#define CB_CAPS_BASE (1u << 1)      // caps present && add has a non-baseline capability
#define CB_CAPS_DROP (1u << 2)      // caps nil || drop lacks "ALL"
#define CB_CAPS_ADD (1u << 3)       // add has something other than NET_BIND_SERVICE
#define CB_HOSTPORT (1u << 4)
#define CB_PRIV (1u << 5)
#define CB_PROCMOUNT (1u << 6)
#define CB_RNR_FALSE (1u << 7)      // runAsNonRoot explicitly false
#define CB_RNR_UNSET (1u << 8)
#define CB_RAU_ZERO (1u << 9)
#define CB_SELINUX (1u << 10)
#define CB_SEC_BAD (1u << 11)       // seccomp set and not RuntimeDefault/Localhost
#define CB_SEC_UNSET (1u << 12)
#define CB_SEC_ANN (1u << 13)       // container seccomp annotation with a forbidden value (1.0)
#define CB_WHP (1u << 14)

// ---- verdict cells (same values as kpe.h enum kpe_verdict) ----
#define KPE_NA_ 0
#define KPE_PASS_ 1
#define KPE_FAIL_ 2
#define KPE_WARN_ 3
#define KPE_ERROR_ 4
#define KPE_SKIP_ 5
#define KPE_PENDING_ 6  // device-internal: matched pattern / condition rule, resolved by a later kernel
#define KPE_UNDECIDED_ 7  // the device cannot decide this cell (a documented device limit, e.g. a
                          // condition list longer than CV_LIST_CAP): the caller evaluates it
#define KPE_XFAIL_ 8  // device-internal: a failing podSecurity cell whose PolicyException has
                      // podSecurity controls (validate_pss.go:88-104), resolved by kpe_pssx_kernel
#define KPE_VERDICT_SLACK 72u  // bytes past the N x R matrix: the pattern kernel's 64-column row
                               // scan reads 17 whole words from a row's start
#define KPE_DEEP_ 0x26  // device-internal: a pattern cell whose walk overflowed the LDS frame stack,
                       // re-walked by kpe_pattern_deep_kernel on the lane-private stack
#define KPE_XDEFER_ 0x10  // device-internal flag (XE_DEFER rules): the exception's match block
                          // held; kpe_cond_kernel applies the exception after the preconditions

// ---- policy program ------------------------------------------------------------------------------
// Rule handlers
#define H_NONE 0u  // no validate handler => no RuleResponse (NA even when matched)
#define H_PSS 1u
#define H_ERROR 2u  // every matching resource gets RuleStatusError (e.g. unparsable PSS version)
#define H_PATTERN 3u  // validate.pattern / validate.anyPattern (validate_resource.go:316-398)
// constant verdicts of rules whose preconditions / deny conditions fold at compile time
// (they read only request.operation, CREATE in the CLI and background scans)
#define H_CONST_SKIP 4u  // preconditions false: RuleSkip (validate_resource.go:125-132)
#define H_CONST_FAIL 5u  // deny conditions true: RuleFail (validate_resource.go:268-279)
#define H_CONST_PASS 6u  // deny conditions false: RulePass
#define H_COND 7u        // deny / foreach-deny evaluated per resource by kpe_cond_kernel (cell PENDING)

// Match terms (AND inside a filter block)
enum KpeTermType {
  T_FALSE = 0,     // constant false ("match cannot be empty", operations w/o CREATE, user info on exclude)
  T_KINDS = 1,     // OR over kind selectors [a, a+b) in the selector table
  T_PRED = 2,      // bit lookup: predicate a over the resource column named by b (KpeCol)
  T_ANNOTATIONS = 3,  // every pair [a, a+b) of the annotation-pair table must be matched by some annotation
  T_SELECTOR = 4,     // label selector a (selector table) over resource labels
  T_NSSELECTOR = 5,   // label selector a over the namespace's labels (not for kind Namespace)
  T_KIND_PRED = 6,    // kind-only selectors folded into one predicate a over D_KIND
  // binding-time forms of T_SELECTOR / T_NSSELECTOR whose requirements have bits in the
  // requirement masks (ScanArgs::selm): a = qbit | nreq << 8 | TSQ_* << 16, b (T_NSSELQ) = the
  // D_KIND ids of "Namespace" | "" << 16 (0xFFFF: not in the corpus). One mask compare per lane,
  // no selector record load in the tile loop.
  T_SELQ = 7,
  T_NSSELQ = 8,
  // binding-time form of T_KINDS / T_KIND_PRED on the wide path: bit a of the row's kind-term
  // mask, looked up once per row in a table over the corpus's distinct GVKs (ScanArgs::kslot_lds)
  T_KSLOT = 9
};
#define TSQ_EXC 1u      // KpeSelector::exc
#define TSQ_STAR 2u     // KpeSelector::star_kind
#define TSQ_INVALID 4u  // KpeSelector::invalid
enum KpeCol { COL_NAME = 0, COL_MNS = 1, COL_NSA = 2 };

typedef struct KpeTerm {
  uint32_t type, a, b, pad;
} KpeTerm;
typedef struct KpeKindSel {
  int32_t pg, pv, pk;  // predicate ids over D_GROUP/D_VERSION/D_KIND, -1 = always true ("*")
  uint32_t sub_ok;     // wildcard.Match(sub, "") (no subresources in background/CLI scans)
} KpeKindSel;
typedef struct KpeAnnPair {
  int32_t pk, pv;  // predicates over D_ANNK / D_ANNV
} KpeAnnPair;
// Label selector (CheckSelector, pkg/utils/match/labels.go:9-24, after
// wildcards.ReplaceInSelector, pkg/engine/wildcards/wildcards.go:13-58): an AND of
// requirements [req0, req0+nreq). Statically invalid selectors and selectors
// that are always true are folded at compile time (T_FALSE / no term).
typedef struct KpeSelector {
  uint32_t req0, nreq;
  int32_t p_kind_ns;     // namespaceSelector: D_KIND predicate "Namespace" (never applies)
  int32_t p_kind_empty;  // namespaceSelector: D_KIND predicate "" (skipped unless kinds has "*")
  uint32_t star_kind;    // namespaceSelector: the block's kinds contain "*"
  uint32_t invalid;      // namespaceSelector that fails to build (false wherever it is evaluated)
  uint32_t exc;          // PolicyException block (pkg/utils/match/match.go:184-193): not checked
                         // for kind Namespace or an empty kind
  uint32_t qbit;         // binding: first bit of the selector's requirements in the per-row
                         // requirement mask (ScanArgs::selm), KPE_NO_QBIT: evaluated per requirement
} KpeSelector;
#define KPE_NO_QBIT 0xFFFFFFFFu
#define SR_EQ 0u        // matchLabels k: v (no wildcards): first label with key k has value v
#define SR_WILD 1u      // matchLabels with wildcards: first label matching both globs, and that
                        // label is a valid key/value (else LabelSelectorAsSelector fails)
#define SR_IN 2u        // matchExpressions In:     key present and value in set
#define SR_NOTIN 3u     // matchExpressions NotIn:  key absent or value not in set
#define SR_EXISTS 4u    // matchExpressions Exists
#define SR_NOTEXIST 5u  // matchExpressions DoesNotExist
typedef struct KpeSelReq {
  uint32_t op;
  int32_t pk, pv;       // predicates over D_LABK / D_LABV (pv unused for EXISTS / NOTEXIST)
  int32_t pk_ok, pv_ok; // SR_WILD: validity predicates (qualified name / label value)
  uint32_t pad[3];
} KpeSelReq;
// A filter (one ResourceFilter / ResourceDescription block) is the AND of the
// distinct terms fterms[t0, t0+nt) (indices into the term table).
typedef struct KpeFilter {
  uint32_t t0, nt;
} KpeFilter;

#define MODE_LEGACY 0u
#define MODE_ANY 1u
#define MODE_ALL 2u

typedef struct KpeRule {
  uint32_t handler;       // H_*
  uint32_t cv_mask;       // PSS: versioned checks to run (version selection done at compile time)
  uint32_t match_mode, match_f0, match_nf;    // filters [f0, f0+nf)
  uint32_t excl_mode, excl_f0, excl_nf;
  int32_t pol_term;       // -1 or term that must hold (namespaced policy: resource ns == policy ns)
  uint32_t policy;        // policy index (ApplyOne grouping)
  uint32_t apply_one;     // spec.applyRules == One
  uint32_t pss_excl0, pss_nexcl;  // PSS exclusions (reserved)
  uint32_t cv_class;      // PSS: index of cv_mask among the program's distinct cv_masks
  uint32_t exc;           // PolicyExceptions of the rule (XE_*): their match block; 0 = none
  uint32_t pad;           // 16 words
} KpeRule;
// KpeRule::exc: a cell whose rule matched (and whose preconditions are constant) is
// RuleSkip "rule skipped due to policy exception" when this block of filters holds
// (pkg/engine/utils/exceptions.go:14-47 MatchesException, validate_resource.go:43-56,
// validate_pss.go:45-58). Filters [f0, f0 + nf), any (OR) or all (AND; nf = 0: always).
#define XE_PRESENT (1u << 31)
#define XE_ALL (1u << 30)
#define XE_PSS (1u << 29)  // the rule's (single) exception has podSecurity controls: a failing PSS
                           // cell becomes KPE_XFAIL_ instead of RuleSkip (ApplyPodSecurityExclusion)
#define XE_DEFER (1u << 28)  // kpe_cond_kernel decides (the exception's conditions or the rule's
                             // preconditions read the resource): a cell whose block holds is
                             // written as KPE_XDEFER_ | its verdict without the exception
#define XE_F0(x) ((x) & 0xFFFFFu)
#define XE_NF(x) (((x) >> 20) & 0xFFu)  // bits 20..27

// ---- podSecurity.exclude (pkg/pss/evaluate.go:72-317), evaluated by kpe_pssx_kernel ----------
// A PSA field error is keyed by its field path with digit runs replaced by "*": a suffix
// code (XF_*) and the container list it names (XT_*, XT_POD for pod-level fields).
// Annotation fields carry the normalised annotation key; container fields the container name.
#define XF_APE 0u         // securityContext.allowPrivilegeEscalation
#define XF_CAPS_ADD 1u    // securityContext.capabilities.add
#define XF_CAPS_DROP 2u   // securityContext.capabilities.drop
#define XF_HOSTPORT 3u    // ports[*].hostPort
#define XF_PRIV 4u        // securityContext.privileged
#define XF_PROCMOUNT 5u   // securityContext.procMount
#define XF_RNR 6u         // securityContext.runAsNonRoot
#define XF_RAU 7u         // securityContext.runAsUser
#define XF_SEL_TYPE 8u    // securityContext.seLinuxOptions.type
#define XF_SEL_USER 9u    // securityContext.seLinuxOptions.user
#define XF_SEL_ROLE 10u   // securityContext.seLinuxOptions.role
#define XF_SECCOMP 11u    // securityContext.seccompProfile.type
#define XF_WHP 12u        // securityContext.windowsOptions.hostProcess
#define XF_HOSTNET 13u    // spec.hostNetwork
#define XF_HOSTPID 14u    // spec.hostPID
#define XF_HOSTIPC 15u    // spec.hostIPC
#define XF_SYSCTL 16u     // spec.securityContext.sysctls[*].name
#define XF_ANN 17u        // metadata.annotations[<key>]
#define XF_VOL 32u        // spec.volumes[*].<source>: XF_VOL + VS_* (XF_VOL + 31: "unknown")
#define XT_POD 3u         // 0 initContainers, 1 containers, 2 ephemeralContainers
#define XKEY(fc, ct) ((fc) | ((ct) << 8))
// restrictedField forms
#define XRF_ANY 0u    // restrictedField "" (with no values)
#define XRF_FIELD 1u  // a fixed field path: key XKEY(fc, ct)
#define XRF_ANN 2u    // metadata.annotations[K]: K against normalised annotation keys
#define XRF_NEVER 3u  // a path no PSA check reports
// constant bad-value matches of an exclude (extractBadValues of bools and the int 0)
#define XV_TRUE 1u
#define XV_FALSE 2u
#define XV_ZERO 4u
typedef struct KpeXExcl {
  uint32_t checks;         // PSA check ids of controlName (pkg/pss/utils/mapping.go), bit per KpeCheck
  int32_t img;             // predicate over D_IMAGE (images); -1: pod-level exclusion
  uint32_t rf_kind, rf_key;  // XRF_*; XRF_FIELD: XKEY; XRF_ANN: index of K in the program's text table
  uint32_t has_values, vconst;  // values non-empty; XV_* bits
  int32_t pv_misc, pv_annv, pv_sys, pv_cap;  // predicates (values) over D_MISC / D_ANNV / D_SYSCTL / D_CAP
  uint32_t pad[2];
} KpeXExcl;  // 16 words
// force: the exclusion list fails Validate (common_types.go:472-478): the last exclude's error
// makes every evaluated pod fail; an earlier one empties the results (every pod passes)
#define XR_FORCE_NONE 0u
#define XR_FORCE_PASS 1u
#define XR_FORCE_FAIL 2u
typedef struct KpeXRule {
  uint32_t col, cv_mask, excl0, nexcl;
  uint32_t force, kx;  // kx: check ids some exclude names (the rule's or its exception's)
  // PolicyException podSecurity controls (KPE_XFAIL_ cells): excludes [xexcl0, + XR_XN(xn)),
  // applied after the rule's to the converted checks (validate_pss.go:88-104, convertChecks
  // :114-135: only a Pod's spec fields still compare), and the fold of invalid entries
  uint32_t xexcl0, xn;
} KpeXRule;
#define XR_XN(x) ((x) & 0xFFFFFFu)
#define XR_XFORCE(x) ((x) >> 24)  // XR_FORCE_NONE; XR_FORCE_PASS here means "every check cleared":
                                  // SKIP; XR_FORCE_FAIL: the last exclude invalid, FAIL

// ---- generic document tape (pattern rules) ---------------------------------------------
// Every resource is also kept as its JSON document (the reference's unstructured map).
// An entry (uint2) is x = kind | (member-name id + 1) << 2 (D_KEY id; 0 = array element /
// root) and y = scalar id (DN_SCALAR) or the tape index of the container's body. A body is
// {count, 0} followed by the count member / element entries, contiguous (so a member
// lookup is one run of independent loads). Corpus::doc_off[r] is resource r's root entry
// (absolute tape index).
#define DN_SCALAR 0u
#define DN_MAP 1u
#define DN_ARR 2u
#define DN_KIND(x) ((x) & 3u)
#define DN_KEY(x) ((x) >> 2)
#define DN_MAX_KEYS 0x3FFFFFFEu

// Scalar table: one entry per distinct (type, value) of the corpus; ids 0/1/2 are null,
// false, true. Attributes are what pattern.go derives from a value (goval.hpp).
#define SC_NULL_ID 0u
#define SC_FALSE_ID 1u
#define SC_TRUE_ID 2u
#define SC_T_NULL 0u
#define SC_T_BOOL 1u
#define SC_T_INT 2u
#define SC_T_FLOAT 3u
#define SC_T_STR 4u
#define SC_TYPE(f) ((f) & 7u)
#define SC_PINT (1u << 3)    // string: strconv.ParseInt ok -> ival
#define SC_PFLOAT (1u << 4)  // string: strconv.ParseFloat ok -> fval
#define SC_DUR (1u << 5)     // convertNumberToString(v) parses as a duration -> dur
#define SC_QTY (1u << 6)     // ... as a quantity -> comparison key (QNEG, qexp = order, qlo/qhi)
#define SC_QNEG (1u << 7)
#define SC_TEXT (1u << 8)    // compareString text valid: text pool [text_off, +text_len)
#define SC_BTRUE (1u << 9)
#define SC_JVALID (1u << 10)  // condition constant string: json.Valid
#define SC_JLIST (1u << 11)   // ... and decodes as a []string (or null): elements = constant list
                              // [ival & 0xFFFFFFFF, + ival >> 32) of the constant-list table
#define SC_JARR (1u << 13)     // corpus string: json.Valid and a JSON array (a []string decode the
                              // device leaves undecided); SC_JVALID alone: valid JSON, not an array
#define SC_RANGE (1u << 14)    // corpus string: GetOperatorFromStringPattern == InRange, its two
                              // endpoints interned as scalars: ival = lo id | hi id << 32
#define SC_RANGEU (1u << 15)   // corpus string: the InRange form with a `|` in it (undecided)
#define SC_PSIMPLE (1u << 16)  // string: as a pattern, one plain condition equal to itself
                              // (no `|` `&`, no operator prefix or range form, trim-invariant)
#define SC_SPQ (1u << 12)     // number: the quantity of its fmt.Sprint text (%v) equals the quantity
                              // of convertNumberToString (%f), so SC_QTY also stands for Sprint
#define SC_T_ARR 5          // condition constants only: text_off = first element (constant list), text_len = count
typedef struct KpeScalar {
  uint32_t flags, text_off, text_len;
  uint32_t sp_len;    // numbers: fmt.Sprint text (%v of the float64) follows the text: [text_off + text_len, +sp_len)
  int64_t ival;
  double fval;
  int64_t dur;
  int64_t qexp;       // quantity comparison key (goval::qty_key): order (digits + exponent)
  uint64_t qlo, qhi;  // ... and the mantissa left-aligned to 38 digits
} KpeScalar;  // 64 bytes

// ---- compiled patterns -------------------------------------------------------------------
// Pattern node
#define PN_LEAF 0u       // y = leaf index
#define PN_MAP 1u        // y = first member, z = number of anchor-phase members | total << 16,
                         // w = inline depth (see PNF_FLAT)
#define PN_ARR_EMPTY 2u  // []: "pattern Array empty"
#define PN_ARR_MAPS 3u   // [map, ...]: y = node of element 0 (validateArrayOfMaps)
#define PN_ARR_LEAF 4u   // [scalar, ...]: y = leaf of element 0 (every element must match)
#define PN_ARR_POS 5u    // [[...], ...]: y = first entry of the node list, z = count (positional)
#define PN_EXLIST 6u     // existence-anchor value: y = node list entry, z = count (PN_BAD entries allowed)
#define PN_BAD 7u        // existence element that is not a map / pattern that is not a list
typedef struct KpePNode {
  uint32_t kind, y, z, w;
} KpePNode;
// Inline depth of a map node (KpePNode::w, 0 = none): a map of at most 8 members each of which is a
// scalar leaf, a negation anchor, a "*" presence check or a map of inline depth d - 1 (so depth 1
// holds leaves only), with no existence anchor, ExpandInMetadata key or AnchorMap slot past the
// 32 tracked, and d <= PNF_MAXDEPTH. The VM validates such a map in its BEGIN step, each level
// from one load of the resource map's body (patvm.inl flat_map), instead of a frame and a step
// per member.
#define PNF_FLAT 1u
#define PNF_MAXDEPTH 3u
#define PNW_DEPTH 0xFFu       // KpePNode::w of a map: the inline depth bits
#define PNW_CHAIN (1u << 8)   // a map whose only member is a plain key (default handler, no flags)
                              // with a map / list value: validateMap's verdict is that value's
                              // (validate.go:118-175 with one member, anchor/handlers.go:23-41), so
                              // the walk descends to it without a frame
// Pattern member (uint4): x = handler | PMF_* | slot << 8, y = member-name id + 1 (per
// binding; 0 = name absent from the corpus), z = value node, w = glob-key predicate
// location (PMF_GLOB) or PRED_NONE
#define PM_DEFAULT 0u
#define PM_COND 1u
#define PM_GLOBAL 2u
#define PM_EXIST 3u
#define PM_EQ 4u
#define PM_NEG 5u
#define PM_HANDLER(x) ((x) & 7u)
#define PMF_STAR (1u << 3)   // default handler whose value is the string "*" (presence check)
#define PMF_GLOB (1u << 4)   // ExpandInMetadata: first resource member matching the glob (string values)
#define PMF_SLOT (1u << 5)   // condition / existence anchor tracked in the AnchorMap
#define PMF_LEAF (1u << 6)   // the member's pattern value is a scalar leaf (PN_LEAF); bound: w = its
                             // leaf-table slot (PatArgs::lslot of the leaf) unless PMF_GLOB / PMF_VKEY
#define PMF_VSTAR (1u << 7)  // default-handler member whose leaf has variables: a value of "*"
                             // is the presence check (anchor/handlers.go:130-133)
#define PM_SLOT(x) (((x) >> 8) & 31u)
#define PMF_XSLOT (1u << 13)  // condition / existence anchor past the 32 AnchorMap slots: a map
                              // holding it makes the cell KPE_UNDECIDED
#define PMF_VKEY (1u << 14)   // a key with {{ }} variables (substitutePatterns renames it per row,
                              // jsonutils/traverse.go:90-117): w = the key's template leaf (PL_VAR /
                              // PL_TMPL; bval bit 0: under ExpandInMetadata, bit 1: the map has other
                              // keys with variables (PVF_GROUP), bit 2: an anchored key, the template
                              // being the whole written key and pad[2] = the anchor text's lengths
                              // before | after the key << 16; pad[0] = template-text offset of the
                              // map's other plain keys (anchored: its other phase-1 anchor keys) in
                              // walk order, [u16 length][bytes] each; pad[1] = their count | this
                              // key's place << 16)
// Leaf
#define PL_BOOL 0u
#define PL_INT 1u
#define PL_FLOAT 2u
#define PL_NIL 3u
#define PL_STR 4u
#define PL_NEVER 5u  // array pattern in leaf position: always false
#define PL_VAR 6u    // a whole-string {{ }} variable: the pattern is the variable's typed value;
                     // c0 = variable slot (per-row value in PatArgs::pvals)
#define PL_TMPL 7u   // a string with variables inside: pieces [c0, c0 + nc) of the template table
// Template piece (uint2): x = PT_TEXT | len << 1 (y = offset in the template text) or PT_VAR
// (y = variable slot; the value's text: a string as is, anything else json.Marshal-ed)
#define PT_TEXT 0u
#define PT_VAR 1u
// Resolved pattern variable of a row (uint2 pvals[row * nvars + slot], written by
// kpe_cond_kernel after the rule's preconditions): x = PVK_*, y = id
#define PVK_NULL 0u
#define PVK_SCAL 1u   // corpus scalar id
#define PVK_CONST 2u  // condition-program constant id
#define PVK_NUM 3u    // y = elementIndex (a float64)
// Pattern variable slot: the query template (condition program) and how the pattern uses it
#define PVF_WHOLE 1u  // a whole-string leaf: a string value must be SC_PSIMPLE
#define PVF_TEXT 2u   // inside a template: numbers must print as json.Marshal does
#define PVF_KEY 4u    // a whole-string variable naming a map key: a string (traverse.go:101-103:
                      // another type is an error; null keeps the key as written: undecided)
#define PVF_GROUP_SH 8u       // bits 8..31: the map's key group when it has several keys with variables
#define PVF_GROUP(f) ((f) >> PVF_GROUP_SH)  // (each one whole-string variable; 0: the only one)
typedef struct KpePVar {
  uint32_t tmpl, flags;
} KpePVar;
typedef struct KpeLeaf {
  uint32_t type, bval, c0, nc;  // PL_STR: conditions [c0, c0 + nc)
  int64_t ival;
  double fval;
  uint32_t exact;               // PL_STR: pattern-operand record of the whole pattern (value == pattern)
  uint32_t pad[3];
} KpeLeaf;  // 40 -> 48 bytes
#define KPE_NO_LSLOT 0xFFFFFFFFu
#define KPE_LTAB_SLOTS 256u  // distinct leaves with a leaf-table slot per program
// String-pattern condition (one `&`-term of one `|`-alternative)
#define PC_OP(x) ((x) & 7u)
#define PC_EQ 0u
#define PC_GE 1u
#define PC_LE 2u
#define PC_NE 3u
#define PC_GT 4u
#define PC_LT 5u
#define PC_NEWGROUP (1u << 3)  // first condition of a `|` alternative
#define PC_OR2 (1u << 4)       // NotInRange: this condition OR the next one (one term)
#define PC_DUR (1u << 5)       // operand parses as a duration
#define PC_QTY (1u << 6)       // operand parses as a quantity
#define PC_QNEG (1u << 7)
typedef struct KpeCond {
  uint32_t op, pat, pad0, pad1;  // pat: operand record (compareString glob)
  int64_t dur, qexp;
  uint64_t qlo, qhi;
} KpeCond;  // 48 bytes
// Pattern rule: roots [r0, r0 + nr) of the root table (uint2: node, anchor slots)
#define PR_ANY 1u        // anyPattern
#define PR_ANY_BAD 2u    // anyPattern that is not a list: RuleStatusError
// KpePatRule::flags >> PR_MEMO_SH: the rule's memo slot (< KPE_PAT_MEMO) when other pattern rules of
// the program carry the same pattern (equal JSON, no variables): a row evaluates it once and
// every rule of the slot takes that verdict (the pattern verdict depends on the row alone);
// PR_NO_MEMO: none
#define PR_MEMO_SH 16
#define PR_NO_MEMO 0xFFFFu
// 16 slots: 2 KiB of LDS per 128-lane block, so 8 blocks fit a CU's 160 KiB with the frame stacks
// (32 slots allowed 7; C5 6.97 -> 6.59 ms, C3 3.23 -> 3.05 ms, profiles/r04_o)
// PatArgs::col2pr entry: pattern rule index + 1 in the low 24 bits (0: not a pattern column), the
// rule's memo slot + 1 in the high 8 (0: none), so a cell's slot needs no rule-record load
#define C2P_RULE(e) ((e) & 0xFFFFFFu)
#define C2P_SLOT(e) (((e) >> 24) - 1u)  // >= KPE_PAT_MEMO: none
#define C2P_MAKE(pi1, slot) ((pi1) | (((slot) < KPE_PAT_MEMO ? (slot) + 1u : 0u) << 24))
#ifndef KPE_PAT_SLOT_ORDER
#define KPE_PAT_SLOT_ORDER 1  // kpe_pattern_kernel evaluates a row's memo slots in slot order first
#endif
#ifndef KPE_PAT_MEMO
#define KPE_PAT_MEMO 16
#endif
// the pattern kernel keeps the memo slots' valid bits in one 32-bit word (patvm.inl memo_ok)
#if KPE_PAT_MEMO > 32
#error "KPE_PAT_MEMO must be <= 32"
#endif
typedef struct KpePatRule {
  uint32_t col, flags, r0, nr;
} KpePatRule;
// Failing-path record of one pattern root (kpe_pattern_traces, include/kpe.h): word 0 =
// component count | KPE_TR_TRUNC | verdict << 16 | KPE_TR_VALID; words 1..15 = components from
// the root: a pattern member index (the key its handler appends to the path), KPE_TC_KEY | D_KEY
// id (an ExpandInMetadata key: the matched resource member's name) or KPE_TC_IDX | array index
#define KPE_TRACE_WORDS 16u
#define KPE_TRACE_ROOTS 4u
#define KPE_TC_IDX 0x80000000u
#define KPE_TC_KEY 0x40000000u
#define KPE_TR_TRUNC 0x100u
#define KPE_TR_VALID 0x1000000u

// ---- condition programs (preconditions / deny / foreach-deny; kpe_cond_kernel) -------------
// A query is the JMESPath expression of a whole-string {{ }} variable (or a foreach `list`),
// compiled to a linear op list (program.cpp cq::QueryParser): a root, then steps. After `[]`
// or `[*]` the following steps apply to every element of the projected list; the nulls they
// produce are dropped when the projection ends (go-jmespath projection semantics).
#define QO_OBJ 0u     // request.object: the resource's document root
#define QO_EL 1u      // element (y = 0xFFFFFFFF: the innermost) / element<y> (foreach nesting y)
#define QO_IDX 2u     // elementIndex / elementIndex<y> (a float64)
#define QO_CONST 3u   // y = constant (request.operation = "CREATE", raw-string / JSON literals)
#define QO_FIELD 4u   // y = field-name index (a binding resolves it to D_KEY id + 1; 0 = absent)
#define QO_INDEX 5u   // y = index (int32; negative counts from the end)
#define QO_FLAT 6u    // `[]`
#define QO_STAR 7u    // `[*]`
#define QO_KEYS 8u    // keys(@) of the current value
#define QO_MSL 9u     // `[a, b, ...]` over the current value; QO_ARG = number of items, each a
                      // QO_ITEM (QO_ARG = its op count) followed by a relative field / index chain
#define QO_ITEM 10u
#define QO_ERROR 11u  // the expression is empty: every evaluation is an error (RuleError)
#define QO_VALS 13u   // `.*`: the member values of an object, then projected like `[*]`
#define QO_LEN 14u    // length() of the current value (functions.go jpfLength): a projection's
                      // items, a string's runes, an array's items, an object's members; other
                      // types an invalid-type error
#define QO_IMG 12u    // images: the resource's images context map (context.go:306-348), absent
                      // when the resource has no images
#define QO_OP(x) ((x) & 0xFFu)
#define QO_ARG(x) ((x) >> 8)
typedef struct KpeCExpr {
  uint32_t op0, nops;  // ops [op0, op0 + nops) (uint2 each)
  uint32_t flags;      // CE_STRICT: a plain field / index chain: a missing member is a NotFoundError
  uint32_t alt;        // `||` right operand (an expression index) or 0xFFFFFFFF
} KpeCExpr;
#define CE_STRICT 1u
#define CE_NONE 0xFFFFFFFFu
// Value template: a condition key / value after variable substitution
#define VT_CONST 0u  // a = constant
#define VT_QUERY 1u  // a = expression
#define VT_ARRAY 2u  // a = first element template, b = count (a list with variables inside)
#define VT_TMPL 3u   // a string with variables inside it: pieces [a, a + b) of CondArgs::tpieces
typedef struct KpeVTmpl {
  uint32_t kind, a, b, pad;
} KpeVTmpl;
// Condition operators (variables/operator/operator.go:27-67)
#define CO_EQ 0u
#define CO_NE 1u
#define CO_ANYIN 2u
#define CO_ALLIN 3u
#define CO_ANYNOTIN 4u
#define CO_ALLNOTIN 5u
#define CO_IN 6u
#define CO_NOTIN 7u
#define CO_NUM 8u   // numeric.go GreaterThan* / LessThan*: aux = CN_* (compareByCondition's operator)
#define CO_DUR 9u   // duration.go Duration*: aux = CN_*
#define CO_BAD 10u  // no operator handler: an evaluation error after the key / value substitution
#define CN_GE 0u
#define CN_GT 1u
#define CN_LE 2u
#define CN_LT 3u
#define CN_NONE 4u  // a non-canonical spelling: compareByCondition's default (false)
typedef struct KpeCCond {
  uint32_t op, key, value;  // key / value: template indices
  uint32_t aux;  // CO_NUM / CO_DUR: CN_*; set operators: 1 + leaf index of an InRange constant value
                 // (validateStringPatterns of the value, pattern program leaf table; the NotInRange
                 // form `a!-b` AnyNotIn uses is the next leaf), 0 = none
} KpeCCond;
// Condition block: AnyAllConditions (any = conds [c0, c0 + nany), all = the next nall), or the
// deprecated list form (nany = 0, all = the list)
#define CB_HAS_ANY 1u
typedef struct KpeCBlock {
  uint32_t c0, nany, nall, flags;
} KpeCBlock;
// A validate.foreach entry (newForEachValidator, validate_resource.go:76-119): the list, its
// preconditions, then one body: deny, pattern / anyPattern (against the innermost scoped element,
// or the resource), or nested entries (nesting + 1)
#define FE_NONE 0u  // no body: a nil response per element
#define FE_DENY 1u  // deny = block
#define FE_PAT 2u   // a = first pattern root, b = roots | PR_* << 16, c = pv0 | npv << 16
#define FE_NEST 3u  // a = first nested entry, b = count
typedef struct KpeCForeach {
  uint32_t list;   // value template (a query)
  uint32_t pre;    // block or CE_NONE
  uint32_t deny;   // block (FE_DENY)
  uint32_t scope;  // elementScope: 0 unset, 1 false, 2 true
  uint32_t kind, a, b, c;
} KpeCForeach;
#define KPE_FE_DEPTH 3  // foreach nesting levels evaluated on the device
#define CR_PRE_ONLY 0u  // only the rule's preconditions are evaluated here (other handler)
#define CR_DENY 1u      // H_COND: validate.deny
#define CR_FOREACH 2u   // H_COND: validate.foreach (deny entries)
#define CR_NONE 3u      // H_COND: a validate block without handler (validation.go:52: the
                        // resource validator returns nil) behind per-resource preconditions
typedef struct KpeCRule {
  uint32_t col, pre, kind, deny;  // pre / deny: block or CE_NONE
  uint32_t fe0, nfe;
  uint32_t pv0, npv;  // pattern rules with variables: slots [pv0, pv0 + npv) resolved after the
                      // preconditions (validate_resource.go:456-476 substitutePatterns)
  uint32_t exc;       // XC_DEFER: the exception's conditions (block; CE_NONE: none, it holds)
  uint32_t xflags;    // XC_*
  uint32_t mslot;     // condition trace slot + 1 (CondArgs::mtrace; 0: none)
} KpeCRule;
// A condition trace word (CondArgs::mtrace, one per row and rule with a slot): where the rule's
// preconditions block (low half) and deny block (high half << 16) stopped, for the messages of
// variables/evaluate.go:31-125 (program.hpp CondMsgs): the index of the first true `any`
// condition (nany: none) and of the first false `all` condition (nall: none), CT_EVAL when the
// block was evaluated without an error and CT_TRUE when it held. Blocks of more than CT_MAXC
// conditions get no slot.
#define CT_ANY(t) ((t) & 0x7Fu)
#define CT_ALL(t) (((t) >> 7) & 0x7Fu)
#define CT_EVAL 0x4000u
#define CT_TRUE 0x8000u
#define CT_MAXC 127u
// A block that raised an error (RuleError texts, validate_resource.go:127,270 and engine.go:279-281):
// CT_ERR without CT_EVAL, the index of the condition that raised it (any conditions first, then
// all; the old list form: its index) and the side: 0 the key's substitution, 1 the value's, 2 the
// operator (variables/evaluate.go:14-27)
#define CT_ERR 0x8000u
#define CT_IS_ERR(t) (((t) & (CT_ERR | CT_EVAL)) == CT_ERR)
#define CT_ERR_COND(t) ((t) & 0x7Fu)
#define CT_ERR_SIDE(t) (((t) >> 7) & 3u)
// validate.foreach rules have four trace words (KpeCRule::mslot .. + 3), written for the element
// that decided a FAIL / ERROR cell (validateElements, validate_resource.go:206-254):
//   word 0: the rule's preconditions (low half, as above) | the deciding element's block << 16
//           (its deny block, or its preconditions for FT_PRE_ERR; CT_* / CT_ERR form)
//   word 1: FT_* path: nesting depth of the element (0 .. KPE_FE_DEPTH - 1), what decided it, and
//           per level l <= depth the foreach entries left in that level's list when it ran (the
//           entry is count - left) and the element index
//   word 2: the element's tape entry (a document node), or 0xFFFFFFFF (a constant element)
//   word 3: the tape entry its patterns validate (the innermost scoped element; 0xFFFFFFFF: the
//           resource root, 0xFFFFFFFE: a constant)
#define KPE_FE_TRACE_WORDS 4u
#define FT_DEPTH(b) ((b) & 3u)
#define FT_KIND(b) (((b) >> 2) & 7u)
#define FT_DENY 1u      // the element's deny block held (FAIL) or raised an error
#define FT_PRE_ERR 2u   // the element's preconditions raised an error
#define FT_PAT 3u       // the entry's pattern / anyPattern on the element failed or errored
#define FT_PVAR_ERR 4u  // the entry's pattern variables failed to substitute
#define FT_SCOPE_ERR 5u // elementScope: true on an element that is not a map (AddElementToContext)
#define FT_VALID 0x20u
#define FT_OVERFLOW 0x40u  // an element index > 31 or more than 7 entries left: no path
#define FT_LEFT(b, l) (((b) >> (8u + 8u * (l))) & 7u)
#define FT_IDX(b, l) (((b) >> (11u + 8u * (l))) & 31u)
// KpeCRule::xflags: the rule's PolicyException is applied here (XE_DEFER), after the
// preconditions: in a cell flagged KPE_XDEFER_ its conditions holding make the cell RuleSkip
// (validate_resource.go:43-56) or, with podSecurity controls (XC_PSS), a failing cell KPE_XFAIL_
// (validate_pss.go:45-104); false or an error: no exception (exceptions.go:33-41)
#define XC_DEFER 1u
#define XC_PSS 2u
