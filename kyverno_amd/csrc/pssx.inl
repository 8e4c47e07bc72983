// podSecurity.exclude on the device: kpe_pssx_kernel's per-pod body. Included inside
// kernels.hip's anonymous namespace.
//
// Restates pkg/pss/evaluate.go for rules with exclusions:
//   EvaluatePod :242-252, ApplyPodSecurityExclusion :255-279, GetPodWithMatchingContainers
//   :283-317 (pod-level exclusions evaluate a copy whose containers are one empty "fake"
//   container; image exclusions a pod of only the matching containers, with no metadata but
//   name / namespace and no pod-level fields), exemptExclusions :72-161 (for every exclude
//   error whose field and bad values qualify, the first default error with the same field -
//   and, for image exclusions, the same container name - is swap-removed), extractBadValues
//   :163-182, parseField :193-204 (fields compare with digit runs replaced by "*").
// The field errors are the PSA v0.29 check errors restated in oracle/pss.hpp (field paths,
// bad values and their order), generated here from the corpus's pod columns.
// Everything is forced inline with single call sites for the heavy parts (gen() and the
// removal loop): the lane's error buffers are private arrays (the patvm.inl constraint).

constexpr uint32_t kXCap = 64;  // errors of one versioned check on one pod view
constexpr uint32_t VW_REAL = 0, VW_SPEC = 1, VW_MATCH = 2;
// bad-value kinds of a generated error (E[].x bits 16..23)
constexpr uint32_t BK_NONE = 0, BK_TRUE = 1, BK_FALSE = 2, BK_ZERO = 3, BK_MISC = 4, BK_ANNV = 5, BK_SYS = 6,
                   BK_CAPS = 7;
// the "fake" container of a pod-level exclusion: no securityContext, no ports
constexpr uint32_t kFakeBits = CX_PRIV_U | CX_APE_U | CX_RNR_U | CX_RAU_U | CX_SEC_NONE | CX_PM_U | CX_SEL_NONE |
                               CX_WHP_NT | CX_NOCAPS | CX_NOHOSTPORT;
// restrictedVolumes precedence (check_restrictedVolumes.go): the first present of these
// sources in VS_* order names the field, else "unknown"
constexpr uint32_t kBadVolumes = (1u << VS_HOSTPATH) | (1u << VS_GCEPD) | (1u << VS_AWSEBS) | (1u << VS_GITREPO) |
                                 (1u << VS_NFS) | (1u << VS_ISCSI) | (1u << VS_GLUSTERFS) | (1u << VS_RBD) |
                                 (1u << VS_FLEXVOLUME) | (1u << VS_CINDER) | (1u << VS_CEPHFS) | (1u << VS_FLOCKER) |
                                 (1u << VS_FC) | (1u << VS_AZUREFILE) | (1u << VS_VSPHERE) | (1u << VS_QUOBYTE) |
                                 (1u << VS_AZUREDISK) | (1u << VS_PHOTONPD) | (1u << VS_PORTWORX) |
                                 (1u << VS_SCALEIO) | (1u << VS_STORAGEOS);
constexpr uint32_t kOkVolumes = (1u << VS_CONFIGMAP) | (1u << VS_CSI) | (1u << VS_DOWNWARDAPI) |
                                (1u << VS_EMPTYDIR) | (1u << VS_EPHEMERAL) | (1u << VS_PVC) | (1u << VS_PROJECTED) |
                                (1u << VS_SECRET);

// versioned checks of PSA check k (KpeCheckVersion bits)
__device__ __forceinline__ uint32_t check_versions(uint32_t k) {
  switch (k) {
    case CK_APE: return (1u << CV_APE_1_8) | (1u << CV_APE_1_25);
    case CK_APPARMOR: return 1u << CV_APPARMOR_1_0;
    case CK_CAPS_BASELINE: return 1u << CV_CAPS_BASELINE_1_0;
    case CK_CAPS_RESTRICTED: return (1u << CV_CAPS_RESTRICTED_1_22) | (1u << CV_CAPS_RESTRICTED_1_25);
    case CK_HOST_NS: return 1u << CV_HOST_NS_1_0;
    case CK_HOST_PATH: return 1u << CV_HOST_PATH_1_0;
    case CK_HOST_PORTS: return 1u << CV_HOST_PORTS_1_0;
    case CK_PRIVILEGED: return 1u << CV_PRIVILEGED_1_0;
    case CK_PROC_MOUNT: return 1u << CV_PROC_MOUNT_1_0;
    case CK_RESTRICTED_VOLUMES: return 1u << CV_RESTRICTED_VOLUMES_1_0;
    case CK_RUN_AS_NON_ROOT: return 1u << CV_RUN_AS_NON_ROOT_1_0;
    case CK_RUN_AS_USER: return 1u << CV_RUN_AS_USER_1_23;
    case CK_SELINUX: return 1u << CV_SELINUX_1_0;
    case CK_SECCOMP_BASELINE: return (1u << CV_SECCOMP_BASELINE_1_0) | (1u << CV_SECCOMP_BASELINE_1_19);
    case CK_SECCOMP_RESTRICTED: return (1u << CV_SECCOMP_RESTRICTED_1_19) | (1u << CV_SECCOMP_RESTRICTED_1_25);
    case CK_SYSCTLS: return (1u << CV_SYSCTLS_1_0) | (1u << CV_SYSCTLS_1_27) | (1u << CV_SYSCTLS_1_29);
    default: return 1u << CV_WIN_HOST_PROCESS_1_0;
  }
}

struct PssxVM {
  const PssxArgs& a;
  int64_t r;
  uint32_t pw, c0, c1, v0, v1, s0, s1, a0, a1;
  uint4 E[kXCap];  // errors of the last gen(): x = XKEY | bk << 16, y = aux, z / w = bad value
  uint32_t ne;
  uint2 D[kXCap];  // the default errors of the check being exempted: x = XKEY, y = aux
  uint32_t nd;
  __device__ __forceinline__ PssxVM(const PssxArgs& args, int64_t row) : a(args), r(row), ne(0), nd(0) {}

  __device__ __forceinline__ bool bit(uint32_t loc, uint32_t id) const {
    if (loc == PRED_NONE || id == KPE_NO_STR) return false;
    return (a.pbuf[loc + (id >> 5)] >> (id & 31u)) & 1u;
  }
  __device__ __forceinline__ uint64_t mask64(uint32_t loc) const {  // predicate over D_CAP (<= 64 ids)
    return loc == PRED_NONE ? 0ull : ((uint64_t)a.pbuf[loc] | ((uint64_t)a.pbuf[loc + 1] << 32));
  }
  __device__ __forceinline__ void emit(uint32_t fc, uint32_t ct, uint32_t aux, uint32_t bk, uint32_t b0 = 0,
                                       uint32_t b1 = 0) {
    if (ne < kXCap) E[ne] = make_uint4(XKEY(fc, ct) | (bk << 16), aux, b0, b1);
    ++ne;
  }
  __device__ __forceinline__ uint32_t norm(uint32_t key) const { return key == KPE_NO_STR ? KPE_NO_STR : a.ann_norm[key]; }
  __device__ __forceinline__ uint32_t ann_value(uint32_t key) const {  // pod annotation value by key id
    if (key == KPE_NO_STR) return KPE_NO_STR;
    for (uint32_t k = a0; k < a1; ++k)
      if (a.pann_k[k] == key) return a.pann_v[k];
    return KPE_NO_STR;
  }

  // The field errors of versioned check cv over a pod view (oracle/pss.hpp order).
  __device__ __forceinline__ void gen(uint32_t cv, uint32_t view, uint32_t img) {
    ne = 0;
    const bool podlvl = view != VW_MATCH;
    const uint32_t w = podlvl ? pw : 0u;
    const bool win = FIELD(w, P_OS_SH, 2) == OS_WINDOWS;
    if (win && (cv == CV_APE_1_25 || cv == CV_CAPS_RESTRICTED_1_25 || cv == CV_SECCOMP_RESTRICTED_1_25)) return;
    // checks of pod-level fields only
    if (cv == CV_APPARMOR_1_0) {
      if (podlvl)
        for (uint32_t k = a0; k < a1; ++k) {
          const uint32_t key = a.pann_k[k], val = a.pann_v[k];
          if (bit(a.pp_apparmor_key, key) && !bit(a.pp_apparmor_ok, val)) emit(XF_ANN, XT_POD, norm(key), BK_ANNV, val);
        }
      return;
    }
    if (cv == CV_HOST_NS_1_0) {
      if (w & P_HOSTNET) emit(XF_HOSTNET, XT_POD, 0, BK_TRUE);
      if (w & P_HOSTPID) emit(XF_HOSTPID, XT_POD, 0, BK_TRUE);
      if (w & P_HOSTIPC) emit(XF_HOSTIPC, XT_POD, 0, BK_TRUE);
      return;
    }
    if (cv == CV_HOST_PATH_1_0 || cv == CV_RESTRICTED_VOLUMES_1_0) {
      if (podlvl)
        for (uint32_t k = v0; k < v1; ++k) {
          const uint32_t src = a.vol_src[k];
          if (cv == CV_HOST_PATH_1_0) {
            if (src & (1u << VS_HOSTPATH)) emit(XF_VOL + VS_HOSTPATH, XT_POD, 0, BK_NONE);
          } else if (!(src & kOkVolumes)) {
            emit(XF_VOL + ((src & kBadVolumes) ? (uint32_t)__builtin_ctz(src & kBadVolumes) : 31u), XT_POD, 0, BK_NONE);
          }
        }
      return;
    }
    if (cv >= CV_SYSCTLS_1_0 && cv <= CV_SYSCTLS_1_29) {
      if (podlvl) {
        const uint32_t loc = a.pp_sysctl[cv - CV_SYSCTLS_1_0];
        for (uint32_t k = s0; k < s1; ++k) {
          const uint32_t id = a.sys_id[k];
          if (!bit(loc, id)) emit(XF_SYSCTL, XT_POD, 0, BK_SYS, id);
        }
      }
      return;
    }
    // runAsNonRoot / seccompProfile_restricted: explicit bad values first and alone, else the
    // implicit (unset) containers
    const bool rnr = cv == CV_RUN_AS_NON_ROOT_1_0;
    const bool secr = cv == CV_SECCOMP_RESTRICTED_1_19 || cv == CV_SECCOMP_RESTRICTED_1_25;
    const uint32_t prnr = FIELD(w, P_RNR_SH, 2), psec = FIELD(w, P_SECCOMP_SH, 3);
    const bool psec_valid = psec == SECCOMP_RUNTIMEDEFAULT || psec == SECCOMP_LOCALHOST;
    const bool psec_bad = psec != SECCOMP_NONE && !psec_valid;
    bool has_bad = rnr ? prnr == TRI_FALSE : psec_bad;
    const bool pod_ok = rnr ? prnr == TRI_TRUE : psec_valid;
    const bool fake = view == VW_SPEC;
    const uint32_t cb = fake ? 0u : c0, ce = fake ? 1u : c1;
    for (uint32_t pass = (rnr || secr) ? 0u : 1u; pass < 2u; ++pass) {
      if (pass == 1u) {  // pod-level errors come before the containers'
        if (rnr && has_bad && prnr == TRI_FALSE) emit(XF_RNR, XT_POD, 0, BK_FALSE);
        if (cv == CV_RUN_AS_USER_1_23 && FIELD(w, P_RAU_SH, 2) == RAU_ZERO) emit(XF_RAU, XT_POD, 0, BK_ZERO);
        if (cv == CV_SELINUX_1_0 && FIELD(w, P_SEL_SH, 3) != SEL_NONE) {
          const uint32_t* pc = a.p_cold + 4 * r;
          if (FIELD(w, P_SEL_SH, 3) == SEL_OTHER) emit(XF_SEL_TYPE, XT_POD, 0, BK_MISC, pc[1]);
          if (w & P_SEL_USER) emit(XF_SEL_USER, XT_POD, 0, BK_MISC, pc[2]);
          if (w & P_SEL_ROLE) emit(XF_SEL_ROLE, XT_POD, 0, BK_MISC, pc[3]);
        }
        if (cv == CV_SECCOMP_BASELINE_1_0 && podlvl) {
          const uint32_t val = ann_value(a.key_pod_sec);
          if (val != KPE_NO_STR && !bit(a.pp_seccomp_ok, val))
            emit(XF_ANN, XT_POD, norm(a.key_pod_sec), BK_ANNV, val);
        }
        if ((cv == CV_SECCOMP_BASELINE_1_19 || (secr && has_bad)) && psec_bad)
          emit(XF_SECCOMP, XT_POD, 0, BK_MISC, a.p_cold[4 * r]);
      }
      for (uint32_t i = cb; i < ce; ++i) {
        uint32_t x, ct, name;
        if (fake) {
          x = kFakeBits, ct = 1u, name = KPE_NO_STR;
        } else {
          if (view == VW_MATCH && !bit(img, a.c_image[i])) continue;
          x = a.crec[2 * i], ct = a.crec[2 * i + 1] >> 16, name = a.c_name[i];
        }
        if (pass == 0u) {  // is there an explicit bad container value
          has_bad = has_bad || (rnr ? (x & CX_RNR_F) != 0u : (x & (CX_SEC_UNC | CX_SEC_OTHER)) != 0u);
          continue;
        }
        switch (cv) {
          case CV_APE_1_8:
          case CV_APE_1_25:
            if (x & CX_APE_U) emit(XF_APE, ct, name, BK_FALSE);
            else if (x & CX_APE_T) emit(XF_APE, ct, name, BK_TRUE);
            break;
          case CV_CAPS_BASELINE_1_0:
          case CV_CAPS_RESTRICTED_1_22:
          case CV_CAPS_RESTRICTED_1_25: {
            const bool base = cv == CV_CAPS_BASELINE_1_0;
            if (!(x & CX_CAPS)) {
              if (!base) emit(XF_CAPS_DROP, ct, name, BK_NONE);
              break;
            }
            const uint32_t cs = (a.crec[2 * i + 1] & 0xFFFFu) * 4u;
            const uint64_t add = (uint64_t)a.capsets[cs] | ((uint64_t)a.capsets[cs + 1] << 32);
            const uint64_t drop = (uint64_t)a.capsets[cs + 2] | ((uint64_t)a.capsets[cs + 3] << 32);
            if (!base && !(drop & mask64(a.pp_all))) emit(XF_CAPS_DROP, ct, name, BK_NONE);
            const uint64_t bad = add & ~mask64(base ? a.pp_caps_ok : a.pp_nbs);
            if (bad) emit(XF_CAPS_ADD, ct, name, BK_CAPS, (uint32_t)bad, (uint32_t)(bad >> 32));
            break;
          }
          case CV_HOST_PORTS_1_0:
            if (x & CX_HOSTPORT)
              for (uint32_t p = a.cport_off[i]; p < a.cport_off[i + 1]; ++p)
                if (a.cport_str[p] != KPE_NO_STR) emit(XF_HOSTPORT, ct, name, BK_MISC, a.cport_str[p]);
            break;
          case CV_PRIVILEGED_1_0:
            if (x & CX_PRIV_T) emit(XF_PRIV, ct, name, BK_TRUE);
            break;
          case CV_PROC_MOUNT_1_0:
            if (x & CX_PM_OTHER) emit(XF_PROCMOUNT, ct, name, BK_MISC, a.c_pm_str[i]);
            break;
          case CV_RUN_AS_NON_ROOT_1_0:
            if (has_bad) {
              if (x & CX_RNR_F) emit(XF_RNR, ct, name, BK_FALSE);
            } else if ((x & CX_RNR_U) && !pod_ok) {
              emit(XF_RNR, ct, name, BK_NONE);
            }
            break;
          case CV_RUN_AS_USER_1_23:
            if (x & CX_RAU_Z) emit(XF_RAU, ct, name, BK_ZERO);
            break;
          case CV_SELINUX_1_0:
            if (x & CX_SEL_OTHER) emit(XF_SEL_TYPE, ct, name, BK_MISC, a.c_selt_str[i]);
            if (x & CX_SEL_USER) emit(XF_SEL_USER, ct, name, BK_MISC, a.c_selu_str[i]);
            if (x & CX_SEL_ROLE) emit(XF_SEL_ROLE, ct, name, BK_MISC, a.c_selr_str[i]);
            break;
          case CV_SECCOMP_BASELINE_1_0:
            if (podlvl) {  // the container's annotation "container.seccomp.security.alpha.kubernetes.io/<name>"
              const uint32_t key = fake ? a.key_fake_sec : a.c_sann_key[i];
              const uint32_t val = fake ? ann_value(a.key_fake_sec) : a.c_sann[i];
              if (val != KPE_NO_STR && !bit(a.pp_seccomp_ok, val)) emit(XF_ANN, XT_POD, norm(key), BK_ANNV, val);
            }
            break;
          case CV_SECCOMP_BASELINE_1_19:
            if (x & (CX_SEC_UNC | CX_SEC_OTHER)) emit(XF_SECCOMP, ct, name, BK_MISC, a.c_sec_str[i]);
            break;
          case CV_SECCOMP_RESTRICTED_1_19:
          case CV_SECCOMP_RESTRICTED_1_25:
            if (has_bad) {
              if (x & (CX_SEC_UNC | CX_SEC_OTHER)) emit(XF_SECCOMP, ct, name, BK_MISC, a.c_sec_str[i]);
            } else if ((x & CX_SEC_NONE) && !pod_ok) {
              emit(XF_SECCOMP, ct, name, BK_NONE);
            }
            break;
          case CV_WIN_HOST_PROCESS_1_0:
            if (x & CX_WHP_T) emit(XF_WHP, ct, name, BK_TRUE);
            break;
          default: break;
        }
      }
    }
    if (cv == CV_WIN_HOST_PROCESS_1_0 && FIELD(w, P_WHP_SH, 2) == TRI_TRUE) emit(XF_WHP, XT_POD, 0, BK_TRUE);
  }

  __device__ __forceinline__ static bool empty_str(const uint32_t* off, uint32_t id) {
    return id == KPE_NO_STR || off[id + 1] == off[id];
  }
  // extractBadValues + wildcard.CheckPatterns(values, v) for every bad value
  __device__ __forceinline__ bool values_ok(const KpeXExcl& e, uint4 x) const {
    if (!e.has_values) return true;
    switch ((x.x >> 16) & 0xFFu) {
      case BK_NONE: return true;
      case BK_TRUE: return e.vconst & XV_TRUE;
      case BK_FALSE: return e.vconst & XV_FALSE;
      case BK_ZERO: return e.vconst & XV_ZERO;
      case BK_MISC: return empty_str(a.misc_off, x.z) || bit((uint32_t)e.pv_misc, x.z);
      case BK_ANNV: return empty_str(a.annv_off, x.z) || bit((uint32_t)e.pv_annv, x.z);
      case BK_SYS: return empty_str(a.sysd_off, x.z) || bit((uint32_t)e.pv_sys, x.z);
      default: {
        const uint64_t bad = (uint64_t)x.z | ((uint64_t)x.w << 32);
        return (bad & ~mask64((uint32_t)e.pv_cap)) == 0ull;
      }
    }
  }
  // exemptExclusions for one exclude over the errors E of its pod view; conv: the defaults went
  // through convertChecks (a PolicyException's excludes), so annotation fields never compare
  __device__ __forceinline__ void exempt(const KpeXExcl& e, bool conv) {
    const bool by_image = e.img != -1;
    const uint32_t rf_ann = e.rf_kind == XRF_ANN ? a.rf_ann[e.rf_key] : KPE_NO_STR;
    const uint32_t n = ne < kXCap ? ne : kXCap;
    for (uint32_t j = 0; j < n && nd; ++j) {
      const uint4 x = E[j];
      const uint32_t key = x.x & 0xFFFFu;
      if (e.rf_kind == XRF_NEVER) break;
      if (conv && key == XKEY(XF_ANN, XT_POD)) continue;  // now spec.template.metadata.annotations[..]
      if (e.rf_kind == XRF_FIELD && key != e.rf_key) continue;
      if (e.rf_kind == XRF_ANN && (key != XKEY(XF_ANN, XT_POD) || x.y != rf_ann || rf_ann == KPE_NO_STR)) continue;
      if (!values_ok(e, x)) continue;
      const bool aux = by_image || key == XKEY(XF_ANN, XT_POD);  // names (image exclusions) / annotation keys
      for (uint32_t d = 0; d < nd; ++d)
        if (D[d].x == key && (!aux || D[d].y == x.y)) {
          D[d] = D[nd - 1];  // evaluate.go:184-187 remove(): swap with the last, truncate
          --nd;
          break;
        }
    }
  }
};

// kpe_pssx_kernel's body for pod r. The scan wrote each exclusion rule's plain PSS verdict
// (KPE_XFAIL_ where a podSecurity PolicyException matched); a failing pod is re-evaluated with
// its exclusions (EvaluatePod), then with the exception's (validate_pss.go:88-104). One gen()
// call site: the loop walks (1) every versioned check on the pod, then per excluded failing
// check (2) its default errors and (3) each naming exclude's errors of every version on that
// exclude's view, the rule's excludes first.
__device__ __forceinline__ void pssx_eval_row(const PssxArgs& a, int64_t r) {
  uint8_t* row = a.verdicts + (size_t)r * a.R;
  PssxVM vm(a, r);
  const uint32_t* rec = a.rec + 4 * r;
  vm.pw = rec[0] & 0xFFFFFu;
  const bool pod = ((rec[0] >> PR_CLASS_SH) & R_CLASS_MASK) == R_CLASS_POD;
  vm.c0 = a.ctr_off[r], vm.c1 = a.ctr_off[r + 1];
  vm.v0 = a.vol_off[r], vm.v1 = a.vol_off[r + 1];
  vm.s0 = a.sys_off[r], vm.s1 = a.sys_off[r + 1];
  vm.a0 = a.pann_off[r], vm.a1 = a.pann_off[r + 1];
  for (uint32_t ri = 0; ri < a.nxr; ++ri) {
    const KpeXRule xr = a.rules[ri];
    const uint8_t cell = row[xr.col];
    const bool xc = cell == KPE_XFAIL_;  // a podSecurity exception matched the pod
    if (cell != KPE_PASS_ && cell != KPE_FAIL_ && !xc) continue;  // not evaluated (NA, error, skip, ...)
    uint32_t* mk = a.masks ? a.masks + (size_t)r * a.R + xr.col : nullptr;
    const uint32_t xforce = XR_XFORCE(xr.xn);
    if (xr.force != XR_FORCE_NONE) {  // an invalid exclude: results nil (EvaluatePod)
      // not allowed under the exception: ApplyPodSecurityExclusion over no checks
      row[xr.col] = xr.force == XR_FORCE_PASS ? KPE_PASS_ : (!xc || xforce == XR_FORCE_FAIL) ? KPE_FAIL_ : KPE_SKIP_;
      if (mk) *mk = 0u;
      continue;
    }
    if (cell == KPE_PASS_ || (!xc && xr.nexcl == 0u)) continue;  // nothing to exempt
    // the exception's excludes can remove errors only when they run (no invalid entry) on a Pod:
    // convertChecks rewrites every field of a controller / CronJob
    const uint32_t total = xr.nexcl + ((xc && xforce == XR_FORCE_NONE && pod) ? XR_XN(xr.xn) : 0u);
    uint32_t ph = 0, rem_v = xr.cv_mask, fails = 0, rem_k = 0, k = 0, vk = 0, ei = 0, rem_x = 0, out = 0, out_rule = 0;
    KpeXExcl ex{};
    bool undec = false, rdone = false, conv = false;
    for (;;) {
      uint32_t cv, view = VW_REAL, img = PRED_NONE;
      if (ph == 0u) {  // every versioned check on the pod (evaluatePSS)
        if (!rem_v) {
          uint32_t fk = 0;
          for (uint32_t c = 0; c < KPE_NUM_CHECKS; ++c)
            if (fails & check_versions(c)) fk |= 1u << c;
          for (uint32_t m = fk & ~xr.kx; m; m &= m - 1u)  // failing checks no exclude names: kept
            out |= 1u << (31u - __builtin_clz(fails & check_versions(__builtin_ctz(m))));
          out_rule = out;
          rem_k = fk & xr.kx;
          ph = 1u;
          continue;
        }
        cv = __builtin_ctz(rem_v);
        rem_v &= rem_v - 1u;
      } else if (ph == 1u) {  // next excluded failing check: its default (last failing version) errors
        if (!rem_k) break;
        k = __builtin_ctz(rem_k);
        rem_k &= rem_k - 1u;
        vk = 31u - __builtin_clz(fails & check_versions(k));
        cv = vk, ei = 0, rem_x = 0, rdone = false;
      } else {  // the next (exclude, version) of check k
        if (!rem_x) {
          while (ei < total && !(a.excl[ei < xr.nexcl ? xr.excl0 + ei : xr.xexcl0 + ei - xr.nexcl].checks & (1u << k)))
            ++ei;
          if (!rdone && (ei >= xr.nexcl || vm.nd == 0u)) {  // the rule's excludes are done
            rdone = true;
            if (vm.nd) out_rule |= 1u << vk;
          }
          if (ei >= total || vm.nd == 0u) {
            if (vm.nd) out |= 1u << vk;  // errors left: the check still fails
            ph = 1u;
            continue;
          }
          conv = ei >= xr.nexcl;
          ex = a.excl[conv ? xr.xexcl0 + ei - xr.nexcl : xr.excl0 + ei];
          ++ei;
          rem_x = xr.cv_mask & check_versions(k);
        }
        cv = __builtin_ctz(rem_x);
        rem_x &= rem_x - 1u;
        view = ex.img == -1 ? VW_SPEC : VW_MATCH;
        img = (uint32_t)ex.img;
      }
      vm.gen(cv, view, img);  // the one call site
      if (ph == 0u) {
        if (vm.ne) fails |= 1u << cv;
        continue;
      }
      if (vm.ne > kXCap) {  // more errors than the lane buffers hold: the caller decides
        undec = true;
        break;
      }
      if (ph == 1u) {
        for (uint32_t j = 0; j < vm.ne; ++j) vm.D[j] = make_uint2(vm.E[j].x & 0xFFFFu, vm.E[j].y);
        vm.nd = vm.ne;
        ph = 2u;
      } else {
        vm.exempt(ex, conv);
      }
    }
    if (undec) {
      row[xr.col] = KPE_UNDECIDED_;
      continue;
    }
    // validate_pss.go:84-110: allowed => pass; else, under the exception, no checks left and no
    // error => skip; the fail response carries the checks from before the exception
    uint8_t v = KPE_PASS_;
    if (out_rule)
      v = (!xc || xforce == XR_FORCE_FAIL || (xforce == XR_FORCE_NONE && out)) ? KPE_FAIL_ : KPE_SKIP_;
    row[xr.col] = v;
    if (mk) *mk = v == KPE_FAIL_ ? out_rule | (xc ? KPE_CVM_XMATCH : 0u) : 0u;
  }
}
