// kss_eval.cuh — per-(pod,node) predicates and raw scores, device side (gfx950).
//
// Each function restates one upstream v1.26.2 plugin step (cited) over the
// interned struct-of-arrays of include/kss.h.  Everything here is integer or
// IEEE double arithmetic compiled with -ffp-contract=off, so results are
// bit-identical to the reference operation order.  One lane evaluates one node;
// pod programs are wave-uniform (read through the scalar cache).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kss.h"

// Debug builds (make debug -> libkss_dbg.so) check every data-dependent global index
// and trap with the offending values; release builds compile the checks away.
#ifdef KSS_DEBUG_BOUNDS
#define KSS_DCHECK(cond, what, a, b)                                                                      \
  do {                                                                                                    \
    if (!(cond)) {                                                                                        \
      printf("KSS_DCHECK %s a=%lld b=%lld block=%d thread=%d\n", what, (long long)(a), (long long)(b),     \
             (int)blockIdx.x, (int)threadIdx.x);                                                          \
      __builtin_trap();                                                                                   \
    }                                                                                                     \
  } while (0)
#else
#define KSS_DCHECK(cond, what, a, b) \
  do {                               \
  } while (0)
#endif

namespace kss {

// Device view of a loaded cluster.  Row r of a [attr][N] matrix starts at r*N.
struct DevCluster {
  int32_t N;
  int32_t n_scalar;
  int32_t n_keys;
  int32_t n_classes;
  int32_t n_terms;
  int32_t node_base;
  int32_t class_cap;
  int32_t term_cap;
  const int64_t* alloc;
  int64_t* requested;
  int64_t* nonzero;
  const int32_t* allowed_pods;
  int32_t* pod_count;
  const uint32_t* node_flags;
  const uint64_t* taint_hard;
  const uint64_t* taint_soft;
  const uint8_t* taint_order;
  const int32_t* label_value;
  const int32_t* key_base;
  const int32_t* key_card;
  const uint32_t* key_flags;
  const int32_t* key_empty;
  const int64_t* value_int;
  const uint8_t* value_is_int;
  int32_t* class_count;
  int32_t* term_count;
  const double* log_table;  // go_log(k + 2), k in [0, N]
  uint64_t* port_used;        // [N] NodeInfo.UsedPorts dictionary bits (mutable: AssumePod adds)
  const int64_t* image_score; // [n_images][N] scaledImageScore, 0 = image absent
  int32_t n_images;
  // volumes (include/kss.h kss_cluster): vol_count [rows][N] and vol_attached [keys][N] are
  // mutable (AssumePod adds), vol_limit [keys][N] static
  int32_t n_vol_rows, n_vol_keys;
  int32_t* vol_count;
  int32_t* vol_attached;
  const int32_t* vol_limit;
  const int32_t* vol_row_key;
  const int32_t* vol_key_plugin;
  // the binder's assume cache for WaitForFirstConsumer claims (kss_cluster pv_owner / claim_node):
  // mutable, with the snapshot's values beside them (ForgetPod restores those)
  int32_t n_pvs, n_wclaims;
  int32_t* pv_owner;
  int32_t* claim_node;
  const int32_t* pv_owner0;
  const int32_t* claim_node0;
  // Shard-resident LDS copies of the hot node columns (set inside the kernel; null on
  // the host and in kernels without a cache).  Slot i holds node nc_lo + i.
  int64_t* nc64;    // [8][nc_cap]: alloc cpu/mem/eph, requested cpu/mem/eph, nonzero cpu/mem
  uint64_t* nct;    // [2][nc_cap]: taint_hard, taint_soft
  int32_t* nc32;    // [3][nc_cap]: pod_count, allowed_pods, node_flags
  int32_t* ncl;     // [n_keys][nc_cap]: label value ids, or null (read from HBM)
  int32_t nc_lo, nc_cap;
};

// One node's hot columns, loaded once per (pod, node) into registers.
// One entry of the scheduling queue's nominator (kss_nominate): a pod nominated to a node by an
// earlier preemption, with what NodeInfo.AddPodInfo and the AddPod PreFilter extensions need.
struct DevNom {
  int32_t node;      // local row
  int32_t prio;      // corev1helpers.PodPriority
  int32_t pod;       // the pod's identity: its index in the podset
  int32_t cls;       // class_count row (labels + namespace)
  int32_t n_terms;   // term_count rows it contributes
  int32_t terms[8];
  int32_t pad;
  uint64_t ports;    // NodeInfo.UsedPorts bits it adds
  int64_t req[KSS_NRES];
};
constexpr int KSS_NOM_MAX = 64;  // entries (one 64-bit activity mask)

struct NodeRow {
  int64_t alloc[3], req[3], nz[2];
  uint64_t th, ts;
  int32_t pods, allowed;
  uint32_t flags;
};

// a[r] for a runtime r in [0, 3) without dynamic register indexing
__device__ __forceinline__ int64_t pick3(const int64_t (&a)[3], int r) { return r == 0 ? a[0] : (r == 1 ? a[1] : a[2]); }

__device__ __forceinline__ NodeRow row_from_hbm(const DevCluster& c, int n) {
  KSS_DCHECK(n >= 0 && n < c.N, "row_from_hbm n", n, c.N);
  NodeRow r;
  const size_t N = (size_t)c.N;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    r.alloc[k] = c.alloc[k * N + n];
    r.req[k] = c.requested[k * N + n];
  }
  r.nz[0] = c.nonzero[n];
  r.nz[1] = c.nonzero[N + n];
  r.th = c.taint_hard[n];
  r.ts = c.taint_soft[n];
  r.pods = c.pod_count[n];
  r.allowed = c.allowed_pods[n];
  r.flags = c.node_flags[n];
  return r;
}

__device__ __forceinline__ NodeRow load_row(const DevCluster& c, int n) {
  if (!c.nc64) return row_from_hbm(c, n);
  NodeRow r;
  const int i = n - c.nc_lo, C = c.nc_cap;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    r.alloc[k] = c.nc64[k * C + i];
    r.req[k] = c.nc64[(3 + k) * C + i];
  }
  r.nz[0] = c.nc64[6 * C + i];
  r.nz[1] = c.nc64[7 * C + i];
  r.th = c.nct[i];
  r.ts = c.nct[C + i];
  r.pods = c.nc32[i];
  r.allowed = c.nc32[C + i];
  r.flags = (uint32_t)c.nc32[2 * C + i];
  return r;
}

__device__ __forceinline__ uint64_t taint_hard_of(const DevCluster& c, int n) {
  return c.nct ? c.nct[n - c.nc_lo] : c.taint_hard[n];
}

__device__ __forceinline__ uint32_t node_flags_of(const DevCluster& c, int n) {
  return c.nc32 ? (uint32_t)c.nc32[2 * c.nc_cap + (n - c.nc_lo)] : c.node_flags[n];
}

// Split grid (node axis over several GPUs, kss_split_*): a launch runs shards
// [w_off, w_off + wl) of the W shards of the cluster; every exchange granule is published to
// each part's inbox (device pointers valid in this process: IPC-mapped for other GPUs) with
// system-scope stores, and polled in the local inbox only.  n <= 1: one launch owns the grid.
constexpr int KSS_MAX_PARTS = 8;
struct XPeers {
  int32_t n;
  int32_t w_off;
  int32_t wl;
  int32_t xcd_local;  // k_simple, one part: every shard on one XCD (xcd_slot), granules published with plain stores
  unsigned long long* inbox[KSS_MAX_PARTS];
  unsigned long long* tl;  // k_spread, one part, many shards: the two-level selectHost exchange's area (null: off)
  int32_t tl_red;          // ... the statistics / filter exchanges in two levels too (spread_exchange_tl)
};


struct DevPods {
  const kss_pod* pods;
  const kss_req* reqs;
  const kss_term* terms;
  const kss_spread* spreads;
  const kss_ipa* ipa;
  const int32_t* ints;
  const kss_vol* vols;
};

__device__ __forceinline__ int32_t label_of(const DevCluster& c, int key, int n) {
  if (c.ncl) return c.ncl[key * c.nc_cap + (n - c.nc_lo)];
  KSS_DCHECK(key >= 0 && key < c.n_keys && n >= 0 && n < c.N, "label_of key/n", key, n);
  return c.label_value[(size_t)key * (size_t)c.N + (size_t)n];
}

// labels.Requirement.Matches over value ids (apimachinery labels/selector.go) and the
// metadata.name field selector (component-helpers nodeaffinity).  g is the global node
// index, lab(key) the node's value id for a label key (-1 absent), ints the pool of
// IN / NOTIN value lists: the HBM path and the LDS path (kss_simple.cuh) share it.
template <class Lab>
__device__ __forceinline__ bool req_match_t(const DevCluster& c, const int32_t* ints, const kss_req& r, int64_t g, Lab lab) {
  const int op = r.op;
  if (op == KSS_OP_FALSE) return false;
  if (op == KSS_OP_TRUE) return true;
  if (op == KSS_OP_NAME_IN) return r.ival >= 0 && g == r.ival;
  if (op == KSS_OP_NAME_NOTIN) return !(r.ival >= 0 && g == r.ival);
  const int32_t v = lab(r.key);
  switch (op) {
    case KSS_OP_MASK:
      if (v < 0) return (r.mask >> 63) & 1ull;
      return v < 63 ? ((r.mask >> v) & 1ull) : false;
    case KSS_OP_IN: {
      if (v < 0) return false;
      for (int i = 0; i < r.list_len; i++)
        if (ints[r.list_off + i] == v) return true;
      return false;
    }
    case KSS_OP_NOTIN: {
      if (v < 0) return true;
      for (int i = 0; i < r.list_len; i++)
        if (ints[r.list_off + i] == v) return false;
      return true;
    }
    case KSS_OP_EXISTS:
      return v >= 0;
    case KSS_OP_DNE:
      return v < 0;
    case KSS_OP_GT:
    case KSS_OP_LT: {
      if (v < 0) return false;
      const int32_t gi = c.key_base[r.key] + v;
      if (!c.value_is_int[gi]) return false;
      const int64_t x = c.value_int[gi];
      return op == KSS_OP_GT ? x > r.ival : x < r.ival;
    }
    default:
      return false;
  }
}

template <class Lab>
__device__ __forceinline__ bool term_match_t(const DevCluster& c, const kss_req* reqs, const int32_t* ints,
                                             const kss_term& t, int64_t g, Lab lab) {
  for (int i = 0; i < t.req_len; i++)
    if (!req_match_t(c, ints, reqs[t.req_off + i], g, lab)) return false;
  return true;
}

// nodeaffinity.RequiredNodeAffinity.Match: nodeSelector AND (OR over terms)
template <class Lab>
__device__ __forceinline__ bool required_affinity_t(const DevCluster& c, const kss_req* reqs, const kss_term* terms,
                                                    const int32_t* ints, const kss_pod& p, int64_t g, Lab lab) {
  for (int i = 0; i < p.sel_len; i++)
    if (!req_match_t(c, ints, reqs[p.sel_off + i], g, lab)) return false;
  if (p.flags & KSS_POD_HAS_REQ_AFFINITY) {
    for (int t = 0; t < p.aff_len; t++)
      if (term_match_t(c, reqs, ints, terms[p.aff_off + t], g, lab)) return true;
    return false;
  }
  return true;
}

// NodeAffinity.Score: PreferredSchedulingTerms.Score
template <class Lab>
__device__ __forceinline__ int64_t na_score_t(const DevCluster& c, const kss_req* reqs, const kss_term* terms,
                                              const int32_t* ints, const kss_pod& p, int64_t g, Lab lab) {
  int64_t s = 0;
  for (int t = 0; t < p.pref_len; t++) {
    const kss_term& term = terms[p.pref_off + t];
    if (term_match_t(c, reqs, ints, term, g, lab)) s += term.weight;
  }
  return s;
}

// the same over HBM (or shard-cache) labels and the pooled pod programs
__device__ __forceinline__ bool required_affinity(const DevCluster& c, const DevPods& P, const kss_pod& p, int n) {
  return required_affinity_t(c, P.reqs, P.terms, P.ints, p, (int64_t)c.node_base + n,
                             [&](int key) { return label_of(c, key, n); });
}

// v1helper.FindMatchingUntoleratedTaint(node.Spec.Taints, tolerations, DoNotScheduleTaintsFilterFunc)
__device__ __forceinline__ int first_untolerated(const DevCluster& c, const kss_pod& p, int n, uint64_t th) {
  const uint64_t untol = th & ~p.tol_hard;
  if (!untol) return -1;
  KSS_DCHECK(n >= 0 && n < c.N, "first_untolerated n", n, c.N);
  const uint8_t* ord = c.taint_order + (size_t)n * KSS_TAINT_ORDER;
#pragma unroll
  for (int i = 0; i < KSS_TAINT_ORDER; i++) {
    const int t = ord[i];
    if (t == 0xFF) break;
    if ((untol >> t) & 1ull) return t;
  }
  return 63 - __clzll(untol);
}

__device__ __forceinline__ int64_t sum_rows(const int32_t* mat, size_t N, const int32_t* rows, int len, int n) {
  int64_t s = 0;
  for (int i = 0; i < len; i++) {
    KSS_DCHECK(rows[i] >= 0 && rows[i] < 4096 && n >= 0 && (size_t)n < N, "sum_rows row/n", rows[i], n);
    s += mat[(size_t)rows[i] * N + (size_t)n];
  }
  return s;
}

// First-failing filter among NodeUnschedulable, NodeName, TaintToleration,
// NodeAffinity, (NodePorts), NodeResourcesFit — the ones that need no per-pod
// cluster-wide state.  Returns 0 when all of them pass.
// nom / here: the nominated pods added to the node (RunFilterPluginsWithNominatedPods' first
// pass: NodeInfo.AddPodInfo of each entry whose bit is set) -- null for the plain pass.
__device__ __forceinline__ int filter_local(const DevCluster& c, const DevPods& P, const kss_pod& p,
                                            uint32_t enabled, int n, const NodeRow& row, uint16_t* detail,
                                            const DevNom* nom = nullptr, uint64_t here = 0) {
  const int xpods = nom ? __popcll(here) : 0;
  uint64_t xports = 0;
  if (nom)
    for (uint64_t m = here; m; m &= m - 1) xports |= nom[__ffsll((unsigned long long)m) - 1].ports;
  // NodeUnschedulable.Filter
  if ((enabled >> KSS_F_NODE_UNSCHEDULABLE) & 1u) {
    if ((row.flags & KSS_NODE_UNSCHEDULABLE) && !(p.flags & KSS_POD_TOL_UNSCHEDULABLE))
      return KSS_F_NODE_UNSCHEDULABLE;
  }
  // NodeName.Fits
  if ((enabled >> KSS_F_NODE_NAME) & 1u) {
    if (p.node_name != -1 && (int64_t)p.node_name != (int64_t)c.node_base + n) return KSS_F_NODE_NAME;
  }
  // TaintToleration.Filter
  if ((enabled >> KSS_F_TAINT_TOLERATION) & 1u) {
    const int t = first_untolerated(c, p, n, row.th);
    if (t >= 0) {
      *detail = (uint16_t)t;
      return KSS_F_TAINT_TOLERATION;
    }
  }
  // NodeAffinity.Filter
  if ((enabled >> KSS_F_NODE_AFFINITY) & 1u) {
    if (!required_affinity(c, P, p, n)) return KSS_F_NODE_AFFINITY;
  }
  // NodePorts.Filter -> fitsPorts: HostPortInfo.CheckConflict of every wanted port
  if ((enabled >> KSS_F_NODE_PORTS) & 1u) {
    if (p.port_conflict && ((c.port_used[n] | xports) & p.port_conflict)) return KSS_F_NODE_PORTS;
  }
  // NodeResourcesFit.Filter -> fitsRequest
  if ((enabled >> KSS_F_NODE_RESOURCES_FIT) & 1u) {
    const size_t N = (size_t)c.N;
    uint32_t bits = 0;
    if ((int64_t)row.pods + xpods + 1 > (int64_t)row.allowed) bits |= KSS_FIT_TOO_MANY_PODS;
    const int nr = 3 + c.n_scalar;
    bool all_zero = true;
    for (int r = 0; r < nr; r++) all_zero &= (p.fit_request[r] == 0);
    if (!all_zero) {
      for (int r = 0; r < nr; r++) {
        const int64_t req = p.fit_request[r];
        if (r >= KSS_RES_SCALAR0 && req == 0) continue;
        int64_t freev = r < 3 ? pick3(row.alloc, r) - pick3(row.req, r)
                              : c.alloc[(size_t)r * N + n] - c.requested[(size_t)r * N + n];
        if (nom)
          for (uint64_t m = here; m; m &= m - 1) freev -= nom[__ffsll((unsigned long long)m) - 1].req[r];
        if (req > freev) bits |= 1u << (r + 1);
      }
    }
    if (bits) {
      *detail = (uint16_t)bits;
      return KSS_F_NODE_RESOURCES_FIT;
    }
  }
  return 0;
}

// The volume filters (VolumeRestrictions, EBSLimits, GCEPDLimits, NodeVolumeLimits,
// AzureDiskLimits, VolumeBinding, VolumeZone: default MultiPoint order) over the pod's volume
// program, whose entries the host sorted into that order (kss/volumes.py).  Returns the first
// failing plugin (detail in *detail) or 0.  Restates, per node:
//   volume_restrictions.go satisfyVolumeConflicts: a pod volume conflicts with a volume of a
//     pod on the node (the host resolved isVolumeConflict into the rows each entry names);
//   non_csi.go nonCSILimits.Filter / csi.go CSILimits.Filter: per limit key, the pod's volumes
//     not already attached on the node (newVolumes minus attachedVolumes) on top of the
//     node's distinct attached ones against the node's limit (CSI: only keys with a new volume);
//   binder.go checkBoundClaims: the bound claims in order; a missing PV or a PV whose node
//     affinity does not match the node's labels ends the walk;
//   volume_zone.go Filter: on nodes carrying a zone label, every zone label of the pod's PVs
//     must name the node's value, volumes in order (per-volume errors as messages).
// One attach-limit key of the pod on node n: its plugin when the node's limit is exceeded.
// nonCSILimits counts existing + new volumes whenever the pod has a volume of the plugin;
// CSILimits checks only keys with a new volume.
__device__ __forceinline__ int limit_exceeded(const DevCluster& c, int key, int n, int64_t newc, uint32_t enabled) {
  const size_t N = (size_t)c.N;
  const int pl = c.vol_key_plugin[key];
  const int32_t lim = c.vol_limit[(size_t)key * N + n];
  if (!((enabled >> pl) & 1u) || lim < 0) return 0;
  if (pl == KSS_F_NODE_VOLUME_LIMITS && newc == 0) return 0;
  return (int64_t)c.vol_attached[(size_t)key * N + n] + newc > (int64_t)lim ? pl : 0;
}

__device__ __forceinline__ bool vb_kind(int k) {
  return k == KSS_VOL_BIND_AFFINITY || k == KSS_VOL_BIND_PV_MISSING || k == KSS_VOL_BIND_WFFC;
}

// pv_helpers.go FindMatchingVolume for delayed claim entry v on node n (candidates: ints[v.a ..],
// {pv, term_off, term_len} triplets in increasing capacity, then name): a PV bound to the claim
// (pv_owner == key + 1: its claimRef, or assumed by AssumePodVolumes) and not chosen by an earlier
// claim of the pod (chosen[0 .. nch): excludedVolumes; a pod can list one claim twice) is returned
// -- or nothing, when its node affinity fails -- wherever it comes; else the first available PV not
// chosen whose node affinity matches.  -1: no match.
template <class Lab>
__device__ __forceinline__ int wffc_match(const DevCluster& c, const kss_req* reqs, const kss_term* terms,
                                          const int32_t* ints, const kss_vol& v, const int (&chosen)[KSS_MAX_WFFC],
                                          int nch, Lab lab) {
  auto node_ok = [&](int i) {  // volumeutil.CheckNodeAffinity(pv, node.Labels)
    const int ta = ints[v.a + 3 * i + 1], tb = ints[v.a + 3 * i + 2];
    if (tb < 0) return true;
    bool ok = false;
    for (int t = 0; t < tb && !ok; t++) ok = term_match_t(c, reqs, ints, terms[ta + t], -1, lab);
    return ok;
  };
  for (int i = 0; i < v.b; i++) {  // excludedVolumes come first: a PV an earlier claim took is skipped
    const int pv = ints[v.a + 3 * i];
    bool taken = false;
    for (int k = 0; k < KSS_MAX_WFFC; k++) taken |= k < nch && chosen[k] == pv;
    if (!taken && c.pv_owner[pv] == v.key + 1) return node_ok(i) ? pv : -1;
  }
  for (int i = 0; i < v.b; i++) {
    const int pv = ints[v.a + 3 * i];
    if (c.pv_owner[pv] != 0) continue;
    bool taken = false;
    for (int k = 0; k < KSS_MAX_WFFC; k++) taken |= k < nch && chosen[k] == pv;
    if (taken || !node_ok(i)) continue;
    return pv;
  }
  return -1;
}

// VolumeBinding.Filter -> binder.go FindPodVolumes on node n over the pod's VolumeBinding
// entries [e0, e1): checkBoundClaims (BIND_AFFINITY / BIND_PV_MISSING in claim order, the first
// failure ends it), then the delayed claims (BIND_WFFC): a claim selected for another node fails
// at once; findMatchingVolumes over the others; checkVolumeProvisions over the selected and the
// unmatched ones.  Returns -1 when satisfied, else the KSS_VB_* detail (the reasons in
// FindPodVolumes' order: node conflict, bind conflict, PV not exist).  pick (optional): per
// BIND_WFFC entry in order, the statically bound PV, or -1 for a provisioned claim
// (AssumePodVolumes' podVolumes).
template <class Lab>
__device__ __forceinline__ int vb_eval(const DevCluster& c, const kss_req* reqs, const kss_term* terms,
                                       const int32_t* ints, const kss_vol* vols, int e0, int e1, int n, Lab lab,
                                       int* pick = nullptr) {
  int bound = 0;  // 1 node conflict, 2 a bound claim's PV does not exist
  for (int e = e0; e < e1 && bound == 0; e++) {
    const kss_vol& v = vols[e];
    if (v.kind == KSS_VOL_BIND_PV_MISSING) {
      bound = 2;
    } else if (v.kind == KSS_VOL_BIND_AFFINITY) {
      bool ok = false;
      for (int t = 0; t < v.b && !ok; t++) ok = term_match_t(c, reqs, ints, terms[v.a + t], -1, lab);
      if (!ok) bound = 1;
    }
  }
  bool unbound_ok = true;
  for (int e = e0; e < e1 && unbound_ok; e++)  // the selected-node fast path
    if (vols[e].kind == KSS_VOL_BIND_WFFC) {
      const int sel = c.claim_node[vols[e].key];
      if (sel != -1 && sel != n) unbound_ok = false;
    }
  if (unbound_ok) {
    int chosen[KSS_MAX_WFFC] = {-1, -1, -1, -1};
    int nch = 0, wi = 0;
    unsigned prov = 0;  // the claims to provision: selected for this node, or without a match
    for (int e = e0; e < e1; e++) {
      const kss_vol& v = vols[e];
      if (v.kind != KSS_VOL_BIND_WFFC) continue;
      int m = -1;
      if (c.claim_node[v.key] == -1) {
        m = wffc_match(c, reqs, terms, ints, v, chosen, nch, lab);
        if (m >= 0 && nch < KSS_MAX_WFFC) chosen[nch++] = m;
        if (m < 0) unbound_ok = false;  // foundMatches false: the provisioning check decides below
      }
      if (m < 0) prov |= 1u << wi;
      if (pick && wi < KSS_MAX_WFFC) pick[wi] = m;
      wi++;
    }
    if (prov) {  // checkVolumeProvisions: a provisioner, and the class's allowedTopologies admit the node
      unbound_ok = true;
      wi = 0;
      for (int e = e0; e < e1 && unbound_ok; e++) {
        const kss_vol& v = vols[e];
        if (v.kind != KSS_VOL_BIND_WFFC) continue;
        if ((prov >> wi) & 1u) {
          if (!(v.count & 1)) {
            unbound_ok = false;
          } else if ((v.count >> 1) > 0) {
            bool ok = false;
            for (int t = 0; t < (v.count >> 1) && !ok; t++) ok = term_match_t(c, reqs, ints, terms[v.row + t], -1, lab);
            unbound_ok = ok;
          }
        }
        wi++;
      }
    }
  }
  if (!unbound_ok) return bound == 1 ? KSS_VB_NODE_BIND : (bound == 2 ? KSS_VB_BIND_PV_NOT_EXIST : KSS_VB_BIND_CONFLICT);
  return bound == 1 ? KSS_VB_NODE_CONFLICT : (bound == 2 ? KSS_VB_PV_NOT_EXIST : -1);
}

// Reserve's AssumePodVolumes (sign 1) on node `local`: the static bindings' PVs become the claims'
// (pv_owner), the provisioned claims select the node (claim_node); Unreserve's
// RevertAssumedPodVolumes (sign -1): the claims' PVs and the claims back to the snapshot's values.
// Every shard of a grid runs it with the same result (the columns are global, not per node).
template <class Lab>
__device__ __forceinline__ void wffc_commit(const DevCluster& c, const kss_req* reqs, const kss_term* terms,
                                            const int32_t* ints, const kss_vol* vols, const kss_pod& p, int local,
                                            int sign, Lab lab) {
  int e0 = -1, e1 = -1;
  for (int e = 0; e < p.vol_len; e++)
    if (vb_kind(vols[p.vol_off + e].kind)) {
      if (e0 < 0) e0 = p.vol_off + e;
      e1 = p.vol_off + e + 1;
    }
  if (e0 < 0) return;
  bool any = false;
  for (int e = e0; e < e1; e++) any |= vols[e].kind == KSS_VOL_BIND_WFFC;
  if (!any) return;
  if (sign > 0) {
    int pick[KSS_MAX_WFFC] = {-1, -1, -1, -1};
    vb_eval(c, reqs, terms, ints, vols, e0, e1, local, lab, pick);
    int wi = 0;
    for (int e = e0; e < e1; e++) {
      const kss_vol& v = vols[e];
      if (v.kind != KSS_VOL_BIND_WFFC) continue;
      if (wi < KSS_MAX_WFFC && pick[wi] >= 0) c.pv_owner[pick[wi]] = v.key + 1;
      else c.claim_node[v.key] = local;
      wi++;
    }
  } else {
    for (int e = e0; e < e1; e++) {
      const kss_vol& v = vols[e];
      if (v.kind != KSS_VOL_BIND_WFFC) continue;
      for (int i = 0; i < v.b; i++) {
        const int pv = ints[v.a + 3 * i];
        if (c.pv_owner[pv] == v.key + 1) c.pv_owner[pv] = c.pv_owner0[pv];
      }
      c.claim_node[v.key] = c.claim_node0[v.key];
    }
  }
}

template <class Lab>
__device__ __forceinline__ int filter_volumes_t(const DevCluster& c, const kss_req* reqs, const kss_term* terms,
                                                const int32_t* ints, const kss_vol* vols, const kss_pod& p,
                                                uint32_t enabled, int n, uint32_t node_flags, uint16_t* detail,
                                                Lab lab) {
  const size_t N = (size_t)c.N;
  int cur = -1;      // the limit key of the open segment
  int64_t newc = 0;  // its new volumes on this node
  for (int e = 0; e < p.vol_len; e++) {
    const kss_vol v = vols[p.vol_off + e];
    if (v.kind != KSS_VOL_LIMIT && cur >= 0) {  // the open segment ends: check it
      if (const int pl = limit_exceeded(c, cur, n, newc, enabled)) return pl;
      cur = -1;
    }
    switch (v.kind) {
      case KSS_VOL_CONFLICT:
        if (((enabled >> KSS_F_VOLUME_RESTRICTIONS) & 1u) && c.vol_count[(size_t)v.row * N + n] > 0)
          return KSS_F_VOLUME_RESTRICTIONS;
        break;
      case KSS_VOL_LIMIT:
        if (v.key != cur) {
          if (cur >= 0)  // the previous key's segment ends
            if (const int pl = limit_exceeded(c, cur, n, newc, enabled)) return pl;
          cur = v.key;
          newc = 0;
        }
        newc += v.row >= 0 ? (c.vol_count[(size_t)v.row * N + n] == 0 ? 1 : 0) : v.count;
        break;
      case KSS_VOL_BIND_AFFINITY:
      case KSS_VOL_BIND_PV_MISSING:
      case KSS_VOL_BIND_WFFC: {  // VolumeBinding: its entries (consecutive) as one FindPodVolumes
        int e1 = e + 1;
        while (e1 < p.vol_len && vb_kind(vols[p.vol_off + e1].kind)) e1++;
        if ((enabled >> KSS_F_VOLUME_BINDING) & 1u) {
          const int d = vb_eval(c, reqs, terms, ints, vols, p.vol_off + e, p.vol_off + e1, n, lab);
          if (d >= 0) {
            *detail = (uint16_t)d;
            return KSS_F_VOLUME_BINDING;
          }
        }
        e = e1 - 1;
        break;
      }
      case KSS_VOL_ZONE:
        if (((enabled >> KSS_F_VOLUME_ZONE) & 1u) && (node_flags & KSS_NODE_VOLUME_ZONE)) {
          for (int k = 0; k < v.b; k++)
            if (!req_match_t(c, ints, reqs[v.a + k], -1, lab)) {
              *detail = 0;
              return KSS_F_VOLUME_ZONE;
            }
        }
        break;
      case KSS_VOL_ZONE_ERROR:
        if (((enabled >> KSS_F_VOLUME_ZONE) & 1u) && (node_flags & KSS_NODE_VOLUME_ZONE)) {
          *detail = (uint16_t)(1 + v.a);
          return KSS_F_VOLUME_ZONE;
        }
        break;
      default:  // AssumePod entries close the program
        return 0;
    }
  }
  if (cur >= 0) return limit_exceeded(c, cur, n, newc, enabled);
  return 0;
}

__device__ __forceinline__ int filter_volumes(const DevCluster& c, const DevPods& P, const kss_pod& p, uint32_t enabled,
                                              int n, uint16_t* detail) {
  if (p.vol_len <= 0) return 0;
  return filter_volumes_t(c, P.reqs, P.terms, P.ints, P.vols, p, enabled, n, node_flags_of(c, n), detail,
                          [&](int key) { return label_of(c, key, n); });
}

// AssumePod (sign 1) / ForgetPod (-1) of one KSS_VOL_OWN row on node `local`: the row's pod
// count moves, and the row's key counts the volume once while some pod on the node uses it.
__device__ __forceinline__ void vol_commit_row(const DevCluster& c, int row, int local, int sign) {
  const size_t N = (size_t)c.N;
  int32_t* cnt = c.vol_count + (size_t)row * N + local;
  const int key = c.vol_row_key[row];
  if (sign > 0) {
    if (key >= 0 && *cnt == 0) c.vol_attached[(size_t)key * N + local] += 1;
    *cnt += 1;
  } else {
    *cnt -= 1;
    if (key >= 0 && *cnt == 0) c.vol_attached[(size_t)key * N + local] -= 1;
  }
}

// Go int64 division a / b for the non-negative operands the scores produce: one f64
// division (exact operands below 2^53, error of the rounded quotient < 1) and an exact
// integer correction; anything else takes the integer division.
__device__ __forceinline__ int64_t div_f53(int64_t a, int64_t b) {
  int64_t q = (int64_t)((double)a / (double)b);
  const int64_t r = a - q * b;
  return r < 0 ? q - 1 : (r >= b ? q + 1 : q);
}

// SMALL = true: the caller guarantees 0 <= a, b < 2^53 (k_simple: the host checks every
// allocatable value and profile weight at load), so the integer fallback is not compiled.
template <bool SMALL = false>
__device__ __forceinline__ int64_t div_i64(int64_t a, int64_t b) {
  if (SMALL || (a >= 0 && b > 0 && a < (1ll << 53) && b < (1ll << 53))) return div_f53(a, b);
  return a / b;
}

// leastRequestedScore / mostRequestedScore
template <bool SMALL = false>
__device__ __forceinline__ int64_t alloc_score(int strategy, int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (strategy == KSS_FIT_MOST_ALLOCATED) {
    if (requested > capacity) requested = capacity;
    return div_i64<SMALL>(requested * 100, capacity);
  }
  if (requested > capacity) return 0;
  return div_i64<SMALL>((capacity - requested) * 100, capacity);
}

// NodeResourcesFit.Score (resourceAllocationScorer.score, useRequested=false)
template <bool SMALL = false>
__device__ __forceinline__ int64_t fit_score(const DevCluster& c, const kss_profile& prof, const kss_pod& p, int n,
                                             const NodeRow& row) {
  const size_t N = (size_t)c.N;
  int64_t node_score = 0, weight_sum = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i >= prof.fit_n) break;
    const int r = prof.fit_res[i];
    const int64_t preq = p.score_req_nz[r];
    if (r >= KSS_RES_SCALAR0 && preq == 0) continue;
    const int64_t alloc = r < 3 ? pick3(row.alloc, r) : c.alloc[(size_t)r * N + n];
    const int64_t base = r == KSS_RES_CPU       ? row.nz[0]
                         : r == KSS_RES_MEMORY  ? row.nz[1]
                         : r == KSS_RES_EPHEMERAL ? row.req[2]
                                                  : c.requested[(size_t)r * N + n];
    if (alloc == 0) continue;
    node_score += alloc_score<SMALL>(prof.fit_strategy, base + preq, alloc) * prof.fit_weight[i];
    weight_sum += prof.fit_weight[i];
  }
  if (weight_sum == 0) return 0;
  return div_i64<SMALL>(node_score, weight_sum);
}

// NodeResourcesBalancedAllocation.Score (balancedResourceScorer, useRequested=true)
__device__ __forceinline__ int64_t ba_score(const DevCluster& c, const kss_profile& prof, const kss_pod& p, int n,
                                            const NodeRow& row) {
  const size_t N = (size_t)c.N;
  double fr[4] = {0.0, 0.0, 0.0, 0.0};
  bool use[4] = {false, false, false, false};
  int nf = 0;
  double total = 0.0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i >= prof.ba_n) break;
    const int r = prof.ba_res[i];
    const int64_t preq = p.score_req[r];
    if (r >= KSS_RES_SCALAR0 && preq == 0) continue;
    const int64_t alloc = r < 3 ? pick3(row.alloc, r) : c.alloc[(size_t)r * N + n];
    const int64_t req = (r < 3 ? pick3(row.req, r) : c.requested[(size_t)r * N + n]) + preq;
    if (alloc == 0) continue;
    double f = (double)req / (double)alloc;
    if (f > 1.0) f = 1.0;
    total += f;
    fr[i] = f;
    use[i] = true;
    nf++;
  }
  double sd = 0.0;
  if (nf == 2) {
    // the two used fractions, in resource order
    double a = 0.0, b = 0.0;
    bool got = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (!use[i]) continue;
      if (!got) {
        a = fr[i];
        got = true;
      } else {
        b = fr[i];
      }
    }
    sd = fabs((a - b) / 2.0);
  } else if (nf > 2) {
    const double mean = total / (double)nf;
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (!use[i]) continue;
      const double d = fr[i] - mean;
      const double sq = d * d;
      sum = sum + sq;
    }
    sd = sqrt(sum / (double)nf);
  }
  const double s = (1.0 - sd) * 100.0;
  return (int64_t)s;
}

// TaintToleration.Score: countIntolerableTaintsPreferNoSchedule
__device__ __forceinline__ int64_t tt_score(const NodeRow& row, const kss_pod& p) {
  return (int64_t)__popcll(row.ts & ~p.tol_soft);
}

// ImageLocality.Score (image_locality.go): calculatePriority(sumImageScores, len(Containers));
// the per-(image, node) scaledImageScore is host-resolved into c.image_score.
__host__ __device__ inline int64_t image_priority(int64_t sum, int n_containers) {
  const int64_t max_t = KSS_IMAGE_MAX_CONTAINER_THRESHOLD * (int64_t)n_containers;
  if (sum < KSS_IMAGE_MIN_THRESHOLD) sum = KSS_IMAGE_MIN_THRESHOLD;
  else if (sum > max_t) sum = max_t;
  return (int64_t)100 * (sum - KSS_IMAGE_MIN_THRESHOLD) / (max_t - KSS_IMAGE_MIN_THRESHOLD);
}

__device__ __forceinline__ int64_t il_score(const DevCluster& c, const DevPods& P, const kss_pod& p, int n) {
  if (p.img_len <= 0) return 0;
  int64_t sum = 0;
  for (int i = 0; i < p.img_len; i++) sum += c.image_score[(size_t)P.ints[p.img_off + i] * (size_t)c.N + (size_t)n];
  return image_priority(sum, p.n_containers);
}

__device__ __forceinline__ int64_t na_score(const DevCluster& c, const DevPods& P, const kss_pod& p, int n) {
  return na_score_t(c, P.reqs, P.terms, P.ints, p, (int64_t)c.node_base + n, [&](int key) { return label_of(c, key, n); });
}

}  // namespace kss
