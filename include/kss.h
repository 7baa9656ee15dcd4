/*
 * kss.h — C ABI of the MI355X-native Filter/Score evaluator (libkss.so).
 *
 * This is the drop-in boundary for the scheduling-cycle hot path of
 * kube-scheduler-simulator (reference snapshot 2025-01-31, upstream scheduler
 * k8s.io/kubernetes v1.26.2 pinned at simulator/go.mod:56).  It replaces, for
 * one pending pod or for a sequential batch of pods:
 *
 *   findNodesThatFitPod -> findNodesThatPassFilters  (HOT LOOP 1)
 *   prioritizeNodes -> RunPreScore/RunScore/Normalize (HOT LOOPS 2-4)
 *   selectHost                                         (mirror: scheduler/scheduler.go:323-344)
 *   Cache.AssumePod -> NodeInfo.AddPod                 (the commit the next pod sees)
 *
 * and the per-call result recording the simulator performs through
 *   wrappedPlugin.Filter/Score/NormalizeScore  simulator/scheduler/plugin/wrappedplugin.go:388-548
 *   resultstore.Store.Add* / GetStoredResult   simulator/scheduler/plugin/resultstore/store.go:133-626
 *
 * Conventions:
 *  - plain C, no exceptions cross the boundary; return 0 on success, <0 on error;
 *  - the library owns device buffers; callers own every host pointer passed in,
 *    and no caller pointer is retained after a call returns;
 *  - strings are interned by the caller (the Go plugin in a real integration,
 *    kss/compile.py here); only dense integer ids cross, except the optional
 *    name tables used to format annotations;
 *  - nodes are given in the scheduler's canonical order (nodeTree.list() zone
 *    round-robin); node index == canonical index.
 *
 * The same structs are consumed by the CPU oracle (oracle/kss_oracle.c), which is
 * test infrastructure only.
 */
#ifndef KSS_H_
#define KSS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSS_ABI_VERSION 5

/* ---- error codes ------------------------------------------------------- */
#define KSS_OK 0
#define KSS_E_INVAL (-22)        /* malformed input / shape mismatch           */
#define KSS_E_NOMEM (-12)        /* host or device allocation failed          */
#define KSS_E_DEVICE (-5)        /* HIP runtime error (maps to framework.Error) */
#define KSS_E_UNSUPPORTED (-95)  /* input outside what the device path supports */
#define KSS_E_RANGE (-34)        /* value outside the exact-arithmetic envelope */
#define KSS_E_NOTFOUND (-2)

/* ---- resources ----------------------------------------------------------
 * Resource vector layout (framework.Resource, ⟨k8s⟩ framework/types.go):
 * MilliCPU, Memory, EphemeralStorage, then up to 4 scalar (extended) resources. */
#define KSS_RES_CPU 0
#define KSS_RES_MEMORY 1
#define KSS_RES_EPHEMERAL 2
#define KSS_RES_SCALAR0 3
#define KSS_NRES 7
#define KSS_MAX_SCALAR 4

/* ---- filter plugins, in default MultiPoint order -------------------------
 * (simulator/scheduler/config/plugin_test.go:15-36).  A node's verdict is the
 * 1-based index of the FIRST failing filter (RunFilterPlugins stops at the first
 * non-success status), 0 when every filter passed. */
enum kss_filter_plugin {
  KSS_F_PASS = 0,
  KSS_F_NODE_UNSCHEDULABLE = 1,
  KSS_F_NODE_NAME = 2,
  KSS_F_TAINT_TOLERATION = 3,
  KSS_F_NODE_AFFINITY = 4,
  KSS_F_NODE_PORTS = 5,
  KSS_F_NODE_RESOURCES_FIT = 6,
  KSS_F_VOLUME_RESTRICTIONS = 7,
  KSS_F_EBS_LIMITS = 8,
  KSS_F_GCEPD_LIMITS = 9,
  KSS_F_NODE_VOLUME_LIMITS = 10,
  KSS_F_AZURE_DISK_LIMITS = 11,
  KSS_F_VOLUME_BINDING = 12,
  KSS_F_VOLUME_ZONE = 13,
  KSS_F_POD_TOPOLOGY_SPREAD = 14,
  KSS_F_INTER_POD_AFFINITY = 15,
  KSS_NFILTER = 15,
  KSS_F_NOT_EVALUATED = 255 /* node excluded by a PreFilterResult / PreFilter failure */
};

/* fail_detail of a node whose verdict is KSS_F_PASS: 0 = feasible (scored when >= 2 feasible
 * nodes); KSS_PASS_NOT_KEPT = the node that ended the search: with percentageOfNodesToScore
 * below 100, findNodesThatPassFilters stops once it finds one feasible node more than
 * numFeasibleNodesToFind; that node's filters ran and passed (filter-result records it) but it is
 * not in the feasible list (no Score / NormalizeScore entry).  Nodes after it in visiting order
 * were never filtered: KSS_F_NOT_EVALUATED. */
#define KSS_PASS_NOT_KEPT 1

/* fail_detail meaning per failing plugin */
#define KSS_FIT_TOO_MANY_PODS (1u << 0)
#define KSS_FIT_CPU (1u << 1)
#define KSS_FIT_MEMORY (1u << 2)
#define KSS_FIT_EPHEMERAL (1u << 3)
#define KSS_FIT_SCALAR0 (1u << 4) /* bit (4+s) for scalar s */
/* TaintToleration: detail = taint-dictionary id of the first untolerated taint */
#define KSS_PTS_CONSTRAINTS_NOT_MATCH 0
#define KSS_PTS_MISSING_LABEL 1
#define KSS_IPA_AFFINITY 0
#define KSS_IPA_ANTI_AFFINITY 1
#define KSS_IPA_EXISTING_ANTI_AFFINITY 2
/* VolumeRestrictions: "node(s) had no available disk"; EBSLimits / GCEPDLimits /
 * NodeVolumeLimits / AzureDiskLimits: "node(s) exceed max volume count" (detail 0) */
#define KSS_VB_NODE_CONFLICT 0 /* VolumeBinding: "node(s) had volume node affinity conflict" */
#define KSS_VB_PV_NOT_EXIST 1  /* "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)" */
#define KSS_VB_BIND_CONFLICT 2 /* "node(s) didn't find available persistent volumes to bind" */
#define KSS_VB_NODE_BIND 3     /* node conflict, then bind conflict (the reasons joined with ", ") */
#define KSS_VB_BIND_PV_NOT_EXIST 4 /* bind conflict, then PV not exist */
/* VolumeZone: detail 0 = "node(s) had no available volume zone", 1 + i = kss_names.messages[i] */

/* ---- score plugins, in default MultiPoint order ------------------------- */
enum kss_score_plugin {
  KSS_S_TAINT_TOLERATION = 0,
  KSS_S_NODE_AFFINITY = 1,
  KSS_S_NODE_RESOURCES_FIT = 2,
  KSS_S_VOLUME_BINDING = 3,
  KSS_S_POD_TOPOLOGY_SPREAD = 4,
  KSS_S_INTER_POD_AFFINITY = 5,
  KSS_S_BALANCED_ALLOCATION = 6,
  KSS_S_IMAGE_LOCALITY = 7,
  KSS_NSCORE = 8
};

/* ---- node flags --------------------------------------------------------- */
#define KSS_NODE_UNSCHEDULABLE (1u << 0) /* node.Spec.Unschedulable */
#define KSS_NODE_HAS_LABELS (1u << 1)    /* len(node.Labels) > 0 (IPA processExistingPod) */
#define KSS_NODE_VOLUME_ZONE (1u << 2)   /* the node carries a VolumeZone label (topology.kubernetes.io /
                                            failure-domain.beta.kubernetes.io zone or region) */

/* ---- label-key flags ---------------------------------------------------- */
#define KSS_KEY_UNIQUE (1u << 0)   /* no two nodes share a value: domain == node */
#define KSS_KEY_HOSTNAME (1u << 1) /* key == "kubernetes.io/hostname" (PTS scoring special case) */

/* Maximum taint dictionary size (uint64 masks) and hard taints per node kept in order. */
#define KSS_MAX_TAINTS 64
#define KSS_TAINT_ORDER 8
/* Maximum domain cardinality of a NON-unique topology key on the device path. */
#define KSS_MAX_BINS 1024
/* Host-port dictionary size (uint64 masks): distinct (hostIP, protocol, hostPort) entries of
 * the snapshot's NodeInfo.UsedPorts and the pending pods' container ports. */
#define KSS_MAX_PORTS 64
/* ImageLocality thresholds (image_locality.go: minThreshold 23 MiB, maxContainerThreshold 1000 MiB) */
#define KSS_IMAGE_MIN_THRESHOLD (23ll * 1024 * 1024)
#define KSS_IMAGE_MAX_CONTAINER_THRESHOLD (1000ll * 1024 * 1024)

/*
 * Cluster snapshot, struct-of-arrays, canonical node order.  All arrays are
 * caller-owned host memory; kss_load_cluster copies them to HBM.
 * Matrices are column-blocked [attribute][node] so that a wavefront reads 64
 * consecutive nodes of one attribute (coalesced).
 */
typedef struct kss_cluster {
  int32_t n_nodes;
  int32_t n_scalar;       /* scalar resource columns in use (0..KSS_MAX_SCALAR) */
  int32_t n_label_keys;   /* referenced label keys (columns of label_value)      */
  int32_t n_label_values; /* size of the value tables                            */
  int32_t n_classes;      /* existing-pod classes (namespace + labels)           */
  int32_t n_terms;        /* existing-pod affinity term types                    */
  int32_t n_taints;       /* taint dictionary size (<= KSS_MAX_TAINTS)            */
  int32_t node_base;      /* global index of row 0 (node-axis sharding); 0 otherwise */

  const int64_t* alloc;        /* [KSS_NRES][n_nodes] Allocatable            */
  const int64_t* requested;    /* [KSS_NRES][n_nodes] Requested              */
  const int64_t* nonzero;      /* [2][n_nodes] NonZeroRequested cpu, memory  */
  const int32_t* allowed_pods; /* [n_nodes] Allocatable.AllowedPodNumber     */
  const int32_t* pod_count;    /* [n_nodes] len(NodeInfo.Pods)               */
  const uint32_t* node_flags;  /* [n_nodes] KSS_NODE_*                       */
  const uint64_t* taint_hard;  /* [n_nodes] dict bits of NoSchedule/NoExecute taints */
  const uint64_t* taint_soft;  /* [n_nodes] dict bits of PreferNoSchedule taints     */
  const uint8_t* taint_order;  /* [n_nodes][KSS_TAINT_ORDER] hard-taint dict ids in node.Spec.Taints order, 0xFF pad */
  const int32_t* label_value;  /* [n_label_keys][n_nodes] key-local value id, -1 = label absent */
  const int32_t* key_base;     /* [n_label_keys] offset of the key's values in the value tables */
  const int32_t* key_card;     /* [n_label_keys] number of distinct values of the key */
  const uint32_t* key_flags;   /* [n_label_keys] KSS_KEY_* */
  const int32_t* key_empty;    /* [n_label_keys] local id of the "" value, or key_card (virtual "missing" domain) */
  const int64_t* value_int;    /* [n_label_values] strconv.ParseInt(value,10,64) */
  const uint8_t* value_is_int; /* [n_label_values] 1 if ParseInt succeeded */
  const int32_t* class_count;  /* [n_classes][n_nodes] #pods of class c on node n */
  const int32_t* term_count;   /* [n_terms][n_nodes]   #occurrences of term type t among pods on node n */
  /* NodePorts: NodeInfo.UsedPorts as bits over the port dictionary (framework.HostPortInfo;
   * hostIP "" -> 0.0.0.0, protocol "" -> TCP).  NULL or n_ports == 0: no host port in use. */
  int32_t n_ports;
  /* ImageLocality: rows of image_score, one per image name a pending pod's container
   * references (normalizedImageName) that some node lists in Status.Images. */
  int32_t n_images;
  const uint64_t* port_used;   /* [n_nodes] */
  const int64_t* image_score;  /* [n_images][n_nodes] scaledImageScore(NodeInfo.ImageStates[name], totalNumNodes),
                                  0 where the node does not list the image */
  /* Volumes (VolumeRestrictions, the attach-limit plugins, VolumeBinding, VolumeZone).
   * A volume row is a volume (by the limit plugins' unique name) or a disk usage (kind,
   * identity, readOnly: VolumeRestrictions) that some pending pod's filter needs to find on a
   * node: vol_count = how many of the node's pods use it.  A key is an attach-limit resource
   * (attachable-volumes-aws-ebs / -gce-pd / -azure-disk, or a CSI driver's
   * attachable-volumes-csi-<driver>) of one limit plugin: vol_attached = the distinct
   * volumes of that key the node's pods use, vol_limit = the node's limit (-1: the plugin
   * does not check the key on this node).  n_vol_rows == n_vol_keys == 0: no volumes. */
  int32_t n_vol_rows;
  int32_t n_vol_keys;
  const int32_t* vol_count;      /* [n_vol_rows][n_nodes] (mutable: AssumePod adds) */
  const int32_t* vol_attached;   /* [n_vol_keys][n_nodes] (mutable) */
  const int32_t* vol_limit;      /* [n_vol_keys][n_nodes] */
  const int32_t* vol_row_key;    /* [n_vol_rows] key the row's volume counts under, -1 (disk usage rows) */
  const int32_t* vol_key_plugin; /* [n_vol_keys] KSS_F_EBS_LIMITS / _GCEPD_ / _NODE_VOLUME_ / _AZURE_DISK_LIMITS */
  /* VolumeBinding for unbound WaitForFirstConsumer claims (binder.go FindPodVolumes): the
   * binder's assume cache as two mutable columns.  A candidate PV is one some pending pod's
   * delayed claim may bind (KSS_VOL_BIND_WFFC lists); a delayed claim is an unbound claim of a
   * WaitForFirstConsumer class some pending pod uses.
   *   pv_owner[v]   0: available; c + 1: bound to delayed claim c (spec.claimRef in the
   *                 snapshot, or AssumePodVolumes' static binding)
   *   claim_node[c] the claim's volume.kubernetes.io/selected-node: -1 none, -2 a node outside
   *                 the snapshot, else the node's canonical index (AssumePodVolumes' provisioning) */
  int32_t n_pvs;
  int32_t n_wclaims;
  const int32_t* pv_owner;   /* [n_pvs] (mutable) */
  const int32_t* claim_node; /* [n_wclaims] (mutable) */
} kss_cluster;

/* ---- pod programs --------------------------------------------------------
 * The host compiles each pod (v1.Pod) once into a fixed record plus entries in
 * shared pools.  All label matching is reduced to predicates over value ids. */

/* label requirement ops (labels.Requirement.Matches / NodeSelectorRequirement) */
enum kss_req_op {
  KSS_OP_FALSE = 0,  /* never matches (e.g. parse error)                      */
  KSS_OP_TRUE = 1,
  KSS_OP_MASK = 2,   /* low-cardinality key: match iff bit(value id) of mask; bit 63 = absent matches */
  KSS_OP_IN = 3,     /* value id in list (absent -> false)                    */
  KSS_OP_NOTIN = 4,  /* value id not in list (absent -> true)                 */
  KSS_OP_EXISTS = 5,
  KSS_OP_DNE = 6,
  KSS_OP_GT = 7,     /* ParseInt(value) >  ival (absent or non-int -> false)  */
  KSS_OP_LT = 8,     /* ParseInt(value) <  ival                               */
  KSS_OP_NAME_IN = 9,    /* matchFields metadata.name In  [value]: node index == ival */
  KSS_OP_NAME_NOTIN = 10 /* matchFields metadata.name NotIn [value]             */
};

typedef struct kss_req {
  int32_t key;      /* label key column (unused for NAME ops / TRUE / FALSE) */
  int32_t op;       /* enum kss_req_op */
  int32_t list_off; /* IN/NOTIN: offset into kss_podset.ints */
  int32_t list_len;
  uint64_t mask;    /* OP_MASK */
  int64_t ival;     /* GT/LT threshold; NAME ops: global node index (-1 = no such node) */
} kss_req;

/* a node-selector term: AND of requirements [req_off, req_off+req_len) */
typedef struct kss_term {
  int32_t req_off;
  int32_t req_len;
  int32_t weight; /* preferred terms: weight; required terms: unused */
  int32_t flags;  /* reserved */
} kss_term;

/* topology spread constraint (after filterTopologySpreadConstraints/buildDefaultConstraints) */
#define KSS_SPREAD_POLICY_AFFINITY_HONOR (1u << 0) /* NodeAffinityPolicy == Honor (default) */
#define KSS_SPREAD_POLICY_TAINTS_HONOR (1u << 1)   /* NodeTaintsPolicy   == Honor (default Ignore) */
typedef struct kss_spread {
  int32_t key;        /* topology key column */
  int32_t max_skew;
  int32_t self_match; /* selector matches the incoming pod's own labels (filter) */
  int32_t flags;      /* KSS_SPREAD_* */
  int32_t cls_off;    /* classes (in the pod's namespace) matching the selector: ints[cls_off..] */
  int32_t cls_len;
  int32_t min_domains; /* 1 unless MinDomainsInPodTopologySpread (off in v1.26) */
  int32_t pad;
} kss_spread;

/* inter-pod affinity program entries */
enum kss_ipa_kind {
  KSS_IPA_EXISTING_ANTI = 0, /* existing pods' required anti-affinity terms matching the incoming pod (rows: term types) */
  KSS_IPA_REQ_AFFINITY = 1,  /* one per incoming required affinity term; rows: classes matching ALL terms */
  KSS_IPA_REQ_ANTI = 2,      /* one per incoming required anti-affinity term; rows: classes matching it */
  KSS_IPA_SCORE_CLASS = 3,   /* incoming preferred (anti-)affinity term: coef = +/-weight; rows: classes */
  KSS_IPA_SCORE_TERM = 4     /* existing pods' terms matched by the incoming pod: coef; rows: term types */
};
typedef struct kss_ipa {
  int32_t kind;
  int32_t key;     /* topology key column */
  int32_t row_off; /* ints[row_off .. row_off+row_len) */
  int32_t row_len;
  int32_t coef;    /* score entries: weight*multiplier */
  int32_t pad;
} kss_ipa;

/* volume program entries, in filter order (kss_pod.vol_off / vol_len): VolumeRestrictions,
 * then the limit plugins (grouped by key, keys in plugin order), VolumeBinding, VolumeZone, and
 * last the AssumePod entries */
enum kss_vol_kind {
  KSS_VOL_CONFLICT = 0,       /* VolumeRestrictions fails where vol_count[row][n] > 0 (isVolumeConflict) */
  KSS_VOL_LIMIT = 1,          /* a new volume under `key`: row >= 0 a shared volume, new where vol_count[row][n] == 0;
                                 row < 0: `count` volumes no other pod uses.  Per key: fail where vol_limit >= 0 and
                                 vol_attached + new > vol_limit (NodeVolumeLimits: only when new > 0) */
  KSS_VOL_BIND_AFFINITY = 2,  /* VolumeBinding bound claim: its PV's required node affinity, terms [a, a + b) (OR) */
  KSS_VOL_BIND_PV_MISSING = 3,/* VolumeBinding bound claim whose PV does not exist */
  KSS_VOL_ZONE = 4,           /* VolumeZone on zone-labelled nodes: requirements [a, a + b) (AND) */
  KSS_VOL_ZONE_ERROR = 5,     /* VolumeZone on zone-labelled nodes: the status message kss_names.messages[a] */
  KSS_VOL_OWN = 6,            /* AssumePod: vol_count[row][n] += 1 (0 -> 1 also adds 1 to the row's key) */
  KSS_VOL_OWN_PRIVATE = 7,    /* AssumePod: vol_attached[key][n] += count */
  KSS_VOL_BIND_WFFC = 8       /* VolumeBinding delayed claim `key` (an unbound WaitForFirstConsumer claim), after the
                                 pod's BIND_AFFINITY / BIND_PV_MISSING entries, in increasing storage request (stable):
                                 candidate PVs ints[a .. a + 3b) as {pv, term_off, term_len} triplets in increasing
                                 capacity, then name (term_len -1: no required node affinity; else its terms, OR, over
                                 the node's labels); count bit 0: its class can provision (a provisioner other than
                                 kubernetes.io/no-provisioner), count >> 1: the class's allowedTopologies as terms
                                 [row, row + (count >> 1)) (0: any node).  FindMatchingVolume: a PV with pv_owner ==
                                 key + 1 is the claim's (its node affinity decides), else the first available one not
                                 chosen by an earlier claim whose affinity matches; a claim with a selected node, or
                                 without a match, is provisioned (checkVolumeProvisions).  AssumePod (Reserve's
                                 AssumePodVolumes) sets pv_owner / claim_node on the chosen node. */
};
#define KSS_MAX_WFFC 4 /* delayed claims per pod */
typedef struct kss_vol {
  int32_t kind;
  int32_t key;
  int32_t row;
  int32_t count;
  int32_t a;
  int32_t b;
} kss_vol;
#define KSS_MAX_VOL_KEYS 64

/* kss_pod.prefilter_status */
#define KSS_PF_OK 0
#define KSS_PF_NODE_AFFINITY_CONFLICT 1 /* NodeAffinity PreFilter: "pod affinity terms conflict" */
#define KSS_PF_ERROR 2                  /* a PreFilter Error (pod-level) */
#define KSS_PF_VOLUME_BINDING 3         /* VolumeBinding PreFilter UnschedulableAndUnresolvable:
                                           kss_names.messages[prefilter_msg] */

/* pod flags */
#define KSS_POD_TOL_UNSCHEDULABLE (1u << 0)  /* tolerates node.kubernetes.io/unschedulable:NoSchedule */
#define KSS_POD_HAS_REQ_AFFINITY (1u << 1)   /* RequiredDuringScheduling node affinity present */
#define KSS_POD_PTS_REQUIRE_ALL (1u << 2)    /* PTS scoring requireAllTopologies */
#define KSS_POD_IPA_SELF_MATCH (1u << 3)     /* podMatchesAllAffinityTerms(required, pod) */
#define KSS_POD_IPA_HAS_PREFERRED (1u << 4)  /* incoming pod has preferred (anti-)affinity terms */
#define KSS_POD_PTS_SCORE_STATE (1u << 5)    /* PTS preScoreState written (always, unless error) */
#define KSS_POD_PREEMPT_NEVER (1u << 6)      /* spec.preemptionPolicy == Never (PodEligibleToPreemptOthers) */

typedef struct kss_pod {
  int64_t fit_request[KSS_NRES];   /* Fit PreFilter computePodResourceRequest                 */
  int64_t score_req_nz[KSS_NRES];  /* LeastAllocated: calculatePodResourceRequest(nonZero)    */
  int64_t score_req[KSS_NRES];     /* BalancedAllocation: calculatePodResourceRequest(useRequested) */
  int64_t commit_req[KSS_NRES];    /* NodeInfo.AddPod Requested delta (calculateResource)     */
  int64_t commit_nz[2];            /* NodeInfo.AddPod NonZeroRequested delta                  */
  uint64_t tol_hard;               /* dict bits of NoSchedule/NoExecute taints tolerated      */
  uint64_t tol_soft;               /* dict bits of PreferNoSchedule taints tolerated by
                                      tolerations with effect "" or PreferNoSchedule          */
  int32_t node_name;               /* spec.nodeName: -1 unset, -2 names no node, else global index */
  uint32_t flags;                  /* KSS_POD_* */
  int32_t sel_off, sel_len;        /* nodeSelector requirements (AND), pool reqs          */
  int32_t aff_off, aff_len;        /* required NodeSelectorTerms (OR), pool terms         */
  int32_t pref_off, pref_len;      /* PreferredSchedulingTerms, pool terms                */
  int32_t spread_off;              /* pool spreads: n_hard DoNotSchedule then n_soft ScheduleAnyway */
  int32_t n_hard, n_soft;
  int32_t ipa_off, ipa_len;        /* pool ipa entries */
  int32_t cls;                     /* the pod's own class (class_count row it joins on commit), -1 none */
  int32_t own_terms_off, own_terms_len; /* term-type rows this pod adds on commit: ints[] */
  int32_t prefilter_status;        /* KSS_PF_* */
  int32_t names_off, names_len;    /* NodeAffinity PreFilterResult node set (ints[], global idx); len<0: all nodes */
  int32_t priority;                /* corev1helpers.PodPriority: spec.priority, 0 when unset (DefaultPreemption) */
  int32_t prefilter_msg;           /* KSS_PF_VOLUME_BINDING: index into kss_names.messages */
  /* NodePorts (nodeports.go): port_conflict = dictionary entries any wanted container host
   * port conflicts with (HostPortInfo.CheckConflict: same protocol and port, and either IP is
   * 0.0.0.0 or both are equal); port_add = the pod's own entries (NodeInfo.AddPod
   * updateUsedPorts).  Both 0 for pods without host ports. */
  uint64_t port_conflict;
  uint64_t port_add;
  /* ImageLocality (image_locality.go): image_score rows of the pod's containers, one entry per
   * container whose normalized image some node lists (ints[img_off .. +img_len)); n_containers =
   * len(pod.Spec.Containers) for calculatePriority's maxThreshold. */
  int32_t img_off, img_len;
  int32_t n_containers;
  int32_t vol_off, vol_len;        /* volume program: pool vols (kss_vol), 0 entries for volume-less pods */
  int32_t uid;                     /* the pod's identity for the nominator (kss_nominate): > 0 a stable caller id
                                      (the Go plugin interns metadata.uid); 0: its index in the podset stands for it */
} kss_pod;

typedef struct kss_podset {
  int32_t n_pods;
  int32_t n_reqs, n_terms, n_spreads, n_ipa, n_ints;
  const kss_pod* pods;
  const kss_req* reqs;
  const kss_term* terms;
  const kss_spread* spreads;
  const kss_ipa* ipa;
  const int32_t* ints;
  int32_t n_vols;
  int32_t pad;
  const kss_vol* vols;
} kss_podset;

/* ---- profile (KubeSchedulerConfiguration profile subset) --------------- */
#define KSS_FIT_LEAST_ALLOCATED 0
#define KSS_FIT_MOST_ALLOCATED 1
typedef struct kss_profile {
  int32_t weight[KSS_NSCORE]; /* score plugin weights as getScorePluginWeight builds them (0 -> 1) */
  uint32_t filter_enabled;    /* bit i = filter plugin i enabled (bit 0 unused) */
  uint32_t score_enabled;     /* bit s = score plugin s enabled */
  int32_t fit_strategy;       /* KSS_FIT_* (NodeResourcesFitArgs.ScoringStrategy.Type) */
  int32_t fit_n;              /* scoring resources */
  int32_t fit_res[4];
  int64_t fit_weight[4];
  int32_t ba_n;               /* NodeResourcesBalancedAllocationArgs.Resources */
  int32_t ba_res[4];
  int32_t hard_pod_affinity_weight; /* InterPodAffinityArgs.HardPodAffinityWeight */
  int32_t pct_nodes_to_score;       /* KubeSchedulerConfiguration.percentageOfNodesToScore, 0..100 (0 = the
                                       adaptive default of v1.26, which the simulator's built-in scheduler
                                       uses: simulator/scheduler/scheduler.go:162,258-275).  100 evaluates
                                       every node (north_star / bench configuration); below 100 the
                                       findNodesThatPassFilters window applies (numFeasibleNodesToFind from
                                       nextStartNodeIndex, Parallelism = 1 order) and batches run on
                                       k_schedule.  SURVEY §8a a1. */
  int32_t system_defaulted;         /* PodTopologySpreadArgs.DefaultingType == System */
  int32_t pad;
} kss_profile;

/* the default v1.26 profile as the simulator builds it (plugins_test.go:184-209,878-1096) */
void kss_default_profile(kss_profile* out);

/* ---- per-pod results ------------------------------------------------------
 * Caller-allocated host arrays of length n_nodes (any may be NULL to skip). */
typedef struct kss_pod_result {
  uint8_t* fail_plugin;  /* [n] enum kss_filter_plugin                          */
  uint16_t* fail_detail; /* [n]                                                 */
  int64_t* raw;          /* [KSS_NSCORE][n] Score() results (feasible nodes)    */
  int64_t* norm;         /* [KSS_NSCORE][n] after NormalizeScore (pre-weight)   */
  int64_t* total;        /* [n] Σ weight·norm                                   */
  int32_t n_feasible;
  int32_t chosen;        /* global node index, -1 if unschedulable */
  int64_t best_total;
  int32_t scored;        /* 1 if prioritizeNodes ran (>= 2 feasible nodes) */
  int32_t status;        /* 0 ok; 1 unschedulable (no feasible); 2 prefilter unschedulable; 3 error */
} kss_pod_result;

/* ---- context -------------------------------------------------------------- */
typedef struct kss_ctx kss_ctx;

typedef struct kss_config {
  int32_t device;          /* HIP device ordinal */
  int32_t max_pods_record; /* capacity of the on-device per-pod result record (0 = no recording) */
  int32_t class_capacity;  /* rows reserved in class_count (>= n_classes; commits may add rows) */
  int32_t term_capacity;   /* rows reserved in term_count */
} kss_config;

int kss_abi_version(void);
const char* kss_last_error(void); /* thread-local message of the last failing call */

/* Tuning and diagnosis options, process-wide (no reference counterpart: the reference reads no
 * such knobs).  The library reads no environment variable: a plugin host's environment changes
 * nothing, and every option keeps its default until set here.  Names: "shards" (shards per
 * cluster, 0 automatic), "xcd" (1: XCD-local grids where the shards fit one XCD), "xcd_shards",
 * "no_simple", "no_spread", "threads", "force_threads", "nodes_per_shard", "static_bytes" (k_static
 * budget; 0: an eighth of free memory), "static_ppb", "fold" (k_spread statistics fold), "no_cache",
 * "coop_launch", "service_general", "service_stamps", "svc_xcd", "svc_no_static", "svc_full_fence",
 * "svc_inline_sweep", "svc_huge", "service_no_diff", "sweep_pipe", "axis_blocks", "axis_no_fold",
 * "trace_path", "xcd_force_fallback" (XCD-local launches report failed placement, so the
 * unrestricted rerun runs: tests).  Read when a context is created (shards, xcd, xcd_shards,
 * no_simple, no_spread, threads, nodes_per_shard, axis_*) or at each launch (the rest).
 * KSS_E_NOTFOUND for an unknown name.  kss_set_stamps_file: per-phase timestamps of every launch
 * of contexts created afterwards are appended to `path` (NULL: off). */
int kss_set_option(const char* name, int64_t value);
int kss_get_option(const char* name, int64_t* value);
int kss_reset_options(void);
int kss_set_stamps_file(const char* path);

kss_ctx* kss_create(const kss_config* cfg, const kss_profile* prof);
void kss_destroy(kss_ctx* ctx);

/* upload a snapshot (replaces any previous one) */
int kss_load_cluster(kss_ctx* ctx, const kss_cluster* cl);
/* NodeInfo-generation delta sync: overwrite rows idx[0..n) of the mutable columns (one
 * packed upload) */
int kss_apply_node_delta(kss_ctx* ctx, const int32_t* idx, int32_t n, const int64_t* requested /*[n][KSS_NRES]*/,
                         const int64_t* nonzero /*[n][2]*/, const int32_t* pod_count /*[n]*/);
/* The class / term count side of the same sync (a pod bound or deleted outside this
 * scheduler, a re-listed node): count[row[i]][node[i]] += value[i] (mode 0) or = value[i]
 * (mode 1).  row r < n_classes is class_count row r, otherwise term_count row r - n_classes.
 * Replaces: the informer's NodeInfo.AddPod / RemovePod on the scheduler cache
 * (simulator/scheduler/scheduler.go:66-104 starts the scheduler that keeps it). */
int kss_apply_count_delta(kss_ctx* ctx, const int32_t* node, const int32_t* row, const int32_t* value, int32_t n,
                          int32_t mode);
/* Volume state (vol_count rows, then vol_attached keys as rows n_vol_rows + k): read back, or
 * the delta sync of pods with volumes bound or deleted outside this context:
 * row[i] < n_vol_rows: vol_count[row][node] += value (mode 0) or = value (mode 1); otherwise
 * vol_attached[row - n_vol_rows][node].  Replaces the informer's NodeInfo.AddPod / RemovePod
 * (the volume plugins re-read NodeInfo.Pods' volumes on every Filter call). */
int kss_read_volume_state(kss_ctx* ctx, int32_t* vol_count /*[n_vol_rows][N] or NULL*/,
                          int32_t* vol_attached /*[n_vol_keys][N] or NULL*/);
int kss_apply_volume_delta(kss_ctx* ctx, const int32_t* node, const int32_t* row, const int32_t* value, int32_t n,
                           int32_t mode);
/* The binder's assume cache (kss_cluster pv_owner / claim_node) read back: what AssumePodVolumes
 * (batch commits, kss_commit) and RevertAssumedPodVolumes (kss_rollback) left.  Replaces the
 * volumebinding plugin's pvCache / pvcCache (binder.go AssumePodVolumes, simulator
 * scheduler's default VolumeBinding, plugin_test.go:28). */
int kss_read_binding_state(kss_ctx* ctx, int32_t* pv_owner /*[n_pvs] or NULL*/, int32_t* claim_node /*[n_wclaims] or NULL*/);
/* read back the mutable columns (requested [KSS_NRES][N], nonzero [2][N], pod_count [N]) */
int kss_read_node_state(kss_ctx* ctx, int64_t* requested, int64_t* nonzero, int32_t* pod_count,
                        int32_t* class_count /*[n_classes][N] or NULL*/, int32_t* term_count /*or NULL*/);
/* NodeInfo.UsedPorts of every row (port dictionary bits, [N]): read back, or overwrite rows
 * idx[0..n) (pods with host ports bound or deleted outside this context).  Replaces the
 * informer's NodeInfo.AddPod / RemovePod updateUsedPorts on the scheduler cache. */
int kss_read_port_state(kss_ctx* ctx, uint64_t* port_used);
int kss_apply_port_delta(kss_ctx* ctx, const int32_t* idx, int32_t n, const uint64_t* port_used);

/* evaluate one pod against the current snapshot (no commit): the PreFilter-time call.  Only
 * the pod's own program is uploaded; the record comes back in one copy. */
int kss_eval_pod(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, kss_pod_result* out);
/* The same evaluation without the copy into caller arrays: `out` points into the context's
 * pinned read-back staging, which the one device->host copy fills directly.  `fields`
 * (KSS_FIELD_*) selects the arrays read back; the others are NULL.  The pointers stay valid
 * until the next call on ctx that runs device work.  Saves the host copy of the per-node
 * arrays (~0.7 MB for the full record at 5k nodes): the plugin reads them in place during
 * the pod's scheduling cycle. */
#define KSS_FIELD_FAIL (1u << 0)
#define KSS_FIELD_DETAIL (1u << 1)
#define KSS_FIELD_RAW (1u << 2)
#define KSS_FIELD_NORM (1u << 3)
#define KSS_FIELD_TOTAL (1u << 4)
#define KSS_FIELD_ALL 0x1Fu
typedef struct kss_pod_view {
  const uint8_t* fail_plugin;  /* [n] */
  const uint16_t* fail_detail; /* [n] */
  const int64_t* raw;          /* [KSS_NSCORE][n] */
  const int64_t* norm;         /* [KSS_NSCORE][n] */
  const int64_t* total;        /* [n] */
  int32_t n_feasible;
  int32_t chosen;
  int64_t best_total;
  int32_t scored;
  int32_t status;
} kss_pod_view;
int kss_eval_pod_view(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, uint32_t fields, kss_pod_view* out);
/* The per-pod path as a persistent service grid: the shape wrappedPlugin.PreFilter ->
 * evaluate, Reserve -> AssumePod, Unreserve -> ForgetPod drives
 * (simulator/scheduler/plugin/wrappedplugin.go:491-518, 616-645) without a kernel launch, an
 * upload or a stream synchronisation per call.  One grid stays resident on the context's
 * device and takes commands from a ring in pinned host memory; the pods are the staged ones
 * (kss_stage_pods: their programs already in HBM), named by index.
 *   kss_service_eval    evaluates pod_index on the current state (filters, raw and normalised
 *                       scores, totals, the selectHost choice): the record fields asked for
 *                       land in a pinned host buffer and `out` points into it (valid until the
 *                       next service call); returns when the record is complete
 *   kss_service_commit  AssumePod of pod_index on node (queued: returns at once; the next
 *                       evaluation sees it), kss_service_rollback its ForgetPod
 *   kss_service_start / kss_service_stop  explicit start (the first eval / commit starts the
 *                       grid too) and stop.  The grid leaves by itself after ~1 s without a
 *                       command and is restarted by the next call.  Every other entry point
 *                       that touches the context's device state stops it first.
 * Results equal kss_eval_pod_view / kss_commit / kss_rollback on the same state.
 * The resident grid runs on a stream with a hardware queue of its own (a CU-masked stream: the
 * runtime's GPU_MAX_HW_QUEUES shared queues are not used), so no other context's or stream's
 * work waits behind it; the grid's workgroups still occupy CUs until it leaves. */
int kss_service_start(kss_ctx* ctx);
int kss_service_stop(kss_ctx* ctx);
int kss_service_eval(kss_ctx* ctx, int32_t pod_index, uint32_t fields, kss_pod_view* out);
/* kss_service_eval with the score rows narrowed on the device before they cross the host link
 * (47 instead of 139 bytes per node): raw and total as int32, normalised scores (0..100) as
 * uint8.  When some value of the pod does not fit (is_wide = 1) the pod is evaluated again
 * into the full record and `wide` holds the kss_service_eval view instead (the narrow
 * pointers are NULL).  Same validity as kss_service_eval. */
typedef struct kss_pod_cview {
  const uint8_t* fail_plugin;  /* [n] */
  const uint16_t* fail_detail; /* [n] */
  const int32_t* raw;          /* [KSS_NSCORE][n] */
  const uint8_t* norm;         /* [KSS_NSCORE][n] */
  const int32_t* total;        /* [n] */
  int32_t n_feasible;
  int32_t chosen;
  int64_t best_total;
  int32_t scored;
  int32_t status;
  int32_t is_wide;
  int32_t pad;
  kss_pod_view wide;
} kss_pod_cview;
int kss_service_eval_compact(kss_ctx* ctx, int32_t pod_index, uint32_t fields, kss_pod_cview* out);
int kss_service_commit(kss_ctx* ctx, int32_t pod_index, int32_t node);
int kss_service_rollback(kss_ctx* ctx, int32_t pod_index, int32_t node);
/* Diagnostics (KSS_SERVICE_STAMPS set when the grid starts): shard 0's s_memrealtime (100 MHz)
 * in the last evaluation when it took the command, relayed it, finished the pod, had its
 * record visible to the host, and had issued its record stores (before the system fence);
 * the k_simple-shaped evaluation adds its node pass done, its statistics exchange done and its
 * record stores issued before the key exchange (out8[5..7], 0 otherwise). */
int kss_service_stamps(kss_ctx* ctx, uint64_t* out8);
/* Which evaluation the service grid runs (set when it starts): 1 the k_simple-shaped chain
 * (staged default-profile pods: no spread / inter-pod programs, host ports, node-cached images,
 * volumes or extended resources; below percentageOfNodesToScore 100 no PreFilterResult node
 * lists, the window running on the same chain) with the record stored from
 * registers, 2 the same on an XCD-local grid (its exchanges in one XCD's L2), 0 the general
 * chain (schedule_pod + the record copy), -1 not started. */
int kss_service_mode(kss_ctx* ctx, int32_t* mode);
/* commit pod ps.pods[pod_index] to node (AssumePod); rollback undoes it (Unreserve/ForgetPod).
 * The deltas travel in the kernel's arguments (no upload). */
int kss_commit(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node);
int kss_rollback(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node);

/* sequential scheduling of ps.pods[0..n) entirely on the device: each pod sees the
 * previous pods' commits.  chosen_out[i] = global node index or -1.  When
 * record != 0 (and max_pods_record >= n) per-pod results stay in HBM for
 * kss_fetch_record / kss_format_annotations. */
#define KSS_SCHED_RECORD (1u << 0)
#define KSS_SCHED_FORCE_MULTI_WG (1u << 1) /* testing: use the multi-workgroup per-pod path */
#define KSS_SCHED_FORCE_SINGLE_WG (1u << 2)
#define KSS_SCHED_GENERAL_KERNEL (1u << 3) /* testing: never use the compact k_simple path */
int kss_schedule_batch(kss_ctx* ctx, const kss_podset* ps, int32_t n, uint32_t flags, int32_t* chosen_out);
int kss_fetch_record(kss_ctx* ctx, int32_t pod_index, kss_pod_result* out);

/* Resident-input variant of kss_schedule_batch: kss_stage_pods validates and copies
 * the pod programs to HBM once; kss_run_staged schedules the first n staged pods
 * (no host->device traffic).  kss_reset_node_state restores every mutable column
 * (requested, nonzero, pod counts, class/term counts) to the snapshot given to
 * kss_load_cluster, on the device (what-if replays, simulator/reset). */
int kss_stage_pods(kss_ctx* ctx, const kss_podset* ps);
int kss_run_staged(kss_ctx* ctx, int32_t n, uint32_t flags, int32_t* chosen_out);
int kss_reset_node_state(kss_ctx* ctx);
/* The scheduler's nextStartNodeIndex (schedule_one.go findNodesThatPassFilters): where the next
 * pod's node search starts, advanced by every evaluated scheduling cycle (kss_eval_pod, batches,
 * the service) by the nodes it processed, modulo the pod's node list.  0 after kss_load_cluster and
 * kss_reset_node_state.  Only percentageOfNodesToScore < 100 reads it.  Replaces the field of
 * pkg/scheduler.Scheduler that simulator/scheduler/scheduler.go:155-168 creates. */
int kss_next_start_node_index(kss_ctx* ctx, int32_t* out);
int kss_set_next_start_node_index(kss_ctx* ctx, int32_t value);

/* The scheduling queue's nominator (PodNominator), the nominations a PostFilter leaves behind:
 * the simulator's scheduler records them when DefaultPreemption nominates a node
 * (simulator/scheduler/plugin/wrappedplugin.go:550-577 returns the PostFilterResult whose
 * NominatedNodeName the scheduler's handleSchedulingFailure stores).
 *   kss_nominate          AddNominatedPod: ps.pods[pod_index] is nominated to global node `node`
 *                         (an earlier nomination of the same pod is replaced).  The pod's identity
 *                         is kss_pod.uid when > 0, otherwise its index in the podset the caller
 *                         schedules from (the staged one for batches, the one passed to
 *                         kss_eval_pod).  At most 64 entries; pods with volumes are refused.
 *   kss_clear_nomination  DeleteNominatedPodIfExists (a PostFilter that found no candidate, a
 *                         lower-priority nomination cleared by prepareCandidate); no-op if absent
 *   kss_nominations       the entries in AddNominatedPod order (*n = count; cap entries copied)
 * Every scheduling cycle (kss_eval_pod, batches, kss_postfilter_pod's dry run) then filters with
 * RunFilterPluginsWithNominatedPods: on a node holding nominees of priority >= the pod's (other
 * than the pod itself) the filters run first with them added (their requests, pod count, host
 * ports, and their labels / required anti-affinity terms in the PodTopologySpread and
 * InterPodAffinity counts of the node's pairs); a failure there is the node's status, otherwise
 * the plain pass decides.  A nominated pod first evaluates its own node (PreferNominatedNode:
 * chosen without scoring when it passes; nextStartNodeIndex restarts at 0).  An assumed pod leaves
 * the nominator (kss_commit, batch commits).  kss_load_cluster / kss_reset_node_state empty it.
 * While it is non-empty batches run on k_schedule and the service grid, node axis and split
 * grids refuse (KSS_E_UNSUPPORTED).  Replaces the nominator of the scheduler that
 * simulator/scheduler/scheduler.go:155-168 creates (pkg/scheduler/internal/queue, v1.26). */
int kss_nominate(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node);
int kss_clear_nomination(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index);
/* ids: the pods' identities (kss_pod.uid when > 0, else -1 - podset index) */
int kss_nominations(kss_ctx* ctx, int32_t* ids, int32_t* nodes, int32_t cap, int32_t* n);

/* many independent clusters (what-if scenarios, KEP-184): clusters[s] with podsets[s];
 * one workgroup per scenario, no inter-scenario communication. chosen_out is [sum n_pods].
 * One-shot form of kss_sweep_create + kss_sweep_run + kss_sweep_destroy. */
int kss_schedule_scenarios(int32_t device, const kss_profile* prof, int32_t n_scen, const kss_cluster* clusters,
                           const kss_podset* podsets, int32_t* chosen_out, double* device_ms);

/* Resident what-if sweep.  kss_sweep_create validates and packs every scenario's
 * snapshot and pod programs into one host image and uploads it with one copy (NULL on
 * error: kss_last_error).  kss_sweep_run restores every scenario's node state to its
 * snapshot on the device and schedules all of them (chosen_out [sum n_pods]; device_ms =
 * reset + launches, HIP events).  Replaces, per scenario, the sequential scheduleOne
 * loop of the simulator's scheduler; the scenario axis of SURVEY 8(e).
 * kss_sweep_info: host wall time of create (pack + upload), the kernel used (1 k_simple,
 * 0 k_schedule) and the uploaded bytes. */
typedef struct kss_sweep kss_sweep;
kss_sweep* kss_sweep_create(int32_t device, const kss_profile* prof, int32_t n_scen, const kss_cluster* clusters,
                            const kss_podset* podsets);
int kss_sweep_run(kss_sweep* sw, int32_t* chosen_out, double* device_ms);
int kss_sweep_info(kss_sweep* sw, double* stage_ms, int32_t* kernel, int64_t* upload_bytes);
void kss_sweep_destroy(kss_sweep* sw);

/* ---- node-axis sharding ----------------------------
 * One context per GPU holds rows [lo, hi) of the cluster (node_base = lo); the pods are
 * staged on every rank (kss_stage_pods).  One pod is two launches on `stream` (a
 * hipStream_t, NULL = the context's stream), never synchronising with the host; the
 * caller runs two collectives between them on the same stream.  With b = i & 1:
 * Fold buffers per rank: stats = int64[KSS_AXIS_SLOTS][KSS_AXIS_STATS], key =
 * int64[KSS_AXIS_SLOTS] (workgroup w folds into slot w % KSS_AXIS_SLOTS; readers reduce
 * over the slots, so the key's all_reduce is an elementwise MAX).
 *   kss_axis_eval(i)    applies the pending AssumePod of pod i-1 (prev_key_dev = key[1-b],
 *                       prev_gathered_dev = its gathered statistics; NULL for i = 0),
 *                       clears key_zero_dev = key[b], then filter + raw scores of the local
 *                       rows, folding {feasible count, max TaintToleration raw, max
 *                       NodeAffinity raw, 0} into the slots of stats_dev = stats[b]
 *   (all_gather stats[b] -> gathered_dev[world][SLOTS][4]; world 1: gathered = stats[b])
 *   kss_axis_select     NormalizeScore with the global statistics, weighted total, local
 *                       selectHost key (total << 32 | 0xFFFFFFFF - global index) max-folded
 *                       into key_dev = key[b]; clears stats_zero_dev = stats[1-b]
 *   (all_reduce key[b] MAX)
 *   kss_axis_commit     after the last pod only: its pending AssumePod.
 * chosen_dev[i] = global node or -1.  stats[0] must be zero before pod 0.  Outcomes are
 * also kept for kss_fetch_meta.  Replaces, per rank, the findNodesThatPassFilters /
 * prioritizeNodes / selectHost / AssumePod sequence of scheduleOne (SURVEY 8(a) a1, a15,
 * a17, a18) over that rank's rows; pods with spread / inter-pod programs return
 * KSS_E_UNSUPPORTED. */
#define KSS_AXIS_SLOTS 32
#define KSS_AXIS_STATS 4
int kss_load_cluster_rows(kss_ctx* ctx, const kss_cluster* cl, int32_t lo, int32_t hi);
int kss_axis_eval(kss_ctx* ctx, int32_t pod_index, int64_t* stats_dev, const int64_t* prev_key_dev,
                  const int64_t* prev_gathered_dev, int32_t world, int64_t* key_zero_dev, int32_t* chosen_dev,
                  void* stream);
int kss_axis_select(kss_ctx* ctx, const int64_t* gathered_dev, int32_t world, int64_t* key_dev, int64_t* stats_zero_dev,
                    void* stream);
int kss_axis_commit(kss_ctx* ctx, int32_t pod_index, const int64_t* key_dev, const int64_t* gathered_dev, int32_t world,
                    int32_t* chosen_dev, void* stream);

/* ---- split grid: the node axis as one persistent grid over several GPUs ----------
 * Every part (one context per GPU, one process per GPU) loads the WHOLE cluster and stages
 * the same pods; part p runs shards [p * shards_per_part, (p + 1) * shards_per_part) of the
 * n_parts * shards_per_part shards of k_simple / k_spread, i.e. owns their node rows.  The
 * per-pod exchanges (statistics, critical paths, the packed selectHost key) are the
 * kernels' own granule exchanges: each granule is stored into every part's inbox (xGMI
 * peer stores) and polled in the local inbox, so a pod costs no launch and no host round
 * trip on any GPU.  Every part ends with the full chosen / outcome vectors; node state is
 * current on each part for its own rows.
 *   kss_split_config  allocates the zeroed inbox (n_parts == 1 clears the split) and moves the
 *                     context to a stream with a hardware queue of its own (parts that share one
 *                     of the runtime's GPU_MAX_HW_QUEUES queues would run one after the other)
 *   kss_split_inbox   the inbox's device pointer / size / IPC handle (KSS_IPC_HANDLE_BYTES)
 *   kss_split_peers   every part's inbox as addressable in this process (in-process parts)
 *   kss_split_open    the same from the parts' IPC handles (one process per GPU)
 * Then kss_run_staged on every part concurrently (all parts' grids must be resident at
 * once).  A split run that fails after launching (an exchange timed out: a peer did not
 * run, or failed) leaves the parts' granule epochs apart; that context then refuses split
 * runs (KSS_E_INVAL) until every part is re-armed: kss_split_config, then the peers again.  Replaces SURVEY 8(e)'s per-pod RCCL packed-argmax all-reduce of the node axis
 * (findNodesThatPassFilters / prioritizeNodes / selectHost per rank's rows,
 * simulator/scheduler/scheduler.go:174-219, 232-267, 323-344). */
#define KSS_SPLIT_MAX_PARTS 8
#define KSS_IPC_HANDLE_BYTES 64
int kss_split_config(kss_ctx* ctx, int32_t n_parts, int32_t part, int32_t shards_per_part);
int kss_split_inbox(kss_ctx* ctx, void** dev_ptr, size_t* bytes, void* ipc_handle /* KSS_IPC_HANDLE_BYTES or NULL */);
int kss_split_peers(kss_ctx* ctx, void* const* inboxes /* [n_parts] */);
int kss_split_open(kss_ctx* ctx, const void* handles /* [n_parts][KSS_IPC_HANDLE_BYTES] */);

/* timing of the last kss_schedule_batch / kss_eval_pod device work (HIP events on the work stream) */
int kss_last_timing(kss_ctx* ctx, double* device_ms, int32_t* launches);
/* device time of the sequential-loop kernel alone in the last batch: the k_simple /
 * k_spread launch(es) without the k_static precompute (k_schedule batches: the whole batch) */
int kss_last_loop_timing(kss_ctx* ctx, double* loop_ms);
/* Node-state hand-off self-check of the last run (k_spread batches over several k_static
 * chunks): every chunk's epilogue stores a position-mixed sum of the node state it writes back,
 * the next chunk's prologue compares the state it loads with it and loads again while they
 * disagree (the run fails with KSS_E_DEVICE if they never agree).  *retries = the repeated
 * loads (0 when every hand-off was consistent at once). */
int kss_last_handoff_retries(kss_ctx* ctx, int32_t* retries);
/* The same hand-off's second copy and diagnosis: every epilogue also stores the node state into
 * a shadow buffer, and odd reload attempts read the shadow; *recovered = the loads the shadow
 * answered.  On a launch's first disagreement the prologue lists each word where the state and
 * its shadow differ, KSS_HANDOFF_DIAG_WORDS int64 per entry: {shard | loading XCC << 32 |
 * storing XCC << 40, array (0-2 requested, 3-4 nonzero, 5 pod count, 6 + r resident count row
 * r), node, state by agent load, by atomic add of 0, by nontemporal load, shadow value, the
 * chunk tag, the word's device address, a 100 MHz timestamp}.  Up to cap entries are copied; *n_entries = the entries listed (<= 64). */
#define KSS_HANDOFF_DIAG_WORDS 10
int kss_last_handoff_diag(kss_ctx* ctx, int32_t* recovered, int64_t* entries, int32_t cap, int32_t* n_entries);
/* The hand-off counters of the last k_spread run (0 for other kernels): out3[0] prologue reloads,
 * out3[1] loads the shadow answered, out3[2] shards whose LAST write-back failed the final check
 * (a trailing launch re-sums every shard's node state in HBM against its epilogue's sum; a
 * failure fails the run with KSS_E_DEVICE and is never repaired).  A clean run is {0, 0, 0}. */
int kss_last_handoff_status(kss_ctx* ctx, int32_t* out3);
/* Diagnosis: the device address and size of each of the context's device buffers, in a fixed
 * order (cluster, pristine copy, pods, per-pod upload, record slot, outcomes, chosen, job,
 * granules, error words, hand-off check, stamps, k_simple records, static words, k_spread
 * records, resident rows, delta staging, node-axis values, bound pods, preemption scratch, the
 * split inbox); *n = the number of entries (at most cap are written). */
int kss_buffer_map(kss_ctx* ctx, uint64_t* base, uint64_t* bytes, int32_t cap, int32_t* n);
/* launch geometry of the last scheduling launch: out[0] shards (workgroups) per cluster,
 * out[1] threads per workgroup, out[2] node slots per lane */
int kss_last_geometry(kss_ctx* ctx, int32_t* out3);
/* XCD-local grid of the last run: out2[0] = 1 when its k_simple shards ran on one XCD (the
 * per-pod exchange in that XCD's L2: a cluster of at most CUs-per-XCD shards, one node per lane;
 * KSS_XCD=0 disables it), out2[1] = the chunks that found fewer workgroups on that XCD than shards
 * and ran again on an unrestricted grid (correctness never rests on placement). */
int kss_last_xcd_local(kss_ctx* ctx, int32_t* out2);
/* kernel of the last scheduling launch: 0 general (k_schedule), 1 compact (k_simple:
 * batches without spread / inter-pod programs and without a record), 2 k_spread (batches
 * with programs, without a record), 3 k_preempt (kss_postfilter_pod); <0 on error */
int kss_last_kernel(kss_ctx* ctx);
/* outcome of pods [first, first+n) of the last scheduling launch, recorded or not:
 * out[5*i .. 5*i+4] = chosen, n_feasible, scored, status, best_total (kss_pod_result) */
int kss_fetch_meta(kss_ctx* ctx, int32_t first, int32_t n, int64_t* out);

/* ---- DefaultPreemption PostFilter dry run ---------------------------------
 * Replaces wrappedPlugin.PostFilter -> DefaultPreemption.PostFilter -> Evaluator.Preempt
 * (simulator/scheduler/plugin/wrappedplugin.go:550-577; upstream
 * pkg/scheduler/framework/preemption/preemption.go, v1.26.2) for a pod whose filters left no
 * feasible node: nodesWherePreemptionMightHelp, SelectVictimsOnNode on every potential node
 * (remove the lower-priority pods, filter, reprieve in MoreImportantPod order) and
 * pickOneNodeForPreemption.  Nothing is evicted: the caller deletes the victims
 * (prepareCandidate) and records the nomination (store.go:436-456 "preemption victim").
 *
 * The bound-pod table gives the victims' identity and order: per node, NodeInfo.Pods order
 * (the table order of the pods on that node).  kss_commit appends the committed pod to the
 * table (id = -1 - pod_index) and kss_rollback removes it the way NodeInfo.RemovePod does
 * (the node's last pod takes its place). */
#define KSS_START_UNSET INT64_MAX  /* status.startTime unset (sorts after every start time) */
typedef struct kss_boundset {
  int32_t n;                 /* bound pods (on nodes of the loaded cluster) */
  int32_t n_ints;
  const int64_t* id;         /* [n] caller ids reported for victims */
  const int32_t* node;       /* [n] global node index */
  const int32_t* priority;   /* [n] corev1helpers.PodPriority */
  const int64_t* start;      /* [n] status.startTime on any monotone integer clock, KSS_START_UNSET if unset */
  const int32_t* cls;        /* [n] the class_count row the pod counts in */
  const int64_t* req;        /* [KSS_NRES][n] the pod's NodeInfo.Requested contribution */
  const int32_t* terms_off;  /* [n] the term_count rows it contributes: ints[terms_off .. +terms_len) */
  const int32_t* terms_len;  /* [n] */
  const int32_t* ints;
  const int64_t* nonzero;    /* [2][n] NodeInfo.NonZeroRequested cpu / memory contribution, or NULL */
  const uint64_t* ports;     /* [n] the NodeInfo.UsedPorts bits it holds, or NULL (none) */
} kss_boundset;
int kss_load_bound(kss_ctx* ctx, const kss_boundset* bs);
/* The informer's RemovePod for pods of the bound-pod table -- the victims a PostFilter named, once
 * the caller deleted them (prepareCandidate; simulator/scheduler/plugin/wrappedplugin.go:550-577
 * records the nomination): every id (a kss_boundset id, or -1 - i for a pod committed from
 * ps.pods[i]) leaves the table and its node (Requested, NonZeroRequested, pod count, class and term
 * counts, host ports).  Loaded pods need the boundset's nonzero array; pods with volumes are
 * refused (KSS_E_UNSUPPORTED: kss_apply_volume_delta is their sync).  An id not in the table is
 * KSS_E_INVAL and nothing is removed. */
int kss_remove_bound(kss_ctx* ctx, const int64_t* ids, int32_t n);

#define KSS_PREEMPT_NOMINATED 0
#define KSS_PREEMPT_NO_CANDIDATE 1   /* FitError: no node where evicting lower-priority pods helps */
#define KSS_PREEMPT_NOT_ELIGIBLE 2   /* preemptionPolicy Never */
#define KSS_PREEMPT_SCHEDULABLE 3    /* a node passes every filter: PostFilter does not run */
typedef struct kss_preempt_result {
  int32_t status;           /* KSS_PREEMPT_* */
  int32_t nominated;        /* global node index, -1 */
  int32_t n_potential;      /* nodes whose filter status is not UnschedulableAndUnresolvable */
  int32_t n_candidates;     /* potential nodes where the pod fits after evicting some pods */
  int32_t n_victims;        /* victims on the nominated node (the first victims_cap are written) */
  int32_t victims_cap;
  int64_t* victims;         /* caller-owned [victims_cap]: boundset ids, in eviction (importance) order */
  int32_t highest_priority; /* pickOneNodeForPreemption criteria of the nominated node */
  int32_t pad;
  int64_t sum_priority;     /* sum of (priority + 2^31) over the victims */
  int64_t earliest_start;   /* earliest start among the highest-priority victims */
} kss_preempt_result;
/* PostFilter dry run of ps.pods[pod_index] against the current snapshot (the state the
 * pod's filters saw): call after kss_eval_pod reported it unschedulable. */
int kss_postfilter_pod(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, kss_preempt_result* out);

/* ---- annotation formatting (store.go GetStoredResult semantics) -------- */
typedef struct kss_names {
  const char* const* node_names;    /* [n_nodes] */
  const char* const* taint_keys;    /* [n_taints] */
  const char* const* taint_values;  /* [n_taints] */
  const char* const* scalar_names;  /* [n_scalar] */
  int32_t n_messages;               /* per-pod status messages (VolumeBinding PreFilter, VolumeZone errors) */
  int32_t pad;
  const char* const* messages;      /* [n_messages] */
} kss_names;
int kss_set_names(kss_ctx* ctx, const kss_names* names);
/* Format the 13 annotation values of one recorded pod result as
 * "key\0value\0key\0value\0...\0\0" into buf.  *need receives the byte count
 * required (call with cap=0 to size).  Formatting is lazy: nothing is produced
 * in the timed scheduling path. */
int kss_format_annotations(kss_ctx* ctx, const kss_pod_result* res, int32_t n_nodes, char* buf, size_t cap,
                           size_t* need);
/* Context-free variant (host only): names and profile passed explicitly. */
int kss_format_annotations_ex(const kss_names* names, const kss_profile* prof, const kss_pod_result* res,
                              int32_t n_nodes, int32_t n_taints, int32_t n_scalar, char* buf, size_t cap, size_t* need);
/* The same two with the pod's NodeAffinity PreFilterResult: store.go:522-534 records
 * PreFilterResult.NodeNames.List() under scheduler-simulator/prefilter-result; ps.pods[pod_index]
 * (names_off/names_len) supplies the node set.  Replaces the AddPreFilterResult path of
 * simulator/scheduler/plugin/resultstore/store.go:522 for pods with matchFields metadata.name. */
int kss_format_pod_annotations(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, const kss_pod_result* res,
                               int32_t n_nodes, char* buf, size_t cap, size_t* need);
int kss_format_pod_annotations_ex(const kss_names* names, const kss_profile* prof, const kss_podset* ps,
                                  int32_t pod_index, const kss_pod_result* res, int32_t n_nodes, int32_t n_taints,
                                  int32_t n_scalar, char* buf, size_t cap, size_t* need);
/* sizeof() of every ABI struct, in header order; returns the count written (ABI self-check) */
int kss_abi_sizes(int32_t* out, int32_t n);
/* Host only (no device): which sequential-loop kernel a staged, unrecorded batch of `ps` on
 * `cl` can take, by its pod programs: out3[0] = 1 k_simple, 2 k_spread, 0 k_schedule only;
 * out3[1] = the first pod that rules out k_spread (-1 none), out3[2] = the reason code
 * (kss_plan_reason).  The launch still checks LDS geometry and value bounds. */
int kss_plan_podset(const kss_cluster* cl, const kss_podset* ps, int32_t* out3);
/* The same with the profile the batch runs under (NULL: kss_plan_podset): a profile with
 * percentageOfNodesToScore below 100 on a cluster of 100+ nodes (the findNodesThatPassFilters
 * window) keeps k_simple only when no pod has a NodeAffinity PreFilterResult list, and rules out
 * k_spread; a profile that scores an extended resource on a cluster that has them rules out both
 * loop kernels (out3[1] = the pod, out3[2] the reason). */
int kss_plan_podset_ex(const kss_cluster* cl, const kss_podset* ps, const kss_profile* prof, int32_t* out3);
const char* kss_plan_reason(int32_t code);
/* Test support: y[i] = the device restatement of Go math.Log (kss_spread.cuh go_log_dev,
 * PodTopologySpread's topologyNormalizingWeight in k_spread) at x[i], i < n, evaluated on
 * `device`; host arrays.  Compared bitwise with the host port (kss_go_log_c) by the tests. */
int kss_device_go_log(int32_t device, const double* x, double* y, int32_t n);

/* ---- synthetic clusters (SplitMix64, seed 0x5EED0000 + config) */
typedef struct kss_synth {
  kss_cluster cluster;
  kss_podset pods;
  void* owner; /* internal */
} kss_synth;
/* config_id 1..5 selects the BASELINE.json recipe; n_nodes/n_pods override sizes when > 0 */
int kss_synth_make(int32_t config_id, uint64_t seed, int32_t n_nodes, int32_t n_pods, kss_synth* out);
void kss_synth_free(kss_synth* s);

#ifdef __cplusplus
}
#endif
#endif /* KSS_H_ */
