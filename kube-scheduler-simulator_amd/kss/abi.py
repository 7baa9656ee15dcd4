"""ctypes mirror of include/kss.h (the C ABI of libkss.so).

Kept byte-for-byte in sync with the header; ``tests/test_abi.py`` checks every
struct size against the library's own ``kss_abi_sizes``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

KSS_OK = 0
KSS_RES_CPU, KSS_RES_MEMORY, KSS_RES_EPHEMERAL, KSS_RES_SCALAR0 = 0, 1, 2, 3
KSS_NRES = 7
KSS_MAX_SCALAR = 4
KSS_MAX_TAINTS = 64
KSS_TAINT_ORDER = 8
KSS_MAX_BINS = 1024
KSS_MAX_PORTS = 64
KSS_SPLIT_MAX_PARTS = 8
KSS_IPC_HANDLE_BYTES = 64
# kss_eval_pod_view fields
KSS_FIELD_FAIL, KSS_FIELD_DETAIL, KSS_FIELD_RAW, KSS_FIELD_NORM, KSS_FIELD_TOTAL = 1, 2, 4, 8, 16
KSS_FIELD_ALL = 0x1F
KSS_IMAGE_MIN_THRESHOLD = 23 * 1024 * 1024
KSS_IMAGE_MAX_CONTAINER_THRESHOLD = 1000 * 1024 * 1024

# filter plugins (default MultiPoint order; simulator/scheduler/config/plugin_test.go:15-36)
FILTER_PLUGINS = [
    None,
    "NodeUnschedulable",
    "NodeName",
    "TaintToleration",
    "NodeAffinity",
    "NodePorts",
    "NodeResourcesFit",
    "VolumeRestrictions",
    "EBSLimits",
    "GCEPDLimits",
    "NodeVolumeLimits",
    "AzureDiskLimits",
    "VolumeBinding",
    "VolumeZone",
    "PodTopologySpread",
    "InterPodAffinity",
]
KSS_F_PASS = 0
KSS_F_NODE_UNSCHEDULABLE = 1
KSS_F_NODE_NAME = 2
KSS_F_TAINT_TOLERATION = 3
KSS_F_NODE_AFFINITY = 4
KSS_F_NODE_PORTS = 5
KSS_F_NODE_RESOURCES_FIT = 6
KSS_F_VOLUME_RESTRICTIONS = 7
KSS_F_EBS_LIMITS = 8
KSS_F_GCEPD_LIMITS = 9
KSS_F_NODE_VOLUME_LIMITS = 10
KSS_F_AZURE_DISK_LIMITS = 11
KSS_F_VOLUME_BINDING = 12
KSS_F_VOLUME_ZONE = 13
KSS_F_POD_TOPOLOGY_SPREAD = 14
KSS_F_INTER_POD_AFFINITY = 15
KSS_NFILTER = 15
KSS_F_NOT_EVALUATED = 255
KSS_PASS_NOT_KEPT = 1  # fail_detail of the passing node that ended a percentageOfNodesToScore search

KSS_FIT_TOO_MANY_PODS = 1 << 0
KSS_FIT_CPU = 1 << 1
KSS_FIT_MEMORY = 1 << 2
KSS_FIT_EPHEMERAL = 1 << 3
KSS_FIT_SCALAR0 = 1 << 4
KSS_PTS_CONSTRAINTS_NOT_MATCH = 0
KSS_PTS_MISSING_LABEL = 1
KSS_IPA_AFFINITY = 0
KSS_IPA_ANTI_AFFINITY = 1
KSS_IPA_EXISTING_ANTI_AFFINITY = 2
KSS_VB_NODE_CONFLICT = 0
KSS_VB_PV_NOT_EXIST = 1
KSS_VB_BIND_CONFLICT = 2
KSS_VB_NODE_BIND = 3
KSS_VB_BIND_PV_NOT_EXIST = 4

SCORE_PLUGINS = [
    "TaintToleration",
    "NodeAffinity",
    "NodeResourcesFit",
    "VolumeBinding",
    "PodTopologySpread",
    "InterPodAffinity",
    "NodeResourcesBalancedAllocation",
    "ImageLocality",
]
KSS_NSCORE = 8
(KSS_S_TAINT_TOLERATION, KSS_S_NODE_AFFINITY, KSS_S_NODE_RESOURCES_FIT, KSS_S_VOLUME_BINDING,
 KSS_S_POD_TOPOLOGY_SPREAD, KSS_S_INTER_POD_AFFINITY, KSS_S_BALANCED_ALLOCATION, KSS_S_IMAGE_LOCALITY) = range(8)

KSS_NODE_UNSCHEDULABLE = 1 << 0
KSS_NODE_HAS_LABELS = 1 << 1
KSS_NODE_VOLUME_ZONE = 1 << 2
KSS_KEY_UNIQUE = 1 << 0
KSS_KEY_HOSTNAME = 1 << 1

(KSS_OP_FALSE, KSS_OP_TRUE, KSS_OP_MASK, KSS_OP_IN, KSS_OP_NOTIN, KSS_OP_EXISTS, KSS_OP_DNE, KSS_OP_GT, KSS_OP_LT,
 KSS_OP_NAME_IN, KSS_OP_NAME_NOTIN) = range(11)
KSS_SPREAD_POLICY_AFFINITY_HONOR = 1 << 0
KSS_SPREAD_POLICY_TAINTS_HONOR = 1 << 1
(KSS_IPA_EXISTING_ANTI, KSS_IPA_REQ_AFFINITY, KSS_IPA_REQ_ANTI, KSS_IPA_SCORE_CLASS, KSS_IPA_SCORE_TERM) = range(5)

(KSS_VOL_CONFLICT, KSS_VOL_LIMIT, KSS_VOL_BIND_AFFINITY, KSS_VOL_BIND_PV_MISSING, KSS_VOL_ZONE, KSS_VOL_ZONE_ERROR,
 KSS_VOL_OWN, KSS_VOL_OWN_PRIVATE, KSS_VOL_BIND_WFFC) = range(9)
KSS_MAX_VOL_KEYS = 64
KSS_MAX_WFFC = 4
KSS_PF_OK, KSS_PF_NODE_AFFINITY_CONFLICT, KSS_PF_ERROR, KSS_PF_VOLUME_BINDING = range(4)

KSS_POD_TOL_UNSCHEDULABLE = 1 << 0
KSS_POD_HAS_REQ_AFFINITY = 1 << 1
KSS_POD_PTS_REQUIRE_ALL = 1 << 2
KSS_POD_IPA_SELF_MATCH = 1 << 3
KSS_POD_IPA_HAS_PREFERRED = 1 << 4
KSS_POD_PTS_SCORE_STATE = 1 << 5
KSS_POD_PREEMPT_NEVER = 1 << 6

KSS_START_UNSET = 2**63 - 1
KSS_PREEMPT_NOMINATED = 0
KSS_PREEMPT_NO_CANDIDATE = 1
KSS_PREEMPT_NOT_ELIGIBLE = 2
KSS_PREEMPT_SCHEDULABLE = 3

KSS_FIT_LEAST_ALLOCATED = 0
KSS_FIT_MOST_ALLOCATED = 1

KSS_SCHED_RECORD = 1 << 0
KSS_SCHED_FORCE_MULTI_WG = 1 << 1
KSS_SCHED_FORCE_SINGLE_WG = 1 << 2
KSS_SCHED_GENERAL_KERNEL = 1 << 3

P = C.POINTER
i32, i64, u32, u64, u8, u16 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_uint8, C.c_uint16


class Cluster(C.Structure):
    _fields_ = [
        ("n_nodes", i32), ("n_scalar", i32), ("n_label_keys", i32), ("n_label_values", i32),
        ("n_classes", i32), ("n_terms", i32), ("n_taints", i32), ("node_base", i32),
        ("alloc", P(i64)), ("requested", P(i64)), ("nonzero", P(i64)), ("allowed_pods", P(i32)),
        ("pod_count", P(i32)), ("node_flags", P(u32)), ("taint_hard", P(u64)), ("taint_soft", P(u64)),
        ("taint_order", P(u8)), ("label_value", P(i32)), ("key_base", P(i32)), ("key_card", P(i32)),
        ("key_flags", P(u32)), ("key_empty", P(i32)), ("value_int", P(i64)), ("value_is_int", P(u8)),
        ("class_count", P(i32)), ("term_count", P(i32)),
        ("n_ports", i32), ("n_images", i32), ("port_used", P(u64)), ("image_score", P(i64)),
        ("n_vol_rows", i32), ("n_vol_keys", i32), ("vol_count", P(i32)), ("vol_attached", P(i32)),
        ("vol_limit", P(i32)), ("vol_row_key", P(i32)), ("vol_key_plugin", P(i32)),
        ("n_pvs", i32), ("n_wclaims", i32), ("pv_owner", P(i32)), ("claim_node", P(i32)),
    ]


class Req(C.Structure):
    _fields_ = [("key", i32), ("op", i32), ("list_off", i32), ("list_len", i32), ("mask", u64), ("ival", i64)]


class Term(C.Structure):
    _fields_ = [("req_off", i32), ("req_len", i32), ("weight", i32), ("flags", i32)]


class Spread(C.Structure):
    _fields_ = [("key", i32), ("max_skew", i32), ("self_match", i32), ("flags", i32), ("cls_off", i32),
                ("cls_len", i32), ("min_domains", i32), ("pad", i32)]


class Ipa(C.Structure):
    _fields_ = [("kind", i32), ("key", i32), ("row_off", i32), ("row_len", i32), ("coef", i32), ("pad", i32)]


class Vol(C.Structure):
    _fields_ = [("kind", i32), ("key", i32), ("row", i32), ("count", i32), ("a", i32), ("b", i32)]


class Pod(C.Structure):
    _fields_ = [
        ("fit_request", i64 * KSS_NRES), ("score_req_nz", i64 * KSS_NRES), ("score_req", i64 * KSS_NRES),
        ("commit_req", i64 * KSS_NRES), ("commit_nz", i64 * 2), ("tol_hard", u64), ("tol_soft", u64),
        ("node_name", i32), ("flags", u32), ("sel_off", i32), ("sel_len", i32), ("aff_off", i32), ("aff_len", i32),
        ("pref_off", i32), ("pref_len", i32), ("spread_off", i32), ("n_hard", i32), ("n_soft", i32),
        ("ipa_off", i32), ("ipa_len", i32), ("cls", i32), ("own_terms_off", i32), ("own_terms_len", i32),
        ("prefilter_status", i32), ("names_off", i32), ("names_len", i32), ("priority", i32), ("prefilter_msg", i32),
        ("port_conflict", u64), ("port_add", u64), ("img_off", i32), ("img_len", i32), ("n_containers", i32),
        ("vol_off", i32), ("vol_len", i32), ("uid", i32),
    ]


class PodSet(C.Structure):
    _fields_ = [("n_pods", i32), ("n_reqs", i32), ("n_terms", i32), ("n_spreads", i32), ("n_ipa", i32),
                ("n_ints", i32), ("pods", P(Pod)), ("reqs", P(Req)), ("terms", P(Term)), ("spreads", P(Spread)),
                ("ipa", P(Ipa)), ("ints", P(i32)), ("n_vols", i32), ("pad", i32), ("vols", P(Vol))]


class Profile(C.Structure):
    _fields_ = [("weight", i32 * KSS_NSCORE), ("filter_enabled", u32), ("score_enabled", u32),
                ("fit_strategy", i32), ("fit_n", i32), ("fit_res", i32 * 4), ("fit_weight", i64 * 4),
                ("ba_n", i32), ("ba_res", i32 * 4), ("hard_pod_affinity_weight", i32),
                ("pct_nodes_to_score", i32), ("system_defaulted", i32), ("pad", i32)]


class PodResult(C.Structure):
    _fields_ = [("fail_plugin", P(u8)), ("fail_detail", P(u16)), ("raw", P(i64)), ("norm", P(i64)),
                ("total", P(i64)), ("n_feasible", i32), ("chosen", i32), ("best_total", i64), ("scored", i32),
                ("status", i32)]


class PodView(C.Structure):
    _fields_ = [("fail_plugin", P(u8)), ("fail_detail", P(u16)), ("raw", P(i64)), ("norm", P(i64)),
                ("total", P(i64)), ("n_feasible", i32), ("chosen", i32), ("best_total", i64), ("scored", i32),
                ("status", i32)]


class PodCView(C.Structure):
    """kss_pod_cview: the compact service record (raw / total int32, norm uint8), or `wide`."""
    _fields_ = [("fail_plugin", P(u8)), ("fail_detail", P(u16)), ("raw", P(i32)), ("norm", P(u8)),
                ("total", P(i32)), ("n_feasible", i32), ("chosen", i32), ("best_total", i64), ("scored", i32),
                ("status", i32), ("is_wide", i32), ("pad", i32), ("wide", PodView)]


class Config(C.Structure):
    _fields_ = [("device", i32), ("max_pods_record", i32), ("class_capacity", i32), ("term_capacity", i32)]


class Names(C.Structure):
    _fields_ = [("node_names", P(C.c_char_p)), ("taint_keys", P(C.c_char_p)), ("taint_values", P(C.c_char_p)),
                ("scalar_names", P(C.c_char_p)), ("n_messages", i32), ("pad", i32), ("messages", P(C.c_char_p))]


class Boundset(C.Structure):
    _fields_ = [("n", i32), ("n_ints", i32), ("id", P(i64)), ("node", P(i32)), ("priority", P(i32)),
                ("start", P(i64)), ("cls", P(i32)), ("req", P(i64)), ("terms_off", P(i32)), ("terms_len", P(i32)),
                ("ints", P(i32)), ("nonzero", P(i64)), ("ports", P(C.c_uint64))]


class PreemptResult(C.Structure):
    _fields_ = [("status", i32), ("nominated", i32), ("n_potential", i32), ("n_candidates", i32),
                ("n_victims", i32), ("victims_cap", i32), ("victims", P(i64)), ("highest_priority", i32),
                ("pad", i32), ("sum_priority", i64), ("earliest_start", i64)]


class Synth(C.Structure):
    _fields_ = [("cluster", Cluster), ("pods", PodSet), ("owner", C.c_void_p)]


POD_DTYPE = np.dtype(Pod)
REQ_DTYPE = np.dtype(Req)
TERM_DTYPE = np.dtype(Term)
SPREAD_DTYPE = np.dtype(Spread)
IPA_DTYPE = np.dtype(Ipa)
VOL_DTYPE = np.dtype(Vol)


def ptr(arr: np.ndarray, ctype):
    """Pointer to a contiguous numpy array (the array must outlive the call)."""
    assert arr.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return arr.ctypes.data_as(P(ctype))


def default_profile() -> Profile:
    """The v1.26 default profile as the simulator builds it.

    Weights: simulator/scheduler/plugin/plugins_test.go:184-204 (TT 3, NA 2, Fit 1,
    PTS 2, IPA 2, BA 1, ImageLocality 1; VolumeBinding has no weight -> 1 by
    getScorePluginWeight, plugins.go:288-303).  Args: plugins_test.go:878-1096.
    """
    p = Profile()
    w = {KSS_S_TAINT_TOLERATION: 3, KSS_S_NODE_AFFINITY: 2, KSS_S_NODE_RESOURCES_FIT: 1, KSS_S_VOLUME_BINDING: 1,
         KSS_S_POD_TOPOLOGY_SPREAD: 2, KSS_S_INTER_POD_AFFINITY: 2, KSS_S_BALANCED_ALLOCATION: 1,
         KSS_S_IMAGE_LOCALITY: 1}
    for k, v in w.items():
        p.weight[k] = v
    p.filter_enabled = sum(1 << i for i in range(1, KSS_NFILTER + 1))
    p.score_enabled = (1 << KSS_NSCORE) - 1
    p.fit_strategy = KSS_FIT_LEAST_ALLOCATED
    p.fit_n = 2
    p.fit_res[0], p.fit_res[1] = KSS_RES_CPU, KSS_RES_MEMORY
    p.fit_weight[0], p.fit_weight[1] = 1, 1
    p.ba_n = 2
    p.ba_res[0], p.ba_res[1] = KSS_RES_CPU, KSS_RES_MEMORY
    p.hard_pod_affinity_weight = 1
    p.pct_nodes_to_score = 100
    p.system_defaulted = 1
    return p
