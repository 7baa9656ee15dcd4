"""Snapshot I/O and the scheduler configuration.

* ``read_snapshot`` / ``write_snapshot``: the simulator's ``ResourcesForSnap`` JSON
  (simulator/snapshot/snapshot.go:32-41: pods, nodes, pvs, pvcs, storageClasses,
  priorityClasses, schedulerConfig, namespaces) <-> the object lists ``kss.compile`` turns
  into the device struct-of-arrays.  Pods with ``spec.nodeName`` are NodeInfo pods (bound);
  the others are pending, in listed order.  A pod without ``spec.priority`` gets its
  PriorityClass's value (the Priority admission plugin the import passes through).
* ``profile_from_config``: a ``KubeSchedulerConfiguration`` (v1; the simulator keeps one
  profile, plugins.go:288-303) -> ``kss_profile``: enabled filter / score plugins from the
  default MultiPoint set merged with the profile's sets as the simulator merges them
  (plugins.go mergePluginSet, :227-283), weights with 0 -> 1 (getScorePluginWeight,
  :288-303), NodeResourcesFitArgs.scoringStrategy, NodeResourcesBalancedAllocationArgs,
  InterPodAffinityArgs.hardPodAffinityWeight, PodTopologySpreadArgs.defaultingType and
  percentageOfNodesToScore (unset: 0, the adaptive default).
* ``sync_deltas``: the NodeInfo-generation delta sync of an updated snapshot onto a loaded
  context (kss_apply_node_delta / kss_apply_count_delta / kss_apply_port_delta) instead of a
  full reload -- the rows whose mutable columns changed.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .compile import CompiledCluster, Unsupported

# v1.26 default MultiPoint plugins (pkg/scheduler/apis/config/v1/default_plugins.go; the
# simulator's test of the list: simulator/scheduler/config/plugin_test.go:15-36)
DEFAULT_MULTIPOINT: List[Tuple[str, int]] = [
    ("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0), ("TaintToleration", 3), ("NodeAffinity", 2),
    ("NodePorts", 0), ("NodeResourcesFit", 1), ("VolumeRestrictions", 0), ("EBSLimits", 0), ("GCEPDLimits", 0),
    ("NodeVolumeLimits", 0), ("AzureDiskLimits", 0), ("VolumeBinding", 0), ("VolumeZone", 0),
    ("PodTopologySpread", 2), ("InterPodAffinity", 2), ("DefaultPreemption", 0),
    ("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("DefaultBinder", 0),
]
SCORE_CAPABLE = set(abi.SCORE_PLUGINS)
FILTER_CAPABLE = set(p for p in abi.FILTER_PLUGINS if p)
RESOURCE_IDS = {"cpu": abi.KSS_RES_CPU, "memory": abi.KSS_RES_MEMORY, "ephemeral-storage": abi.KSS_RES_EPHEMERAL}


# ----------------------------------------------------------------------------- snapshot
@dataclass
class Snapshot:
    nodes: List[dict]
    bound: List[dict]
    pending: List[dict]
    namespaces: Dict[str, Dict[str, str]]
    priority_classes: Dict[str, int] = field(default_factory=dict)
    scheduler_config: Optional[dict] = None
    pvs: List[dict] = field(default_factory=list)
    pvcs: List[dict] = field(default_factory=list)
    storage_classes: List[dict] = field(default_factory=list)

    def storage(self) -> dict:
        """The volume plugins' objects for kss.compile (Compiler(storage=...)).  ResourcesForSnap
        carries no CSINodes (snapshot.go:32-41): CSI attach limits come from allocatable only."""
        return {"pvs": list(self.pvs), "pvcs": list(self.pvcs), "storage_classes": list(self.storage_classes),
                "csinodes": []}


def _resolve_priority(pod: dict, classes: Dict[str, int], default: Optional[int]) -> dict:
    spec = pod.get("spec") or {}
    if "priority" in spec:
        return pod
    name = spec.get("priorityClassName")
    value = classes.get(name) if name else default
    if value is None:
        return pod
    pod = dict(pod)
    pod["spec"] = dict(spec, priority=int(value))
    return pod


def read_snapshot(src) -> Snapshot:
    """ResourcesForSnap from a dict, a JSON string or a file path."""
    if isinstance(src, str):
        src = json.loads(src) if src.lstrip().startswith("{") else json.load(open(src))
    pcs = {}
    default = None
    for pc in src.get("priorityClasses") or []:
        nm = (pc.get("metadata") or {}).get("name")
        pcs[nm] = int(pc.get("value") or 0)
        if pc.get("globalDefault"):
            default = int(pc.get("value") or 0)
    nodes = list(src.get("nodes") or [])
    bound, pending = [], []
    for p in src.get("pods") or []:
        p = _resolve_priority(p, pcs, default)
        (bound if (p.get("spec") or {}).get("nodeName") else pending).append(p)
    ns = {}
    for n in src.get("namespaces") or []:
        md = n.get("metadata") or {}
        ns[md.get("name", "")] = dict(md.get("labels") or {})
    for p in bound + pending:
        ns.setdefault((p.get("metadata") or {}).get("namespace") or "default", {})
    return Snapshot(nodes=nodes, bound=bound, pending=pending, namespaces=ns, priority_classes=pcs,
                    scheduler_config=src.get("schedulerConfig"), pvs=list(src.get("pvs") or []),
                    pvcs=list(src.get("pvcs") or []), storage_classes=list(src.get("storageClasses") or []))


def write_snapshot(snap: Snapshot) -> dict:
    """The ResourcesForSnap JSON object of a snapshot (bound pods, then pending ones)."""
    return {"pods": list(snap.bound) + list(snap.pending), "nodes": list(snap.nodes), "pvs": list(snap.pvs),
            "pvcs": list(snap.pvcs), "storageClasses": list(snap.storage_classes),
            "priorityClasses": [{"metadata": {"name": k}, "value": v} for k, v in sorted(snap.priority_classes.items())],
            "schedulerConfig": snap.scheduler_config,
            "namespaces": [{"metadata": {"name": k, "labels": v}} for k, v in sorted(snap.namespaces.items())]}


# ----------------------------------------------------------------------------- profile
def merge_plugin_set(default_enabled: Sequence[Tuple[str, int]], custom: Optional[dict]) -> List[Tuple[str, int]]:
    """simulator/scheduler/plugin/plugins.go mergePluginSet: the default set minus the
    disabled plugins ("*": all), defaults re-configured by the custom set updated in place,
    the other custom plugins appended."""
    custom = custom or {}
    disabled = {p.get("name") for p in custom.get("disabled") or []}
    enabled_custom = {p.get("name"): (i, p) for i, p in enumerate(custom.get("enabled") or [])}
    replaced = set()
    out = []
    if "*" not in disabled:
        for name, w in default_enabled:
            if name in disabled:
                continue
            if name in enabled_custom:
                i, p = enabled_custom[name]
                w = int(p.get("weight") or 0)
                replaced.add(i)
            out.append((name, w))
    for i, p in enumerate(custom.get("enabled") or []):
        if i not in replaced:
            out.append((p.get("name"), int(p.get("weight") or 0)))
    return out


def _args_of(profile: dict, name: str) -> dict:
    for pc in profile.get("pluginConfig") or []:
        if pc.get("name") == name:
            return pc.get("args") or {}
    return {}


def _resource_id(name: str, scalars: Sequence[str]) -> int:
    if name in RESOURCE_IDS:
        return RESOURCE_IDS[name]
    if name in scalars:
        return abi.KSS_RES_SCALAR0 + list(scalars).index(name)
    raise Unsupported(f"scoring resource {name!r} is not a column of the compiled cluster")


def store_weights_from_config(cfg: Optional[dict]) -> Dict[str, int]:
    """The weights the simulator's result store applies to finalscore annotations
    (getScorePluginWeight, plugins.go:288-303, over the configuration ConvertForSimulator
    produced, plugins.go:173-195): the profile's Score.Enabled entries, then the MultiPoint set
    merged with the in-tree defaults, each assignment overwriting the previous one -- so a
    plugin listed in both takes its MultiPoint weight -- and 0 -> 1.

    These can differ from the weights the framework schedules with (``profile_from_config``:
    a plugin configured at the Score extension point keeps that weight over its MultiPoint
    one): the simulator then records finalscores that are not the ones it selected the node
    by.  The device schedules with the framework's weights; the formatter takes these."""
    plugins = (((cfg or {}).get("profiles") or [{}])[0].get("plugins")) or {}
    multi = merge_plugin_set(DEFAULT_MULTIPOINT, plugins.get("multiPoint"))
    user_score = [(p.get("name"), int(p.get("weight") or 0)) for p in (plugins.get("score") or {}).get("enabled") or []]
    out: Dict[str, int] = {}
    for n, w in user_score + multi:
        out[n] = w if w != 0 else 1
    return out


def store_profile_from_config(cfg: Optional[dict], scalars: Sequence[str] = ()) -> abi.Profile:
    """``profile_from_config`` with the result store's weights (``store_weights_from_config``):
    the profile to format annotations with (kss_format_*_ex)."""
    prof = profile_from_config(cfg, scalars)
    w = store_weights_from_config(cfg)
    for s, n in enumerate(abi.SCORE_PLUGINS):
        if prof.score_enabled & (1 << s):
            prof.weight[s] = w.get(n, prof.weight[s])
    return prof


def profile_from_config(cfg: Optional[dict], scalars: Sequence[str] = (),
                        pct_nodes_to_score: Optional[int] = None) -> abi.Profile:
    """kss_profile of a KubeSchedulerConfiguration's (first) profile; None -> the default plugins.
    Weights follow the framework (the Score extension point's entry wins over MultiPoint's);
    the result store's annotation weights are ``store_weights_from_config``.

    percentageOfNodesToScore: the simulator's scheduler keeps only Profiles and Extenders of the
    configuration it is given and resets every other field to the v1 defaults
    (filterOutNonAllowedChangesOnCfg, simulator/scheduler/scheduler.go:258-275, applied at
    :163), so it always runs with 0 -- the adaptive numFeasibleNodesToFind -- whatever the
    configuration (or its absence) says.  The profile follows that: 0, unless the caller opts in
    to another value with ``pct_nodes_to_score`` (the north_star / bench workloads use 100).  The
    configuration's own field is still validated (ValidateKubeSchedulerConfiguration: 0..100)."""
    if pct_nodes_to_score is not None and not 0 <= int(pct_nodes_to_score) <= 100:
        raise Unsupported("percentageOfNodesToScore must be between 0 and 100")
    pct = 0 if pct_nodes_to_score is None else int(pct_nodes_to_score)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    if not cfg:
        return prof
    profiles = cfg.get("profiles") or [{}]
    if len(profiles) > 1:
        raise Unsupported("one scheduler profile only (plugins.go getScorePluginWeight reads profiles[0])")
    p0 = profiles[0]
    # v1.26 has the global field only (profiles gained their own in v1.27); validated, then reset
    # by the simulator (see above)
    cfg_pct = cfg.get("percentageOfNodesToScore")
    if cfg_pct is not None and not 0 <= int(cfg_pct) <= 100:
        raise Unsupported("percentageOfNodesToScore must be between 0 and 100 (ValidateKubeSchedulerConfiguration)")
    plugins = p0.get("plugins") or {}
    multi = merge_plugin_set(DEFAULT_MULTIPOINT, plugins.get("multiPoint"))
    names = [n for n, _ in multi]
    # per-extension-point sets: MultiPoint plugins are expanded, then filter / score
    # disabled entries remove them and enabled entries add them
    filt = merge_plugin_set([(n, 0) for n in names if n in FILTER_CAPABLE], plugins.get("filter"))
    score = merge_plugin_set([(n, w) for n, w in multi if n in SCORE_CAPABLE], plugins.get("score"))
    for n, _ in multi + filt + score:
        if n not in FILTER_CAPABLE | SCORE_CAPABLE | {"PrioritySort", "DefaultPreemption", "DefaultBinder"}:
            raise Unsupported(f"plugin {n!r} has no device restatement")
    prof.filter_enabled = 0
    for n, _ in filt:
        if n in FILTER_CAPABLE:
            prof.filter_enabled |= 1 << abi.FILTER_PLUGINS.index(n)
    prof.score_enabled = 0
    for s in range(abi.KSS_NSCORE):
        prof.weight[s] = 0
    weights = {}
    for n, w in score + [(n, w) for n, w in multi if n in SCORE_CAPABLE]:
        weights.setdefault(n, w)
    for n, _ in score:
        s = abi.SCORE_PLUGINS.index(n)
        prof.score_enabled |= 1 << s
        prof.weight[s] = weights[n] if weights[n] != 0 else 1  # getScorePluginWeight: 0 -> 1
    fit = _args_of(p0, "NodeResourcesFit").get("scoringStrategy") or {}
    typ = fit.get("type", "LeastAllocated")
    if typ not in ("LeastAllocated", "MostAllocated"):
        raise Unsupported(f"NodeResourcesFit scoring strategy {typ!r}")
    prof.fit_strategy = abi.KSS_FIT_LEAST_ALLOCATED if typ == "LeastAllocated" else abi.KSS_FIT_MOST_ALLOCATED
    res = fit.get("resources") or [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]
    if len(res) > 4:
        raise Unsupported("more than 4 NodeResourcesFit scoring resources")
    prof.fit_n = len(res)
    for i, r in enumerate(res):
        prof.fit_res[i] = _resource_id(r.get("name"), scalars)
        prof.fit_weight[i] = int(r.get("weight") or 1)
    ba = _args_of(p0, "NodeResourcesBalancedAllocation").get("resources") or [{"name": "cpu"}, {"name": "memory"}]
    if len(ba) > 4:
        raise Unsupported("more than 4 BalancedAllocation resources")
    prof.ba_n = len(ba)
    for i, r in enumerate(ba):
        prof.ba_res[i] = _resource_id(r.get("name"), scalars)
    ipa = _args_of(p0, "InterPodAffinity")
    prof.hard_pod_affinity_weight = int(ipa.get("hardPodAffinityWeight", 1))
    pts = _args_of(p0, "PodTopologySpread")
    dt = pts.get("defaultingType", "System")
    if dt == "List" and pts.get("defaultConstraints"):
        raise Unsupported("PodTopologySpread List defaulting with default constraints")
    prof.system_defaulted = 1 if dt == "System" else 0
    prof.pct_nodes_to_score = pct
    return prof


# ----------------------------------------------------------------------------- deltas
def sync_deltas(ctx, old: CompiledCluster, new: CompiledCluster) -> Dict[str, int]:
    """Bring a context loaded with `old` to `new` (same nodes, same dictionaries; bound pods
    added or removed): overwrite the node rows whose requested / non-zero / pod count
    changed, add the class / term count differences, overwrite changed UsedPorts.  Returns
    the number of rows / cells sent."""
    if old.node_names != new.node_names or old.classes != new.classes or old.terms != new.terms \
            or old.ports != new.ports or old.scalars != new.scalars:
        raise ValueError("sync_deltas needs the same nodes and dictionaries; reload the cluster instead")
    a, b = old.arrays, new.arrays
    N = new.n_nodes
    changed = np.zeros(N, bool)
    changed |= (a["requested"][:, :N] != b["requested"][:, :N]).any(axis=0)
    changed |= (a["nonzero"][:, :N] != b["nonzero"][:, :N]).any(axis=0)
    changed |= a["pod_count"][:N] != b["pod_count"][:N]
    idx = np.nonzero(changed)[0].astype(np.int32)
    if len(idx):
        ctx.apply_node_delta(idx, b["requested"][:, idx].T, b["nonzero"][:, idx].T, b["pod_count"][idx])
    nodes, rows, vals = [], [], []
    nc = len(new.classes)
    for off, key, nrow in ((0, "class_count", nc), (nc, "term_count", len(new.terms))):
        if nrow == 0:
            continue
        d = b[key][:nrow, :N].astype(np.int64) - a[key][:nrow, :N].astype(np.int64)
        r, n = np.nonzero(d)
        rows.extend((r + off).tolist())
        nodes.extend(n.tolist())
        vals.extend(d[r, n].tolist())
    if nodes:
        ctx.apply_count_delta(nodes, rows, vals)
    pidx = np.nonzero(a["port_used"][:N] != b["port_used"][:N])[0].astype(np.int32)
    if len(pidx):
        ctx.apply_port_delta(pidx, b["port_used"][pidx])
    return {"rows": int(len(idx)), "count_cells": len(nodes), "port_rows": int(len(pidx))}
