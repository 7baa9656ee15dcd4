"""Host-side compiler: Kubernetes objects -> the packed SoA the C ABI consumes.

This is the host glue a cgo plugin would run at PreFilter time:
it interns strings (label keys/values, taints, pod label classes, affinity term
types) into dense ids and compiles each pod into a fixed ``kss_pod`` record plus
pool entries.  Objects are k8s-shaped dicts (``metadata``/``spec``/``status``),
so fixtures read like the reference's own YAML (web/components/lib/templates).

Upstream semantics restated here (k8s.io/kubernetes v1.26.2, not vendored):
  * node order: internal/cache nodeTree.list() zone round-robin, utilnode.GetZoneKey
  * requests: noderesources.computePodResourceRequest, resource_allocation
    calculatePodResourceRequest, framework.calculateResource, schedutil.GetRequestForResource
  * taints: v1helper.TolerationsTolerateTaint / Toleration.ToleratesTaint
  * node affinity: component-helpers nodeaffinity (GetRequiredNodeAffinity,
    NewLazyErrorNodeSelector, NewPreferredSchedulingTerms, nodeSelectorRequirementsAsSelector)
  * topology spread: filterTopologySpreadConstraints / buildDefaultConstraints
  * inter-pod affinity: framework.NewPodInfo affinity terms, AffinityTerm.Matches,
    mergeAffinityTermNamespacesIfNotEmpty
  * volumes: kss/volumes.py (VolumeRestrictions, the attach-limit plugins, VolumeBinding,
    VolumeZone) from the snapshot's PVs, claims, StorageClasses and CSINodes
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .quantity import milli_value, value
from .selectors import (EVERYTHING, NOTHING, Selector, SelectorError, label_selector_as_selector, parse_int,
                        selector_from_set)

LABEL_HOSTNAME = "kubernetes.io/hostname"
LABEL_ZONE = "topology.kubernetes.io/zone"
LABEL_REGION = "topology.kubernetes.io/region"
LABEL_ZONE_BETA = "failure-domain.beta.kubernetes.io/zone"
LABEL_REGION_BETA = "failure-domain.beta.kubernetes.io/region"
TAINT_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"
DEFAULT_SPREAD_SELECTOR_ANN = "kss.x-k8s.io/default-spread-selector"  # stands in for helper.DefaultSelector

DEFAULT_MILLI_CPU = 100               # schedutil.DefaultMilliCPURequest
DEFAULT_MEMORY = 200 * 1024 * 1024    # schedutil.DefaultMemoryRequest

NATIVE_RESOURCES = ("cpu", "memory", "ephemeral-storage", "pods")


class CompileError(ValueError):
    pass


class Unsupported(CompileError):
    pass


# ---------------------------------------------------------------------------
# small helpers over k8s-shaped dicts
# ---------------------------------------------------------------------------
def meta(o) -> dict:
    return o.get("metadata") or {}


def spec(o) -> dict:
    return o.get("spec") or {}


def labels_of(o) -> Dict[str, str]:
    return dict(meta(o).get("labels") or {})


def name_of(o) -> str:
    return meta(o).get("name", "")


def ns_of(o) -> str:
    return meta(o).get("namespace") or "default"


def zone_key(node) -> str:
    """utilnode.GetZoneKey."""
    lb = labels_of(node)
    zone = lb.get(LABEL_ZONE_BETA, lb.get(LABEL_ZONE, ""))
    region = lb.get(LABEL_REGION_BETA, lb.get(LABEL_REGION, ""))
    if region == "" and zone == "":
        return ""
    return region + ":\x00:" + zone


def pod_priority(p) -> int:
    """corev1helpers.PodPriority: spec.priority (the Priority admission plugin resolves
    priorityClassName into it), 0 when unset."""
    v = spec(p).get("priority")
    if v is None:
        return 0
    v = int(v)
    if not -(2**31) <= v < 2**31:
        raise CompileError(f"priority {v} out of int32 range")
    return v


def pod_start(p) -> int:
    """status.startTime (RFC 3339, seconds) as Unix nanoseconds; KSS_START_UNSET when unset
    (GetPodStartTime falls back to time.Now(): later than any recorded start)."""
    st = (p.get("status") or {}).get("startTime")
    if not st:
        return abi.KSS_START_UNSET
    from datetime import datetime, timezone
    t = datetime.strptime(st, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=timezone.utc)
    return int(t.timestamp()) * 10**9


def node_tree_order(nodes: Sequence[dict]) -> List[int]:
    """internal/cache nodeTree: zones in first-seen order, round-robin, insertion order within a zone."""
    zones: List[str] = []
    tree: Dict[str, List[int]] = {}
    for i, n in enumerate(nodes):
        z = zone_key(n)
        if z not in tree:
            tree[z] = []
            zones.append(z)
        tree[z].append(i)
    out: List[int] = []
    idx = 0
    while len(out) < len(nodes):
        for z in zones:
            if idx < len(tree[z]):
                out.append(tree[z][idx])
        idx += 1
    return out


def is_scalar_resource_name(name: str) -> bool:
    """schedutil/v1helper IsScalarResourceName: extended, hugepages-, attachable-volumes-."""
    if name in NATIVE_RESOURCES:
        return False
    if name.startswith("hugepages-") or name.startswith("attachable-volumes-"):
        return True
    # IsExtendedResourceName: fully-qualified, not in the kubernetes.io namespace, not requests.*
    if "/" not in name:
        return False
    if name.startswith("requests."):
        return False
    domain = name.split("/", 1)[0]
    return not (domain == "kubernetes.io" or domain.endswith(".kubernetes.io"))


def tolerates(tol: dict, key: str, value: str, effect: str) -> bool:
    """v1.Toleration.ToleratesTaint."""
    te = tol.get("effect") or ""
    if te and te != effect:
        return False
    tk = tol.get("key") or ""
    if tk and tk != key:
        return False
    op = tol.get("operator") or ""
    if op in ("", "Equal"):
        return (tol.get("value") or "") == value
    if op == "Exists":
        return True
    return False


def tolerations_tolerate(tols, key, value, effect) -> bool:
    return any(tolerates(t, key, value, effect) for t in (tols or []))


# ---------------------------------------------------------------------------
# pod requests
# ---------------------------------------------------------------------------
def _requests(c) -> dict:
    return ((c.get("resources") or {}).get("requests")) or {}


def _q(res: dict, name: str, milli: bool) -> int:
    return milli_value(res[name]) if milli else value(res[name])


def resource_add(vec: List[int], res: dict, scalars: List[str]):
    """framework.Resource.Add (cpu MilliValue, others Value)."""
    for name, q in res.items():
        if name == "cpu":
            vec[0] += milli_value(q)
        elif name == "memory":
            vec[1] += value(q)
        elif name == "ephemeral-storage":
            vec[2] += value(q)
        elif name in scalars:
            vec[3 + scalars.index(name)] += value(q)


def resource_set_max(vec: List[int], res: dict, scalars: List[str]):
    """framework.Resource.SetMaxResource."""
    for name, q in res.items():
        if name == "cpu":
            vec[0] = max(vec[0], milli_value(q))
        elif name == "memory":
            vec[1] = max(vec[1], value(q))
        elif name == "ephemeral-storage":
            vec[2] = max(vec[2], value(q))
        elif name in scalars:
            i = 3 + scalars.index(name)
            vec[i] = max(vec[i], value(q))


def compute_pod_resource_request(pod, scalars) -> List[int]:
    """noderesources.computePodResourceRequest (== calculateResource's Resource part)."""
    vec = [0] * abi.KSS_NRES
    sp = spec(pod)
    for c in sp.get("containers") or []:
        resource_add(vec, _requests(c), scalars)
    for c in sp.get("initContainers") or []:
        resource_set_max(vec, _requests(c), scalars)
    if sp.get("overhead"):
        resource_add(vec, sp["overhead"], scalars)
    return vec


def get_request_for_resource(r: int, res: dict, non_zero: bool, scalars) -> int:
    """schedutil.GetRequestForResource."""
    if r == 0:
        if "cpu" not in res and non_zero:
            return DEFAULT_MILLI_CPU
        return milli_value(res["cpu"]) if "cpu" in res else 0
    if r == 1:
        if "memory" not in res and non_zero:
            return DEFAULT_MEMORY
        return value(res["memory"]) if "memory" in res else 0
    if r == 2:
        return value(res["ephemeral-storage"]) if "ephemeral-storage" in res else 0
    s = r - 3
    if s < len(scalars) and scalars[s] in res:
        return value(res[scalars[s]])
    return 0


def calculate_pod_resource_request(pod, r: int, non_zero: bool, scalars) -> int:
    """resource_allocation.go calculatePodResourceRequest (v1.26: overhead adds quantity.Value())."""
    sp = spec(pod)
    req = 0
    for c in sp.get("containers") or []:
        req += get_request_for_resource(r, _requests(c), non_zero, scalars)
    for c in sp.get("initContainers") or []:
        v = get_request_for_resource(r, _requests(c), non_zero, scalars)
        if req < v:
            req = v
    oh = sp.get("overhead")
    if oh:
        nm = _resource_name(r, scalars)
        if nm in oh:
            req += value(oh[nm])
    return req


def _resource_name(r: int, scalars) -> str:
    return ("cpu", "memory", "ephemeral-storage")[r] if r < 3 else (scalars[r - 3] if r - 3 < len(scalars) else "")


def calculate_nonzero(pod) -> Tuple[int, int]:
    """framework.calculateResource non0CPU / non0Mem."""
    sp = spec(pod)
    c0 = m0 = 0
    for c in sp.get("containers") or []:
        res = _requests(c)
        c0 += get_request_for_resource(0, res, True, [])
        m0 += get_request_for_resource(1, res, True, [])
    for c in sp.get("initContainers") or []:
        res = _requests(c)
        c0 = max(c0, get_request_for_resource(0, res, True, []))
        m0 = max(m0, get_request_for_resource(1, res, True, []))
    oh = sp.get("overhead")
    if oh:
        if "cpu" in oh:
            c0 += milli_value(oh["cpu"])
        if "memory" in oh:
            m0 += value(oh["memory"])
    return c0, m0


# ---------------------------------------------------------------------------
# affinity terms
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class AffinityTerm:
    """framework.AffinityTerm after NewPodInfo (and, for incoming pods, namespace merging)."""

    namespaces: frozenset
    selector: Selector
    ns_selector: Selector
    topology_key: str

    def matches(self, ns: str, pod_labels: Dict[str, str], ns_labels: Optional[Dict[str, str]]) -> bool:
        """AffinityTerm.Matches."""
        if ns in self.namespaces or self.ns_selector.matches(ns_labels if ns_labels is not None else {}):
            return self.selector.matches(pod_labels)
        return False

    def canonical(self) -> str:
        return "|".join([",".join(sorted(self.namespaces)), self.selector.canonical(), self.ns_selector.canonical(),
                         self.topology_key])


def new_affinity_term(pod, term: dict) -> AffinityTerm:
    """framework.newAffinityTerm + getNamespacesFromPodAffinityTerm."""
    sel = label_selector_as_selector(term.get("labelSelector"))
    nsl = term.get("namespaces") or []
    nssel_raw = term.get("namespaceSelector")
    if len(nsl) == 0 and nssel_raw is None:
        names = frozenset([ns_of(pod)])
    else:
        names = frozenset(nsl)
    nssel = label_selector_as_selector(nssel_raw)
    return AffinityTerm(names, sel, nssel, term.get("topologyKey", ""))


def pod_affinity_terms(pod):
    """(required affinity, required anti, preferred affinity [(w,term)], preferred anti [(w,term)])."""
    aff = spec(pod).get("affinity") or {}
    pa = aff.get("podAffinity") or {}
    pn = aff.get("podAntiAffinity") or {}
    ra = [new_affinity_term(pod, t) for t in pa.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
    rn = [new_affinity_term(pod, t) for t in pn.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
    wa = [(int(w["weight"]), new_affinity_term(pod, w["podAffinityTerm"]))
          for w in pa.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
    wn = [(int(w["weight"]), new_affinity_term(pod, w["podAffinityTerm"]))
          for w in pn.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
    return ra, rn, wa, wn


def merge_namespaces(t: AffinityTerm, namespaces: Dict[str, Dict[str, str]]) -> AffinityTerm:
    """InterPodAffinity.mergeAffinityTermNamespacesIfNotEmpty."""
    if t.ns_selector.empty():
        return t
    names = set(t.namespaces)
    for nsname, nslabels in namespaces.items():
        if t.ns_selector.matches(nslabels):
            names.add(nsname)
    return AffinityTerm(frozenset(names), t.selector, NOTHING, t.topology_key)


# ---------------------------------------------------------------------------
# the compiled cluster
def host_ports(pod) -> List[Tuple[str, str, int]]:
    """nodeports.go getContainerPorts / NodeInfo.updateUsedPorts (v1.26: spec.containers only),
    HostPortInfo.sanitize: hostIP "" -> 0.0.0.0, protocol "" -> TCP; hostPort <= 0 is ignored
    (HostPortInfo.Add / CheckConflict)."""
    out = []
    for c in spec(pod).get("containers") or []:
        for port in c.get("ports") or []:
            hp = int(port.get("hostPort") or 0)
            if hp <= 0:
                continue
            out.append((port.get("hostIP") or "0.0.0.0", port.get("protocol") or "TCP", hp))
    return out


def ports_conflict(want: Tuple[str, str, int], used: Tuple[str, str, int]) -> bool:
    """HostPortInfo.CheckConflict of one wanted port against one used entry: the same
    (protocol, port), and the wanted IP is 0.0.0.0 (checks every IP) or the used entry's IP
    is 0.0.0.0 or equal."""
    if (want[1], want[2]) != (used[1], used[2]):
        return False
    return want[0] == "0.0.0.0" or used[0] in ("0.0.0.0", want[0])


def normalized_image_name(name: str) -> str:
    """image_locality.go normalizedImageName: append ":latest" when the name has no tag."""
    if name.rfind(":") <= name.rfind("/"):
        name = name + ":latest"
    return name


def node_image_states(nodes: Sequence[dict]) -> List[Dict[str, Tuple[int, int]]]:
    """NodeInfo.ImageStates of each node (input = cache add order) as the v1.26 scheduler
    cache builds them (internal/cache/cache.go addNodeImageStates): the image's size is the
    first adding node's SizeBytes, and NumNodes is copied when the node is added
    (createImageStateSummary), i.e. the nodes listing the name among those added so far.
    [verify] against a Go build: later releases recount NumNodes at snapshot time."""
    size: Dict[str, int] = {}
    seen: Dict[str, set] = {}
    out = []
    for n in nodes:
        summ: Dict[str, Tuple[int, int]] = {}
        for image in ((n.get("status") or {}).get("images") or []):
            for nm in image.get("names") or []:
                if nm not in size:
                    size[nm] = int(image.get("sizeBytes") or 0)
                    seen[nm] = set()
                seen[nm].add(name_of(n))
                if nm not in summ:
                    summ[nm] = (size[nm], len(seen[nm]))
        out.append(summ)
    return out


# ---------------------------------------------------------------------------
@dataclass
class CompiledCluster:
    node_names: List[str]
    order: List[int]                     # canonical -> input index
    scalars: List[str]
    label_keys: List[str]
    key_values: List[List[str]]
    taints: List[Tuple[str, str, str]]
    classes: List[Tuple[str, Tuple[Tuple[str, str], ...]]]
    terms: List[Tuple[str, int, AffinityTerm]]   # (kind, weight, term)
    arrays: Dict[str, np.ndarray]
    namespaces: Dict[str, Dict[str, str]]
    bound: Dict[str, np.ndarray] = field(default_factory=dict)     # the kss_boundset arrays
    bound_names: List[Tuple[str, str]] = field(default_factory=list)  # (namespace, name) per bound id
    ports: List[Tuple[str, str, int]] = field(default_factory=list)   # host-port dictionary (ip, protocol, port)
    images: List[str] = field(default_factory=list)                   # image_score rows (image names)
    vol_rows: list = field(default_factory=list)                      # vol_count rows (volumes.VolumeCompiler.rows)
    vol_keys: List[str] = field(default_factory=list)                 # attach-limit keys
    pvs: List[str] = field(default_factory=list)                      # candidate PVs of WaitForFirstConsumer claims (pv_owner)
    wclaims: List[Tuple[str, str]] = field(default_factory=list)      # those claims (namespace, name) (claim_node)
    _keep: list = field(default_factory=list)

    @property
    def n_nodes(self) -> int:
        return len(self.node_names)

    def as_struct(self, node_base: int = 0) -> abi.Cluster:
        a = self.arrays
        c = abi.Cluster()
        c.n_ports = len(self.ports)
        c.n_images = len(self.images)
        c.port_used = abi.ptr(a["port_used"], abi.u64)
        c.image_score = abi.ptr(a["image_score"], abi.i64)
        c.n_vol_rows = len(self.vol_rows)
        c.n_vol_keys = len(self.vol_keys)
        for name in ("vol_count", "vol_attached", "vol_limit", "vol_row_key", "vol_key_plugin", "pv_owner", "claim_node"):
            setattr(c, name, abi.ptr(a[name], abi.i32))
        c.n_pvs = len(self.pvs)
        c.n_wclaims = len(self.wclaims)
        c.n_nodes = self.n_nodes
        c.n_scalar = len(self.scalars)
        c.n_label_keys = len(self.label_keys)
        c.n_label_values = int(a["value_int"].shape[0])
        c.n_classes = len(self.classes)
        c.n_terms = len(self.terms)
        c.n_taints = len(self.taints)
        c.node_base = node_base
        for name, ct in (("alloc", abi.i64), ("requested", abi.i64), ("nonzero", abi.i64), ("allowed_pods", abi.i32),
                         ("pod_count", abi.i32), ("node_flags", abi.u32), ("taint_hard", abi.u64),
                         ("taint_soft", abi.u64), ("taint_order", abi.u8), ("label_value", abi.i32),
                         ("key_base", abi.i32), ("key_card", abi.i32), ("key_flags", abi.u32), ("key_empty", abi.i32),
                         ("value_int", abi.i64), ("value_is_int", abi.u8), ("class_count", abi.i32),
                         ("term_count", abi.i32)):
            setattr(c, name, abi.ptr(a[name], ct))
        return c

    def as_boundset(self) -> abi.Boundset:
        """The bound pods (NodeInfo.Pods order per node) for the PostFilter dry run."""
        b = self.bound
        s = abi.Boundset()
        s.n = len(self.bound_names)
        s.n_ints = int(sum(int(x) for x in b["terms_len"][:s.n]))
        for name, ct in (("id", abi.i64), ("node", abi.i32), ("priority", abi.i32), ("start", abi.i64),
                         ("cls", abi.i32), ("req", abi.i64), ("terms_off", abi.i32), ("terms_len", abi.i32),
                         ("ints", abi.i32), ("nonzero", abi.i64), ("ports", abi.u64)):
            setattr(s, name, abi.ptr(b[name], ct))
        return s


@dataclass
class CompiledPods:
    pods: np.ndarray
    reqs: np.ndarray
    terms: np.ndarray
    spreads: np.ndarray
    ipa: np.ndarray
    ints: np.ndarray
    names: List[Tuple[str, str]]   # (namespace, name)
    counts: Tuple[int, int, int, int, int] = (0, 0, 0, 0, 0)  # real pool sizes (arrays are padded to >= 1)
    vols: Optional[np.ndarray] = None   # kss_vol pool
    n_vols: int = 0
    messages: List[str] = field(default_factory=list)  # kss_names.messages (VolumeBinding PreFilter, VolumeZone)

    @property
    def n(self) -> int:
        return int(self.pods.shape[0])

    def as_struct(self) -> abi.PodSet:
        s = abi.PodSet()
        s.n_pods = self.n
        s.n_reqs, s.n_terms, s.n_spreads, s.n_ipa, s.n_ints = self.counts
        s.pods = self.pods.ctypes.data_as(abi.P(abi.Pod))
        s.reqs = self.reqs.ctypes.data_as(abi.P(abi.Req))
        s.terms = self.terms.ctypes.data_as(abi.P(abi.Term))
        s.spreads = self.spreads.ctypes.data_as(abi.P(abi.Spread))
        s.ipa = self.ipa.ctypes.data_as(abi.P(abi.Ipa))
        s.ints = self.ints.ctypes.data_as(abi.P(abi.i32))
        if self.vols is None:
            self.vols = np.zeros(1, dtype=abi.VOL_DTYPE)
        s.n_vols = self.n_vols
        s.vols = self.vols.ctypes.data_as(abi.P(abi.Vol))
        return s


def _nonempty(a: np.ndarray) -> np.ndarray:
    """ctypes needs a valid pointer even for empty pools."""
    if a.shape[0] == 0:
        return np.zeros(1, dtype=a.dtype)
    return np.ascontiguousarray(a)


class Compiler:
    """Compile nodes + bound pods + pending pods.

    ``nodes`` in insertion order; ``bound_pods`` carry spec.nodeName; ``pending``
    in queue order; ``namespaces`` maps namespace name -> labels.
    """

    def __init__(self, nodes: Sequence[dict], bound_pods: Sequence[dict] = (), pending: Sequence[dict] = (),
                 namespaces: Optional[Dict[str, Dict[str, str]]] = None, hard_pod_affinity_weight: int = 1,
                 system_defaulted: bool = True, device_limits: bool = True, storage: Optional[dict] = None):
        """storage: {"pvs", "pvcs", "storage_classes", "csinodes"} object lists for the volume plugins."""
        self.nodes_in = list(nodes)
        self.bound = list(bound_pods)
        self.pending = list(pending)
        self.namespaces = dict(namespaces or {})
        for p in self.bound + self.pending:
            self.namespaces.setdefault(ns_of(p), {})
        self.hard_w = hard_pod_affinity_weight
        self.system_defaulted = system_defaulted
        self.device_limits = device_limits
        self.storage = storage

    # -------------------------------------------------------------- cluster
    def compile(self) -> Tuple[CompiledCluster, CompiledPods]:
        order = node_tree_order(self.nodes_in)
        nodes = [self.nodes_in[i] for i in order]
        names = [name_of(n) for n in nodes]
        if len(set(names)) != len(names):
            raise CompileError("duplicate node names")
        self.node_index = {nm: i for i, nm in enumerate(names)}
        N = len(nodes)
        # volume programs (kss/volumes.py): built from the canonical node order and NodeInfo pods
        self.vc = None
        if self.storage or any(spec(p).get("volumes") for p in self.bound + self.pending):
            from .volumes import VolumeCompiler
            bound_on = [(p, self.node_index[spec(p).get("nodeName")]) for p in self.bound
                        if spec(p).get("nodeName") in self.node_index]
            self.vc = VolumeCompiler(self.storage, nodes, bound_on, self.pending)

        # scalar resources (sorted)
        sc = set()
        for n in nodes:
            for r in ((n.get("status") or {}).get("allocatable") or {}):
                if is_scalar_resource_name(r):
                    sc.add(r)
        for p in self.bound + self.pending:
            sp = spec(p)
            for c in (sp.get("containers") or []) + (sp.get("initContainers") or []):
                for r in _requests(c):
                    if is_scalar_resource_name(r):
                        sc.add(r)
        scalars = sorted(sc)
        if len(scalars) > abi.KSS_MAX_SCALAR:
            raise Unsupported(f"more than {abi.KSS_MAX_SCALAR} scalar resources: {scalars}")
        self.scalars = scalars

        # pod affinity terms of every pod (bound pods' terms become term types)
        self.pod_terms = {}
        for p in self.bound + self.pending:
            self.pod_terms[id(p)] = pod_affinity_terms(p)

        # referenced label keys
        keys = set()
        for p in self.bound + self.pending:
            sp = spec(p)
            keys.update((sp.get("nodeSelector") or {}).keys())
            na = ((sp.get("affinity") or {}).get("nodeAffinity")) or {}
            req = na.get("requiredDuringSchedulingIgnoredDuringExecution") or {}
            for t in req.get("nodeSelectorTerms") or []:
                for e in t.get("matchExpressions") or []:
                    keys.add(e.get("key", ""))
            for w in na.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
                for e in (w.get("preference") or {}).get("matchExpressions") or []:
                    keys.add(e.get("key", ""))
            for c in sp.get("topologySpreadConstraints") or []:
                keys.add(c.get("topologyKey", ""))
            ra, rn, wa, wn = self.pod_terms[id(p)]
            for t in ra + rn:
                keys.add(t.topology_key)
            for _, t in wa + wn:
                keys.add(t.topology_key)
            if self.system_defaulted and DEFAULT_SPREAD_SELECTOR_ANN in (meta(p).get("annotations") or {}):
                keys.update((LABEL_HOSTNAME, LABEL_ZONE))
        if self.vc is not None:
            keys.update(self.vc.label_keys())
        label_keys = sorted(keys)
        self.key_index = {k: i for i, k in enumerate(label_keys)}

        node_labels = [labels_of(n) for n in nodes]
        key_values: List[List[str]] = []
        self.value_index: List[Dict[str, int]] = []
        label_value = np.full((len(label_keys), max(N, 1)), -1, dtype=np.int32)[:, :N].copy()
        key_card = np.zeros(len(label_keys), dtype=np.int32)
        key_flags = np.zeros(len(label_keys), dtype=np.uint32)
        key_empty = np.zeros(len(label_keys), dtype=np.int32)
        key_base = np.zeros(len(label_keys), dtype=np.int32)
        vint: List[int] = []
        visint: List[int] = []
        for k, key in enumerate(label_keys):
            vals = sorted({lb[key] for lb in node_labels if key in lb})
            vi = {v: i for i, v in enumerate(vals)}
            key_values.append(vals)
            self.value_index.append(vi)
            present = 0
            for n, lb in enumerate(node_labels):
                if key in lb:
                    label_value[k, n] = vi[lb[key]]
                    present += 1
            key_card[k] = len(vals)
            key_base[k] = len(vint)
            key_empty[k] = vi.get("", len(vals))
            if present == len(vals) and "" not in vi:
                key_flags[k] |= abi.KSS_KEY_UNIQUE
            if key == LABEL_HOSTNAME:
                key_flags[k] |= abi.KSS_KEY_HOSTNAME
            for v in vals:
                iv = parse_int(v)
                vint.append(iv if iv is not None else 0)
                visint.append(1 if iv is not None else 0)
        self.key_card = key_card

        # taint dictionary
        tset = set()
        for n in nodes:
            for t in (spec(n).get("taints") or []):
                tset.add((t.get("key", ""), t.get("value") or "", t.get("effect", "")))
        taints = sorted(tset)
        if len(taints) > abi.KSS_MAX_TAINTS:
            raise Unsupported(f"more than {abi.KSS_MAX_TAINTS} distinct taints")
        tidx = {t: i for i, t in enumerate(taints)}
        self.taints = taints
        taint_hard = np.zeros(N, dtype=np.uint64)
        taint_soft = np.zeros(N, dtype=np.uint64)
        taint_order = np.full((N, abi.KSS_TAINT_ORDER), 0xFF, dtype=np.uint8)
        for i, n in enumerate(nodes):
            k = 0
            for t in (spec(n).get("taints") or []):
                tt = (t.get("key", ""), t.get("value") or "", t.get("effect", ""))
                b = np.uint64(1) << np.uint64(tidx[tt])
                if tt[2] in ("NoSchedule", "NoExecute"):
                    taint_hard[i] |= b
                    if k >= abi.KSS_TAINT_ORDER:
                        raise Unsupported(f"node {names[i]}: more than {abi.KSS_TAINT_ORDER} NoSchedule/NoExecute taints")
                    taint_order[i, k] = tidx[tt]
                    k += 1
                elif tt[2] == "PreferNoSchedule":
                    taint_soft[i] |= b

        # node resources
        alloc = np.zeros((abi.KSS_NRES, N), dtype=np.int64)
        allowed = np.zeros(N, dtype=np.int32)
        flags = np.zeros(N, dtype=np.uint32)
        for i, n in enumerate(nodes):
            al = (n.get("status") or {}).get("allocatable") or {}
            if "cpu" in al:
                alloc[0, i] = milli_value(al["cpu"])
            if "memory" in al:
                alloc[1, i] = value(al["memory"])
            if "ephemeral-storage" in al:
                alloc[2, i] = value(al["ephemeral-storage"])
            for s, nm in enumerate(scalars):
                if nm in al:
                    alloc[3 + s, i] = value(al[nm])
            allowed[i] = value(al["pods"]) if "pods" in al else 0
            if spec(n).get("unschedulable"):
                flags[i] |= abi.KSS_NODE_UNSCHEDULABLE
            if node_labels[i]:
                flags[i] |= abi.KSS_NODE_HAS_LABELS
        if self.vc is not None:
            flags |= self.vc.node_zone_flags()

        # classes and term types over all pods (bound + pending)
        cls_set = set()
        term_set = set()
        for p in self.bound + self.pending:
            cls_set.add(self._class_key(p))
            ra, rn, wa, wn = self.pod_terms[id(p)]
            for t in ra:
                term_set.add(("RA", 0, t))
            for t in rn:
                term_set.add(("RN", 0, t))
            for w, t in wa:
                term_set.add(("PA", w, t))
            for w, t in wn:
                term_set.add(("PN", w, t))
        classes = sorted(cls_set)
        self.class_index = {c: i for i, c in enumerate(classes)}
        terms = sorted(term_set, key=lambda x: (x[0], x[1], x[2].canonical()))
        self.term_index = {t: i for i, t in enumerate(terms)}
        self.classes = classes
        self.terms = terms

        requested = np.zeros((abi.KSS_NRES, N), dtype=np.int64)
        nonzero = np.zeros((2, N), dtype=np.int64)
        pod_count = np.zeros(N, dtype=np.int32)
        class_count = np.zeros((len(classes), N), dtype=np.int32)
        term_count = np.zeros((len(terms), N), dtype=np.int32)
        bt = dict(id=[], node=[], priority=[], start=[], cls=[], req=[], terms_off=[], terms_len=[], ints=[], nz=[])
        bound_names = []
        for p in self.bound:
            nn = spec(p).get("nodeName")
            if nn not in self.node_index:
                continue  # pods bound to unknown nodes are not in any NodeInfo
            i = self.node_index[nn]
            req = compute_pod_resource_request(p, scalars)
            own = self._own_terms(p)
            bt["id"].append(len(bound_names))
            bt["node"].append(i)
            bt["priority"].append(pod_priority(p))
            bt["start"].append(pod_start(p))
            bt["cls"].append(self.class_index[self._class_key(p)])
            bt["req"].append(req)
            bt["terms_off"].append(len(bt["ints"]))
            bt["terms_len"].append(len(own))
            bt["ints"].extend(own)
            bound_names.append((ns_of(p), name_of(p)))
            requested[:, i] += np.array(req, dtype=np.int64)
            c0, m0 = calculate_nonzero(p)
            bt["nz"].append((c0, m0))
            nonzero[0, i] += c0
            nonzero[1, i] += m0
            pod_count[i] += 1
            class_count[self.class_index[self._class_key(p)], i] += 1
            for t in self._own_terms(p):
                term_count[t, i] += 1

        # NodePorts: the host-port dictionary over NodeInfo.UsedPorts and the pending pods' ports
        pset = set()
        for p in self.bound:
            if spec(p).get("nodeName") in self.node_index:
                pset.update(host_ports(p))
        for p in self.pending:
            pset.update(host_ports(p))
        ports = sorted(pset)
        if len(ports) > abi.KSS_MAX_PORTS:
            raise Unsupported(f"more than {abi.KSS_MAX_PORTS} distinct host ports")
        self.ports = ports
        self.port_index = {e: i for i, e in enumerate(ports)}
        port_used = np.zeros(N, dtype=np.uint64)
        bound_ports = []  # per table row (the bound pods on known nodes, in order)
        for p in self.bound:
            nn = spec(p).get("nodeName")
            if nn in self.node_index:
                bits = np.uint64(0)
                for e in host_ports(p):
                    bits |= np.uint64(1) << np.uint64(self.port_index[e])
                port_used[self.node_index[nn]] |= bits
                bound_ports.append(bits)
        # ImageLocality: rows for the normalized container images of pending pods that some
        # node lists; scaledImageScore per (row, node) with totalNumNodes = N
        states = node_image_states(self.nodes_in)
        canon_states = [states[i] for i in order]
        listed = set().union(*[set(st) for st in states]) if states else set()
        want = set()
        for p in self.pending:
            for c in spec(p).get("containers") or []:
                nm = normalized_image_name(c.get("image") or "")
                if nm in listed:
                    want.add(nm)
        images = sorted(want)
        self.images = images
        self.image_index = {nm: i for i, nm in enumerate(images)}
        image_score = np.zeros((len(images), N), dtype=np.int64)
        for r, nm in enumerate(images):
            for i, st in enumerate(canon_states):
                if nm in st:
                    sz, num = st[nm]
                    image_score[r, i] = int(float(sz) * (float(num) / float(N)))  # scaledImageScore

        vc = self.vc
        arrays = dict(alloc=alloc, requested=requested, nonzero=nonzero, allowed_pods=allowed, pod_count=pod_count,
                      node_flags=flags, taint_hard=taint_hard, taint_soft=taint_soft, taint_order=taint_order,
                      label_value=label_value, key_base=key_base, key_card=key_card, key_flags=key_flags,
                      key_empty=key_empty, value_int=np.array(vint, dtype=np.int64),
                      value_is_int=np.array(visint, dtype=np.uint8), class_count=class_count, term_count=term_count,
                      port_used=port_used, image_score=image_score,
                      vol_count=vc.vol_count if vc else np.zeros((0, N), np.int32),
                      vol_attached=vc.vol_attached if vc else np.zeros((0, N), np.int32),
                      vol_limit=vc.vol_limit if vc else np.zeros((0, N), np.int32),
                      vol_row_key=vc.vol_row_key if vc else np.zeros(0, np.int32),
                      vol_key_plugin=vc.vol_key_plugin if vc else np.zeros(0, np.int32),
                      pv_owner=vc.pv_owner if vc else np.zeros(0, np.int32),
                      claim_node=vc.claim_node if vc else np.zeros(0, np.int32))
        arrays = {k: (np.zeros(1, dtype=v.dtype) if v.size == 0 else np.ascontiguousarray(v))
                  for k, v in arrays.items()}
        nb = len(bound_names)
        bound = dict(id=np.array(bt["id"], dtype=np.int64), node=np.array(bt["node"], dtype=np.int32),
                     priority=np.array(bt["priority"], dtype=np.int32), start=np.array(bt["start"], dtype=np.int64),
                     cls=np.array(bt["cls"], dtype=np.int32),
                     req=np.ascontiguousarray(np.array(bt["req"], dtype=np.int64).reshape(nb, abi.KSS_NRES).T),
                     terms_off=np.array(bt["terms_off"], dtype=np.int32),
                     terms_len=np.array(bt["terms_len"], dtype=np.int32), ints=np.array(bt["ints"], dtype=np.int32),
                     nonzero=np.ascontiguousarray(np.array(bt["nz"], dtype=np.int64).reshape(nb, 2).T),
                     ports=np.array(bound_ports, dtype=np.uint64))
        bound = {k: (np.zeros(1, dtype=v.dtype) if v.size == 0 else np.ascontiguousarray(v)) for k, v in bound.items()}
        self.cc = CompiledCluster(node_names=names, order=order, scalars=scalars, label_keys=label_keys,
                                  key_values=key_values, taints=taints, classes=classes, terms=terms, arrays=arrays,
                                  namespaces=self.namespaces, bound=bound, bound_names=bound_names, ports=ports,
                                  images=images, vol_rows=list(vc.rows) if vc else [], vol_keys=list(vc.keys) if vc else [],
                                  pvs=list(vc.pv_names) if vc else [],
                                  wclaims=[vc.claim_key(pvc) for pvc in vc.wclaims] if vc else [])
        self.node_labels = node_labels
        self.key_flags = key_flags
        pods = self._compile_pods(self.pending)
        return self.cc, pods

    def _class_key(self, p):
        return (ns_of(p), tuple(sorted(labels_of(p).items())))

    def _own_terms(self, p) -> List[int]:
        ra, rn, wa, wn = self.pod_terms[id(p)]
        out = [self.term_index[("RA", 0, t)] for t in ra]
        out += [self.term_index[("RN", 0, t)] for t in rn]
        out += [self.term_index[("PA", w, t)] for w, t in wa]
        out += [self.term_index[("PN", w, t)] for w, t in wn]
        return out

    # -------------------------------------------------------------- pods
    def _compile_pods(self, pods: Sequence[dict]) -> CompiledPods:
        self._reqs: List[tuple] = []
        self._terms: List[tuple] = []
        self._spreads: List[tuple] = []
        self._ipa: List[tuple] = []
        self._ints: List[int] = []
        self._vols: List[tuple] = []
        recs = np.zeros(len(pods), dtype=abi.POD_DTYPE)
        names = []
        for i, p in enumerate(pods):
            self._compile_pod(p, recs[i])
            self._compile_volumes(i, recs[i])
            names.append((ns_of(p), name_of(p)))

        def arr(rows, dt):
            a = np.zeros(len(rows), dtype=dt)
            for j, r in enumerate(rows):
                a[j] = r
            return _nonempty(a)

        return CompiledPods(pods=recs, reqs=arr(self._reqs, abi.REQ_DTYPE), terms=arr(self._terms, abi.TERM_DTYPE),
                            spreads=arr(self._spreads, abi.SPREAD_DTYPE), ipa=arr(self._ipa, abi.IPA_DTYPE),
                            ints=_nonempty(np.array(self._ints, dtype=np.int32)), names=names,
                            counts=(len(self._reqs), len(self._terms), len(self._spreads), len(self._ipa),
                                    len(self._ints)),
                            vols=arr(self._vols, abi.VOL_DTYPE), n_vols=len(self._vols),
                            messages=list(self.vc.messages) if self.vc else [])

    def _list(self, vals: Sequence[int]) -> Tuple[int, int]:
        off = len(self._ints)
        self._ints.extend(int(v) for v in vals)
        return off, len(vals)

    def _req(self, key: str, op: str, vals: Sequence[str]) -> tuple:
        """Compile one NodeSelectorRequirement / label requirement into a kss_req row.

        Raises SelectorError for what labels.NewRequirement rejects."""
        if op in ("In", "NotIn", "="):
            if len(vals) == 0:
                raise SelectorError("values set can't be empty")
        elif op in ("Exists", "DoesNotExist"):
            if len(vals) != 0:
                raise SelectorError("values set must be empty")
        elif op in ("Gt", "Lt"):
            if len(vals) != 1 or parse_int(vals[0]) is None:
                raise SelectorError("for 'Gt', 'Lt' operators, exactly one integer value is required")
        else:
            raise SelectorError(f"{op} is not a valid node selector operator")
        k = self.key_index[key]
        vi = self.value_index[k]
        card = int(self.key_card[k])
        if op == "=":
            op = "In"
        if card <= 62:
            values = self.cc_values(k)
            mask = 0
            for j, v in enumerate(values):
                if requirement_on_value(op, vals, v):
                    mask |= 1 << j
            if requirement_on_value(op, vals, None):
                mask |= 1 << 63
            return (k, abi.KSS_OP_MASK, 0, 0, mask, 0)
        if op in ("In", "NotIn"):
            ids = sorted({vi[v] for v in vals if v in vi})
            off, ln = self._list(ids)
            return (k, abi.KSS_OP_IN if op == "In" else abi.KSS_OP_NOTIN, off, ln, 0, 0)
        if op == "Exists":
            return (k, abi.KSS_OP_EXISTS, 0, 0, 0, 0)
        if op == "DoesNotExist":
            return (k, abi.KSS_OP_DNE, 0, 0, 0, 0)
        return (k, abi.KSS_OP_GT if op == "Gt" else abi.KSS_OP_LT, 0, 0, 0, parse_int(vals[0]))

    def cc_values(self, k: int) -> List[str]:
        return sorted(self.value_index[k], key=lambda v: self.value_index[k][v])

    def _field_req(self, key: str, op: str, vals: Sequence[str]) -> tuple:
        """nodeSelectorRequirementsAsFieldSelector over {metadata.name: node.Name}."""
        if op not in ("In", "NotIn"):
            raise SelectorError("not a valid field selector operator")
        if len(vals) != 1:
            raise SelectorError("must have one element")
        if key != "metadata.name":
            # fields.Set{"metadata.name": name}.Get(key) == "" for any other key
            eq = vals[0] == ""
            res = eq if op == "In" else not eq
            return (0, abi.KSS_OP_TRUE if res else abi.KSS_OP_FALSE, 0, 0, 0, 0)
        idx = self.node_index.get(vals[0], -1)
        return (0, abi.KSS_OP_NAME_IN if op == "In" else abi.KSS_OP_NAME_NOTIN, 0, 0, 0, idx)

    def _term(self, term: dict, weight: int) -> Optional[tuple]:
        """newNodeSelectorTerm; returns None for an empty term (skipped by the parser)."""
        me = term.get("matchExpressions") or []
        mf = term.get("matchFields") or []
        if not me and not mf:
            return None
        off = len(self._reqs)
        rows = []
        try:
            for e in me:
                rows.append(self._req(e.get("key", ""), e.get("operator", ""), tuple(e.get("values") or ())))
            for e in mf:
                rows.append(self._field_req(e.get("key", ""), e.get("operator", ""), tuple(e.get("values") or ())))
        except SelectorError:
            rows = [(0, abi.KSS_OP_FALSE, 0, 0, 0, 0)]  # a term with parse errors never matches
        self._reqs.extend(rows)
        return (off, len(rows), weight, 0)

    def _pv_term(self, term: dict) -> Optional[tuple]:
        """A PersistentVolume's required node-affinity term as CheckNodeAffinity evaluates it:
        MatchNodeSelectorTerms against a node carrying only the labels, so matchFields never
        constrain (nodeSelectorTerm.match skips them on empty fields); their parse errors
        still void the term."""
        me = term.get("matchExpressions") or []
        mf = term.get("matchFields") or []
        if not me and not mf:
            return None
        off = len(self._reqs)
        rows = []
        try:
            for e in me:
                rows.append(self._req(e.get("key", ""), e.get("operator", ""), tuple(e.get("values") or ())))
            for e in mf:
                self._field_req(e.get("key", ""), e.get("operator", ""), tuple(e.get("values") or ()))
        except SelectorError:
            rows = [(0, abi.KSS_OP_FALSE, 0, 0, 0, 0)]
        if not rows:
            rows = [(0, abi.KSS_OP_TRUE, 0, 0, 0, 0)]
        self._reqs.extend(rows)
        return (off, len(rows), 0, 0)

    def _compile_volumes(self, j: int, rec):
        """The pod's VolumeBinding PreFilter status and its volume program (kss/volumes.py)."""
        rec["vol_off"], rec["vol_len"] = len(self._vols), 0
        if self.vc is None:
            return
        msg, _ = self.vc.prefilter(j)
        # RunPreFilterPlugins order: NodeAffinity's conflict comes first; a NodeAffinity parse
        # error of a preferred term surfaces only at PreScore, after this PreFilter
        if msg is not None and rec["prefilter_status"] != abi.KSS_PF_NODE_AFFINITY_CONFLICT:
            rec["prefilter_status"] = abi.KSS_PF_VOLUME_BINDING
            rec["prefilter_msg"] = self.vc.message(msg)

        def pv_terms(terms):
            off = len(self._terms)
            for t in terms:
                tt = self._pv_term(t)
                if tt is not None:
                    self._terms.append(tt)
            return off, len(self._terms) - off

        def zone_reqs(cons):
            off = len(self._reqs)
            for key, vals in cons:
                self._reqs.append(self._req(key, "In", tuple(vals)))
            return off, len(self._reqs) - off

        prog = self.vc.program(j, pv_terms, zone_reqs, self._list)
        self._vols.extend(prog)
        rec["vol_len"] = len(prog)

    def _classes_matching(self, pred) -> List[int]:
        return [i for i, (ns, lb) in enumerate(self.classes) if pred(ns, dict(lb))]

    def _compile_pod(self, p, rec):
        sp = spec(p)
        ns = ns_of(p)
        plabels = labels_of(p)
        # NodePorts PreFilter (getContainerPorts) and the pod's own UsedPorts entries
        conflict = add = 0
        for w in host_ports(p):
            add |= 1 << self.port_index[w]
            for e, j in self.port_index.items():
                if ports_conflict(w, e):
                    conflict |= 1 << j
        rec["port_conflict"] = conflict
        rec["port_add"] = add
        # ImageLocality: one image_score row per container whose normalized image a node lists
        conts = sp.get("containers") or []
        rows = [self.image_index[nm] for nm in (normalized_image_name(c.get("image") or "") for c in conts)
                if nm in self.image_index]
        rec["n_containers"] = len(conts)
        rec["img_off"], rec["img_len"] = self._list(rows) if rows else (0, 0)
        scal = self.scalars
        rec["fit_request"][:] = compute_pod_resource_request(p, scal)
        rec["commit_req"][:] = rec["fit_request"]
        for r in range(abi.KSS_NRES):
            rec["score_req_nz"][r] = calculate_pod_resource_request(p, r, True, scal)
            rec["score_req"][r] = calculate_pod_resource_request(p, r, False, scal)
        rec["commit_nz"][:] = calculate_nonzero(p)
        tols = sp.get("tolerations") or []
        th = ts = 0
        for j, (k, v, e) in enumerate(self.taints):
            if e in ("NoSchedule", "NoExecute") and tolerations_tolerate(tols, k, v, e):
                th |= 1 << j
            if e == "PreferNoSchedule":
                # getAllTolerationPreferNoSchedule: tolerations with effect "" or PreferNoSchedule
                pns = [t for t in tols if (t.get("effect") or "") in ("", "PreferNoSchedule")]
                if tolerations_tolerate(pns, k, v, e):
                    ts |= 1 << j
        rec["tol_hard"] = th
        rec["tol_soft"] = ts
        flags = 0
        if tolerations_tolerate(tols, TAINT_UNSCHEDULABLE, "", "NoSchedule"):
            flags |= abi.KSS_POD_TOL_UNSCHEDULABLE
        nn = sp.get("nodeName") or ""
        rec["node_name"] = -1 if nn == "" else self.node_index.get(nn, -2)
        rec["prefilter_status"] = 0
        rec["names_off"], rec["names_len"] = 0, -1

        # nodeSelector (labels.SelectorFromSet)
        rec["sel_off"] = len(self._reqs)
        sel = sp.get("nodeSelector") or {}
        for k, v in sel.items():
            self._reqs.append(self._req(k, "In", (v,)))
        rec["sel_len"] = len(self._reqs) - rec["sel_off"]

        na = ((sp.get("affinity") or {}).get("nodeAffinity")) or {}
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
        rec["aff_off"] = len(self._terms)
        if req is not None:
            flags |= abi.KSS_POD_HAS_REQ_AFFINITY
            for t in req.get("nodeSelectorTerms") or []:
                tr = self._term(t, 0)
                if tr is not None:
                    self._terms.append(tr)
            # NodeAffinity.PreFilter: PreFilterResult when every term names nodes via metadata.name In
            nodenames = None
            for t in req.get("nodeSelectorTerms") or []:
                tn = None
                for r in t.get("matchFields") or []:
                    if r.get("key") == "metadata.name" and r.get("operator") == "In":
                        s = set(r.get("values") or [])
                        tn = s if tn is None else (tn & s)
                if tn is None:
                    nodenames = None
                    break
                if len(tn) == 0:
                    rec["prefilter_status"] = 1  # errReasonConflict
                    nodenames = None
                    break
                nodenames = tn if nodenames is None else (nodenames | tn)
            if nodenames:
                missing = sorted(n for n in nodenames if n not in self.node_index)
                if missing:
                    # findNodesThatFitPod: NodeInfos().Get(name) fails -> a scheduling error, not a FitError
                    raise Unsupported(f"PreFilterResult names nodes absent from the snapshot: {missing[:3]}")
                idx = sorted(self.node_index[n] for n in nodenames)
                rec["names_off"], rec["names_len"] = self._list(idx)
        rec["aff_len"] = len(self._terms) - rec["aff_off"]

        rec["pref_off"] = len(self._terms)
        for w in na.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
            wt = int(w.get("weight", 0))
            pref = w.get("preference") or {}
            if wt == 0:
                continue
            tr = self._term(pref, wt)
            if tr is not None:
                if self._reqs[tr[0]][1] == abi.KSS_OP_FALSE and tr[1] == 1 and _term_has_error(pref):
                    rec["prefilter_status"] = 2  # preferred-term parse error -> framework Error
                self._terms.append(tr)
        rec["pref_len"] = len(self._terms) - rec["pref_off"]

        self._compile_spread(p, rec)
        flags |= self._spread_flags
        self._compile_ipa(p, rec)
        flags |= self._ipa_flags
        if (spec(p).get("preemptionPolicy") or "") == "Never":
            flags |= abi.KSS_POD_PREEMPT_NEVER
        rec["priority"] = pod_priority(p)
        rec["flags"] = flags
        rec["cls"] = self.class_index[self._class_key(p)]
        own = self._own_terms(p)
        rec["own_terms_off"], rec["own_terms_len"] = self._list(own)

    def _spread_classes(self, ns: str, sel: Selector) -> List[int]:
        if sel.empty():
            return []  # countPodsMatchSelector: selector.Empty() -> 0
        return self._classes_matching(lambda cns, lb: cns == ns and sel.matches(lb))

    def _compile_spread(self, p, rec):
        sp = spec(p)
        ns = ns_of(p)
        plabels = labels_of(p)
        cons = sp.get("topologySpreadConstraints") or []
        self._spread_flags = abi.KSS_POD_PTS_SCORE_STATE
        hard, soft = [], []
        if cons:
            self._spread_flags |= abi.KSS_POD_PTS_REQUIRE_ALL
            for c in cons:
                try:
                    sel = label_selector_as_selector(c.get("labelSelector"))
                except SelectorError as exc:
                    raise CompileError(f"bad spread selector: {exc}") from exc
                ent = (c.get("topologyKey", ""), int(c.get("maxSkew", 1)), sel, c.get("nodeAffinityPolicy"),
                       c.get("nodeTaintsPolicy"))
                if c.get("whenUnsatisfiable") == "DoNotSchedule":
                    hard.append(ent)
                elif c.get("whenUnsatisfiable") == "ScheduleAnyway":
                    soft.append(ent)
        else:
            if not self.system_defaulted:
                self._spread_flags |= abi.KSS_POD_PTS_REQUIRE_ALL
            ann = (meta(p).get("annotations") or {}).get(DEFAULT_SPREAD_SELECTOR_ANN)
            if self.system_defaulted and ann:
                import json
                sel = label_selector_as_selector(json.loads(ann))
                if not sel.empty():
                    soft = [(LABEL_HOSTNAME, 3, sel, None, None), (LABEL_ZONE, 5, sel, None, None)]
        if len(hard) > 8 or len(soft) > 8:
            raise Unsupported("more than 8 spread constraints per kind")
        rec["spread_off"] = len(self._spreads)
        for key, skew, sel, nap, ntp in hard + soft:
            fl = 0
            if (nap or "Honor") == "Honor":
                fl |= abi.KSS_SPREAD_POLICY_AFFINITY_HONOR
            if (ntp or "Ignore") == "Honor":
                fl |= abi.KSS_SPREAD_POLICY_TAINTS_HONOR
            off, ln = self._list(self._spread_classes(ns, sel))
            self._spreads.append((self.key_index[key], skew, 1 if sel.matches(plabels) else 0, fl, off, ln, 1, 0))
        rec["n_hard"] = len(hard)
        rec["n_soft"] = len(soft)

    def _compile_ipa(self, p, rec):
        ns = ns_of(p)
        plabels = labels_of(p)
        nslabels = self.namespaces.get(ns, {})
        ra, rn, wa, wn = self.pod_terms[id(p)]
        ra = [merge_namespaces(t, self.namespaces) for t in ra]
        rn = [merge_namespaces(t, self.namespaces) for t in rn]
        wa = [(w, merge_namespaces(t, self.namespaces)) for w, t in wa]
        wn = [(w, merge_namespaces(t, self.namespaces)) for w, t in wn]
        self._ipa_flags = 0
        rec["ipa_off"] = len(self._ipa)
        # existing pods' required anti-affinity terms that match the incoming pod, grouped by key
        by_key: Dict[int, List[int]] = {}
        for tid, (kind, w, t) in enumerate(self.terms):
            if kind == "RN" and t.matches(ns, plabels, nslabels):
                by_key.setdefault(self.key_index[t.topology_key], []).append(tid)
        for k in sorted(by_key):
            off, ln = self._list(by_key[k])
            self._ipa.append((abi.KSS_IPA_EXISTING_ANTI, k, off, ln, 0, 0))
        # incoming required affinity: classes matching ALL terms (with nil nsLabels)
        if ra:
            allc = self._classes_matching(lambda cns, lb: all(t.matches(cns, lb, None) for t in ra))
            off, ln = self._list(allc)
            for t in ra:
                self._ipa.append((abi.KSS_IPA_REQ_AFFINITY, self.key_index[t.topology_key], off, ln, 0, 0))
            if all(t.matches(ns, plabels, None) for t in ra):
                self._ipa_flags |= abi.KSS_POD_IPA_SELF_MATCH
        for t in rn:
            off, ln = self._list(self._classes_matching(lambda cns, lb, t=t: t.matches(cns, lb, None)))
            self._ipa.append((abi.KSS_IPA_REQ_ANTI, self.key_index[t.topology_key], off, ln, 0, 0))
        # scoring (InterPodAffinity.PreScore / processExistingPod)
        if wa or wn:
            self._ipa_flags |= abi.KSS_POD_IPA_HAS_PREFERRED
        for sign, lst in ((1, wa), (-1, wn)):
            for w, t in lst:
                off, ln = self._list(self._classes_matching(lambda cns, lb, t=t: t.matches(cns, lb, None)))
                self._ipa.append((abi.KSS_IPA_SCORE_CLASS, self.key_index[t.topology_key], off, ln, sign * w, 0))
        groups: Dict[Tuple[int, int], List[int]] = {}
        for tid, (kind, w, t) in enumerate(self.terms):
            if kind == "RA":
                if self.hard_w <= 0:
                    continue
                coef = self.hard_w
            elif kind == "PA":
                coef = w
            elif kind == "PN":
                coef = -w
            else:
                continue
            if t.matches(ns, plabels, nslabels):
                groups.setdefault((self.key_index[t.topology_key], coef), []).append(tid)
        for (k, coef) in sorted(groups):
            off, ln = self._list(groups[(k, coef)])
            self._ipa.append((abi.KSS_IPA_SCORE_TERM, k, off, ln, coef, 0))
        rec["ipa_len"] = len(self._ipa) - rec["ipa_off"]


def _term_has_error(pref: dict) -> bool:
    for e in pref.get("matchExpressions") or []:
        op = e.get("operator")
        vals = e.get("values") or []
        if op in ("In", "NotIn") and not vals:
            return True
        if op in ("Exists", "DoesNotExist") and vals:
            return True
        if op in ("Gt", "Lt") and (len(vals) != 1 or parse_int(vals[0]) is None):
            return True
        if op not in ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"):
            return True
    for e in pref.get("matchFields") or []:
        if e.get("operator") not in ("In", "NotIn") or len(e.get("values") or []) != 1:
            return True
    return False


def requirement_on_value(op: str, vals, v: Optional[str]) -> bool:
    """Requirement.Matches evaluated for a single node value (None = label absent)."""
    if op == "In":
        return v is not None and v in vals
    if op == "NotIn":
        return v is None or v not in vals
    if op == "Exists":
        return v is not None
    if op == "DoesNotExist":
        return v is None
    if op in ("Gt", "Lt"):
        if v is None:
            return False
        lv = parse_int(v)
        rv = parse_int(vals[0])
        if lv is None or rv is None:
            return False
        return lv > rv if op == "Gt" else lv < rv
    return False


def compile_cluster(nodes, bound_pods=(), pending=(), namespaces=None, **kw):
    """Convenience: returns (CompiledCluster, CompiledPods, Compiler)."""
    c = Compiler(nodes, bound_pods, pending, namespaces, **kw)
    cc, cp = c.compile()
    return cc, cp, c
