"""Object-level ORACLE (TEST INFRASTRUCTURE ONLY) — pure Python, small cases.

An independent restatement of the scheduling cycle of kube-scheduler-simulator
(upstream k8s.io/kubernetes v1.26.2, pinned at /root/reference/simulator/go.mod:56;
not vendored, unbuildable here) working directly on Kubernetes-shaped objects
(dicts with metadata/spec/status).  It shares no code with the product package:
quantity parsing, selectors and every plugin are re-written here from the
upstream function they cite.  It also formats the simulator's annotations the
way resultstore.Store.GetStoredResult does
(/root/reference/simulator/scheduler/plugin/resultstore/store.go:133-198) with
Go encoding/json string escaping and sorted map keys.

Pinned by the reference's own known answer (README.md:61-79): see
tests/test_oracle_known_answer.py.  Tie-break in selectHost: max total, lowest
canonical node index (reference: random reservoir sampling,
/root/reference/scheduler/scheduler.go:323-344).

Used only by tests/ (checker), never by the product.
"""
from __future__ import annotations

import math
import re
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

# ---------------------------------------------------------------------------
# quantities (apimachinery resource.Quantity) — independent restatement
# ---------------------------------------------------------------------------
_SUF = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60,
        "n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": 1, "k": 10**3,
        "M": 10**6, "G": 10**9, "T": 10**12, "P": 10**15, "E": 10**18}


def qparse(s) -> Fraction:
    if isinstance(s, int):
        return Fraction(s)
    s = str(s)
    m = re.match(r"^([+-]?\d*\.?\d*)([eE][+-]?\d+|[A-Za-z]*)$", s)
    if not m:
        raise ValueError(s)
    num, suf = m.group(1), m.group(2)
    val = Fraction(num)
    if suf[:1] in ("e", "E"):
        return val * Fraction(10) ** int(suf[1:])
    return val * _SUF[suf]


def qvalue(s) -> int:
    return math.ceil(qparse(s))


def qmilli(s) -> int:
    return math.ceil(qparse(s) * 1000)


# ---------------------------------------------------------------------------
# labels
# ---------------------------------------------------------------------------
def _parse_int64(s):
    if not isinstance(s, str) or not re.fullmatch(r"[+-]?[0-9]+", s):
        return None
    v = int(s)
    return v if -(2**63) <= v < 2**63 else None


def req_match(key, op, values, labels) -> bool:
    """labels.Requirement.Matches."""
    has = key in labels
    if op in ("In", "="):
        return has and labels[key] in values
    if op == "NotIn":
        return (not has) or labels[key] not in values
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    if op in ("Gt", "Lt"):
        if not has or len(values) != 1:
            return False
        a, b = _parse_int64(labels[key]), _parse_int64(values[0])
        if a is None or b is None:
            return False
        return a > b if op == "Gt" else a < b
    return False


class LSel:
    """metav1.LabelSelectorAsSelector result: None -> nothing, {} -> everything."""

    def __init__(self, ls):
        if ls is None:
            self.kind = "nothing"
            self.reqs = []
            return
        ml = ls.get("matchLabels") or {}
        me = ls.get("matchExpressions") or []
        if not ml and not me:
            self.kind = "everything"
            self.reqs = []
            return
        self.kind = "reqs"
        self.reqs = [(k, "=", [v]) for k, v in ml.items()] + [(e["key"], e["operator"], list(e.get("values") or []))
                                                             for e in me]

    def empty(self):
        return self.kind == "everything"

    def matches(self, labels):
        labels = labels or {}
        if self.kind == "nothing":
            return False
        return all(req_match(k, op, v, labels) for k, op, v in self.reqs)


# ---------------------------------------------------------------------------
# cluster model: NodeInfo
# ---------------------------------------------------------------------------
def _spec(o):
    return o.get("spec") or {}


def _meta(o):
    return o.get("metadata") or {}


def _labels(o):
    return dict(_meta(o).get("labels") or {})


def _ns(o):
    return _meta(o).get("namespace") or "default"


def _name(o):
    return _meta(o).get("name", "")


SCALAR_PREFIX_EXCLUDE = ("cpu", "memory", "ephemeral-storage", "pods")


def _is_scalar(name):
    if name in SCALAR_PREFIX_EXCLUDE:
        return False
    if name.startswith("hugepages-") or name.startswith("attachable-volumes-"):
        return True
    if "/" not in name or name.startswith("requests."):
        return False
    d = name.split("/", 1)[0]
    return not (d == "kubernetes.io" or d.endswith(".kubernetes.io"))


class Resource:
    """framework.Resource."""

    def __init__(self):
        self.milli_cpu = 0
        self.memory = 0
        self.ephemeral = 0
        self.allowed_pods = 0
        self.scalars: Dict[str, int] = {}

    def add(self, rl):
        for k, q in (rl or {}).items():
            if k == "cpu":
                self.milli_cpu += qmilli(q)
            elif k == "memory":
                self.memory += qvalue(q)
            elif k == "ephemeral-storage":
                self.ephemeral += qvalue(q)
            elif k == "pods":
                self.allowed_pods += qvalue(q)
            elif _is_scalar(k):
                self.scalars[k] = self.scalars.get(k, 0) + qvalue(q)

    def set_max(self, rl):
        for k, q in (rl or {}).items():
            if k == "cpu":
                self.milli_cpu = max(self.milli_cpu, qmilli(q))
            elif k == "memory":
                self.memory = max(self.memory, qvalue(q))
            elif k == "ephemeral-storage":
                self.ephemeral = max(self.ephemeral, qvalue(q))
            elif k == "pods":
                self.allowed_pods = max(self.allowed_pods, qvalue(q))
            elif _is_scalar(k):
                self.scalars[k] = max(self.scalars.get(k, 0), qvalue(q))


def _creq(c):
    return ((c.get("resources") or {}).get("requests")) or {}


def get_request_for_resource(res_name, requests, non_zero) -> int:
    """schedutil.GetRequestForResource."""
    if res_name == "cpu":
        if "cpu" not in requests and non_zero:
            return 100
        return qmilli(requests["cpu"]) if "cpu" in requests else 0
    if res_name == "memory":
        if "memory" not in requests and non_zero:
            return 200 * 1024 * 1024
        return qvalue(requests["memory"]) if "memory" in requests else 0
    return qvalue(requests[res_name]) if res_name in requests else 0


def calculate_resource(pod):
    """framework.calculateResource -> (Resource, non0CPU, non0Mem)."""
    res = Resource()
    c0 = m0 = 0
    for c in _spec(pod).get("containers") or []:
        res.add(_creq(c))
        c0 += get_request_for_resource("cpu", _creq(c), True)
        m0 += get_request_for_resource("memory", _creq(c), True)
    for c in _spec(pod).get("initContainers") or []:
        res.set_max(_creq(c))
        c0 = max(c0, get_request_for_resource("cpu", _creq(c), True))
        m0 = max(m0, get_request_for_resource("memory", _creq(c), True))
    oh = _spec(pod).get("overhead")
    if oh:
        res.add(oh)
        if "cpu" in oh:
            c0 += qmilli(oh["cpu"])
        if "memory" in oh:
            m0 += qvalue(oh["memory"])
    return res, c0, m0


class AffTerm:
    """framework.AffinityTerm."""

    def __init__(self, pod, t):
        self.selector = LSel(t.get("labelSelector"))
        nsl = t.get("namespaces") or []
        if not nsl and t.get("namespaceSelector") is None:
            self.namespaces = {_ns(pod)}
        else:
            self.namespaces = set(nsl)
        self.ns_selector = LSel(t.get("namespaceSelector"))
        self.topology_key = t.get("topologyKey", "")

    def matches(self, pod, ns_labels):
        if _ns(pod) in self.namespaces or self.ns_selector.matches(ns_labels or {}):
            return self.selector.matches(_labels(pod))
        return False


class PodInfo:
    """framework.PodInfo with parsed affinity terms."""

    def __init__(self, pod):
        self.pod = pod
        aff = _spec(pod).get("affinity") or {}
        pa = aff.get("podAffinity") or {}
        pn = aff.get("podAntiAffinity") or {}
        self.required_affinity = [AffTerm(pod, t) for t in pa.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
        self.required_anti = [AffTerm(pod, t) for t in pn.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
        self.preferred_affinity = [(int(w["weight"]), AffTerm(pod, w["podAffinityTerm"]))
                                   for w in pa.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
        self.preferred_anti = [(int(w["weight"]), AffTerm(pod, w["podAffinityTerm"]))
                               for w in pn.get("preferredDuringSchedulingIgnoredDuringExecution") or []]


def _container_host_ports(pod):
    """(hostIP, protocol, hostPort) of the pod's containers' ports, HostPortInfo-sanitized
    (framework/types.go: "" -> 0.0.0.0 / TCP; hostPort <= 0 never added nor checked)."""
    out = []
    for c in _spec(pod).get("containers") or []:
        for cp in c.get("ports") or []:
            port = int(cp.get("hostPort") or 0)
            if port > 0:
                out.append((cp.get("hostIP") or "0.0.0.0", cp.get("protocol") or "TCP", port))
    return out


def check_conflict(used, ip, protocol, port) -> bool:
    """framework.HostPortInfo.CheckConflict over a set of (ip, protocol, port)."""
    if ip == "0.0.0.0":
        return any((pr, po) == (protocol, port) for _, pr, po in used)
    return ("0.0.0.0", protocol, port) in used or (ip, protocol, port) in used


class NodeInfo:
    def __init__(self, node):
        self.node = node
        self.pods: List[PodInfo] = []
        self.used_ports = set()
        self.requested = Resource()
        self.nz_cpu = 0
        self.nz_mem = 0
        al = (node.get("status") or {}).get("allocatable") or {}
        self.allocatable = Resource()
        self.allocatable.add(al)

    def add_pod(self, pod):
        """NodeInfo.AddPod."""
        res, c0, m0 = calculate_resource(pod)
        self.requested.milli_cpu += res.milli_cpu
        self.requested.memory += res.memory
        self.requested.ephemeral += res.ephemeral
        for k, v in res.scalars.items():
            self.requested.scalars[k] = self.requested.scalars.get(k, 0) + v
        self.nz_cpu += c0
        self.nz_mem += m0
        self.pods.append(PodInfo(pod))
        self.used_ports.update(_container_host_ports(pod))  # updateUsedPorts(pod, true)

    def remove_pod(self, pod):
        """NodeInfo.RemovePod: resources back, removeFromSlice (swap with the last element)."""
        for i, pi in enumerate(self.pods):
            if pi.pod is pod:
                self.pods[i] = self.pods[-1]
                self.pods.pop()
                break
        else:
            raise KeyError("pod not on node")
        res, c0, m0 = calculate_resource(pod)
        self.requested.milli_cpu -= res.milli_cpu
        self.requested.memory -= res.memory
        self.requested.ephemeral -= res.ephemeral
        for k, v in res.scalars.items():
            self.requested.scalars[k] = self.requested.scalars.get(k, 0) - v
        self.nz_cpu -= c0
        self.nz_mem -= m0
        self.used_ports.difference_update(_container_host_ports(pod))  # HostPortInfo.Remove

    def clone(self):
        c = NodeInfo.__new__(NodeInfo)
        c.node = self.node
        c.pods = list(self.pods)
        c.requested = Resource()
        c.requested.milli_cpu, c.requested.memory = self.requested.milli_cpu, self.requested.memory
        c.requested.ephemeral = self.requested.ephemeral
        c.requested.scalars = dict(self.requested.scalars)
        c.requested.allowed_pods = self.requested.allowed_pods
        c.nz_cpu, c.nz_mem = self.nz_cpu, self.nz_mem
        c.allocatable = self.allocatable
        c.used_ports = set(self.used_ports)
        c.image_states = getattr(self, "image_states", {})
        return c


def zone_key(node):
    lb = _labels(node)
    z = lb.get("failure-domain.beta.kubernetes.io/zone", lb.get("topology.kubernetes.io/zone", ""))
    r = lb.get("failure-domain.beta.kubernetes.io/region", lb.get("topology.kubernetes.io/region", ""))
    if not r and not z:
        return ""
    return r + ":\x00:" + z


def node_tree_list(nodes):
    """internal/cache nodeTree.list."""
    zones, tree = [], {}
    for n in nodes:
        z = zone_key(n)
        if z not in tree:
            zones.append(z)
            tree[z] = []
        tree[z].append(n)
    out, i = [], 0
    while len(out) < len(nodes):
        for z in zones:
            if i < len(tree[z]):
                out.append(tree[z][i])
        i += 1
    return out


# ---------------------------------------------------------------------------
# plugins (⟨k8s⟩ pkg/scheduler/framework/plugins/*)
# ---------------------------------------------------------------------------
def tolerates(tol, taint):
    """v1.Toleration.ToleratesTaint."""
    if tol.get("effect") and tol.get("effect") != taint.get("effect"):
        return False
    if tol.get("key") and tol.get("key") != taint.get("key"):
        return False
    op = tol.get("operator") or ""
    if op in ("", "Equal"):
        return (tol.get("value") or "") == (taint.get("value") or "")
    return op == "Exists"


def tolerations_tolerate(tols, taint):
    return any(tolerates(t, taint) for t in tols or [])


def find_untolerated(taints, tols, flt):
    for t in taints or []:
        if flt(t) and not tolerations_tolerate(tols, t):
            return t
    return None


def _do_not_schedule(t):
    return t.get("effect") in ("NoSchedule", "NoExecute")


class NodeSelectorTerms:
    """component-helpers nodeaffinity.nodeSelector (LazyErrorNodeSelector)."""

    def __init__(self, terms):
        self.terms = []  # list of (label reqs, field reqs, err)
        for t in terms:
            me, mf = t.get("matchExpressions") or [], t.get("matchFields") or []
            if not me and not mf:
                continue  # isEmptyNodeSelectorTerm
            self.terms.append(self._parse(me, mf))

    @staticmethod
    def _parse(me, mf):
        err = False
        lreqs, freqs = [], []
        for e in me:
            op, vals = e.get("operator"), list(e.get("values") or [])
            if op not in ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"):
                err = True
            elif op in ("In", "NotIn") and not vals:
                err = True
            elif op in ("Exists", "DoesNotExist") and vals:
                err = True
            elif op in ("Gt", "Lt") and (len(vals) != 1 or _parse_int64(vals[0]) is None):
                err = True
            lreqs.append((e.get("key"), op, vals))
        for e in mf:
            op, vals = e.get("operator"), list(e.get("values") or [])
            if op not in ("In", "NotIn") or len(vals) != 1:
                err = True
            freqs.append((e.get("key"), op, vals))
        return lreqs, freqs, err

    @staticmethod
    def term_match(term, node):
        lreqs, freqs, err = term
        if err:
            return False
        lb = _labels(node)
        if lreqs and not all(req_match(k, op, v, lb) for k, op, v in lreqs):
            return False
        fields = {"metadata.name": _name(node)} if _name(node) else {}
        if freqs and fields:
            for k, op, v in freqs:
                got = fields.get(k, "")
                if op == "In" and got != v[0]:
                    return False
                if op == "NotIn" and got == v[0]:
                    return False
        return True

    def match(self, node):
        return any(self.term_match(t, node) for t in self.terms)


def required_node_affinity_match(pod, node):
    """nodeaffinity.GetRequiredNodeAffinity(pod).Match(node)."""
    sel = _spec(pod).get("nodeSelector") or {}
    lb = _labels(node)
    for k, v in sel.items():
        if lb.get(k) != v or k not in lb:
            return False
    na = ((_spec(pod).get("affinity") or {}).get("nodeAffinity")) or {}
    req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
    if req is not None:
        return NodeSelectorTerms(req.get("nodeSelectorTerms") or []).match(node)
    return True


MSG = {
    "NodeUnschedulable": "node(s) were unschedulable",
    "NodeName": "node(s) didn't match the requested node name",
    "NodeAffinity": "node(s) didn't match Pod's node affinity/selector",
    "NodePorts": "node(s) didn't have free ports for the requested pod ports",  # nodeports.go ErrReason
    "PTS": "node(s) didn't match pod topology spread constraints",
    "PTS_LABEL": "node(s) didn't match pod topology spread constraints (missing required label)",
    "IPA_AFF": "node(s) didn't match pod affinity rules",
    "IPA_ANTI": "node(s) didn't match pod anti-affinity rules",
    "IPA_EXIST": "node(s) didn't satisfy existing pods anti-affinity rules",
}

FILTERS = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
           "VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits", "VolumeBinding",
           "VolumeZone", "PodTopologySpread", "InterPodAffinity"]
SCORES = ["TaintToleration", "NodeAffinity", "NodeResourcesFit", "VolumeBinding", "PodTopologySpread",
          "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"]
NORMALIZING = {"TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity"}
PREFILTERS = ["NodeAffinity", "NodePorts", "NodeResourcesFit", "VolumeRestrictions", "VolumeBinding",
              "PodTopologySpread", "InterPodAffinity"]
PRESCORES = ["TaintToleration", "NodeAffinity", "PodTopologySpread", "InterPodAffinity"]
DEFAULT_WEIGHTS = {"TaintToleration": 3, "NodeAffinity": 2, "NodeResourcesFit": 1, "VolumeBinding": 1,
                   "PodTopologySpread": 2, "InterPodAffinity": 2, "NodeResourcesBalancedAllocation": 1,
                   "ImageLocality": 1}


def num_feasible_nodes_to_find(num_all_nodes: int, pct: int) -> int:
    """Scheduler.numFeasibleNodesToFind (pkg/scheduler/schedule_one.go, v1.26.2)."""
    min_feasible_nodes_to_find, min_feasible_nodes_percentage_to_find = 100, 5
    if num_all_nodes < min_feasible_nodes_to_find or pct >= 100:
        return num_all_nodes
    adaptive = pct
    if adaptive <= 0:
        adaptive = 50 - num_all_nodes // 125
        if adaptive < min_feasible_nodes_percentage_to_find:
            adaptive = min_feasible_nodes_percentage_to_find
    num_nodes = num_all_nodes * adaptive // 100
    if num_nodes < min_feasible_nodes_to_find:
        return min_feasible_nodes_to_find
    return num_nodes


def go_log(x: float) -> float:
    """Go math.Log (src/math/log.go)."""
    Ln2Hi, Ln2Lo = 6.93147180369123816490e-01, 1.90821492927058770002e-10
    L1, L2, L3, L4 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01, 2.222219843214978396e-01
    L5, L6, L7 = 1.818357216161805012e-01, 1.531383769920937332e-01, 1.479819860511658591e-01
    f1, ki = math.frexp(x)
    if f1 < math.sqrt(2) / 2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f)


def go_round(x: float) -> int:
    """math.Round: half away from zero."""
    return int(math.floor(abs(x) + 0.5)) * (1 if x >= 0 else -1)


# ----------------------------------------------------------- AddPod / RemovePod extensions
# The PreFilter extensions both RunFilterPluginsWithNominatedPods (addNominatedPods) and
# SelectVictimsOnNode (k8s_preemption) drive on a cloned cycle state.
MAX_INT32 = 2**31 - 1


def pod_priority(pod) -> int:
    """corev1helpers.PodPriority: spec.priority (set by the Priority admission plugin), 0 if unset."""
    p = _spec(pod).get("priority")
    return int(p) if p is not None else 0


class CriticalPaths:
    """podtopologyspread criticalPaths: [2]{TopologyValue, MatchNum}, newCriticalPaths = MaxInt32."""

    def __init__(self):
        self.p = [["", MAX_INT32], ["", MAX_INT32]]

    def update(self, val, num):
        p = self.p
        i = 0 if val == p[0][0] else (1 if val == p[1][0] else -1)
        if i >= 0:
            p[i][1] = num
            if p[0][1] > p[1][1]:
                p[0], p[1] = p[1], p[0]
        else:
            if num < p[0][1]:
                p[1] = p[0]
                p[0] = [val, num]
            elif num < p[1][1]:
                p[1] = [val, num]

    def min(self):
        return self.p[0][1]


def _pts_state(st):
    """Clone of the PodTopologySpread preFilterState with criticalPaths built as calPreFilterState
    does (update over every pair); `mins` mirrors paths[key][0] for Oracle.pts_filter."""
    if not st["cons"]:
        return dict(cons=[])
    pair_num = dict(st["pair_num"])
    paths: Dict[str, CriticalPaths] = {}
    for (k, v), num in pair_num.items():
        paths.setdefault(k, CriticalPaths()).update(v, num)
    return dict(cons=st["cons"], pair_num=pair_num, paths=paths, mins={k: cp.min() for k, cp in paths.items()})


def _pts_update(st, victim, preemptor, node, delta):
    """podtopologyspread preFilterState.updateWithPod (v1.26)."""
    if not st["cons"] or _ns(victim) != _ns(preemptor):
        return
    lb = _labels(node)
    if not all(c["key"] in lb for c in st["cons"]):
        return
    if not required_node_affinity_match(preemptor, node):
        return
    plabels = _labels(victim)
    for c in st["cons"]:
        if not c["sel"].matches(plabels):
            continue
        pair = (c["key"], lb[c["key"]])
        st["pair_num"][pair] = st["pair_num"].get(pair, 0) + delta
        st["paths"].setdefault(c["key"], CriticalPaths()).update(lb[c["key"]], st["pair_num"][pair])
        st["mins"][c["key"]] = st["paths"][c["key"]].min()


def _ipa_state(st):
    return dict(pinfo=st["pinfo"], existing=dict(st["existing"]), aff=dict(st["aff"]), anti=dict(st["anti"]))


def _tm_update(m, node, key, value):
    """topologyToMatchedTermCount.update: delete the pair when it reaches zero."""
    lb = _labels(node)
    if key in lb:
        pair = (key, lb[key])
        m[pair] = m.get(pair, 0) + value
        if m[pair] == 0:
            del m[pair]


def _ipa_update(o, st, victim_pi, preemptor, node, mult):
    """interpodaffinity preFilterState.updateWithPod (v1.26)."""
    pinfo = st["pinfo"]
    nsl = o.namespaces.get(_ns(preemptor), {})
    for t in victim_pi.required_anti:
        if t.matches(preemptor, nsl):
            _tm_update(st["existing"], node, t.topology_key, mult)
    if pinfo.required_affinity and all(t.matches(victim_pi.pod, None) for t in pinfo.required_affinity):
        for t in pinfo.required_affinity:
            _tm_update(st["aff"], node, t.topology_key, mult)
    for t in pinfo.required_anti:
        if t.matches(victim_pi.pod, None):
            _tm_update(st["anti"], node, t.topology_key, mult)



class Oracle:
    """Sequential scheduler over objects; one schedule_one() per pending pod."""

    def __init__(self, nodes, bound_pods=(), namespaces=None, weights=None, hard_pod_affinity_weight=1,
                 system_defaulted=True, fit_strategy="LeastAllocated", fit_resources=(("cpu", 1), ("memory", 1)),
                 ba_resources=("cpu", "memory"), storage=None, percentage_of_nodes_to_score=100):
        """storage: k8s_volumes.Storage (PVs, PVCs, StorageClasses, CSINodes) for the volume plugins.
        percentage_of_nodes_to_score: KubeSchedulerConfiguration.percentageOfNodesToScore (0: the
        adaptive default the simulator's built-in scheduler runs with)."""
        import k8s_volumes
        self.storage = storage if storage is not None else k8s_volumes.Storage()
        self.nodes = node_tree_list(list(nodes))
        self.infos = [NodeInfo(n) for n in self.nodes]
        # NodeInfo.ImageStates as the v1.26 cache builds them while nodes are added (input
        # order): size of the first node listing the name, NumNodes counted at that node's add
        states, size, holders = {}, {}, {}
        for n in nodes:
            summ = {}
            for im in ((n.get("status") or {}).get("images") or []):
                for nm in im.get("names") or []:
                    if nm not in size:
                        size[nm], holders[nm] = int(im.get("sizeBytes") or 0), set()
                    holders[nm].add(_name(n))
                    summ.setdefault(nm, (size[nm], len(holders[nm])))
            states[_name(n)] = summ
        for ni in self.infos:
            ni.image_states = states[_name(ni.node)]
        self.by_name = {_name(n): i for i, n in enumerate(self.nodes)}
        self.namespaces = dict(namespaces or {})
        for p in bound_pods:
            nn = _spec(p).get("nodeName")
            if nn in self.by_name:
                self.infos[self.by_name[nn]].add_pod(p)
        self.weights = dict(weights or DEFAULT_WEIGHTS)
        self.hard_w = hard_pod_affinity_weight
        self.system_defaulted = system_defaulted
        self.fit_strategy = fit_strategy
        self.fit_resources = list(fit_resources)
        self.ba_resources = list(ba_resources)
        self.pct = percentage_of_nodes_to_score
        self.next_start = 0  # Scheduler.nextStartNodeIndex
        # the scheduling queue's nominator: [(pod key, pod, node index)] in AddNominatedPod order
        self.nominated: List[Tuple[Tuple[str, str], dict, int]] = []

    # ----------------------------------------------------------- nominator
    @staticmethod
    def _key(pod) -> Tuple[str, str]:
        return (_ns(pod), _name(pod))  # the pod's UID in this restatement

    def nominate(self, pod, i: int):
        """PodNominator.AddNominatedPod (a pod's earlier nomination is replaced)."""
        self.clear_nomination(pod)
        self.nominated.append((self._key(pod), pod, i))

    def clear_nomination(self, pod):
        """PodNominator.DeleteNominatedPodIfExists."""
        k = self._key(pod)
        self.nominated = [e for e in self.nominated if e[0] != k]

    def nomination_of(self, pod) -> Optional[int]:
        """status.nominatedNodeName as a node index (None when the pod is not nominated)."""
        k = self._key(pod)
        for kk, _, i in self.nominated:
            if kk == k:
                return i
        return None

    def assume(self, pod, i: int):
        """Reserve's VolumeBinding.AssumePodVolumes (the binder's assume cache: WaitForFirstConsumer
        claims' static bindings and provisioning decisions on node i), Cache.AssumePod ->
        NodeInfo.AddPod, then SchedulingQueue.DeleteNominatedPodIfExists (schedule_one.go assume)."""
        if _spec(pod).get("volumes"):
            _, claims = self.storage.binding_prefilter(pod)
            self.storage.assume(claims, self.infos[i].node, NodeSelectorTerms)
        self.infos[i].add_pod(pod)
        self.clear_nomination(pod)

    def forget(self, pod, i: int):
        """Unreserve: VolumeBinding.Unreserve (RevertAssumedPodVolumes) and Cache.ForgetPod ->
        NodeInfo.RemovePod."""
        if _spec(pod).get("volumes"):
            _, claims = self.storage.binding_prefilter(pod)
            self.storage.revert(claims)
        self.infos[i].remove_pod(pod)

    def filter_with_nominated(self, pod, i: int, ni: "NodeInfo", pts_st, ipa_st, vb_claims=None):
        """framework.RunFilterPluginsWithNominatedPods (v1.26 runtime/framework.go) over NodeInfo ni
        of node i: a first pass with every nominated pod of equal or higher priority (other than
        the pod itself) added to a clone of ni and of the cycle state (addNominatedPods: AddPodInfo
        and RunPreFilterExtensionAddPod -- the PodTopologySpread / InterPodAffinity updateWithPod),
        then, when it passed and some pod was added, a second pass on the unmodified ni and state.
        The record is the simulator's per-plugin map (store.go:423 AddFilterResult overwrites): a
        plugin the second pass never reached keeps the first pass's "passed"."""
        prio = pod_priority(pod)
        k = self._key(pod)
        noms = [q for kk, q, n in self.nominated if n == i and kk != k and pod_priority(q) >= prio]
        if not noms:
            return self.filter_node(pod, ni, pts_st, ipa_st, vb_claims)
        ni1 = ni.clone()
        pts1 = _pts_state(pts_st)
        ipa1 = _ipa_state(ipa_st)
        for q in noms:
            ni1.add_pod(q)
            _pts_update(pts1, q, pod, ni.node, 1)
            _ipa_update(self, ipa1, PodInfo(q), pod, ni.node, 1)
        failed, rec = self.filter_node(pod, ni1, pts1, ipa1, vb_claims)
        if failed is not None:
            return failed, rec
        failed2, rec2 = self.filter_node(pod, ni, pts_st, ipa_st, vb_claims)
        rec.update(rec2)
        return failed2, rec

    # ----------------------------------------------------------- ImageLocality
    def image_locality_score(self, pod, ni) -> int:
        """image_locality.go Score: calculatePriority(sumImageScores(...), len(Containers))."""
        total = len(self.infos)
        conts = _spec(pod).get("containers") or []
        s = 0
        for c in conts:
            nm = c.get("image") or ""
            if nm.rfind(":") <= nm.rfind("/"):  # normalizedImageName
                nm += ":latest"
            st = ni.image_states.get(nm)
            if st is not None:
                s += int(float(st[0]) * (float(st[1]) / float(total)))  # scaledImageScore
        mb = 1024 * 1024
        lo, hi = 23 * mb, 1000 * mb * len(conts)
        s = lo if s < lo else (hi if s > hi else s)
        return 100 * (s - lo) // (hi - lo) if hi != lo else 0

    # ----------------------------------------------------------- NodeResourcesFit
    def fit_filter(self, pod, ni: NodeInfo) -> Optional[str]:
        """noderesources.fitsRequest."""
        req = calculate_resource(pod)[0]
        reasons = []
        if len(ni.pods) + 1 > ni.allocatable.allowed_pods:
            reasons.append("Too many pods")
        if req.milli_cpu == 0 and req.memory == 0 and req.ephemeral == 0 and not req.scalars:
            return ", ".join(reasons) if reasons else None
        if req.milli_cpu > ni.allocatable.milli_cpu - ni.requested.milli_cpu:
            reasons.append("Insufficient cpu")
        if req.memory > ni.allocatable.memory - ni.requested.memory:
            reasons.append("Insufficient memory")
        if req.ephemeral > ni.allocatable.ephemeral - ni.requested.ephemeral:
            reasons.append("Insufficient ephemeral-storage")
        for name in sorted(req.scalars):  # map order upstream; sorted here (deterministic)
            q = req.scalars[name]
            if q == 0:
                continue
            if q > ni.allocatable.scalars.get(name, 0) - ni.requested.scalars.get(name, 0):
                reasons.append(f"Insufficient {name}")
        return ", ".join(reasons) if reasons else None

    def _pod_request(self, pod, res_name, non_zero):
        """resource_allocation calculatePodResourceRequest (v1.26)."""
        r = 0
        for c in _spec(pod).get("containers") or []:
            r += get_request_for_resource(res_name, _creq(c), non_zero)
        for c in _spec(pod).get("initContainers") or []:
            r = max(r, get_request_for_resource(res_name, _creq(c), non_zero))
        oh = _spec(pod).get("overhead")
        if oh and res_name in oh:
            r += qvalue(oh[res_name])
        return r

    def _alloc_req(self, ni, pod, res_name, use_requested):
        """calculateResourceAllocatableRequest."""
        pr = self._pod_request(pod, res_name, not use_requested)
        if pr == 0 and _is_scalar(res_name):
            return 0, 0
        if res_name == "cpu":
            base = ni.requested.milli_cpu if use_requested else ni.nz_cpu
            return ni.allocatable.milli_cpu, base + pr
        if res_name == "memory":
            base = ni.requested.memory if use_requested else ni.nz_mem
            return ni.allocatable.memory, base + pr
        if res_name == "ephemeral-storage":
            return ni.allocatable.ephemeral, ni.requested.ephemeral + pr
        if res_name in ni.allocatable.scalars:
            return ni.allocatable.scalars[res_name], ni.requested.scalars.get(res_name, 0) + pr
        return 0, 0

    def fit_score(self, pod, ni):
        node_score = weight_sum = 0
        for name, w in self.fit_resources:
            alloc, req = self._alloc_req(ni, pod, name, False)
            if alloc == 0:
                continue
            if self.fit_strategy == "MostAllocated":
                rq = min(req, alloc)
                s = rq * 100 // alloc
            else:
                s = 0 if req > alloc else (alloc - req) * 100 // alloc
            node_score += s * w
            weight_sum += w
        return 0 if weight_sum == 0 else node_score // weight_sum

    def ba_score(self, pod, ni):
        fr = []
        total = 0.0
        for name in self.ba_resources:
            alloc, req = self._alloc_req(ni, pod, name, True)
            if alloc == 0:
                continue
            f = float(req) / float(alloc)
            if f > 1:
                f = 1.0
            total += f
            fr.append(f)
        std = 0.0
        if len(fr) == 2:
            std = abs((fr[0] - fr[1]) / 2)
        elif len(fr) > 2:
            mean = total / float(len(fr))
            acc = 0.0
            for f in fr:
                acc = acc + (f - mean) * (f - mean)
            std = math.sqrt(acc / float(len(fr)))
        return int((1 - std) * float(100))

    # ----------------------------------------------------------- PodTopologySpread
    def _spread_constraints(self, pod, action):
        cons = _spec(pod).get("topologySpreadConstraints") or []
        out = []
        if cons:
            for c in cons:
                if c.get("whenUnsatisfiable") == action:
                    out.append(dict(key=c["topologyKey"], max_skew=int(c.get("maxSkew", 1)),
                                    sel=LSel(c.get("labelSelector")),
                                    aff_honor=(c.get("nodeAffinityPolicy") or "Honor") == "Honor",
                                    taint_honor=(c.get("nodeTaintsPolicy") or "Ignore") == "Honor"))
            return out
        ann = (_meta(pod).get("annotations") or {}).get("kss.x-k8s.io/default-spread-selector")
        if self.system_defaulted and ann and action == "ScheduleAnyway":
            import json
            sel = LSel(json.loads(ann))
            if sel.empty():
                return []
            return [dict(key="kubernetes.io/hostname", max_skew=3, sel=sel, aff_honor=True, taint_honor=False),
                    dict(key="topology.kubernetes.io/zone", max_skew=5, sel=sel, aff_honor=True, taint_honor=False)]
        return []

    @staticmethod
    def _count_match(ni, sel, ns):
        """countPodsMatchSelector."""
        if sel.empty():
            return 0
        return sum(1 for pi in ni.pods if _ns(pi.pod) == ns and sel.matches(_labels(pi.pod)))

    def _inclusion_ok(self, c, pod, node):
        if c["aff_honor"] and not required_node_affinity_match(pod, node):
            return False
        if c["taint_honor"] and find_untolerated(_spec(node).get("taints"), _spec(pod).get("tolerations"),
                                                _do_not_schedule) is not None:
            return False
        return True

    def pts_prefilter(self, pod):
        """calPreFilterState."""
        cons = self._spread_constraints(pod, "DoNotSchedule")
        if not cons:
            return dict(cons=[])
        pair_num: Dict[Tuple[str, str], int] = {}
        for ni in self.infos:
            lb = _labels(ni.node)
            if not all(c["key"] in lb for c in cons):
                continue
            # tpCounts[pair] = count: constraints on one key overwrite each other per node
            tp_counts: Dict[Tuple[str, str], int] = {}
            for c in cons:
                if not self._inclusion_ok(c, pod, ni.node):
                    continue
                pair = (c["key"], lb[c["key"]])
                tp_counts[pair] = self._count_match(ni, c["sel"], _ns(pod))
            for pair, cnt in tp_counts.items():
                pair_num[pair] = pair_num.get(pair, 0) + cnt
        mins = {}
        for (k, v), num in pair_num.items():
            mins[k] = min(mins.get(k, 2**31 - 1), num)
        return dict(cons=cons, pair_num=pair_num, mins=mins)

    def pts_filter(self, st, pod, node) -> Optional[str]:
        if not st["cons"]:
            return None
        lb = _labels(node)
        for c in st["cons"]:
            if c["key"] not in lb:
                return MSG["PTS_LABEL"]
            mn = st["mins"].get(c["key"], 2**31 - 1)
            self_match = 1 if c["sel"].matches(_labels(pod)) else 0
            num = st["pair_num"].get((c["key"], lb[c["key"]]), 0)
            if num + self_match - mn > c["max_skew"]:
                return MSG["PTS"]
        return None

    def pts_prescore(self, pod, feasible):
        """PodTopologySpread.PreScore + initPreScoreState."""
        cons = self._spread_constraints(pod, "ScheduleAnyway")
        require_all = bool(_spec(pod).get("topologySpreadConstraints")) or not self.system_defaulted
        st = dict(cons=cons, ignored=set(), pair_counts={}, weights=[])
        if not cons:
            return st
        topo_size = [0] * len(cons)
        for i in feasible:
            lb = _labels(self.nodes[i])
            if require_all and not all(c["key"] in lb for c in cons):
                st["ignored"].add(i)
                continue
            for ci, c in enumerate(cons):
                if c["key"] == "kubernetes.io/hostname":
                    continue
                pair = (c["key"], lb.get(c["key"], ""))
                if pair not in st["pair_counts"]:
                    st["pair_counts"][pair] = 0
                    topo_size[ci] += 1
        for ci, c in enumerate(cons):
            sz = topo_size[ci]
            if c["key"] == "kubernetes.io/hostname":
                sz = len(feasible) - len(st["ignored"])
            st["weights"].append(go_log(float(sz + 2)))
        for ni in self.infos:
            lb = _labels(ni.node)
            if require_all and not all(c["key"] in lb for c in cons):
                continue
            for c in cons:
                if not self._inclusion_ok(c, pod, ni.node):
                    continue
                pair = (c["key"], lb.get(c["key"], ""))
                if pair not in st["pair_counts"]:
                    continue
                st["pair_counts"][pair] += self._count_match(ni, c["sel"], _ns(pod))
        return st

    def pts_score(self, st, pod, i):
        if i in st["ignored"]:
            return 0
        ni = self.infos[i]
        lb = _labels(ni.node)
        score = 0.0
        for ci, c in enumerate(st["cons"]):
            if c["key"] in lb:
                if c["key"] == "kubernetes.io/hostname":
                    cnt = self._count_match(ni, c["sel"], _ns(pod))
                else:
                    cnt = st["pair_counts"][(c["key"], lb[c["key"]])]
                score += float(cnt) * st["weights"][ci] + float(c["max_skew"] - 1)
        return go_round(score)

    # ----------------------------------------------------------- InterPodAffinity
    def _merge(self, t: AffTerm):
        if t.ns_selector.empty():
            return t
        for name, lbs in self.namespaces.items():
            if t.ns_selector.matches(lbs):
                t.namespaces.add(name)
        t.ns_selector = LSel(None)
        return t

    def ipa_prefilter(self, pod):
        pinfo = PodInfo(pod)
        for t in pinfo.required_affinity + pinfo.required_anti:
            self._merge(t)
        nsl = self.namespaces.get(_ns(pod), {})
        existing: Dict[Tuple[str, str], int] = {}
        for ni in self.infos:
            lb = _labels(ni.node)
            for ep in ni.pods:
                for t in ep.required_anti:
                    if t.matches(pod, nsl) and t.topology_key in lb:
                        pair = (t.topology_key, lb[t.topology_key])
                        existing[pair] = existing.get(pair, 0) + 1
        aff: Dict[Tuple[str, str], int] = {}
        anti: Dict[Tuple[str, str], int] = {}
        if pinfo.required_affinity or pinfo.required_anti:
            for ni in self.infos:
                lb = _labels(ni.node)
                for ep in ni.pods:
                    if pinfo.required_affinity and all(t.matches(ep.pod, None) for t in pinfo.required_affinity):
                        for t in pinfo.required_affinity:
                            if t.topology_key in lb:
                                pair = (t.topology_key, lb[t.topology_key])
                                aff[pair] = aff.get(pair, 0) + 1
                    for t in pinfo.required_anti:
                        if t.matches(ep.pod, None) and t.topology_key in lb:
                            pair = (t.topology_key, lb[t.topology_key])
                            anti[pair] = anti.get(pair, 0) + 1
        return dict(pinfo=pinfo, existing={k: v for k, v in existing.items() if v != 0},
                    aff={k: v for k, v in aff.items() if v != 0}, anti={k: v for k, v in anti.items() if v != 0})

    def ipa_filter(self, st, pod, node) -> Optional[str]:
        lb = _labels(node)
        pinfo = st["pinfo"]
        # satisfyPodAffinity
        pods_exist = True
        for t in pinfo.required_affinity:
            if t.topology_key in lb:
                if st["aff"].get((t.topology_key, lb[t.topology_key]), 0) <= 0:
                    pods_exist = False
            else:
                return MSG["IPA_AFF"]
        if not pods_exist:
            self_all = bool(pinfo.required_affinity) and all(t.matches(pod, None) for t in pinfo.required_affinity)
            if not (len(st["aff"]) == 0 and self_all):
                return MSG["IPA_AFF"]
        # satisfyPodAntiAffinity
        if st["anti"]:
            for t in pinfo.required_anti:
                if t.topology_key in lb and st["anti"].get((t.topology_key, lb[t.topology_key]), 0) > 0:
                    return MSG["IPA_ANTI"]
        # satisfyExistingPodsAntiAffinity
        if st["existing"]:
            for k, v in lb.items():
                if st["existing"].get((k, v), 0) > 0:
                    return MSG["IPA_EXIST"]
        return None

    def ipa_prescore(self, pod):
        pinfo = PodInfo(pod)
        for _, t in pinfo.preferred_affinity + pinfo.preferred_anti:
            self._merge(t)
        nsl = self.namespaces.get(_ns(pod), {})
        topo: Dict[str, Dict[str, int]] = {}

        def process(term, weight, target, ns_labels, node, mult):
            if term.matches(target, ns_labels):
                lb = _labels(node)
                if term.topology_key in lb:
                    d = topo.setdefault(term.topology_key, {})
                    d[lb[term.topology_key]] = d.get(lb[term.topology_key], 0) + weight * mult

        for ni in self.infos:
            node = ni.node
            if not _labels(node):
                continue
            for ep in ni.pods:
                for w, t in pinfo.preferred_affinity:
                    process(t, w, ep.pod, None, node, 1)
                for w, t in pinfo.preferred_anti:
                    process(t, w, ep.pod, None, node, -1)
                if self.hard_w > 0:
                    for t in ep.required_affinity:
                        process(t, self.hard_w, pod, nsl, node, 1)
                for w, t in ep.preferred_affinity:
                    process(t, w, pod, nsl, node, 1)
                for w, t in ep.preferred_anti:
                    process(t, w, pod, nsl, node, -1)
        return topo

    # ----------------------------------------------------------- runFilterPlugins
    def filter_node(self, pod, ni: NodeInfo, pts_st, ipa_st, vb_claims=None):
        """framework.RunFilterPlugins over one NodeInfo: (first failing plugin or None, the
        per-plugin record up to it).  vb_claims: VolumeBinding's bound claims from PreFilter."""
        node = ni.node
        st = self.storage
        sp = _spec(pod)
        tols = sp.get("tolerations") or []
        rec = {}
        for pl in FILTERS:
            msg = None
            if pl == "NodeUnschedulable":
                tol = tolerations_tolerate(tols, {"key": "node.kubernetes.io/unschedulable", "effect": "NoSchedule"})
                if _spec(node).get("unschedulable") and not tol:
                    msg = MSG["NodeUnschedulable"]
            elif pl == "NodeName":
                nn = sp.get("nodeName") or ""
                if nn and nn != _name(node):
                    msg = MSG["NodeName"]
            elif pl == "TaintToleration":
                t = find_untolerated(_spec(node).get("taints"), tols, _do_not_schedule)
                if t is not None:
                    msg = "node(s) had untolerated taint {%s: %s}" % (t.get("key", ""), t.get("value") or "")
            elif pl == "NodeAffinity":
                if not required_node_affinity_match(pod, node):
                    msg = MSG["NodeAffinity"]
            elif pl == "NodePorts":
                if any(check_conflict(ni.used_ports, *w) for w in _container_host_ports(pod)):
                    msg = MSG["NodePorts"]
            elif pl == "NodeResourcesFit":
                msg = self.fit_filter(pod, ni)
            elif pl == "VolumeRestrictions":
                msg = st.restrictions_filter(pod, [pi.pod for pi in ni.pods])
            elif pl in ("EBSLimits", "GCEPDLimits", "AzureDiskLimits"):
                msg = st.non_csi_filter(pl, pod, ni)
            elif pl == "NodeVolumeLimits":
                msg = st.csi_filter(pod, ni)
            elif pl == "VolumeBinding":
                msg = st.binding_filter(vb_claims, node, NodeSelectorTerms)
            elif pl == "VolumeZone":
                msg = st.zone_filter(pod, node)
            elif pl == "PodTopologySpread":
                msg = self.pts_filter(pts_st, pod, node)
            elif pl == "InterPodAffinity":
                msg = self.ipa_filter(ipa_st, pod, node)
            rec[pl] = "passed" if msg is None else msg
            if msg is not None:
                return pl, rec
        return None, rec

    # ----------------------------------------------------------- schedulePod
    def schedule_one(self, pod, commit=True):
        ann_filter: Dict[str, Dict[str, str]] = {}
        res = dict(filter=ann_filter, score={}, finalscore={}, prefilter_status={}, prescore={}, selected=None,
                   n_feasible=0, fail={}, raw={}, norm={}, total={}, scored=False, status="ok",
                   prefilter_result={})
        sp = _spec(pod)
        # RunPreFilterPlugins (multipoint order); NodeAffinity may return a PreFilterResult
        node_subset = None
        na = ((sp.get("affinity") or {}).get("nodeAffinity")) or {}
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
        conflict = False
        if req is not None and (req.get("nodeSelectorTerms") or []):
            names = set()
            for t in req.get("nodeSelectorTerms") or []:
                tn = None
                for r in t.get("matchFields") or []:
                    if r.get("key") == "metadata.name" and r.get("operator") == "In":
                        s = set(r.get("values") or [])
                        tn = s if tn is None else tn & s
                if tn is None:
                    names = None
                    break
                if not tn:
                    conflict = True
                    break
                names |= tn
            if not conflict and names:
                node_subset = names
        vb_claims = None
        for pl in PREFILTERS:
            if pl == "NodeAffinity" and conflict:
                res["prefilter_status"][pl] = "pod affinity terms conflict"
                res["status"] = "prefilter"
                return res
            if pl == "NodeAffinity" and node_subset is not None:
                res["prefilter_result"]["NodeAffinity"] = sorted(node_subset)
            if pl == "VolumeBinding":
                msg, vb_claims = self.storage.binding_prefilter(pod)
                if msg is not None:
                    res["prefilter_status"][pl] = msg
                    res["status"] = "prefilter"
                    return res
            res["prefilter_status"][pl] = "success"
        pts_st = self.pts_prefilter(pod)
        ipa_st = self.ipa_prefilter(pod)
        res["_pts_st"], res["_ipa_st"] = pts_st, ipa_st  # the cycle state PostFilter sees
        feasible = []
        tols = sp.get("tolerations") or []
        # PreferNominatedNode (findNodesThatFitPod -> evaluateNominatedNode): a pod nominated by an
        # earlier preemption first runs findNodesThatPassFilters on [that node] alone -- before and
        # regardless of the PreFilterResult set; its one-node list resets nextStartNodeIndex to 0
        # ((start + processed) % 1).  A feasible node is the answer without scoring; otherwise the
        # node's status stays in the diagnosis (the full search overwrites it if it gets there)
        nom = self.nomination_of(pod)
        if nom is not None:
            failed, rec = self.filter_with_nominated(pod, nom, self.infos[nom], pts_st, ipa_st, vb_claims)
            ann_filter[_name(self.infos[nom].node)] = rec
            res["fail"][nom] = failed
            res["nominated_eval"] = nom
            self.next_start = 0
            if failed is None:
                res["n_feasible"] = 1
                res["selected"] = nom
                if commit:
                    self.assume(pod, nom)
                return res
        # findNodesThatPassFilters (schedule_one.go, v1.26) with Parallelism = 1: the node list (the
        # PreFilterResult set in canonical order -- upstream ranges over a Go map here) is checked
        # one node at a time from nextStartNodeIndex; the feasible node that makes the count exceed
        # numFeasibleNodesToFind cancels the search and is dropped (its filters ran: it is recorded).
        node_list = [i for i, ni in enumerate(self.infos) if node_subset is None or _name(ni.node) in node_subset]
        m = len(node_list)
        num_to_find = num_feasible_nodes_to_find(m, self.pct)
        # diagnosis.NodeToStatusMap, keyed by node: it already holds evaluateNominatedNode's failure,
        # which the full search overwrites (one entry) only if it visits that node again
        feasible_len, statuses = 0, ({nom} if nom is not None else set())
        res["dropped"] = None
        for j in range(m):
            i = node_list[(self.next_start + j) % m]
            ni = self.infos[i]
            failed, rec = self.filter_with_nominated(pod, i, ni, pts_st, ipa_st, vb_claims)
            ann_filter[_name(ni.node)] = rec
            res["fail"][i] = failed
            if failed is None:
                feasible_len += 1
                if feasible_len > num_to_find:  # cancel(); atomic.AddInt32(&feasibleNodesLen, -1)
                    feasible_len -= 1
                    res["dropped"] = i
                    break
                feasible.append(i)
            else:
                statuses.add(i)
        if m:
            self.next_start = (self.next_start + feasible_len + len(statuses)) % m
        feasible.sort()  # selectHost's deterministic tie-break is the canonical index, not the visit order
        res["n_feasible"] = len(feasible)
        if not feasible:
            res["status"] = "unschedulable"
            return res
        if len(feasible) == 1:
            res["selected"] = feasible[0]
            if commit:
                self.assume(pod, feasible[0])
            return res
        res["scored"] = True
        for pl in PRESCORES:
            res["prescore"][pl] = "success"
        pts_sc = self.pts_prescore(pod, feasible)
        topo = self.ipa_prescore(pod)
        tol_pns = [t for t in tols if (t.get("effect") or "") in ("", "PreferNoSchedule")]
        raw = {pl: {} for pl in SCORES}
        for i in feasible:
            ni = self.infos[i]
            node = ni.node
            raw["TaintToleration"][i] = sum(1 for t in _spec(node).get("taints") or []
                                            if t.get("effect") == "PreferNoSchedule"
                                            and not tolerations_tolerate(tol_pns, t))
            s = 0
            pref = na.get("preferredDuringSchedulingIgnoredDuringExecution") or []
            for w in pref:
                if int(w.get("weight", 0)) == 0:
                    continue
                tt = NodeSelectorTerms([w.get("preference") or {}])
                if tt.terms and NodeSelectorTerms.term_match(tt.terms[0], node):
                    s += int(w["weight"])
            raw["NodeAffinity"][i] = s
            raw["NodeResourcesFit"][i] = self.fit_score(pod, ni)
            raw["VolumeBinding"][i] = 0
            raw["PodTopologySpread"][i] = self.pts_score(pts_sc, pod, i)
            lb = _labels(node)
            raw["InterPodAffinity"][i] = sum(vals.get(lb[k], 0) for k, vals in topo.items() if k in lb)
            raw["NodeResourcesBalancedAllocation"][i] = self.ba_score(pod, ni)
            raw["ImageLocality"][i] = self.image_locality_score(pod, ni)
        norm = {pl: dict(v) for pl, v in raw.items()}

        def default_normalize(d, reverse):
            mx = max([0] + [v for v in d.values()])
            if mx == 0:
                if reverse:
                    for k in d:
                        d[k] = 100
                return
            for k in d:
                s = 100 * d[k] // mx if d[k] >= 0 else -((-100 * d[k]) // mx)
                d[k] = 100 - s if reverse else s

        default_normalize(norm["TaintToleration"], True)
        default_normalize(norm["NodeAffinity"], False)
        d = norm["PodTopologySpread"]
        ign = pts_sc["ignored"]
        vals = [d[i] for i in feasible if i not in ign]
        mn = min(vals) if vals else 2**63 - 1
        mx = max([0] + vals)
        for i in feasible:
            if i in ign:
                d[i] = 0
            elif mx == 0:
                d[i] = 100
            else:
                d[i] = 100 * (mx + mn - d[i]) // mx
        if topo:
            d = norm["InterPodAffinity"]
            mn, mx = min(d.values()), max(d.values())
            diff = mx - mn
            for i in feasible:
                d[i] = int(float(100) * (float(d[i] - mn) / float(diff))) if diff > 0 else 0
        best, bi = None, None
        for i in feasible:
            t = sum(norm[pl][i] * self.weights[pl] for pl in SCORES)
            res["total"][i] = t
            if best is None or t > best:
                best, bi = t, i
        res["raw"], res["norm"] = raw, norm
        for i in feasible:
            nm = _name(self.nodes[i])
            res["score"][nm] = {pl: str(raw[pl][i]) for pl in SCORES}
            res["finalscore"][nm] = {pl: str(norm[pl][i] * self.weights[pl]) for pl in SCORES}
        res["selected"] = bi
        if commit:
            self.assume(pod, bi)
        return res

    # ----------------------------------------------------------- annotations
    def annotations(self, res, nominated: Optional[int] = None) -> Dict[str, str]:
        """store.GetStoredResult for a pod scheduled by the default profile (bind assumed successful).
        `nominated`: the node DefaultPreemption nominated (k8s_preemption.preempt), if any."""
        sel = self.nodes[res["selected"]] if res["selected"] is not None else None
        post = {}
        if sel is None:
            # FitError -> RunPostFilterPlugins: DefaultPreemption (wrapped) records every node of the
            # NodeToStatusMap, the nominated one with PostFilterNominatedMessage (store.go:436-456).
            if res["status"] == "prefilter":
                post = {_name(n): {} for n in self.nodes}
            else:
                post = {nm: {} for nm in res["filter"]}
            if nominated is not None:
                post[_name(self.nodes[nominated])] = {"DefaultPreemption": "preemption victim"}
        out = {
            "scheduler-simulator/prefilter-result": go_json(res["prefilter_result"]),
            "scheduler-simulator/prefilter-result-status": go_json(res["prefilter_status"]),
            "scheduler-simulator/filter-result": go_json(res["filter"]),
            "scheduler-simulator/postfilter-result": go_json(post),
            "scheduler-simulator/prescore-result": go_json(res["prescore"]),
            "scheduler-simulator/score-result": go_json(res["score"]),
            "scheduler-simulator/finalscore-result": go_json(res["finalscore"]),
            "scheduler-simulator/reserve-result": go_json({"VolumeBinding": "success"} if sel else {}),
            "scheduler-simulator/permit-result": "{}",
            "scheduler-simulator/permit-result-timeout": "{}",
            "scheduler-simulator/prebind-result": go_json({"VolumeBinding": "success"} if sel else {}),
            "scheduler-simulator/bind-result": go_json({"DefaultBinder": "success"} if sel else {}),
            "scheduler-simulator/selected-node": _name(sel) if sel else "",
        }
        return out


def go_json_string(s: str) -> str:
    """encoding/json string encoding with HTML escaping (Go's default Marshal)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_json(v) -> str:
    """json.Marshal for map[string]string / map[string]map[string]string / map[string][]string."""
    if isinstance(v, dict):
        return "{" + ",".join(go_json_string(k) + ":" + go_json(v[k]) for k in sorted(v)) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(go_json(x) for x in v) + "]"
    return go_json_string(str(v))
