"""Seeded random clusters whose pending pods carry every kind of PodTopologySpread /
InterPodAffinity program the device path supports (test infrastructure).

Unlike the BASELINE generators (kss/synth.py: one zone constraint, one hostname constraint,
one app selector), these mix per pod:

  * 0-2 DoNotSchedule and 0-3 ScheduleAnyway constraints over hostname (unique key),
    zone / rack (shared keys, some nodes without the label) and instance type, maxSkew
    1-3, NodeAffinityPolicy / NodeTaintsPolicy Honor or Ignore, matchLabels or
    matchExpressions selectors;
  * required pod affinity and anti-affinity, preferred affinity and anti-affinity with
    weights, over the same keys;
  * bound pods carrying required anti-affinity (existing-pod filter), and required /
    preferred (anti-)affinity terms (existing-pod scores);
  * NoExecute / NoSchedule / PreferNoSchedule taints, tolerations, nodeSelector, required
    and preferred node affinity, spec.nodeName, a second namespace, small pod limits;
  * every node-affinity operator (In / NotIn / Exists / DoesNotExist / Gt / Lt), matchFields
    metadata.name In (PreFilterResult) and NotIn, an extended resource (example.com/gpu) on
    some nodes, ephemeral-storage requests against small disks, init-container requests.

A quarter of the pods with constraints also carry a second constraint of the same kind on
a key they already use (v1.26 keys the counts by topology pair: test_spread_same_key.py).
"""
import random
from typing import Dict, List, Tuple

ZONES = ["z0", "z1", "z2", "z3"]
RACKS = ["r%d" % i for i in range(6)]
ITYPES = ["small", "large", "gpu"]
K_HOST = "kubernetes.io/hostname"
K_ZONE = "topology.kubernetes.io/zone"
K_RACK = "example.com/rack"
K_ITYPE = "node.kubernetes.io/instance-type"
K_TIER = "example.com/tier"
K_ACCEL = "example.com/accelerator"
R_GPU = "example.com/gpu"
# extended (scalar) resources beyond the first, used with make(..., n_extended=k)
R_MORE = ["example.com/fpga", "hugepages-2Mi", "vendor.io/nic"]
APPS = 6


def _node(i: int, r: random.Random, extended: bool = True) -> dict:
    name = "n%05d" % i
    labels: Dict[str, str] = {}
    if r.random() >= 0.02:
        labels[K_HOST] = name
        if r.random() >= 0.05:
            labels[K_ZONE] = ZONES[r.randrange(len(ZONES))]
        if r.random() >= 0.10:
            labels[K_RACK] = RACKS[r.randrange(len(RACKS))]
        labels[K_ITYPE] = ITYPES[r.randrange(len(ITYPES))]
        if r.random() < 0.8:
            labels[K_TIER] = str(r.randint(0, 30))
        if r.random() < 0.3:
            labels[K_ACCEL] = "yes"
    taints = []
    if r.random() < 0.10:
        taints.append({"key": "dedicated", "value": "infra", "effect": "NoSchedule"})
    if r.random() < 0.04:
        taints.append({"key": "evict", "value": "yes", "effect": "NoExecute"})
    if r.random() < 0.08:
        taints.append({"key": "spot", "value": "true", "effect": "PreferNoSchedule"})
    cores = r.choice([2, 4, 8, 16])
    spec: Dict = {}
    if taints:
        spec["taints"] = taints
    if r.random() < 0.02:
        spec["unschedulable"] = True
    alloc = {"cpu": str(cores), "memory": "%dGi" % (cores * 4),
             "ephemeral-storage": r.choice(["50Gi", "50Gi", "1Gi"]), "pods": str(r.choice([4, 8, 16, 110]))}
    if r.random() < 0.3 and extended:
        alloc[R_GPU] = r.choice(["1", "2", "4"])
    return {"metadata": {"name": name, "labels": labels}, "spec": spec, "status": {"allocatable": alloc}}


def _more_extended(nodes, pods, bound, k: int, r: random.Random):
    """k - 1 more extended resources: on some nodes (as allocatable), asked for by some pods."""
    for res in R_MORE[:max(k - 1, 0)]:
        for n in nodes:
            if r.random() < 0.4:
                n["status"]["allocatable"][res] = r.choice(["1", "2", "3"]) if "/" in res else r.choice(["4Mi", "8Mi"])
        for p in pods + bound:
            if r.random() < 0.15:
                req = p["spec"]["containers"][0]["resources"]["requests"]
                req[res] = "1" if "/" in res else r.choice(["2Mi", "4Mi"])
                if r.random() < 0.1:
                    req[res] = "0" if "/" in res else "0Mi"  # a zero request: fitsRequest skips it


def _sel(r: random.Random) -> dict:
    if r.random() < 0.7:
        return {"matchLabels": {"app": "a%d" % r.randrange(APPS)}}
    vals = sorted({"a%d" % r.randrange(APPS) for _ in range(2)})
    return {"matchExpressions": [{"key": "app", "operator": "In", "values": vals}]}


def _term(r: random.Random, keys: List[str]) -> dict:
    return {"labelSelector": _sel(r), "topologyKey": r.choice(keys)}


def _requests(r: random.Random, extended: bool = True) -> dict:
    if r.random() < 0.05:
        return {}
    req = {"cpu": "%dm" % r.choice([100, 250, 500, 1000]), "memory": "%dMi" % r.choice([128, 256, 512, 1024])}
    if r.random() < 0.1:
        req["ephemeral-storage"] = r.choice(["256Mi", "768Mi"])
    if r.random() < 0.1 and extended:
        req[R_GPU] = "1"
    return req


def _node_expr(r: random.Random) -> dict:
    u = r.randrange(6)
    if u == 0:
        return {"key": K_ZONE, "operator": "In", "values": sorted(set(r.sample(ZONES, 2)))}
    if u == 1:
        return {"key": K_ITYPE, "operator": "NotIn", "values": [r.choice(ITYPES)]}
    if u == 2:
        return {"key": K_ACCEL, "operator": r.choice(["Exists", "DoesNotExist"])}
    if u == 3:
        return {"key": K_TIER, "operator": r.choice(["Gt", "Lt"]), "values": [str(r.randint(5, 25))]}
    if u == 4:
        return {"key": K_RACK, "operator": "NotIn", "values": sorted(set(r.sample(RACKS, 3)))}
    return {"key": K_RACK, "operator": "In", "values": [r.choice(RACKS)]}


def _bound(i: int, k: int, node: str, r: random.Random, extended: bool = True) -> dict:
    spec: Dict = {"nodeName": node, "containers": [{"name": "c", "resources": {"requests": _requests(r, extended)}}]}
    aff: Dict = {}
    u = r.random()
    if u < 0.15:
        aff["podAntiAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": [_term(r, [K_HOST, K_ZONE])]}
    elif u < 0.30:
        aff["podAffinity"] = {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": r.randint(1, 100), "podAffinityTerm": _term(r, [K_ZONE, K_RACK, K_HOST])}]}
    elif u < 0.38:
        aff["podAntiAffinity"] = {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": r.randint(1, 100), "podAffinityTerm": _term(r, [K_ZONE, K_RACK])}]}
    elif u < 0.45:
        aff["podAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": [_term(r, [K_ZONE, K_RACK])]}
    if aff:
        spec["affinity"] = aff
    ns = "default" if r.random() < 0.9 else "other"
    return {"metadata": {"name": "b%05d-%d" % (i, k), "namespace": ns, "labels": {"app": "a%d" % r.randrange(APPS)}},
            "spec": spec}


def _spread(r: random.Random, key: str, hard: bool) -> dict:
    c = {"maxSkew": r.randint(1, 3), "topologyKey": key,
         "whenUnsatisfiable": "DoNotSchedule" if hard else "ScheduleAnyway", "labelSelector": _sel(r)}
    if r.random() < 0.25:
        c["nodeAffinityPolicy"] = r.choice(["Honor", "Ignore"])
    if r.random() < 0.25:
        c["nodeTaintsPolicy"] = r.choice(["Honor", "Ignore"])
    return c


def _pending(j: int, r: random.Random, node_names: List[str], extended: bool = True) -> dict:
    spec: Dict = {"containers": [{"name": "c", "resources": {"requests": _requests(r, extended)}}]}
    if r.random() < 0.08:
        spec["initContainers"] = [{"name": "i", "resources": {"requests": {"cpu": r.choice(["1", "2500m"])}}}]
    tols = []
    if r.random() < 0.3:
        tols.append({"key": "dedicated", "operator": "Exists", "effect": "NoSchedule"})
    if r.random() < 0.2:
        tols.append({"key": "evict", "operator": "Equal", "value": "yes", "effect": "NoExecute"})
    if r.random() < 0.3:
        tols.append({"key": "spot", "operator": "Exists", "effect": "PreferNoSchedule"})
    if tols:
        spec["tolerations"] = tols
    if r.random() < 0.1:
        spec["nodeSelector"] = {K_ITYPE: r.choice(ITYPES)}
    aff: Dict = {}
    na: Dict = {}
    u = r.random()
    if u < 0.15:
        terms = [{"matchExpressions": [_node_expr(r) for _ in range(r.choice([1, 1, 2]))]}
                 for _ in range(r.choice([1, 1, 2]))]
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
    elif u < 0.18:  # PreFilterResult: one node name per term (the field selector takes one value)
        terms = [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": [r.choice(node_names)]}]}
                 for _ in range(r.choice([1, 2, 3]))]
        if r.random() < 0.5:
            terms[0]["matchExpressions"] = [_node_expr(r)]
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
    elif u < 0.20:
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [{"matchFields": [
            {"key": "metadata.name", "operator": "NotIn", "values": [r.choice(node_names)]}]}]}
    if r.random() < 0.2:
        na["preferredDuringSchedulingIgnoredDuringExecution"] = [
            {"weight": r.randint(1, 100), "preference": {"matchExpressions": [_node_expr(r)]}}
            for _ in range(r.choice([1, 1, 2]))]
    if na:
        aff["nodeAffinity"] = na
    hard = r.sample([K_ZONE, K_RACK, K_HOST], r.choice([0, 0, 1, 1, 2]))
    soft = r.sample([K_ZONE, K_RACK, K_HOST, K_ITYPE], r.choice([0, 1, 1, 2, 3]))
    if hard and r.random() < 0.25:  # a second DoNotSchedule constraint on a key already used
        hard.append(r.choice(hard))
    if soft and len(soft) < 4 and r.random() < 0.25:
        soft.append(r.choice(soft))
    tsc = [_spread(r, k, True) for k in hard] + [_spread(r, k, False) for k in soft]
    r.shuffle(tsc)
    if tsc:
        spec["topologySpreadConstraints"] = tsc
    pa: Dict = {}
    pn: Dict = {}
    if r.random() < 0.12:
        pa["requiredDuringSchedulingIgnoredDuringExecution"] = [_term(r, [K_ZONE, K_RACK])]
    if r.random() < 0.2:
        pn["requiredDuringSchedulingIgnoredDuringExecution"] = [_term(r, [K_HOST, K_ZONE])]
    if r.random() < 0.3:
        pa["preferredDuringSchedulingIgnoredDuringExecution"] = [
            {"weight": r.randint(1, 100), "podAffinityTerm": _term(r, [K_ZONE, K_RACK, K_HOST])}]
    if r.random() < 0.2:
        pn["preferredDuringSchedulingIgnoredDuringExecution"] = [
            {"weight": r.randint(1, 100), "podAffinityTerm": _term(r, [K_ZONE, K_RACK, K_ITYPE])}]
    if pa:
        aff["podAffinity"] = pa
    if pn:
        aff["podAntiAffinity"] = pn
    if aff:
        spec["affinity"] = aff
    if r.random() < 0.02:
        spec["nodeName"] = r.choice(node_names)
    ns = "default" if r.random() < 0.9 else "other"
    return {"metadata": {"name": "p%05d" % j, "namespace": ns, "labels": {"app": "a%d" % r.randrange(APPS)}},
            "spec": spec}


def make(seed: int, n_nodes: int, n_pods: int, bound_per_node: Tuple[int, int] = (0, 3), extended: bool = True,
         n_extended: int = 1, programs: bool = True):
    """(nodes, bound_pods, pending_pods) for one seed.  extended=False leaves the extended
    resources out; n_extended (1-4) adds more of them; programs=False strips every
    PodTopologySpread / InterPodAffinity term (pending and bound pods: a k_simple batch)."""
    r = random.Random(seed)
    nodes = [_node(i, r, extended) for i in range(n_nodes)]
    names = [n["metadata"]["name"] for n in nodes]
    bound = []
    for i, nm in enumerate(names):
        for k in range(r.randint(*bound_per_node)):
            bound.append(_bound(i, k, nm, r, extended))
    pods = [_pending(j, r, names, extended) for j in range(n_pods)]
    if extended and n_extended > 1:
        _more_extended(nodes, pods, bound, n_extended, r)
    if not programs:
        for p in pods + bound:
            p["spec"].pop("topologySpreadConstraints", None)
            aff = p["spec"].get("affinity")
            if aff:
                aff.pop("podAffinity", None)
                aff.pop("podAntiAffinity", None)
                if not aff:
                    p["spec"].pop("affinity")
    return nodes, bound, pods
