"""Seeded synthetic clusters, as Kubernetes-shaped objects.

SplitMix64 with seed 0x5EED0000 + config id.  Every node and pod consumes a FIXED
number of draws, so the C++ generator (csrc/kss_synth.cpp, which emits the SoA
directly for bench-scale configs) produces the same cluster; tests compare the
two through the oracle.  The object form can also be written in the simulator's
ResourcesForSnap JSON shape (simulator/snapshot/snapshot.go:32-41) and imported
into the reference with POST /api/v1/import where Go is available.

Configs (BASELINE.json):
  1: 100 nodes / 1,000 pods, default profile
  2: 5,000 nodes / 10,000 pods, default profile
  3: 5,000 nodes in 3 zones, 2 pre-bound pods per node from 100 apps, pending pods
     with zone DoNotSchedule spread, hostname ScheduleAnyway spread, hostname
     anti-affinity, preferred zone affinity, zone self-affinity
  4: 100,000 nodes / 20,000 pods, default profile + zone DoNotSchedule spread
  5: one scenario of the 4,096 x (1,000 nodes / 1,000 pods) sweep (seed + scenario)
"""
from __future__ import annotations

from typing import Dict, List, Tuple

M64 = (1 << 64) - 1
SEED_BASE = 0x5EED0000
DEFAULT_SIZES = {1: (100, 1000), 2: (5000, 10000), 3: (5000, 10000), 4: (100000, 20000), 5: (1000, 1000)}

CORES = (4, 8, 16, 32, 64)
INSTANCE = ("small", "medium", "large", "xlarge")
ZONES = ("zone-a", "zone-b", "zone-c")
POD_CPU = ("100m", "250m", "500m", "1", "2")
POD_MEM = ("128Mi", "256Mi", "512Mi", "1Gi", "2Gi", "4Gi")


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def rnd(self, n: int) -> int:
        return self.next() % n


def cores_of(c: int) -> int:
    return 4 if c < 1 else 8 if c < 4 else 16 if c < 7 else 32 if c < 9 else 64


def make_node(i: int, r: SplitMix64) -> dict:
    c = r.rnd(10)
    mm = r.rnd(2)
    it = r.rnd(4)
    gen = 1 + r.rnd(5)
    ded = r.rnd(100) < 10
    spot = r.rnd(100) < 5
    uns = r.rnd(100) < 2
    cores = cores_of(c)
    mult = 8 if mm else 4
    name = "node-%06d" % i
    taints = []
    if ded:
        taints.append({"key": "dedicated", "value": "gpu", "effect": "NoSchedule"})
    if spot:
        taints.append({"key": "spot", "value": "true", "effect": "PreferNoSchedule"})
    node = {
        "metadata": {"name": name, "labels": {
            "kubernetes.io/hostname": name,
            "topology.kubernetes.io/zone": ZONES[i % 3],
            "node.kubernetes.io/instance-type": INSTANCE[it],
            "example.com/gen": str(gen),
        }},
        "spec": {"taints": taints} if taints else {},
        "status": {"allocatable": {"cpu": str(cores), "memory": "%dGi" % (cores * mult),
                                   "ephemeral-storage": "100Gi", "pods": "110"}},
    }
    if uns:
        node["spec"]["unschedulable"] = True
    return node


def _app_sel(k: int) -> dict:
    return {"matchLabels": {"app": "app-%d" % (k % 100)}}


def make_pod(j: int, r: SplitMix64, config: int) -> dict:
    noreq = r.rnd(100) < 5
    ci = r.rnd(5)
    mi = r.rnd(6)
    tded = r.rnd(100) < 10
    tspot = r.rnd(100) < 30
    sel = r.rnd(100) < 20
    sit = r.rnd(4)
    raff = r.rnd(100) < 20
    rk = r.rnd(2)
    z1 = r.rnd(3)
    z2o = r.rnd(2)
    has_pref = r.rnd(100) < 30
    npref = 1 + r.rnd(3)
    prefs = [(1 + r.rnd(100), r.rnd(3), r.rnd(5)) for _ in range(3)]
    app = pz = ph = anti = pref = selfaff = None
    if config == 3:
        app = r.rnd(100)
        pz = r.rnd(100) < 50
        ph = r.rnd(100) < 50
        anti = r.rnd(100) < 30
        pref = r.rnd(100) < 30
        selfaff = r.rnd(100) < 10
    elif config == 4:
        app = r.rnd(100)
        pz = r.rnd(100) < 50

    spec: Dict = {"containers": [{"name": "c0", "resources": {
        "requests": {} if noreq else {"cpu": POD_CPU[ci], "memory": POD_MEM[mi]}}}]}
    tols = []
    if tded:
        tols.append({"key": "dedicated", "operator": "Equal", "value": "gpu", "effect": "NoSchedule"})
    if tspot:
        tols.append({"key": "spot", "operator": "Exists", "effect": "PreferNoSchedule"})
    if tols:
        spec["tolerations"] = tols
    if sel:
        spec["nodeSelector"] = {"node.kubernetes.io/instance-type": INSTANCE[sit]}
    na: Dict = {}
    if raff:
        if rk == 0:
            expr = {"key": "topology.kubernetes.io/zone", "operator": "In",
                    "values": [ZONES[z1], ZONES[(z1 + 1 + z2o) % 3]]}
        else:
            expr = {"key": "example.com/gen", "operator": "Gt", "values": ["2"]}
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [{"matchExpressions": [expr]}]}
    if has_pref:
        terms = []
        for t in range(npref):
            w, k, v = prefs[t]
            if k == 0:
                expr = {"key": "node.kubernetes.io/instance-type", "operator": "In", "values": [INSTANCE[v % 4]]}
            elif k == 1:
                expr = {"key": "topology.kubernetes.io/zone", "operator": "In", "values": [ZONES[v % 3]]}
            else:
                expr = {"key": "example.com/gen", "operator": "Lt", "values": [str(1 + v)]}
            terms.append({"weight": w, "preference": {"matchExpressions": [expr]}})
        na["preferredDuringSchedulingIgnoredDuringExecution"] = terms
    aff: Dict = {}
    if na:
        aff["nodeAffinity"] = na
    labels: Dict[str, str] = {}
    if app is not None:
        labels["app"] = "app-%d" % app
        tsc = []
        if pz:
            tsc.append({"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone",
                        "whenUnsatisfiable": "DoNotSchedule", "labelSelector": _app_sel(app)})
        if ph:
            tsc.append({"maxSkew": 1, "topologyKey": "kubernetes.io/hostname",
                        "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": _app_sel(app)})
        if tsc:
            spec["topologySpreadConstraints"] = tsc
        if anti:
            aff["podAntiAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": _app_sel(app), "topologyKey": "kubernetes.io/hostname"}]}
        pa: Dict = {}
        if pref:
            pa["preferredDuringSchedulingIgnoredDuringExecution"] = [
                {"weight": 50, "podAffinityTerm": {"labelSelector": _app_sel(app + 1),
                                                   "topologyKey": "topology.kubernetes.io/zone"}}]
        if selfaff:
            pa["requiredDuringSchedulingIgnoredDuringExecution"] = [
                {"labelSelector": _app_sel(app), "topologyKey": "topology.kubernetes.io/zone"}]
        if pa:
            aff["podAffinity"] = pa
    if aff:
        spec["affinity"] = aff
    return {"metadata": {"name": "pod-%06d" % j, "namespace": "default", "labels": labels}, "spec": spec}


def make_cluster(config: int, n_nodes: int = 0, n_pods: int = 0, seed: int = -1) -> Tuple[List[dict], List[dict], List[dict]]:
    """Returns (nodes, bound_pods, pending_pods)."""
    dn, dp = DEFAULT_SIZES[config]
    n_nodes = n_nodes or dn
    n_pods = n_pods or dp
    if seed < 0:
        seed = SEED_BASE + config
    r = SplitMix64(seed)
    nodes = [make_node(i, r) for i in range(n_nodes)]
    bound = []
    if config == 3:
        for i in range(n_nodes):
            for k in range(2):
                app = r.rnd(100)
                bound.append({"metadata": {"name": "ex-%06d-%d" % (i, k), "namespace": "default",
                                           "labels": {"app": "app-%d" % app}},
                              "spec": {"nodeName": nodes[i]["metadata"]["name"],
                                       "containers": [{"name": "c0", "resources": {
                                           "requests": {"cpu": "100m", "memory": "128Mi"}}}]}})
    pods = [make_pod(j, r, config) for j in range(n_pods)]
    return nodes, bound, pods


def to_resources_for_snap(nodes, bound, pods) -> dict:
    """simulator/snapshot ResourcesForSnap JSON shape (snapshot.go:32-41)."""
    return {"pods": bound + pods, "nodes": nodes, "pvs": [], "pvcs": [], "storageClasses": [],
            "priorityClasses": [], "schedulerConfig": None, "namespaces": [{"metadata": {"name": "default"}}]}
