"""Hand-derived DefaultPreemption fixtures (test infrastructure).

Each pending pod selects one node group (nodeSelector group=G), so the nodes of the other
groups fail NodeAffinity (UnschedulableAndUnresolvable: never potential).  Nodes have 2 CPU;
the expectations follow SelectVictimsOnNode / pickOneNodeForPreemption (v1.26) by hand:

  G1 highest victim priority   a: low-1 (prio 1, 1000m, t0), low-2 (prio 1, 1000m, t10)
                               b: mid (prio 5, 1500m), low (prio 1, 500m)
       p1 (prio 10, 1000m): a: remove both, reprieve low-1 (2000 fits), low-2 evicted;
       b: reprieve mid fails (2500), low reprieved -> victims [mid].  Highest victim
       priority 1 < 5 -> nominate a, victims [a-low-2].
  G2 sum of priorities         d: two prio-1 pods of 1000m; e: one prio-1 pod of 2000m.
       p2 (prio 10, 1500m): d evicts both (each reprieve overflows), e evicts one; equal
       highest priority, sums 2(1 + 2^31) > 1 + 2^31 -> e.
  G3 latest earliest start     f: prio-1 pod 2000m started 2024-01-01; g: the same started
       2024-06-01.  p3: one victim each, equal sums and counts -> the later start: g.
  G4 no candidate              h: prio-100 pod of 2000m.  p4 (prio 10): no lower-priority
       pod -> FitError, nothing nominated.
  G1 again, preemptionPolicy Never: p5 is not eligible.
  G5 anti-affinity             i: low-priority app=x pod; j: prio-100 app=x pod.  p6 (prio 10,
       required anti-affinity to app=x per hostname) fails InterPodAffinity on both
       (Unschedulable); i: removing the pod clears the count, reprieving it fails -> victim;
       j has nothing to evict -> nominate i.
  G6 existing anti-affinity    k: low-priority pod with required anti-affinity to app=web per
       hostname.  p7 (app=web, prio 10) fails "existing pods anti-affinity" -> evict it -> k.
  G7 spread skew (hostname)    m: two low-priority app=y pods; n: prio-100 pod of 2000m.
       p8 (app=y, DoNotSchedule hostname maxSkew 1, prio 10): m 2 + 1 - 0 > 1 fails PTS, n
       fails Fit.  m: both removed -> 0 + 1 - 0 fits; reprieving either gives 2 > 1 -> two
       victims, in importance order (the earlier start first).
  G8 spread skew (zone)        zone za: q1 two low-priority app=z pods; zone zb: q2 with a
       prio-100 pod of 2000m.  p9 (app=z, DoNotSchedule zone maxSkew 1): za 2 + 1 - 0 > 1,
       q2 fails Fit.  q1: removing both gives za = 0 -> fits; each reprieve gives 2 > 1 ->
       two victims; nominate q1.
"""

G = "group"
HOST = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"


def node(name, group, zone=None):
    lb = {HOST: name, G: group}
    if zone:
        lb[ZONE] = zone
    return {"metadata": {"name": name, "labels": lb}, "spec": {},
            "status": {"allocatable": {"cpu": "2", "memory": "8Gi", "pods": "110"}}}


def pod(name, prio, cpu=None, node_name=None, start=None, group=None, labels=None, **spec):
    s = {"containers": [{"name": "c", "resources": {"requests": {"cpu": cpu} if cpu else {}}}], "priority": prio}
    if node_name:
        s["nodeName"] = node_name
    if group:
        s["nodeSelector"] = {G: group}
    s.update(spec)
    out = {"metadata": {"name": name, "namespace": "default", "labels": dict(labels or {})}, "spec": s}
    if start:
        out["status"] = {"startTime": start}
    return out


T0, T10 = "2024-01-01T00:00:00Z", "2024-01-01T00:00:10Z"


def _anti(app, key=HOST):
    return {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": app}}, "topologyKey": key}]}}


def _spread(app, key):
    return [{"maxSkew": 1, "topologyKey": key, "whenUnsatisfiable": "DoNotSchedule",
             "labelSelector": {"matchLabels": {"app": app}}}]


def fixture():
    nodes = [node("a", "g1"), node("b", "g1"), node("d", "g2"), node("e", "g2"), node("f", "g3"), node("g", "g3"),
             node("h", "g4"), node("i", "g5"), node("j", "g5"), node("k", "g6"), node("m", "g7"), node("n", "g7"),
             node("q1", "g8", zone="za"), node("q2", "g8", zone="zb")]
    bound = [pod("a-low-1", 1, "1000m", "a", T0), pod("a-low-2", 1, "1000m", "a", T10),
             pod("b-mid", 5, "1500m", "b", T0), pod("b-low", 1, "500m", "b", T0),
             pod("d-1", 1, "1000m", "d", T0), pod("d-2", 1, "1000m", "d", T0),
             pod("e-1", 1, "2000m", "e", T0),
             pod("f-1", 1, "2000m", "f", "2024-01-01T00:00:00Z"), pod("g-1", 1, "2000m", "g", "2024-06-01T00:00:00Z"),
             pod("h-1", 100, "2000m", "h", T0),
             pod("i-x", 1, "100m", "i", T0, labels={"app": "x"}), pod("j-x", 100, "100m", "j", T0, labels={"app": "x"}),
             pod("k-guard", 1, "100m", "k", T0, affinity=_anti("web")),
             pod("m-y1", 1, "100m", "m", T0, labels={"app": "y"}), pod("m-y2", 1, "100m", "m", T10, labels={"app": "y"}),
             pod("n-1", 100, "2000m", "n", T0),
             pod("q1-z1", 1, "100m", "q1", T10, labels={"app": "z"}), pod("q1-z2", 1, "100m", "q1", T0, labels={"app": "z"}),
             pod("q2-1", 100, "2000m", "q2", T0)]
    pods = [pod("p1", 10, "1000m", group="g1"),
            pod("p2", 10, "1500m", group="g2"),
            pod("p3", 10, "1500m", group="g3"),
            pod("p4", 10, "1000m", group="g4"),
            pod("p5", 10, "1000m", group="g1", preemptionPolicy="Never"),
            pod("p6", 10, "100m", group="g5", affinity=_anti("x")),
            pod("p7", 10, "100m", group="g6", labels={"app": "web"}),
            pod("p8", 10, "100m", group="g7", labels={"app": "y"}, topologySpreadConstraints=_spread("y", HOST)),
            pod("p9", 10, "100m", group="g8", labels={"app": "z"}, topologySpreadConstraints=_spread("z", ZONE))]
    expect = [("nominated", "a", ["a-low-2"]),
              ("nominated", "e", ["e-1"]),
              ("nominated", "g", ["g-1"]),
              ("no_candidate", None, []),
              ("not_eligible", None, []),
              ("nominated", "i", ["i-x"]),
              ("nominated", "k", ["k-guard"]),
              ("nominated", "m", ["m-y1", "m-y2"]),
              ("nominated", "q1", ["q1-z2", "q1-z1"])]
    return nodes, bound, pods, expect


# --------------------------------------------------------------------------------------
# Seeded saturated clusters: every node nearly full of pods of mixed priority (and start
# times), pending pods of higher and lower priority, some with a hostname / zone spread
# constraint or pod anti-affinity, a few with preemptionPolicy Never.
def saturated(seed: int, n_nodes: int, n_pods: int):
    import random
    r = random.Random(seed)
    zones = ["z%d" % i for i in range(4)]
    nodes, bound, pods = [], [], []
    for i in range(n_nodes):
        name = "n%04d" % i
        cores = r.choice([2, 4, 8])
        lb = {HOST: name, ZONE: r.choice(zones)}
        nodes.append({"metadata": {"name": name, "labels": lb}, "spec": {},
                      "status": {"allocatable": {"cpu": str(cores), "memory": "%dGi" % (4 * cores),
                                                 "pods": str(r.choice([8, 16, 110]))}}})
        used = 0
        k = 0
        while used < cores * 1000 - 250:
            cpu = r.choice([250, 500, 1000, 1500])
            if used + cpu > cores * 1000:
                break
            used += cpu
            spec = {"nodeName": name, "priority": r.choice([0, 10, 10, 100, 1000]),
                    "containers": [{"name": "c", "resources": {"requests": {"cpu": "%dm" % cpu,
                                                                             "memory": "%dMi" % r.choice([256, 512])}}}]}
            if r.random() < 0.05:
                spec["affinity"] = _anti("a%d" % r.randrange(3))
            pod_ = {"metadata": {"name": "%s-b%d" % (name, k), "namespace": "default",
                                 "labels": {"app": "a%d" % r.randrange(3)}}, "spec": spec}
            if r.random() < 0.8:
                pod_["status"] = {"startTime": "2024-01-%02dT%02d:00:00Z" % (r.randint(1, 28), r.randint(0, 23))}
            bound.append(pod_)
            k += 1
    for j in range(n_pods):
        spec = {"priority": r.choice([0, 10, 100, 100, 1000, 5000]),
                "containers": [{"name": "c", "resources": {"requests": {"cpu": "%dm" % r.choice([500, 1000, 2000, 3000]),
                                                                         "memory": "512Mi"}}}]}
        u = r.random()
        if u < 0.15:
            spec["topologySpreadConstraints"] = _spread("a%d" % r.randrange(3), r.choice([HOST, ZONE]))
        elif u < 0.3:
            spec["affinity"] = _anti("a%d" % r.randrange(3), r.choice([HOST, ZONE]))
        if r.random() < 0.05:
            spec["preemptionPolicy"] = "Never"
        pods.append({"metadata": {"name": "p%04d" % j, "namespace": "default", "labels": {"app": "a%d" % r.randrange(3)}},
                     "spec": spec})
    return nodes, bound, pods
