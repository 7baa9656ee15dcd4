"""Hand-derived fixtures, one per filter branch and reason string (test infrastructure).

Every expectation below was worked out by hand from the upstream function it names
(kube-scheduler v1.26, the version the simulator vendors: reference go.mod
k8s.io/kubernetes v1.26.x), not produced by either oracle.  tests/test_edge_fixtures.py
checks both oracles (and the lazy annotation formatter) against them;
tests/test_gpu_edge_fixtures.py checks the device path through the C-ABI.

Each fixture is (nodes, bound, pods, expect) with one `expect` entry per pending pod,
scheduled in order (each AssumePod is visible to the next pod):

  filter   {node: None | (plugin, message)} -- None passes every filter plugin; a node left
           out was not evaluated (PreFilterResult); the annotation record then holds
           "passed" for every plugin before the failing one (runFilterPlugins stops there).
  selected node name, "" (unschedulable) or absent (decided by scores not derived here).
  extra    annotation keys compared as decoded JSON.
  pts      {node: (raw, normalized)} PodTopologySpread score pairs.
"""
import json

FILTERS = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
           "VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits", "VolumeBinding",
           "VolumeZone", "PodTopologySpread", "InterPodAffinity"]

HOST = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"
DEFAULT_SPREAD_SELECTOR_ANN = "kss.x-k8s.io/default-spread-selector"

M_UNSCHED = "node(s) were unschedulable"
M_NAME = "node(s) didn't match the requested node name"
M_AFF = "node(s) didn't match Pod's node affinity/selector"
M_PTS = "node(s) didn't match pod topology spread constraints"
M_PTS_LABEL = "node(s) didn't match pod topology spread constraints (missing required label)"
M_IPA_AFF = "node(s) didn't match pod affinity rules"
M_IPA_ANTI = "node(s) didn't match pod anti-affinity rules"
M_IPA_EXIST = "node(s) didn't satisfy existing pods anti-affinity rules"
M_PORTS = "node(s) didn't have free ports for the requested pod ports"


def node(name, zone=None, cpu="4", mem="8Gi", pods="110", eph="10Gi", extra=None, labels=None, taints=None,
         unschedulable=False, images=None):
    lb = {HOST: name}
    if zone is not None:
        lb[ZONE] = zone
    lb.update(labels or {})
    alloc = {"cpu": cpu, "memory": mem, "pods": pods, "ephemeral-storage": eph}
    alloc.update(extra or {})
    spec = {}
    if taints:
        spec["taints"] = taints
    if unschedulable:
        spec["unschedulable"] = True
    status = {"allocatable": alloc}
    if images:
        status["images"] = images
    return {"metadata": {"name": name, "labels": lb}, "spec": spec, "status": status}


def pod(name, requests=None, labels=None, node_name=None, init=None, annotations=None, **spec):
    s = {"containers": [{"name": "c", "resources": {"requests": dict(requests or {})}}]}
    if init:
        s["initContainers"] = [{"name": "i", "resources": {"requests": dict(init)}}]
    if node_name:
        s["nodeName"] = node_name
    s.update(spec)
    md = {"name": name, "namespace": "default", "labels": dict(labels or {})}
    if annotations:
        md["annotations"] = dict(annotations)
    return {"metadata": md, "spec": s}


def record(fail=None):
    """The filter-result record of one node: "passed" up to the failing plugin."""
    out = {}
    for pl in FILTERS:
        if fail is not None and pl == fail[0]:
            out[pl] = fail[1]
            return out
        out[pl] = "passed"
    return out


def filter_result(spec):
    return {n: record(f) for n, f in spec.items()}


def _sel(app):
    return {"matchLabels": {"app": app}}


def _req_na(*terms):
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": list(terms)}}}


# --------------------------------------------------------------------------------------
# NodeUnschedulable (nodeunschedulable/node_unschedulable.go Filter): spec.unschedulable
# fails unless the pod tolerates {node.kubernetes.io/unschedulable, NoSchedule}.
# NodeName (nodename/node_name.go Fits): spec.nodeName must equal the node's name.
def fx_unschedulable_and_nodename():
    nodes = [node("a", unschedulable=True), node("b"), node("c")]
    tol = [{"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"}]
    pods = [pod("p-plain"),
            pod("p-pinned", node_name="c"),
            pod("p-tolerates", tolerations=tol, node_name="a"),
            pod("p-pinned-unsched", node_name="a")]
    expect = [
        {"filter": {"a": ("NodeUnschedulable", M_UNSCHED), "b": None, "c": None}},
        {"filter": {"a": ("NodeUnschedulable", M_UNSCHED), "b": ("NodeName", M_NAME), "c": None}, "selected": "c"},
        {"filter": {"a": None, "b": ("NodeName", M_NAME), "c": ("NodeName", M_NAME)}, "selected": "a"},
        # NodeUnschedulable runs before NodeName: a fails on unschedulable, b and c on the name.
        {"filter": {"a": ("NodeUnschedulable", M_UNSCHED), "b": ("NodeName", M_NAME), "c": ("NodeName", M_NAME)},
         "selected": ""},
    ]
    return nodes, [], pods, expect


# --------------------------------------------------------------------------------------
# TaintToleration (tainttoleration/taint_toleration.go Filter, v1helper.FindMatchingUntoleratedTaint
# over NoSchedule + NoExecute): message "node(s) had untolerated taint {key: value}" for the
# first untolerated taint in the node's order.  PreferNoSchedule only scores: Score counts the
# untolerated PreferNoSchedule taints, NormalizeScore reverses (100 - 100*c/max).
def fx_taints():
    nodes = [node("a", taints=[{"key": "k1", "value": "v1", "effect": "NoSchedule"}]),
             node("b", taints=[{"key": "k2", "effect": "NoExecute"}]),
             node("c", taints=[{"key": "k3", "value": "v3", "effect": "PreferNoSchedule"}]),
             node("d"),
             node("e", taints=[{"key": "k3", "value": "v3", "effect": "PreferNoSchedule"},
                               {"key": "k1", "value": "other", "effect": "NoSchedule"},
                               {"key": "k2", "value": "x", "effect": "NoExecute"}])]
    tol_all = [{"key": "k1", "operator": "Equal", "value": "v1", "effect": "NoSchedule"},
               {"key": "k2", "operator": "Exists"}]
    pods = [pod("p-none"), pod("p-tolerates", tolerations=tol_all)]
    expect = [
        # c and d feasible; TaintToleration raw c=1 d=0 -> normalized c=0 d=100 (x3 weight decides).
        {"filter": {"a": ("TaintToleration", "node(s) had untolerated taint {k1: v1}"),
                    "b": ("TaintToleration", "node(s) had untolerated taint {k2: }"),
                    "c": None, "d": None,
                    "e": ("TaintToleration", "node(s) had untolerated taint {k1: other}")},
         "selected": "d"},
        # k1=v1 Equal tolerates a but not e's k1=other; Exists with no effect tolerates every k2.
        {"filter": {"a": None, "b": None, "c": None, "d": None,
                    "e": ("TaintToleration", "node(s) had untolerated taint {k1: other}")},
         "selected": "a"},  # a, b empty and untainted for scoring; a comes first; d holds p-none
    ]
    return nodes, [], pods, expect


# --------------------------------------------------------------------------------------
# NodeAffinity (nodeaffinity/node_affinity.go PreFilter + Filter; component-helpers
# nodeaffinity.NodeSelectorRequirementsAsSelector / matchFields): nodeSelector AND required
# terms; terms ORed, expressions ANDed; In / NotIn (absent key matches NotIn) / Exists /
# DoesNotExist / Gt / Lt (integer compare); matchFields metadata.name In narrows the node set
# in PreFilter (PreFilterResult -> nodes outside it are never evaluated); an empty
# intersection inside one term is "pod affinity terms conflict" (UnschedulableAndUnresolvable).
def fx_node_affinity():
    nodes = [node("a", labels={"env": "prod", "tier": "5"}),
             node("b", labels={"env": "dev", "tier": "10"}),
             node("c", labels={"tier": "3"}),
             node("d", labels={"env": "prod", "gpu": "yes", "tier": "20"})]

    def expr(key, op, *values):
        e = {"key": key, "operator": op}
        if values:
            e["values"] = list(values)
        return e

    def name_field(op, *values):
        return {"key": "metadata.name", "operator": op, "values": list(values)}

    F = ("NodeAffinity", M_AFF)
    pods, expect = [], []

    def case(name, want, selected=None, node_selector=None, extra=None, **aff_kw):
        kw = {}
        if aff_kw.get("terms") is not None:
            kw["affinity"] = _req_na(*aff_kw["terms"])
        if node_selector:
            kw["nodeSelector"] = node_selector
        pods.append(pod(name, **kw))
        e = {"filter": want}
        if selected is not None:
            e["selected"] = selected
        if extra:
            e["extra"] = extra
        expect.append(e)

    case("in", {"a": None, "b": F, "c": F, "d": None}, terms=[{"matchExpressions": [expr("env", "In", "prod")]}])
    case("notin", {"a": F, "b": None, "c": None, "d": F}, terms=[{"matchExpressions": [expr("env", "NotIn", "prod")]}])
    case("exists", {"a": F, "b": F, "c": F, "d": None}, selected="d",
         terms=[{"matchExpressions": [expr("gpu", "Exists")]}])
    case("dne", {"a": None, "b": None, "c": None, "d": F}, terms=[{"matchExpressions": [expr("gpu", "DoesNotExist")]}])
    case("gt", {"a": F, "b": None, "c": F, "d": None}, terms=[{"matchExpressions": [expr("tier", "Gt", "5")]}])
    case("lt", {"a": F, "b": F, "c": None, "d": F}, selected="c", terms=[{"matchExpressions": [expr("tier", "Lt", "5")]}])
    case("or-terms", {"a": F, "b": None, "c": F, "d": None},
         terms=[{"matchExpressions": [expr("env", "In", "dev")]}, {"matchExpressions": [expr("gpu", "Exists")]}])
    case("and-exprs", {"a": F, "b": F, "c": F, "d": None}, selected="d",
         terms=[{"matchExpressions": [expr("env", "In", "prod"), expr("tier", "Gt", "10")]}])
    case("selector-and-affinity", {"a": None, "b": F, "c": F, "d": F}, selected="a", node_selector={"env": "prod"},
         terms=[{"matchExpressions": [expr("tier", "Lt", "10")]}])
    case("selector-missing-key", {"a": F, "b": F, "c": F, "d": F}, selected="", node_selector={"zone": "x"})
    # matchFields metadata.name In -> PreFilterResult {b}; a, c and d are never evaluated.
    case("fields-in", {"b": None}, selected="b", terms=[{"matchFields": [name_field("In", "b")]}],
         extra={"scheduler-simulator/prefilter-result": {"NodeAffinity": ["b"]}})
    # Two values: PreFilter still narrows to {b, c}, but nodeSelectorRequirementsAsFieldSelector
    # accepts exactly one value per field requirement, so the term is a parse error and matches
    # no node (LazyErrorNodeSelector).
    case("fields-in-two-values", {"b": F, "c": F}, selected="", terms=[{"matchFields": [name_field("In", "b", "c")]}],
         extra={"scheduler-simulator/prefilter-result": {"NodeAffinity": ["b", "c"]}})
    # NotIn narrows nothing in PreFilter; the filter rejects a.
    case("fields-notin", {"a": F, "b": None, "c": None, "d": None},
         terms=[{"matchFields": [name_field("NotIn", "a")]}],
         extra={"scheduler-simulator/prefilter-result": {}})
    # fields and expressions ANDed in each term: PreFilterResult {a, b}; the expression rejects a.
    case("fields-and-expr", {"a": F, "b": None}, selected="b",
         terms=[{"matchFields": [name_field("In", "a")], "matchExpressions": [expr("env", "In", "dev")]},
                {"matchFields": [name_field("In", "b")], "matchExpressions": [expr("env", "In", "dev")]}],
         extra={"scheduler-simulator/prefilter-result": {"NodeAffinity": ["a", "b"]}})
    # union over terms: {a} | {d}
    case("fields-union", {"a": None, "d": None},
         terms=[{"matchFields": [name_field("In", "a")]}, {"matchFields": [name_field("In", "d")]}],
         extra={"scheduler-simulator/prefilter-result": {"NodeAffinity": ["a", "d"]}})
    # a term without a name field makes every node eligible (no PreFilterResult).
    case("fields-or-open-term", {"a": None, "b": F, "c": F, "d": None},
         terms=[{"matchFields": [name_field("In", "a")]}, {"matchExpressions": [expr("gpu", "Exists")]}],
         extra={"scheduler-simulator/prefilter-result": {}})
    # {a} & {b} = {} inside one term: PreFilter conflict; nothing is filtered.
    case("fields-conflict", {}, selected="",
         terms=[{"matchFields": [name_field("In", "a"), name_field("In", "b")]}],
         extra={"scheduler-simulator/prefilter-result-status": {"NodeAffinity": "pod affinity terms conflict"},
                "scheduler-simulator/postfilter-result": {"a": {}, "b": {}, "c": {}, "d": {}}})
    return nodes, [], pods, expect


# --------------------------------------------------------------------------------------
# NodeResourcesFit (noderesources/fit.go fitsRequest): "Too many pods" first (pod count +1 >
# allowed), then -- only if the pod requests anything -- cpu, memory, ephemeral-storage and
# each scalar resource in turn; the status message joins the reasons with ", ".  The pod
# request is max(sum(containers), max(initContainers)) (+ overhead) (computePodResourceRequest).
def fx_resources():
    GPU = "example.com/gpu"
    nodes = [node("a", pods="1", extra={GPU: "2"}),
             node("b", extra={GPU: "2"}),
             node("c", extra={GPU: "2"}),
             node("d", eph="256Mi", extra={GPU: "2"}),
             node("e", extra={GPU: "2"}),
             node("f"),
             node("g", cpu="100m", mem="256Mi", pods="1", extra={GPU: "2"}),
             node("h", extra={GPU: "2"})]
    bound = [pod("a-0", node_name="a"),
             pod("b-0", {"cpu": "3900m"}, node_name="b"),
             pod("c-0", {"memory": "7936Mi"}, node_name="c"),
             pod("e-0", {GPU: "2"}, node_name="e"),
             pod("g-0", node_name="g")]
    big = {"cpu": "200m", "memory": "512Mi", "ephemeral-storage": "512Mi", GPU: "1"}
    pods = [pod("p-big", big), pod("p-empty"), pod("p-init", {"cpu": "100m"}, init={"cpu": "3500m"})]
    TMP = ("NodeResourcesFit", "Too many pods")
    expect = [
        {"filter": {"a": TMP,
                    "b": ("NodeResourcesFit", "Insufficient cpu"),
                    "c": ("NodeResourcesFit", "Insufficient memory"),
                    "d": ("NodeResourcesFit", "Insufficient ephemeral-storage"),
                    "e": ("NodeResourcesFit", "Insufficient " + GPU),
                    "f": ("NodeResourcesFit", "Insufficient " + GPU),
                    "g": ("NodeResourcesFit", "Too many pods, Insufficient cpu, Insufficient memory"),
                    "h": None},
         "selected": "h"},
        # zero requests: only the pod count is checked
        {"filter": {"a": TMP, "b": None, "c": None, "d": None, "e": None, "f": None, "g": TMP, "h": None}},
        # effective request 3500m cpu (the init container): b has 100m free, g 100m total; h
        # holds p-big (200m) -> 3800m free passes.
        {"filter": {"a": TMP, "b": ("NodeResourcesFit", "Insufficient cpu"), "c": None, "d": None, "e": None,
                    "f": None, "g": ("NodeResourcesFit", "Too many pods, Insufficient cpu"), "h": None}},
    ]
    return nodes, bound, pods, expect


# --------------------------------------------------------------------------------------
# PodTopologySpread Filter (podtopologyspread/filtering.go): a node lacking a constraint's key
# fails with the "(missing required label)" reason; otherwise matchNum + selfMatch - minMatch
# must not exceed maxSkew.  Zones z1 = {a}, z2 = {b}; c has no zone label; a holds 2 x app=x.
def fx_spread_filter():
    nodes = [node("a", zone="z1"), node("b", zone="z2"), node("c")]
    bound = [pod("x0", labels={"app": "x"}, node_name="a"), pod("x1", labels={"app": "x"}, node_name="a")]
    con = [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule", "labelSelector": _sel("x")}]
    pods = [pod("p%d" % i, labels={"app": "x"}, topologySpreadConstraints=con) for i in range(3)]
    LBL = ("PodTopologySpread", M_PTS_LABEL)
    SKEW = ("PodTopologySpread", M_PTS)
    expect = [
        {"filter": {"a": SKEW, "b": None, "c": LBL}, "selected": "b"},  # z1 2+1-0 = 3 > 1
        {"filter": {"a": SKEW, "b": None, "c": LBL}, "selected": "b"},  # z1 2+1-1 = 2 > 1; z2 1+1-1 = 1
        {"filter": {"a": None, "b": None, "c": LBL}},                   # 2+1-2 = 1 on both zones
    ]
    return nodes, bound, pods, expect


# --------------------------------------------------------------------------------------
# System-defaulted PodTopologySpread (podtopologyspread/scoring.go with
# defaultConstraints = {hostname maxSkew 3, zone maxSkew 5} ScheduleAnyway, selector from
# helper.DefaultSelector -- here the kss annotation standing in for the owning workload).
# requireAllTopologies = false: a node without a zone label is NOT ignored; its pair
# (zone, "") still counts in the zone topoSize, and it scores the hostname term only.
#
# Zones z1 = {a, b}, z2 = {c}, d has no zone.  Bound app=web: 2 on a, 1 on c.
#   P1 (system default): topoSize zone 3 (z1, z2, ""), hostname 4 -> weights log 5, log 6.
#     a: 2 log 6 + 2 + 2 log 5 + 4 = 12.80 -> 13     b: 0 + 2 + 2 log 5 + 4 = 9.22 -> 9
#     c: log 6 + 2 + log 5 + 4 = 9.40 -> 9           d: 0 + 2 = 2
#     NormalizeScore 100 * (max + min - s) / max, max 13 min 2: 15, 46, 46, 100.
#   P2 (the same constraints written explicitly): requireAllTopologies -> d ignored (0, 0);
#     topoSize zone 2, hostname 3 -> weights log 4, log 5; P1 sits on d and is not counted.
#     a: 2 log 5 + 2 + 2 log 4 + 4 = 11.99 -> 12    b: 2 + 2 log 4 + 4 = 8.77 -> 9
#     c: log 5 + 2 + log 4 + 4 = 9.00 -> 9           max 12 min 9: 75, 100, 100.
def fx_system_default_spread():
    nodes = [node("a", zone="z1"), node("b", zone="z1"), node("c", zone="z2"), node("d")]
    web = {"app": "web"}
    bound = [pod("w0", labels=web, node_name="a"), pod("w1", labels=web, node_name="a"),
             pod("w2", labels=web, node_name="c")]
    ann = {DEFAULT_SPREAD_SELECTOR_ANN: json.dumps(_sel("web"))}
    explicit = [{"maxSkew": 3, "topologyKey": HOST, "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": _sel("web")},
                {"maxSkew": 5, "topologyKey": ZONE, "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": _sel("web")}]
    pods = [pod("p-default", labels=web, annotations=ann), pod("p-explicit", labels=web, topologySpreadConstraints=explicit)]
    allpass = {n: None for n in "abcd"}
    expect = [
        {"filter": allpass, "selected": "d", "pts": {"a": (13, 15), "b": (9, 46), "c": (9, 46), "d": (2, 100)}},
        {"filter": allpass, "pts": {"a": (12, 75), "b": (9, 100), "c": (9, 100), "d": (0, 0)}},
    ]
    return nodes, bound, pods, expect


# --------------------------------------------------------------------------------------
# InterPodAffinity Filter (interpodaffinity/filtering.go): satisfyPodAffinity, then
# satisfyPodAntiAffinity, then satisfyExistingPodsAntiAffinity, each with its own reason.
# Zones z1 = {a, b}, z2 = {c, d}; a holds app=db, c holds app=guard with required
# anti-affinity to app=web over zones.
def fx_interpod():
    nodes = [node("a", zone="z1"), node("b", zone="z1"), node("c", zone="z2"), node("d", zone="z2")]
    guard_aff = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": _sel("web"), "topologyKey": ZONE}]}}
    bound = [pod("db", {"cpu": "100m"}, labels={"app": "db"}, node_name="a"),
             pod("guard", {"cpu": "100m"}, labels={"app": "guard"}, node_name="c", affinity=guard_aff)]
    want_db = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": _sel("db"), "topologyKey": ZONE}]}}
    avoid_db = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": _sel("db"), "topologyKey": HOST}]}}
    want_nothing = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": _sel("nobody"), "topologyKey": ZONE}]}}
    pods = [pod("p-aff", labels={"app": "web"}, affinity=want_db),
            pod("p-web", labels={"app": "web"}),
            pod("p-anti", labels={"app": "cache"}, affinity=avoid_db),
            pod("p-none", labels={"app": "cache"}, affinity=want_nothing)]
    AFF = ("InterPodAffinity", M_IPA_AFF)
    EXIST = ("InterPodAffinity", M_IPA_EXIST)
    expect = [
        {"filter": {"a": None, "b": None, "c": AFF, "d": AFF}},
        {"filter": {"a": None, "b": None, "c": EXIST, "d": EXIST}},
        {"filter": {"a": ("InterPodAffinity", M_IPA_ANTI), "b": None, "c": None, "d": None}},
        # no pod matches the affinity term and the pod does not match its own term
        {"filter": {n: AFF for n in "abcd"}, "selected": ""},
    ]
    return nodes, bound, pods, expect


# --------------------------------------------------------------------------------------
# internal/cache/node_tree.go: zones in first-seen order, round-robin over zones, insertion
# order inside a zone; selectHost ties go to the lowest index in that order.  Input order
# n1(z1) n2(z1) n3(z2) n4(-) n5(z1) -> tree order n1 n3 n4 n2 n5.  Zero-request pods on
# identical nodes: each pod's AssumePod lowers its node's NodeResourcesFit score by 2
# (nonzero 100m / 200Mi: 97 -> 95 on 4 CPU / 8Gi), so five pods fill the nodes in tree
# order and the sixth returns to n1.
TREE_ORDER = ["n1", "n3", "n4", "n2", "n5"]


def fx_node_tree_order():
    nodes = [node("n1", zone="z1"), node("n2", zone="z1"), node("n3", zone="z2"), node("n4"), node("n5", zone="z1")]
    pods = [pod("p%d" % i) for i in range(6)]
    allpass = {n: None for n in TREE_ORDER}
    expect = [{"filter": allpass, "selected": s} for s in TREE_ORDER + ["n1"]]
    return nodes, [], pods, expect


# --------------------------------------------------------------------------------------
# NodePorts (nodeports/node_ports.go: PreFilter getContainerPorts over spec.containers, Filter
# fitsPorts -> framework.HostPortInfo.CheckConflict, reason ErrReason; NodeInfo.AddPod adds the
# pod's container host ports to UsedPorts).  HostPortInfo.sanitize: hostIP "" -> 0.0.0.0,
# protocol "" -> TCP; a wanted 0.0.0.0 port conflicts with the same protocol/port on any IP, a
# specific IP only with 0.0.0.0 or the same IP; hostPort 0 (containerPort only) never
# conflicts; init containers' ports are not collected in v1.26.
# Zero-request pods on identical 4-CPU / 8Gi nodes: NodeResourcesFit is 97 / 95 / 92 with
# 0 / 1 / 2 pods on the node (non-zero defaults 100m / 200Mi), every other score is equal.
def _ports(*pp):
    return [dict(zip(("hostPort", "protocol", "hostIP", "containerPort"), p)) for p in pp]


def _cpod(name, ports, node_name=None, init_ports=None):
    spec = {"containers": [{"name": "c", "resources": {"requests": {}}, "ports": ports}]}
    if init_ports:
        spec["initContainers"] = [{"name": "i", "resources": {"requests": {}}, "ports": init_ports}]
    return pod(name, node_name=node_name, **spec)


def fx_node_ports():
    nodes = [node("a"), node("b"), node("c"), node("d")]
    bound = [_cpod("web-a", _ports((8080, "", "", 80)), node_name="a"),
             _cpod("dns-b", _ports((53, "UDP", "10.0.0.2", 53)), node_name="b"),
             _cpod("x-c", _ports((9090, "TCP", "10.0.0.3", 9090)), node_name="c")]
    pods = [_cpod("p-8080", _ports((8080, "TCP", "", 8080), (0, "", "", 9000))),  # 0.0.0.0:8080 vs a
            _cpod("p-8080-again", _ports((8080, "", "", 8080))),                    # a, and d after p-8080
            _cpod("p-udp53-any", _ports((53, "UDP", "", 53))),                      # any IP: b's 10.0.0.2
            _cpod("p-specific", _ports((9090, "TCP", "10.0.0.3", 1), (53, "UDP", "10.0.0.2", 2))),
            _cpod("p-tcp53", _ports((53, "TCP", "", 53)), init_ports=_ports((8080, "", "", 1)))]
    P = ("NodePorts", M_PORTS)
    expect = [
        {"filter": {"a": P, "b": None, "c": None, "d": None}, "selected": "d"},          # Fit 95 95 97
        {"filter": {"a": P, "b": None, "c": None, "d": P}, "selected": "b"},             # tie 95: b first
        {"filter": {"a": None, "b": P, "c": None, "d": None}, "selected": "a"},          # tie 95: a first
        # 10.0.0.3:9090 vs c (same IP); 10.0.0.2/UDP/53 vs b (same IP) and vs a's 0.0.0.0/UDP/53
        {"filter": {"a": P, "b": P, "c": P, "d": None}, "selected": "d"},
        # TCP 53 conflicts with no UDP entry; the init container's 8080 is not collected
        {"filter": {"a": None, "b": None, "c": None, "d": None}, "selected": "c"},      # Fit 92 92 95 92
    ]
    return nodes, bound, pods, expect


# --------------------------------------------------------------------------------------
# ImageLocality (imagelocality/image_locality.go Score): calculatePriority(sumImageScores,
# len(Containers)) = 100 * (clamp(sum, 23Mi, 1000Mi * #containers) - 23Mi) / (max - 23Mi)
# (int64), sum over containers of scaledImageScore = int64(float64(size) * NumNodes/N) for
# the node's ImageStates[normalizedImageName(image)] (":latest" appended when the name has
# no tag after its last "/").  v1.26 cache (cache.go addNodeImageStates /
# createImageStateSummary): the size is the first adding node's SizeBytes and NumNodes is
# copied when the node is added (input order a, b, c, d): a app:v1 (300Mi, 1) base:latest
# (100Mi, 1); b app:v1 (300Mi -- b's own 999Mi is ignored --, 2); c base:latest (100Mi, 2).
MI = 1024 * 1024


def fx_image_locality():
    nodes = [node("a", images=[{"names": ["app:v1"], "sizeBytes": 300 * MI},
                               {"names": ["base:latest"], "sizeBytes": 100 * MI}]),
             node("b", images=[{"names": ["app:v1"], "sizeBytes": 999 * MI}]),
             node("c", images=[{"names": ["base:latest"], "sizeBytes": 100 * MI}]),
             node("d")]

    def ipod(name, *images):
        return pod(name, containers=[{"name": "c%d" % i, "image": im, "resources": {"requests": {}}}
                                     for i, im in enumerate(images)])
    pods = [ipod("p-app", "app:v1"),                         # a 75Mi -> 5, b 150Mi -> 12
            ipod("p-base", "base"),                          # base:latest: a 25Mi -> 0, c 50Mi -> 2
            ipod("p-two", "app:v1", "registry:5000/base"),   # 2 containers, max 2000Mi: a 2, b 6
            ipod("p-app-twice", "app:v1", "app:v1")]         # a 150Mi -> 6, b 300Mi -> 14
    # Totals differ by NodeResourcesFit + ImageLocality only.  Non-zero defaults apply per
    # container (100m / 200Mi each), so a two-container pod requests 200m / 400Mi.
    allpass = {n: None for n in "abcd"}
    expect = [
        {"filter": allpass, "selected": "b", "il": {"a": 5, "b": 12, "c": 0, "d": 0}},   # Fit 97 everywhere
        {"filter": allpass, "selected": "c", "il": {"a": 0, "b": 0, "c": 2, "d": 0}},    # Fit 97 95 97 97
        # Fit 95 92 92 95 (b, c: 100m + 200m): totals 97 98 92 95
        {"filter": allpass, "selected": "b", "il": {"a": 2, "b": 6, "c": 0, "d": 0}},
        # Fit 95 87 92 95 (b: 300m + 200m): totals 101 101 92 95, the tie goes to a
        {"filter": allpass, "selected": "a", "il": {"a": 6, "b": 14, "c": 0, "d": 0}},
    ]
    return nodes, [], pods, expect


FIXTURES = {
    "unschedulable_and_nodename": fx_unschedulable_and_nodename,
    "taints": fx_taints,
    "node_affinity": fx_node_affinity,
    "resources": fx_resources,
    "spread_filter": fx_spread_filter,
    "system_default_spread": fx_system_default_spread,
    "interpod": fx_interpod,
    "node_tree_order": fx_node_tree_order,
    "node_ports": fx_node_ports,
    "image_locality": fx_image_locality,
}


def check_expect(ann, exp, pts=None, where=""):
    """Compare one pod's annotations (and optional PTS (raw, norm) per node) with `exp`."""
    got = json.loads(ann["scheduler-simulator/filter-result"])
    assert got == filter_result(exp["filter"]), where
    if "selected" in exp:
        assert ann["scheduler-simulator/selected-node"] == exp["selected"], where
    for k, v in (exp.get("extra") or {}).items():
        assert json.loads(ann[k]) == v, (where, k)
    if "il" in exp:
        sc = json.loads(ann["scheduler-simulator/score-result"])
        for n, v in exp["il"].items():
            assert sc[n]["ImageLocality"] == str(v), (where, n, sc[n]["ImageLocality"])
    if "pts" in exp and pts is not None:
        for n, (raw, norm) in exp["pts"].items():
            assert pts[n] == (raw, norm), (where, n, pts[n])
