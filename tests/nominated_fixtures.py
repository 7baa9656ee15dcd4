"""Hand-derived fixture for nominated pods (test data, derived from the v1.26 rules the oracles
restate: runtime/framework.go RunFilterPluginsWithNominatedPods / addNominatedPods,
schedule_one.go findNodesThatFitPod -> evaluateNominatedNode, assume -> DeleteNominatedPodIfExists).

Three nodes of 4 CPUs; n1 holds a 1-CPU pod, n3 a 3-CPU pod.  The nominator holds "big" (priority
100, 3 CPUs) on n2 and "mid" (priority 50, 1 CPU) on n3 -- as a preemption would have left them.
Pods are scheduled in index order:

  0 low  (prio 0, 2 CPUs)   n2 fails NodeResourcesFit in the first pass (big's 3 CPUs added), n3
                            is full anyway -> n1.
  1 aff  (prio 0, 0.1 CPU, required pod affinity to app=big on the hostname key, not matching
         itself)            n1: InterPodAffinity; n2: the first pass passes (big counts for the
                            affinity), the second fails InterPodAffinity; n3: the first pass fails
                            NodeResourcesFit (mid fills it) -> unschedulable.
  2 eq   (prio 50, 0.5 CPU) big (100) and mid (50 >= 50) both count: n3 fails NodeResourcesFit;
                            n1 and n2 pass; scoring sees no nominee: n2 (empty) wins.
  3 high (prio 200, 2 CPUs) no nominee counts (both below 200): n2 has 3.5 CPUs free -> n2.
  4 mid  (nominated to n3)  PreferNominatedNode: n3 alone is evaluated and fits -> n3; its
                            nomination leaves the nominator.
  5 big  (nominated to n2)  n2 has 1.5 CPUs free: fails; the full search finds nothing ->
                            unschedulable, the nomination stays (no PostFilter here).
"""


def _node(name):
    return {"metadata": {"name": name, "labels": {"kubernetes.io/hostname": name}},
            "status": {"allocatable": {"cpu": "4", "memory": "16Gi", "pods": "110"}}}


def _pod(name, cpu, prio, labels=None, node=None, affinity=None):
    p = {"metadata": {"name": name, "namespace": "default", "labels": dict(labels or {})},
         "spec": {"priority": prio, "containers": [{"name": "c", "image": "busybox",
                                                     "resources": {"requests": {"cpu": cpu, "memory": "64Mi"}}}]}}
    if node:
        p["spec"]["nodeName"] = node
    if affinity:
        p["spec"]["affinity"] = affinity
    return p


def fixture():
    nodes = [_node("n1"), _node("n2"), _node("n3")]
    bound = [_pod("b1", "1", 0, node="n1"), _pod("b3", "3", 0, node="n3")]
    aff = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "big"}}, "topologyKey": "kubernetes.io/hostname"}]}}
    pods = [_pod("low", "2", 0, {"app": "low"}),
            _pod("aff", "100m", 0, {"app": "aff"}, affinity=aff),
            _pod("eq", "500m", 50, {"app": "eq"}),
            _pod("high", "2", 200, {"app": "high"}),
            _pod("mid", "1", 50, {"app": "mid"}),
            _pod("big", "3", 100, {"app": "big"})]
    noms = [(5, "n2"), (4, "n3")]
    NRF, IPA = "NodeResourcesFit", "InterPodAffinity"
    expect = [
        (0, {"selected": "n1", "fail": {"n2": NRF, "n3": NRF, "n1": None}}),
        (1, {"selected": None, "fail": {"n1": IPA, "n2": IPA, "n3": NRF}}),
        (2, {"selected": "n2", "fail": {"n1": None, "n2": None, "n3": NRF}}),
        (3, {"selected": "n2", "fail": {"n1": NRF, "n2": None, "n3": NRF}}),
        (4, {"selected": "n3", "evaluated": ["n3"], "nominated_left": ["big"]}),
        (5, {"selected": None, "fail": {"n1": NRF, "n2": NRF, "n3": NRF}, "nominated_left": ["big"]}),
    ]
    return nodes, bound, pods, noms, expect


def window_fixture():
    """nextStartNodeIndex after a failed evaluateNominatedNode (hand-derived from v1.26
    findNodesThatPassFilters: processedNodes = feasibleNodesLen + len(diagnosis.NodeToStatusMap),
    the map keyed by node and already holding the nominated node's status).

    120 empty nodes w000..w119 of 4 CPUs, except w119 which a 4-CPU pod fills; percentageOfNodesToScore
    50 -> numFeasibleNodesToFind = max(60, 100) = 100.  Both pods are nominated to w119.

      0 p (1 CPU)  evaluateNominatedNode: w119 fails NodeResourcesFit, the one-node list sets the
                   cursor to 0.  The full search visits w000..w100 and stops at w100 (the 101st
                   feasible node: filtered, dropped); w101..w119 are not reached, so w119's entry is
                   the map's 101st -> processed 100 + 1, cursor 101.
      1 q (1 CPU, matchFields metadata.name In w000 | ... | w009: a 10-node PreFilterResult list, no
                   window)  w119 fails (NodeAffinity first), cursor 0; the search visits the 10 listed nodes (all
                   feasible) and the map holds w119 alone -> processed 10 + 1, cursor 11 % 10 = 1.
    Returns nodes, bound, pods, nominations [(pod, node name)], pct, expected cursor after each pod."""
    nodes = [_node("w%03d" % i) for i in range(120)]
    bound = [_pod("fill", "4", 0, node="w119")]
    # one term per name (a field selector's In takes exactly one value); the terms' union is the list
    names = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["w%03d" % i]}]} for i in range(10)]}}}
    pods = [_pod("p", "1", 0, {"app": "p"}), _pod("q", "1", 0, {"app": "q"}, affinity=names)]
    return nodes, bound, pods, [(0, "w119"), (1, "w119")], 50, [101, 1]
