"""DefaultPreemption PostFilter dry run (ORACLE, TEST INFRASTRUCTURE ONLY) — pure Python.

Restates, over k8s_oracle.Oracle's NodeInfos and cycle state, the PostFilter the simulator
wraps at /root/reference/simulator/scheduler/plugin/wrappedplugin.go:550-577 (the default
MultiPoint profile enables DefaultPreemption, simulator/scheduler/config/plugin_test.go:32).
The plugin lives in the pinned dependency k8s.io/kubernetes v1.26.2
(/root/reference/simulator/go.mod:56; not vendored here), so every step cites the upstream
function it restates:

  pkg/scheduler/framework/preemption/preemption.go
    Evaluator.Preempt                 eligibility -> findCandidates -> SelectCandidate
    findCandidates                    nodesWherePreemptionMightHelp + DryRunPreemption
    nodesWherePreemptionMightHelp     drop nodes whose status is UnschedulableAndUnresolvable
    DryRunPreemption                  SelectVictimsOnNode on every potential node
    SelectCandidate / pickOneNodeForPreemption
  pkg/scheduler/framework/plugins/defaultpreemption/default_preemption.go
    PodEligibleToPreemptOthers        preemptionPolicy Never
    SelectVictimsOnNode               remove lower-priority pods, filter, reprieve in order
  pkg/scheduler/framework/plugins/podtopologyspread/filtering.go
    preFilterState.updateWithPod, criticalPaths.update (RemovePod / AddPod extensions)
  pkg/scheduler/framework/plugins/interpodaffinity/filtering.go
    preFilterState.updateWithPod, topologyToMatchedTermCount.update
  pkg/scheduler/util/utils.go         MoreImportantPod, GetPodStartTime, GetEarliestPodStartTime

Deterministic where upstream is not (both documented in DESIGN.md, "PostFilter"):
  * DryRunPreemption starts at a random offset and stops once max(10% of the potential
    nodes, 100) candidates are found; here every potential node is evaluated, which is
    upstream's result whenever there are at most 100 potential nodes;
  * pods without status.startTime get GetPodStartTime = time.Now() upstream (clock-dependent
    order); here they sort after every pod with a start time and tie with each other;
    sort.Slice ties keep NodeInfo order (Go's pdqsort is an insertion sort below 13
    elements, so this is upstream's order whenever a node has at most 12 potential victims);
  * pickOneNodeForPreemption iterates a Go map (random order) and keeps the first node on a
    full tie; here candidates are visited in canonical node order.
No PodDisruptionBudgets (the simulator's snapshot carries none: every victim is
non-violating).  SelectVictimsOnNode filters with RunFilterPluginsWithNominatedPods
(Oracle.filter_with_nominated): the nominator's pods of equal or higher priority on the node
take part in the first pass; they are never victims (they are not in NodeInfo.Pods).
"""
from __future__ import annotations

from datetime import datetime, timezone
from typing import Dict, List, Optional

import k8s_oracle as ko
from k8s_oracle import (CriticalPaths, _ipa_state, _ipa_update, _pts_state, _pts_update,  # noqa: F401
                        _tm_update, pod_priority)

MAX_INT32 = 2**31 - 1
NOMINATED_MESSAGE = "preemption victim"  # resultstore PostFilterNominatedMessage (store.go:34)

# Filter reasons returned with UnschedulableAndUnresolvable in v1.26 (the rest are Unschedulable).
UNRESOLVABLE = {
    ("NodeUnschedulable", None), ("NodeName", None), ("TaintToleration", None), ("NodeAffinity", None),
    ("PodTopologySpread", ko.MSG["PTS_LABEL"]), ("InterPodAffinity", ko.MSG["IPA_AFF"]),
}


def pod_start_ns(pod) -> Optional[int]:
    """status.startTime as Unix nanoseconds (RFC 3339, second precision), None if unset."""
    st = (pod.get("status") or {}).get("startTime")
    if not st:
        return None
    t = datetime.strptime(st, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=timezone.utc)
    return int(t.timestamp()) * 10**9


def _start_key(pod) -> float:
    s = pod_start_ns(pod)
    return float("inf") if s is None else s


def more_important(p1, p2) -> bool:
    """util.MoreImportantPod: higher priority, then earlier start time."""
    a, b = pod_priority(p1), pod_priority(p2)
    if a != b:
        return a > b
    return _start_key(p1) < _start_key(p2)


def _sorted_by_importance(pods: List) -> List:
    """sort.Slice(MoreImportantPod), as the insertion sort Go uses below 13 elements (stable)."""
    out = list(pods)
    for i in range(1, len(out)):
        j = i
        while j > 0 and more_important(out[j].pod, out[j - 1].pod):
            out[j], out[j - 1] = out[j - 1], out[j]
            j -= 1
    return out


def _unresolvable(plugin: str, msg: str) -> bool:
    return (plugin, None) in UNRESOLVABLE or (plugin, msg) in UNRESOLVABLE


def select_victims_on_node(o: ko.Oracle, pod, i: int, pts_st, ipa_st):
    """SelectVictimsOnNode: (victim PodInfos in reprieve order, or None when the node is no candidate)."""
    ni = o.infos[i].clone()
    node = ni.node
    pts = _pts_state(pts_st)
    ipa = _ipa_state(ipa_st)
    prio = pod_priority(pod)
    potential = [pi for pi in o.infos[i].pods if pod_priority(pi.pod) < prio]  # NodeInfo order
    if not potential:
        return None  # "No preemption victims found for incoming pod"
    for pi in potential:
        ni.remove_pod(pi.pod)
        _pts_update(pts, pi.pod, pod, node, -1)
        _ipa_update(o, ipa, pi, pod, node, -1)
    if o.filter_with_nominated(pod, i, ni, pts, ipa)[0] is not None:
        return None
    victims = []
    for pi in _sorted_by_importance(potential):  # no PDBs: every pod is non-violating
        ni.add_pod(pi.pod)
        _pts_update(pts, pi.pod, pod, node, 1)
        _ipa_update(o, ipa, pi, pod, node, 1)
        if o.filter_with_nominated(pod, i, ni, pts, ipa)[0] is not None:
            ni.remove_pod(pi.pod)
            _pts_update(pts, pi.pod, pod, node, -1)
            _ipa_update(o, ipa, pi, pod, node, -1)
            victims.append(pi)
    return victims or None  # success with no victims is an error status upstream


def pick_one_node(cands: Dict[int, List]) -> Optional[int]:
    """pickOneNodeForPreemption over {node index: victims}, visited in canonical order."""
    if not cands:
        return None
    nodes = sorted(cands)  # every NumPDBViolations is 0
    hp = {n: pod_priority(cands[n][0].pod) for n in nodes}
    m = min(hp.values())
    nodes = [n for n in nodes if hp[n] == m]
    if len(nodes) == 1:
        return nodes[0]
    sp = {n: sum(pod_priority(v.pod) + MAX_INT32 + 1 for v in cands[n]) for n in nodes}
    m = min(sp.values())
    nodes = [n for n in nodes if sp[n] == m]
    if len(nodes) == 1:
        return nodes[0]
    nv = {n: len(cands[n]) for n in nodes}
    m = min(nv.values())
    nodes = [n for n in nodes if nv[n] == m]
    if len(nodes) == 1:
        return nodes[0]

    def earliest(vs):  # GetEarliestPodStartTime: earliest start among the highest-priority victims
        top = max(pod_priority(v.pod) for v in vs)
        return min(_start_key(v.pod) for v in vs if pod_priority(v.pod) == top)

    best, best_t = nodes[0], earliest(cands[nodes[0]])
    for n in nodes[1:]:
        t = earliest(cands[n])
        if t > best_t:  # After(latestStartTime)
            best, best_t = n, t
    return best


def preempt(o: ko.Oracle, pod, res) -> dict:
    """Evaluator.Preempt for a pod whose scheduling cycle `res` (Oracle.schedule_one) failed.
    Returns {status, nominated, victims, n_potential, n_candidates, candidates}."""
    out = dict(status="no_candidate", nominated=None, victims=[], n_potential=0, n_candidates=0, candidates={})
    if res["selected"] is not None:
        out["status"] = "schedulable"
        return out
    if (ko._spec(pod).get("preemptionPolicy") or "") == "Never":
        out["status"] = "not_eligible"
        return out
    if res["status"] == "prefilter":
        return out  # every node carries the PreFilter's UnschedulableAndUnresolvable status
    pts_st, ipa_st = res["_pts_st"], res["_ipa_st"]
    cands: Dict[int, List] = {}
    for i, ni in enumerate(o.infos):
        name = ko._name(ni.node)
        rec = res["filter"].get(name)
        if rec is not None:
            plugin = next(reversed(rec))
            if _unresolvable(plugin, rec[plugin]):
                continue
        out["n_potential"] += 1
        v = select_victims_on_node(o, pod, i, pts_st, ipa_st)
        if v:
            cands[i] = v
    out["n_candidates"] = len(cands)
    out["candidates"] = cands
    best = pick_one_node(cands)
    if best is not None:
        out["status"] = "nominated"
        out["nominated"] = best
        out["victims"] = [(ko._ns(v.pod), ko._name(v.pod)) for v in cands[best]]
    return out


def schedule_with_preemption(nodes, bound, pods, **kw):
    """Sequential cycles as Oracle.schedule_one does; every unschedulable pod also gets its
    PostFilter dry run against the state it was filtered in (nothing is evicted)."""
    o = ko.Oracle(nodes, bound, **kw)
    out = []
    for p in pods:
        r = o.schedule_one(p)
        pre = preempt(o, p, r) if r["selected"] is None else None
        out.append((r, pre, o.annotations(r, pre["nominated"] if pre else None)))
    return o, out



def schedule_with_nominations(nodes, bound, pods, retries=1, **kw):
    """The sequence as the simulator's scheduler runs it with DefaultPreemption and a nominator.
    An unschedulable pod's PostFilter result is acted on the way the scheduler does:
      * nominated: prepareCandidate deletes the victims (the informer's RemovePod follows) and
        clears the nominations of lower-priority pods nominated to that node
        (getLowerPriorityNominatedPods -> ClearNominatedNodeName); handleSchedulingFailure records
        the pod in the nominator (AddNominatedPod) and it is retried after the pods already
        queued (at most `retries` times);
      * no candidate: the PostFilterResult's empty NominatedNodeName clears the pod's nomination;
      * not eligible: the nomination stays (ModeNoop).
    Returns (oracle, [(pod index, cycle result, PostFilter result or None)]) in cycle order."""
    o = ko.Oracle(nodes, bound, **kw)
    queue = list(range(len(pods)))
    tries = [0] * len(pods)
    out = []
    while queue:
        j = queue.pop(0)
        p = pods[j]
        r = o.schedule_one(p)
        pre = None
        if r["selected"] is None:
            pre = preempt(o, p, r)
            if pre["status"] == "nominated":
                node = pre["nominated"]
                for pi in pre["candidates"][node]:
                    o.infos[node].remove_pod(pi.pod)
                prio = pod_priority(p)
                for _, q, n in list(o.nominated):
                    if n == node and pod_priority(q) < prio:
                        o.clear_nomination(q)
                o.nominate(p, node)
                if tries[j] < retries:
                    tries[j] += 1
                    queue.append(j)
            elif pre["status"] == "no_candidate":
                o.clear_nomination(p)
        out.append((j, r, pre))
    return o, out
