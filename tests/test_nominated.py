"""Nominated pods (the scheduling queue's nominator) in both oracles: RunFilterPluginsWithNominatedPods
(two filter passes on nodes holding nominees of equal or higher priority), PreferNominatedNode (a
nominated pod tries its node first) and DeleteNominatedPodIfExists on assume.  The SoA C oracle and
the object oracle agree per node and per pod on seeded clusters; the hand-derived fixture pins the
object oracle (tests/nominated_fixtures.py)."""
import copy
import random

import pytest

import k8s_oracle as ko
import nominated_fixtures as nf
from crosscheck import run_both
from kss import synth


def with_priorities(pods, seed, levels=(0, 0, 10, 100, 1000)):
    rnd = random.Random(seed)
    out = []
    for p in pods:
        p = copy.deepcopy(p)
        p["spec"]["priority"] = rnd.choice(levels)
        out.append(p)
    return out


def nominations_for(pods, n_nodes, n_check, seed, inside=3, outside=6):
    """`inside` nominations of pods scheduled in the checked prefix (PreferNominatedNode, removal on
    assume) and `outside` of pods after it (nominees only), on random nodes; the nominees get the
    highest priority level so most pods see them."""
    rnd = random.Random(seed)
    noms = []
    for j in rnd.sample(range(n_check), inside) + rnd.sample(range(n_check, len(pods)), outside):
        noms.append((j, rnd.randrange(n_nodes)))
    for j, _ in noms[inside:]:
        pods[j]["spec"]["priority"] = 1000
    return noms


@pytest.mark.parametrize("seed,config,n_nodes,n_pods,n_check", [(1, 1, 40, 160, 120), (2, 1, 12, 120, 90),
                                                                  (3, 5, 30, 120, 100)])
def test_nominees_default_profile(seed, config, n_nodes, n_pods, n_check):
    nodes, bound, pods = synth.make_cluster(config, n_nodes, n_pods)
    pods = with_priorities(pods, seed)
    noms = nominations_for(pods, n_nodes, n_check, seed)
    run_both(nodes, bound, pods, n_check=n_check, nominations=noms)


@pytest.mark.parametrize("seed", [4, 5])
def test_nominees_spread_and_interpod(seed):
    """The nominees' labels enter the PodTopologySpread pair counts (criticalPaths update) and
    the InterPodAffinity counts (existing anti-affinity, affinity, anti-affinity) of their node."""
    nodes, bound, pods = synth.make_cluster(3, 40, 160)
    pods = with_priorities(pods, seed)
    noms = nominations_for(pods, 40, 120, seed, inside=4, outside=10)
    run_both(nodes, bound, pods, n_check=120, nominations=noms)


@pytest.mark.parametrize("seed", range(4))
def test_nominees_program_fuzz(seed):
    import progfuzz
    nodes, bound, pods = progfuzz.make(2000 + seed, 50, 110)
    pods = with_priorities(pods, seed)
    noms = nominations_for(pods, 50, 90, seed, inside=4, outside=12)
    run_both(nodes, bound, pods, n_check=90, nominations=noms)


def test_nominees_with_window():
    """percentageOfNodesToScore 30 over 250 nodes: PreferNominatedNode resets nextStartNodeIndex;
    a nominated node the window never reaches keeps its evaluateNominatedNode record."""
    nodes, bound, pods = synth.make_cluster(1, 250, 160)
    pods = with_priorities(pods, 9)
    noms = nominations_for(pods, 250, 120, 9, inside=8, outside=10)
    run_both(nodes, bound, pods, n_check=120, pct=30, nominations=noms)


def test_fixture_object_oracle():
    """The hand-derived fixture (nominated_fixtures.fixture): every expected outcome, record and
    nomination change, on the object oracle."""
    nodes, bound, pods, noms, expect = nf.fixture()
    o = ko.Oracle(nodes, bound)
    for j, n in noms:
        o.nominate(pods[j], o.by_name[n])
    for (j, want) in expect:
        r = o.schedule_one(pods[j])
        sel = ko._name(o.nodes[r["selected"]]) if r["selected"] is not None else None
        assert sel == want["selected"], (j, sel, want)
        for node, plugin in want.get("fail", {}).items():
            assert r["fail"].get(o.by_name[node], "NOTEVAL") == plugin, (j, node)
        if "nominated_left" in want:
            assert sorted(ko._name(p) for _, p, _ in o.nominated) == want["nominated_left"], j
        if "evaluated" in want:
            assert sorted(ko._name(o.nodes[i]) for i in r["fail"]) == want["evaluated"], j


def test_fixture_c_oracle():
    """The same fixture through the C oracle (one batch: the nominator as the fixture leaves it)."""
    nodes, bound, pods, noms, expect = nf.fixture()
    order = [j for j, _ in expect]
    assert order == list(range(len(order)))  # the fixture schedules pods in index order
    name_noms = [(j, n) for j, n in noms]
    from kss.compile import compile_cluster
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    idx = {n: i for i, n in enumerate(cc.node_names)}
    import oracle_c
    from kss import abi
    chosen, res, st = oracle_c.schedule(abi.default_profile(), cc.as_struct(), cp.as_struct(), len(order), cc.n_nodes,
                                        n_classes=len(cc.classes), n_terms=len(cc.terms),
                                        nominations=[(j, idx[n]) for j, n in name_noms])
    for j, want in expect:
        got = cc.node_names[chosen[j]] if chosen[j] >= 0 else None
        assert got == want["selected"], (j, got, want)
    left = sorted(cp.names[j][1] for j, _ in st["nominations"])
    assert left == expect[-1][1]["nominated_left"]


def test_window_fixture_cursor_counts_the_nominated_status():
    """nominated_fixtures.window_fixture: the nominated node's failure counts in processedNodes when
    the search does not reach that node again (window stop; outside the PreFilterResult list), in
    both oracles."""
    nodes, bound, pods, noms, pct, cursors = nf.window_fixture()
    o = ko.Oracle(nodes, bound, percentage_of_nodes_to_score=pct)
    for j, n in noms:
        o.nominate(pods[j], o.by_name[n])
    for j, want in enumerate(cursors):
        r = o.schedule_one(pods[j])
        assert r["selected"] is not None and r["fail"][o.by_name["w119"]] == ("NodeResourcesFit", "NodeAffinity")[j], j
        assert o.next_start == want, (j, o.next_start)
    r0 = None
    from kss.compile import compile_cluster
    from kss import abi
    import oracle_c
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    idx = {n: i for i, n in enumerate(cc.node_names)}
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    for n_run, want in ((1, cursors[0]), (2, cursors[1])):
        ch, res, st = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), n_run, cc.n_nodes,
                                        n_classes=len(cc.classes), n_terms=len(cc.terms),
                                        nominations=[(j, idx[n]) for j, n in noms])
        assert st["next_start"] == want, (n_run, st["next_start"])
        if n_run == 1:
            r0 = res
    # pod 0's record: w100 ended the search (passed, dropped), w101..w118 never visited
    assert int(r0.fail_plugin[0, idx["w100"]]) == 0 and int(r0.fail_detail[0, idx["w100"]]) == abi.KSS_PASS_NOT_KEPT
    assert all(int(r0.fail_plugin[0, idx["w%03d" % i]]) == abi.KSS_F_NOT_EVALUATED for i in range(101, 119))
