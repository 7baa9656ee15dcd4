"""Helpers comparing the object-level oracle with the SoA-level C oracle (test infrastructure)."""
import numpy as np

import k8s_oracle
import oracle_c
from kss import abi
from kss.compile import compile_cluster

FILTER_CODE = {name: i for i, name in enumerate(abi.FILTER_PLUGINS) if name}


def run_both(nodes, bound, pods, n_check=None, storage=None, pct=100, nominations=()):
    """Schedule `pods` sequentially with both oracles and assert identical per-pod results.
    storage: {"pvs", "pvcs", "storage_classes", "csinodes"} for the volume plugins.
    pct: percentageOfNodesToScore (below 100: the findNodesThatPassFilters window; the C oracle
    filters every node and windows afterwards, the object oracle visits nodes one at a time).
    nominations: [(index into pods, node index)] in the nominator's order (the nominated pods
    need not be among the first n_check)."""
    cc, cp, comp = compile_cluster(nodes, bound, pods, storage=storage)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    chosen, res, _ = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes,
                                       n_classes=len(cc.classes), n_terms=len(cc.terms), nominations=nominations)
    st = None
    if storage:
        import k8s_volumes
        st = k8s_volumes.Storage(storage.get("pvs") or (), storage.get("pvcs") or (),
                                 storage.get("storage_classes") or (), storage.get("csinodes") or ())
    o = k8s_oracle.Oracle(nodes, bound, storage=st, percentage_of_nodes_to_score=pct)
    assert [k8s_oracle._name(n) for n in o.nodes] == cc.node_names
    for a, b in nominations:
        o.nominate(pods[a], b)
    n_check = len(pods) if n_check is None else n_check
    for j in range(n_check):
        r = o.schedule_one(pods[j])
        m = res.meta(j)
        sel = r["selected"]
        assert (chosen[j] if chosen[j] >= 0 else None) == sel, (j, chosen[j], sel)
        assert m["n_feasible"] == r["n_feasible"], j
        for i in range(cc.n_nodes):
            want = r["fail"].get(i, "NOTEVAL")
            got = int(res.fail_plugin[j, i])
            if want == "NOTEVAL":
                assert got == abi.KSS_F_NOT_EVALUATED, (j, i, got)
            else:
                assert got == (0 if want is None else FILTER_CODE[want]), (j, i, want, got)
                if want is None:  # the node that ended the search: filtered, not kept
                    assert (int(res.fail_detail[j, i]) == abi.KSS_PASS_NOT_KEPT) == (r.get("dropped") == i), (j, i)
        if r["scored"]:
            assert m["scored"] == 1
            for s, pl in enumerate(abi.SCORE_PLUGINS):
                for i, v in r["raw"][pl].items():
                    assert int(res.raw[j, s, i]) == v, (j, pl, i)
                    assert int(res.norm[j, s, i]) == r["norm"][pl][i], (j, pl, i)
    return cc, cp, chosen, res
