"""The volume plugins on CPU: both oracles (object-level oracle/k8s_volumes.py and the SoA-level
C oracle over kss/volumes.py's compiled programs) and the lazy annotation formatter against
the hand-derived fixtures of tests/volume_fixtures.py (disk conflicts, the in-tree and CSI
attach limits, VolumeBinding PreFilter / Filter, VolumeZone), and against each other on
random clusters with volumes (tests/volume_fuzz.py)."""
import json

import pytest

import edge_fixtures as ef
import k8s_oracle
import k8s_volumes
import volume_fixtures as vf
from crosscheck import run_both
from kss import abi
from kss.compile import Unsupported, compile_cluster
from test_format import _format_from_oracle


def _oracle(nodes, bound, st):
    return k8s_oracle.Oracle(nodes, bound, storage=k8s_volumes.Storage(
        st["pvs"], st["pvcs"], st["storage_classes"], st["csinodes"]))


@pytest.mark.parametrize("name", sorted(vf.FIXTURES))
def test_object_oracle_matches_hand_derived(name):
    nodes, bound, pods, expect, st = vf.FIXTURES[name]()
    o = _oracle(nodes, bound, st)
    for j, (p, exp) in enumerate(zip(pods, expect)):
        ef.check_expect(o.annotations(o.schedule_one(p)), exp, where=(name, j))


@pytest.mark.parametrize("name", sorted(vf.FIXTURES))
def test_c_oracle_and_formatter_match_hand_derived(name):
    nodes, bound, pods, expect, st = vf.FIXTURES[name]()
    cc, cp, chosen, res = run_both(nodes, bound, pods, storage=st)  # the two oracles agree first
    prof = abi.default_profile()
    o = _oracle(nodes, bound, st)
    for j, exp in enumerate(expect):
        ann = _format_from_oracle(cc, cp, res, j, prof, pod_aware=True)
        assert ann == o.annotations(o.schedule_one(pods[j])), (name, j)  # all 13 values, byte for byte
        ef.check_expect(ann, exp, where=(name, j))


def test_every_volume_reason_is_covered():
    seen, pre = set(), set()
    for fx in vf.FIXTURES.values():
        for exp in fx()[3]:
            seen.update(f[1] for f in exp["filter"].values() if f is not None)
            st = (exp.get("extra") or {}).get("scheduler-simulator/prefilter-result-status")
            if st:
                pre.add(st["VolumeBinding"])
    for msg in (vf.M_DISK, vf.M_MAXVOL, vf.M_VB_CONFLICT, vf.M_VB_NOPV, vf.M_ZONE, vf.M_VB_BIND,
                vf.M_VB_CONFLICT + ", " + vf.M_VB_BIND):
        assert msg in seen, msg
    assert vf.M_UNBOUND in pre
    plugins = {f[0] for fx in vf.FIXTURES.values() for exp in fx()[3] for f in exp["filter"].values() if f}
    assert {"VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits",
            "VolumeBinding", "VolumeZone"} <= plugins


def test_volume_rows_and_keys():
    """Shared volumes get vol_count rows, private ones count on the chosen node only; the
    attach-limit keys follow the plugin order."""
    nodes, bound, pods, _, st = vf.fx_csi_limits()
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    assert cc.vol_keys == ["attachable-volumes-csi-ebs.csi.aws.com"]
    shared = sorted(u for kind, (k, u) in cc.vol_rows if kind == "vol")
    assert shared == ["ebs.csi.aws.com/h-1", "ebs.csi.aws.com/h-2", "ebs.csi.aws.com/h-3"]
    a = cc.arrays
    assert list(a["vol_attached"][0]) == [1, 1, 0]  # x's h-1 on a, y's unbound u-1 on b
    assert list(a["vol_limit"][0]) == [1, 3, -1]


def test_intree_rbd_provisioner_is_not_a_csi_driver():
    """csi-translation-lib (v1.26) lists the in-tree RBD plugin: with migration off, an unbound
    claim whose StorageClass provisioner is kubernetes.io/rbd has no CSI driver
    (getCSIDriverInfoFromSC returns ""), so it counts toward no attach-limit key, while a CSI
    provisioner's claim does; an inline rbd volume on a node whose CSINode lists the plugin as
    migrated is refused like the other migratable sources (parity unpinned: the translation
    lib is not vendored under the reference)."""
    nodes = [ef.node("a"), ef.node("b")]
    st = vf.storage(pvs=[vf.pv("pv-1", vf.csi("ebs.csi.aws.com", "h-1"))],
                    pvcs=[vf.pvc("u-rbd", bound=False, sc="rbd-sc"), vf.pvc("u-csi", bound=False, sc="csi-sc"),
                          vf.pvc("c-1", "pv-1")],
                    scs=[{"metadata": {"name": "rbd-sc"}, "provisioner": "kubernetes.io/rbd",
                          "volumeBindingMode": "Immediate"},
                         {"metadata": {"name": "csi-sc"}, "provisioner": "ebs.csi.aws.com",
                          "volumeBindingMode": "Immediate"}],
                    csinodes=[{"metadata": {"name": n}, "spec": {"drivers": [
                        {"name": "ebs.csi.aws.com", "allocatable": {"count": 5}},
                        {"name": "kubernetes.io/rbd", "allocatable": {"count": 5}}]}} for n in "ab"])
    bound = [vf.vpod("x", vf.claim("u-rbd"), node_name="a"), vf.vpod("y", vf.claim("u-csi"), node_name="b")]
    cc, cp, _ = compile_cluster(nodes, bound, [vf.vpod("p", vf.claim("c-1"))], storage=st)
    assert cc.vol_keys == ["attachable-volumes-csi-ebs.csi.aws.com"]
    assert list(cc.arrays["vol_attached"][0]) == [0, 1]
    mig = [{"metadata": {"name": "a", "annotations": {"storage.alpha.kubernetes.io/migrated-plugins":
                                                      "kubernetes.io/rbd"}}, "spec": {"drivers": []}}]
    with pytest.raises(Unsupported, match="migrated"):
        compile_cluster([ef.node("a")], [], [vf.vpod("p", vf.rbd(["m1"], "p", "img"))],
                        storage=vf.storage(csinodes=mig))


def test_refusals():
    nodes = [ef.node("a")]
    wffc = {"metadata": {"name": "late"}, "provisioner": "x", "volumeBindingMode": "WaitForFirstConsumer"}
    claims = [vf.pvc(f"u{i}", bound=False, sc="late") for i in range(abi.KSS_MAX_WFFC + 1)]
    st = vf.storage(pvcs=claims, scs=[wffc])
    compile_cluster(nodes, [], [vf.vpod("p", *[vf.claim(f"u{i}") for i in range(abi.KSS_MAX_WFFC)])], storage=st)
    with pytest.raises(Unsupported, match="WaitForFirstConsumer"):  # one delayed claim too many
        compile_cluster(nodes, [], [vf.vpod("p", *[vf.claim(f"u{i}") for i in range(abi.KSS_MAX_WFFC + 1)])],
                        storage=st)
    twice = vf.storage(pvs=[vf.wpv("x", 1, "late", claim_ref="u0"), vf.wpv("y", 1, "late", claim_ref="u0")],
                       pvcs=claims, scs=[wffc])
    with pytest.raises(Unsupported, match="pre-bound"):
        compile_cluster(nodes, [], [vf.vpod("p", vf.claim("u0"))], storage=twice)
    mig = [{"metadata": {"name": "a", "annotations": {"storage.alpha.kubernetes.io/migrated-plugins":
                                                      "kubernetes.io/aws-ebs"}}, "spec": {"drivers": []}}]
    with pytest.raises(Unsupported, match="migrated"):
        compile_cluster(nodes, [], [vf.vpod("p", vf.ebs("v"))], storage=vf.storage(csinodes=mig))


def test_long_csi_driver_key():
    """GetCSIAttachLimitKey: names reaching 63 characters keep 23 characters and 16 hex of sha1."""
    from kss.volumes import csi_attach_limit_key
    d = "a-very-long-csi-driver-name.storage.example.com"
    k = csi_attach_limit_key(d)
    assert k == k8s_volumes.csi_attach_limit_key(d)
    assert k.startswith("attachable-volumes-csi-a-very-long-csi-driver") and len(k) == 23 + 23 + 16
    assert csi_attach_limit_key("ebs.csi.aws.com") == "attachable-volumes-csi-ebs.csi.aws.com"


@pytest.mark.parametrize("seed", range(12))
def test_oracles_agree_on_random_volume_clusters(seed):
    """The object-level restatement (objects, NodeInfo.Pods re-read per filter call) and the
    C oracle over the compiled volume rows agree on every per-node verdict, score and
    choice, pod after pod (each AssumePod visible to the next pod)."""
    import volume_fuzz
    nodes, bound, pods, st = volume_fuzz.make(seed)
    cc, cp, chosen, res = run_both(nodes, bound, pods, storage=st)
    fails = {int(f) for f in res.fail_plugin.ravel()}
    assert cp.n_vols > 0 and len(cc.vol_rows) > 0
    if seed == 0:  # the generator reaches the volume plugins' failures
        assert fails & {abi.KSS_F_VOLUME_RESTRICTIONS, abi.KSS_F_VOLUME_BINDING, abi.KSS_F_VOLUME_ZONE}


def test_snapshot_round_trip_with_volumes():
    """ResourcesForSnap (snapshot.go:32-41) carries pvs / pvcs / storageClasses: written, read
    back and compiled, it schedules like the objects it came from."""
    from kss import snapshot
    import volume_fuzz
    nodes, bound, pods, st = volume_fuzz.make(5)
    snap = snapshot.Snapshot(nodes=nodes, bound=bound, pending=pods, namespaces={"default": {}},
                             pvs=st["pvs"], pvcs=st["pvcs"], storage_classes=st["storage_classes"])
    back = snapshot.read_snapshot(json.dumps(snapshot.write_snapshot(snap)))
    st2 = back.storage()
    assert st2["pvs"] == st["pvs"] and st2["pvcs"] == st["pvcs"]
    run_both(back.nodes, back.bound, back.pending, storage=st2)


def test_plan_names_volumes():
    """kss_plan_podset (host only): volume programs keep a batch on k_schedule, and say so."""
    from kss import native
    nodes, bound, pods, _, st = vf.fx_volume_zone()
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    plan = native.plan_podset(cc.as_struct(), cp.as_struct())
    assert plan["kernel"] == "k_schedule" and "volumes" in plan["reason"], plan


def test_wffc_assume_cache_final_state():
    """Both oracles end the WaitForFirstConsumer fixture with the hand-derived assume cache: each
    claim's static binding (pv_owner) and the provisioned claim's selected node (claim_node)."""
    import oracle_c
    nodes, bound, pods, _, st = vf.fx_wait_for_first_consumer()
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    _, _, fs = oracle_c.schedule(abi.default_profile(), cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes,
                                 record=False, n_classes=len(cc.classes), n_terms=len(cc.terms))
    claim_of = {i + 1: name for i, (_, name) in enumerate(cc.wclaims)}
    got = {claim_of[o]: cc.pvs[v] for v, o in enumerate(fs["pv_owner"]) if o}
    assert got == vf.WFFC_FINAL_BINDINGS
    sel = {cc.wclaims[c][1]: cc.node_names[n] for c, n in enumerate(fs["claim_node"]) if n >= 0}
    assert sel == vf.WFFC_FINAL_SELECTED
    o = _oracle(nodes, bound, st)
    for p in pods:
        o.schedule_one(p)
    assert {ref[1]: pv for pv, ref in o.storage.pv_ref.items()} == vf.WFFC_FINAL_BINDINGS
    assert o.storage.selected == {("default", k): v for k, v in vf.WFFC_FINAL_SELECTED.items()}


@pytest.mark.parametrize("seed", range(16))
def test_oracles_agree_on_random_wffc_clusters(seed):
    """WaitForFirstConsumer claims on random clusters (tests/volume_fuzz.py wffc=True): the object
    oracle's FindPodVolumes / AssumePodVolumes and the C oracle over the compiled candidate lists
    agree pod after pod, and on the assume cache they leave."""
    import oracle_c
    import volume_fuzz
    nodes, bound, pods, st = volume_fuzz.make(100 + seed, wffc=True)
    cc, cp, chosen, res = run_both(nodes, bound, pods, storage=st)
    assert cc.wclaims and cp.n_vols > 0
    _, _, fs = oracle_c.schedule(abi.default_profile(), cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes,
                                 record=False, n_classes=len(cc.classes), n_terms=len(cc.terms))
    o = _oracle(nodes, bound, st)
    for p in pods:
        o.schedule_one(p)
    claim_of = {i + 1: name for i, (_, name) in enumerate(cc.wclaims)}
    got = {cc.pvs[v]: claim_of[int(x)] for v, x in enumerate(fs["pv_owner"]) if x}
    want = {pv: ref[1] for pv, ref in o.storage.pv_ref.items() if pv in set(cc.pvs)}
    assert got == want
    sel = {cc.wclaims[c][1]: int(n) for c, n in enumerate(fs["claim_node"]) if n != -1}
    want_sel = {k[1]: (cc.node_names.index(v) if v in cc.node_names else -2) for k, v in o.storage.selected.items()
                if k in set(cc.wclaims)}
    assert sel == want_sel


def test_random_wffc_clusters_reach_every_branch():
    """Across the seeds the WaitForFirstConsumer fuzz reaches bind conflicts, the combined node +
    bind conflict reason, static bindings and provisioning (both assume-cache columns move)."""
    import oracle_c
    import volume_fuzz
    details, moved_pv, moved_claim = set(), False, False
    for seed in range(16):
        nodes, bound, pods, st = volume_fuzz.make(100 + seed, wffc=True)
        cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
        ch, res, fs = oracle_c.schedule(abi.default_profile(), cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes,
                                        record=True, n_classes=len(cc.classes), n_terms=len(cc.terms))
        vb = res.fail_plugin == abi.KSS_F_VOLUME_BINDING
        details |= {int(d) for d in res.fail_detail[vb]}
        moved_pv |= bool((fs["pv_owner"] != cc.arrays["pv_owner"][:len(cc.pvs)]).any())
        moved_claim |= bool((fs["claim_node"] != cc.arrays["claim_node"][:len(cc.wclaims)]).any())
    assert {abi.KSS_VB_BIND_CONFLICT} <= details, details
    assert moved_pv and moved_claim
