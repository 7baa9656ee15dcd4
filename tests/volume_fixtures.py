"""Hand-derived fixtures for the volume plugins (test infrastructure).

Every expectation was worked out by hand from the v1.26 upstream function it names (not
produced by either oracle); tests/test_volumes.py checks both oracles and the formatter
against them, tests/test_gpu_volumes.py the device through the C-ABI.  Same shape as
tests/edge_fixtures.py, plus the storage objects:

    (nodes, bound, pods, expect, storage)

Scores: every pod here requests nothing, so NodeResourcesFit (LeastAllocated over
NonZeroRequested: 100m / 200Mi per pod) ranks nodes by their pod count and ties go to the
lowest canonical index (BalancedAllocation is 100 everywhere, the other plugins constant).
"""
from edge_fixtures import HOST, ZONE, node, pod

REGION = "topology.kubernetes.io/region"
BETA_ZONE = "failure-domain.beta.kubernetes.io/zone"
IT = "node.kubernetes.io/instance-type"
BIND = {"pv.kubernetes.io/bind-completed": "yes"}

M_DISK = "node(s) had no available disk"                          # volume_restrictions.go ErrReasonDiskConflict
M_MAXVOL = "node(s) exceed max volume count"                      # nodevolumelimits ErrReasonMaxVolumeCountExceeded
M_VB_CONFLICT = "node(s) had volume node affinity conflict"       # volumebinding ErrReasonNodeConflict
M_VB_NOPV = "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)"  # ErrReasonPVNotExist
M_ZONE = "node(s) had no available volume zone"                   # volume_zone.go ErrReasonConflict
M_UNBOUND = "pod has unbound immediate PersistentVolumeClaims"
M_VB_BIND = "node(s) didn't find available persistent volumes to bind"  # volumebinding ErrReasonBindConflict


def vpod(name, *volumes, node_name=None):
    return pod(name, node_name=node_name, volumes=[dict(v, name="v%d" % i) for i, v in enumerate(volumes)])


def gce(pd, ro=False):
    return {"gcePersistentDisk": {"pdName": pd, "readOnly": ro}}


def ebs(vid, ro=False):
    return {"awsElasticBlockStore": {"volumeID": vid, "readOnly": ro}}


def azure(disk):
    return {"azureDisk": {"diskName": disk, "diskURI": "uri/" + disk}}


def rbd(monitors, pool, image, ro=False):
    return {"rbd": {"monitors": list(monitors), "pool": pool, "image": image, "readOnly": ro}}


def claim(name):
    return {"persistentVolumeClaim": {"claimName": name}}


def pvc(name, volume=None, bound=True, sc=None, phase=None):
    md = {"name": name, "namespace": "default"}
    if bound and volume:
        md["annotations"] = dict(BIND)
    spec = {}
    if volume:
        spec["volumeName"] = volume
    if sc is not None:
        spec["storageClassName"] = sc
    out = {"metadata": md, "spec": spec}
    if phase:
        out["status"] = {"phase": phase}
    return out


def pv(name, source=None, labels=None, affinity_terms=None):
    spec = dict(source or {})
    if affinity_terms is not None:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": list(affinity_terms)}}
    return {"metadata": {"name": name, "labels": dict(labels or {})}, "spec": spec}


def csi(driver, handle):
    return {"csi": {"driver": driver, "volumeHandle": handle}}


def storage(pvs=(), pvcs=(), scs=(), csinodes=()):
    return {"pvs": list(pvs), "pvcs": list(pvcs), "storage_classes": list(scs), "csinodes": list(csinodes)}


def _all(names, v=None):
    return {n: v for n in names}


# --------------------------------------------------------------------------------------
# VolumeRestrictions (volume_restrictions.go satisfyVolumeConflicts / isVolumeConflict):
# GCE PD and iSCSI conflict unless both mounts are read-only, an AWS EBS volume conflicts
# with any other mount of it, RBD conflicts when the monitor lists overlap, pool and image
# match, and not both are read-only.  Only inline pod volumes are checked.
def fx_disk_conflict():
    nodes = [node(n) for n in "abcd"]
    bound = [vpod("gce-rw", gce("disk-1"), node_name="a"),
             vpod("gce-ro", gce("disk-2", ro=True), node_name="b"),
             vpod("ebs-ro", ebs("vol-9", ro=True), node_name="c"),
             vpod("rbd-rw", rbd(["m1", "m2"], "p", "img"), node_name="d")]
    pods = [vpod("p-gce1-ro", gce("disk-1", ro=True)),   # RO vs a's RW: a fails
            vpod("p-gce2-ro", gce("disk-2", ro=True)),   # RO vs RO on b: no conflict
            vpod("p-gce1-rw", gce("disk-1")),            # RW vs a's RW and b's RO (p-gce1-ro)
            vpod("p-ebs", ebs("vol-9")),                 # EBS: c's read-only mount still conflicts
            vpod("p-rbd-ro", rbd(["m2", "m3"], "p", "img", ro=True)),  # m2 shared, d's mount RW
            vpod("p-rbd-other", rbd(["m2"], "p", "img2"))]             # another image: no conflict
    D = ("VolumeRestrictions", M_DISK)
    expect = [
        {"filter": {"a": D, "b": None, "c": None, "d": None}, "selected": "b"},   # b c d one pod each
        {"filter": _all("abcd"), "selected": "a"},                                # b has two pods
        {"filter": {"a": D, "b": D, "c": None, "d": None}, "selected": "c"},
        {"filter": {"a": None, "b": None, "c": D, "d": None}, "selected": "d"},   # a b c two pods, d one
        {"filter": {"a": None, "b": None, "c": None, "d": D}, "selected": "a"},   # every node two pods
        {"filter": _all("abcd"), "selected": "b"},                                # a three pods
    ]
    return nodes, bound, pods, expect, storage()


# --------------------------------------------------------------------------------------
# EBSLimits / GCEPDLimits / AzureDiskLimits (non_csi.go nonCSILimits.Filter): when the pod
# has a volume of the plugin, len(existing) + len(new \ existing) > the node's limit fails,
# even with nothing new (c below, already over its limit).  Limits: allocatable
# attachable-volumes-<plugin> over getMaxVolumeFunc's default (EBS: 25 for instance types
# matching ^[cmr]5.*|t3|z1d, else 39; GCE PD and Azure Disk 16).  PVC-backed volumes count by
# their PV's id and are not VolumeRestrictions' concern.
def fx_non_csi_limits():
    nodes = [node("a", labels={IT: "m5.large"}, extra={"attachable-volumes-aws-ebs": "2"}),
             node("b", labels={IT: "t3.small"}, extra={"attachable-volumes-azure-disk": "0"}),
             node("c", extra={"attachable-volumes-aws-ebs": "1", "attachable-volumes-gce-pd": "0"})]
    bound = [vpod("two-a", ebs("vol-1"), ebs("vol-2"), node_name="a"),
             vpod("two-c", ebs("vol-5"), ebs("vol-6"), node_name="c")]
    st = storage(pvs=[pv("pv-1", ebs("vol-1")), pv("pv-5", ebs("vol-5"))],
                 pvcs=[pvc("c-1", "pv-1"), pvc("c-5", "pv-5")])
    pods = [vpod("p-new", ebs("vol-3")),          # a: 2 + 1 > 2; c: 2 + 1 > 1
            vpod("p-pvc1", claim("c-1")),         # vol-1 already on a: 2 + 0; c: 2 + 1 > 1
            vpod("p-pvc5", claim("c-5")),         # c: 2 + 0 > 1 (nothing new, still over); a: 3 > 2
            vpod("p-gce-az", gce("pd-x"), azure("az-1"))]  # c: GCE 0 + 1 > 0; b: Azure 0 + 1 > 0
    E, G, A = ("EBSLimits", M_MAXVOL), ("GCEPDLimits", M_MAXVOL), ("AzureDiskLimits", M_MAXVOL)
    expect = [
        {"filter": {"a": E, "b": None, "c": E}, "selected": "b"},
        {"filter": {"a": None, "b": None, "c": E}, "selected": "a"},   # a, b one pod each: a first
        {"filter": {"a": E, "b": None, "c": E}, "selected": "b"},
        {"filter": {"a": None, "b": A, "c": G}, "selected": "a"},     # GCEPDLimits runs before AzureDiskLimits
    ]
    return nodes, bound, pods, expect, st


# --------------------------------------------------------------------------------------
# NodeVolumeLimits (csi.go CSILimits.Filter): per CSI driver key
# attachable-volumes-csi-<driver>, attached + new > limit fails, only for keys with a new
# volume; limits from CSINode.spec.drivers[].allocatable.count (a: 1, b: 3; c: no CSINode,
# no limit).  An unbound claim of a bound pod counts through its StorageClass's provisioner
# (getCSIDriverInfoFromSC): y's claim u-1 is attached on b.
def fx_csi_limits():
    drv = "ebs.csi.aws.com"
    nodes = [node(n) for n in "abc"]
    csinodes = [{"metadata": {"name": "a"}, "spec": {"drivers": [{"name": drv, "allocatable": {"count": 1}}]}},
                {"metadata": {"name": "b"}, "spec": {"drivers": [{"name": drv, "allocatable": {"count": 3}}]}}]
    st = storage(pvs=[pv("pv-1", csi(drv, "h-1")), pv("pv-2", csi(drv, "h-2")), pv("pv-3", csi(drv, "h-3"))],
                 pvcs=[pvc("c-1", "pv-1"), pvc("c-2", "pv-2"), pvc("c-3", "pv-3"),
                       pvc("u-1", bound=False, sc="csi-sc")],
                 scs=[{"metadata": {"name": "csi-sc"}, "provisioner": drv, "volumeBindingMode": "Immediate"}],
                 csinodes=csinodes)
    bound = [vpod("x", claim("c-1"), node_name="a"), vpod("y", claim("u-1"), node_name="b")]
    pods = [vpod("p-c2", claim("c-2")),                  # a: 1 + 1 > 1; b: 1 (u-1) + 1 <= 3
            vpod("p-c1", claim("c-1")),                  # a: h-1 attached, nothing new: passes at its limit
            vpod("p-c1c3", claim("c-1"), claim("c-3")),  # a: 1 + 1 (h-3) > 1; b: 1 + 2 <= 3
            vpod("p-c3", claim("c-3")),                  # b: h-3 attached by p-c1c3, nothing new
            vpod("p-c2-again", claim("c-2"))]            # b: 3 + 1 > 3; a: 1 + 1 > 1
    L = ("NodeVolumeLimits", M_MAXVOL)
    expect = [
        {"filter": {"a": L, "b": None, "c": None}, "selected": "c"},   # b has y
        {"filter": _all("abc"), "selected": "a"},                      # one pod each: a first
        {"filter": {"a": L, "b": None, "c": None}, "selected": "b"},   # b (y) and c (p-c2): b first
        {"filter": {"a": L, "b": None, "c": None}, "selected": "c"},   # b two pods, c one
        {"filter": {"a": L, "b": L, "c": None}, "selected": "c"},
    ]
    return nodes, bound, pods, expect, st


# --------------------------------------------------------------------------------------
# VolumeBinding (volume_binding.go PreFilter / Filter -> binder.go checkBoundClaims):
# PreFilter rejects a pod whose claim is missing, lost or unbound-immediate
# (UnschedulableAndUnresolvable, every node); Filter walks the bound claims in order and
# stops at a PV that does not exist or whose required node affinity does not match the
# node's labels (CheckNodeAffinity: the node's labels only, so matchFields never constrain).
def fx_volume_binding():
    nodes = [node("a", zone="zone-a"), node("b", zone="zone-b"), node("c", zone="zone-c")]
    za = [{"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["zone-a"]}]}]
    zbc = [{"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["zone-b"]}]},
           {"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["zone-c"]}]}]
    host_c = [{"matchExpressions": [{"key": HOST, "operator": "In", "values": ["c"]}],
               "matchFields": [{"key": "metadata.name", "operator": "In", "values": ["a"]}]}]
    st = storage(pvs=[pv("pv-za", affinity_terms=za), pv("pv-zbc", affinity_terms=zbc),
                      pv("pv-hostc", affinity_terms=host_c)],
                 pvcs=[pvc("c-za", "pv-za"), pvc("c-zbc", "pv-zbc"), pvc("c-hostc", "pv-hostc"),
                       pvc("c-missing", "pv-gone"), pvc("c-unbound", bound=False),
                       pvc("c-lost", "pv-gone", phase="Lost")])
    pods = [vpod("p-za", claim("c-za")),
            vpod("p-zbc-za", claim("c-zbc"), claim("c-za")),
            vpod("p-hostc", claim("c-hostc")),
            vpod("p-za-missing", claim("c-za"), claim("c-missing")),
            vpod("p-unbound", claim("c-unbound")),
            vpod("p-nopvc", claim("nope")),
            vpod("p-lost", claim("c-lost"))]
    C, N = ("VolumeBinding", M_VB_CONFLICT), ("VolumeBinding", M_VB_NOPV)

    def pre(msg):
        return {"scheduler-simulator/prefilter-result-status": {
            "NodeAffinity": "success", "NodePorts": "success", "NodeResourcesFit": "success",
            "VolumeRestrictions": "success", "VolumeBinding": msg}}
    expect = [
        {"filter": {"a": None, "b": C, "c": C}, "selected": "a"},
        {"filter": {"a": C, "b": C, "c": C}, "selected": ""},
        {"filter": {"a": C, "b": C, "c": None}, "selected": "c"},
        {"filter": {"a": N, "b": C, "c": C}, "selected": ""},
        {"filter": {}, "selected": "", "extra": pre(M_UNBOUND)},
        {"filter": {}, "selected": "", "extra": pre('persistentvolumeclaim "nope" not found')},
        {"filter": {}, "selected": "",
         "extra": pre('persistentvolumeclaim "c-lost" bound to non-existent persistentvolume "pv-gone"')},
    ]
    return nodes, [], pods, expect, st


# --------------------------------------------------------------------------------------
# VolumeZone (volume_zone.go Filter): a node without any of the four zone / region labels
# passes; otherwise every zone / region label of the pod's bound PVs must contain the
# node's value for that key ("" when the node lacks it); values split on "__"
# (LabelZonesToSet), and a label that fails to parse is ignored.
def fx_volume_zone():
    nodes = [node("a", zone="zone-a"), node("b", zone="zone-b"), node("c"), node("d", labels={REGION: "r1"})]
    st = storage(pvs=[pv("pv-a", labels={ZONE: "zone-a"}), pv("pv-ab", labels={ZONE: "zone-a__zone-b"}),
                      pv("pv-bad", labels={ZONE: "zone-a__"}), pv("pv-r", labels={REGION: "r1"}),
                      pv("pv-beta", labels={BETA_ZONE: "zone-b"})],
                 pvcs=[pvc("c-a", "pv-a"), pvc("c-ab", "pv-ab"), pvc("c-bad", "pv-bad"), pvc("c-r", "pv-r"),
                       pvc("c-beta", "pv-beta")])
    pods = [vpod("p-a", claim("c-a")), vpod("p-ab", claim("c-ab")), vpod("p-bad", claim("c-bad")),
            vpod("p-r", claim("c-r")), vpod("p-beta", claim("c-beta"))]
    Z = ("VolumeZone", M_ZONE)
    expect = [
        {"filter": {"a": None, "b": Z, "c": None, "d": Z}, "selected": "a"},
        {"filter": {"a": None, "b": None, "c": None, "d": Z}, "selected": "b"},
        {"filter": _all("abcd"), "selected": "c"},
        {"filter": {"a": Z, "b": Z, "c": None, "d": None}, "selected": "d"},
        {"filter": {"a": Z, "b": Z, "c": None, "d": Z}, "selected": "c"},
    ]
    return nodes, [], pods, expect, st


# --------------------------------------------------------------------------------------
# VolumeBinding for unbound WaitForFirstConsumer claims (binder.go FindPodVolumes, v1.26):
# claims selected for another node (volume.kubernetes.io/selected-node) fail at once; the others
# go by increasing request (findMatchingVolumes) to FindMatchingVolume -- a PV pre-bound to the
# claim (claimRef) answers by its node affinity alone, else the smallest Available PV of the class
# with enough capacity, the claim's access modes, a matching node affinity, and not chosen by an
# earlier claim of the pod or bound (assumed) to another claim; claims left over must be
# provisionable (checkVolumeProvisions: a provisioner other than kubernetes.io/no-provisioner whose
# class's allowedTopologies admit the node).  Reserve's AssumePodVolumes then binds the chosen PVs
# to the claims and marks provisioned claims selected for the node, which later pods see.
# Reasons: node conflict (bound claims) before bind conflict, joined with ", ".
GI = 1 << 30


def wpv(name, gib, sc, zone=None, claim_ref=None):
    spec = {"capacity": {"storage": f"{gib}Gi"}, "storageClassName": sc, "accessModes": ["ReadWriteOnce"],
            "local": {"path": "/mnt/" + name}}
    if zone is not None:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": [
            {"matchExpressions": [{"key": ZONE, "operator": "In", "values": [zone]}]}]}}
    if claim_ref is not None:
        spec["claimRef"] = {"namespace": "default", "name": claim_ref}
    return {"metadata": {"name": name}, "spec": spec, "status": {"phase": "Available"}}


def wpvc(name, gib, sc):
    return {"metadata": {"name": name, "namespace": "default"},
            "spec": {"storageClassName": sc, "accessModes": ["ReadWriteOnce"],
                     "resources": {"requests": {"storage": f"{gib}Gi"}}}}


def wsc(name, provisioner, zones=None):
    sc = {"metadata": {"name": name}, "provisioner": provisioner, "volumeBindingMode": "WaitForFirstConsumer"}
    if zones is not None:
        sc["allowedTopologies"] = [{"matchLabelExpressions": [{"key": ZONE, "values": list(zones)}]}]
    return sc


def fx_wait_for_first_consumer():
    nodes = [node("a", zone="zone-a"), node("b", zone="zone-b"), node("c", zone="zone-c")]
    za = [{"matchExpressions": [{"key": ZONE, "operator": "In", "values": ["zone-a"]}]}]
    st = storage(
        pvs=[wpv("pv-a-5", 5, "local", "zone-a"), wpv("pv-a-10", 10, "local", "zone-a"),
             wpv("pv-b-20", 20, "local", "zone-b"), wpv("pv-c-8", 8, "local", "zone-c"),
             wpv("pv-pre", 1, "local", "zone-a", claim_ref="l-pre"), wpv("pv-w-3", 3, "wffc", "zone-c"),
             wpv("pv2-a-6", 6, "local2", "zone-a"), wpv("pv2-a-7", 7, "local2", "zone-a"),
             wpv("pv2-b-7", 7, "local2", "zone-b"), pv("pv-za", affinity_terms=za)],
        pvcs=[wpvc("l-4", 4, "local"), wpvc("l-4b", 4, "local"), wpvc("l-9", 9, "local"), wpvc("l-15", 15, "local"),
              wpvc("d-1", 1, "wffc-b"), wpvc("w-2", 2, "wffc"), wpvc("l-pre", 1, "local"), wpvc("x-7", 7, "local2"),
              wpvc("x-6", 6, "local2"), pvc("c-za", "pv-za")],
        scs=[wsc("local", "kubernetes.io/no-provisioner"), wsc("local2", "kubernetes.io/no-provisioner"),
             wsc("wffc", "csi.example.com"), wsc("wffc-b", "csi.example.com", zones=["zone-b"])])
    pods = [vpod("p1", claim("l-4")),     # every node has a PV (a: pv-a-5, the smallest); a (ties)
            vpod("p2", claim("l-4b")),    # a: pv-a-5 taken, pv-a-10; b: pv-b-20; c: pv-c-8; b (a has p1)
            vpod("p3", claim("l-9")),     # 9Gi: pv-a-10 on a; b's pv-b-20 is p2's: no PV, no provisioner
            vpod("p4", claim("l-15")),    # only pv-b-20 is large enough, and it is taken: nowhere
            vpod("p5", claim("d-1")),     # no PV: provisioned where wffc-b's topology allows, b
            vpod("p6", claim("d-1")),     # d-1 is now selected for b: the other nodes fail at once
            vpod("p7", claim("w-2")),     # pv-w-3 on c, provisioning elsewhere (no topology); c (no pods)
            vpod("p8", claim("l-pre")),   # pv-pre is pre-bound: only its zone-a node, though pv-c-8 is free
            vpod("p9", claim("c-za"), claim("l-15")),  # bound pv-za (zone-a) and an impossible claim
            vpod("p10", claim("x-7"), claim("x-6"))]   # x-6 first: a gets pv2-a-6 + pv2-a-7; b's pv2-b-7 once
    B = ("VolumeBinding", M_VB_BIND)
    NB = ("VolumeBinding", M_VB_CONFLICT + ", " + M_VB_BIND)
    expect = [
        {"filter": _all("abc"), "selected": "a"},
        {"filter": _all("abc"), "selected": "b"},
        {"filter": {"a": None, "b": B, "c": B}, "selected": "a"},
        {"filter": _all("abc", B), "selected": ""},
        {"filter": {"a": B, "b": None, "c": B}, "selected": "b"},
        {"filter": {"a": B, "b": None, "c": B}, "selected": "b"},
        {"filter": _all("abc"), "selected": "c"},           # pods: a 2, b 3, c 0
        {"filter": {"a": None, "b": B, "c": B}, "selected": "a"},
        {"filter": {"a": B, "b": NB, "c": NB}, "selected": ""},
        {"filter": {"a": None, "b": B, "c": B}, "selected": "a"},
    ]
    return nodes, [], pods, expect, st


# the assume cache after the fixture's pods (claim -> its PV; claims selected for a node)
WFFC_FINAL_BINDINGS = {"l-4": "pv-a-5", "l-4b": "pv-b-20", "l-9": "pv-a-10", "w-2": "pv-w-3", "l-pre": "pv-pre",
                       "x-6": "pv2-a-6", "x-7": "pv2-a-7"}
WFFC_FINAL_SELECTED = {"d-1": "b"}


FIXTURES = {
    "disk_conflict": fx_disk_conflict,
    "non_csi_limits": fx_non_csi_limits,
    "csi_limits": fx_csi_limits,
    "volume_binding": fx_volume_binding,
    "volume_zone": fx_volume_zone,
    "wait_for_first_consumer": fx_wait_for_first_consumer,
}
