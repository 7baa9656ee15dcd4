"""Random clusters with volumes (test infrastructure): nodes with zone / region / instance-type
labels and attach limits (allocatable and CSINode counts), PVs of CSI drivers, EBS and GCE PD
with zone labels and node affinity, claims bound / bound to a missing PV / unbound, and pods
mixing inline disks (GCE PD, EBS, RBD, iSCSI; read-only or not) with claims, shared between
pods.  Every shape the volume plugins distinguish shows up at these sizes; nothing the
device path refuses (CSI migration) is generated.  wffc=True adds unbound WaitForFirstConsumer
claims (a no-provisioner class with local PVs, a CSI class with allowedTopologies or none), PVs
of several sizes with zone affinity, pre-bound (claimRef) PVs and claims already selected for a
node (or for a node outside the snapshot), shared between pods."""
import random

import volume_fixtures as vf
from edge_fixtures import node

ZONES = ["zone-a", "zone-b", "zone-c"]
DRIVERS = ["ebs.csi.aws.com", "pd.csi.storage.gke.io"]


def make(seed: int, n_nodes: int = 12, n_bound: int = 16, n_pods: int = 40, wffc: bool = False):
    rng = random.Random(seed)
    nodes, csinodes = [], []
    for i in range(n_nodes):
        name = "n%02d" % i
        labels, extra = {}, {}
        r = rng.random()
        zone = None
        if r < 0.6:
            zone = rng.choice(ZONES)
        elif r < 0.75:
            labels[vf.REGION] = rng.choice(["r1", "r2"])
        elif r < 0.85:
            labels[vf.BETA_ZONE] = rng.choice(ZONES)
        if rng.random() < 0.5:
            labels[vf.IT] = rng.choice(["m5.large", "t3.small", "c4.xlarge", "z1d.metal"])
        for key in ("attachable-volumes-aws-ebs", "attachable-volumes-gce-pd", "attachable-volumes-azure-disk"):
            if rng.random() < 0.3:
                extra[key] = str(rng.randint(0, 3))
        nodes.append(node(name, zone=zone, labels=labels, extra=extra))
        if rng.random() < 0.6:
            drivers = [{"name": d, "allocatable": {"count": rng.randint(0, 3)}}
                       for d in DRIVERS if rng.random() < 0.7]
            csinodes.append({"metadata": {"name": name}, "spec": {"drivers": drivers}})
    # PVs and claims
    pvs, pvcs = [], []
    for k in range(24):
        kind = rng.choice(["csi", "csi", "ebs", "gce", "plain"])
        src = {"csi": lambda: vf.csi(rng.choice(DRIVERS), "h-%d" % k), "ebs": lambda: vf.ebs("pv-vol-%d" % (k % 9)),
               "gce": lambda: vf.gce("pv-pd-%d" % (k % 7)), "plain": lambda: {}}[kind]()
        labels = {}
        if rng.random() < 0.35:
            zs = rng.sample(ZONES, rng.randint(1, 2))
            labels[rng.choice([vf.ZONE, vf.BETA_ZONE])] = "__".join(zs) + ("__" if rng.random() < 0.1 else "")
        if rng.random() < 0.15:
            labels[vf.REGION] = rng.choice(["r1", "r2"])
        aff = None
        if rng.random() < 0.3:
            aff = [{"matchExpressions": [{"key": vf.ZONE, "operator": "In", "values": rng.sample(ZONES, 2)}]}]
            if rng.random() < 0.3:
                aff.append({"matchExpressions": [{"key": "kubernetes.io/hostname", "operator": "In",
                                                  "values": ["n%02d" % rng.randrange(n_nodes)]}],
                            "matchFields": [{"key": "metadata.name", "operator": "In", "values": ["zz"]}]})
        pvs.append(vf.pv("pv-%d" % k, src, labels=labels, affinity_terms=aff))
        pvcs.append(vf.pvc("c-%d" % k, "pv-%d" % k))
    pvcs += [vf.pvc("c-missing-%d" % k, "pv-none-%d" % k) for k in range(3)]
    pvcs += [vf.pvc("c-unbound", bound=False), vf.pvc("c-sc", bound=False, sc="fast")]
    scs = [{"metadata": {"name": "fast"}, "provisioner": DRIVERS[0], "volumeBindingMode": "Immediate"},
           {"metadata": {"name": "gp"}, "provisioner": "kubernetes.io/aws-ebs", "volumeBindingMode": "Immediate"}]
    pvcs.append(vf.pvc("c-gp", bound=False, sc="gp"))
    n_w = 0
    if wffc:  # WaitForFirstConsumer: classes, candidate PVs, delayed claims
        scs.append(vf.wsc("lw", "kubernetes.io/no-provisioner"))
        scs.append(vf.wsc("cw", DRIVERS[1], zones=rng.sample(ZONES, rng.randint(1, 2)) if rng.random() < 0.7 else None))
        n_w = 12
        for k in range(16):
            cls = "lw" if k < 11 else "cw"
            zone = rng.choice(ZONES) if rng.random() < 0.8 else None
            ref = "w-%d" % rng.randrange(n_w) if rng.random() < 0.12 else None
            pv = vf.wpv("wpv-%d" % k, rng.randint(1, 16), cls, zone=zone, claim_ref=ref)
            if rng.random() < 0.1:
                pv["status"]["phase"] = "Released"
            pvs.append(pv)
        for k in range(n_w):
            c = vf.wpvc("w-%d" % k, rng.randint(1, 12), "lw" if rng.random() < 0.7 else "cw")
            if rng.random() < 0.15:
                c["metadata"]["annotations"] = {"volume.kubernetes.io/selected-node":
                                                rng.choice(["n%02d" % rng.randrange(n_nodes), "gone"])}
            pvcs.append(c)
        seen_ref = set()
        for pv in pvs:  # at most one PV pre-bound to a claim (the device path refuses two)
            ref = pv["spec"].get("claimRef")
            if ref:
                if ref["name"] in seen_ref:
                    del pv["spec"]["claimRef"]
                seen_ref.add(ref["name"])

    def volumes(pending):
        out = []
        for _ in range(rng.choice([0, 1, 1, 2, 2, 3])):
            r = rng.random()
            if r < 0.12:
                out.append(vf.gce("pd-%d" % rng.randrange(4), ro=rng.random() < 0.5))
            elif r < 0.22:
                out.append(vf.ebs("vol-%d" % rng.randrange(5), ro=rng.random() < 0.3))
            elif r < 0.27:
                out.append(vf.rbd(rng.sample(["m1", "m2", "m3"], rng.randint(1, 2)), rng.choice(["p", "q"]),
                                  "img-%d" % rng.randrange(2), ro=rng.random() < 0.5))
            elif r < 0.32:
                out.append({"iscsi": {"iqn": "iqn-%d" % rng.randrange(2), "targetPortal": "t", "lun": 0,
                                      "readOnly": rng.random() < 0.5}})
            elif r < 0.36:
                out.append(vf.azure("az-%d" % rng.randrange(3)))
            elif n_w and pending and r < 0.70:
                out.append(vf.claim("w-%d" % rng.randrange(n_w)))
            elif r < 0.94 or not pending:
                out.append(vf.claim("c-%d" % rng.randrange(24)))
            else:
                out.append(vf.claim(rng.choice(["c-missing-0", "c-missing-1", "c-unbound", "c-sc", "nope"])))
        return out

    bound = [vf.vpod("b%02d" % i, *volumes(False), node_name="n%02d" % rng.randrange(n_nodes))
             for i in range(n_bound)]
    bound.append(vf.vpod("b-gp", vf.claim("c-gp"), node_name="n00"))  # an unbound in-tree claim (matchProvisioner)
    pods = [vf.vpod("p%03d" % i, *volumes(True)) for i in range(n_pods)]
    return nodes, bound, pods, vf.storage(pvs, pvcs, scs, csinodes)
