"""Seeded random clusters exercising NodePorts and ImageLocality (test infrastructure).

Nodes list images in Status.Images (shared names with differing sizes, untagged and
registry-port names); bound pods hold container host ports (wildcard and specific IPs, TCP /
UDP, hostPort 0); pending pods want host ports and run containers whose images some nodes
list.  tests/test_portimage.py checks the two oracles against each other on these clusters
and tests/test_gpu_portimage.py the device path (k_schedule batches, the per-pod API,
commit / rollback of UsedPorts) against the C oracle.
"""
import random

MI = 1024 * 1024
IMAGES = ["app:v1", "app:v2", "base:latest", "base", "registry:5000/tool", "registry:5000/tool:latest", "big:1"]
IPS = ["", "0.0.0.0", "10.0.0.1", "10.0.0.2"]
PROTOS = ["", "TCP", "UDP"]
PORTS = [53, 80, 8080, 9090]


def _port(r):
    return {"containerPort": r.choice([80, 443, 9000]), "hostPort": r.choice(PORTS + [0]),
            "protocol": r.choice(PROTOS), "hostIP": r.choice(IPS)}


def _containers(r, allow_ports=True, n=None):
    out = []
    for i in range(n if n is not None else r.choice([1, 1, 2, 3])):
        c = {"name": "c%d" % i, "image": r.choice(IMAGES),
             "resources": {"requests": {"cpu": r.choice(["100m", "250m", "500m"]),
                                        "memory": r.choice(["128Mi", "256Mi", "1Gi"])}}}
        if allow_ports and r.random() < 0.5:
            c["ports"] = [_port(r) for _ in range(r.choice([1, 1, 2]))]
        out.append(c)
    return out


def make(seed, n_nodes=12, n_bound=10, n_pods=30):
    r = random.Random(seed)
    nodes = []
    for i in range(n_nodes):
        imgs = []
        for nm in r.sample(IMAGES, r.choice([0, 1, 2, 3])):
            imgs.append({"names": [nm], "sizeBytes": r.choice([30, 400, 800, 1500, 3000]) * MI})
        st = {"allocatable": {"cpu": r.choice(["4", "8"]), "memory": r.choice(["8Gi", "16Gi"]), "pods": "20",
                              "ephemeral-storage": "20Gi"}}
        if imgs:
            st["images"] = imgs
        lb = {"kubernetes.io/hostname": "n%02d" % i}
        if i % 4:
            lb["topology.kubernetes.io/zone"] = "z%d" % (i % 3)
        nodes.append({"metadata": {"name": "n%02d" % i, "labels": lb}, "spec": {}, "status": st})
    bound = []
    for j in range(n_bound):
        bound.append({"metadata": {"name": "b%02d" % j, "namespace": "default", "labels": {"app": "b"}},
                      "spec": {"nodeName": "n%02d" % r.randrange(n_nodes), "containers": _containers(r)}})
    pods = []
    for j in range(n_pods):
        spec = {"containers": _containers(r)}
        if r.random() < 0.2:
            spec["initContainers"] = _containers(r, n=1)
        pods.append({"metadata": {"name": "p%02d" % j, "namespace": "default", "labels": {"app": "p"}}, "spec": spec})
    return nodes, bound, pods
